// TEST INFRASTRUCTURE ONLY: the reference's HDR decoder, OpenglRayTracing/hdrloader.cpp, compiled
// unmodified from /root/reference by oracle/ref_build.py (oracle/_ref/ref_hdr; the file is
// #included whole, so its static scanline decoders are callable here), run on a .hdr file; writes
// width, height (int32) and the width * height * 3 float32 colours to a binary file, which
// tests/golden/make_ref_fixtures.py turns into tests/golden/ref/hdr_decode_*.json.
//
// HDRLoader::load itself mis-parses on LP64: it reads the resolution line with sscanf("%ld") into
// ints (hdrloader.cpp:66), and the 8-byte store for the width overwrites the height (a height of 0
// here). On the reference's own platform (MSVC, LLP64: long is 32 bits) the same line parses both.
// So this harness follows load() (hdrloader.cpp:28-91) with the resolution read into longs and
// calls the reference's own decrunch / workOnRGBE (hdrloader.cpp:105-191) for every scanline in
// load()'s order: every pixel value comes from the reference's code.
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "hdrloader.cpp"

int main(int argc, char** argv) {
  if (argc != 3) {
    std::fprintf(stderr, "usage: ref_hdr in.hdr out.bin\n");
    return 2;
  }
  FILE* file = std::fopen(argv[1], "rb");
  if (!file) return 1;
  char str[16];
  if (std::fread(str, 10, 1, file) != 1 || std::memcmp(str, "#?RADIANCE", 10)) return 1;  // load(): magic
  std::fseek(file, 1, SEEK_CUR);
  char c = 0, oldc;
  while (true) {  // load(): the header, up to an empty line
    oldc = c;
    c = (char)std::fgetc(file);
    if (c == 0xa && oldc == 0xa) break;
  }
  char reso[200];
  int i = 0;
  while (i < 199) {  // load(): the resolution line
    c = (char)std::fgetc(file);
    reso[i++] = c;
    if (c == 0xa) break;
  }
  reso[i] = 0;
  long h = 0, w = 0;
  if (std::sscanf(reso, "-Y %ld +X %ld", &h, &w) != 2 || w <= 0 || h <= 0) return 1;
  float* cols = new float[(size_t)w * h * 3];
  RGBE* scanline = new RGBE[w];
  float* p = cols;
  for (long y = h - 1; y >= 0; y--) {  // load()'s scanline loop
    if (decrunch(scanline, (int)w, file) == false) break;
    workOnRGBE(scanline, (int)w, p);
    p += w * 3;
  }
  std::fclose(file);
  FILE* o = std::fopen(argv[2], "wb");
  if (!o) return 1;
  const int wh[2] = {(int)w, (int)h};
  std::fwrite(wh, sizeof(int), 2, o);
  std::fwrite(cols, sizeof(float), (size_t)w * h * 3, o);
  std::fclose(o);
  std::printf("%ld %ld\n", w, h);
  return 0;
}
