// Which hardware queue does each HIP stream get? (diagnostic for the frames-in-flight pipeline)
// Creates streams in the order given by argv, launches a short spin kernel on each, and prints
// nothing: run under rocprofv3 --kernel-trace and read Queue_Id per kernel (tag = blockIdx count).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
__global__ void spin(int tag, long long cycles) {
  const long long t0 = clock64();
  while (clock64() - t0 < cycles) {
  }
  (void)tag;
}
int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 6;
  std::vector<hipStream_t> s(n);
  for (int k = 0; k < n; k++) hipStreamCreateWithFlags(&s[k], hipStreamNonBlocking);
  for (int rep = 0; rep < 2; rep++)
    for (int k = 0; k < n; k++) hipLaunchKernelGGL(spin, dim3(k + 1), dim3(64), 0, s[k], k, 2000000LL);
  hipDeviceSynchronize();
  printf("queue_map: %d streams done\n", n);
  return 0;
}
