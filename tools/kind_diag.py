#!/usr/bin/env python3
"""Fetch counts of both runtime-tree record kinds against the CPU restatement.

Round 1 reported that a version choosing the runtime tree's record kind at run
time made the fetch-counting kernel (PT_FLAG_COUNT_FETCHES: always the uploaded
tree, its top staged in LDS) disagree with the oracle. The suspected
mechanism: the LDS copy of the staged tree's top sized by the
runtime tree's record kind (3 float4 per node when quantized) while the
uploaded tree (4 float4 per node) is the one staged, leaving device nodes
96..127 of that copy unwritten. A build reconstructing it (tried once this
round) ended without a result -- a walk through unwritten LDS can read
anywhere -- and was not run again. The product sizes the copy from the staged
tree's own kind; this tool checks that both record kinds count exactly:

    python tools/tune.py --build kquant:PT_QUANT_NODES=1     # here
    python tools/kind_diag.py kquant ; python tools/kind_diag.py base   # GPU box

Prints the GPU fetch counts of c2 at 480x270 beside the CPU restatement's (the
oracle, test infrastructure) and exits 1 when any total differs by more than
test_fetch_counts_match_oracle's 1e-3.
"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def main():
    variant = sys.argv[1] if len(sys.argv) > 1 else "base"
    from opengl_ray_tracing_amd import _native
    if variant != "base":
        _native.use_variant(variant)
    import oracle  # test infrastructure: the checker
    from opengl_ray_tracing_amd import FLAG_COUNT_FETCHES, Renderer, orbit_camera, scenes
    import numpy as np
    cfg, tris, nodes, hdr = scenes.build_config("c2")
    w, h = 480, 270
    eye, rot = orbit_camera(*cfg.camera)
    with Renderer(w, h, cfg.integrator, max_bounce=cfg.max_bounce, flags=FLAG_COUNT_FETCHES) as r:
        r.upload_scene(tris, nodes)
        r.upload_env(hdr)
        r.render_frame(eye, rot, 0)
        st = r.stats()
    orc = oracle.Oracle(tris, nodes, hdr)
    _, cnt = orc.render(w, h, cfg.integrator, 0, eye, rot, accum=np.zeros((h, w, 4), np.float32),
                        max_bounce=cfg.max_bounce)
    rows = {k: (int(a), int(b)) for k, a, b in [("rays", st.rays, cnt.rays), ("nodes", st.node_fetch, cnt.nodes),
                                                ("tris", st.tri_fetch, cnt.tris), ("mats", st.mat_fetch, cnt.mats),
                                                ("texels", st.tex_fetch, cnt.texels)]}
    bad = [k for k, (a, b) in rows.items() if abs(a - b) > 1e-3 * b + 2]
    print(json.dumps({"variant": variant, "gpu_vs_oracle": rows, "mismatch": bad}))
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
