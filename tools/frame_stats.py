#!/usr/bin/env python3
"""Per-frame kernel time, traversal tree and split items of one config on the GPU
(what the runtime's probe and the adaptive tile splitting did frame by frame).

    python tools/frame_stats.py c4 [frames]
"""
import sys
sys.path.insert(0, '.')
from opengl_ray_tracing_amd import Renderer, orbit_camera, scenes
cfg, tris, nodes, hdr = scenes.build_config(sys.argv[1])
eye, rot = orbit_camera(*cfg.camera)
with Renderer(cfg.width, cfg.height, cfg.integrator, max_bounce=cfg.max_bounce) as r:
    r.upload_scene(tris, nodes); r.upload_env(hdr)
    for f in range(int(sys.argv[2]) if len(sys.argv) > 2 else 40):
        r.render_frame(eye, rot, f)
        st = r.stats()
        print(f, 'ms %.3f' % st.kernel_ms, 'tree', st.runtime_tree, 'split', st.split_items)
