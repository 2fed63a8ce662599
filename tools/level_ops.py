"""Per-level cost of the trace kernel (config 3, 1080p): rays per level and the counted
kernels' test / cycle counters, as differences between renders of depth d and d - 1
(tuning count=trace: only the trace kernels count).  python tools/level_ops.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rust_tracer_amd import DeviceScene, SceneDesc  # noqa: E402

s = DeviceScene(SceneDesc.synth_config(3), tuning="count=trace")
s.set_scan_counting(True)
prev_ops, prev_nodes = None, 0
keys = DeviceScene.SCAN_OPS
print("level rays " + " ".join(k for k in keys))
for d in range(1, 9):
    s.scan_ops(reset=True)
    _, c, ms, _ = s.render(1920, 1080, d)
    ops = s.scan_ops()
    rays = c["node_rays"] - prev_nodes
    if prev_ops is not None:
        delta = {k: ops[k] - prev_ops[k] for k in keys}
    else:
        delta = ops
    print(d - 1, rays, " ".join(f"{k}={delta[k] / max(rays, 1):.1f}" for k in keys), flush=True)
    prev_ops, prev_nodes = ops, c["node_rays"]
