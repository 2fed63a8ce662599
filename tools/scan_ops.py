"""Per-frame test counts of the scans (rt_scene_scan_ops), hierarchy on vs off.

usage: python tools/scan_ops.py [config=3] [width=1920] [height=1080] [depth=8]
Prints, per mode, the lane-weighted counts of each test kind, per traced ray (node +
shadow), and the frame's kernel time.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rust_tracer_amd import DeviceScene, SceneDesc


def run(config, w, h, depth, bvh):
    s = DeviceScene(SceneDesc.synth_config(config), tuning=None if bvh else "bvh=0")
    s.render(w, h, depth)
    s.set_scan_counting(True)
    s.scan_ops(reset=True)
    _, cnt, ms, _ = s.render(w, h, depth)
    ops = s.scan_ops()
    rays = cnt["node_rays"] + cnt["shadow_rays"]
    print(f"bvh={bvh} kernel {ms:.2f} ms  node rays {cnt['node_rays']} shadow rays {cnt['shadow_rays']}")
    for k, v in ops.items():
        if k.startswith("cycles"):
            share = v / max(1, ops["cycles_scans"])
            print(f"   {k:14s} {v:14d}  share of scan cycles {share:6.3f}")
        else:
            print(f"   {k:14s} {v:14d}  per ray {v / rays:9.2f}")
    s.close()


if __name__ == "__main__":
    a = [int(x) for x in sys.argv[1:]]
    config, w, h, depth = (a + [3, 1920, 1080, 8][len(a):])[:4]
    run(config, w, h, depth, True)
    if not os.environ.get("SKIP_LINEAR"):
        run(config, w, h, depth, False)
