"""Per-level frequency of the scan's divergent hit paths (RT_DIAG build).
Level k statistics = stats(depth k+1) - stats(depth k).
usage: RT_LIB=rust_tracer_amd/librt_hip_stats.so python tools/scan_stats.py [config] [max_depth]"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rust_tracer_amd import DeviceScene, SceneDesc, abi  # noqa: E402

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 3
maxd = int(sys.argv[2]) if len(sys.argv) > 2 else 8
L = abi.lib()
L.rt_debug_scan_stats.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
s = DeviceScene(SceneDesc.synth_config(cfg))
s.render(1920, 1080, 1)
st = (C.c_ulonglong * 40)()
L.rt_debug_scan_stats(st, 1)
prev = [0] * 16
prev_scans = 0
names = ["wave-scans", "dsph-pair solve", "gsph solve", "tri-pair finish", "cube-tri pass"]
print(f"config {cfg}: per level, hit-path entries per wave-scan")
print("lvl  lane-scans  wave-scans lanes/ws " + " ".join(f"{n:>16s}" for n in names[1:]))
for d in range(1, maxd + 1):
    _, cnt, ms, _ = s.render(1920, 1080, d)
    L.rt_debug_scan_stats(st, 1)
    cur = list(st)
    scans = cnt["node_rays"] + cnt["shadow_rays"]
    dl = [c - p for c, p in zip(cur, prev)] if False else cur
    # stats were reset, so `cur` is the whole depth-d frame; subtract the depth-(d-1) frame
    lvl = [c - p for c, p in zip(cur, prev)]
    ds = scans - prev_scans
    ws = max(1, lvl[0])
    print(f"{d-1:3d} {ds:11d} {lvl[0]:10d} {ds / ws:8.1f} " + " ".join(f"{lvl[i] / ws:16.2f}" for i in range(1, 5))
          + f"   frame {ms:.1f} ms")
    prev, prev_scans = cur, scans
