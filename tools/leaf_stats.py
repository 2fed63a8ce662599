"""Leaf occupancy of the wave-uniform walk (RT_DIAG build, tools/scan_stats.sh):
of the lanes active at each leaf visit, how many had their own box test admit the leaf.
usage: RT_LIB=rust_tracer_amd/librt_hip_stats.so python tools/leaf_stats.py [config]"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rust_tracer_amd import DeviceScene, SceneDesc, abi  # noqa: E402

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 3
L = abi.lib()
L.rt_debug_scan_stats.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
s = DeviceScene(SceneDesc.synth_config(cfg))
st = (C.c_ulonglong * 40)()
for depth in (1, 2, 8):
    L.rt_debug_scan_stats(st, 1)
    _, cnt, ms, _ = s.render(1920, 1080, depth)
    L.rt_debug_scan_stats(st, 1)
    v = list(st)
    rays = cnt["node_rays"] + cnt["shadow_rays"]
    print(f"config {cfg} depth {depth}: rays {rays}, wave scans {v[0]}, leaf visits {v[7]} "
          f"({v[7] / max(1, v[0]):.2f} per wave scan)")
    for name, b, n in (("trace", 5, cnt["node_rays"]), ("shadow", 8, cnt["shadow_rays"])):
        print(f"  {name}: leaf visits {v[b + 2]}, lanes at leaves {v[b]}, needing the leaf {v[b + 1]}: "
              f"occupancy {v[b + 1] / max(1, v[b]):.3f}; per ray needed {v[b + 1] / max(1, n):.2f}, "
              f"executed {v[b] / max(1, n):.2f}")
    print(f"  hit points: inside the Morton cube {v[11]}, outside {v[12]} (level 0: {v[13]} / {v[14]})")
    print(f"  shadow rays a hierarchy walk serves (no light buffer, undecided after the planes): {v[15]} "
          f"of {cnt['shadow_rays']} ({v[15] / max(1, cnt['shadow_rays']):.3f}); by D / R in (0,3] (3,6] (6,12] "
          f"(12,25] (25,50] (50,inf): {v[16:22]}; light farther than 45: {v[22]}")
    print(f"  trace walks' lanes by D / R (same buckets): {v[23:29]}; leaf visits of trace waves whose farthest "
          f"lane is within 3 R / 12 R / beyond: {v[29:32]}")
    print(f"  leaf-major planning (trace rays): leaves a ray's own box tests admit with no nearest-hit bound "
          f"{v[32] / max(1, v[33]):.2f} per ray, with its final nearest hit as the bound {v[34] / max(1, v[33]):.2f} "
          f"({v[33]} walks)")
    print(f"  hit paths per wave scan: dsph {v[1] / max(1, v[0]):.2f} gsph {v[2] / max(1, v[0]):.2f} "
          f"tri {v[3] / max(1, v[0]):.2f} cube-tri {v[4] / max(1, v[0]):.2f}")
