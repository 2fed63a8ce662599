"""Digest of the scene image rt_scene_create would upload (rt_scene_layout_digest: the host
build alone, no GPU) for the benchmark and stress scenes under several tunings, with the
build time.  Used to check that a change to the scene builder leaves the device image
unchanged (run before and after, compare the JSON)."""
import ctypes as C
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rust_tracer_amd import SceneDesc, abi  # noqa: E402


def scenes():
    from tests.test_gpu_cull_stress import stress_scene
    out = [("config2", SceneDesc.synth_config(2)), ("config3", SceneDesc.synth_config(3)),
           ("my_scene", SceneDesc.my_scene())]
    for seed, scale, near, sl in [(11, 1.0, False, False), (12, 0.01, True, True), (13, 1000.0, False, True)]:
        out.append((f"stress{seed}", stress_scene(seed, scale, near, sl)))
    return out


def main():
    tunings = sys.argv[2:] if len(sys.argv) > 2 else ["", "lb_tiers=1", "lb_near_all=0", "lb_reach=0", "lb_res=32"]
    L = abi.lib()
    res = {}
    for name, d in scenes():
        for tun in tunings:
            dg, nb = C.c_uint64(), C.c_uint64()
            t = time.perf_counter()
            st = L.rt_scene_layout_digest(d.ptr(), tun.encode(), C.byref(dg), C.byref(nb))
            ms = 1e3 * (time.perf_counter() - t)
            res[f"{name}|{tun}"] = {"status": st, "digest": f"{dg.value:016x}", "bytes": nb.value}
            print(f"{name:10s} {tun:16s} st {st} digest {dg.value:016x} bytes {nb.value:>11d} {ms:8.1f} ms", flush=True)
    if len(sys.argv) > 1 and sys.argv[1] != "-":
        json.dump(res, open(sys.argv[1], "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
