"""Where the shadow kernel's time goes, per 64-entry task (a task-clock build, RT_TASK_CLOCK).

Renders one rank's share of config 3 (rt_render_bands_async, block-cyclic 8-row bands) and
reads the shadow kernel's task clock of that pass: per task its wall time, the mean and
largest distance of its origins from the scene ball's centre (in scene radii) and its
first lane's light.  A wave of the persistent grid takes tasks w, w + G, w + 2G, ..., so the
kernel lasts at least as long as its slowest wave's tasks together.
usage: RT_LIB=rust_tracer_amd/librt_hip_clock.so python tools/shadow_tail.py [world ...]
       (default worlds 1 8; build: tools/build_variant.sh clock -DRT_TASK_CLOCK=1)"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from rust_tracer_amd import DeviceScene, SceneDesc, abi, band_rows_per_rank  # noqa: E402

WORDS = 2 + 4 * (1 << 20)


def main():
    worlds = [int(x) for x in sys.argv[1:]] or [1, 8]
    L = abi.lib()
    L.rt_debug_shadow_clock.argtypes = [C.POINTER(C.c_uint32), C.c_uint32]
    s = DeviceScene(SceneDesc.synth_config(3))
    w, h = 1920, 1080
    cam = abi.camera(w, h)
    stream = torch.cuda.current_stream().cuda_stream
    buf = np.zeros(WORDS, dtype=np.uint32)
    for world in worlds:
        rpr = band_rows_per_rank(h, 8, world)
        img = torch.zeros((rpr, w, 3), dtype=torch.float32, device="cuda")
        cnt = torch.zeros(3, dtype=torch.int64, device="cuda")
        for _ in range(3):
            s.render_bands_async(cam, 8, 8, 0, world, img.data_ptr(), cnt.data_ptr(), stream)
            torch.cuda.synchronize()
        if L.rt_debug_shadow_clock(buf.ctypes.data_as(C.POINTER(C.c_uint32)), WORDS):
            raise SystemExit("rt_debug_shadow_clock failed")
        n, g = int(buf[0]), int(buf[1])
        tasks = (n + 63) // 64
        rec = buf[2:2 + 4 * tasks].reshape(tasks, 4)
        us = rec[:, 0].astype(np.float64) / 100.0  # 100 MHz ticks
        dmean = rec[:, 1].view(np.float32)
        dmax = rec[:, 2].view(np.float32)
        light = rec[:, 3] >> 8
        wave_sum = np.bincount(np.arange(tasks) % g, weights=us, minlength=g)
        print(f"world {world}: {n} shadow entries, {tasks} tasks over {g} waves "
              f"({tasks / g:.1f} per wave); task us mean {us.mean():.2f} p50 {np.median(us):.2f} "
              f"p99 {np.percentile(us, 99):.1f} max {us.max():.1f}; slowest wave {wave_sum.max():.1f} us "
              f"(mean wave {wave_sum.mean():.1f})", flush=True)
        for lo, hi in ((0, 5), (5, 20), (20, 50), (50, 100), (100, 200), (200, 1e9)):
            m = (us >= lo) & (us < hi)
            print(f"   tasks {lo:>4}-{hi if hi < 1e9 else 'inf':>4} us: {int(m.sum()):7d}  time {us[m].sum() / 1e3:8.3f} ms  "
                  f"origin distance mean {float(dmean[m].mean()) if m.any() else 0:.2f} R", flush=True)
        top = np.argsort(-us)[:16]
        print("   slowest tasks: position in queue, us, origin distance mean / max (R), light", flush=True)
        for i in top:
            print(f"     {i / tasks:6.3f}  {us[i]:7.1f}  {dmean[i]:6.2f} / {dmax[i]:6.2f}  {int(light[i])}", flush=True)
        wmax = int(np.argmax(wave_sum))
        wt = us[wmax::g]
        print(f"   slowest wave {wmax}: tasks " + " ".join(f"{x:.0f}" for x in wt), flush=True)
    s.close()


if __name__ == "__main__":
    main()
