"""Where each trace level's time goes, per task (the task-clock build, RT_TASK_CLOCK).

Renders one rank's share of config 3 (rt_render_bands_async, block-cyclic 8-row bands) and
reads the trace kernels' task clocks of that pass: per level and task its wall time (from its
iteration's start to the next's), the mean distance of its origins from the scene ball's
centre (scene radii), its lanes and whether they start inside a sphere / cube.  A level lasts
at least as long as its slowest wave's tasks together.
usage: RT_LIB=rust_tracer_amd/librt_hip_clock.so python tools/trace_tail.py [world ...]
       (default worlds 1 8; build: tools/build_variant.sh clock -DRT_TASK_CLOCK=1)"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from rust_tracer_amd import DeviceScene, SceneDesc, abi, band_rows_per_rank  # noqa: E402

TASKS = 1 << 16
LEVEL_WORDS = 4 + 4 * TASKS


def main():
    worlds = [int(x) for x in sys.argv[1:]] or [1, 8]
    L = abi.lib()
    L.rt_debug_trace_clock.argtypes = [C.POINTER(C.c_uint32), C.c_uint32]
    s = DeviceScene(SceneDesc.synth_config(3))
    w, h, depth = 1920, 1080, 8
    cam = abi.camera(w, h)
    stream = torch.cuda.current_stream().cuda_stream
    buf = np.zeros(16 * LEVEL_WORDS, dtype=np.uint32)
    for world in worlds:
        rpr = band_rows_per_rank(h, 8, world)
        img = torch.zeros((rpr, w, 3), dtype=torch.float32, device="cuda")
        cnt = torch.zeros(3, dtype=torch.int64, device="cuda")
        for _ in range(3):
            s.render_bands_async(cam, depth, 8, 0, world, img.data_ptr(), cnt.data_ptr(), stream)
            torch.cuda.synchronize()
        if L.rt_debug_trace_clock(buf.ctypes.data_as(C.POINTER(C.c_uint32)), buf.size):
            raise SystemExit("rt_debug_trace_clock failed")
        print(f"world {world}:", flush=True)
        for lvl in range(depth):
            blk = buf[lvl * LEVEL_WORDS:(lvl + 1) * LEVEL_WORDS]
            n, g, wd = int(blk[0]), int(blk[1]), int(blk[2])
            if n == 0 or wd == 0:
                continue
            tasks = min((n + wd - 1) // wd, TASKS)
            rec = blk[4:4 + 4 * tasks].reshape(tasks, 4)
            us = rec[:, 0].astype(np.float64) / 100.0  # 100 MHz ticks
            dmean = rec[:, 1].view(np.float32)
            lanes = rec[:, 2] & 0xFFFF
            inside = (rec[:, 2] >> 16) & 1
            wave_sum = np.bincount(np.arange(tasks) % g, weights=us, minlength=g)
            top = np.argsort(-us)[:5]
            print(f"  level {lvl}: {n} rays, {tasks} tasks of {wd} over {g} waves; task us mean {us.mean():.1f} "
                  f"p50 {np.median(us):.1f} p99 {np.percentile(us, 99):.1f} max {us.max():.1f}; slowest wave "
                  f"{wave_sum.max():.1f} us; tasks > 2x p50: {int((us > 2 * np.median(us)).sum())}", flush=True)
            print("     slowest: " + "; ".join(
                f"pos {i / tasks:.3f} {us[i]:.0f} us D {dmean[i]:.1f} R lanes {int(lanes[i])}{' in' if inside[i] else ''}"
                for i in top), flush=True)
    s.close()


if __name__ == "__main__":
    main()
