"""Per wave-iteration wall-clock records of the trace kernel (RT_TASK_CLOCK debug build
path): where a level's time goes when it has fewer tasks than wave slots.
usage: python tools/task_clock.py [config=3] [world=1,8]
Prints per level: wave iterations, ticks (10 ns) median / p90 / p99 / max, and the
slowest iterations' task bases."""
import ctypes as C
import os
import sys

os.environ.setdefault("RT_TASK_CLOCK", "400000")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from rust_tracer_amd import DeviceScene, SceneDesc, abi, band_rows_per_rank  # noqa: E402


def main():
    config = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    worlds = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "1,8").split(",")]
    w, h, depth = 1920, 1080, (4 if config == 2 else 8)
    cap = int(os.environ["RT_TASK_CLOCK"])
    s = DeviceScene(SceneDesc.synth_config(config))
    cam = abi.camera(w, h)
    stream = torch.cuda.current_stream().cuda_stream
    L = abi.lib()
    out = np.zeros(4 + 4 * cap, dtype=np.uint32)
    for world in worlds:
        rpr = band_rows_per_rank(h, 8, world)
        buf = torch.zeros((rpr, w, 3), dtype=torch.float32, device="cuda")
        cnt = torch.zeros(3, dtype=torch.int64, device="cuda")
        for _ in range(3):
            s.render_bands_async(cam, depth, 8, 0, world, buf.data_ptr(), cnt.data_ptr(), stream)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        s.render_bands_async(cam, depth, 8, 0, world, buf.data_ptr(), cnt.data_ptr(), stream)
        b.record()
        torch.cuda.synchronize()
        assert L.rt_debug_task_clock(out.ctypes.data_as(C.POINTER(C.c_uint32)), cap) == 0
        n = min(int(out[0]), cap)
        rec = out[4:4 + 4 * n].reshape(n, 4)
        t0 = int(rec[:, 1].astype(np.int64).min())
        print(f"world {world}: {n} wave iterations recorded (last frame, {a.elapsed_time(b):.3f} ms; "
              f"times in ticks from the frame's first task)")
        for lv in range(depth):
            r = rec[rec[:, 0] == lv]
            if len(r) == 0:
                continue
            t = np.sort(r[:, 2].astype(np.float64))
            q = lambda p: t[min(len(t) - 1, int(p * len(t)))]  # noqa: E731
            st = r[:, 1].astype(np.int64)
            en = st + r[:, 2].astype(np.int64)
            print(f"  level {lv}: iters {len(t):6d}  ticks med {q(0.5):7.0f} p90 {q(0.9):7.0f} p99 {q(0.99):7.0f} "
                  f"max {t[-1]:7.0f}  first start {st.min() - t0:8d}  last start {st.max() - t0:8d}  "
                  f"last end {en.max() - t0:8d}", flush=True)
            # where the slow tasks sit in the sorted queue: mean ticks per decile of the queue
            # position, and the deciles of the slowest 1% (inside rays sort last)
            b = r[:, 1].astype(np.float64)
            pos = (b - b.min()) / max(1.0, float(b.max() - b.min()) + 64.0)
            dec = np.minimum((pos * 10).astype(int), 9)
            tk = r[:, 2].astype(np.float64)
            means = [tk[dec == d].mean() if np.any(dec == d) else 0.0 for d in range(10)]
            slow = dec[tk >= np.quantile(tk, 0.99)]
            print("    mean ticks per queue decile: " + " ".join(f"{m:6.0f}" for m in means) +
                  "   slowest 1% by decile: " + " ".join(str(int(np.sum(slow == d))) for d in range(10)), flush=True)
            t0 = int(en.max())
    s.close()


if __name__ == "__main__":
    main()
