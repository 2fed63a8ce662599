"""Time one rank's share of a frame (rt_render_bands_async, block-cyclic bands) on one GPU,
for world sizes 1..8: the strong-scaling ceiling of the multi-GPU path before the gather.
usage: python tools/band_share_time.py [config=3] [width height]
   (env WORLDS=1,2,4,8; KT=1 adds the per-kind kernel times of the timed renders,
   rt_scene_kernel_times: trace / sorts / shadow / combine launch groups, ms per share)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from rust_tracer_amd import DeviceScene, SceneDesc, abi, band_rows_per_rank  # noqa: E402


def main():
    config = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    w = int(sys.argv[2]) if len(sys.argv) > 2 else 1920
    h = int(sys.argv[3]) if len(sys.argv) > 3 else 1080
    depth = 4 if config == 2 else 8
    s = DeviceScene(SceneDesc.synth_config(config))
    kt = os.environ.get("KT", "0") == "1"
    if kt:
        s.set_kernel_timing(True)
    cam = abi.camera(w, h)
    stream = torch.cuda.current_stream().cuda_stream
    base = None
    worlds = [int(x) for x in os.environ.get("WORLDS", "1,2,4,8").split(",")]
    for world in worlds:
        rpr = band_rows_per_rank(h, 8, world)
        buf = torch.zeros((rpr, w, 3), dtype=torch.float32, device="cuda")
        cnt = torch.zeros(3, dtype=torch.int64, device="cuda")
        times = []
        for it in range(8):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            s.render_bands_async(cam, depth, 8, 0, world, buf.data_ptr(), cnt.data_ptr(), stream)
            b.record()
            torch.cuda.synchronize()
            if it >= 2:
                times.append(a.elapsed_time(b))
            elif kt:
                s.kernel_times(reset=True)
        t = sorted(times)[len(times) // 2]
        base = base or t
        print(f"{w}x{h} world {world}: rank-0 share {t:.3f} ms  -> ideal speedup {base / t:.2f} (x{world})", flush=True)
        if kt:
            d = s.kernel_times(reset=True)
            n = len(times)
            print("   kernel ms per share: " + "  ".join(f"{k} {d[k] / n:.3f}" for k in DeviceScene.KERNEL_KINDS), flush=True)
    s.close()


if __name__ == "__main__":
    main()
