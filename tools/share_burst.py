"""One rank's share of a K-frame burst (bench.py's timed region) on one GPU, no gather:
K frames in passes of B frames over F slots, for world sizes / B values.
usage: python tools/share_burst.py  (env WORLDS=8,4,2 BATCHES=4,5,8 FLIGHT=4 K=20 REPS=3 GRID_SHARE=75)"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from rust_tracer_amd import DeviceScene, SceneDesc, abi, band_rows_per_rank  # noqa: E402


def main():
    w, h, depth = 1920, 1080, 8
    worlds = [int(x) for x in os.environ.get("WORLDS", "8,4,2").split(",")]
    batches = [int(x) for x in os.environ.get("BATCHES", "4,5,8").split(",")]
    F = int(os.environ.get("FLIGHT", "4"))
    K = int(os.environ.get("K", "20"))
    reps = int(os.environ.get("REPS", "3"))
    desc = SceneDesc.synth_config(3)
    scenes = [DeviceScene(desc) for _ in range(F)]
    share = int(os.environ.get("GRID_SHARE", "75"))  # as FramePipeline with passes in flight
    if F > 1:
        for s in scenes:
            s.set_grid_share(share)
    streams = [torch.cuda.Stream() for _ in scenes]
    cnt = torch.zeros(3, dtype=torch.int64, device="cuda")
    cam = abi.camera(w, h)
    for world in worlds:
        rpr = band_rows_per_rank(h, 8, world)
        for b in batches:
            bufs = [torch.zeros((b, rpr, w, 3), dtype=torch.float32, device="cuda") for _ in scenes]
            # an animation, as bench.py's default: frame i's camera origin x = 0.01 (i mod 64)
            cams = []
            for i in range(b):
                c = abi.camera(w, h)
                c.origin[0] = 0.01 * i
                cams.append(c)

            def burst(k):
                p = 0
                while k > 0:
                    n = min(b, k)
                    k -= n
                    i = p % F
                    p += 1
                    scenes[i].render_bands_batch_async(cams[:n], depth, 8, 0, world, bufs[i].data_ptr(),
                                                       cnt.data_ptr(), streams[i].cuda_stream)
            burst(F * b)  # sizes every slot's workspace
            torch.cuda.synchronize()
            ts = []
            for _ in range(reps):
                t0 = time.perf_counter()
                burst(K)
                torch.cuda.synchronize()
                ts.append((time.perf_counter() - t0) / K * 1e3)
            print(f"world {world} K {K} batch {b} inflight {F}: {min(ts):.3f} ms per share-frame "
                  f"(all {', '.join(f'{t:.3f}' for t in ts)})", flush=True)
    for s in scenes:
        s.close()


if __name__ == "__main__":
    main()
