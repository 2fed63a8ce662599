"""Throughput of one rank's share of a frame with F frames in flight (F scene handles,
each with its own workspace, on F HIP streams), for world sizes 1..8, on one GPU.
At small shares a trace level has fewer tasks than wave slots and its slowest task sets
its length (Multi-GPU); frames in flight fill the idle slots.
usage: python tools/inflight_time.py [config=3] [width height]   (env WORLDS, FLIGHTS)"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from rust_tracer_amd import DeviceScene, SceneDesc, abi, band_rows_per_rank  # noqa: E402


def main():
    config = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    w = int(sys.argv[2]) if len(sys.argv) > 2 else 1920
    h = int(sys.argv[3]) if len(sys.argv) > 3 else 1080
    depth = 4 if config == 2 else 8
    desc = SceneDesc.synth_config(config)
    cam = abi.camera(w, h)
    worlds = [int(x) for x in os.environ.get("WORLDS", "1,2,4,8").split(",")]
    flights = [int(x) for x in os.environ.get("FLIGHTS", "1,2,3").split(",")]
    frames = int(os.environ.get("FRAMES", "24"))
    scenes = [DeviceScene(desc) for _ in range(max(flights))]
    streams = [torch.cuda.Stream() for _ in scenes]
    for world in worlds:
        rpr = band_rows_per_rank(h, 8, world)
        bufs = [torch.zeros((rpr, w, 3), dtype=torch.float32, device="cuda") for _ in scenes]
        cnts = [torch.zeros(3, dtype=torch.int64, device="cuda") for _ in scenes]
        base = None
        for f in flights:
            for rep in range(2):  # rep 0 warms every workspace up
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for k in range(frames):
                    i = k % f
                    scenes[i].render_bands_async(cam, depth, 8, 0, world, bufs[i].data_ptr(), cnts[i].data_ptr(),
                                                 streams[i].cuda_stream)
                torch.cuda.synchronize()
                dt = (time.perf_counter() - t0) / frames * 1e3
            same = all(torch.equal(bufs[0], bufs[i]) for i in range(1, f))
            base = base or dt
            print(f"world {world} in-flight {f}: {dt:.3f} ms per share-frame  ({base / dt:.2f}x)  identical={same}",
                  flush=True)
    for s in scenes:
        s.close()


if __name__ == "__main__":
    main()
