"""Frame batches (rt_render_bands_batch_async): B frames per pipeline pass x F passes in
flight.  Checks every batched frame against rt_render_bands_async of its own camera, then
times ms per frame of one rank's share for world sizes 1..8 on one GPU.
usage: python tools/batch_time.py [config=3]   (env WORLDS, BATCHES, FLIGHTS, FRAMES)"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from rust_tracer_amd import DeviceScene, SceneDesc, abi, band_rows_per_rank  # noqa: E402


def cams_for(w, h, b):
    out = []
    for k in range(b):
        c = abi.camera(w, h)
        c.origin[0] = c.origin[0] + 0.05 * k   # a camera path: frame k moves 0.05 along x
        out.append(c)
    return out


def main():
    config = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    w, h, depth = 1920, 1080, 4 if config == 2 else 8
    desc = SceneDesc.synth_config(config)
    worlds = [int(x) for x in os.environ.get("WORLDS", "1,8").split(",")]
    batches = [int(x) for x in os.environ.get("BATCHES", "1,2,4").split(",")]
    flights = [int(x) for x in os.environ.get("FLIGHTS", "1,4").split(",")]
    nframes = int(os.environ.get("FRAMES", "32"))
    scenes = [DeviceScene(desc) for _ in range(max(flights))]
    streams = [torch.cuda.Stream() for _ in scenes]
    for world in worlds:
        rpr = band_rows_per_rank(h, 8, world)
        # parity: a batch of 4 frames with 4 cameras == 4 single-frame band renders
        cams = cams_for(w, h, 4)
        cnt = torch.zeros(3, dtype=torch.int64, device="cuda")
        one = torch.zeros((4, rpr, w, 3), dtype=torch.float32, device="cuda")
        st = torch.cuda.current_stream().cuda_stream
        for k in range(4):
            scenes[0].render_bands_async(cams[k], depth, 8, world - 1, world, one[k].data_ptr(), cnt.data_ptr(), st)
        c1 = cnt.clone()
        cnt.zero_()
        bat = torch.zeros((4, rpr, w, 3), dtype=torch.float32, device="cuda")
        scenes[0].render_bands_batch_async(cams, depth, 8, world - 1, world, bat.data_ptr(), cnt.data_ptr(), st)
        torch.cuda.synchronize()
        same = torch.equal(one.view(torch.int32), bat.view(torch.int32)) and torch.equal(c1, cnt)
        print(f"world {world}: batch of 4 cameras == 4 single renders: {same} (counters {cnt.tolist()})",
              flush=True)
        if not same:
            sys.exit(1)
        for b in batches:
            bufs = [torch.zeros((b, rpr, w, 3), dtype=torch.float32, device="cuda") for _ in scenes]
            cams = cams_for(w, h, b)
            for f in flights:
                for rep in range(2):
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    passes = nframes // b
                    for k in range(passes):
                        i = k % f
                        if b == 1:
                            scenes[i].render_bands_async(cams[0], depth, 8, 0, world, bufs[i].data_ptr(),
                                                         cnt.data_ptr(), streams[i].cuda_stream)
                        else:
                            scenes[i].render_bands_batch_async(cams, depth, 8, 0, world, bufs[i].data_ptr(),
                                                               cnt.data_ptr(), streams[i].cuda_stream)
                    torch.cuda.synchronize()
                    dt = (time.perf_counter() - t0) / (passes * b) * 1e3
                print(f"world {world} batch {b} in-flight {f}: {dt:.3f} ms per share-frame", flush=True)
    for s in scenes:
        s.close()


if __name__ == "__main__":
    main()
