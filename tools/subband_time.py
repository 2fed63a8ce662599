"""K animation frames (bench.py's cameras) over 4 slots, split two ways (ms per frame):
  frames: slot i renders frames [i*K/4, (i+1)*K/4) whole (bench.py today);
  bands S: slot i renders sub-band i % S (rank i % S of a world of S) of frame group i // S,
           i.e. each pass mixes S times as many frames, each a 1/S share.
WORLD=W (default 1): rank 0's share of a W-rank run instead (slots render rank 0 of W, or
virtual rank j of W*S -- the rank's S sub-shares); F=slots (default 4).  Times are per
frame of the share.
usage: python tools/subband_time.py [K] [reps]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rust_tracer_amd import DeviceScene, SceneDesc, abi  # noqa: E402
from rust_tracer_amd.dist import FrameTiler  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
REPS = int(sys.argv[2]) if len(sys.argv) > 2 else 5
W, H, DEPTH = 1920, 1080, 8
F = int(os.environ.get("F", "4"))
WORLD = int(os.environ.get("WORLD", "1"))
dev = torch.device("cuda", 0)
scene = DeviceScene(SceneDesc.synth_config(3))
scenes = [scene] + [scene.clone(0) for _ in range(F - 1)]
for s in scenes:
    s.set_grid_share(75)
streams = [torch.cuda.Stream(device=dev) for _ in range(F)]


def cam(i):
    c = abi.camera(W, H)
    c.origin[0] = 0.01 * (i % 64)
    return c


def plan(mode):
    """[(slot, rank, world, [frame indices])] passes in enqueue order"""
    if mode == "frames":
        q = -(-K // F)
        return [(i, 0, WORLD, list(range(i * q, min(K, (i + 1) * q)))) for i in range(F)]
    S = int(mode[5:])
    groups = F // S
    q = -(-K // groups)
    out = []
    for g in range(groups):
        fr = list(range(g * q, min(K, (g + 1) * q)))
        mf = int(abi.lib().rt_max_frames())
        chunks = [fr[k:k + mf] for k in range(0, len(fr), mf)]
        for ch in chunks:
            for j in range(S):
                out.append((g * S + j, j, WORLD * S, ch))
    return out


tilers = {}


def tiler(slot, rank, world):
    key = (slot, rank, world)
    if key not in tilers:
        tilers[key] = FrameTiler(scenes[slot], W, H, DEPTH, 8, rank, world, dev,
                                  batch=int(abi.lib().rt_max_frames()))
    return tilers[key]


def run(mode, base):
    main = torch.cuda.current_stream(dev)
    for s in streams:
        s.wait_stream(main)
    for slot, rank, world, fr in plan(mode):
        with torch.cuda.stream(streams[slot]):
            tiler(slot, rank, world).render_local(len(fr), [cam(base + f) for f in fr])
    for s in streams:
        main.wait_stream(s)


modes = (os.environ.get("MODES") or "frames bands2 bands4").split()
for m in modes:  # workspaces sized, kernels loaded
    run(m, 0)
    run(m, 0)
torch.cuda.synchronize()
res = {m: [] for m in modes}
base = 0
for r in range(REPS):
    for m in modes:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(m, base)
        torch.cuda.synchronize()
        res[m].append((time.perf_counter() - t0) * 1e3 / K)
        base += K
for m in modes:
    v = sorted(res[m])
    print(f"K={K} WORLD={WORLD} F={F} {m:7s} ms/frame median {v[len(v) // 2]:.4f} min {v[0]:.4f} "
          f"-> {W * H / (v[len(v) // 2] / 1e3) / 1e6:.1f} Mpixels/s  all {[round(x, 3) for x in res[m]]}")
for s in scenes:
    s.sync_status()
