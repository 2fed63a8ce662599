#!/usr/bin/env python3
"""bench.py -- Mpixels/s of the MI355X render path on BASELINE.json's headline workload.

Workload (BASELINE.json configs[2]): synth(seed=2) = 600
spheres + 25 cubes (300 triangles) + 100 loose triangles + my_scene's 2 textured planes,
3 point lights; 1920x1080; depth 8 (reference semantics: primary + 7 secondary levels,
src/render.rs:43-45).  Synthetic scene, no dataset.

A step = one full frame: every rank renders its block-cyclic row bands with the HIP
level-synchronous pipeline (culling hierarchy + ordered ray queues), then (N > 1) the bands are gathered to rank 0 over RCCL and un-permuted.
The frame is fixed as N grows ("scaling": "strong").  Consecutive frames are rendered with
--inflight F frames in flight: F scene handles (one workspace each) on F HIP streams, so
the latency-bound tails of one frame's trace levels overlap the next frames' work, and
each pass renders --batch B frames in one pipeline (rt_render_bands_batch_async: the frame
index sits above every queue-key bit, so each frame's rays stay contiguous in the queues).  Every frame is rendered
and (N > 1) gathered in full; `pass_latency_ms` reports one pass's own duration beside
the throughput.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

Prints ONE JSON line on rank 0 with `roofline` (VALU f32, the bound of this path: see
DESIGN.md) and `cpu_baseline` (the CPU oracle -- a C++ restatement of the reference's
single-threaded render.rs -- timed on a bounded row sample, rank 0, N = 1 only).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402  (first: one HIP runtime per process, see rust_tracer_amd/abi.py)
import torch.distributed as dist  # noqa: E402

METRIC = "Mpixels/sec (primary+8 bounces) at 1920×1080; fraction of HBM roofline"
PEAK_F32_TFLOPS = 157.3      # MI355X FP32 vector peak (MI355X_MICROARCH.md)
PEAK_HBM_GBPS = 8000.0       # MI355X HBM3E peak
# f32 flops of each test the scans count (rt_scene_scan_ops; DESIGN.md "Roofline").
# Reference tests -- the ray-primitive tests Scene::intersect performs (SURVEY.md §8(d):
# sphere 57, triangle 52, cube 33 for the ray transform + 12 x 52, plane 49):
REF_TEST_FLOPS = {"dsph_pairs": 2 * 57, "gsph": 57, "tri_pairs": 2 * 52, "cube_boxes": 33, "cubes": 12 * 52,
                  "planes": 49}
# ... as the device executes them: a translate-scale sphere's pt_mul / vec3_mul drop their
# 24 x*0 terms (57 -> 33 flops, rt_scan.hpp sph_pair); the others as the reference's
EXEC_TEST_FLOPS = dict(REF_TEST_FLOPS, dsph_pairs=2 * 33)
# Hierarchy work the reference never performs: 12 FMAs = 24 flops per 2-wide child-box test,
# 12 per cube's object-space box test, 6 per grazing cone test, 48 per 8-normal grazing test
OVERHEAD_FLOPS = {"node_pairs": 24, "cube_box_slab": 12, "graze_cones": 6, "graze_normals": 48}
OVERHEAD_COUNTER = {"cube_box_slab": "cube_boxes"}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    # K = 64 timed frames by default: every slot runs a pass of 16 frames (K = 20 is one pass
    # of 5 per slot: 1051 - 1062 Mpixels/s; 2 passes of 8 per slot at K = 64: 1077 - 1095;
    # round-3 A/B run r3_steps, profiles/r3ab/, round-3 A/B run r3_steps2, profiles/r3ab/)
    p.add_argument("--steps", type=int, default=64)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--config", type=int, default=3, help="BASELINE config (2..5 synth scenes)")
    p.add_argument("--width", type=int, default=None, help="default: the config's (1920 / 3840)")
    p.add_argument("--height", type=int, default=None, help="default: the config's (1080 / 2160)")
    p.add_argument("--depth", type=int, default=None, help="default: the config's (4 / 8)")
    p.add_argument("--spp", type=int, default=None, help="samples per pixel (default: 64 for config 5, else 1)")
    p.add_argument("--seed", type=int, default=None, help="jitter seed (default: 3 for config 5)")
    p.add_argument("--band-rows", type=int, default=8)
    p.add_argument("--batch", type=int, default=None,
                   help="frames per pipeline pass (rt_render_bands_batch_async, <= 32; default: the timed "
                        "frames spread evenly over the slots, q = ceil(steps / inflight) per slot in equal "
                        "passes of up to 32 frames (rt_max_frames()) (a divisor of q where one is close) within 16 x 1080p of pixels "
                        "per pass and rank; 1 for spp > 1, whose samples are batched inside each pass)")
    p.add_argument("--sub-bands", type=int, default=None,
                   help="slots as groups of S band shares of the rank's rows, each rendering its rows of "
                        "every frame of its group's passes (N = 1: in place, rt_render_bands_direct_async; "
                        "N > 1: one gather per group pass): S times the frames per pass at the same rays in "
                        "flight.  Default (spp 1, N <= 4): the first S of (4, 2) -- (2, 4) at N = 4 -- that "
                        "divides the slots and whose groups still take the timed frames in one pass each "
                        "(ceil(K / (F / S)) <= rt_max_frames()): K = 20 gives 1 group x 4 shares x 20 frames "
                        "(N = 4: 2 groups x 2 shares x 10), K = 64 2 groups x 2 shares x 32 frames; otherwise 1")
    p.add_argument("--inflight", type=int, default=None,
                   help="frames in flight (F scene handles / HIP streams; default 4 = the box's hardware "
                        "queues per process; 3 from 4 ranks up when no band-share plan applies); 1 = one at a time")
    p.add_argument("--cpu-baseline", type=int, default=1, help="0 to skip the CPU oracle timing")
    p.add_argument("--cpu-threads", type=int, default=None,
                   help="threads of the multi-core CPU baseline (default: every core in the affinity mask)")
    p.add_argument("--cpu-rows-step", type=int, default=None,
                   help="CPU baseline renders every k-th row of the frame")
    p.add_argument("--backend", default="nccl", help="nccl (RCCL) or gloo (CPU rehearsal)")
    p.add_argument("--check", type=int, default=1,
                   help="rank 0 compares the timed passes' assembled frames with a single-launch render "
                        "(untimed, on the device; 0 to skip)")
    p.add_argument("--animate", type=int, default=1,
                   help="1 (default): every frame its own camera (an animation: the origin moves 0.01 along x per "
                        "frame, 64-frame cycle) -- no two frames of a batch share rays; 0: K renders of one camera "
                        "(the reference's bench -n loop); the frame check renders each frame's own camera")
    p.add_argument("--force-gather", type=int, default=0,
                   help="at N = 1 under torchrun: assemble every pass through the process group's gather "
                        "and the un-permute kernel anyway (a one-rank RCCL communicator; tests the N > 1 "
                        "exchange on one GPU)")
    p.add_argument("--emulate-rank", type=int, default=None,
                   help="one process on one GPU standing in for rank R of a --gpus N run: the same pass "
                        "plan and slots, no process group and no gather (tools/scale_projection.py projects "
                        "the N-GPU step from every rank's time); no checks, no extras")
    p.add_argument("--output", choices=("f32", "rgb8"), default="f32",
                   help="f32 frames (the parity contract), or Color::as_u8 bytes only: fused into the "
                        "render and gathered at 3 B per pixel (N > 1)")
    p.add_argument("--seam-stats", type=int, default=1,
                   help="N = 1: also time one frame at a time, rt_render with its host copy, the scene "
                        "build, and the depth-9 reading of 'primary+8 bounces' (untimed extras)")
    p.add_argument("--grid-share", type=int, default=None,
                   help="%% of the chip each pass's persistent trace grids take with passes in flight "
                        "(FramePipeline grid_share; default 50 for band-share groups, 75 otherwise)")
    p.add_argument("--forest", type=int, default=1,
                   help="N = 1, spp 1: also time the ray-forest path at the benchmark size (seam.forest: "
                        "rt_forest_create, render_forest, render_forest_filter after a one-shape edit)")
    p.add_argument("--count-frame", type=int, default=1,
                   help="0: skip the instrumented (counting) frame; roofline test counts are then null "
                        "(used by the rocprofv3 counter passes so they see only the default kernels)")
    p.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"),
                   help="rocprofv3 FETCH_SIZE/WRITE_SIZE summary for the render kernel")
    a = p.parse_args()
    # BASELINE.json configs: 2 = 1080p depth 4 (100 spheres); 3 = 1080p
    # depth 8 (1k primitives); 4 = 4K depth 8; 5 = 4K depth 8, 64 jittered spp, seed 3
    big = a.config in (4, 5)
    a.width = a.width or (3840 if big else 1920)
    a.height = a.height or (2160 if big else 1080)
    a.depth = a.depth if a.depth is not None else (4 if a.config == 2 else 8)
    a.spp = a.spp or (64 if a.config == 5 else 1)
    a.seed = a.seed if a.seed is not None else (3 if a.config == 5 else 0)
    if a.cpu_rows_step is None:  # ~86k pixel samples of CPU work (~6 s on config 3)
        a.cpu_rows_step = max(1, -(-a.width * a.height * a.spp // 86400))
    return a


def scene_label(config):
    if config == 2:
        return "synth seed 1 (100 spheres, 2 planes, 3 point lights)"
    return "synth seed 2 (600 spheres, 25 cubes, 100 triangles, 2 planes, 3 point lights)"


def oracle_rows_check(gpu, cpu, rows):
    """The GPU frame against the oracle on the rows the CPU baseline rendered (untimed;
    tolerance 1e-4 per channel, north_star): max |diff|, NaN agreement, bit-exact share."""
    import numpy as np
    g, c = gpu[rows].astype(np.float64), cpu[rows].astype(np.float64)
    nan_g, nan_c = np.isnan(g), np.isnan(c)
    d = np.abs(g - c)
    d[nan_g & nan_c] = 0.0
    same = np.array_equal(gpu[rows].view(np.uint32), cpu[rows].view(np.uint32))
    exact = float(np.mean(np.all(gpu[rows].view(np.uint32) == cpu[rows].view(np.uint32), axis=-1)))
    mx = float(np.nanmax(d)) if d.size else 0.0
    ok = bool(np.array_equal(nan_g, nan_c)) and mx <= 1e-4
    return {"rows": len(rows), "pixels": int(len(rows) * gpu.shape[1]), "max_abs_diff": mx,
            "nan_pattern_equal": bool(np.array_equal(nan_g, nan_c)), "bit_exact_pixel_frac": round(exact, 6),
            "all_bit_exact": bool(same), "tolerance": 1e-4, "ok": ok}


def cpu_baseline(args, desc, gpu_frame=None):
    """Single-threaded CPU oracle (the reference's algorithm, restated in C++) on every
    k-th row of the same frame.  Mpixels/s = rendered pixels / wall time.  With the GPU's
    single-launch frame, the rendered rows double as a parity check (`oracle_check`)."""
    from oracle.oracle import OracleScene
    o = OracleScene(desc)
    rows = range(0, args.height, args.cpu_rows_step)
    t0 = time.perf_counter()
    img, cnt = o.render(args.width, args.height, args.depth, rows=(0, args.height, args.cpu_rows_step),
                        threads=1, spp=args.spp, seed=args.seed)
    dt = time.perf_counter() - t0
    check = oracle_rows_check(gpu_frame, img, list(rows)) if gpu_frame is not None else None
    return {
        "oracle_check": check,
        "value": round(cnt["pixels"] / args.spp / dt / 1e6, 6),
        "unit": "Mpixels/s",
        "cores": 1,
        "kind": "port",
        "sample": f"{len(rows)} of {args.height} rows (every {args.cpu_rows_step}th) of the "
                  f"benchmark frame, {cnt['pixels'] // args.spp} pixels x {args.spp} spp, {dt:.1f} s, single thread "
                  f"(C++ restatement of src/render.rs, g++ -O2 -ffp-contract=off); "
                  f"host: {os.cpu_count()} logical CPUs",
        "seconds": round(dt, 2),
        "multicore": cpu_baseline_mt(args, o, label=f"every core this process may use: affinity mask "
                                                     f"{len(os.sched_getaffinity(0))} CPUs, cgroup CPU quota "
                                                     f"{cpu_quota_cores() or 'none'}"),
    }


def cpu_quota_cores():
    """CPUs' worth of time the cgroup grants this process (cgroup v2 cpu.max), or None."""
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            return max(1, int(int(quota) // int(period)))
    except Exception:
        pass
    return None


def cpu_threads(args):
    """Every host core this process may run on (OpenMP over all host
    cores): the affinity mask, capped by the cgroup's CPU quota (the GPU box shows 256 CPUs
    in the mask but grants 16 CPUs of time; more threads than that only contend)."""
    if args.cpu_threads:
        return args.cpu_threads
    n = len(os.sched_getaffinity(0))
    q = cpu_quota_cores()
    return min(n, q) if q else n


def cpu_baseline_mt(args, o, threads=None, label="every host core this process may use"):
    """The same oracle, rows dealt over T host threads (pixel-parallel over
    the host cores), on every k/T-th row: about the single-thread run's wall time."""
    threads = threads or cpu_threads(args)
    if threads <= 1:
        return None
    step = max(1, args.cpu_rows_step // threads)
    rows = range(0, args.height, step)
    t0 = time.perf_counter()
    _, cnt = o.render(args.width, args.height, args.depth, rows=(0, args.height, step), threads=threads,
                      spp=args.spp, seed=args.seed)
    dt = time.perf_counter() - t0
    return {
        "value": round(cnt["pixels"] / args.spp / dt / 1e6, 6),
        "unit": "Mpixels/s",
        "cores": threads,
        "sample": f"{len(rows)} of {args.height} rows (every {step}th), {cnt['pixels'] // args.spp} pixels x "
                  f"{args.spp} spp, {dt:.1f} s, {threads} threads ({label})",
        "seconds": round(dt, 2),
    }


def seam_stats(args, scene, pipe, tiler, dev):
    """Numbers of the drop-in seam beside the throughput headline (untimed extras, N = 1):
    - one frame at a time: the pipeline with nothing overlapping it (HIP events);
    - rt_render: the reference's render() seam (src/render.rs:31) with its device-to-host
      copy of the float frame, wall clock per call (main.rs:250-253 times render only);
    - the drop-in render() (the C++ mirror of render.rs:31) called repeatedly on one Scene:
      the first call builds the device scene, later ones reuse it (render_call_ms);
    - the scene build: rt_scene_create (host hierarchy, light buffers, grazing masks, upload)
      and rt_scene_clone (a second handle, device-to-device);
    - 'primary+8 bounces' read literally: depth 9 (reference depth 8 = primary + 7 levels,
      render.rs:43-45), frames in flight as the headline."""
    out = {}
    main = torch.cuda.current_stream(dev)
    # one frame at a time and the rt_render seam: the whole chip for the one pass
    # (FramePipeline gives each of its passes 75%)
    scene.set_grid_share(100)
    tiler.step()
    torch.cuda.synchronize()
    n1 = 5
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(main)
    for _ in range(n1):
        tiler.step()
    e1.record(main)
    torch.cuda.synchronize()
    # one pipeline pass over the whole frame (rt_render_bands_async)
    out["one_pass_ms"] = round(e0.elapsed_time(e1) / n1, 4)
    # one frame at a time through the stream-ordered seam (rt_render_frame_async: rt_render's
    # two band shares side by side, forked from and joined into this stream), checked bit for
    # bit against the single pass
    out["one_frame_at_a_time_ms"] = out["one_pass_ms"]
    if args.spp == 1 and args.output != "rgb8":
        try:  # an untimed extra: a failure here is reported, never the headline's end
            from rust_tracer_amd.dist import FrameTiler
            side = torch.cuda.Stream(dev)  # a created stream (rt_api.h: not the legacy null stream)
            with torch.cuda.stream(side):
                ft = FrameTiler(scene, args.width, args.height, args.depth, device=dev, split=True)
                for _ in range(3):  # the meeting row settles between synchronised calls
                    ft.step()
                    torch.cuda.synchronize()
                e0.record(side)
                for _ in range(n1):
                    ft.step()
                e1.record(side)
            torch.cuda.synchronize()
            scene.sync_status()
            out["one_frame_at_a_time_ms"] = round(e0.elapsed_time(e1) / n1, 4)
            out["one_frame_split_identical"] = bool(torch.equal(ft.frame, tiler.frame))
            del ft
        except Exception as e:  # noqa: BLE001
            out["one_frame_split_error"] = repr(e)[:200]
    out["one_frame_at_a_time_mpixels_per_s"] = round(args.width * args.height / (out["one_frame_at_a_time_ms"] / 1e3) / 1e6, 3)
    if args.spp == 1:
        scene.render(args.width, args.height, args.depth)  # sizes rt_render's frame buffers
        walls = []
        for _ in range(3):
            t0 = time.perf_counter()
            scene.render(args.width, args.height, args.depth)
            walls.append((time.perf_counter() - t0) * 1e3)
        out["rt_render_with_host_copy_ms"] = round(min(walls), 3)
        out["rt_render_with_host_copy_mpixels_per_s"] = round(args.width * args.height / (min(walls) / 1e3) / 1e6, 3)
        # the same seam into a page-locked caller buffer (rt_host_alloc: a RenderBuffer
        # allocated for DMA)
        from rust_tracer_amd import HostFrame
        hf = HostFrame(args.width, args.height)
        scene.render(args.width, args.height, args.depth, out=hf.array)
        walls = []
        for _ in range(3):
            t0 = time.perf_counter()
            scene.render(args.width, args.height, args.depth, out=hf.array)
            walls.append((time.perf_counter() - t0) * 1e3)
        hf.close()
        out["rt_render_pinned_host_copy_ms"] = round(min(walls), 3)
        # the drop-in render() itself (render.rs:31-38): the C++ host mirror's
        # render(camera, scene, buffer, depth) called again and again on ONE Scene -- the
        # reference's bench loop (main.rs:137-140, render_scene_basic :244-261).  The first call
        # builds the device scene; later calls find it unchanged (rt_scene_update) and cost a
        # frame: flatten + compare, rt_render, the frame into the RenderBuffer (pageable)
        if args.config in (2, 3, 4):
            try:  # an untimed extra
                from rust_tracer_amd import mirror_render_calls
                ms, up, _, _ = mirror_render_calls(args.config, args.width, args.height, args.depth, 7,
                                                   device=dev.index)
                later = sorted(ms[1:])
                out["render_call_first_ms"] = round(ms[0], 3)
                out["render_call_ms"] = round(later[len(later) // 2], 3)  # median of calls 2..7
                out["render_call_min_ms"] = round(later[0], 3)
                out["render_call_updates"] = up
            except Exception as e:  # noqa: BLE001
                out["render_call_error"] = repr(e)[:200]
    if args.spp == 1 and args.forest:
        try:  # an untimed extra
            out["forest"] = forest_stats(args, scene)
        except Exception as e:  # noqa: BLE001
            out["forest_error"] = repr(e)[:200]
    t0 = time.perf_counter()
    c = scene.clone(dev.index)
    out["scene_clone_ms"] = round((time.perf_counter() - t0) * 1e3, 2)
    c.close()
    # rt_scene_create again, the process's HIP runtime warm (the headline's scene_create_ms is
    # the process's first, with the runtime's first allocations and stream in it)
    from rust_tracer_amd import DeviceScene as _DS, SceneDesc as _SD
    _desc = _SD.synth_config(args.config)
    walls = []
    for _ in range(2):
        t0 = time.perf_counter()
        _s = _DS(_desc, device=dev.index)
        walls.append((time.perf_counter() - t0) * 1e3)
        _s.close()
    out["scene_create_warm_ms"] = round(min(walls), 2)
    if pipe.inflight > 1:
        scene.set_grid_share(pipe.grid_share)
    if args.spp == 1:
        # the other workload beside the headline: an animation (every frame its own camera,
        # the origin moving 0.01 per frame along x) when the headline repeats one camera, or
        # the repeated camera when the headline is the animation; frames in flight and frames
        # per pass as the headline
        from rust_tracer_amd import abi as _abi

        def cam(i):
            c = _abi.camera(args.width, args.height)
            if not args.animate:
                c.origin[0] = 0.01 * (i % 64)
            return c
        pipe.run(pipe.round_frames, cameras=cam)
        torch.cuda.synchronize()
        k = pipe.round_frames  # whole passes on every slot, as the headline's K frames
        e0.record(main)
        pipe.run(k, cameras=cam)
        e1.record(main)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / k
        tag = "identical_frames" if args.animate else "distinct_cameras"
        out[f"{tag}_ms_per_frame"] = round(ms, 4)
        out[f"{tag}_mpixels_per_s"] = round(args.width * args.height / (ms / 1e3) / 1e6, 3)
    if args.spp == 1 and args.depth == 8:
        for t in pipe.tilers:
            t.depth = 9
        pipe.run(pipe.round_frames)
        torch.cuda.synchronize()
        k = pipe.round_frames
        e0.record(main)
        pipe.run(k)
        e1.record(main)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / k
        for t in pipe.tilers:
            t.depth = args.depth
        out["depth9_ms_per_frame"] = round(ms, 4)
        out["depth9_mpixels_per_s"] = round(args.width * args.height / (ms / 1e3) / 1e6, 3)
    return out


def forest_stats(args, scene, edit_shapes=(20, 725)):
    """The ray-forest path at the benchmark size (render_tree.rs; the reference's bench -f mode,
    main.rs:170-204): generate_ray_forest once (rt_forest_create), render_forest (the whole
    forest shaded), and render_forest_filter after a one-shape material edit (the GUI's
    re-shade, gui.rs:163-236) -- for a small sphere (shape 20) and for the floor plane (shape
    725) -- wall clock of the C-ABI call (with its host copies of the float frame) and device
    time of its kernels (rt_forest_timings), plus the share of the trees each edit re-shades.
    Each edited material is restored afterwards."""
    import numpy as np
    w, h, depth = args.width, args.height, args.depth
    out = {}
    t0 = time.perf_counter()
    f = scene.forest(w, h, depth)
    out["forest_create_ms"] = round((time.perf_counter() - t0) * 1e3, 3)
    out["forest_build_device_ms"] = round(f.timings()["build_ms"], 4)
    img = f.render()
    walls, dev = [], []
    for _ in range(3):
        t0 = time.perf_counter()
        img = f.render()
        walls.append((time.perf_counter() - t0) * 1e3)
        dev.append(f.timings()["shade_ms"])
    out["forest_render_ms"] = round(min(walls), 3)
    out["forest_render_device_ms"] = round(min(dev), 4)
    edits = []
    base = scene.desc.editable()
    for shape in edit_shapes:
        if shape >= len(base.shapes):
            continue
        k = int(base.shapes[shape].material)
        old = base.materials[k]
        m = type(old).from_buffer_copy(old)  # same kind (rt_scene_set_material keeps kinds)
        m.reflectivity = float(np.float32(0.4 if old.reflectivity < 0.2 else 0.1))
        m.power = float(np.float32(old.power * 1.5))
        scene.set_material(k, m)
        try:
            walls, dev = [], []
            for _ in range(3):
                t0 = time.perf_counter()
                got = f.render_filter([shape], img)
                walls.append((time.perf_counter() - t0) * 1e3)
                dev.append(f.timings()["shade_ms"])
            n = f.trees_with(shape)
            edits.append({"shape": shape, "kind": ("sphere", "plane", "triangle", "cube")[base.shapes[shape].kind],
                          "filter_ms": round(min(walls), 3), "filter_device_ms": round(min(dev), 4),
                          "trees_reshaded": n, "tree_fraction": round(n / (w * h), 6),
                          "pixels_changed": int(np.count_nonzero((got != img).any(axis=2)))})
        finally:
            scene.set_material(k, old)
    out["filter"] = edits
    st = f.stats()
    out["forest_trees"] = st["num_trees"]
    out["forest_intersections"] = st["num_intersections"]
    f.close()
    out["note"] = ("wall: the C-ABI call incl. its host copies of the float frame (render: one device-to-host "
                   "copy; filter: the caller's frame up and back); device: HIP events around the forest_mark / "
                   "forest_shade_level kernels (build: trace + shadow passes)")
    return out


def test_flops(ops):
    """(reference tests at the reference's flop counts, as executed, hierarchy tests) of a
    scan_ops dict."""
    ref_f = sum(ops[k] * REF_TEST_FLOPS[k] for k in REF_TEST_FLOPS)
    exec_f = sum(ops[k] * EXEC_TEST_FLOPS[k] for k in EXEC_TEST_FLOPS)
    over_f = sum(ops[OVERHEAD_COUNTER.get(k, k)] * OVERHEAD_FLOPS[k] for k in OVERHEAD_FLOPS)
    return ref_f, exec_f, over_f


def kernel_roofline(args, pipe, reps=5):
    """Per-kernel roofline at one frame at a time (the regime whose kernel times are exclusive):
    one untimed pass of the whole frame counted twice (trace-kernel tests, shadow-kernel tests;
    Tune::count), then `reps` uncounted passes with every launch group bracketed by HIP events on
    the pass's stream (rt_scene_kernel_times).  achieved = the kernel's executed test flops per
    frame / its summed launch time per frame, against the 157.3 TFLOP/s f32 peak.  The same
    kernel's exclusive time in profiles/<tag>/kernel_trace_trace1.csv (rocprofv3, one frame at a
    time) is the cross-check (`exclusive_kernel_ms_per_frame`)."""
    whole = pipe.whole_tiler()
    sc = whole.scene
    sc.set_grid_share(100)
    out = {"regime": "one frame at a time (one pipeline pass of the whole frame on one stream, full-chip grids)"}
    try:
        flops = {}
        for kind in ("trace", "shadow"):
            sc.set_tuning(f"count={kind}")
            sc.set_scan_counting(True)
            sc.scan_ops(reset=True)
            whole.step()
            torch.cuda.synchronize()
            ops = sc.scan_ops(reset=True)
            sc.set_scan_counting(False)
            sc.set_tuning("count=all")
            ref_f, exec_f, over_f = test_flops(ops)
            flops[kind] = {"reference_tests_executed": exec_f, "hierarchy_tests": over_f,
                           "reference_tests_at_reference_flops": ref_f}
        whole.step()
        torch.cuda.synchronize()
        sc.set_kernel_timing(True)
        sc.kernel_times(reset=True)
        for _ in range(reps):
            whole.step()
        torch.cuda.synchronize()
        kt = sc.kernel_times(reset=True)
        sc.set_kernel_timing(False)
    finally:
        sc.set_grid_share(pipe.grid_share if pipe.inflight > 1 else 100)
    ms = {k: kt[k] / reps for k in sc.KERNEL_KINDS}
    for kind, name in (("trace", "trace_level_kernel"), ("shadow", "shadow_kernel")):
        f = flops[kind]["reference_tests_executed"] + flops[kind]["hierarchy_tests"]
        t = ms[kind]
        out[name] = {"flops_per_frame": f, "flops_breakdown": flops[kind], "ms_per_frame": round(t, 4),
                     "achieved_TFLOPs": round(f / (t / 1e3) / 1e12, 3) if t > 0 else None,
                     "frac": round(f / (t / 1e3) / 1e12 / PEAK_F32_TFLOPS, 4) if t > 0 else None}
    out["kernel_ms_per_frame"] = {k: round(v, 4) for k, v in ms.items()}
    out["launch_groups_per_frame"] = kt["launch_groups"] / reps
    out["frame_ms"] = round(sum(ms.values()), 4)
    return out


def load_traffic(path, workload, frames_per_pass):
    """The profile (tools/profile.sh -> profiles/pmc_traffic.json) of THESE sources and this
    pass size, or (None, why not): counters measured on other code are not replayed."""
    from rust_tracer_amd.provenance import sources_sha
    try:
        with open(path) as f:
            t = json.load(f)
    except Exception as e:  # noqa: BLE001
        return None, f"no profile ({e!r:.80})"
    if t.get("workload") != workload:
        return None, "the profile is of another workload"
    sha = sources_sha()
    if t.get("sources_sha") != sha:
        return None, f"profile of sources {t.get('sources_sha')}, these are {sha}: stale, not replayed"
    entry = (t.get("per_pass_size") or {}).get(str(frames_per_pass))
    if entry is None:
        return None, f"the profile has no {frames_per_pass}-frame pass entry"
    return dict(entry, profile=t.get("profile"), sources_sha=sha, commit=t.get("commit"),
                exclusive_kernel_ms_per_frame=t.get("exclusive_kernel_ms_per_frame"),
                exclusive_source=t.get("exclusive_source")), None


def main():
    args = parse()
    # stdout carries exactly the one JSON line: libraries that print banners to fd 1 (RCCL's
    # "RCCL version : ..." at communicator creation) write to stderr instead
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    emulate = args.emulate_rank is not None
    if emulate:  # rank R of an N-GPU run, alone on this GPU: no process group, no exchange
        assert world == 1 and 0 <= args.emulate_rank < args.gpus
        world, rank = args.gpus, args.emulate_rank
        args.check = args.seam_stats = args.cpu_baseline = args.count_frame = 0
    use_pg = (world > 1 and not emulate) or bool(args.force_gather)
    if use_pg:
        # one process per GPU; ranks share a device only in a --backend gloo rehearsal
        torch.cuda.set_device(local_rank % torch.cuda.device_count())
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", torch.cuda.current_device()))
        else:
            dist.init_process_group(args.backend)
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    import ctypes as C
    from rust_tracer_amd import DeviceScene, SceneDesc, abi, band_rows_per_rank
    from rust_tracer_amd.dist import FramePipeline

    desc = SceneDesc.synth_config(args.config)
    _d = desc.ptr().contents
    scene_soa_bytes = (_d.n_shapes * C.sizeof(abi.rt_shape) + _d.n_materials * C.sizeof(abi.rt_material)
                       + _d.n_lights * C.sizeof(abi.rt_light))
    torch.cuda.synchronize()
    t_sc = time.perf_counter()
    scene = DeviceScene(desc, device=dev.index)   # host build (hierarchy, light buffers) + upload
    scene_create_ms = (time.perf_counter() - t_sc) * 1e3
    # 4 passes in flight, as band-share groups where a group still takes its frames in one pass
    # per slot.  Round 4 (config 3, tools/subband_time.py, profiles/r4m/subband.txt): at K = 20,
    # 4 x 5 whole frames 1.977 ms per frame, 2 groups x 2 shares x 10 frames 1.929, 1 group x 4
    # shares x 20 frames 1.886; with the light-buffer tiers (profiles/r4k64/): K = 64: 1 / 2 / 4
    # shares 1237 - 1253 / 1264 - 1269 / 1259 - 1263 Mpixels/s.  At N > 1 every rank played
    # alone on one MI355X (tools/emulate_ab.py / tools/scale_projection.py, round 6, K = 20,
    # profiles/r6ab/r6k_plans.log, profiles/r6share/): N = 4: 2 groups x 2 shares x 10 frames,
    # slowest rank 0.453 ms per frame, against 0.470 for 3 x 7 whole shares (the same 34 bands
    # on rank 0).  N = 8: 3 x 7 whole shares -- a rank's share then holds 16 - 17 of the 135
    # 8-row bands; as 4 band shares (32 virtual ranks, rank-major) the 7 leftover bands all land
    # on ranks 0 - 1 (20 / 19 bands against 16): 0.334 ms on rank 0 against 0.280, and per band
    # the shares are no faster (0.0170 vs 0.0165 ms).  A short burst that no group plan holds in
    # one pass per slot takes 3 whole-share passes from N = 4 up (bigger passes amortise each
    # level's fixed latency; round 3, profiles/r3ab/r3_share2.txt)
    inflight = max(1, args.inflight or 4)
    if args.sub_bands is None:
        sub = 1
        if args.spp == 1 and world <= 4:
            from rust_tracer_amd import abi as _abi0
            mf = int(_abi0.lib().rt_max_frames())
            for cand in ((2, 4) if world == 4 else (4, 2)):
                if inflight % cand == 0 and -(-args.steps // (inflight // cand)) <= mf:
                    sub = cand
                    break
        if sub == 1 and args.inflight is None and world >= 4 and -(-args.steps // 4) < 8:
            inflight = 3
    else:
        sub = max(1, args.sub_bands)
    groups = max(1, inflight // sub)
    if args.batch is None:
        # The timed K frames are spread evenly over the F slots: q = ceil(K / F) frames per
        # slot, in r = ceil(q / cap) passes of B frames -- a divisor of q when one is near
        # ceil(q / r), so that every slot runs the same passes.  Up to rt_max_frames() (32)
        # frames per pass within 16 x 1080p of pixels per pass and rank (bounded workspace,
        # ~1.1 KB per pixel).
        # Round 2, ms per share-frame on one MI355X at K = 20 (tools/share_burst.py): N = 1:
        # B = 2 / 4 / 5 / 8: 2.46 / 2.51 / 2.31 / 2.36; N = 8: 0.533 / 0.464 / 0.389 / 0.381
        # (DESIGN.md "Frame batches")
        share = band_rows_per_rank(args.height, args.band_rows, world) * args.width // sub
        if args.spp > 1:
            cap = 1
        else:  # up to 32 frames (RT_MAX_FRAMES), within 16 x 1080p of pixels per pass and rank
            # (~37 GB of workspace per slot, ~150 GB for 4 slots of the 288 GB): at K = 64, 4 x 16
            # 1118 - 1126 vs 4 x 8 1077 - 1084 Mpixels/s (round-3 A/B run r3_steps2, profiles/r3ab/).  Passes in flight
            # come first: at K = 20 bigger passes lost (4 x 5: 1027 / 1033, 3 x 7: 1018 / 1017,
            # 2 x 10: 750, 1 x 16: 796)
            from rust_tracer_amd import abi as _abi1
            cap = max(1, min(int(_abi1.lib().rt_max_frames()), (16 * 1920 * 1088) // share))
        q = -(-args.steps // groups)
        r = -(-q // cap)
        b = -(-q // r)
        for d in range(b, 0, -1):
            if 2 * d < b:
                break
            if q % d == 0:
                b = d
                break
        args.batch = max(1, b)
    pipe = FramePipeline(scene, desc, args.width, args.height, args.depth, args.band_rows, rank, world, dev,
                         spp=args.spp, seed=args.seed, inflight=inflight, batch=args.batch,
                         rgb8=args.output == "rgb8", force_gather=bool(args.force_gather), sub_bands=sub,
                         emulate=emulate, grid_share=args.grid_share)
    batch = pipe.batch
    tilers = pipe.tilers
    tiler = tilers[0]
    main_stream = torch.cuda.current_stream(dev)

    def barrier():
        if use_pg:
            if args.backend == "nccl":
                dist.barrier(device_ids=[dev.index])
            else:
                dist.barrier()

    from rust_tracer_amd import abi as _abi

    def anim_cam(i):
        c = _abi.camera(args.width, args.height)
        c.origin[0] = 0.01 * (i % 64)
        return c

    def run_frames(n, lat=None):
        pipe.run(n, lat, cameras=anim_cam if args.animate else None)

    # slot set-up (untimed, like the scene upload): each slot's workspace is sized by its
    # first full pass
    run_frames(pipe.round_frames)
    run_frames(args.warmup)
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    # one instrumented pass (untimed) counts the scans' tests: the timed passes' size and
    # cameras (a batch's waves mix its frames' rays, so the tests a wave runs depend on the
    # pass), per frame; frames are deterministic, so the timed passes run these tests, uncounted
    ops = None
    ops_by_kernel = None
    if args.count_frame:
        # the same pass counted twice: the trace kernels' tests, then the shadow kernel's
        # (Tune::count), so that the flops split by kernel; their sum is every test of the pass
        counted = [t.scene for t in pipe.group_tilers(0)]  # one pass of group 0 (all its shares)
        ops, ops_by_kernel = {}, {}
        for kind in ("trace", "shadow"):
            for sc in counted:
                sc.set_tuning(f"count={kind}")
                sc.set_scan_counting(True)
                sc.scan_ops(reset=True)
            pipe.render_pass(0, [anim_cam(i) for i in range(batch)] if args.animate
                             else [_abi.camera(args.width, args.height)] * batch)
            torch.cuda.synchronize()
            part = {}
            for sc in counted:
                for k, v in sc.scan_ops().items():
                    part[k] = part.get(k, 0.0) + v / batch
                sc.set_scan_counting(False)
                sc.set_tuning("count=all")
            ops_by_kernel[kind] = part
            for k, v in part.items():
                ops[k] = ops.get(k, 0.0) + v
    # per-kernel rates at one frame at a time (exclusive kernel times, live HIP events)
    per_kernel = kernel_roofline(args, pipe) if (args.count_frame and world == 1 and args.spp == 1) else None
    pipe.zero_counters()

    lat = []  # one (start, end) event pair per pass
    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    t0 = time.perf_counter()
    ev[0].record(main_stream)
    run_frames(args.steps, lat)
    ev[1].record(main_stream)
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0

    # the timed region's HIP events (main stream, joined with every slot stream) / K: the
    # render pipeline's time per frame at steady state; one frame's own span beside it
    kernel_ms = ev[0].elapsed_time(ev[1]) / args.steps
    latency_ms = sum(a.elapsed_time(b) for a, b in lat) / max(1, len(lat))  # one pass of `batch` frames
    # each pass's (start, end) in ms from the timed region's start: how the passes overlap
    pass_spans = [[round(ev[0].elapsed_time(a), 3), round(ev[0].elapsed_time(b), 3)] for a, b in lat]
    cnt = pipe.counters.double()
    local_scans = float(cnt[0] + cnt[1]) / args.steps   # this rank's launch (for the roofline)
    red_dev = dev if args.backend == "nccl" else torch.device("cpu")
    stats = torch.tensor([elapsed, kernel_ms], dtype=torch.float64, device=red_dev)
    cnt = cnt.to(red_dev)
    if use_pg:
        dist.all_reduce(stats, op=dist.ReduceOp.MAX)
        dist.all_reduce(cnt, op=dist.ReduceOp.SUM)
    frame_check = None
    frame_checked = 0
    single_ref = None
    if args.check:
        # the timed passes' assembled frames of every slot (pipe.frames() first checks every
        # slot's overflow status), then a fresh single frame, against one rt_render_spp launch
        # of the whole frame -- bit for bit, compared on the device
        # copies: tiler.step() below re-renders into slot 0's buffers
        frames = [f.clone() for f in pipe.frames()]
        fcams = pipe.frame_cameras()
        whole = pipe.whole_tiler()
        single = whole.step()
        if rank == 0:
            frames.append(single)
            fcams.append(whole.last_cams[0])
        torch.cuda.synchronize()
        if rank == 0:
            refs = {}
            frame_check = True
            for f, c in zip(frames, fcams):
                key = tuple(c.origin)
                if key not in refs:
                    ref, _, _, ref8 = scene.render(args.width, args.height, args.depth, device=dev.index,
                                                   spp=args.spp, seed=args.seed, want_u8=args.output == "rgb8",
                                                   cam=c)
                    if single_ref is None and key == tuple(_abi.camera(args.width, args.height).origin):
                        single_ref = ref
                    refs[key] = (torch.from_numpy(ref8).to(dev) if args.output == "rgb8"
                                 else torch.from_numpy(ref).to(dev).view(torch.int32))
                r = refs[key]
                same = torch.equal(f, r) if args.output == "rgb8" else torch.equal(f.contiguous().view(torch.int32), r)
                frame_check = frame_check and bool(same)
            frame_checked = len(frames)
            if single_ref is None:  # the oracle row check needs Camera::new's frame
                single_ref = scene.render(args.width, args.height, args.depth, device=dev.index, spp=args.spp,
                                          seed=args.seed)[0]
    seam = seam_stats(args, scene, pipe, pipe.whole_tiler(), dev) if (args.seam_stats and world == 1) else None
    for t in tilers:  # every stream-ordered pass of the run, incl. the timed ones, was complete
        t.scene.sync_status()
    if seam is not None:
        seam["scene_create_ms"] = round(scene_create_ms, 2)
    # the whole job's time: the slowest rank's timed region (max over ranks)
    elapsed, kernel_ms_max = stats.tolist()
    node_rays, shadow_rays, pixels = cnt.tolist()

    if emulate:
        # one rank's share of the timed region (tools/scale_projection.py takes the max over ranks)
        sys.stdout.flush()
        os.write(json_fd, (json.dumps({"emulated": {"world": world, "rank": rank}, "steps": args.steps,
                                       "ms_per_step": round(elapsed / args.steps * 1e3, 4),
                                       "kernel_ms_per_step": round(kernel_ms, 4), "frames_per_pass": batch,
                                       "passes_in_flight": inflight, "sub_bands": sub,
                                       "pass_latency_ms": round(latency_ms, 4),
                                       "rows_per_rank": band_rows_per_rank(args.height, args.band_rows, world),
                                       "node_rays_per_step": node_rays / args.steps}) + "\n").encode())
        return
    if rank == 0:
        steps = args.steps
        mpix = args.width * args.height * steps / elapsed / 1e6
        # rank 0's launch: the tests its scans ran (culled) -- the reference's tests as the device
        # executes them plus the hierarchy's own tests; beside it the reference tests at the
        # reference's flop counts
        flops = None
        if ops:
            ref_f, exec_f, over_f = test_flops(ops)
            flops = {"reference_tests_at_reference_flops": ref_f, "reference_tests_executed": exec_f,
                     "hierarchy_tests": over_f,
                     "by_kernel": {("trace_level_kernel" if k == "trace" else "shadow_kernel"):
                                   dict(zip(("reference_tests_at_reference_flops", "reference_tests_executed",
                                             "hierarchy_tests"), test_flops(v)))
                                   for k, v in ops_by_kernel.items()}}
        per_launch_flops = flops["reference_tests_executed"] + flops["hierarchy_tests"] if flops else None
        achieved = per_launch_flops / (kernel_ms / 1e3) / 1e12 if ops else None
        # what the reference's linear scan would need for the same rays (F_alg per scan)
        brute_flops = local_scans * scene.flops_per_scan
        workload = (f"config{args.config}: {scene_label(args.config)}, {args.width}x{args.height}, "
                    f"depth {args.depth}" + (f", {args.spp} spp (jitter seed {args.seed})" if args.spp > 1 else ""))
        traffic, traffic_note = load_traffic(args.traffic_json, workload, batch if sub == 1 else f"{batch}/{sub}")
        roofline = {
            "bound": "valu",
            "achieved": round(achieved, 3) if ops else None,
            "peak": PEAK_F32_TFLOPS,
            "unit": "TFLOP/s",
            "frac": round(achieved / PEAK_F32_TFLOPS, 4) if ops else None,
            "traffic": traffic["bytes_per_launch"] if traffic else None,
            "kernel": ("one frame: trace_level_kernel per level + queue sorts + shadow_kernel + "
                       "combine_level_kernel per level"),
            "kernel_ms": round(kernel_ms, 4),
            "kernel_ms_is": (f"timed-region HIP events / steps ({inflight} passes of {batch} frames"
                             + (f", each 1/{sub} of the rows," if sub > 1 else "") + " in flight)"
                             if inflight * batch > 1 else "timed-region HIP events / steps"),
            "flops_per_launch": per_launch_flops,
            "flops_is": ("the counted tests as executed: reference tests (translate-scale spheres at 33 flops, "
                         "their x*0 terms dropped; SURVEY.md §8(d) counts otherwise) + hierarchy tests"),
            "flops_breakdown": flops,
            "frac_reference_tests_only": (round(flops["reference_tests_executed"] / (kernel_ms / 1e3) / 1e12 /
                                                PEAK_F32_TFLOPS, 4) if flops else None),
            "tests_per_launch": {k: round(v) for k, v in ops.items() if not k.startswith("cycles")} if ops else None,
            "cycles_per_launch": {k: round(v) for k, v in ops.items() if k.startswith("cycles")} if ops else None,
            # the dominant kernels' own rates, one frame at a time (live HIP events per launch
            # group, bench.py kernel_roofline); the headline's frac above is the whole frame's
            # executed tests over the frames-in-flight step time
            "per_kernel": per_kernel,
            "culling": {"hierarchy": scene.uses_bvh,
                        "linear_scan_flops_per_launch": brute_flops,
                        "linear_scan_equivalent_TFLOPs": round(brute_flops / (kernel_ms / 1e3) / 1e12, 3)},
            # structural ceilings of the algorithmic frac: the reference never
            # fuses a*b+c (-ffp-contract=off: no FMA), and unpacked f32 issues one lane op per
            # cycle where the 157.3 peak counts 2-wide packed FMA
            "ceilings": {"no_fma_contraction": 0.5, "unpacked": 0.25},
            # executed-instruction view beside the algorithmic frac: the profile's
            # SQ_INSTS_VALU per frame (wave instructions, packed ones counted once) over the
            # VALU issue slots of this frame time (1024 SIMDs x 2.4 GHz)
            "executed_valu": ({
                "sq_insts_valu_per_frame": traffic["sq_insts_valu_per_frame"],
                "issue_slots_per_frame": round(1024 * 2.4e9 * kernel_ms / 1e3),
                "issue_frac": round(traffic["sq_insts_valu_per_frame"] / (1024 * 2.4e9 * kernel_ms / 1e3), 4),
                "wave_cycle_shares": traffic.get("wave_cycle_shares"),
                "source": traffic.get("sq_source"),
            } if traffic and traffic.get("sq_insts_valu_per_frame") else None),
            "profile": ({"path": traffic["profile"], "sources_sha": traffic["sources_sha"],
                         "commit": traffic["commit"], "frames_per_pass": batch, "sub_bands": sub} if traffic else None),
            "traffic_note": traffic_note,
            # exclusive per-kernel times (one frame at a time, nothing overlapping) of the profile
            "exclusive_kernel_ms_per_frame": traffic.get("exclusive_kernel_ms_per_frame") if traffic else None,
            "hbm": {
                # B_alg = S_scene + W H 12 / world per launch (the float frame; S_scene
                # = the reference scene's own records: shapes, materials, lights as the C ABI
                # describes them), once per sample; the device scene's acceleration data (hierarchy,
                # light-buffer and shape-buffer record copies) is the builder's, reported apart
                "algorithmic_bytes_per_launch": round(args.spp * (scene_soa_bytes + args.width * args.height * 12 / world)),
                "scene_soa_bytes": scene_soa_bytes,
                "accel_bytes": scene.device_bytes,
                "achieved_GBps": round((traffic["bytes_per_launch"] / (kernel_ms / 1e3) / 1e9), 3)
                if traffic else None,
                "peak_GBps": PEAK_HBM_GBPS,
                "frac": round(traffic["bytes_per_launch"] / (kernel_ms / 1e3) / 1e9 / PEAK_HBM_GBPS, 6)
                if traffic else None,
                "frac_is": "the counters' HBM bytes (intermediate queue state included) over the step time",
                # SURVEY.md §8(d)'s algorithmic bytes over the step time: the useful-work fraction
                "frac_algorithmic": round(args.spp * (scene_soa_bytes + args.width * args.height * 12 / world)
                                          / (elapsed / steps) / 1e9 / PEAK_HBM_GBPS, 6),
                "traffic_over_algorithmic": (round(traffic["bytes_per_launch"] /
                                                   (args.spp * (scene_soa_bytes + args.width * args.height * 12 / world)), 1)
                                             if traffic else None),
            },
        }
        out = {
            "metric": METRIC,
            "value": round(mpix, 3),
            "unit": "Mpixels/s",
            "n_gpus": world,
            "steps": steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded scene, SURVEY.md §8(d))",
            "config": {
                "workload": workload,
                "width": args.width, "height": args.height, "depth": args.depth,
                "leaf_primitives": 100 if args.config == 2 else 1000,
                "spp": args.spp, "seed": args.seed, "band_rows": args.band_rows,
                "frames": ("animation: frame i's camera origin x = 0.01 (i mod 64)" if args.animate
                           else "K renders of Camera::new (the reference's bench -n loop, main.rs:137-140)"),
                "frames_in_flight": groups * batch, "passes_in_flight": inflight,
                "frames_per_pass": batch, "sub_bands": sub, "pass_latency_ms": round(latency_ms, 4),
                "pass_spans_ms": pass_spans,
                "output": args.output,
                "msamples_per_s": round(args.width * args.height * args.spp * steps / elapsed / 1e6, 3),
                "parallelism": f"row-bands x{world}" + (f" (x{sub} band shares per device)" if sub > 1 else "") + ((" + RCCL gather" if args.backend == "nccl"
                                                          else f" + {args.backend} gather (rehearsal)")
                                                         if world > 1 else ""),
                "workspace_bytes_per_slot": max(t.scene.workspace_bytes for t in tilers),
                "workspace_bytes_all_slots": sum(t.scene.workspace_bytes for t in tilers),
                "node_rays_per_frame": node_rays / steps,
                "shadow_rays_per_frame": shadow_rays / steps,
            },
            "roofline": roofline,
            "cpu_baseline": None,
        }
        if frame_check is not None:
            out["frame_check"] = frame_check
            out["frame_check_frames"] = frame_checked
        if seam is not None:
            out["seam"] = seam
        if world == 1 and args.cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args, desc, single_ref)
        sys.stdout.flush()
        os.write(json_fd, (json.dumps(out) + "\n").encode())
    if use_pg:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
