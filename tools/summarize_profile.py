"""Turn a gpurun_out/<tag>/ profiling run (tools/gpu_profile.sh) into committed evidence:

  profiles/<tag>/kernel_stats.csv         rocprofv3 --kernel-trace --stats summary
  profiles/<tag>/kernel_trace_render.csv  per-dispatch durations of the render kernels
  profiles/<tag>/pmc_*.csv                the render kernels' PMC rows (SQ, FETCH_SIZE, WRITE_SIZE)
  profiles/<tag>/summary.md               what the numbers say
  profiles/pmc_traffic.json               HBM bytes per frame, read by bench.py (`traffic`)

usage: python tools/summarize_profile.py TAG
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RENDER = ("trace_level_kernel", "shadow_kernel", "combine_level_kernel", "wave_init_kernel", "render_kernel",
          "rocprim", "fillBufferAligned", "sort_count_kernel", "sort_scan_kernel", "sort_scatter_kernel")


def family(kernel_name):
    """short family name of a render-pipeline dispatch (None if not one)"""
    if ("trace_level_kernel<true" in kernel_name or "shadow_kernel<true, true>" in kernel_name
            or "shadow_kernel<false, true>" in kernel_name):
        return "instrumented variant (counted frame only)"
    for k in RENDER:
        if k in kernel_name:
            if k == "rocprim":
                return "queue sort (rocPRIM onesweep)"
            if k.startswith("sort_"):
                return "queue sort (device radix: " + k + ")"
            if k == "fillBufferAligned":
                return "sort lookback reset (fill)"
            return k
    return None


def trace_frames(keep):
    """per-frame ms of each render kernel family, and the timed frames' wall span per frame"""
    # kernel-trace: split the dispatches into frames at each wave_init (bench.py: slot
    # set-up + warm-up + one counted frame + timed frames); frames in flight (bench.py
    # --inflight) run on their own streams, so the split is per stream; a family's ms per
    # frame averages the frames it ran in (the counted frame runs the instrumented kernels)
    frame_sums = []
    open_frame = {}
    for r in sorted(keep, key=lambda r: int(r["Start_Timestamp"])):
        fam = family(r["Kernel_Name"])
        sid = r.get("Stream_Id", "0")
        if fam == "wave_init_kernel" or sid not in open_frame:
            open_frame[sid] = defaultdict(int)
            frame_sums.append(open_frame[sid])
        open_frame[sid][fam] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    # the timed frames: every dispatch after the counted (instrumented) frame; their wall
    # span / their number is what bench.py's timed-region HIP events measure per frame
    inst_end = max((int(r["End_Timestamp"]) for r in keep
                    if family(r["Kernel_Name"]).startswith("instrumented")), default=0)
    timed = [r for r in keep if int(r["Start_Timestamp"]) > inst_end]
    n_timed = sum(1 for r in timed if "wave_init_kernel" in r["Kernel_Name"])
    span_ms = ((max(int(r["End_Timestamp"]) for r in timed) - min(int(r["Start_Timestamp"]) for r in timed))
               / max(1, n_timed) / 1e6) if timed else 0.0
    fams = {f for fs in frame_sums for f in fs}
    fam_ms = {f: sum(fs[f] for fs in frame_sums if f in fs) / sum(1 for fs in frame_sums if f in fs) / 1e6
              for f in fams}
    timed_ms = sum(v for f, v in fam_ms.items() if not f.startswith("instrumented"))
    return len(frame_sums), fam_ms, timed_ms, n_timed, span_ms


def render_rows(path):
    rows = list(csv.DictReader(open(path)))
    return [r for r in rows if any(k in r["Kernel_Name"] for k in RENDER)]


def main(tag):
    src = os.path.join(ROOT, "gpurun_out", tag)
    dst = os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
    rows = list(csv.DictReader(open(os.path.join(src, "trace", "run_kernel_trace.csv"))))
    keep = [r for r in rows if any(k in r["Kernel_Name"] for k in RENDER)]
    fields = ["Dispatch_Id", "Kernel_Name", "Start_Timestamp", "End_Timestamp", "VGPR_Count", "SGPR_Count",
              "Scratch_Size", "Grid_Size_X", "Workgroup_Size_X"]
    with open(os.path.join(dst, "kernel_trace_render.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=fields + ["Duration_ns"])
        w.writeheader()
        for r in keep:
            d = {k: r[k] for k in fields}
            d["Kernel_Name"] = family(r["Kernel_Name"]) if "rocprim" in r["Kernel_Name"] else r["Kernel_Name"]
            d["Duration_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            w.writerow(d)
    bench = json.load(open(os.path.join(src, "bench.json")))
    fpp = int(bench["config"].get("frames_per_pass", 1))  # frames per pipeline pass (wave_init)
    pmc = {}
    pmc_frames = {}
    for p in ("pmc_sq", "pmc_fetch", "pmc_write"):
        rr = list(csv.DictReader(open(os.path.join(src, p, "run_counter_collection.csv"))))
        kept = [r for r in rr if any(k in r["Kernel_Name"] for k in RENDER)]
        with open(os.path.join(dst, p + ".csv"), "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
            w.writeheader()
            for r in kept:
                w.writerow({k: r[k] for k in ["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"]})
        agg = defaultdict(float)
        for r in kept:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
        # frames in this pass (bench.py --steps 4 --warmup 0 --inflight 1 --count-frame 0:
        # full passes of frames_per_pass frames, one wave_init each)
        inits = {r["Dispatch_Id"] for r in kept if "wave_init_kernel" in r["Kernel_Name"]}
        for k in agg:
            pmc_frames[k] = max(1, len(inits)) * fpp
        pmc.update({k: v / pmc_frames[k] for k, v in agg.items()})
    frames, fam_ms, timed_ms, n_timed, span_ms = trace_frames(keep)
    # passes -> frames (the instrumented counted frame is a one-frame pass)
    fam_ms = {f: (v if f.startswith("instrumented") else v / fpp) for f, v in fam_ms.items()}
    timed_ms /= fpp
    span_ms /= fpp
    n_timed *= fpp
    fetch_b = pmc.get("FETCH_SIZE", 0.0) * 1024
    write_b = pmc.get("WRITE_SIZE", 0.0) * 1024
    traffic = {
        "workload": bench["config"]["workload"],
        "bytes_per_launch": fetch_b * 2 + write_b,
        "launch": "one frame of the render pipeline (all trace + combine dispatches)",
        "fetch_size_bytes_raw": fetch_b,
        "fetch_size_bytes_x2": fetch_b * 2,
        "write_size_bytes": write_b,
        "correction": "FETCH_SIZE x 2 per MI355X_MICROARCH.md (gfx950 tallies 128-B requests at 64 B); "
                      "WRITE_SIZE as reported",
        "source": f"profiles/{tag}/pmc_fetch.csv, pmc_write.csv",
    }
    json.dump(traffic, open(os.path.join(ROOT, "profiles", "pmc_traffic.json"), "w"), indent=1)
    sq = {k: v for k, v in pmc.items() if k.startswith("SQ_")}
    frame_ms = bench["roofline"]["kernel_ms"]
    lines = [
        f"# Profile {tag}: {bench['config']['workload']}",
        "",
        f"bench.py: **{bench['value']} Mpixels/s**, {bench['ms_per_step']} ms/frame, render pipeline "
        f"{frame_ms} ms (HIP events), algorithmic {bench['roofline']['achieved']} TFLOP/s = "
        f"{bench['roofline']['frac']:.3f} of 157.3 (f32 vector peak).",
        "",
        f"## rocprofv3 --kernel-trace --stats ({frames} frames: warm-up + counted + timed; ms per frame)",
        "",
        "| kernel family | ms per frame |",
        "|---|---|",
    ] + [f"| {k} | {v:.3f} |" for k, v in sorted(fam_ms.items(), key=lambda x: -x[1])] + [
        "",
        f"Sum of the default kernels per frame: {timed_ms:.3f} ms (kernel-busy time; with "
        f"{bench['config'].get('frames_in_flight', 1)} frames in flight, {fpp} per pass, the frames' kernels "
        f"overlap).",
        "",
        f"Timed frames ({n_timed}) in the trace run: wall span per frame {span_ms:.3f} ms "
        f"(bench HIP events over the timed region: {frame_ms} ms per frame; the tracer's per-dispatch "
        f"bookkeeping stretches overlapped frames -- at --inflight 1 below the two agree).",
        "",
    ]
    t1 = os.path.join(src, "trace1", "run_kernel_trace.csv")
    b1 = os.path.join(src, "bench1.json")
    if os.path.exists(t1) and os.path.exists(b1):
        bench1 = json.load(open(b1))
        shutil.copy(os.path.join(src, "trace1", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats_inflight1.csv"))
        shutil.copy(b1, os.path.join(dst, "bench_inflight1.json"))
        f1, fam1, sum1, nt1, span1 = trace_frames(render_rows(t1))
        lines += [
            "## One frame at a time (bench.py --inflight 1; rocprofv3 kernel trace of the same command)",
            "",
            f"bench.py --inflight 1: {bench1['value']} Mpixels/s, render pipeline {bench1['roofline']['kernel_ms']} ms "
            f"per frame (HIP events).",
            "",
            "| kernel family | ms per frame |",
            "|---|---|",
        ] + [f"| {k} | {v:.3f} |" for k, v in sorted(fam1.items(), key=lambda x: -x[1])] + [
            "",
            f"Sum of the default kernels per frame: {sum1:.3f} ms; timed frames ({nt1}) wall span per frame "
            f"{span1:.3f} ms (bench HIP events: {bench1['roofline']['kernel_ms']} ms).",
            "",
        ]
    lines += [
        "## PMC (per frame, separate passes, render kernels only)",
        "",
        "| counter | value |",
        "|---|---|",
    ] + [f"| {k} | {v:.4g} |" for k, v in sorted(sq.items())] + [
        f"| FETCH_SIZE (KB) | {pmc.get('FETCH_SIZE', 0):.6g} |",
        f"| WRITE_SIZE (KB) | {pmc.get('WRITE_SIZE', 0):.6g} |",
        "",
        f"HBM traffic per frame: {traffic['bytes_per_launch'] / 1e6:.1f} MB (FETCH x2 + WRITE) -> "
        f"{traffic['bytes_per_launch'] / (frame_ms / 1e3) / 1e9:.1f} GB/s = "
        f"{traffic['bytes_per_launch'] / (frame_ms / 1e3) / 8e12 * 100:.3f} % of 8 TB/s.",
    ]
    if "SQ_INSTS_VALU" in sq and "SQ_WAVE_CYCLES" in sq:
        lines += [
            "",
            f"VALU instructions per frame: {sq['SQ_INSTS_VALU']:.3g}; SALU {sq.get('SQ_INSTS_SALU', 0):.3g}; "
            f"SMEM {sq.get('SQ_INSTS_SMEM', 0):.3g}.  Wave-cycle shares: active VALU "
            f"{sq.get('SQ_ACTIVE_INST_VALU', 0) / sq['SQ_WAVE_CYCLES']:.2f}, waiting (s_waitcnt) "
            f"{sq.get('SQ_WAIT_ANY', 0) / sq['SQ_WAVE_CYCLES']:.2f}, issue-stalled "
            f"{sq.get('SQ_WAIT_INST_ANY', 0) / sq['SQ_WAVE_CYCLES']:.2f}.",
        ]
    open(os.path.join(dst, "summary.md"), "w").write("\n".join(lines) + "\n")
    shutil.copy(os.path.join(src, "bench.json"), os.path.join(dst, "bench.json"))
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1])
