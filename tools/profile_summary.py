"""Summarise a tools/profile.sh run: per-kernel ms per frame (the driver's frames in flight, and
one frame at a time -- exclusive times), per-kernel HBM bytes per frame (FETCH_SIZE x 2 +
WRITE_SIZE, MI355X_MICROARCH.md's gfx950 correction) and SQ wave-cycle shares for passes of
1, 5 and 16 frames.  Copies the evidence to profiles/TAG/ and writes profiles/pmc_traffic.json
(what bench.py replays for roofline.traffic / executed_valu, keyed by the sources' hash and
the pass size).

usage: python tools/profile_summary.py TAG
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def fam(name):
    n = name.split("(")[0].replace("void ", "").replace("rtdev::", "")
    if n.startswith("trace_level_kernel<true") or "shadow_kernel<true, true>" in n or "shadow_kernel<false, true>" in n:
        return "instrumented (counted frame)"
    return n.split("<")[0]


def one(pattern):
    f = glob.glob(pattern, recursive=True)
    return f[0] if f else None


def trace_table(d, frames):
    f = one(os.path.join(d, "**", "*kernel_trace.csv"))
    if not f:
        return {}, None, []
    rows = list(csv.DictReader(open(f)))
    tot = defaultdict(int)
    n = defaultdict(int)
    for r in rows:
        k = fam(r["Kernel_Name"])
        tot[k] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        n[k] += 1
    return {k: v / 1e6 / frames for k, v in tot.items()}, f, rows


def pmc_table(d, counter):
    f = one(os.path.join(d, "**", "*counter_collection.csv"))
    if not f:
        return {}, None
    tot = defaultdict(float)
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == counter:
            tot[fam(r["Kernel_Name"])] += float(r["Counter_Value"])
    return tot, f


def main():
    tag = sys.argv[1]
    src = os.path.join(ROOT, "gpurun_out", tag)
    dst = os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    bench = json.load(open(os.path.join(src, "bench.json")))
    sha = open(os.path.join(src, "sources_sha.txt")).read().strip()
    for fn in ("bench.json", "cpu_max.txt", "sources_sha.txt"):
        if os.path.exists(os.path.join(src, fn)):
            shutil.copy(os.path.join(src, fn), os.path.join(dst, fn))
    out = [f"# Profile {tag}: {bench['config']['workload']}", "",
           f"Sources: `{sha}` (rust_tracer_amd/provenance.py).", ""]
    out.append(f"bench.py --steps 20 --warmup 5 (the driver's line): **{bench['value']} Mpixels/s** "
               f"({bench['ms_per_step']} ms/frame, {bench['config']['passes_in_flight']} passes x "
               f"{bench['config']['frames_per_pass']} frames in flight).")
    out.append("")
    # trace runs: slot set-up (inflight x batch frames) + warm-up + timed frames; the trace run
    # repeats bench.json's own arguments (tools/profile.sh)
    f4 = bench["config"]["frames_in_flight"]
    t4, f_t4, _ = trace_table(os.path.join(src, "trace"), bench["steps"] + bench["warmup"] + f4)
    t1, f_t1, _ = trace_table(os.path.join(src, "trace1"), 6 + 1 + 1)
    out += ["## rocprofv3 --kernel-trace (ms of kernel time per frame)", "",
            "In flight the passes overlap, so those times are not exclusive (they sum to more than a "
            "frame); one frame at a time they are.", "",
            f"| kernel | {f4} frames in flight ({bench['config']['passes_in_flight']} passes x "
            f"{bench['config']['frames_per_pass']}) | one frame at a time (exclusive) |", "|---|---|---|"]
    for k in sorted(set(t4) | set(t1), key=lambda k: -t1.get(k, 0)):
        out.append(f"| {k} | {t4.get(k, 0):.3f} | {t1.get(k, 0):.3f} |")
    out.append(f"| **sum** | {sum(t4.values()):.3f} | {sum(t1.values()):.3f} |")
    for name, f in (("trace", f_t4), ("trace1", f_t1)):
        if f:
            shutil.copy(f, os.path.join(dst, f"kernel_trace_{name}.csv"))
            st = one(os.path.join(src, name, "**", "*kernel_stats.csv"))
            if st:
                shutil.copy(st, os.path.join(dst, f"kernel_stats_{name}.csv"))
    import subprocess
    commit = os.environ.get("PROFILE_COMMIT") or subprocess.run(
        ["git", "-C", ROOT, "rev-parse", "--short=12", "HEAD"], capture_output=True, text=True).stdout.strip()
    from rust_tracer_amd.provenance import sources_sha
    if sources_sha() != sha:
        print(f"warning: the tree's sources ({sources_sha()}) are not the profiled ones ({sha})")
    # PMC passes: (suffix, frames per pass, frames rendered in the run: the slot's set-up pass + steps)
    # (b1: --steps 4 after a 1-frame set-up pass; bN: --steps N after an N-frame set-up pass)
    # (bNsS: N-frame passes over S band shares of the device, bench.py --sub-bands S: entry "N/S")
    import re
    runs = []
    for d in sorted(os.listdir(src)):
        m = re.fullmatch(r"pmc_fetch_b(\d+)(?:s(\d+))?", d)
        if m:
            n, s = int(m.group(1)), int(m.group(2) or 1)
            runs.append((d[len("pmc_fetch"):], n if s == 1 else f"{n}/{s}", 2 * n))
    runs.sort(key=lambda r: (isinstance(r[1], str), r[2]))
    result = {}
    for suf, per_pass, pmc_frames in runs:
        fe, f_fe = pmc_table(os.path.join(src, "pmc_fetch" + suf), "FETCH_SIZE")
        wr, f_wr = pmc_table(os.path.join(src, "pmc_write" + suf), "WRITE_SIZE")
        label = (f"{per_pass} frame{'s' if per_pass > 1 else ''} per pass" if isinstance(per_pass, int) else
                 f"{per_pass.split('/')[0]} frames per pass over {per_pass.split('/')[1]} band shares")
        out += ["", f"## HBM bytes per frame, {label} (MB; FETCH_SIZE x 2 + WRITE_SIZE, KB counters)", "",
                "| kernel | fetch x2 | write | total |", "|---|---|---|---|"]
        tf = tw = 0.0
        for k in sorted(set(fe) | set(wr), key=lambda k: -(2 * fe.get(k, 0) + wr.get(k, 0))):
            a, b = 2 * fe.get(k, 0) / 1024 / pmc_frames, wr.get(k, 0) / 1024 / pmc_frames
            tf += a
            tw += b
            out.append(f"| {k} | {a:.1f} | {b:.1f} | {a + b:.1f} |")
        out.append(f"| **all** | {tf:.1f} | {tw:.1f} | {tf + tw:.1f} |")
        for f, n in ((f_fe, f"pmc_fetch{suf}.csv"), (f_wr, f"pmc_write{suf}.csv")):
            if f:
                shutil.copy(f, os.path.join(dst, n))
        sq = {}
        per_kernel = []
        f_sq = one(os.path.join(src, "pmc_sq" + suf, "**", "*counter_collection.csv"))
        if f_sq:
            shutil.copy(f_sq, os.path.join(dst, f"pmc_sq{suf}.csv"))
            tot = defaultdict(float)
            byk = defaultdict(lambda: defaultdict(float))
            for r in csv.DictReader(open(f_sq)):
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
                byk[fam(r["Kernel_Name"])][r["Counter_Name"]] += float(r["Counter_Value"])
            sq = {k: v / pmc_frames for k, v in tot.items()}
            wc = sq.get("SQ_WAVE_CYCLES", 0) or 1
            out += ["", f"## SQ per frame, {label} (all render kernels)", "", "| counter | value |", "|---|---|"]
            for k, v in sorted(sq.items()):
                out.append(f"| {k} | {v:.4g} |")
            out.append("")
            out.append(f"Wave-cycle shares: VALU active {sq.get('SQ_ACTIVE_INST_VALU', 0) / wc:.3f}, "
                       f"waiting (s_waitcnt) {sq.get('SQ_WAIT_ANY', 0) / wc:.3f}, "
                       f"issue-stalled {sq.get('SQ_WAIT_INST_ANY', 0) / wc:.3f}.")
            out += ["", "| kernel | wave-cycles share | VALU active | s_waitcnt | issue-stalled |", "|---|---|---|---|---|"]
            for k, v in sorted(byk.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
                w = v.get("SQ_WAVE_CYCLES", 0)
                if w < 0.01 * tot.get("SQ_WAVE_CYCLES", 1):
                    continue
                out.append(f"| {k} | {w / tot['SQ_WAVE_CYCLES']:.3f} | {v.get('SQ_ACTIVE_INST_VALU', 0) / w:.3f} | "
                           f"{v.get('SQ_WAIT_ANY', 0) / w:.3f} | {v.get('SQ_WAIT_INST_ANY', 0) / w:.3f} |")
        traffic = (tf + tw) * 1024 * 1024
        wc = sq.get("SQ_WAVE_CYCLES", 0) or 1
        result[per_pass] = {"bytes_per_launch": traffic, "fetch_size_bytes_x2": tf * 1024 * 1024,
                            "write_size_bytes": tw * 1024 * 1024,
                            "sq_insts_valu_per_frame": sq.get("SQ_INSTS_VALU"),
                            "wave_cycle_shares": {"valu_active": round(sq.get("SQ_ACTIVE_INST_VALU", 0) / wc, 4),
                                                  "waiting_s_waitcnt": round(sq.get("SQ_WAIT_ANY", 0) / wc, 4),
                                                  "issue_stalled": round(sq.get("SQ_WAIT_INST_ANY", 0) / wc, 4)}
                            if sq else None,
                            "source": f"profiles/{tag}/pmc_fetch{suf}.csv, pmc_write{suf}.csv, pmc_sq{suf}.csv"}
    # bench.py picks the entry of its own pass size (the driver's K = 20: 5 frames per pass)
    doc = {"workload": bench["config"]["workload"], "sources_sha": sha, "commit": commit,
           "profile": f"profiles/{tag}",
           "launch": "one frame of the render pipeline (every kernel of the frame), per frame of an "
                     "N-frame pass (per_pass_size[N])",
           "correction": "FETCH_SIZE x 2 per MI355X_MICROARCH.md (gfx950 tallies 128-B requests at 64 B); "
                         "WRITE_SIZE as reported",
           "exclusive_kernel_ms_per_frame": {k: round(v, 4) for k, v in sorted(t1.items(), key=lambda kv: -kv[1])},
           "exclusive_source": f"profiles/{tag}/kernel_trace_trace1.csv (one frame at a time)",
           "in_flight_kernel_ms_per_frame": {k: round(v, 4) for k, v in sorted(t4.items(), key=lambda kv: -kv[1])},
           "per_pass_size": {str(k): v for k, v in result.items()}}
    json.dump(doc, open(os.path.join(ROOT, "profiles", "pmc_traffic.json"), "w"), indent=1)
    open(os.path.join(dst, "summary.md"), "w").write("\n".join(out) + "\n")
    print("\n".join(out))


if __name__ == "__main__":
    main()
