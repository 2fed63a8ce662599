"""Project the N-GPU bench line from one GPU (the driver's 8-GPU run is the
measurement, this is a projection).

For N = 1, 2, 4, 8 every rank r of an N-rank `bench.py --gpus N` run is played alone on this
GPU (`bench.py --emulate-rank r`): the same pass plan (passes in flight, frames per pass, band
shares), the same rows (block-cyclic 8-row bands), no process group and no gather.  The N-GPU
step time is projected as the slowest rank's time per frame; the gather to rank 0 is reported
beside it as a bound, not measured (xGMI is not on this one-GPU box): rank 0 receives
(N - 1) / N of the float frame per frame over N - 1 links, at an assumed 50 GB/s effective per
link (the 153 GB/s link peak of MI355X_MICROARCH.md derated for a many-to-one gather), and the
gather of one pass overlaps the rendering of the other passes in flight.

usage: python tools/scale_projection.py [K=20] > gpurun_out/TAG/scale_projection.json
       (env WORLDS=1,2,4,8; progress on stderr)
"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
W, H = 1920, 1080
LINK_GBPS = 50.0


def run(args):
    t0 = time.time()
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                         timeout=300, cwd=ROOT)
    if out.returncode != 0:
        sys.stderr.write(out.stderr[-2000:])
        raise SystemExit(f"bench.py {' '.join(args)} failed: {out.returncode}")
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1]
    sys.stderr.write(f"  {' '.join(args)}: {time.time() - t0:.0f} s\n")
    sys.stderr.flush()
    return json.loads(line)


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    worlds = [int(x) for x in os.environ.get("WORLDS", "1,2,4,8").split(",")]
    common = ["--steps", str(k), "--warmup", "2"]
    res = {"k": k, "workload": "config 3, 1920x1080, depth 8 (bench.py defaults for each N)", "worlds": {}}
    base = None
    for n in worlds:
        if n == 1:
            d = run(common + ["--cpu-baseline", "0", "--seam-stats", "0", "--check", "0", "--count-frame", "0"])
            ranks = [d["ms_per_step"]]
            plan = {"passes_in_flight": d["config"]["passes_in_flight"], "frames_per_pass": d["config"]["frames_per_pass"],
                    "sub_bands": d["config"]["sub_bands"]}
        else:
            ranks, plan = [], None
            for r in range(n):
                d = run(common + ["--gpus", str(n), "--emulate-rank", str(r)])
                ranks.append(d["ms_per_step"])
                plan = {"passes_in_flight": d["passes_in_flight"], "frames_per_pass": d["frames_per_pass"],
                        "sub_bands": d["sub_bands"]}
        slowest = max(ranks)
        gather_ms = 0.0 if n == 1 else (W * H * 12 * (n - 1) / n) / ((n - 1) * LINK_GBPS * 1e9) * 1e3
        entry = {"rank_ms_per_frame": ranks, "projected_ms_per_frame": round(slowest, 4),
                 "projected_mpixels_per_s": round(W * H / (slowest / 1e3) / 1e6, 1),
                 "gather_bound_ms_per_frame": round(gather_ms, 4),
                 "projected_mpixels_per_s_if_gather_serialised": round(W * H / ((slowest + gather_ms) / 1e3) / 1e6, 1),
                 "plan": plan}
        if base is None:
            base = slowest
        entry["projected_speedup"] = round(base / slowest, 3)
        entry["projected_efficiency"] = round(base / slowest / n, 3)
        res["worlds"][str(n)] = entry
        sys.stderr.write(f"N = {n}: {json.dumps(entry)}\n")
        sys.stderr.flush()
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
