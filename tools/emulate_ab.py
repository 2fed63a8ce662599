"""A/B of the N-GPU pass plan on one GPU: one rank of an N-rank bench.py run played alone
(bench.py --emulate-rank), for several plans, alternating, REPS times.

usage: python tools/emulate_ab.py N RANK PLAN [PLAN ...]
   PLAN: extra bench.py arguments joined by commas, e.g. --inflight=3,--batch=7 or
   --inflight=4,--sub-bands=4; "default" = bench.py's own plan for N
   (env K=20 timed frames, REPS=2)
Prints the rank's ms per frame for every run and the mean per plan."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    n, rank = int(sys.argv[1]), int(sys.argv[2])
    plans = [("" if p == "default" else p) for p in (sys.argv[3:] or ["default"])]
    k = os.environ.get("K", "20")
    reps = int(os.environ.get("REPS", "2"))
    res = {p: [] for p in plans}
    for _ in range(reps):
        for p in plans:
            args = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--emulate-rank", str(rank),
                    "--steps", k, "--warmup", "2"] + [a for a in p.split(",") if a]
            out = subprocess.run(args, capture_output=True, text=True, timeout=300, cwd=ROOT)
            if out.returncode != 0:
                sys.stderr.write(out.stderr[-1500:])
                raise SystemExit(f"failed: {p}")
            d = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1])
            res[p].append(d["ms_per_step"])
            print(f"N={n} rank={rank} [{p or 'default'}] ms/frame {d['ms_per_step']} (F={d['passes_in_flight']} "
                  f"B={d['frames_per_pass']} S={d['sub_bands']})", flush=True)
    for p, v in res.items():
        print(f"MEAN N={n} [{p or 'default'}] {sum(v) / len(v):.4f} ms/frame over {len(v)}", flush=True)


if __name__ == "__main__":
    main()
