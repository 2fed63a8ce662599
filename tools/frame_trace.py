"""Per-dispatch timeline of the last frame in a rocprofv3 --kernel-trace CSV.

usage: python tools/frame_trace.py DIR [first_kernel_substring=wave_init]
Prints start offset, duration, VGPRs and scratch of every dispatch from the last
occurrence of the first kernel on, then the per-kernel totals.
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(n):
    n = re.sub(r"\(.*", "", n)
    n = re.sub(r"<.*", "", n)
    return n.split("::")[-1][-34:]


def main():
    d = sys.argv[1]
    first = sys.argv[2] if len(sys.argv) > 2 else "wave_init"
    path = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
    last = rows[idx[-1]:]
    t0 = int(last[0]["Start_Timestamp"])
    tot = defaultdict(float)
    for r in last:
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        name = short(r["Kernel_Name"])
        tot[name] += dur
        print(f"{(int(r['Start_Timestamp']) - t0) / 1e3:9.1f} {dur:8.1f} us  {name:34s} "
              f"vgpr {r['VGPR_Count']} scratch {r['Scratch_Size']}")
    print("--- totals (us)")
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
        print(f"{v:9.1f}  {k}")


if __name__ == "__main__":
    main()
