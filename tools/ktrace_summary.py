"""Summarise a tools/ktrace.sh run: per-kernel ms per frame, per config (frames are
grouped by wave_init dispatches)."""
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
frames, cur = [], None
for r in rows:
    name = r["Kernel_Name"].split("(")[0].replace("rtdev::", "")
    if "rocprim" in name:  # library sort kernels: keep the stage name only
        import re
        m = re.findall(r"(radix_sort_\w+|merge_sort_\w+|onesweep_\w+|histogram\w*|scan\w*)", name)
        name = "sort:" + (m[0] if m else "other")
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    if "wave_init" in name:
        cur = collections.OrderedDict()
        frames.append(cur)
    if cur is None:
        continue
    key = name
    if key in cur:
        i = 1
        while f"{key}#{i}" in cur:
            i += 1
        key = f"{key}#{i}"
    cur[key] = d
for i, f in enumerate(frames):
    tot = sum(f.values())
    fam = collections.OrderedDict()
    for k, v in f.items():
        b = k.split("#")[0]
        fam[b] = fam.get(b, 0.0) + v
    print(f"frame {i}: total {tot:.2f} ms | " + " ".join(f"{k.replace('_kernel','')}={v:.2f}" for k, v in f.items()))
    print(f"   families: " + " ".join(f"{k.replace('_kernel','')}={v:.2f}" for k, v in fam.items()))
