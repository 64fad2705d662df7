"""Summarise a rocprofv3 --pmc CSV (per-kernel mean of each counter over dispatches)."""
import collections
import csv
import glob
import os
import sys

for d in sys.argv[1:]:
    hits = sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True))
    if not hits:
        print(d, "no counter_collection.csv")
        continue
    rows = list(csv.DictReader(open(hits[0])))
    agg = collections.defaultdict(list)
    info = {}
    for r in rows:
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][-60:]
        agg[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
        info[k] = (r["Grid_Size"], r["VGPR_Count"], r["Accum_VGPR_Count"], r["LDS_Block_Size"])
    print(d)
    for (k, c), v in sorted(agg.items()):
        if "elementwise" in k or "fill" in k.lower() or "normal" in k:
            continue
        print(f"  {k:60s} {c:24s} {sum(v) / len(v):14.0f}  (n={len(v)}) grid/vgpr/agpr/lds={info[k]}")
