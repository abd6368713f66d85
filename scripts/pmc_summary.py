"""Summarise rocprofv3 --pmc csv passes: per-dispatch averages for the trace kernel."""
import collections
import csv
import glob
import sys

root = sys.argv[1]
agg = collections.defaultdict(list)
meta = {}
for f in sorted(glob.glob(f"{root}/p*/p*_counter_collection.csv")):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if "trace_kernel" not in r["Kernel_Name"]:
            continue
        per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        meta = {k: r[k] for k in ("Kernel_Name", "VGPR_Count", "SGPR_Count", "LDS_Block_Size", "Scratch_Size")}
        meta["dur_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    for (d, c), v in per.items():
        agg[c].append(v)
print(meta)
for c in sorted(agg):
    v = agg[c]
    print(f"{c:40s} {sum(v) / len(v):.4g}  (n={len(v)})")
