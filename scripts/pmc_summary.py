"""Summarise rocprofv3 --pmc csv passes: per-dispatch averages for the trace kernel.

usage: python scripts/pmc_summary.py <dir with p*/ passes> [kernel-name substring, default: the
production (COUNT=0) instances, i.e. names containing "trace_kernel" and not ", 1, " as COUNT]"""
import collections
import csv
import glob
import sys

root = sys.argv[1]
want = sys.argv[2] if len(sys.argv) > 2 else None


def match(name):
    if want is not None:
        return want in name
    if "trace_kernel" not in name:
        return False
    targs = name[name.index("<") + 1:name.index(">")].split(",")
    if "trace_kernel_wf" in name:  # <SAMPLER, COUNT, F, LDSM>
        return targs[1].strip() == "0"
    return len(targs) >= 4 and targs[3].strip() == "0"  # COUNT=0: the timed kernel, not the counting pass
agg = collections.defaultdict(list)
meta = {}
for f in sorted(glob.glob(f"{root}/p*/p*_counter_collection.csv")):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if not match(r["Kernel_Name"]):
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
