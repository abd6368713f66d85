"""HBM traffic per launch of the timed trace kernel from two rocprofv3 --pmc passes (FETCH_SIZE
and WRITE_SIZE cannot share a pass on gfx950), corrected as MI355X_MICROARCH.md §HBM says:
FETCH_SIZE/WRITE_SIZE are KiB; FETCH_SIZE under-reports wide reads by 2x on gfx950, so the
read side is reported both as measured and doubled, and `traffic` uses the doubled figure.

usage: python scripts/pmc_traffic.py <fetch_csv_dir> <write_csv_dir> <kernel_substring> <workload> <out.json>
"""
import csv
import glob
import json
import sys


def per_dispatch(d, counter, kernel):
    vals = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter:
                key = (f, r["Dispatch_Id"])
                vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    return list(vals.values())


fetch_dir, write_dir, kernel, workload, out = sys.argv[1:6]
fk = per_dispatch(fetch_dir, "FETCH_SIZE", kernel)
wk = per_dispatch(write_dir, "WRITE_SIZE", kernel)
if not fk or not wk:
    raise SystemExit(f"no {kernel} dispatches with FETCH_SIZE/WRITE_SIZE under {fetch_dir} / {write_dir}")
fetch = sum(fk) / len(fk) * 1024.0
write = sum(wk) / len(wk) * 1024.0
res = {"workload": workload, "kernel": kernel, "dispatches": [len(fk), len(wk)],
       "fetch_bytes_measured": fetch, "fetch_bytes_corrected": 2.0 * fetch, "write_bytes": write,
       "traffic": 2.0 * fetch + write,
       "note": "per launch; FETCH_SIZE x2 (gfx950 wide-read correction) + WRITE_SIZE, KiB -> bytes"}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))
