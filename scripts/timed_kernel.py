"""Name of the timed trace kernel in a rocprofv3 kernel_stats.csv: the COUNT=0 instance (4th
template argument) with the most total time, as "trace_kernel_lds<1, 16, false, 0, 0, false>".

usage: python scripts/timed_kernel.py <kt_kernel_stats.csv>
"""
import csv
import re
import sys

best = None
for r in csv.DictReader(open(sys.argv[1])):
    m = re.search(r"(trace_kernel\w*<\d+, \d+, (?:true|false), 0, \d+, (?:true|false)>)", r["Name"])
    if m and (best is None or float(r["TotalDurationNs"]) > best[0]):
        best = (float(r["TotalDurationNs"]), m.group(1))
if best is None:
    raise SystemExit("no COUNT=0 trace kernel in " + sys.argv[1])
print(best[1])
