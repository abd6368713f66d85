#!/bin/bash
# Copy the roofline evidence of a scripts/gpu.sh call into profiles/<round>_roofline/:
# gpurun_out/<tag>/m_<name>/roofline.json -> <name>.json, its rocprofv3 kernel-trace summary ->
# <name>_kernel_stats.csv (names: the measure task's workload with '/' -> '_').
# usage: bash scripts/collect_roofline.sh <tag> <round>
set -e
tag=$1; round=$2
out=profiles/${round}_roofline
mkdir -p "$out"
for d in gpurun_out/$tag/m_*/; do
    name=$(basename "$d"); name=${name#m_}
    name=$(echo "$name" | sed 's/_--batch_/_batch/; s/[^A-Za-z0-9_]//g')
    [ -f "$d/roofline.json" ] || { echo "no record in $d"; continue; }
    cp "$d/roofline.json" "$out/$name.json"
    stats=$(find "$d/kt" -name "*kernel_stats.csv" | sort | head -n 1)
    [ -n "$stats" ] && cp "$stats" "$out/${name}_kernel_stats.csv"
    echo "$out/$name.json"
done
