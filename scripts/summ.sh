#!/bin/bash
# one line per bench log: value, ms/step, batch, calls, launch ms, options, image check, streams
for f in "$@"; do
  printf '%s: ' "$(basename "$f")"
  grep -h '"value"' "$f" | python3 -c '
import sys,json
d=json.loads(sys.stdin.read()); r=d["roofline"]
print(d["value"], d["ms_per_step"], "batch", d["config"].get("batch"), "launch_ms", r["avg_launch_ms"], d.get("options"), (d["image_check"] or {}).get("ok"), [t for t in r["launch"].split() if t.startswith("streams")])' 2>/dev/null || tail -1 "$f"
done
