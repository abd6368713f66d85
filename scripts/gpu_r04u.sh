# Round 4: the shading gate on the headline's 1/8 and 1/4 sample shares (short launches).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
run() {  # <name> <args...>
  local name=$1; shift
  scripts/gpu_step.sh 200 $O/$name.log timeout -k 10 180 python bench.py --no-cpu-baseline --no-reference-order "$@" || return 1
  echo "$name $* => $(grep -h '"value"' $O/$name.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"])')" | tee -a $O/summary.txt
}
for rep in 1 2; do
  for w in 56 48 52 60; do run n8_w${w}_$rep --steps 80 --as-rank-of 8 --opt wait_lanes=$w || exit 1; done
  for w in 56 52 60; do run n4_w${w}_$rep --steps 40 --as-rank-of 4 --opt wait_lanes=$w || exit 1; done
done
