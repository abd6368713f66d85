# Round 4, call 9: features2 near vs wide at its own spp (the auto rule), and two chunkings of the
# headline's 1/8 share.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
run() {  # <name> <args...>
  local name=$1; shift
  scripts/gpu_step.sh 300 $O/$name.log timeout -k 10 280 python bench.py --no-cpu-baseline --no-reference-order "$@" || return 1
  echo "$name $* => $(grep -h '"value"' $O/$name.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"].get("avg_launch_ms"), d["roofline"]["launch"].split("chunk=")[1].split()[0], d["config"]["traversal"])')" | tee -a $O/summary.txt
}
F2="--scene assets/scenes/features2/features2.json --width 1920 --height 1080 --spp 512 --steps 2 --warmup 1"
for rep in 1 2; do
  run f2_wide_$rep $F2 || exit 1
  run f2_near_$rep $F2 --traversal near || exit 1
done
run n8_c2 --steps 80 --as-rank-of 8 || exit 1
run n8_c3 --steps 80 --as-rank-of 8 --opt chunk=3 || exit 1
run n8_c2m1 --steps 80 --as-rank-of 8 --opt chunk=2 --opt chunk_min=1 || exit 1
run n8_c2_again --steps 80 --as-rank-of 8 || exit 1
