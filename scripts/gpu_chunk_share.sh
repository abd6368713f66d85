# The headline's 1/N sample shares (--as-rank-of N) under chunk-table options: which chunking keeps a
# share's per-GPU rate closest to the full launch's.  usage: bash scripts/gpu_chunk_share.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
run() {  # <name> <args...>
  local name=$1; shift
  scripts/gpu_step.sh 120 $O/$name.log timeout -k 10 110 python bench.py --no-cpu-baseline --no-reference-order "$@" || return 1
  echo "$name $* => $(grep -h '"value"' $O/$name.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"].get("avg_launch_ms"))')" | tee -a $O/summary.txt
}
run full --steps 10 || exit 1
for n in 8 4; do
  st=$((10 * n))
  run n${n}_default --steps $st --as-rank-of $n || exit 1
  for o in chunk=4 chunk=16 chunk_min=2 chunk_min=4; do
    run n${n}_${o/=/} --steps $st --as-rank-of $n --opt $o || exit 1
  done
done
