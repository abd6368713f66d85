# Per-GPU throughput of the N-GPU shares of the headline workload on one GPU:
# a sample shard (256/N spp of every tile), a tile share (1/N of the tiles, 256 spp) and the
# hybrids (1/G of the tiles at 256 G/N spp). Efficiency = share rate / full-launch rate.
# usage: bash scripts/gpu_split.sh <tag> [extra bench args]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; shift
mkdir -p $O
run() {  # name steps "--opt k=v ..." bench-args...
  local name=$1 steps=$2 opts=$3; shift 3
  scripts/gpu_step.sh 120 $O/$name.log timeout -k 10 110 python bench.py --no-cpu-baseline --no-reference-order --steps $steps $opts "$@" || exit 1
  echo "$name $opts $* => $(grep -h '"value"' $O/$name.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["value"],1), d["ms_per_step"], d["roofline"]["avg_launch_ms"])')" | tee -a $O/summary.txt
}
run full 10 "" --spp 256 "$@"
for N in 2 4 8; do
  run n${N}_samples $((10*N)) "--as-rank-of $N" --spp 256 "$@"
  G=2
  while [ $G -le $N ]; do
    run n${N}_tiles${G} $((10*N)) "--as-rank-of $N --tile-groups $G" --spp 256 "$@"
    G=$((G*2))
  done
done
