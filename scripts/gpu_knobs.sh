# Sweep of runtime knobs (env "NAME=VALUE ..." per run; "-" = defaults) on the headline workload,
# or on the one BENCH_ARGS names (e.g. BENCH_ARGS="--scene ... --width ... --spp ...")
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; shift
mkdir -p $O
i=0
for cfg in "$@"; do
  i=$((i+1))
  if [ "$cfg" = "-" ]; then envs=""; else envs="$cfg"; fi
  env $envs scripts/gpu_step.sh 120 $O/k$i.log timeout -k 10 100 python bench.py --no-cpu-baseline --steps 3 $BENCH_ARGS || exit 1
  echo "$cfg => $(grep -h '"value"' $O/k$i.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"])')" | tee -a $O/summary.txt
done
