# Samples per work unit (the chunk option) on full launches and on the headline's 1/N shares.
# usage: bash scripts/gpu_chunk_full.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
run() {  # <name> <args...>
  local name=$1; shift
  scripts/gpu_step.sh 150 $O/$name.log timeout -k 10 140 python bench.py --no-cpu-baseline --no-reference-order "$@" || return 1
  echo "$name $* => $(grep -h '"value"' $O/$name.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"].get("avg_launch_ms"), d["roofline"]["launch"].split("chunk=")[1].split()[0])')" | tee -a $O/summary.txt
}
for rep in 1 2; do
  run cb_default_$rep --steps 10 || exit 1
  for c in 2 4 8 16 32; do run cb_chunk${c}_$rep --steps 10 --opt chunk=$c || exit 1; done
done
for n in 8 2; do
  st=$((10 * n))
  for c in 2 4 8; do run n${n}_chunk$c --steps $st --as-rank-of $n --opt chunk=$c || exit 1; done
done
run n2_default --steps 20 --as-rank-of 2 || exit 1
F2="--scene assets/scenes/features2/features2.json --width 1920 --height 1080 --spp 128 --steps 2 --warmup 1"
B1="--scene assets/scenes/bathroom1/bathroom1.json --width 1920 --height 1080 --spp 128 --steps 2 --warmup 1"
EC="--scene assets/scenes/ecosys/ecosys.json --width 3840 --height 2160 --spp 16 --steps 2 --warmup 1"
run f2_default $F2 || exit 1
for c in 4 8 16; do run f2_chunk$c $F2 --opt chunk=$c || exit 1; done
run b1_default $B1 || exit 1
for c in 4 8 16; do run b1_chunk$c $B1 --opt chunk=$c || exit 1; done
run ec_default $EC || exit 1
for c in 2 4; do run ec_chunk$c $EC --opt chunk=$c || exit 1; done
