# Round 4, call 2: configs 3-5 bench lines (+ roofline records) in the traversal bench.py picks,
# the 8-GPU configs' one-GPU shares (--as-rank-of 8) at their spec sample counts, and the N-share
# efficiencies of the headline (scripts/gpu_split.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
T=${TRAV:-near}
mkdir -p $O
run() {  # <name> <workload> <bench args...>
  local name=$1 wl=$2; shift 2
  scripts/gpu_step.sh 600 $O/bench_$name.log timeout -k 10 580 python bench.py --no-cpu-baseline --steps 2 --warmup 1 --traversal $T "$@" || return 1
  MEASURE_STEPS=1 MEASURE_WARMUP=0 bash scripts/gpu_measure.sh $O/$name "$wl" --traversal $T "$@" || return 1
}
run f2 "features2 path 1920x1080 512 samples/launch traversal=$T" --scene assets/scenes/features2/features2.json --width 1920 --height 1080 --spp 512 || exit 1
run b1 "bathroom1 path 1920x1080 1024 samples/launch traversal=$T" --scene assets/scenes/bathroom1/bathroom1.json --width 1920 --height 1080 --spp 1024 || exit 1
run ec "ecosys path 3840x2160 64 samples/launch traversal=$T" --scene assets/scenes/ecosys/ecosys.json --width 3840 --height 2160 --spp 64 || exit 1
scripts/gpu_step.sh 300 $O/b1_rank_of_8.log timeout -k 10 280 python bench.py --no-cpu-baseline --steps 1 --warmup 1 --traversal $T --scene assets/scenes/bathroom1/bathroom1.json --width 1920 --height 1080 --spp 1024 --as-rank-of 8 || exit 1
scripts/gpu_step.sh 300 $O/ec_rank_of_8.log timeout -k 10 280 python bench.py --no-cpu-baseline --steps 1 --warmup 0 --traversal $T --scene assets/scenes/ecosys/ecosys.json --width 3840 --height 2160 --spp 4096 --as-rank-of 8 || exit 1
bash scripts/gpu_split.sh $1/split || exit 1
