# Round 4, call 2: the headline bench line + its roofline record on the final build, then configs
# 3-5 (traversal auto -> wide in HBM mode) bench lines + roofline records.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
scripts/gpu_step.sh 400 $O/bench.log python bench.py || exit 1
bash scripts/gpu_measure.sh $O/cb "cornellbox path 1280x720 256 samples/launch traversal=near" || exit 1
run() {  # <name> <workload> <bench args...>
  local name=$1 wl=$2; shift 2
  scripts/gpu_step.sh 600 $O/bench_$name.log timeout -k 10 580 python bench.py --no-cpu-baseline --steps 2 --warmup 1 "$@" || return 1
  MEASURE_STEPS=1 MEASURE_WARMUP=0 bash scripts/gpu_measure.sh $O/$name "$wl" "$@" || return 1
}
run f2 "features2 path 1920x1080 512 samples/launch traversal=wide" --scene assets/scenes/features2/features2.json --width 1920 --height 1080 --spp 512 || exit 1
run b1 "bathroom1 path 1920x1080 1024 samples/launch traversal=wide" --scene assets/scenes/bathroom1/bathroom1.json --width 1920 --height 1080 --spp 1024 || exit 1
run ec "ecosys path 3840x2160 64 samples/launch traversal=wide" --scene assets/scenes/ecosys/ecosys.json --width 3840 --height 2160 --spp 64 || exit 1
