# A/B after inline light chains: the primitive-favouring vote bias (JT_VOTE_P 2 / 5 vs 3) and the
# mesh kernels' pops per node iteration (JT_NODE_REPEAT 2 / 4 vs 3).
# usage: bash scripts/gpu_ab_knobs3.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
run() {  # name lib bench-args...
  local name=$1 lib=$2; shift 2
  local L=julia-raytracer_amd/build/libjtrace_hip.so
  [ "$lib" != base ] && L=julia-raytracer_amd/build/libjtrace_hip_$lib.so
  JTRACE_LIB=$L scripts/gpu_step.sh 200 $O/$name.log python bench.py --no-cpu-baseline --no-reference-order "$@" || exit 1
  echo "$name $lib => $(grep -h '"value"' $O/$name.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["value"],1), d["ms_per_step"])')" | tee -a $O/summary.txt
}
F2="--steps 2 --warmup 1 --scene assets/scenes/features2/features2.json --width 1920 --height 1080 --spp 64"
B1="--steps 2 --warmup 1 --scene assets/scenes/bathroom1/bathroom1.json --width 1920 --height 1080 --spp 128"
EC="--steps 2 --warmup 1 --scene assets/scenes/ecosys/ecosys.json --width 3840 --height 2160 --spp 16"
for r in 1 2; do
  for lib in base vp2 vp5; do run cb_${lib}_$r $lib --steps 10; done
  for lib in base vp2 vp5 nrm2 nrm4; do run f2_${lib}_$r $lib $F2; run b1_${lib}_$r $lib $B1; run ec_${lib}_$r $lib $EC; done
done
