# A/B of the previous build (libjtrace_hip_prev.so) and the current one: FT_NOIL ecosys kernel and
# first pops per kernel; chunk sizes on the headline. GPU suite first.
# usage: bash scripts/gpu_ab_noil.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
scripts/gpu_step.sh 600 $O/pytest.log python -u -m pytest tests -x -v -m gpu -rf --timeout 300 --timeout-method thread || exit 1
grep -q " passed" $O/pytest.log && ! grep -q -E "[0-9]+ failed" $O/pytest.log || { echo "GPU tests failed"; exit 1; }
run() {  # name lib env bench-args...
  local name=$1 lib=$2 envs=$3; shift 3
  local L=julia-raytracer_amd/build/libjtrace_hip.so
  [ "$lib" != base ] && L=julia-raytracer_amd/build/libjtrace_hip_$lib.so
  env JTRACE_LIB=$L $envs scripts/gpu_step.sh 200 $O/$name.log python bench.py --no-cpu-baseline --no-reference-order "$@" || exit 1
  echo "$name $lib $envs => $(grep -h '"value"' $O/$name.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["value"],1), d["ms_per_step"])')" | tee -a $O/summary.txt
}
EC="--steps 2 --warmup 1 --scene assets/scenes/ecosys/ecosys.json --width 3840 --height 2160 --spp 16"
F2="--steps 2 --warmup 1 --scene assets/scenes/features2/features2.json --width 1920 --height 1080 --spp 64"
B1="--steps 2 --warmup 1 --scene assets/scenes/bathroom1/bathroom1.json --width 1920 --height 1080 --spp 128"
for r in 1 2; do
  for lib in prev base; do run ec_${lib}_$r $lib "" $EC; run f2_${lib}_$r $lib "" $F2; run b1_${lib}_$r $lib "" $B1; run cb_${lib}_$r $lib "" --steps 10; done
done
for ch in 32 128; do run cb_c$ch base "JT_CHUNK=$ch" --steps 10; done
