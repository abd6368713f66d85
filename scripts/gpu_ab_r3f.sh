# A/B after inline light chains: first-pop count and node-repeat builds, the gate on features2 /
# bathroom1 around the new defaults, and the strong-scaling shard sizes (256/N spp per GPU).
# usage: bash scripts/gpu_ab_r3f.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
run() {  # name lib env bench-args...
  local name=$1 lib=$2 envs=$3; shift 3
  local L=julia-raytracer_amd/build/libjtrace_hip.so
  [ "$lib" != base ] && L=julia-raytracer_amd/build/libjtrace_hip_$lib.so
  env JTRACE_LIB=$L $envs scripts/gpu_step.sh 200 $O/$name.log python bench.py --no-cpu-baseline --no-reference-order "$@" || exit 1
  echo "$name $lib $envs => $(grep -h '"value"' $O/$name.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["value"],1), d["ms_per_step"])')" | tee -a $O/summary.txt
}
F2="--steps 2 --warmup 1 --scene assets/scenes/features2/features2.json --width 1920 --height 1080 --spp 64"
B1="--steps 2 --warmup 1 --scene assets/scenes/bathroom1/bathroom1.json --width 1920 --height 1080 --spp 128"
for r in 1 2; do
  for lib in base fp2 nr3 nr5; do run cb_${lib}_$r $lib "" --steps 10; done
  for lib in base fp2; do run f2_${lib}_$r $lib "" $F2; run b1_${lib}_$r $lib "" $B1; done
done
for w in 60 64; do run f2_w$w base "JT_WAIT_LANES=$w" $F2; done
for w in 36 44; do run b1_w$w base "JT_WAIT_LANES=$w" $B1; done
run s256 base "" --steps 10 --spp 256
run s128 base "" --steps 20 --spp 128
run s64 base "" --steps 40 --spp 64
run s32 base "" --steps 80 --spp 32
run s32_c16 base "JT_CHUNK=16" --steps 80 --spp 32
run s32_c4 base "JT_CHUNK=4" --steps 80 --spp 32
