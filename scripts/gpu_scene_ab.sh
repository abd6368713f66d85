# GPU tests, then the large-scene bench lines (configs 3-5, reduced spp) under each setting given
# ("VAR=value[,VAR2=value]" or "default").  usage: bash scripts/gpu_scene_ab.sh <tag> [setting ...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tag=$1; shift
mkdir -p gpurun_out/$tag
if [ -z "$NO_TESTS" ]; then
  scripts/gpu_step.sh 900 gpurun_out/$tag/pytest.log python -m pytest tests -q -m gpu -rf --timeout 600 || exit 1
fi
F2="--scene assets/scenes/features2/features2.json --width 1920 --height 1080 --spp 64"
B1="--scene assets/scenes/bathroom1/bathroom1.json --width 1920 --height 1080 --spp 32"
EC="--scene assets/scenes/ecosys/ecosys.json --width 3840 --height 2160 --spp 8"
for cfg in "$@"; do
  for sc in F2 B1 EC; do
    ( if [ "$cfg" != default ]; then IFS=','; for kv in $cfg; do export "$kv"; done; unset IFS; fi
      scripts/gpu_step.sh 300 gpurun_out/$tag/bench_${sc}_$(echo $cfg | tr ',=/' '_-_').log python bench.py --no-cpu-baseline ${!sc} --steps 2 --warmup 1 ) || exit 1
  done
done
