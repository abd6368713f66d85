# GPU tests, the headline bench (config 2) and informational bench lines for configs 3-5.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tag=$1
mkdir -p gpurun_out/$tag
scripts/gpu_step.sh 1200 gpurun_out/$tag/pytest.log python -m pytest tests -q -m gpu -rf --timeout 900 || exit 1
scripts/gpu_step.sh 600 gpurun_out/$tag/bench_cb.log python bench.py --no-cpu-baseline || exit 1
scripts/gpu_step.sh 600 gpurun_out/$tag/bench_f2.log python bench.py --no-cpu-baseline --scene assets/scenes/features2/features2.json --width 1920 --height 1080 --spp 64 --steps 2 --warmup 1 || exit 1
scripts/gpu_step.sh 600 gpurun_out/$tag/bench_b1.log python bench.py --no-cpu-baseline --scene assets/scenes/bathroom1/bathroom1.json --width 1920 --height 1080 --spp 32 --steps 2 --warmup 1 || exit 1
scripts/gpu_step.sh 600 gpurun_out/$tag/bench_ec.log python bench.py --no-cpu-baseline --scene assets/scenes/ecosys/ecosys.json --width 3840 --height 2160 --spp 8 --steps 2 --warmup 1 || exit 1
