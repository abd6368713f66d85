set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_step.sh 240 gpurun_out/smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit 1
scripts/gpu_step.sh 600 gpurun_out/pytest_gpu.log python -m pytest tests -m gpu -q -x -s || exit 1
scripts/gpu_step.sh 400 gpurun_out/bench1.log python bench.py --steps 2 --warmup 1 || exit 1
