set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_step.sh 600 gpurun_out/pytest_gpu.log python -m pytest tests -m gpu -q -x -s || exit 1
scripts/gpu_step.sh 400 gpurun_out/bench2.log python bench.py --steps 3 --warmup 1 || exit 1
