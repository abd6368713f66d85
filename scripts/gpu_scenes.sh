set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_step.sh 900 gpurun_out/pytest_gpu_scenes.log python -m pytest tests -q -m gpu -s -rf --timeout 600 || exit 1
