set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_step.sh 300 gpurun_out/stamps_now.log python scripts/stamps.py 64 || exit 1
scripts/gpu_step.sh 300 gpurun_out/stamps_now_naive.log python scripts/stamps.py 64 naive || exit 1
