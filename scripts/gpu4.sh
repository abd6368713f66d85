set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for w in 32 48; do
  JT_WAIT_LANES=$w scripts/gpu_step.sh 300 gpurun_out/stamps_lds_w$w.log python scripts/stamps.py 64 || exit 1
done
