# Diagnostic stamps of the megakernel (JT_STAMPS build)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
mkdir -p $O
scripts/gpu_step.sh 120 $O/stamps_mk.log timeout -k 10 100 python scripts/stamps.py 32 || exit 1
cat $O/stamps_*.log
