# Diagnostic stamps of the megakernel and WF bodies (JT_STAMPS build)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
mkdir -p $O
scripts/gpu_step.sh 120 $O/stamps_mk.log timeout -k 10 100 python scripts/stamps.py 32 || exit 1
for g in 5 8; do
JT_WF=1 JT_WF_GROUPS=$g scripts/gpu_step.sh 120 $O/stamps_wf_g$g.log timeout -k 10 100 python scripts/stamps_wf.py 32 || exit 1
done
cat $O/stamps_*.log
