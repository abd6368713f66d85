# Round 4, call 11: the GPU suite on per-instance root records (JT_WIDE_IROOT) and the depth rule
# of auto; A/B of the instance-root copies and the two direct child-word variants on the deep
# HBM-mode scenes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
scripts/gpu_step.sh 600 $O/tests.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" $O/tests.log && ! grep -q "failed\|error" $O/tests.log || { echo "GPU tests not green: stopping"; exit 1; }
AB_SCENES="b1 ec" AB_B1_SPP=128 AB_EC_SPP=16 bash scripts/gpu_lib_ab.sh $1/ab base noiroot direct2 direct1 || exit 1
