# Round 4, call 10: the GPU suite on the wide traversal's direct child-word entries
# (JT_WIDE_DIRECT), their A/B on the HBM-mode scenes, features2 near vs wide again.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
scripts/gpu_step.sh 600 $O/tests.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" $O/tests.log && ! grep -q "failed\|error" $O/tests.log || { echo "GPU tests not green: stopping"; exit 1; }
AB_SCENES="b1 ec f2" AB_F2_SPP=128 AB_B1_SPP=128 AB_EC_SPP=16 bash scripts/gpu_lib_ab.sh $1/ab_direct base nodirect || exit 1
AB_SCENES="f2" AB_F2_SPP=512 AB_ARGS="--traversal near" bash scripts/gpu_lib_ab.sh $1/f2_near base || exit 1
AB_SCENES="f2" AB_F2_SPP=512 bash scripts/gpu_lib_ab.sh $1/f2_wide base || exit 1
