# Round 4, call 4: GPU parity on the register-held next entry (JT_BIN_NXT), the headline bench line
# (with its CPU baseline), an A/B of JT_BIN_NXT on the binary-order kernels, then the 8-GPU
# configs' one-GPU shares (after an A/B of the parked path weight, JT_PARK_W) and the headline's N-share efficiencies.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
scripts/gpu_step.sh 600 $O/tests.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" $O/tests.log && ! grep -q "failed\|error" $O/tests.log || { echo "GPU tests not green: stopping"; exit 1; }
scripts/gpu_step.sh 400 $O/bench.log python bench.py || exit 1
AB_SCENES="cb" bash scripts/gpu_lib_ab.sh $1/ab_cb base nonxt || exit 1
AB_SCENES="f2 b1" AB_ARGS="--traversal near" bash scripts/gpu_lib_ab.sh $1/ab_near base nonxt || exit 1
AB_F2_SPP=128 AB_B1_SPP=128 AB_EC_SPP=16 bash scripts/gpu_lib_ab.sh $1/ab_parkw base parkw parkw3 || exit 1
bash scripts/calls/gpu_r04f.sh $1/shares || exit 1
