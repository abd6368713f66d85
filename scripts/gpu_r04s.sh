# Round 4: combinations of the scheduling knobs that gained in r04r (no first pop at the sample
# hand-out; 2 pops per node iteration and vote bias 4 in the HBM kernels) on all four scenes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
AB_SCENES="cb" bash scripts/gpu_lib_ab.sh $1/ab_cb base i0 i0v4 || exit 1
AB_SCENES="f2 b1 ec" AB_F2_SPP=128 AB_B1_SPP=128 AB_EC_SPP=16 bash scripts/gpu_lib_ab.sh $1/ab_hbm base i0 i0n2 i0v4 i0n2v4 || exit 1
