# light-hit steps in the environment kernels (JT_LSTEP_ENV): GPU parity subset, then A/B at the configs' spp
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ls
scripts/gpu_step.sh 600 gpurun_out/ls/pytest2.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scenes.py tests/test_gpu_traversal.py tests/test_gpu_variants.py -x -q -m gpu --timeout 300 --timeout-method thread || exit 1
AB_F2_SPP=512 AB_B1_SPP=1024 AB_EC_SPP=64 AB_SCENES="f2 ec" bash scripts/gpu_lib_ab.sh ls/ab2 base nols
