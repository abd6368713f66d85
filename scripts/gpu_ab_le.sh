# light-element records for light_hit: GPU parity subset, then A/B against HEAD
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/le
scripts/gpu_step.sh 600 gpurun_out/le/pytest.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scenes.py tests/test_gpu_variants.py tests/test_gpu_traversal.py -x -q -m gpu --timeout 300 --timeout-method thread || exit 1
AB_SCENES="f2 b1 cb" bash scripts/gpu_lib_ab.sh le/ab base head
