# pinned 16-B record rows (node, light, instance, shape): GPU parity subset, then A/B against the previous load pattern
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/nb1
scripts/gpu_step.sh 600 gpurun_out/nb1/pytest2.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scenes.py tests/test_gpu_traversal.py -x -q -m gpu --timeout 300 --timeout-method thread || exit 1
AB_SCENES="f2 b1 ec cb" bash scripts/gpu_lib_ab.sh nb1/ab2 base head
