# Round 4 check: the GPU suite on the current build (per-lane work items + wide traversal), then
# A/B of the work-item body against the tile-unit body, then wide vs near traversal per scene.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
scripts/gpu_step.sh 900 $O/pytest.log python -u -m pytest tests -x -v -m gpu -rf --timeout 300 --timeout-method thread || exit 1
tail -3 $O/pytest.log
grep -q "failed\|error" $O/pytest.log && { echo "GPU tests failed: stopping"; exit 1; }
AB_SCENES="cb f2 b1 ec" bash scripts/gpu_lib_ab.sh $1/ab base tiles nofuse || exit 1
bash scripts/gpu_wide.sh $1/wide skip-tests || exit 1
