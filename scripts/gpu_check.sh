# Quick GPU check of the current tree: the GPU test suite (optionally a -k filter), smoke and a
# short headline bench.  usage: bash scripts/gpu_check.sh <tag> [pytest -k expression]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
K=${2:+-k "$2"}
scripts/gpu_step.sh 900 $O/pytest.log python -u -m pytest tests -x -v -m gpu -rf --timeout 300 --timeout-method thread $K || exit 1
scripts/gpu_step.sh 120 $O/smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit 1
scripts/gpu_step.sh 300 $O/bench.log python bench.py --steps 10 --no-cpu-baseline || exit 1
