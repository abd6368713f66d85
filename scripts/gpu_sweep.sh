# pytest -m gpu, then the bench at several JT_WAIT_LANES values, then the stamps diagnostic.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tag=$1; shift
mkdir -p gpurun_out/$tag
scripts/gpu_step.sh 900 gpurun_out/$tag/pytest.log python -m pytest tests -q -m gpu -rf --timeout 600 || exit 1
for w in "$@"; do
  JT_WAIT_LANES=$w scripts/gpu_step.sh 300 gpurun_out/$tag/bench_w$w.log python bench.py --no-cpu-baseline || exit 1
done
scripts/gpu_step.sh 300 gpurun_out/$tag/stamps.log python scripts/stamps.py 64 || exit 1
