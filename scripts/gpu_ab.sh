# A/B: GPU test suite on the default library, then the bench on each library variant given.
# usage: bash scripts/gpu_ab.sh <tag> [variant.so ...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tag=$1; shift
mkdir -p gpurun_out/$tag
scripts/gpu_step.sh 900 gpurun_out/$tag/pytest.log python -m pytest tests -q -m gpu -rf --timeout 600 || exit 1
scripts/gpu_step.sh 300 gpurun_out/$tag/bench_default.log python bench.py --no-cpu-baseline || exit 1
for v in "$@"; do
  JTRACE_LIB=$v scripts/gpu_step.sh 300 gpurun_out/$tag/bench_$(basename $v .so).log python bench.py --no-cpu-baseline || exit 1
done
