# pytest -m gpu, then the bench under each "VAR=value[,VAR2=value]" setting given.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tag=$1; shift
mkdir -p gpurun_out/$tag
if [ -z "$NO_TESTS" ]; then
  scripts/gpu_step.sh 900 gpurun_out/$tag/pytest.log python -m pytest tests -q -m gpu -rf --timeout 600 || exit 1
fi
for cfg in "$@"; do
  ( IFS=','; for kv in $cfg; do export "$kv"; done
    scripts/gpu_step.sh 300 gpurun_out/$tag/bench_$(echo $cfg | tr ',=/' '_-_').log python bench.py --no-cpu-baseline ) || exit 1
done
