# bench each library variant given (no tests). usage: bash scripts/gpu_bench_variants.sh <tag> v1.so v2.so ...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tag=$1; shift
mkdir -p gpurun_out/$tag
for v in "$@"; do
  JTRACE_LIB=$v scripts/gpu_step.sh 300 gpurun_out/$tag/bench_$(basename $v .so).log python bench.py --no-cpu-baseline || exit 1
done
