# One GPU call of round work: the GPU test suite, the headline bench (with its CPU baseline) and
# the roofline evidence of the headline workload.  usage: bash scripts/gpu_round.sh <tag> [skip-tests]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tag=$1
O=gpurun_out/$tag
mkdir -p $O
if [ "$2" != "skip-tests" ]; then
  scripts/gpu_step.sh 900 $O/pytest.log python -u -m pytest tests -x -v -m gpu -rf --timeout 300 --timeout-method thread || exit 1
fi
scripts/gpu_step.sh 400 $O/bench.log python bench.py || exit 1
bash scripts/gpu_measure.sh $O/cb "cornellbox path 1280x720 256 samples/launch traversal=near" || exit 1
nproc > $O/host.txt; lscpu | grep -E "Model name|Socket|Core|Thread" >> $O/host.txt
