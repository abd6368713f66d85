# Round evidence of the current build in one call: GPU suite, smoke, headline bench (with CPU
# baseline) and its roofline passes, configs 3-5 bench lines and roofline passes, stamps.
# usage: bash scripts/gpu_final.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
scripts/gpu_step.sh 600 $O/pytest.log python -u -m pytest tests -x -v -m gpu -rf --timeout 300 --timeout-method thread || exit 1
grep -q " passed" $O/pytest.log && ! grep -q -E "[0-9]+ failed" $O/pytest.log || { echo "GPU tests failed"; exit 1; }
scripts/gpu_step.sh 120 $O/smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit 1
scripts/gpu_step.sh 400 $O/bench.log python bench.py || exit 1
bash scripts/gpu_measure.sh $O/cb "cornellbox path 1280x720 256 samples/launch traversal=near" || exit 1
bash scripts/gpu_scenes.sh $1/scenes || exit 1
scripts/gpu_step.sh 120 $O/stamps.log timeout -k 10 100 python scripts/stamps.py 32 || exit 1
nproc > $O/host.txt; lscpu | grep -E "Model name|Socket|Core|Thread" >> $O/host.txt
