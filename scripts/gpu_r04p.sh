# Round 4, final build, call 1 of 2: the GPU suite, then the roofline records of the headline, its
# 1/2, 1/4, 1/8 sample shares and configs 3-5 at their own spp (auto traversal: near for
# cornellbox and features2, wide for bathroom1 and ecosys).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
scripts/gpu_step.sh 600 $O/tests.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" $O/tests.log && ! grep -q "failed\|error" $O/tests.log || { echo "GPU tests not green: stopping"; exit 1; }
bash scripts/gpu_measure.sh $O/cb "cornellbox path 1280x720 256 samples/launch traversal=near" || exit 1
for n in 2 4 8; do
  bash scripts/gpu_measure.sh $O/cb_n$n "cornellbox path 1280x720 $((256 / n)) samples/launch traversal=near" --as-rank-of $n || exit 1
done
MEASURE_STEPS=1 MEASURE_WARMUP=0 bash scripts/gpu_measure.sh $O/f2 "features2 path 1920x1080 512 samples/launch traversal=near" --scene assets/scenes/features2/features2.json --width 1920 --height 1080 --spp 512 || exit 1
MEASURE_STEPS=1 MEASURE_WARMUP=0 bash scripts/gpu_measure.sh $O/b1 "bathroom1 path 1920x1080 1024 samples/launch traversal=wide" --scene assets/scenes/bathroom1/bathroom1.json --width 1920 --height 1080 --spp 1024 || exit 1
MEASURE_STEPS=1 MEASURE_WARMUP=0 bash scripts/gpu_measure.sh $O/ec "ecosys path 3840x2160 64 samples/launch traversal=wide" --scene assets/scenes/ecosys/ecosys.json --width 3840 --height 2160 --spp 64 || exit 1
