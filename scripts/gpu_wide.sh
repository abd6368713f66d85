# The wide traversal on the GPU: its parity tests, then bench lines near vs wide per scene.
# usage: bash scripts/gpu_wide.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
if [ "$2" != "skip-tests" ]; then
  scripts/gpu_step.sh 300 $O/pytest_trav.log python -u -m pytest tests/test_gpu_traversal.py -x -v -m gpu -rf --timeout 120 --timeout-method thread || exit 1
  grep -q " passed" $O/pytest_trav.log && ! grep -q "FAILED\|Error" $O/pytest_trav.log || { echo "traversal tests failed"; exit 1; }
fi
run() {  # name bench-args...
  local name=$1; shift
  scripts/gpu_step.sh 240 $O/$name.log timeout -k 10 220 python bench.py --no-cpu-baseline --no-reference-order "$@" || exit 1
  echo "$name => $(grep -h '"value"' $O/$name.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["value"],1), d["roofline"]["per_ray"])')" | tee -a $O/summary.txt
}
for t in near wide; do
  run cb_$t --traversal $t --steps 10
  run b1_$t --traversal $t --scene assets/scenes/bathroom1/bathroom1.json --width 1920 --height 1080 --spp 64 --steps 2 --warmup 1
  run ec_$t --traversal $t --scene assets/scenes/ecosys/ecosys.json --width 3840 --height 2160 --spp 8 --steps 2 --warmup 1
  run f2_$t --traversal $t --scene assets/scenes/features2/features2.json --width 1920 --height 1080 --spp 64 --steps 2 --warmup 1
done
