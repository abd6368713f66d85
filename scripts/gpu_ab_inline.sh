# Inline light chains (DScene::light_inline) A/B: the GPU suite with the default (inline on where
# the scene allows it), then bench lines with JT_LIGHT_INLINE=0 / 1 alternating on the four configs.
# usage: bash scripts/gpu_ab_inline.sh <tag> [skip-tests]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
if [ "$2" != "skip-tests" ]; then
  scripts/gpu_step.sh 600 $O/pytest.log python -u -m pytest tests -x -v -m gpu -rf --timeout 300 --timeout-method thread || exit 1
  grep -q " passed" $O/pytest.log && ! grep -q -E "[0-9]+ failed" $O/pytest.log || { echo "GPU tests failed"; exit 1; }
fi
run() {  # name inline bench-args...
  local name=$1 inl=$2; shift 2
  JT_LIGHT_INLINE=$inl scripts/gpu_step.sh 200 $O/${name}_$inl.log python bench.py --no-cpu-baseline --no-reference-order "$@" || exit 1
  echo "$name inline=$inl => $(grep -h '"value"' $O/${name}_$inl.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["value"],1), d["ms_per_step"], d["roofline"]["launch"].split()[-1])')" | tee -a $O/summary.txt
}
for r in 1 2; do
  for inl in 0 1; do
    run cb $inl --steps 10
    run f2 $inl --steps 2 --warmup 1 --scene assets/scenes/features2/features2.json --width 1920 --height 1080 --spp 64
    run b1 $inl --steps 2 --warmup 1 --scene assets/scenes/bathroom1/bathroom1.json --width 1920 --height 1080 --spp 128
  done
done
