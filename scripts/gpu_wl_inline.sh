# GPU suite, then the shading-gate threshold (JT_WAIT_LANES) re-swept with inline light chains:
# the light queries no longer wait in the traversal loop, so the gate's best value may move.
# usage: bash scripts/gpu_wl_inline.sh <tag> [skip-tests]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
if [ "$2" != "skip-tests" ]; then
  scripts/gpu_step.sh 600 $O/pytest.log python -u -m pytest tests -x -v -m gpu -rf --timeout 300 --timeout-method thread || exit 1
  grep -q " passed" $O/pytest.log && ! grep -q -E "[0-9]+ failed" $O/pytest.log || { echo "GPU tests failed"; exit 1; }
fi
run() {  # name W bench-args...
  local name=$1 w=$2; shift 2
  JT_WAIT_LANES=$w scripts/gpu_step.sh 200 $O/${name}_$w.log python bench.py --no-cpu-baseline --no-reference-order "$@" || exit 1
  echo "$name W=$w => $(grep -h '"value"' $O/${name}_$w.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["value"],1), d["ms_per_step"], d["roofline"]["kernel"])')" | tee -a $O/summary.txt
}
F2="--steps 2 --warmup 1 --scene assets/scenes/features2/features2.json --width 1920 --height 1080 --spp 64"
B1="--steps 2 --warmup 1 --scene assets/scenes/bathroom1/bathroom1.json --width 1920 --height 1080 --spp 128"
for w in 40 48 56 60 64; do run cb $w --steps 10; done
for w in 32 40 48 56; do run f2 $w $F2; done
for w in 24 32 40 48; do run b1 $w $B1; done
run ec 16 --steps 2 --warmup 1 --scene assets/scenes/ecosys/ecosys.json --width 3840 --height 2160 --spp 8
