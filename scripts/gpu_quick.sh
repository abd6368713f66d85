# Tests + smoke + headline bench + quick scene lines (configs 3-5 at reduced spp), one call.
# usage: bash scripts/gpu_quick.sh <tag> [skip-tests]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
if [ "$2" != "skip-tests" ]; then
  scripts/gpu_step.sh 900 $O/pytest.log python -u -m pytest tests -x -v -m gpu -rf --timeout 300 --timeout-method thread || exit 1
  scripts/gpu_step.sh 120 $O/smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit 1
fi
scripts/gpu_step.sh 300 $O/cb.log python bench.py --steps 10 --no-cpu-baseline || exit 1
scripts/gpu_step.sh 200 $O/f2.log python bench.py --no-cpu-baseline --no-reference-order --steps 2 --warmup 1 --scene assets/scenes/features2/features2.json --width 1920 --height 1080 --spp 64 || exit 1
scripts/gpu_step.sh 200 $O/b1.log python bench.py --no-cpu-baseline --no-reference-order --steps 2 --warmup 1 --scene assets/scenes/bathroom1/bathroom1.json --width 1920 --height 1080 --spp 128 || exit 1
scripts/gpu_step.sh 200 $O/ec.log python bench.py --no-cpu-baseline --no-reference-order --steps 2 --warmup 1 --scene assets/scenes/ecosys/ecosys.json --width 3840 --height 2160 --spp 8 || exit 1
for f in cb f2 b1 ec; do python -c "
import json
for l in open('$O/$f.log'):
    if l.startswith('{'):
        d=json.loads(l); print('$f', d['value'], 'ms/step', d['ms_per_step'])
"; done
