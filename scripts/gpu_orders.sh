# Both BVH child orders (reference, near) on the headline and configs 3-5 (reduced spp), bench
# lines only, plus the traversal tests with their printed statistics.
# usage: bash scripts/gpu_orders.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
scripts/gpu_step.sh 300 $O/pytest_trav.log python -u -m pytest tests/test_gpu_traversal.py -x -v -s -m gpu --timeout 120 --timeout-method thread -k "near_vs" || exit 1
for order in reference near; do
  scripts/gpu_step.sh 200 $O/cb_$order.log python bench.py --no-cpu-baseline --steps 5 --traversal $order || exit 1
  scripts/gpu_step.sh 200 $O/f2_$order.log python bench.py --no-cpu-baseline --steps 2 --warmup 1 --scene assets/scenes/features2/features2.json --width 1920 --height 1080 --spp 64 --traversal $order || exit 1
  scripts/gpu_step.sh 200 $O/b1_$order.log python bench.py --no-cpu-baseline --steps 2 --warmup 1 --scene assets/scenes/bathroom1/bathroom1.json --width 1920 --height 1080 --spp 128 --traversal $order || exit 1
  scripts/gpu_step.sh 200 $O/ec_$order.log python bench.py --no-cpu-baseline --steps 2 --warmup 1 --scene assets/scenes/ecosys/ecosys.json --width 3840 --height 2160 --spp 8 --traversal $order || exit 1
done
python - << 'PY'
import json, glob, os
O = os.environ.get("O_DIR")
PY
for f in $O/*_reference.log $O/*_near.log; do python -c "
import json,sys
for l in open('$f'):
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']; print('$f'.split('/')[-1], d['value'], 'ms/step', d['ms_per_step'], 'per_ray', r['per_ray'])
"; done
# optional library A/B on the same box: ORDERS_AB="<lib> ..." (lib .so names under julia-raytracer_amd/build)
if [ -n "$ORDERS_AB" ]; then
  AB_SCENES="cb f2 b1" bash scripts/gpu_lib_ab.sh $1/ab base $ORDERS_AB || exit 1
fi
