# Round 4, the final build in one call: the GPU suite, the roofline records (headline, its 1/2,
# 1/4, 1/8 shares, configs 3-5 at their own spp) copied into profiles/r04_roofline on the box so
# that the bench lines after them pick them up, the bench lines, smoke() and the N=2/4 rehearsal.
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
for s in cb cb_n2 cb_n4 cb_n8 f2 b1 ec; do cp $O/$s/roofline.json profiles/r04_roofline/${s}_final.json; done
scripts/gpu_step.sh 400 $O/bench.log python bench.py || exit 1
for n in 2 4 8; do scripts/gpu_step.sh 200 $O/bench_n$n.log timeout -k 10 180 python bench.py --no-cpu-baseline --no-reference-order --steps $((10 * n)) --as-rank-of $n || exit 1; done
scripts/gpu_step.sh 600 $O/bench_f2.log timeout -k 10 580 python bench.py --no-cpu-baseline --steps 2 --warmup 1 --scene assets/scenes/features2/features2.json --width 1920 --height 1080 --spp 512 || exit 1
scripts/gpu_step.sh 600 $O/bench_b1.log timeout -k 10 580 python bench.py --no-cpu-baseline --steps 2 --warmup 1 --scene assets/scenes/bathroom1/bathroom1.json --width 1920 --height 1080 --spp 1024 || exit 1
scripts/gpu_step.sh 600 $O/bench_ec.log timeout -k 10 580 python bench.py --no-cpu-baseline --steps 2 --warmup 1 --scene assets/scenes/ecosys/ecosys.json --width 3840 --height 2160 --spp 64 || exit 1
scripts/gpu_step.sh 300 $O/smoke.log timeout -k 10 280 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
bash scripts/gpu_rehearse.sh $1/rehearse || exit 1
