# Round 4, call 8: roofline records of the final build — the headline, its 1/2, 1/4, 1/8 sample
# shares (the workloads the SCALE lines' ranks run) and configs 3-5 at their own spp — then the
# bench lines that pick them up, and a chunk=1 check on the 1/8 share.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
bash scripts/gpu_measure.sh $O/cb "cornellbox path 1280x720 256 samples/launch traversal=near" || exit 1
for n in 2 4 8; do
  bash scripts/gpu_measure.sh $O/cb_n$n "cornellbox path 1280x720 $((256 / n)) samples/launch traversal=near" --as-rank-of $n || exit 1
done
MEASURE_STEPS=1 MEASURE_WARMUP=0 bash scripts/gpu_measure.sh $O/f2 "features2 path 1920x1080 512 samples/launch traversal=wide" --scene assets/scenes/features2/features2.json --width 1920 --height 1080 --spp 512 || exit 1
MEASURE_STEPS=1 MEASURE_WARMUP=0 bash scripts/gpu_measure.sh $O/b1 "bathroom1 path 1920x1080 1024 samples/launch traversal=wide" --scene assets/scenes/bathroom1/bathroom1.json --width 1920 --height 1080 --spp 1024 || exit 1
MEASURE_STEPS=1 MEASURE_WARMUP=0 bash scripts/gpu_measure.sh $O/ec "ecosys path 3840x2160 64 samples/launch traversal=wide" --scene assets/scenes/ecosys/ecosys.json --width 3840 --height 2160 --spp 64 || exit 1
mkdir -p profiles/r04_roofline
for s in cb cb_n2 cb_n4 cb_n8 f2 b1 ec; do cp $O/$s/roofline.json profiles/r04_roofline/${s}_final.json; done
scripts/gpu_step.sh 400 $O/bench.log python bench.py || exit 1
for n in 2 4 8; do scripts/gpu_step.sh 200 $O/bench_n$n.log timeout -k 10 180 python bench.py --no-cpu-baseline --no-reference-order --steps $((10 * n)) --as-rank-of $n || exit 1; done
scripts/gpu_step.sh 200 $O/bench_n8_chunk1.log timeout -k 10 180 python bench.py --no-cpu-baseline --no-reference-order --steps 80 --as-rank-of 8 --opt chunk=1 || exit 1
scripts/gpu_step.sh 600 $O/bench_f2.log timeout -k 10 580 python bench.py --no-cpu-baseline --steps 2 --warmup 1 --scene assets/scenes/features2/features2.json --width 1920 --height 1080 --spp 512 || exit 1
scripts/gpu_step.sh 600 $O/bench_b1.log timeout -k 10 580 python bench.py --no-cpu-baseline --steps 2 --warmup 1 --scene assets/scenes/bathroom1/bathroom1.json --width 1920 --height 1080 --spp 1024 || exit 1
scripts/gpu_step.sh 600 $O/bench_ec.log timeout -k 10 580 python bench.py --no-cpu-baseline --steps 2 --warmup 1 --scene assets/scenes/ecosys/ecosys.json --width 3840 --height 2160 --spp 64 || exit 1
