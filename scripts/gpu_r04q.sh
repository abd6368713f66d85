# Round 4, final build, call 2 of 2 (the records of call 1 committed under profiles/r04_roofline):
# the bench lines that pick them up — the headline with its CPU baseline, its 1/N shares, configs
# 3-5 with their reference-order lines — and the smoke entry point.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
scripts/gpu_step.sh 400 $O/bench.log python bench.py || exit 1
for n in 2 4 8; do scripts/gpu_step.sh 200 $O/bench_n$n.log timeout -k 10 180 python bench.py --no-cpu-baseline --no-reference-order --steps $((10 * n)) --as-rank-of $n || exit 1; done
scripts/gpu_step.sh 600 $O/bench_f2.log timeout -k 10 580 python bench.py --no-cpu-baseline --steps 2 --warmup 1 --scene assets/scenes/features2/features2.json --width 1920 --height 1080 --spp 512 || exit 1
scripts/gpu_step.sh 600 $O/bench_b1.log timeout -k 10 580 python bench.py --no-cpu-baseline --steps 2 --warmup 1 --scene assets/scenes/bathroom1/bathroom1.json --width 1920 --height 1080 --spp 1024 || exit 1
scripts/gpu_step.sh 600 $O/bench_ec.log timeout -k 10 580 python bench.py --no-cpu-baseline --steps 2 --warmup 1 --scene assets/scenes/ecosys/ecosys.json --width 3840 --height 2160 --spp 64 || exit 1
scripts/gpu_step.sh 300 $O/smoke.log timeout -k 10 280 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
bash scripts/gpu_rehearse.sh $1/rehearse || exit 1
