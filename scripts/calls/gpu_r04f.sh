# Round 4, call 3: the 8-GPU configs' one-GPU shares (--as-rank-of 8) at their spec sample counts,
# the headline's N-share efficiencies, the near-order lines of configs 3-5 for comparison.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
scripts/gpu_step.sh 300 $O/b1_rank_of_8.log timeout -k 10 280 python bench.py --no-cpu-baseline --steps 1 --warmup 1 --scene assets/scenes/bathroom1/bathroom1.json --width 1920 --height 1080 --spp 1024 --as-rank-of 8 || exit 1
scripts/gpu_step.sh 300 $O/ec_rank_of_8.log timeout -k 10 280 python bench.py --no-cpu-baseline --steps 1 --warmup 0 --scene assets/scenes/ecosys/ecosys.json --width 3840 --height 2160 --spp 4096 --as-rank-of 8 || exit 1
bash scripts/gpu_split.sh $1/split || exit 1
