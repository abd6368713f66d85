set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_step.sh 600 gpurun_out/pytest_gpu.log python -m pytest tests -m gpu -q -x -s || exit 1
for w in 32 48 64; do
  JT_WAIT_LANES=$w scripts/gpu_step.sh 300 gpurun_out/bench_lds_w$w.log python bench.py --steps 3 --warmup 1 --no-cpu-baseline || exit 1
done
JT_LDS_SCENE=0 JT_WAIT_LANES=48 scripts/gpu_step.sh 300 gpurun_out/bench_hbm_w48.log python bench.py --steps 3 --warmup 1 --no-cpu-baseline || exit 1
