# Multi-rank bench rehearsal on a one-GPU box: 2 and 4 ranks of bench.py under torch.distributed.run,
# both on GPU 0, reducing through gloo (JT_BENCH_BACKEND=gloo: RCCL cannot put two ranks on one
# GPU). Exercises the driver's N>1 launch, sharding, barrier/max timing and the reduce.
# usage: bash scripts/gpu_rehearse.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
JT_BENCH_BACKEND=gloo JT_BENCH_DEVICE=0 scripts/gpu_step.sh 300 $O/rehearsal_n2_gloo_one_gpu.log python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline || exit 1
JT_BENCH_BACKEND=gloo JT_BENCH_DEVICE=0 scripts/gpu_step.sh 300 $O/rehearsal_n4_gloo_one_gpu.log python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 4 --steps 3 --warmup 1 --no-cpu-baseline || exit 1
