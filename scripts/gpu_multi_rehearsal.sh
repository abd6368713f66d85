# N-rank rehearsal of bench.py's distributed path on a one-GPU box: every rank on cuda:0, the
# reduce through gloo (RCCL cannot put two ranks on one device). The driver's 8-GPU run uses
# RCCL; this checks sharding, the running-mean view, the reduce and the JSON line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/multi
for n in 2 4; do
  JT_BENCH_BACKEND=gloo JT_BENCH_DEVICE=0 scripts/gpu_step.sh 300 gpurun_out/multi/bench_n$n.log \
    python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29500 + n)) \
    bench.py --gpus $n --steps 2 --warmup 1 --no-cpu-baseline || exit 1
done
