# Round 4, call 1: the GPU suite, wide vs near per scene, the headline bench line (with its
# image signature), the headline roofline record, the N=2 rehearsal with the image check.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
scripts/gpu_step.sh 600 $O/pytest.log python -u -m pytest tests -x -v -m gpu -rf --timeout 300 --timeout-method thread || exit 1
tail -2 $O/pytest.log
grep -q " failed\| error" $O/pytest.log && { echo "GPU tests failed: stopping"; exit 1; }
bash scripts/gpu_wide.sh $1/wide skip-tests || exit 1
AB_SCENES="b1 ec" AB_ARGS="--traversal wide" bash scripts/gpu_lib_ab.sh $1/abpk base nopk || exit 1
scripts/gpu_step.sh 300 $O/signature.log python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-reference-order --write-signature || exit 1
cp profiles/image_signatures.json $O/ || exit 1
scripts/gpu_step.sh 400 $O/bench.log python bench.py || exit 1
bash scripts/gpu_measure.sh $O/cb "cornellbox path 1280x720 256 samples/launch traversal=near" || exit 1
JT_BENCH_BACKEND=gloo JT_BENCH_DEVICE=0 scripts/gpu_step.sh 300 $O/rehearsal_n2.log python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline || exit 1
nproc > $O/host.txt; lscpu | grep -E "Model name|Socket|Core|Thread" >> $O/host.txt
