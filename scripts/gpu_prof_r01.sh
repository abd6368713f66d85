# Round-1 measurement: full bench (with the CPU baseline), kernel-trace stats, and the two PMC
# passes for HBM traffic (FETCH_SIZE and WRITE_SIZE need separate passes on gfx950).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r01
B="bench.py --steps 3 --warmup 1 --no-cpu-baseline"
scripts/gpu_step.sh 600 gpurun_out/r01/bench.log python bench.py || exit 1
scripts/gpu_step.sh 300 gpurun_out/r01/kt.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r01/kt -o kt -- python3 $B || exit 1
scripts/gpu_step.sh 300 gpurun_out/r01/fetch.log rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r01/fetch -o fetch -- python3 $B || exit 1
scripts/gpu_step.sh 300 gpurun_out/r01/write.log rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r01/write -o write -- python3 $B || exit 1
nproc > gpurun_out/r01/host.txt; lscpu | grep -E "Model name|Socket|Core|Thread" >> gpurun_out/r01/host.txt
