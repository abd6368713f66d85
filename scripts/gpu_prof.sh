set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
B="bench.py --steps 2 --warmup 1 --no-cpu-baseline"
scripts/gpu_step.sh 120 gpurun_out/prof/counters_list.txt rocprofv3 -L || exit 1
scripts/gpu_step.sh 300 gpurun_out/prof/kt.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/kt -o kt -- python3 $B || exit 1
scripts/gpu_step.sh 300 gpurun_out/prof/pmc1.log rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d gpurun_out/prof/pmc1 -o pmc1 -- python3 $B || exit 1
scripts/gpu_step.sh 300 gpurun_out/prof/pmc2.log rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_FLAT SQ_INSTS_BRANCH SQ_INSTS_VALU_TRANS_F32 --output-format csv -d gpurun_out/prof/pmc2 -o pmc2 -- python3 $B || exit 1
scripts/gpu_step.sh 300 gpurun_out/prof/pmc3.log rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/prof/pmc3 -o pmc3 -- python3 $B || exit 1
scripts/gpu_step.sh 300 gpurun_out/prof/pmc4.log rocprofv3 --pmc WRITE_SIZE TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum --output-format csv -d gpurun_out/prof/pmc4 -o pmc4 -- python3 $B || exit 1
