# Roofline evidence for one bench workload: rocprofv3 kernel-trace stats, the FETCH_SIZE and
# WRITE_SIZE passes (separate on gfx950), an SQ instruction pass, a TA/TD/TCP/TCC pass (busy,
# stalls, L1 accesses, L2 hits/misses) and an SQ wait-state pass (issue stalls, LDS), each its own
# rocprofv3 run with no tracing domains, then scripts/roofline.py combines them.
# usage: bash scripts/gpu_measure.sh <outdir> <workload string> <bench args...>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=$1; workload=$2; shift 2
mkdir -p $out
B="bench.py --steps ${MEASURE_STEPS:-2} --warmup ${MEASURE_WARMUP:-1} --no-cpu-baseline --no-reference-order $*"
scripts/gpu_step.sh 300 $out/kt.log rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt -o kt -- python3 $B || exit 1
scripts/gpu_step.sh 300 $out/fetch.log timeout -s KILL 280 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/fetch -o fetch -- python3 $B || exit 1
scripts/gpu_step.sh 300 $out/write.log timeout -s KILL 280 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/write -o write -- python3 $B || exit 1
scripts/gpu_step.sh 300 $out/p1.log timeout -s KILL 280 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $out/pmc/p1 -o p1 -- python3 $B || exit 1
scripts/gpu_step.sh 300 $out/p2.log timeout -s KILL 280 rocprofv3 --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d $out/pmc/p2 -o p2 -- python3 $B || exit 1
scripts/gpu_step.sh 300 $out/p3.log timeout -s KILL 280 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $out/pmc/p3 -o p3 -- python3 $B || exit 1
python scripts/roofline.py make --stats "$(find $out/kt -name "*kernel_stats.csv" | sort | head -n 1)" --fetch $out/fetch --write $out/write --pmc $out/pmc --workload "$workload" --out $out/roofline.json
