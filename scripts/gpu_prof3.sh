set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${PROF_OUT:-gpurun_out/prof3}
mkdir -p $OUT
B="bench.py --steps 1 --warmup 0 --no-cpu-baseline ${BENCH_ARGS:-}"
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  scripts/gpu_step.sh 300 $OUT/p$i.log rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o p$i -- python3 $B || exit 1
done <<'GROUPS'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE
SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU SQ_IFETCH
TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum
TD_TD_BUSY_sum TD_TC_STALL_sum
TD_LOAD_WAVEFRONT_sum TD_COALESCABLE_WAVEFRONT_sum
TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum
GROUPS
