# PMC passes (one rocprofv3 --pmc run per counter group, no tracing domains) of the bench on
# cornellbox (LDS mode, 64 spp) and bathroom1 (HBM mode, 16 spp).  usage: bash scripts/gpu_pmc.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tag=$1
run_groups() {  # <outdir> <bench args...>; groups on stdin
  local out=$1; shift
  mkdir -p $out
  local i=0
  while read -r grp; do
    [ -z "$grp" ] && continue
    i=$((i+1))
    scripts/gpu_step.sh 120 $out/p$i.log timeout -s KILL 100 rocprofv3 --pmc $grp --output-format csv -d $out/p$i -o p$i -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline "$@" || return 1
  done
}
run_groups gpurun_out/$tag/cb --spp 64 <<'GROUPS' || exit 1
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE
SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU SQ_IFETCH
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VSKIPPED SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA
GROUPS
run_groups gpurun_out/$tag/b1 --spp 16 --scene assets/scenes/bathroom1/bathroom1.json --width 1920 --height 1080 <<'GROUPS' || exit 1
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE
SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU SQ_IFETCH
TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum
TD_TD_BUSY_sum TD_TC_STALL_sum
TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum
TCC_HIT_sum TCC_MISS_sum
GROUPS
python scripts/pmc_summary.py gpurun_out/$tag/cb > gpurun_out/$tag/cb_summary.txt
python scripts/pmc_summary.py gpurun_out/$tag/b1 > gpurun_out/$tag/b1_summary.txt
