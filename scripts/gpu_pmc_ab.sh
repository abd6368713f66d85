# PMC comparison of two library builds on the headline workload (32 spp, one pass each):
#   scripts/gpu_pmc_ab.sh <out> <variant .so name under julia-raytracer_amd/build>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
B="bench.py --steps 1 --warmup 0 --no-cpu-baseline --spp 32"
C1="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
C2="SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
for v in base $2; do
  if [ $v != base ]; then export JTRACE_LIB=$GRAFT_REPO_ROOT/julia-raytracer_amd/build/libjtrace_hip_$v.so; fi
  scripts/gpu_step.sh 120 $O/$v.p1.log timeout -s KILL 100 rocprofv3 --pmc $C1 --output-format csv -d $O/$v/p1 -o p1 -- python3 $B || exit 1
  scripts/gpu_step.sh 120 $O/$v.p2.log timeout -s KILL 100 rocprofv3 --pmc $C2 --output-format csv -d $O/$v/p2 -o p2 -- python3 $B || exit 1
  python scripts/pmc_summary.py $O/$v > $O/${v}_summary.txt
done
