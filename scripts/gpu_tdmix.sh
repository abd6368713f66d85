# The HBM-mode kernels' load-mix ceiling (scripts/td_mix_bench.hip): rates, then TD busy and the
# L2 hit rate of every dispatch in its own PMC pass.
# usage: bash scripts/gpu_tdmix.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
scripts/gpu_step.sh 120 $O/rates.log timeout -k 10 100 julia-raytracer_amd/build/td_mix_bench || exit 1
scripts/gpu_step.sh 120 $O/pmc.log timeout -s KILL 100 rocprofv3 --pmc TD_TD_BUSY_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d $O/pmc -o pmc -- julia-raytracer_amd/build/td_mix_bench || exit 1
scripts/gpu_step.sh 120 $O/kt.log timeout -k 10 100 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- julia-raytracer_amd/build/td_mix_bench || exit 1
