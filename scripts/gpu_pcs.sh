set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pcs
B="bench.py --steps 1 --warmup 0 --no-cpu-baseline --spp 64"
scripts/gpu_step.sh 300 gpurun_out/pcs/stoch.log rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles --pc-sampling-interval 1048576 --output-format csv -d gpurun_out/pcs/stoch -o stoch -- python3 $B || exit 1
scripts/gpu_step.sh 300 gpurun_out/pcs/host.log rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 100 --output-format csv -d gpurun_out/pcs/host -o host -- python3 $B || exit 1
ls -la gpurun_out/pcs/*/ > gpurun_out/pcs/ls.txt
