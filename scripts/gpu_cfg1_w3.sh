set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/c1
scripts/gpu_step.sh 300 gpurun_out/c1/bench_naive_cfg1.log python bench.py --sampler naive --width 256 --height 256 --spp 16 --cpu-spp 16 --steps 5 --warmup 2 || exit 1
JTRACE_LIB=julia-raytracer_amd/build/libjtrace_hip_w3.so scripts/gpu_step.sh 300 gpurun_out/c1/bench_w3.log python bench.py --no-cpu-baseline || exit 1
scripts/gpu_step.sh 300 gpurun_out/c1/bench_default.log python bench.py --no-cpu-baseline || exit 1
