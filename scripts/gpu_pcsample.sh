# PC sampling of the headline kernel (diagnostic): rocprofv3's host-trap PC sampler over a short
# bench run of a line-table build (make variant V=lines X=-gline-tables-only), then the samples
# are attributed to source lines by scripts/pc_lines.py.  usage: bash scripts/gpu_pcsample.sh <tag> [bench args]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1; shift
mkdir -p $O
L=$GRAFT_REPO_ROOT/julia-raytracer_amd/build/libjtrace_hip_lines.so
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
JTRACE_LIB=$L scripts/gpu_step.sh 200 $O/pcs.log timeout -s KILL 180 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 1 --output-format csv -d $O/pcs -o pcs -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-reference-order "$@" || exit 1
ls -R $O/pcs | head -20
