# Scene bench lines for several library builds (A/B): bash scripts/gpu_ab_libs.sh <tag> <lib suffixes...>
# ("cur" = build/libjtrace_hip.so, X = build/libjtrace_hip_X.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1; shift
mkdir -p $O
B="python bench.py --no-cpu-baseline --steps 2 --warmup 1"
for lib in "$@"; do
  if [ $lib = cur ]; then unset JTRACE_LIB; else export JTRACE_LIB=$PWD/julia-raytracer_amd/build/libjtrace_hip_$lib.so; fi
  scripts/gpu_step.sh 200 $O/b1_$lib.log timeout -k 10 180 $B --scene assets/scenes/bathroom1/bathroom1.json --width 1920 --height 1080 --spp 32 || exit 1
  scripts/gpu_step.sh 200 $O/ec_$lib.log timeout -k 10 180 $B --scene assets/scenes/ecosys/ecosys.json --width 3840 --height 2160 --spp 8 || exit 1
  scripts/gpu_step.sh 200 $O/f2_$lib.log timeout -k 10 180 $B --scene assets/scenes/features2/features2.json --width 1920 --height 1080 --spp 64 || exit 1
  scripts/gpu_step.sh 200 $O/cb_$lib.log timeout -k 10 180 $B || exit 1
done
for f in $O/*.log; do grep -h '"value"' $f | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('$f'.split('/')[-1], d['value'])"; done
