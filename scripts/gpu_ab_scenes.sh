# A/B of the large-scene (HBM-mode) kernels: parity tests, then scene bench lines for the
# current library and build/libjtrace_hip_base.so (the previous commit), interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
scripts/gpu_step.sh 600 $O/pytest.log timeout -k 10 580 python -u -m pytest tests/test_gpu_scenes.py tests/test_gpu_parity.py -x -v -m gpu --timeout 300 --timeout-method thread || exit 1
grep -q " failed" $O/pytest.log && exit 1
B="python bench.py --no-cpu-baseline --steps 2 --warmup 1"
for lib in cur base; do
  if [ $lib = base ]; then export JTRACE_LIB=$PWD/julia-raytracer_amd/build/libjtrace_hip_base.so; fi
  scripts/gpu_step.sh 200 $O/b1_$lib.log timeout -k 10 180 $B --scene assets/scenes/bathroom1/bathroom1.json --width 1920 --height 1080 --spp 32 || exit 1
  scripts/gpu_step.sh 200 $O/ec_$lib.log timeout -k 10 180 $B --scene assets/scenes/ecosys/ecosys.json --width 3840 --height 2160 --spp 8 || exit 1
  scripts/gpu_step.sh 200 $O/f2_$lib.log timeout -k 10 180 $B --scene assets/scenes/features2/features2.json --width 1920 --height 1080 --spp 64 || exit 1
done
for f in $O/*_cur.log $O/*_base.log; do grep -h '"value"' $f | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['roofline']['kernel'], d['time_to_first_pixel_s'])"; done
