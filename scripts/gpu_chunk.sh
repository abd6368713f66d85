# Work-unit size (JT_CHUNK samples per 8x8 tile unit) at the configs' own spp: does a longer unit
# shrink the per-unit tail (lanes done with their pixel's chunk while the wave still runs it)?
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/chunk
mkdir -p $O
run() {  # tag chunk bench-args...
  local tag=$1 ch=$2; shift 2
  JT_CHUNK=$ch scripts/gpu_step.sh 240 $O/${tag}_$ch.log timeout -k 10 220 python bench.py --no-cpu-baseline --no-reference-order --steps 1 --warmup 1 "$@" || exit 1
  echo "$tag chunk=$ch => $(grep -h '"value"' $O/${tag}_$ch.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["value"],1), d["ms_per_step"])')" | tee -a $O/summary.txt
}
for ch in 64 128 256; do run f2 $ch --scene assets/scenes/features2/features2.json --width 1920 --height 1080 --spp 512; done
for ch in 64 128 256; do run b1 $ch --scene assets/scenes/bathroom1/bathroom1.json --width 1920 --height 1080 --spp 1024; done
for ch in 16 32 64; do run ec $ch --scene assets/scenes/ecosys/ecosys.json --width 3840 --height 2160 --spp 64; done
for ch in 64 128 256; do run cb $ch --steps 5; done
