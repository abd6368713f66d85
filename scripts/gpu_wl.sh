# wait_lanes (shading-gate threshold) sweep at the configs' own spp, current build
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-wl3}
mkdir -p $O
run() {  # tag W bench-args...
  local tag=$1 w=$2; shift 2
  JT_WAIT_LANES=$w scripts/gpu_step.sh 240 $O/${tag}_$w.log timeout -k 10 220 python bench.py --no-cpu-baseline --no-reference-order --steps 1 --warmup 1 "$@" || exit 1
  echo "$tag W=$w => $(grep -h '"value"' $O/${tag}_$w.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["value"],1), d["ms_per_step"], d["roofline"]["launch"].split("chunk=")[1].split()[0])')" | tee -a $O/summary.txt
}
F2="--scene assets/scenes/features2/features2.json --width 1920 --height 1080 --spp 512"
B1="--scene assets/scenes/bathroom1/bathroom1.json --width 1920 --height 1080 --spp 1024"
EC="--scene assets/scenes/ecosys/ecosys.json --width 3840 --height 2160 --spp 64"
for w in 24 32 40 48; do run b1 $w $B1; done
for w in 8 16 24 32; do run ec $w $EC; done
for w in 32 40 48 56; do run f2 $w $F2; done
