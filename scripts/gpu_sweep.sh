# Sweep of the shading gate (wait_lanes) and node-repeat-free knobs on the work-item body, per scene.
# usage: bash scripts/gpu_sweep.sh <tag> [scenes...]   (cb f2 b1 ec)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; shift
mkdir -p $O
SC=${*:-cb}
args() {
  case $1 in
    f2) echo "--scene assets/scenes/features2/features2.json --width 1920 --height 1080 --spp 64 --steps 2 --warmup 1" ;;
    b1) echo "--scene assets/scenes/bathroom1/bathroom1.json --width 1920 --height 1080 --spp 64 --steps 2 --warmup 1" ;;
    ec) echo "--scene assets/scenes/ecosys/ecosys.json --width 3840 --height 2160 --spp 8 --steps 2 --warmup 1" ;;
    cb) echo "--steps 10" ;;
  esac
}
for sc in $SC; do
  for wl in 40 48 52 56 60 64; do
    scripts/gpu_step.sh 200 $O/${sc}_wl$wl.log timeout -k 10 180 python bench.py --no-cpu-baseline --no-reference-order --traversal ${TRAV:-near} --opt wait_lanes=$wl $(args $sc) || exit 1
    echo "$sc wait_lanes=$wl => $(grep -h '"value"' $O/${sc}_wl$wl.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["value"],1))')" | tee -a $O/summary.txt
  done
done
