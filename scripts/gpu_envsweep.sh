# Environment-knob sweep: each line of $2 (a file) is "<scene> <ENV=VAL ...>"; scenes at the
# configs' own spp (cb: the headline). usage: bash scripts/gpu_envsweep.sh <tag> <file>
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
mkdir -p $O
args() {
  case $1 in
    f2) echo "--scene assets/scenes/features2/features2.json --width 1920 --height 1080 --spp 512" ;;
    b1) echo "--scene assets/scenes/bathroom1/bathroom1.json --width 1920 --height 1080 --spp 1024" ;;
    ec) echo "--scene assets/scenes/ecosys/ecosys.json --width 3840 --height 2160 --spp 64" ;;
    cb) echo "--steps 4" ;;
  esac
}
n=0
while read -r sc envs; do
  [ -z "$sc" ] && continue
  n=$((n + 1))
  env $envs scripts/gpu_step.sh 240 $O/run$n.log timeout -k 10 220 python bench.py --no-cpu-baseline --no-reference-order --steps 1 --warmup 1 $(args $sc) || exit 1
  echo "$sc $envs => $(grep -h '"value"' $O/run$n.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["value"],1), d["ms_per_step"])')" | tee -a $O/summary.txt
done < $2
