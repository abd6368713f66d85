# features2 with light-hit steps: wait_lanes and light_lanes at 512 spp
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/f2tune
mkdir -p $O
F2="--scene assets/scenes/features2/features2.json --width 1920 --height 1080 --spp 512"
for cfg in "48 2" "40 2" "32 2" "56 2" "48 4" "40 4"; do
  set -- $cfg
  JT_WAIT_LANES=$1 JT_LIGHT_LANES=$2 scripts/gpu_step.sh 240 $O/f2_$1_$2.log timeout -k 10 220 python bench.py --no-cpu-baseline --no-reference-order --steps 1 --warmup 1 $F2 || exit 1
  echo "f2 W=$1 L=$2 => $(grep -h '"value"' $O/f2_$1_$2.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["value"],1), d["ms_per_step"])')" | tee -a $O/summary.txt
done
