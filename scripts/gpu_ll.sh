# light_lanes (light-hit step threshold) sweep on bathroom1 (the HBM-mode scene with light-hit steps)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-ll}
mkdir -p $O
B1="--scene assets/scenes/bathroom1/bathroom1.json --width 1920 --height 1080 --spp 1024"
for l in 2 4 8 16 65; do
  JT_LIGHT_LANES=$l scripts/gpu_step.sh 240 $O/b1_$l.log timeout -k 10 220 python bench.py --no-cpu-baseline --no-reference-order --steps 1 --warmup 1 $B1 || exit 1
  echo "b1 light_lanes=$l => $(grep -h '"value"' $O/b1_$l.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["value"],1), d["ms_per_step"])')" | tee -a $O/summary.txt
done
