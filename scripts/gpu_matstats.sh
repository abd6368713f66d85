# material coherence of shading phases (diagnostic stamps build, never timed numbers)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/mat
mkdir -p $O
for s in "features2 1920 1080 32" "bathroom1 1920 1080 32" "coffee 1280 720 32" "staircase2 1280 720 32" "features1 1280 720 32" "materials1 1280 720 32" "materials2 1280 720 32" "cornellbox 1280 720 32"; do
  set -- $s
  scripts/gpu_step.sh 200 $O/$1.log timeout -k 10 180 python scripts/stamps.py $4 path --scene assets/scenes/$1/$1.json --width $2 --height $3 || exit 1
done
cat $O/*.log | grep -E "spp|distinct|traversal phase"
