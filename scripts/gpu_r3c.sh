# round-3 evidence: GPU suite, headline bench (CPU baseline, reference-order line), cornellbox
# roofline record, then configs 3-5 at their sizes with roofline records
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu_round.sh $1 || exit 1
bash scripts/gpu_scenes.sh $1/scenes || exit 1
