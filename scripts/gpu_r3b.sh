# round-3 evidence call: tests, bench, cornellbox roofline record, PC sampling of cornellbox
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu_round.sh $1 || exit 1
