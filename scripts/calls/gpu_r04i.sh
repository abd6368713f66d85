# Round 4, call 6: the multi-rank bench rehearsal with the pipelined reduce (N=2, 4 on one GPU over
# gloo), then the chunk sweep on full launches and the headline's shares.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash scripts/gpu_rehearse.sh $1/rehearse || exit 1
bash scripts/gpu_chunk_full.sh $1/chunk || exit 1
