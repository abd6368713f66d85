# Round 4, call 5: the headline bench line (with its CPU baseline), the AMDGPU register-pressure
# trackers build A/B, the 1/N-share chunking sweep, the load-mix ceiling microbenchmark.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
scripts/gpu_step.sh 400 $O/bench.log python bench.py || exit 1
AB_SCENES="cb f2 b1 ec" AB_F2_SPP=128 AB_B1_SPP=128 AB_EC_SPP=16 bash scripts/gpu_lib_ab.sh $1/ab_trk base trk || exit 1
bash scripts/gpu_chunk_share.sh $1/chunk || exit 1
bash scripts/gpu_tdmix.sh $1/tdmix || exit 1
