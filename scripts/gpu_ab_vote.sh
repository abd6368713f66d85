# step-kind vote bias (prim step when np * P >= nn * N) at reduced spp
set -o pipefail
cd $GRAFT_REPO_ROOT
AB_SCENES="f2 b1 ec cb" bash scripts/gpu_lib_ab.sh ${1:-vote} ${2:-vp2 vp3 vp4 vp8 vp64}
