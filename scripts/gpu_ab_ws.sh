# shading gate scaled with the unit's remaining lanes (JT_WAIT_SCALE): A/B at the configs' spp
set -o pipefail
cd $GRAFT_REPO_ROOT
AB_F2_SPP=512 AB_B1_SPP=1024 AB_EC_SPP=64 AB_SCENES="cb f2 b1 ec" bash scripts/gpu_lib_ab.sh ws/ab base ws0
