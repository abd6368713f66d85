# wide vs near per scene (after the wide_take scratch fix), features2 items vs tiles
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash scripts/gpu_wide.sh $1/wide skip-tests || exit 1
AB_SCENES="f2" bash scripts/gpu_lib_ab.sh $1/ab base tiles || exit 1
