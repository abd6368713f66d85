set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_step.sh 300 gpurun_out/diag_features1.log python scripts/diag_scene.py features1 || exit 1
scripts/gpu_step.sh 600 gpurun_out/hdr_experiment.log python scripts/hdr_experiment.py 256 || exit 1
