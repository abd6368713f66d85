# texel pairs + LDS decode LUTs: GPU parity (scenes with textures), then A/B against HEAD
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/tex
scripts/gpu_step.sh 600 gpurun_out/tex/pytest.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scenes.py tests/test_gpu_variants.py tests/test_gpu_alias.py -x -q -m gpu --timeout 300 --timeout-method thread || exit 1
AB_SCENES="f2 b1 ec" bash scripts/gpu_lib_ab.sh tex/ab base head
