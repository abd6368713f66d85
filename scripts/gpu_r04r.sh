# Round 4: smoke() on the final build (checked against the oracle in the order the library
# resolved), then an A/B of the traversal scheduling knobs after the round's scheduling changes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
scripts/gpu_step.sh 300 $O/smoke.log timeout -k 10 280 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
grep -q "smoke ok" $O/smoke.log || { echo "smoke failed: stopping"; exit 1; }
AB_SCENES="cb" bash scripts/gpu_lib_ab.sh $1/ab_cb base nr3 nr5 vp2 vp4 fp2 if0 || exit 1
AB_SCENES="b1 ec" AB_B1_SPP=128 AB_EC_SPP=16 bash scripts/gpu_lib_ab.sh $1/ab_hbm base hnr2 hnr4 vp2 vp4 if0 || exit 1
