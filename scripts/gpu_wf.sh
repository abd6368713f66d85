# WF body: bitwise tests against the megakernel body, then bench sweeps (experiment launcher)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
scripts/gpu_step.sh 300 $O/pytest_wf.log timeout -k 10 280 python -u -m pytest tests/test_gpu_wf.py -x -v --timeout 60 --timeout-method thread || exit 1
grep -q " passed" $O/pytest_wf.log || exit 1
grep -q "failed" $O/pytest_wf.log && exit 1
scripts/gpu_step.sh 120 $O/bench_mk.log timeout -k 10 100 python bench.py --no-cpu-baseline --steps 2 || exit 1
for cfg in "5 56 8 1" "5 40 8 1" "5 64 8 1" "5 56 8 2" "6 56 8 1" "4 56 8 1" "5 56 16 1" "5 56 4 1"; do
  set -- $cfg
  JT_WF=1 JT_WF_GROUPS=$1 JT_WAIT_LANES=$2 JT_WF_REFILL=$3 JT_WF_SHADERS=$4 scripts/gpu_step.sh 120 $O/bench_wf_g$1_w$2_r$3_s$4.log timeout -k 10 100 python bench.py --no-cpu-baseline --steps 2 || exit 1
done
JT_WF=1 JT_WF_GROUPS=5 scripts/gpu_step.sh 120 $O/stamps_wf.log timeout -k 10 100 python scripts/stamps_wf.py 32 || exit 1
grep -h '"value"' $O/bench_*.log | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['value'], d['roofline']['launch'][:40], d['roofline']['launch'].split('wait_lanes=')[1].split()[0], d['roofline']['launch'].split('wf_groups=')[1])"
cat $O/stamps_wf.log
