# Round 4, call 7: the GPU suite on the automatic chunk of a sixteenth of the launch, the headline
# bench line, the new chunk against the round-3 rule at the configs' own spp, the headline's 1/N
# share efficiencies.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
scripts/gpu_step.sh 600 $O/tests.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" $O/tests.log && ! grep -q "failed\|error" $O/tests.log || { echo "GPU tests not green: stopping"; exit 1; }
scripts/gpu_step.sh 400 $O/bench.log python bench.py || exit 1
run() {  # <name> <args...>
  local name=$1; shift
  scripts/gpu_step.sh 300 $O/$name.log timeout -k 10 280 python bench.py --no-cpu-baseline --no-reference-order "$@" || return 1
  echo "$name $* => $(grep -h '"value"' $O/$name.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"].get("avg_launch_ms"), d["roofline"]["launch"].split("chunk=")[1].split()[0])')" | tee -a $O/summary.txt
}
F2="--scene assets/scenes/features2/features2.json --width 1920 --height 1080 --spp 512 --steps 2 --warmup 1"
B1="--scene assets/scenes/bathroom1/bathroom1.json --width 1920 --height 1080 --spp 1024 --steps 1 --warmup 1"
EC="--scene assets/scenes/ecosys/ecosys.json --width 3840 --height 2160 --spp 64 --steps 2 --warmup 1"
for rep in 1 2; do
  run f2_new_$rep $F2 || exit 1
  run f2_old_$rep $F2 --opt chunk=128 || exit 1
  run ec_new_$rep $EC || exit 1
  run ec_old_$rep $EC --opt chunk=64 || exit 1
done
run b1_new $B1 || exit 1
run b1_old $B1 --opt chunk=256 || exit 1
run cb_full --steps 10 || exit 1
for n in 2 4 8; do run cb_n$n --steps $((10 * n)) --as-rank-of $n || exit 1; done
