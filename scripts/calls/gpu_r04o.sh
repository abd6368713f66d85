# Round 4, call 12: the shading gate (wait_lanes) re-swept after the work items, the short chunks
# and the auto traversal, on every bench scene.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
run() {  # <name> <args...>
  local name=$1; shift
  scripts/gpu_step.sh 300 $O/$name.log timeout -k 10 280 python bench.py --no-cpu-baseline --no-reference-order "$@" || return 1
  echo "$name $* => $(grep -h '"value"' $O/$name.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); l=d["roofline"]["launch"]; print(d["value"], d["ms_per_step"], l.split("wait_lanes=")[1].split()[0], d["config"]["traversal"])')" | tee -a $O/summary.txt
}
for rep in 1 2; do
  run cb_default_$rep --steps 10 || exit 1
  for w in 48 52 60 64; do run cb_w${w}_$rep --steps 10 --opt wait_lanes=$w || exit 1; done
done
F2="--scene assets/scenes/features2/features2.json --width 1920 --height 1080 --spp 128 --steps 2 --warmup 1"
B1="--scene assets/scenes/bathroom1/bathroom1.json --width 1920 --height 1080 --spp 128 --steps 2 --warmup 1"
EC="--scene assets/scenes/ecosys/ecosys.json --width 3840 --height 2160 --spp 16 --steps 2 --warmup 1"
run f2_default $F2 || exit 1
for w in 48 56 64; do run f2_w$w $F2 --opt wait_lanes=$w || exit 1; done
run b1_default $B1 || exit 1
for w in 16 24 40 48; do run b1_w$w $B1 --opt wait_lanes=$w || exit 1; done
run ec_default $EC || exit 1
for w in 8 24 32; do run ec_w$w $EC --opt wait_lanes=$w || exit 1; done
