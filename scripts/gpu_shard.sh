# Per-GPU throughput of the strong-scaling shards: bench.py at N ranks renders 256/N samples per
# GPU (samples [r*256/N, (r+1)*256/N)), so the one-GPU rate at 32/64/128 spp bounds the N=8/4/2
# efficiency. Also the work-unit size at 32 spp (options chunk, chunk_min).
# usage: bash scripts/gpu_shard.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
mkdir -p $O
run() {  # name "--opt k=v ..." bench-args...
  local name=$1 opts=$2; shift 2
  scripts/gpu_step.sh 120 $O/$name.log python bench.py --no-cpu-baseline --no-reference-order $opts "$@" || exit 1
  echo "$name $opts => $(grep -h '"value"' $O/$name.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["value"],1), d["ms_per_step"])')" | tee -a $O/summary.txt
}
run s256 "" --steps 10 --spp 256
run s128 "" --steps 20 --spp 128
run s64 "" --steps 40 --spp 64
run s32 "" --steps 80 --spp 32
run s32_c4 "--opt chunk=4" --steps 80 --spp 32
run s32_c16 "--opt chunk=16" --steps 80 --spp 32
run s32_c8m4 "--opt chunk=8 --opt chunk_min=4" --steps 80 --spp 32
run s32_c16m4 "--opt chunk=16 --opt chunk_min=4" --steps 80 --spp 32
run s64_c8 "--opt chunk=8" --steps 40 --spp 64
run s64_c32m8 "--opt chunk=32 --opt chunk_min=8" --steps 40 --spp 64
