# The one GPU driver: every gpurun call of this repository runs `bash scripts/gpu.sh <tag> <task>...`
# (outputs under gpurun_out/<tag>/; the results DESIGN.md cites are copied to profiles/).
#
# tasks, run in order; the call stops at the first GPU fault, abort or timeout (scripts/gpu_step.sh):
#   tests[:<pytest -k expr>]   the GPU test suite (or the tests matching the expression)
#   smoke                      __graft_entry__.smoke()
#   bench:<w>[:<extra args>]   one bench.py line for workload <w> (table below), with its CPU and
#                              reference-order legs unless the extra args skip them
#   quick:<w>[:<extra args>]   a bench.py line without the CPU / reference-order legs (A/B runs)
#   measure:<w>[:<extra args>] the roofline evidence of workload <w> (scripts/gpu_measure.sh)
#   sig:<w>                    write workload <w>'s one-GPU image signature (bench --write-signature)
#   ab:<w>:<lib>,<lib>...      A/B of library builds (build/libjtrace_hip[_<lib>].so, "base" = the
#                              product build), each twice, interleaved
#   prof:<w>                   rocprofv3 --kernel-trace --stats of a short bench run of workload <w>
#   stamps:<w>                 the JT_STAMPS build's per-phase wave clocks (scripts/stamps.py)
#   tdmix[:<args>]             the vector-memory gather ceilings (scripts/td_mix_bench.hip, built
#                              by `make -C julia-raytracer_amd td-mix`): rates, then TD busy / L2 hits
#   rehearse:<N>               N ranks of bench.py under torch.distributed.run on this one GPU,
#                              reducing through gloo (RCCL cannot put two ranks on one GPU)
#   host                       the box's CPU description
# workloads: cb (the headline, cornellbox path 1280x720x256), cb1 (config 1: naive 256x256x16),
#   f2 (features2 1920x1080x512), b1 (bathroom1 1920x1080x1024), ec (ecosys 3840x2160 at 64 spp),
#   ec8 (ecosys 3840x2160 at its 1/8 share, 512 spp), b1s/f2s/ecs (64/64/8 spp short forms),
#   f1s/m2s (features1 / materials2 1280x720x64: the general FT_ALL kernels);
#   a suffix /N[gG] makes it rank 0's share of an N-rank run (G tile groups), e.g. cb/8, cb/8g8.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
tag=$1
shift
O=gpurun_out/$tag
mkdir -p "$O"

wargs() {  # bench.py arguments of a workload name
    local base=${1%%/*} share=""
    [ "$base" != "$1" ] && share=${1#*/}
    local a
    case $base in
        cb) a="" ;;
        cb1) a="--width 256 --height 256 --spp 16 --sampler naive" ;;
        f2) a="--scene assets/scenes/features2/features2.json --width 1920 --height 1080 --spp 512" ;;
        f2s) a="--scene assets/scenes/features2/features2.json --width 1920 --height 1080 --spp 64" ;;
        b1) a="--scene assets/scenes/bathroom1/bathroom1.json --width 1920 --height 1080 --spp 1024" ;;
        b1s) a="--scene assets/scenes/bathroom1/bathroom1.json --width 1920 --height 1080 --spp 64" ;;
        ec) a="--scene assets/scenes/ecosys/ecosys.json --width 3840 --height 2160 --spp 64" ;;
        ecs) a="--scene assets/scenes/ecosys/ecosys.json --width 3840 --height 2160 --spp 8" ;;
        ec8) a="--scene assets/scenes/ecosys/ecosys.json --width 3840 --height 2160 --spp 4096" ;;
        f1s) a="--scene assets/scenes/features1/features1.json --width 1280 --height 720 --spp 64" ;;
        m2s) a="--scene assets/scenes/materials2/materials2.json --width 1280 --height 720 --spp 64" ;;
        *) echo "unknown workload $base" >&2; return 1 ;;
    esac
    if [ -n "$share" ]; then
        local n=${share%%g*} g=1
        [ "$share" != "$n" ] && g=${share#*g}
        a="$a --as-rank-of $n --tile-groups $g"
    fi
    echo "$a"
}
steps() {  # timed steps / warmup of a workload: about 1-4 s of GPU time
    case ${1%%/*} in
        cb|cb1) echo "--steps 10 --warmup 2" ;;
        f2|b1s|f2s|ecs|f1s|m2s) echo "--steps 3 --warmup 1" ;;
        *) echo "--steps 1 --warmup 1" ;;
    esac
}
S=scripts/gpu_step.sh
for task in "$@"; do
    kind=${task%%:*}
    rest=${task#*:}
    [ "$rest" = "$task" ] && rest=""
    w=${rest%%:*}
    extra=${rest#*:}
    [ "$extra" = "$rest" ] && extra=""
    name=$(echo "$w${extra:+_$extra}" | tr '/ ' '__')
    case $kind in
        tests)
            if [ -n "$rest" ]; then
                $S 1100 "$O/pytest.log" python -u -m pytest tests -x -v -m gpu -rf -rP --timeout 240 --timeout-method thread -k "$rest" || exit 1
            else
                $S 1100 "$O/pytest.log" python -u -m pytest tests -x -v -m gpu -rf -rP --timeout 240 --timeout-method thread || exit 1
            fi ;;
        smoke)
            $S 300 "$O/smoke.log" python -c "import __graft_entry__ as g; g.smoke()" || exit 1 ;;
        bench)
            $S 600 "$O/bench_$name.log" python bench.py $(wargs "$w") $(steps "$w") $extra || exit 1 ;;
        quick)
            $S 400 "$O/quick_$name.log" python bench.py --no-cpu-baseline --no-reference-order $(wargs "$w") $(steps "$w") $extra || exit 1 ;;
        sig)
            $S 400 "$O/sig_$name.log" python bench.py --no-cpu-baseline --no-reference-order --write-signature $(wargs "$w") --steps 1 --warmup 0 || exit 1
            cp profiles/image_signatures.json "$O/image_signatures.json" ;;
        measure)
            wl=$(python bench.py --print-workload $(wargs "$w") $extra) || exit 1
            bash scripts/gpu_measure.sh "$O/m_$name" "$wl" $(wargs "$w") $extra || exit 1 ;;
        ab)
            for rep in 1 2; do
                for lib in $(echo "$extra" | tr ',' ' '); do
                    if [ "$lib" = base ]; then L=julia-raytracer_amd/build/libjtrace_hip.so; else L=julia-raytracer_amd/build/libjtrace_hip_$lib.so; fi
                    JTRACE_LIB=$L $S 400 "$O/ab_${name}_${lib}_$rep.log" python bench.py --no-cpu-baseline --no-reference-order $(wargs "$w") $(steps "$w") || exit 1
                    echo "$w $lib rep$rep => $(grep -h '"value"' "$O/ab_${name}_${lib}_$rep.log" | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["value"],1))')" | tee -a "$O/ab_summary.txt"
                done
            done ;;
        prof)
            $S 300 "$O/prof_$name.log" rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$name" -o kt -- python3 bench.py --no-cpu-baseline --no-reference-order $(wargs "$w") --steps 2 --warmup 1 || exit 1 ;;
        stamps)
            $S 400 "$O/stamps_$name.log" python scripts/stamps.py $(wargs "$w") || exit 1 ;;
        tdmix)
            TD=julia-raytracer_amd/build/td_mix_bench
            $S 200 "$O/tdmix_rates$name.log" timeout -k 10 180 $TD $w $extra || exit 1
            $S 200 "$O/tdmix_pmc$name.log" timeout -s KILL 180 rocprofv3 --pmc TD_TD_BUSY_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d "$O/tdmix_pmc$name" -o pmc -- $TD $w $extra || exit 1 ;;
        rehearse)
            JT_BENCH_BACKEND=gloo JT_BENCH_DEVICE=0 $S 300 "$O/rehearsal_n${w}_gloo_one_gpu.log" python -m torch.distributed.run --nnodes=1 --nproc-per-node "$w" --master-addr 127.0.0.1 --master-port $((29500 + w)) bench.py --gpus "$w" --steps 3 --warmup 1 --no-cpu-baseline || exit 1 ;;
        host)
            { nproc; lscpu | grep -E "Model name|Socket|Core|Thread"; rocm-smi --showproductname 2>/dev/null | head -20; } > "$O/host.txt" 2>&1 ;;
        *) echo "unknown task $task" >&2; exit 2 ;;
    esac
done
