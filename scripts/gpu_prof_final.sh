# Round-end evidence for the current kernel, in one call: GPU test suite, the headline bench with
# the CPU baseline, rocprofv3 kernel-trace stats and the FETCH_SIZE / WRITE_SIZE passes of the same
# bench command, PMC passes (cornellbox, bathroom1) and the large-scene bench lines.
# Afterwards (in the container): bash scripts/collect_profiles.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/final
mkdir -p $O
B="bench.py --steps 3 --warmup 1 --no-cpu-baseline"
scripts/gpu_step.sh 900 $O/pytest.log python -m pytest tests -q -m gpu -rf --timeout 600 || exit 1
scripts/gpu_step.sh 300 $O/kt.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 $B || exit 1
scripts/gpu_step.sh 300 $O/fetch.log timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o fetch -- python3 $B || exit 1
scripts/gpu_step.sh 300 $O/write.log timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o write -- python3 $B || exit 1
# traffic of this build's timed kernel (COUNT=0, the most total time) before the bench line, which reads it
K=$(python3 scripts/timed_kernel.py $O/kt/kt_kernel_stats.csv) || exit 1
python3 scripts/pmc_traffic.py $O/fetch $O/write "$K" "cornellbox path 1280x720 256 samples/launch" $O/traffic.json || exit 1
cp $O/traffic.json profiles/${ROUND:-r01}_traffic.json
scripts/gpu_step.sh 600 $O/bench.log python bench.py || exit 1
bash scripts/gpu_pmc.sh final/pmc || exit 1
NO_TESTS=1 bash scripts/gpu_scene_ab.sh final/scenes default || exit 1
nproc > $O/host.txt; lscpu | grep -E "Model name|Socket|Core|Thread" >> $O/host.txt
