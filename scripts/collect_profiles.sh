# Copy the round-end evidence written by scripts/gpu_prof_final.sh (gpurun_out/final) into profiles/.
set -e
cd "$(dirname "$0")/.."
O=gpurun_out/final
R=${ROUND:-r01}
grep '^{' $O/bench.log > profiles/${R}_bench.log
cp $O/kt/kt_kernel_stats.csv profiles/${R}_kernel_stats.csv
cp $O/traffic.json profiles/${R}_traffic.json
mkdir -p profiles/${R}_pmc profiles/${R}_scenes
cp $O/pmc/cb_summary.txt profiles/${R}_pmc/cornellbox_lds_64spp.txt
cp $O/pmc/b1_summary.txt profiles/${R}_pmc/bathroom1_hbm_1920x1080_16spp.txt
for s in F2 B1 EC; do grep -h '^{' $O/scenes/bench_${s}_default.log > profiles/${R}_scenes/bench_$(echo $s | tr A-Z a-z).log; done
cp $O/pytest.log profiles/${R}_pytest_gpu.log
cp $O/host.txt profiles/${R}_host.txt
echo "collected into profiles/ (${R})"
