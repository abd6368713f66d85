# A/B of library builds on the large scenes (HBM mode): each build twice, interleaved.
# usage: bash scripts/gpu_lib_ab.sh <tag> <lib>...   (lib "base" = build/libjtrace_hip.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; shift
mkdir -p $O
SCENES=${AB_SCENES:-"f2 b1 ec"}
args() {
  case $1 in
    f2) echo "--scene assets/scenes/features2/features2.json --width 1920 --height 1080 --spp ${AB_F2_SPP:-64}" ;;
    b1) echo "--scene assets/scenes/bathroom1/bathroom1.json --width 1920 --height 1080 --spp ${AB_B1_SPP:-64}" ;;
    ec) echo "--scene assets/scenes/ecosys/ecosys.json --width 3840 --height 2160 --spp ${AB_EC_SPP:-8}" ;;
    cb) echo "--steps 10" ;;
  esac
}
for rep in 1 2; do
  for sc in $SCENES; do
    for lib in "$@"; do
      if [ "$lib" = base ]; then L=julia-raytracer_amd/build/libjtrace_hip.so; else L=julia-raytracer_amd/build/libjtrace_hip_$lib.so; fi
      JTRACE_LIB=$L scripts/gpu_step.sh 240 $O/${sc}_${lib}_$rep.log timeout -k 10 220 python bench.py --no-cpu-baseline --no-reference-order --steps 2 --warmup 1 $(args $sc) ${AB_ARGS:-} || exit 1
      echo "$sc $lib rep$rep => $(grep -h '"value"' $O/${sc}_${lib}_$rep.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["value"],1))')" | tee -a $O/summary.txt
    done
  done
done
