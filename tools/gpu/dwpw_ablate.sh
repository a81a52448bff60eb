# dwpw ablation sweep: the fused kernel's launch time per epilogue mode under diagnostics builds
# (conv_dwpw.hip MLIC_DPABL bits: 1 one MFMA per k-step, 2 no depthwise math, 4 no stores, 16 all tap
# rows = centre row).  Libraries built on the CPU side as mlic_amd/libmlic_hip_dp<N>.so.
#   bash tools/gpu/dwpw_ablate.sh "1 2 4 7 16 23"
cd "$GRAFT_REPO_ROOT"
set -o pipefail
timeout -k 10 120 python3 -u tools/gpu/dwpw_ab.py base || exit $?
for N in $1; do
  MLIC_HIP_LIB=$PWD/mlic_amd/libmlic_hip_dp$N.so timeout -k 10 120 python3 -u tools/gpu/dwpw_ab.py dp$N || exit $?
done
