set -o pipefail
for lib in r0 r1 r2; do
  for rep in 1 2; do
    for c in "2 192 68 120 65" "3 192 20 96 64" "1 160 36 64 65"; do
      if [ -n "$lib" ]; then export MLIC_HIP_LIB=$PWD/mlic_amd/libmlic_hip_$lib.so; else unset MLIC_HIP_LIB; fi
      echo "lib=${lib:-main} rep=$rep"; timeout -k 10 60 python3 tools/gpu/dwpw2_diag.py $c || exit 1
    done
  done
done
export MLIC_HIP_LIB=$PWD/mlic_amd/libmlic_hip_r3.so D2_REF_NORES=1
for rep in 1 2; do for c in "2 192 68 120 65" "3 192 20 96 64" "1 160 36 64 65"; do echo "lib=r3 rep=$rep"; timeout -k 10 60 python3 tools/gpu/dwpw2_diag.py $c || exit 1; done; done
