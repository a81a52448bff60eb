# round 6: packed-attention output digests of two builds (MLIC_HIP_LIB=old vs the in-tree library), small grids saved
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/lacmp
OLD=$PWD/mlic_amd/libmlic_hip_la0.so
MLIC_HIP_LIB=$OLD timeout -k 10 60 python3 tools/gpu/la_hash.py gpurun_out/lacmp/old &&
timeout -k 10 60 python3 tools/gpu/la_hash.py gpurun_out/lacmp/new
