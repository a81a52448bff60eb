cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools_debug_lrp.py > gpurun_out/debug_lrp.log 2>&1
echo rc=$? >> gpurun_out/debug_lrp.log
