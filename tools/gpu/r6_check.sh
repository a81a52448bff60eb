cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6a
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_conv.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "dwpw or narrow or coder_lists or lanes_do_not" > gpurun_out/r6a/tests.log 2>&1; rc=$?; tail -3 gpurun_out/r6a/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u bench.py > gpurun_out/r6a/bench.json 2> gpurun_out/r6a/bench.err || { echo bench failed; tail -20 gpurun_out/r6a/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r6a/bench.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['step_frac']); print(json.dumps(d.get('decode')))"
