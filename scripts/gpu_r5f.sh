cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dyn.py tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread > gpurun_out/dyn_tests.log 2>&1; rc=$?; tail -3 gpurun_out/dyn_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/dyn_tests.log | head -20; exit $rc; }
timeout -k 10 300 python -u bench.py --dist-c --channels 16 --steps 5 --warmup 2 --gather on > gpurun_out/bench_distc.log 2>&1 || { echo "distc rc=$?"; tail -20 gpurun_out/bench_distc.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/bench_distc.log').read().strip().splitlines()[-1]);print(d['n_gpus'],d['rccl_ranks'],d['value'],d['roofline']['frac'],d.get('with_gather'))"
