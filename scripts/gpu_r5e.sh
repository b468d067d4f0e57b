cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fir_dyn.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_fir_long.py tests/test_gpu_filtfilt.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fir_tests.log 2>&1; rc=$?; tail -3 gpurun_out/fir_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/fir_tests.log | head; exit $rc; }
timeout -k 10 400 python -u scripts/ab2.py --libs scripts/ab/base.so,scripts/ab/fir2d.so --cases fir --check --rounds 8 > gpurun_out/ab2_fir.jsonl 2> gpurun_out/ab2_fir.err; echo "rc=$?"; cat gpurun_out/ab2_fir.jsonl; tail -3 gpurun_out/ab2_fir.err
