cd $GRAFT_REPO_ROOT
bash scripts/gpu_dist_check.sh > gpurun_out/dist_check.out 2>&1; echo "dist_check rc=$?" >> gpurun_out/dist_check.out
cat gpurun_out/dist_check.out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fir_dyn.py tests/test_gpu_fullsize.py -k "fir or Fir" -x -q --timeout 120 --timeout-method thread > gpurun_out/fir_tests.log 2>&1; echo "fir tests rc=$?"; tail -2 gpurun_out/fir_tests.log
timeout -k 10 400 python -u scripts/ab2.py --libs scripts/ab/prev.so,scripts/ab/bankfix.so,scripts/ab/ldpol.so --cases fir --check --rounds 6 > gpurun_out/ab2.jsonl 2> gpurun_out/ab2.err; echo "ab rc=$?"; cat gpurun_out/ab2.jsonl; tail -3 gpurun_out/ab2.err
