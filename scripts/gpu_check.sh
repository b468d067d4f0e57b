cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
if [ $rc -le 1 ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 &&
  timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench1.log 2>&1
  echo "bench rc=$?" >> gpurun_out/bench1.log
fi
tail -5 gpurun_out/gpu_tests.log; tail -2 gpurun_out/smoke.log; tail -3 gpurun_out/bench1.log
