# quick GPU iteration: selected tests then selected kbench cases
#   bash scripts/gpu_iter.sh "<pytest -k expr or file list>" "<kbench cases>"
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest $1 -x -v --timeout 120 --timeout-method thread > gpurun_out/iter_tests.log 2>&1
rc=$?
tail -15 gpurun_out/iter_tests.log
[ $rc -ne 0 ] && exit $rc
if [ -n "$2" ]; then
  timeout -k 10 400 python -u scripts/kbench.py --reps 10 --rounds 2 --cases "$2" > gpurun_out/iter_kbench.log 2>&1
  rc=$?
  cat gpurun_out/iter_kbench.log | tail -30
  exit $rc
fi
