# GPU call: same-buffer A/B of library builds (scripts/ab2.py) after the -m gpu suite.
#   bash scripts/gpu_ab2.sh <libs comma-separated> <cases> [skip-tests]
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
if [ -z "$3" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
  rc=$?
  tail -3 gpurun_out/gpu_tests.log
  [ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/gpu_tests.log | head -20; exit $rc; }
fi
timeout -k 10 900 python -u scripts/ab2.py --libs "$1" --cases "$2" --check > gpurun_out/ab2.jsonl 2> gpurun_out/ab2.err
rc=$?
cat gpurun_out/ab2.jsonl
[ $rc -ne 0 ] && tail -20 gpurun_out/ab2.err
exit $rc
