#!/bin/bash
# One GPU call: the -m gpu suite (all of it: failures are listed, not fatal),
# one default bench.py run, then kbench A/B cases ($KB_CASES).  Each GPU step
# has its own time limit; a crash, abort or timeout of any step ends the call.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests.log
grep -E "^FAILED|^ERROR" gpurun_out/gpu_tests.log | head -30
[ $rc -gt 1 ] && exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?
cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
[ $rc -ne 0 ] && exit $rc
if [ -n "$KB_CASES" ]; then
  timeout -k 10 400 python scripts/kbench.py --cases $KB_CASES --rounds 3 --reps 20 > gpurun_out/kb.jsonl 2> gpurun_out/kb.err
  rc=$?
  cat gpurun_out/kb.jsonl; tail -3 gpurun_out/kb.err
  exit $rc
fi
