#!/bin/bash
# One parametrised GPU call (replaces the round-5 one-off gpu_r5*.sh runners).
#   bash scripts/gpu_run.sh tests                     -m gpu suite only
#   bash scripts/gpu_run.sh ab <libs> <cases> [tests] same-buffer A/B (scripts/ab2.py), optionally after the suite
#   bash scripts/gpu_run.sh bench                     the suite, then bench + rocprof (scripts/gpu_bench_prof.sh)
#   bash scripts/gpu_run.sh pytest <pytest args...>   selected GPU tests
# Each GPU step has its own time limit; any failure ends the call.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
{ nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; grep -m1 "model name" /proc/cpuinfo; echo "OMP=$OMP_NUM_THREADS"; } > gpurun_out/box.txt
suite() {
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
  local rc=$?
  tail -3 gpurun_out/gpu_tests.log
  [ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/gpu_tests.log | head -20; exit $rc; }
  return 0
}
case "$1" in
  tests) suite ;;
  ab)
    [ "$4" = "tests" ] && suite
    timeout -k 10 900 python -u scripts/ab2.py --libs "$2" --cases "$3" --check > gpurun_out/ab2.jsonl 2> gpurun_out/ab2.err
    rc=$?; cat gpurun_out/ab2.jsonl; [ $rc -ne 0 ] && tail -20 gpurun_out/ab2.err; exit $rc ;;
  bench) suite; bash scripts/gpu_bench_prof.sh ;;
  pytest) shift
    timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread "$@" > gpurun_out/pytest_sel.log 2>&1
    rc=$?; tail -15 gpurun_out/pytest_sel.log; exit $rc ;;
  *) echo "usage: $0 tests|ab|bench|pytest ..."; exit 2 ;;
esac
