#!/bin/bash
# One GPU call: the -m gpu suite, then (only if it passed) the bench + rocprof
# kernel-stats + PMC passes (scripts/gpu_bench_prof.sh).  Each GPU step has its
# own time limit; any failure ends the call.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
{ nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; grep -m1 "model name" /proc/cpuinfo; echo "OMP=$OMP_NUM_THREADS"; } > gpurun_out/box.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/gpu_tests.log | head -20; exit $rc; }
[ "$1" = "tests" ] && exit 0
bash scripts/gpu_bench_prof.sh
