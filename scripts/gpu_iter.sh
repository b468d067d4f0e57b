#!/bin/bash
# Iteration run on the GPU box: parity tests, then kernel micro-benchmarks.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q --timeout=600 ${PYTEST_ARGS} ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
tail -15 gpurun_out/gpu_tests.log
if [ $rc -le 1 ]; then
  timeout -k 10 300 python scripts/kbench.py ${KBENCH_ARGS} > gpurun_out/kbench.log 2>&1
  echo "kbench rc=$?" >> gpurun_out/kbench.log
  cat gpurun_out/kbench.log
fi
