#!/bin/bash
# GPU call: the -m gpu suite, then an A/B of two library builds (scripts/abbench.py).
#   bash scripts/gpu_ab.sh <cases> [pairs]      A = scripts/ab/prev.so, B = the in-tree library
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/gpu_tests.log | head -20; exit $rc; }
timeout -k 10 900 python -u scripts/abbench.py --a scripts/ab/prev.so --b vv-dsp_amd/lib/libvvdsp_amd.so \
    --cases "$1" --pairs "${2:-3}" > gpurun_out/ab.jsonl 2> gpurun_out/ab.err
rc=$?
cat gpurun_out/ab.jsonl
[ $rc -ne 0 ] && tail -20 gpurun_out/ab.err
exit $rc
