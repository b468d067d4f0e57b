#!/bin/bash
# kbench cases only (lab / model / product A/B), one process, own time limit.
#   bash scripts/gpu_kb.sh "<cases>" [rounds] [reps]     -> gpurun_out/kb.jsonl
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u scripts/kbench.py --rounds "${2:-3}" --reps "${3:-10}" --cases "$1" > gpurun_out/kb.jsonl 2> gpurun_out/kb.err
rc=$?
cat gpurun_out/kb.jsonl
[ $rc -ne 0 ] && tail -20 gpurun_out/kb.err
exit $rc
