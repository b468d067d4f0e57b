#!/bin/bash
# rocprofv3 kernel trace of a few kbench cases: bash scripts/prof_case.sh <cases> <outdir>
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$2
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 scripts/kbench.py --rounds 2 --reps 10 --cases $1 > $O/trace.log 2>&1 || { echo "trace rc=$?"; tail -5 $O/trace.log; exit 1; }
find $O/trace -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
cut -d, -f1-4 $O/kernel_stats.csv | head -20
grep case $O/trace.log
