#!/bin/bash
# rocprofv3 kernel trace + PMC passes (each pass its own run, no --pmc beside
# any other trace domain) over kbench cases:
#   bash scripts/prof_pmc_case.sh <cases> <outdir>     (writes gpurun_out/<outdir>/)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$2
mkdir -p $O
CMD="python3 scripts/kbench.py --rounds 2 --reps 10 --cases $1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- $CMD > $O/trace.log 2>&1 || { echo "trace rc=$?"; tail -5 $O/trace.log; exit 1; }
i=0
for grp in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace -d $O/pmc$i -o run --output-format csv -- $CMD > $O/pmc$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pmc pass $i rc=$rc"; tail -3 $O/pmc$i.log; exit $rc; fi
done
python3 scripts/pmc_summary.py $O > $O/summary.txt
find $O/trace -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
grep case $O/trace.log
cat $O/summary.txt
