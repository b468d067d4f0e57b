#!/bin/bash
# rocprofv3 kernel trace + PMC passes over scripts/ab2.py cases of the in-tree library
# (one counter group per rocprofv3 run, never combined with other trace domains).
#   bash scripts/gpu_pmc_ab.sh <cases> [outdir]      -> <outdir>/summary.txt (scripts/pmc_summary.py)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${2:-gpurun_out/pmcab}
mkdir -p $O
LIB=${LIB:-vv-dsp_amd/lib/libvvdsp_amd.so}   # a build spec as scripts/ab2.py takes it (path[@KNOB=V])
AB="python3 scripts/ab2.py --libs $LIB --cases $1 --rounds 1 --reps 10"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- $AB > $O/trace.log 2>&1 || { echo "trace rc=$?"; tail -5 $O/trace.log; exit 1; }
i=0
for grp in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace -d $O/pmc$i -o run --output-format csv -- $AB > $O/pmc$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pmc pass $i rc=$rc"; tail -3 $O/pmc$i.log; exit $rc; fi
done
python3 scripts/pmc_summary.py $O > $O/summary.txt
grep '^{' $O/trace.log
head -120 $O/summary.txt
