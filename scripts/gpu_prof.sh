#!/bin/bash
# Profiling run on the GPU box: kernel trace + stats, then PMC counter passes
# (one counter group per rocprofv3 run; never combined with sys/runtime traces).
#   CASES=stft,c2c1024 OUT=gpurun_out/prof bash scripts/gpu_prof.sh
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/prof}
mkdir -p $OUT
CASES=${CASES:-stft,c2c1024,fir}
KB="python3 scripts/kbench.py --cases $CASES --rounds 1 --reps 5"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $KB > $OUT/trace.log 2>&1 || exit 1
i=0
while IFS= read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace -d $OUT/pmc$i -o run --output-format csv -- $KB > $OUT/pmc$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pmc pass $i ($grp) rc=$rc"; tail -3 $OUT/pmc$i.log; [ $rc -ge 124 ] && exit $rc; fi
done <<EOF
${GROUPS_OVERRIDE:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS
SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_WR GRBM_GUI_ACTIVE
TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TC_STALL_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum
TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_sum TCP_TCC_READ_REQ_sum TCC_EA0_WRREQ_STALL_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_sum
FETCH_SIZE
WRITE_SIZE}
EOF
python3 scripts/pmc_summary.py $OUT > $OUT/summary.txt 2>&1
cat $OUT/summary.txt
