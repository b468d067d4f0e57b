#!/bin/bash
# Profiling run on the GPU box: kernel trace + stats, then PMC counter passes
# (one counter group per rocprofv3 run; never combined with sys/runtime traces).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
CASES=${CASES:-stft,c2c1024,fir}
KB="python3 scripts/kbench.py --cases $CASES --rounds 1 --reps 5"
rocprofv3 -L > gpurun_out/prof/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/trace -o run --output-format csv -- $KB > gpurun_out/prof/trace.log 2>&1 || exit 1
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace -d gpurun_out/prof/pmc$i -o run --output-format csv -- $KB > gpurun_out/prof/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 gpurun_out/prof/pmc$i.log; }
done
ls -R gpurun_out/prof | head -50
