#!/bin/bash
# Round measurement on the GPU box: the driver's bench command, then the
# rocprofv3 kernel-trace/stats and PMC (FETCH_SIZE, WRITE_SIZE) passes of the
# same command, each pass on its own (no --pmc beside any other trace domain).
#   bash scripts/gpu_bench_prof.sh           (writes gpurun_out/bprof/)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/bprof
mkdir -p $O
timeout -k 10 500 python3 bench.py > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
CMD="python3 bench.py --steps 20 --warmup 25 --no-cpu --legs c2c,fir"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- $CMD > $O/trace.log 2>&1 || { echo "trace rc=$?"; tail -5 $O/trace.log; exit 1; }
i=0
for grp in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace -d $O/pmc$i -o run --output-format csv -- $CMD > $O/pmc$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pmc pass $i rc=$rc"; tail -3 $O/pmc$i.log; [ $rc -ge 124 ] && exit $rc; fi
done
BOX="$(rocm-smi --showproductname 2>/dev/null | grep -m1 -o 'MI3[0-9A-Z]*' || echo MI355X)"
python3 scripts/pmc_summary.py $O --json $O/bench_pmc.json --channels 256 --box "$BOX, $(date -u +%F)" \
  --tail vvh::k_stft_pair=20 --tail vvh::k_c2c=50 --tail vvh::k_fir_r32=50 > $O/summary.txt
find $O/trace -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
head -40 $O/summary.txt
