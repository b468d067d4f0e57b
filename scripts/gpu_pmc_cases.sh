#!/bin/bash
# rocprofv3 PMC passes over kbench cases, split per case (kbench --mark + scripts/pmc_cases.py).
#   bash scripts/gpu_pmc_cases.sh "<cases>" "<pass1 counters>" ["<pass2 counters>" ...]
# Every pass is its own process (so its own buffer placement): the kernel-trace
# duration of each case is printed beside its counters.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/pmccases
mkdir -p $O
cases="$1"
shift
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace -d $O/p$i -o run --output-format csv -- \
      python3 scripts/kbench.py --mark --rounds 2 --reps 5 --cases "$cases" > $O/p$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pass $i rc=$rc"; tail -5 $O/p$i.log; exit $rc; fi
  echo "== pass $i: $grp"
  grep '^{' $O/p$i.log
  python3 scripts/pmc_cases.py $O/p$i --cases "$cases" --kernel "${KERNEL:-vvh::k_stft_pair}"
done
