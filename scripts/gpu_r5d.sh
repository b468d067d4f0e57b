cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/ab2.py --libs scripts/ab/c3a.so,scripts/ab/c3b.so@MAG_R32=1,scripts/ab/c3c.so@STFT_CPS=1 --cases stft60,stft60x10 --check --rounds 6 > gpurun_out/ab2_cfg3.jsonl 2> gpurun_out/ab2_cfg3.err; echo "rc=$?"; cat gpurun_out/ab2_cfg3.jsonl; tail -3 gpurun_out/ab2_cfg3.err
timeout -k 10 120 python -u scripts/cfg3_trace.py > gpurun_out/cfg3_plain.txt 2>&1; cat gpurun_out/cfg3_plain.txt | tail -2
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cfg3 -o cfg3 -- python3 scripts/cfg3_trace.py > gpurun_out/cfg3_prof.txt 2>&1; echo "prof rc=$?"; tail -2 gpurun_out/cfg3_prof.txt
find gpurun_out/prof_cfg3 -name "*stats*" | head
