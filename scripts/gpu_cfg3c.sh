# GPU call: config 3's streaming ceiling (scripts/cfg3_ceiling.py)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/cfg3_ceiling.py > gpurun_out/cfg3c.jsonl 2> gpurun_out/cfg3c.err
rc=$?; cat gpurun_out/cfg3c.jsonl; [ $rc -ne 0 ] && tail -20 gpurun_out/cfg3c.err; exit $rc
