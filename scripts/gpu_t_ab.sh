# GPU call: selected -m gpu tests (pattern $1), then an ab2 run ($2 libs, $3 cases)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$1" > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/gpu_tests.log | head -20; exit $rc; }
bash scripts/gpu_ab2.sh "$2" "$3" skip
