cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2 3; do timeout -k 10 120 ./vv-dsp_amd/bin/vv_dsp_dist_check --loopback 3 > gpurun_out/dl$i.txt 2> gpurun_out/dl$i.err; echo "run $i rc=$?"; tail -c 600 gpurun_out/dl$i.err; done
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist_c.py -x -v --timeout 200 --timeout-method thread > gpurun_out/distc_pytest.log 2>&1; echo "rc=$?"; grep -E "_stderr|assert" gpurun_out/distc_pytest.log | head -10
