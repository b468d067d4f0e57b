cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 ./vv-dsp_amd/bin/vv_dsp_dist_check > gpurun_out/distc_all.txt 2>&1; echo "rc=$?"; tail -3 gpurun_out/distc_all.txt
timeout -k 10 120 ./vv-dsp_amd/bin/vv_dsp_dist_check --loopback 3 > gpurun_out/distc_loop.txt 2>&1; echo "rc=$?"; tail -3 gpurun_out/distc_loop.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist_c.py -x -q --timeout 200 --timeout-method thread 2>&1 | tail -3
