cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 ./vv-dsp_amd/bin/vv_dsp_dist_check > gpurun_out/distc_all.txt 2>&1; echo "rc=$?"; tail -3 gpurun_out/distc_all.txt
timeout -k 10 120 ./vv-dsp_amd/bin/vv_dsp_dist_check --loopback 3 > gpurun_out/distc_loop.txt 2>&1; echo "rc=$?"; tail -3 gpurun_out/distc_loop.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist_c.py -x -q --timeout 200 --timeout-method thread 2>&1 | tail -3
timeout -k 10 500 python3 bench.py --no-cpu > gpurun_out/bench_r5h.json 2> gpurun_out/bench_r5h.err; echo "bench rc=$?"
python3 -c "
import json;d=json.loads(open('gpurun_out/bench_r5h.json').read().strip().splitlines()[-1])
print('headline', d['roofline']['frac'], d['ms_per_step'])
for k in ('fft_c2c_1024','fir_ols_257','stft_config3','config5_shard_32ch'):
    v=d[k]; print(k, v.get('frac'), v.get('ms_avg'), v.get('ms_avg_isolated'))
"
