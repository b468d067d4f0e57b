cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_pitch.py tests/test_gpu_stft_mel.py tests/test_gpu_pow_r32.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pitch_tests.log 2>&1; rc=$?; tail -5 gpurun_out/pitch_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/pitch_tests.log | head -20; exit $rc; }
timeout -k 10 500 python -u scripts/ab2.py --libs scripts/ab/noexp.so,scripts/ab/k1.so@MAG_R32=1,scripts/ab/k2.so@STFT_CPS=1 --cases stft60,stft60x10 --check --rounds 5 > gpurun_out/ab2_cfg3.jsonl 2> gpurun_out/ab2_cfg3.err; echo "rc=$?"; cat gpurun_out/ab2_cfg3.jsonl; tail -3 gpurun_out/ab2_cfg3.err
timeout -k 10 500 python -u scripts/ab2.py --libs scripts/ab/pitch.so,scripts/ab/pitch_r32.so@POW_R32=1 --cases stftpow,stftpow544 --check --rounds 5 > gpurun_out/ab2_pitch.jsonl 2> gpurun_out/ab2_pitch.err; echo "rc=$?"; cat gpurun_out/ab2_pitch.jsonl; tail -3 gpurun_out/ab2_pitch.err
