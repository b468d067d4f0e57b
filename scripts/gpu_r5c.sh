cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_pitch.py tests/test_gpu_stft_mel.py tests/test_gpu_pow_r32.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pitch_tests.log 2>&1; rc=$?; tail -5 gpurun_out/pitch_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/pitch_tests.log | head -20; exit $rc; }
timeout -k 10 600 python -u scripts/ab2.py --libs scripts/ab/r5m.so,scripts/ab/r5m_old.so@MEL_R32=0+POW_R32=0 --cases logmel,mfcc --check --rounds 5 > gpurun_out/ab2_mel.jsonl 2> gpurun_out/ab2_mel.err; echo "rc=$?"; cat gpurun_out/ab2_mel.jsonl; tail -3 gpurun_out/ab2_mel.err
timeout -k 10 500 python -u scripts/ab2.py --libs scripts/ab/r5p.so,scripts/ab/r5p_old.so@POW_R32=0 --cases stftpow,stftpow544 --check --rounds 5 > gpurun_out/ab2_pitch.jsonl 2> gpurun_out/ab2_pitch.err; echo "rc=$?"; cat gpurun_out/ab2_pitch.jsonl; tail -3 gpurun_out/ab2_pitch.err
