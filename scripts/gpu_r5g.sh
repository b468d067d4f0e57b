cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_stft_mel.py tests/test_gpu_parity.py tests/test_gpu_pitch.py -x -q --timeout 300 --timeout-method thread > gpurun_out/mel_tests.log 2>&1; rc=$?; tail -3 gpurun_out/mel_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/mel_tests.log | head -20; exit $rc; }
timeout -k 10 600 python -u scripts/ab2.py --libs scripts/ab/tail.so,scripts/ab/tail2.so --cases logmel,mfcc --check --rounds 5 > gpurun_out/ab2_tail.jsonl 2> gpurun_out/ab2_tail.err; echo "rc=$?"; cat gpurun_out/ab2_tail.jsonl; tail -3 gpurun_out/ab2_tail.err
