cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/ab2.py --libs scripts/ab/noexp.so,scripts/ab/k1.so@MAG_R32=1,scripts/ab/k2.so@STFT_CPS=1,scripts/ab/k3.so@POW_R32=1 --cases stft60,stft60x10,stft,stftpow --check --rounds 5 > gpurun_out/ab2_cfg3.jsonl 2> gpurun_out/ab2_cfg3.err; echo "rc=$?"; cat gpurun_out/ab2_cfg3.jsonl; tail -3 gpurun_out/ab2_cfg3.err
