# Round 5: the multi-GPU layer on the one-GPU box -- dist tests, bench node
# mode at N = 1 (--dist-c), torchrun ranks mode at world 1, the refusal at
# --gpus 2, and whether RCCL accepts two ranks on one device (expected: no).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 120 --timeout-method thread > gpurun_out/dist_tests.log 2>&1
echo "dist tests rc=$?" >> gpurun_out/dist_tests.log
tail -3 gpurun_out/dist_tests.log
grep -q "dist tests rc=0" gpurun_out/dist_tests.log || exit 1
timeout -k 10 300 python -u bench.py --dist-c --channels 8 --steps 5 --warmup 2 > gpurun_out/bench_distc.log 2>&1 || { echo "distc rc=$?"; tail -20 gpurun_out/bench_distc.log; exit 1; }
tail -c 1500 gpurun_out/bench_distc.log; echo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --dist-c --channels 8 --steps 5 --warmup 2 > gpurun_out/bench_ranks1.log 2>&1 || { echo "ranks rc=$?"; tail -20 gpurun_out/bench_ranks1.log; exit 1; }
tail -c 1500 gpurun_out/bench_ranks1.log; echo
timeout -k 10 120 python bench.py --gpus 2 --steps 1 --warmup 0 > gpurun_out/bench_gpus2.log 2>&1; echo "gpus2 rc=$? (expected non-zero)"; tail -2 gpurun_out/bench_gpus2.log
timeout -k 10 120 python -c "
import sys; sys.path.insert(0, 'vv-dsp_amd')
import torch, vvdsp_amd as vv
try:
    d = vv.Dist.all([0, 0]); print('two ranks on one device: accepted, comm_count', d.comm_count(0))
except Exception as e:
    print('two ranks on one device: refused:', e)
" > gpurun_out/dup_probe.log 2>&1; tail -3 gpurun_out/dup_probe.log
