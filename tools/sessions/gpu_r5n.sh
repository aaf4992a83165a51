#!/bin/bash
# round 5: N>1 rehearsal on one GPU (gloo): self-launched ranks and torchrun, each with the CPU baseline
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
MCODEC_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 20 --warmup 3 > gpurun_out/bench_multi2_self.log 2>&1
rc=$?; tail -1 gpurun_out/bench_multi2_self.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
MCODEC_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 3 > gpurun_out/bench_multi2_torchrun.log 2>&1
rc=$?; grep '"metric"' gpurun_out/bench_multi2_torchrun.log | tail -1 | cut -c1-300; exit $rc
