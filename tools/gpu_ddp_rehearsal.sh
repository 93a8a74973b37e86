#!/bin/bash
# Two ranks on the one GPU over gloo: the N > 1 bench path (staged backward + overlapped
# all-reduce) against the sequential all-reduce path; both must end on the same loss.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_octo_gpu.py -k staged > gpurun_out/ddp_test.log 2>&1 &&
MMT_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 3 --warmup 1 --batch 64 --overlap-stages 3 > gpurun_out/ddp_s3.log 2>&1 &&
MMT_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 2 --steps 3 --warmup 1 --batch 64 --overlap-stages 1 > gpurun_out/ddp_s1.log 2>&1
