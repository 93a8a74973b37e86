#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for s in 1 3 1 3; do
MMT_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 2962$s bench.py --gpus 2 --steps 3 --warmup 1 --batch 64 --overlap-stages $s > gpurun_out/ddp_x.log 2>&1 || exit 1
echo "S=$s $(grep -o '"final_loss": [0-9.]*' gpurun_out/ddp_x.log)"
done
