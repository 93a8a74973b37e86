#!/bin/bash
# Two gloo ranks on the one GPU, deterministic mode: the N > 1 bench path with the T5 next-step
# overlap on and off must end on the same loss bit for bit (staged S = 3 and S = 1)
set -o pipefail
export TMPDIR=/tmp MMT_DETERMINISTIC=1 MMT_DIST_BACKEND=gloo
mkdir -p gpurun_out
rm -f gpurun_out/ddp_t5_check.txt
p=29620
for s in 3 1; do
  for pipe in 1 0; do
    p=$((p+1))
    MMT_T5_PIPELINE=$pipe timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $p bench.py --gpus 2 --steps 3 --warmup 1 --batch 64 --overlap-stages $s > gpurun_out/ddp_t5_$s$pipe.log 2>&1 || exit 1
    echo "S=$s MMT_T5_PIPELINE=$pipe $(grep -o '"final_loss": [0-9.]*' gpurun_out/ddp_t5_$s$pipe.log)" >> gpurun_out/ddp_t5_check.txt
  done
done
