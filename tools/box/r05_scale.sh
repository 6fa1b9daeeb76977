#!/bin/bash
# Round 5: multi-rank rehearsal of the driver's scaling run on the 1-GPU box: 1/2/4/8
# ranks on ONE shared broker (gloo control plane; the box's 16-CPU quota is
# shared by every rank), with per-job payload variants and the S3 content check.
set -o pipefail
OUT=${OUT:-gpurun_out/r05_scale}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python bench.py --gpus 1 --steps 100 --warmup 10 --no-gpu-probe > $OUT/n1.log 2>&1 || exit $?
for n in 2 4 8; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $((29500 + n)) bench.py --gpus $n --steps 100 --warmup 10 --no-gpu-probe --dist-backend gloo \
      > $OUT/n$n.log 2>&1 || exit $?
done
for n in 1 2 4 8; do echo "n=$n $(grep -o '"value": [0-9.]*' $OUT/n$n.log) $(grep -o '"jobs_per_rank": [^]]*]' $OUT/n$n.log) $(grep -o '"broker_core_share": [0-9.]*' $OUT/n$n.log)"; done
