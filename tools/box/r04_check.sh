#!/bin/bash
# Current tree on the box: the multi-GPU collective path (torchrun, RCCL
# max-reduce) with one rank, the GPU tests, smoke, and the driver's command.
set -o pipefail
OUT=${OUT:-gpurun_out/r04_check}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.log 2>&1 &&
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29633 bench.py --gpus 1 --dist-always --steps 20 --warmup 5 > $OUT/rccl_1rank.log 2>&1 &&
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.build(); g.smoke()" > $OUT/smoke.log 2>&1
rc=$?
tail -2 $OUT/pytest_gpu.log; tail -1 $OUT/smoke.log
for f in $OUT/bench_driver.log $OUT/rccl_1rank.log; do
  echo "$(basename $f) $(grep -o '"value": [0-9.]*\|"collectives": "[^"]*"' $f | tr '\n' ' ')"
done
exit $rc
