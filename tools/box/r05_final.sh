#!/bin/bash
# Round-5 tree on one MI355X box: GPU tests, build()+smoke(), the driver's bench form, a 300-job run,
# the reference's cleanup-off mode, and the RCCL 1-rank collective path (torchrun).
set -o pipefail
OUT=${OUT:-gpurun_out/r05_final}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.build(); g.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $OUT/bench_driver.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe > $OUT/bench_300.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe --cleanup off --no-reference-mode > $OUT/bench_300_cleanup_off.log 2>&1 &&
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29543 bench.py --gpus 1 --steps 100 --warmup 5 --dist-always --no-gpu-probe > $OUT/rccl_1rank.log 2>&1
rc=$?
tail -3 $OUT/pytest_gpu.log; tail -2 $OUT/smoke.log
for f in $OUT/bench_*.log $OUT/rccl_1rank.log; do echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"reference_mode": {"cleanup": false, "jobs_per_sec": [0-9.]*' $f)"; done
exit $rc
