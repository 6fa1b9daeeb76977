#!/bin/bash
# Round 5, end of session: GPU tests, build()+smoke(), the driver's bench form
# three times, the RCCL one-rank path, the reference (cleanup-off) mode.
set -o pipefail
OUT=${OUT:-gpurun_out/r05_final_check}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.build(); g.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 200 python bench.py > $OUT/bench_default_1.log 2>&1 &&
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver_1.log 2>&1 &&
timeout -k 10 200 python bench.py > $OUT/bench_default_2.log 2>&1 &&
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver_2.log 2>&1 &&
timeout -k 10 200 python bench.py > $OUT/bench_default_3.log 2>&1 &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 1 --dist-always > $OUT/bench_rccl.log 2>&1
rc=$?
tail -2 $OUT/pytest_gpu.log; tail -1 $OUT/smoke.log
for f in $OUT/bench_*.log; do
  echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | head -1) ref_mode=$(grep -o '"reference_mode": {"cleanup": false, "jobs_per_sec": [0-9.]*' $f | grep -o '[0-9.]*$')"
done
exit $rc
