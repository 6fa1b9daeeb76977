#!/bin/bash
# GPU footprint round: GPU tests (lazy + idle-released HBM, torch-free load,
# streamed hybrid claims), smoke, worker RSS at job 1 with the GPU warm-up on,
# and hybrid resume time A/B: this tree vs .ab/r04_old (the hasher before
# these changes, its own native build: tools/ab_tree.sh --build HEAD~1 r04_old).
set -o pipefail
OUT=${OUT:-gpurun_out/r04_gpu}
mkdir -p $OUT
export TMPDIR=/tmp
ROOT=$PWD
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.build(); g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
timeout -k 10 300 python -m tritondl.soak --jobs 40 --torrent-jobs 2 --fail-every 0 --sample-every 1 --warmup 1 \
    --out $OUT/rss_job1.jsonl > $OUT/rss_job1.log 2>&1 || { tail -20 $OUT/rss_job1.log; exit 1; }
head -3 $OUT/rss_job1.jsonl | cut -c1-200
for rep in 1 2; do
  (cd .ab/r04_old && timeout -k 10 400 python -u tools/bench_resume.py --gb 8 --version 1 --device hybrid --reps 3) \
      > $OUT/resume_old_$rep.log 2>&1 || exit $?
  timeout -k 10 400 python -u tools/bench_resume.py --gb 8 --version 1 --device hybrid --reps 3 \
      > $OUT/resume_new_$rep.log 2>&1 || exit $?
done
for f in $OUT/resume_*.log; do echo "== $(basename $f)"; grep warm $f | cut -c1-200; done
exit 0
