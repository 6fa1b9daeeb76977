#!/bin/bash
# http headline: open-ended GET (default) vs a 2.5 MiB bounded GET probe with
# the rest as parallel Range streams, alternated x4, 300 timed jobs each.
set -o pipefail
OUT=${OUT:-gpurun_out/r04_probe_ab}
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2 3 4; do
  for pk in -1 2560; do
    timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe --probe-kb $pk \
        >> $OUT/http_probe$pk.log 2>&1 || exit $?
  done
done
python tools/bench_summary.py $OUT/*.log
for f in $OUT/*.log; do echo "$f"; grep -o '"job_spans_ms_p50": {[^}]*}' $f; done
