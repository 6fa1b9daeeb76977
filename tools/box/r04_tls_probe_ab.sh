#!/bin/bash
# https headline: one open-ended GET (default) vs a bounded GET probe with the
# rest of the file as parallel Range streams (decryption spread over cores).
set -o pipefail
OUT=${OUT:-gpurun_out/r04_tls_probe_ab}
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for pk in -1 2560 1024; do
    timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe --tls --probe-kb $pk \
        >> $OUT/tls_probe$pk.log 2>&1 || exit $?
  done
done
timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe --probe-kb 2560 >> $OUT/http_probe2560.log 2>&1
timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe >> $OUT/http_default.log 2>&1
python tools/bench_summary.py $OUT/*.log
for f in $OUT/*.log; do echo "$f $(grep -o '"job_spans_ms_p50": {[^}]*}' $f | head -1)"; done
