#!/bin/bash
# A/B: bounded GET probe + in-order stripes pulled by 4 streams, http and https, 10 MiB job.
set -o pipefail
OUT=gpurun_out/r02_stripe_ab
mkdir -p $OUT
export TMPDIR=/tmp
run() { timeout -k 10 200 python -u bench.py --steps 200 --warmup 10 --no-gpu-probe "$@"; }
for tls in "" "--tls"; do
  t=$( [ -n "$tls" ] && echo https || echo http )
  run $tls --probe-kb 0 > $OUT/${t}_base.log 2>&1 || exit $?
  for cfg in "1024 1024" "1024 512" "2048 1024" "512 512"; do
    set -- $cfg
    run $tls --probe-kb $1 --stripe-kb $2 > $OUT/${t}_p$1_s$2.log 2>&1 || exit $?
  done
done
for f in $OUT/*.log; do echo "== $f"; grep -E '^\{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['job_spans_ms_p50'])"; done
