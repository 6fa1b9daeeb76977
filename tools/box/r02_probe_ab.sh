#!/bin/bash
# A/B of the bounded GET probe (parallel Range streams for a 10 MiB file), http and https.
set -o pipefail
OUT=gpurun_out/r02_probe_ab
mkdir -p $OUT
export TMPDIR=/tmp
for tls in "" "--tls"; do
  for kb in 0 1024 2560; do
    tag=$( [ -n "$tls" ] && echo https || echo http )_probe${kb}
    timeout -k 10 200 python -u bench.py --steps 200 --warmup 10 --no-gpu-probe --probe-kb $kb $tls > $OUT/$tag.log 2>&1 || exit $?
  done
done
for f in $OUT/*.log; do echo "== $f"; grep -E '^\{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['job_spans_ms_p50'])"; done
