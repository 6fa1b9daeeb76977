#!/bin/bash
# Parallel multipart PUT for a 10 MiB object (2 x 5 MiB parts) A/B, https and http.
set -o pipefail
OUT=gpurun_out/r02_mpu_ab
mkdir -p $OUT
export TMPDIR=/tmp
run() { timeout -k 10 200 python -u bench.py --steps 300 --warmup 10 --no-gpu-probe "$@"; }
run --tls > $OUT/https_base.log 2>&1 &&
run --tls --s3-part-mb 5 --s3-multipart-mb 8 > $OUT/https_mpu.log 2>&1 &&
run --tls --s3-part-mb 5 --s3-multipart-mb 8 --probe-kb 2560 > $OUT/https_mpu_p2_5m.log 2>&1 &&
run > $OUT/http_base.log 2>&1 &&
run --s3-part-mb 5 --s3-multipart-mb 8 > $OUT/http_mpu.log 2>&1 &&
run --tls > $OUT/https_base2.log 2>&1
rc=$?
for f in $OUT/*.log; do echo "== $f"; grep -E '^\{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d.get('value'), d.get('cpu_ms_per_job'), d.get('job_spans_ms_p50'))"; done
exit $rc
