#!/bin/bash
# Round 5: the https job with more than one job in flight (the fakes' single TLS streams bound one
# job at a time); per-stage worker CPU and fake core shares for each.
set -o pipefail
OUT=${OUT:-gpurun_out/r05_https2}
mkdir -p $OUT
export TMPDIR=/tmp
b() { local name=$1; shift; timeout -k 10 240 python bench.py --no-gpu-probe --no-reference-mode "$@" > $OUT/$name.log 2>&1; }
b https_c1 --steps 300 --warmup 10 --tls &&
b https_c2 --steps 400 --warmup 10 --tls --concurrency 2 &&
b https_c4 --steps 600 --warmup 20 --tls --concurrency 4 &&
b https_c2_probe2560 --steps 400 --warmup 10 --tls --concurrency 2 --probe-kb 2560 &&
b http_c2 --steps 400 --warmup 10 --concurrency 2 &&
b http_c4 --steps 600 --warmup 20 --concurrency 4 &&
TRITONDL_BENCH_LOOP_PROFILE=$OUT/loop.prof b http_c1_loopprof --steps 600 --warmup 20
rc=$?
python -c "import pstats; pstats.Stats('$OUT/loop.prof').sort_stats('tottime').print_stats(40)" > $OUT/loop_top.txt 2>&1
for f in $OUT/*.log; do
  python - "$f" <<'PY'
import json, sys
f = sys.argv[1]
try:
    d = json.loads([l for l in open(f) if l.startswith("{")][-1])
except Exception:
    print(f, "no result"); sys.exit(0)
c = d.get("cpu_ms_per_job") or {}
print(f.split("/")[-1][:-4], d["value"], "p50", d.get("job_latency_ms_p50"), "recv", c.get("worker_recv"),
      "send", c.get("worker_send"), "worker", c.get("worker"), "origin", c.get("origin"), "s3", c.get("s3"),
      "share", d.get("fake_core_share"))
PY
done
exit $rc
