#!/bin/bash
# Round 5: where the https job's time goes (worker pumps vs each fake), and what moves it.
set -o pipefail
OUT=${OUT:-gpurun_out/r05_https}
mkdir -p $OUT
export TMPDIR=/tmp
# three idle L3 domains on one NUMA node: one for the worker, two for the fakes
read RANK FAKES < <(python - <<'PY'
from tritondl.parallel import topology as t
doms = t.l3_domains()
busy = t.domain_busy(doms)
order = t.idle_first(doms, busy)
node = t.numa_node_of(order[0][0])
same = [d for d in order if t.numa_node_of(d[0]) == node]
f = lambda d: ",".join(map(str, d))
print(f(same[0]), f(same[1] + same[2]))
PY
)
echo "rank cpus $RANK; fake cpus $FAKES"
b() { local name=$1; shift; timeout -k 10 240 python bench.py --no-gpu-probe --no-reference-mode "$@" > $OUT/$name.log 2>&1; }
b http_default --steps 300 --warmup 10 &&
b https_default --steps 300 --warmup 10 --tls &&
b https_fakes_2ccd --steps 300 --warmup 10 --tls --cpus "$RANK" --fake-cpus "$FAKES" &&
b https_no_content_check --steps 300 --warmup 10 --tls --no-content-check &&
b https_probe2560 --steps 300 --warmup 10 --tls --probe-kb 2560 &&
b https_probe2560_fakes_2ccd --steps 300 --warmup 10 --tls --probe-kb 2560 --cpus "$RANK" --fake-cpus "$FAKES" &&
b https_multipart5 --steps 300 --warmup 10 --tls --s3-multipart-mb 8 --s3-part-mb 5 &&
b https_probe_multipart_fakes_2ccd --steps 300 --warmup 10 --tls --probe-kb 2560 --s3-multipart-mb 8 --s3-part-mb 5 --cpus "$RANK" --fake-cpus "$FAKES" &&
b https_default_again --steps 300 --warmup 10 --tls
rc=$?
for f in $OUT/*.log; do
  python - "$f" <<'PY'
import json, sys
f = sys.argv[1]
try:
    d = json.loads([l for l in open(f) if l.startswith("{")][-1])
except Exception as e:
    print(f, "no result"); sys.exit(0)
print(f.split("/")[-1][:-4], d["value"], "fetched", d["job_spans_ms_p50"].get("fetched"), "upload", d["job_spans_ms_p50"].get("upload"),
      "cpu", d.get("cpu_ms_per_job"), "share", d.get("fake_core_share"))
PY
done
exit $rc
