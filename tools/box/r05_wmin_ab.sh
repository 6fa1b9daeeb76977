#!/bin/bash
# Round 5: signed PUT sender, writev for any ready run (TRITONDL_ZC_WRITE_MIN=1,
# default) vs sendfile (no copy) while it keeps up and writev only from 2 / 4
# ready frames.  Alternated 300-job runs.
set -o pipefail
OUT=${OUT:-gpurun_out/r05_wmin_ab}
mkdir -p $OUT
export TMPDIR=/tmp
b() { local name=$1; shift; TRITONDL_ZC_TRACE=1 timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe \
      --no-reference-mode "$@" > $OUT/$name.log 2>&1; }
for i in 1 2 3; do
  b min1_$i && TRITONDL_ZC_WRITE_MIN=2 b min2_$i && TRITONDL_ZC_WRITE_MIN=4 b min4_$i || break
done
rc=$?
for f in $OUT/*.log; do
  python3 - "$f" <<'PY'
import re, sys
f = sys.argv[1]
txt = open(f).read()
v = re.search(r'"value": ([0-9.]+)', txt)
rows = [dict((k, float(x)) for k, x in re.findall(r"(\w+)=([0-9.]+)", l)) for l in txt.splitlines() if l.startswith("zc-trace")][-300:]
d = sorted(r["sent_last_us"] - r["cov_last_us"] for r in rows)
print(f.split("/")[-1], v.group(1) if v else "?", "landed->written p50 %.0f us" % d[len(d)//2] if d else "")
PY
done
exit $rc
