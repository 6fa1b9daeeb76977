#!/bin/bash
# Round 5: the 1 GiB job (4 Range streams, 16 MiB parts x 4 in flight) with the
# round-5 sender changes (frontier-aware claims, batched writev) vs each of them
# off.  Alternated 6-job runs.
set -o pipefail
OUT=${OUT:-gpurun_out/r05_gib_ab}
mkdir -p $OUT
export TMPDIR=/tmp
b() { local name=$1; shift; timeout -k 10 240 python bench.py --file-mb 1024 --steps 6 --warmup 1 --no-gpu-probe \
      --no-reference-mode "$@" > $OUT/$name.log 2>&1; }
for i in 1 2 3; do
  b now_$i &&
  TRITONDL_SHA_MB_FOLLOW=0 b nofollow_$i &&
  TRITONDL_ZC_WRITE_BATCH=0 b nobatch_$i || break
done
rc=$?
for f in $OUT/*.log; do
  echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"ingest_MB_per_sec": [0-9.]*' $f | head -1)"
done
exit $rc
