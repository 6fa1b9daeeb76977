#!/bin/bash
# Round 5, end of session: does batching still help the 10 MiB headline now that
# the sender follows the download (frontier-aware claims) and sends its final
# frame first?  6 alternated 300-job runs each, batched (default) vs not.
set -o pipefail
OUT=${OUT:-gpurun_out/r05_batch_ab3}
mkdir -p $OUT
export TMPDIR=/tmp
b() { local name=$1; shift; timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe \
      --no-reference-mode "$@" > $OUT/$name.log 2>&1; }
for i in 1 2 3 4 5 6; do
  b batch_$i && TRITONDL_ZC_WRITE_BATCH=0 b sendfile_$i || break
done
rc=$?
for f in $OUT/*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | head -1)"; done
exit $rc
