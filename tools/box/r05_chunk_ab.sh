#!/bin/bash
# Round 5 (measurement for the next round): aws-chunked payload chunk of the
# signed streaming PUT, minio-go's 64 KiB (default) vs 256 KiB vs 1 MiB.
# Fewer, larger frames mean fewer chunk signatures and frame headers for the
# S3 side to check.  Alternated 300-job traced runs.
set -o pipefail
OUT=${OUT:-gpurun_out/r05_chunk_ab}
mkdir -p $OUT
export TMPDIR=/tmp
b() { local name=$1; shift; TRITONDL_TRACE=1 timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe \
      --no-reference-mode "$@" > $OUT/$name.log 2>&1; }
for i in 1 2 3; do
  b c64_$i &&
  TRITONDL_S3_CHUNK_KB=256 b c256_$i &&
  TRITONDL_S3_CHUNK_KB=1024 b c1024_$i || break
done
rc=$?
for f in $OUT/*.log; do
  echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"put_pump_start": [0-9.]*, "get_pump_end": [0-9.]*, "put_sent": [0-9.]*' $f | head -1)"
done
exit $rc
