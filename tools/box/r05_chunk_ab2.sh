#!/bin/bash
# Round 5 (measurement for the next round): aws-chunked payload chunk of the
# signed streaming PUT, minio-go's 64 KiB (default) vs 32 KiB vs 16 KiB (r05_chunk_ab: 256 KiB and 1 MiB lost).
# Fewer, larger frames mean fewer chunk signatures and frame headers for the
# S3 side to check.  Alternated 300-job traced runs, all arms without the
# bench's content check (the fake checks content by 64 KiB leaf digests).
set -o pipefail
OUT=${OUT:-gpurun_out/r05_chunk_ab2}
mkdir -p $OUT
export TMPDIR=/tmp
b() { local name=$1; shift; TRITONDL_TRACE=1 timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe \
      --no-reference-mode --no-content-check "$@" > $OUT/$name.log 2>&1; }
for i in 1 2 3; do
  b c64_$i &&
  TRITONDL_S3_CHUNK_KB=32 b c32_$i &&
  TRITONDL_S3_CHUNK_KB=16 b c16_$i || break
done
rc=$?
for f in $OUT/*.log; do
  echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"put_pump_start": [0-9.]*, "get_pump_end": [0-9.]*, "put_sent": [0-9.]*' $f | head -1)"
done
exit $rc
