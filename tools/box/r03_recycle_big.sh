#!/bin/bash
# Spare-file recycling on the 1 GiB job (files up to the 1 GiB pool budget are
# kept) vs delete (TRITONDL_RECYCLE_BYTES=0), alternated x3; then headline x2
# each to check the 10 MiB result holds at this tree.
set -o pipefail
OUT=${OUT:-gpurun_out/r03_recycle_big}
mkdir -p $OUT
export TMPDIR=/tmp
big() {
  local name=$1; shift
  timeout -k 10 200 python bench.py --steps 12 --warmup 2 --file-mb 1024 --no-gpu-probe "$@" > $OUT/big_$name.log 2>&1 || return $?
}
hd() {
  local name=$1; shift
  timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe "$@" > $OUT/head_$name.log 2>&1 || return $?
}
for rep in 1 2 3; do
  big recycle_$rep && TRITONDL_RECYCLE_BYTES=0 big delete_$rep || exit $?
done
for rep in 1 2; do
  hd recycle_$rep && TRITONDL_RECYCLE_BYTES=0 hd delete_$rep || exit $?
done
for f in $OUT/big_*.log $OUT/head_*.log; do
  n=$(basename $f .log)
  echo "$n $(grep -o '"value": [0-9.]*' $f) $(grep -o '"ingest_MB_per_sec": [0-9.]*' $f) $(grep -o '"cpu_ms_per_job[^}]*' $f)"
done
exit 0
