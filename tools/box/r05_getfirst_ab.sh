#!/bin/bash
# Round 5: the get-first default confirmed in the driver's own form (`python
# bench.py`, no flags), alternated with the upload-first order (TRITONDL_GET_FIRST=0).
# (Historical: TRITONDL_GET_FIRST was removed once the single-stream fetch ran
# inline, r05_inline_ab.sh; on this tree both arms run the same order.)
set -o pipefail
OUT=${OUT:-gpurun_out/r05_getfirst_ab}
mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2 3 4 5; do
  timeout -k 10 200 python bench.py > $OUT/getfirst_$i.log 2>&1 &&
  TRITONDL_GET_FIRST=0 timeout -k 10 200 python bench.py > $OUT/uploadfirst_$i.log 2>&1 || break
done
rc=$?
for f in $OUT/*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | head -1)"; done
exit $rc
