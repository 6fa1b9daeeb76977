#!/usr/bin/env bash
# HTTP/2 striping A/B on an MI355X box: HTTP/1.1 vs HTTP/2 native (4 connections / 1) vs asyncio.
# Usage (repo root, GPU box): bash tools/h2_box2.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/r06_h2_box2}
mkdir -p "$out"
export TMPDIR=/tmp
echo "[$(date +%T)] h2_ab"
timeout -k 10 900 python tools/h2_ab.py --runs 3 --out "$out/h2_ab" > "$out/h2_ab.log" 2>&1 || exit 1
echo "[$(date +%T)] h2_ab done"
tail -n 6 "$out/h2_ab.log"
