#!/bin/bash
# fp32 ingest encode (configs[2], K10 at M = 65536) and more K10 tiles for the small E5 shapes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/misc; export TMPDIR=/tmp
for dt in float32 bfloat16; do
  timeout -k 10 400 python -u bench.py --mode ingest --e5-dtype $dt --steps 5 --warmup 2 --out gpurun_out/misc/ingest_$dt.json > gpurun_out/misc/ingest_$dt.log 2>&1 || { tail -20 gpurun_out/misc/ingest_$dt.log; exit 1; }
  tail -1 gpurun_out/misc/ingest_$dt.log | cut -c1-300
done
TILES="8x8 4x8" bash tools/k10_tiles.sh
