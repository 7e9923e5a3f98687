#!/bin/bash
# round 5: FFN-up tile at the ingest shape (M = 65536): 192 x 192 (product pick) vs 128 x 128 (CM_K10_TILE=8x8,
# the tile qkv / o / down already use there); ingest encode alternating + kernel summaries
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/uptile; export TMPDIR=/tmp
for r in 1 2; do
  for v in pick 8x8; do
    E=""; [ $v = 8x8 ] && E="CM_K10_TILE=8x8"
    env $E timeout -k 10 300 python -u bench.py --mode ingest --e5-dtype float32 --seq-len 256 --steps 10 --warmup 3 > gpurun_out/uptile/ingest_$v.log 2>&1 || { tail -20 gpurun_out/uptile/ingest_$v.log; exit 1; }
    echo "$v $(tail -1 gpurun_out/uptile/ingest_$v.log | cut -c1-170)"
  done
done
CM_K10_TILE=8x8 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/uptile/prof -o run --output-format csv -- python3 bench.py --mode ingest --e5-dtype float32 --seq-len 256 --steps 5 --warmup 2 > gpurun_out/uptile/prof.log 2>&1 || { tail -20 gpurun_out/uptile/prof.log; exit 1; }
python3 tools/kstats.py gpurun_out/uptile/prof > gpurun_out/uptile/kernels.txt && head -8 gpurun_out/uptile/kernels.txt | cut -c1-150
