#!/bin/bash
# round 5: every projection on 192 x 192 tiles at the ingest shape (CM_K10_TILE=12x12) vs the product pick (qkv, o, down on 128 x 128)
# ingest encode alternating + kernel summaries
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/alltile; export TMPDIR=/tmp
for r in 1 2; do
  for v in pick 12x12; do
    E=""; [ $v = 12x12 ] && E="CM_K10_TILE=12x12"
    env $E timeout -k 10 300 python -u bench.py --mode ingest --e5-dtype float32 --seq-len 256 --steps 10 --warmup 3 > gpurun_out/alltile/ingest_$v.log 2>&1 || { tail -20 gpurun_out/alltile/ingest_$v.log; exit 1; }
    echo "$v $(tail -1 gpurun_out/alltile/ingest_$v.log | cut -c1-170)"
  done
done
CM_K10_TILE=12x12 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/alltile/prof -o run --output-format csv -- python3 bench.py --mode ingest --e5-dtype float32 --seq-len 256 --steps 5 --warmup 2 > gpurun_out/alltile/prof.log 2>&1 || { tail -20 gpurun_out/alltile/prof.log; exit 1; }
python3 tools/kstats.py gpurun_out/alltile/prof > gpurun_out/alltile/kernels.txt && head -8 gpurun_out/alltile/kernels.txt | cut -c1-150
