#!/bin/bash
# GPU: per-kernel times of one BM25 search at the bench shape (+ dbg=3 floor).
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
CM_BM25_DEBUG=3 timeout -k 10 300 python tools/bm25_probe.py > gpurun_out/probe_3.log 2>&1 || exit 1
tail -1 gpurun_out/probe_3.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/k2prof -o k2 --output-format csv -- python3 tools/bm25_probe.py --reps 3 > gpurun_out/k2prof.log 2>&1 || exit 1
f=$(find gpurun_out/k2prof -name '*kernel_stats.csv' | head -1); cp "$f" gpurun_out/k2_kernel_stats.csv
cut -d, -f1-4 gpurun_out/k2_kernel_stats.csv | head -12
