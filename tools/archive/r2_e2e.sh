#!/bin/bash
# GPU: drop-in e2e bench (retrieve_batch strings -> dicts + single-query latency) and the C3 ingest
# lines (bf16 and fp32 E5 forward).
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=${ROUND:-r02}
timeout -k 10 300 python -u bench.py --mode ingest --batch 256 --seq-len 256 --steps 10 --warmup 3 --out gpurun_out/bench_${R}_c3_ingest_bf16.json > gpurun_out/bench_${R}_c3.log 2>&1 || { tail -20 gpurun_out/bench_${R}_c3.log; exit 1; }
tail -1 gpurun_out/bench_${R}_c3.log | cut -c1-200
timeout -k 10 300 python -u bench.py --mode ingest --e5-dtype float32 --batch 256 --seq-len 256 --steps 5 --warmup 2 --out gpurun_out/bench_${R}_c3_ingest_fp32.json > gpurun_out/bench_${R}_c3f.log 2>&1 || { tail -20 gpurun_out/bench_${R}_c3f.log; exit 1; }
tail -1 gpurun_out/bench_${R}_c3f.log | cut -c1-200
timeout -k 10 600 python -u bench.py --mode e2e --docs-per-gpu ${E2E_DOCS:-200000} --batch 256 --steps 10 --warmup 2 --out gpurun_out/bench_${R}_e2e.json > gpurun_out/bench_${R}_e2e.log 2>&1 || { tail -30 gpurun_out/bench_${R}_e2e.log; exit 1; }
grep "\[bench\]" gpurun_out/bench_${R}_e2e.log
