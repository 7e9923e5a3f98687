#!/bin/bash
# GPU: BM25 parity tests (both strategies), then the 10M probe (full vs pruned), then the bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py -x -q -k "bm25" --timeout 300 --timeout-method thread > gpurun_out/bm25_tests.log 2>&1 || { tail -40 gpurun_out/bm25_tests.log; exit 1; }
tail -2 gpurun_out/bm25_tests.log
timeout -k 10 400 python -u tools/bm25_probe.py --reps 5 > gpurun_out/bm25_probe.log 2>&1 || { tail -20 gpurun_out/bm25_probe.log; exit 1; }
cat gpurun_out/bm25_probe.log | grep -v amdgpu.ids
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 500 python -u bench.py --steps 10 --warmup 3 --out gpurun_out/bench_v3.json > gpurun_out/bench_v3.log 2>&1 || { tail -20 gpurun_out/bench_v3.log; exit 1; }
  grep "\[bench\]" gpurun_out/bench_v3.log | tail -4
fi
