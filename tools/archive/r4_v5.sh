#!/bin/bash
# GPU: K1q v5 (epilogue pipelined one tile behind the MFMAs): parity (K1q tests, 10M hybrid sample),
# scan probe (Gaussian queries), headline bench without side legs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/v5; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_q8.py \
  "tests/test_gpu_scale.py::test_hybrid_10m_sample" > gpurun_out/v5/pytest_q8.log 2>&1 || { tail -40 gpurun_out/v5/pytest_q8.log; exit 1; }
tail -2 gpurun_out/v5/pytest_q8.log
for rep in 1 2; do
  timeout -k 10 300 python tools/dense_probe.py --path 5 --reps 7 > gpurun_out/v5/probe.log 2>&1 || { tail -20 gpurun_out/v5/probe.log; exit 1; }
  grep docs= gpurun_out/v5/probe.log | cut -c1-150 | tee -a gpurun_out/v5/probe.txt
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --e5-other-leg 0 --ingest-leg 0 --dense-legs 0 --cpu-baseline 0 --out gpurun_out/v5/bench.json > gpurun_out/v5/bench.log 2>&1 || { tail -30 gpurun_out/v5/bench.log; exit 1; }
grep "steps in" gpurun_out/v5/bench.log | cut -c1-330
