#!/bin/bash
# round 4, GPU box: K1q v4 (batched hit tests, staged candidates, unconditional re-rank loads),
# radix-select seed, sliced filtered-BM25 df: scan probes, the whole GPU suite (K1c default), the
# K1q tests with CM_DENSE_Q8=1, the headline A/B, the filtered single-query latency at 1M.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/c4; export TMPDIR=/tmp
for kind in 5 3; do
  timeout -k 10 300 python tools/dense_probe.py --path $kind --reps 7 > gpurun_out/c4/probe.log 2>&1 || { tail -20 gpurun_out/c4/probe.log; exit 1; }
  grep docs= gpurun_out/c4/probe.log | cut -c1-150 | tee -a gpurun_out/c4/probe.txt
done
for f in variants/lib_k1c_*.so; do   # K1c without appends (K1C_NOHIT) and with a 6-slot ring
  CLASSMATE_HIP_LIB=$PWD/$f timeout -k 10 300 python tools/dense_probe.py --path 3 --reps 7 > gpurun_out/c4/probe.log 2>&1 || { tail -20 gpurun_out/c4/probe.log; exit 1; }
  grep docs= gpurun_out/c4/probe.log | sed "s/^/$(basename $f .so) /" | cut -c1-150 | tee -a gpurun_out/c4/probe.txt
done
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/c4/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/c4/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/c4/pytest_gpu.log
CM_DENSE_Q8=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_q8.py \
  "tests/test_gpu_scale.py::test_hybrid_10m_sample" > gpurun_out/c4/pytest_q8.log 2>&1 || { tail -40 gpurun_out/c4/pytest_q8.log; exit 1; }
tail -2 gpurun_out/c4/pytest_q8.log
CM_DENSE_Q8=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --e5-other-leg 0 --ingest-leg 0 --dense-legs 0 --cpu-baseline 0 --out gpurun_out/c4/bench_q8.json > gpurun_out/c4/bench_q8.log 2>&1 || { tail -30 gpurun_out/c4/bench_q8.log; exit 1; }
grep "steps in" gpurun_out/c4/bench_q8.log | cut -c1-330
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --e5-other-leg 0 --ingest-leg 0 --dense-legs 0 --cpu-baseline 0 --out gpurun_out/c4/bench_k1c.json > gpurun_out/c4/bench_k1c.log 2>&1 || { tail -30 gpurun_out/c4/bench_k1c.log; exit 1; }
grep "steps in" gpurun_out/c4/bench_k1c.log | cut -c1-330
timeout -k 10 400 python -u bench.py --mode e2e --docs-per-gpu 1000000 --steps 3 --warmup 1 --e2e-latency-queries 32 \
  --out gpurun_out/c4/e2e_1m.json > gpurun_out/c4/e2e_1m.log 2>&1 || { tail -30 gpurun_out/c4/e2e_1m.log; exit 1; }
grep "retrieve()" gpurun_out/c4/e2e_1m.log
