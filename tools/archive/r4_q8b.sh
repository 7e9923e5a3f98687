#!/bin/bash
# round 4, GPU box: K1q v2 (tile metadata through the LDS-DMA ring, quick reject) -- parity with K1q
# automatic, the headline under rocprofv3 --kernel-trace --stats on K1q, then the K1q / K1c A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/q8b; export TMPDIR=/tmp
TAG=${TAG:-q8b}
for kind in 5 3; do
  timeout -k 10 300 python tools/dense_probe.py --path $kind --reps 7 > gpurun_out/q8b/probe.log 2>&1 || { tail -20 gpurun_out/q8b/probe.log; exit 1; }
  grep docs= gpurun_out/q8b/probe.log | cut -c1-150 | tee -a gpurun_out/q8b/probe.txt
done
CM_DENSE_Q8=1 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_q8.py tests/test_gpu_growth.py \
  "tests/test_gpu_scale.py::test_hybrid_10m_sample" "tests/test_gpu_scale.py::test_dense_1m_x_768" > gpurun_out/q8b/pytest.log 2>&1 || { tail -40 gpurun_out/q8b/pytest.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/q8b/pytest.log | tail -16
CM_DENSE_Q8=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/q8b/$TAG -o hl --output-format csv -- \
  python3 bench.py --steps 20 --warmup 5 --dense-legs 0 --e5-other-leg 0 --ingest-leg 0 --cpu-baseline 0 \
  --out gpurun_out/q8b/${TAG}_prof.json > gpurun_out/q8b/${TAG}_prof.log 2>&1 || { tail -30 gpurun_out/q8b/${TAG}_prof.log; exit 1; }
python3 tools/kstats.py gpurun_out/q8b/$TAG > gpurun_out/q8b/${TAG}_kernel_summary.txt && head -24 gpurun_out/q8b/${TAG}_kernel_summary.txt
CM_DENSE_Q8=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --e5-other-leg 0 --ingest-leg 0 --cpu-baseline 0 --out gpurun_out/q8b/bench_q8.json > gpurun_out/q8b/bench_q8.log 2>&1 || { tail -30 gpurun_out/q8b/bench_q8.log; exit 1; }
grep "\[bench\]" gpurun_out/q8b/bench_q8.log | cut -c1-330
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --e5-other-leg 0 --ingest-leg 0 --dense-legs 0 --cpu-baseline 0 --out gpurun_out/q8b/bench_k1c.json > gpurun_out/q8b/bench_k1c.log 2>&1 || { tail -30 gpurun_out/q8b/bench_k1c.log; exit 1; }
grep "\[bench\]" gpurun_out/q8b/bench_k1c.log | cut -c1-330
