#!/bin/bash
# round 4, GPU box: the i8 MFMA operand map, then K1q parity (1M + the 10M hybrid sample + growth)
# with the matching build, then the bench headline on K1q and on K1c (A/B, same box)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/q8; export TMPDIR=/tmp
timeout -k 10 60 ./tools/mfma_i8_probe > gpurun_out/q8/probe.txt 2>&1 || { cat gpurun_out/q8/probe.txt; exit 1; }
cat gpurun_out/q8/probe.txt
if grep -q "map H1: ran, 0 of 256" gpurun_out/q8/probe.txt; then echo "map 1 (product build; any k permutation shared by A and B is exact)";
elif grep -q "map H2: ran, 0 of 256" gpurun_out/q8/probe.txt; then echo "map 2 (variant build)"; export CLASSMATE_HIP_LIB=$PWD/variants/lib_q8map2.so;
else echo "neither operand map matches: stop"; exit 1; fi
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_q8.py tests/test_gpu_growth.py \
  "tests/test_gpu_scale.py::test_hybrid_10m_sample" "tests/test_gpu_scale.py::test_dense_1m_x_768" > gpurun_out/q8/pytest.log 2>&1 || { tail -40 gpurun_out/q8/pytest.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/q8/pytest.log | tail -16
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --e5-other-leg 0 --ingest-leg 0 --cpu-baseline 1 --out gpurun_out/q8/bench_q8.json > gpurun_out/q8/bench_q8.log 2>&1 || { tail -30 gpurun_out/q8/bench_q8.log; exit 1; }
grep "\[bench\]" gpurun_out/q8/bench_q8.log | cut -c1-330
CM_DENSE_Q8=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --e5-other-leg 0 --ingest-leg 0 --dense-legs 0 --cpu-baseline 0 --out gpurun_out/q8/bench_k1c.json > gpurun_out/q8/bench_k1c.log 2>&1 || { tail -30 gpurun_out/q8/bench_k1c.log; exit 1; }
grep "\[bench\]" gpurun_out/q8/bench_k1c.log | cut -c1-330
