#!/bin/bash
# round 5: K8 split with the planes written per 16-row block (CM_LN_RB=1) vs per-lane 8-byte pieces (0):
# producer/E5 tests, ingest encode + headline step alternating, ingest kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/ln; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gemm.py tests/test_gpu_engine.py -k "producers or e5 or E5 or layernorm or planes" > gpurun_out/ln/pytest.log 2>&1 || { tail -40 gpurun_out/ln/pytest.log; exit 1; }
tail -1 gpurun_out/ln/pytest.log
for r in 1 2; do
  for v in 1 0; do
    CM_LN_RB=$v timeout -k 10 300 python -u bench.py --mode ingest --e5-dtype float32 --seq-len 256 --steps 10 --warmup 3 > gpurun_out/ln/ingest_$v.log 2>&1 || { tail -20 gpurun_out/ln/ingest_$v.log; exit 1; }
    echo "rb=$v $(tail -1 gpurun_out/ln/ingest_$v.log | cut -c1-170)"
  done
done
for r in 1 2; do
  for v in 1 0; do
    CM_LN_RB=$v timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --e5-other-leg 0 --dense-legs 0 --cpu-baseline 0 --ingest-leg 0 > gpurun_out/ln/bench_$v.log 2>&1 || { tail -20 gpurun_out/ln/bench_$v.log; exit 1; }
    echo "rb=$v $(grep 'steps in' gpurun_out/ln/bench_$v.log | cut -c1-150)"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ln/prof -o run --output-format csv -- python3 bench.py --mode ingest --e5-dtype float32 --seq-len 256 --steps 5 --warmup 2 > gpurun_out/ln/prof.log 2>&1 || { tail -20 gpurun_out/ln/prof.log; exit 1; }
python3 tools/kstats.py gpurun_out/ln/prof > gpurun_out/ln/kernels.txt && head -8 gpurun_out/ln/kernels.txt | cut -c1-150
