#!/bin/bash
# round 5: K10 planes epilogues with packed f16 conversions (f16x3_split2) -- GEMM / producer / E5 tests,
# ingest encode and headline step (compare with profiles/r05_ln_ab.txt rb=1 lines), ingest kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/epi; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gemm.py tests/test_gpu_engine.py -k "gemm or f16x3 or attention or e5 or E5 or planes or producers or layernorm" > gpurun_out/epi/pytest.log 2>&1 || { tail -40 gpurun_out/epi/pytest.log; exit 1; }
tail -1 gpurun_out/epi/pytest.log
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --mode ingest --e5-dtype float32 --seq-len 256 --steps 10 --warmup 3 > gpurun_out/epi/ingest.log 2>&1 || { tail -20 gpurun_out/epi/ingest.log; exit 1; }
  echo "ingest $(tail -1 gpurun_out/epi/ingest.log | cut -c1-170)"
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --e5-other-leg 0 --dense-legs 0 --cpu-baseline 0 --ingest-leg 0 > gpurun_out/epi/bench.log 2>&1 || { tail -20 gpurun_out/epi/bench.log; exit 1; }
  echo "step $(grep 'steps in' gpurun_out/epi/bench.log | cut -c1-150)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/epi/prof -o run --output-format csv -- python3 bench.py --mode ingest --e5-dtype float32 --seq-len 256 --steps 5 --warmup 2 > gpurun_out/epi/prof.log 2>&1 || { tail -20 gpurun_out/epi/prof.log; exit 1; }
python3 tools/kstats.py gpurun_out/epi/prof > gpurun_out/epi/kernels.txt && head -8 gpurun_out/epi/kernels.txt | cut -c1-150
