#!/bin/bash
# round 4, GPU box: K9L accuracy tests, the API-only VMM probe, K10 schedule variants vs the product
# (accuracy tests, GEMM + E5 timings twice), the fp32 ingest encode per-kernel profile
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/r4c; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -x -v --timeout 200 --timeout-method thread -k "long_attention or e5" > gpurun_out/r4c/k9l_tests.log 2>&1 || { tail -30 gpurun_out/r4c/k9l_tests.log; exit 1; }
grep -E "long attention|passed|failed" gpurun_out/r4c/k9l_tests.log | tail -14
timeout -k 10 60 ./tools/vmm_api_probe > gpurun_out/r4c/vmm_api_probe.txt 2>&1 || { cat gpurun_out/r4c/vmm_api_probe.txt; exit 1; }
cat gpurun_out/r4c/vmm_api_probe.txt
bash tools/r4_k10v.sh || exit 1
timeout -k 10 400 env CM_E2E_PROFILE=1 python -u bench.py --mode e2e --docs-per-gpu 1000000 --steps 10 --warmup 3 --out gpurun_out/r4c/e2e_1m.json > gpurun_out/r4c/e2e_1m.log 2>&1 || { tail -30 gpurun_out/r4c/e2e_1m.log; exit 1; }
grep -E "retrieve" gpurun_out/r4c/e2e_1m.log | tail -5
