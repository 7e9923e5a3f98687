#!/bin/bash
# round 5: K9P softmax in the log2 domain (fma + v_exp per score, mask as nibbles, unmasked instance) --
# attention/E5 tests, ingest K9P vs K9L, ingest kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/k9p2; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gemm.py -k "planes or attention or e5 or qkv" > gpurun_out/k9p2/pytest.log 2>&1 || { tail -40 gpurun_out/k9p2/pytest.log; exit 1; }
tail -1 gpurun_out/k9p2/pytest.log
grep -E "planes attention" gpurun_out/k9p2/pytest.log | head -12
for v in 1 0 1; do
  CM_E5_PLANES_ATTN=$v timeout -k 10 300 python -u bench.py --mode ingest --e5-dtype float32 --seq-len 256 --steps 10 --warmup 3 > gpurun_out/k9p2/ingest_$v.log 2>&1 || { tail -20 gpurun_out/k9p2/ingest_$v.log; exit 1; }
  echo "planes=$v $(tail -1 gpurun_out/k9p2/ingest_$v.log | cut -c1-200)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/k9p2/prof -o run --output-format csv -- python3 bench.py --mode ingest --e5-dtype float32 --seq-len 256 --steps 5 --warmup 2 > gpurun_out/k9p2/prof.log 2>&1 || { tail -20 gpurun_out/k9p2/prof.log; exit 1; }
python3 tools/kstats.py gpurun_out/k9p2/prof > gpurun_out/k9p2/kernels.txt && head -8 gpurun_out/k9p2/kernels.txt | cut -c1-150
