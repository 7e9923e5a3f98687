#!/bin/bash
# round 4, GPU box: the whole GPU suite + smoke, the default bench (now with the fp32 ingest leg),
# the per-row-bound band analysis, the 10M drop-in e2e with ask_question-shaped filters
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/r4b; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4b/pytest.log 2>&1 || { tail -40 gpurun_out/r4b/pytest.log; exit 1; }
tail -2 gpurun_out/r4b/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4b/smoke.log 2>&1 || { tail -20 gpurun_out/r4b/smoke.log; exit 1; }
tail -1 gpurun_out/r4b/smoke.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --out gpurun_out/r4b/bench.json > gpurun_out/r4b/bench.log 2>&1 || { tail -30 gpurun_out/r4b/bench.log; exit 1; }
grep "\[bench\]" gpurun_out/r4b/bench.log | cut -c1-300
timeout -k 10 300 python3 tools/int8_band.py --out gpurun_out/r4b/int8_band.json > gpurun_out/r4b/int8_band.log 2>&1 || { tail -30 gpurun_out/r4b/int8_band.log; exit 1; }
timeout -k 10 900 python -u bench.py --mode e2e --docs-per-gpu 10000000 --steps 10 --warmup 3 --out gpurun_out/r4b/e2e.json > gpurun_out/r4b/e2e.log 2>&1 || { tail -30 gpurun_out/r4b/e2e.log; exit 1; }
grep -E "retrieve" gpurun_out/r4b/e2e.log | tail -5
