#!/bin/bash
# round 5: q8 + BM25 engine tests on the shared-LDS K1q / 256-thread merge tree, the headline bench,
# and a kernel trace of the batch-1 E5 encode (tools/e5_b1_probe.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/c2 gpurun_out/e5b1; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_q8.py tests/test_gpu_engine.py > gpurun_out/c2/pytest.log 2>&1 || { tail -30 gpurun_out/c2/pytest.log; exit 1; }
tail -2 gpurun_out/c2/pytest.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --e5-other-leg 0 --ingest-leg 0 --dense-legs 0 --cpu-baseline 0 > gpurun_out/c2/bench.log 2>&1 || { tail -20 gpurun_out/c2/bench.log; exit 1; }
grep "steps in" gpurun_out/c2/bench.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/e5b1/tr -o tr --output-format csv -- python3 -u tools/e5_b1_probe.py > gpurun_out/e5b1/probe.log 2>&1 || { tail -20 gpurun_out/e5b1/probe.log; exit 1; }
cat gpurun_out/e5b1/probe.log | grep "E5 encode"
