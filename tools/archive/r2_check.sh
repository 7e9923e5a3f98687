#!/bin/bash
# GPU session: scale parity tests (all reported), the rest of -m gpu, then the bench.
# Each GPU step has its own limit; the chain stops at the first failure of a step that faults.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TESTS:-tests/test_gpu_scale.py}
timeout -k 10 900 python -u -m pytest $T -v -s --timeout 400 --timeout-method thread > gpurun_out/pytest_scale.log 2>&1
rc=$?
tail -25 gpurun_out/pytest_scale.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "scale tests rc=$rc"; exit 1; fi
if [ "${REST:-1}" = "1" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --deselect tests/test_gpu_scale.py > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
fi
if [ "${BENCH:-1}" = "1" ]; then
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
grep "\[bench\]" gpurun_out/bench.log; tail -1 gpurun_out/bench.log > gpurun_out/bench.json
fi
