#!/bin/bash
# GPU: the whole GPU suite + smoke on the current tree
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/suite; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/suite/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/suite/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/suite/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/suite/smoke.log 2>&1 || { tail -20 gpurun_out/suite/smoke.log; exit 1; }
tail -1 gpurun_out/suite/smoke.log
