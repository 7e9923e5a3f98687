#!/bin/bash
# round 4, GPU box: new GPU tests (C5 8-rank split, growth policy, BM25-only device items), the
# headline step alone under rocprofv3, the 1-byte-plane band analysis, the 8-rank bench rehearsal
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/r4; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_c5.py \
  tests/test_gpu_growth.py tests/test_gpu_dropin.py > gpurun_out/r4/pytest1.log 2>&1 || { tail -40 gpurun_out/r4/pytest1.log; exit 1; }
tail -3 gpurun_out/r4/pytest1.log
BAND=1 bash tools/r4_prof.sh || exit 1
NP=8 DOCS=1000000 TMO=400 bash tools/mgpu_rehearsal.sh || exit 1
