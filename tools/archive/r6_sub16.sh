#!/bin/bash
# Round 6: K2b over planned 16-doc sub-blocks -- BM25 parity tests (engine, drop-in, multi-device, 10M sample),
# the standalone probe, then the headline step with the sub-block plan on / off (CM_BM25_SUB16_OFF=1), alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/sub16; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_engine.py tests/test_gpu_dropin.py \
  tests/test_gpu_multidev.py "tests/test_gpu_scale.py::test_hybrid_10m_sample" > gpurun_out/sub16/tests.log 2>&1 \
  || { echo "tests failed"; tail -40 gpurun_out/sub16/tests.log; exit 1; }
tail -1 gpurun_out/sub16/tests.log
for v in on off on off; do
  if [ $v = off ]; then export CM_BM25_SUB16_OFF=1; else unset CM_BM25_SUB16_OFF; fi
  timeout -k 10 300 python tools/bm25_probe.py --paths 2 --reps 5 2>&1 | grep "path=2" | sed "s/^/$v /" | cut -c1-200
done
unset CM_BM25_SUB16_OFF
ENVS="on off=CM_BM25_SUB16_OFF=1" REPS=2 bash tools/r6_env_ab.sh
