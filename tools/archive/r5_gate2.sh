#!/bin/bash
# round 5: BM25 scoring gated on the dense search's seed pass (--bm25-gate 2, cm_dense_set_seed_event)
# vs on the end of the encode (--bm25-gate 1, product), alternating; engine tests first
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/gate2; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_engine.py -k "gate or gated or q8 or coarse" > gpurun_out/gate2/pytest.log 2>&1 || { tail -30 gpurun_out/gate2/pytest.log; exit 1; }
tail -1 gpurun_out/gate2/pytest.log
for r in 1 2 3; do
  for g in 2 1; do
    timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --bm25-gate $g --e5-other-leg 0 --dense-legs 0 --cpu-baseline 0 --ingest-leg 0 > gpurun_out/gate2/bench_$g.log 2>&1 || { tail -20 gpurun_out/gate2/bench_$g.log; exit 1; }
    echo "gate=$g $(grep 'steps in' gpurun_out/gate2/bench_$g.log | cut -c1-330)"
  done
done
