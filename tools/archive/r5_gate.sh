#!/bin/bash
# round 5: BM25 query preparation beside the encode, scoring gated on it (--bm25-gate 1) vs the whole search
# after the encode (0); headline-only bench, alternating, one box; then a trace of the gated step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/gate; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_engine.py -k "bm25 or BM25" > gpurun_out/gate/pytest.log 2>&1 || { tail -40 gpurun_out/gate/pytest.log; exit 1; }
tail -1 gpurun_out/gate/pytest.log
for r in 1 2 3; do
  for g in 1 0; do
    timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --e5-other-leg 0 --ingest-leg 0 --dense-legs 0 --cpu-baseline 0 --bm25-gate $g > gpurun_out/gate/bench_$g.log 2>&1 || { tail -20 gpurun_out/gate/bench_$g.log; exit 1; }
    grep "steps in" gpurun_out/gate/bench_$g.log | sed "s/^/gate=$g /" | cut -c1-200
  done
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/gate/hl -o hl --output-format csv -- python3 -u bench.py --steps 20 --warmup 5 --e5-other-leg 0 --ingest-leg 0 --dense-legs 0 --cpu-baseline 0 > gpurun_out/gate/trace.log 2>&1 || { tail -30 gpurun_out/gate/trace.log; exit 1; }
python3 tools/trace_step.py gpurun_out/gate/hl/hl_kernel_trace.csv dense_q8_scan_kernel 15 | grep -v "short_att\|add_layernorm" | tail -40
