#!/bin/bash
# round 4, GPU box: where the filtered single-query retrieve() time goes -- e2e mode at 1M chunks,
# host cProfile of the latency legs (CM_E2E_PROFILE_LAT) and, separately, the kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/filt; export TMPDIR=/tmp
CM_E2E_PROFILE_LAT=1 timeout -k 10 400 python -u bench.py --mode e2e --docs-per-gpu 1000000 --steps 3 --warmup 1 \
  --e2e-latency-queries 32 --out gpurun_out/filt/e2e_1m.json > gpurun_out/filt/e2e_1m.log 2>&1 || { tail -30 gpurun_out/filt/e2e_1m.log; exit 1; }
grep "\[bench\]" gpurun_out/filt/e2e_1m.log | tail -5
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/filt/kt -o e2e --output-format csv -- \
  python3 bench.py --mode e2e --docs-per-gpu 1000000 --steps 3 --warmup 1 --e2e-latency-queries 32 \
  --out gpurun_out/filt/e2e_1m_prof.json > gpurun_out/filt/e2e_1m_prof.log 2>&1 || { tail -30 gpurun_out/filt/e2e_1m_prof.log; exit 1; }
python3 tools/kstats.py gpurun_out/filt/kt > gpurun_out/filt/kernel_summary.txt && head -40 gpurun_out/filt/kernel_summary.txt
