#!/bin/bash
# round 5 final tree: the default bench under rocprofv3 --kernel-trace --stats (the headline roofline kernel's
# launch time from the trace beside bench.py's HIP-event figure)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/ftr; export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/ftr/tr -o tr --output-format csv -- python3 -u bench.py --out gpurun_out/ftr/bench.json > gpurun_out/ftr/bench.log 2>&1 || { tail -30 gpurun_out/ftr/bench.log; exit 1; }
grep -E "steps in|c2p|c4_dense" gpurun_out/ftr/bench.log | cut -c1-200
python3 tools/kstats.py gpurun_out/ftr/tr > gpurun_out/ftr/kernels.txt && head -30 gpurun_out/ftr/kernels.txt | cut -c1-150
