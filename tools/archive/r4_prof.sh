#!/bin/bash
# round 4, GPU box: (1) the headline step alone under rocprofv3 --kernel-trace --stats (no side legs,
# so every K1c launch in the summary is the 10M x B=256 one), (2) the 1-byte-plane band analysis.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/r4prof; export TMPDIR=/tmp
TAG=${TAG:-r04}
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r4prof/$TAG -o hl --output-format csv -- \
  python3 bench.py --steps 20 --warmup 5 --dense-legs 0 --e5-other-leg 0 --cpu-baseline 0 \
  --out gpurun_out/r4prof/${TAG}_headline.json > gpurun_out/r4prof/${TAG}_headline.log 2>&1 || { tail -30 gpurun_out/r4prof/${TAG}_headline.log; exit 1; }
grep "\[bench\]" gpurun_out/r4prof/${TAG}_headline.log | tail -3
python3 tools/kstats.py gpurun_out/r4prof/$TAG > gpurun_out/r4prof/${TAG}_kernel_summary.txt && head -30 gpurun_out/r4prof/${TAG}_kernel_summary.txt
if [ -n "$BAND" ]; then
  timeout -k 10 300 python3 tools/int8_band.py --out gpurun_out/r4prof/int8_band.json > gpurun_out/r4prof/int8_band.log 2>&1 || { tail -30 gpurun_out/r4prof/int8_band.log; exit 1; }
  cat gpurun_out/r4prof/int8_band.log
fi
