#!/bin/bash
# round 5: shard-merge kernel + C5 tests, K1q-s seed-sample sweep, step schedule A/B, cliff leg in the default bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/misc; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parallel.py tests/test_gpu_c5.py > gpurun_out/misc/pytest_par.log 2>&1 || { tail -40 gpurun_out/misc/pytest_par.log; exit 1; }
tail -1 gpurun_out/misc/pytest_par.log
bash tools/r5_q8s_sample.sh || exit 1
for s in after with after with; do
  if [ $s = with ]; then fl=--bm25-with-e5; else fl=; fi
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --e5-other-leg 0 --ingest-leg 0 --dense-legs 0 --cpu-baseline 0 $fl > gpurun_out/misc/sched_$s.log 2>&1 || { tail -20 gpurun_out/misc/sched_$s.log; exit 1; }
  grep "steps in" gpurun_out/misc/sched_$s.log | sed "s/^/bm25-$s-e5 /" | cut -c1-400
done
timeout -k 10 600 python -u bench.py --e5-other-leg 0 --ingest-leg 0 --out gpurun_out/misc/bench_cliff.json > gpurun_out/misc/bench_cliff.log 2>&1 || { tail -20 gpurun_out/misc/bench_cliff.log; exit 1; }
grep -E "steps in|c2p|c4_|c2_" gpurun_out/misc/bench_cliff.log | cut -c1-300
