# round-3 check on the GPU box: K10/attention tests + E5 timing, default bench (N=1), N=2 rehearsal
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/r3; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -x -q -s --timeout 200 --timeout-method thread > gpurun_out/r3/gemm_tests.log 2>&1 || { tail -30 gpurun_out/r3/gemm_tests.log; exit 1; }
grep -E "attention|E5 f16x3|passed|failed" gpurun_out/r3/gemm_tests.log
E5_DTYPE=float32 timeout -k 10 200 python tools/e5_probe.py 2>&1 | grep "graph unpadded=True"
timeout -k 10 600 python -u bench.py --steps ${STEPS:-10} --warmup 3 --out gpurun_out/r3/bench.json > gpurun_out/r3/bench.log 2>&1 || { tail -30 gpurun_out/r3/bench.log; exit 1; }
grep "\[bench\]" gpurun_out/r3/bench.log | cut -c1-250
if [ "${MGPU:-1}" = 1 ]; then DOCS=1000000 bash tools/mgpu_rehearsal.sh; fi
