# K10 check on the GPU box: GEMM + E5 parity tests, then the timing probe
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/k10; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_engine.py -x -v -s --timeout 200 --timeout-method thread -k "f16x3 or e5 or layernorm or attention" > gpurun_out/k10/pytest.log 2>&1 || { tail -40 gpurun_out/k10/pytest.log; exit 1; }
grep -E "K10|E5|passed|failed" gpurun_out/k10/pytest.log | tail -20
timeout -k 10 300 python -u tools/k10_probe.py > gpurun_out/k10/probe.log 2>&1 || { tail -20 gpurun_out/k10/probe.log; exit 1; }
cat gpurun_out/k10/probe.log
