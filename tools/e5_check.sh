set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/e5; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_dropin.py -x -q --timeout 120 --timeout-method thread -k "layernorm or e5 or attention" > gpurun_out/e5/pytest.log 2>&1 || { tail -30 gpurun_out/e5/pytest.log; exit 1; }
tail -2 gpurun_out/e5/pytest.log
timeout -k 10 200 python -u tools/e5_probe.py > gpurun_out/e5/fused.log 2>&1 || { tail -20 gpurun_out/e5/fused.log; exit 1; }
grep "graph unpadded=True" gpurun_out/e5/fused.log
CM_E5_FUSED_LN=0 timeout -k 10 200 python -u tools/e5_probe.py > gpurun_out/e5/torch.log 2>&1 || { tail -20 gpurun_out/e5/torch.log; exit 1; }
grep "graph unpadded=True" gpurun_out/e5/torch.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-baseline 0 > gpurun_out/e5/bench.log 2>&1 || { tail -20 gpurun_out/e5/bench.log; exit 1; }
grep '\[bench\] 20 steps' gpurun_out/e5/bench.log | cut -c1-120
