#!/bin/bash
# round 5: K1q-s first look -- dense tests, then probe timings at 10M x 768 (auto = K1q-s for nq <= 32,
# forced batched K1q for comparison)
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD/classmate-rag_amd:$PWD
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_q8.py \
  "tests/test_gpu_engine.py::test_dense_coarse_certificate" "tests/test_gpu_engine.py::test_dense_shapes" \
  "tests/test_gpu_engine.py::test_dense_batched_split_paths" > gpurun_out/r5_q8s_tests.log 2>&1 || { tail -30 gpurun_out/r5_q8s_tests.log; exit 1; }
tail -3 gpurun_out/r5_q8s_tests.log
for b in 1 16 32; do
  timeout -k 10 300 python -u tools/dense_probe.py --batch $b --k 10 --reps 9 2>&1 | tail -1
done
for p in 5 4; do
  timeout -k 10 300 python -u tools/dense_probe.py --batch 16 --k 10 --reps 9 --path $p 2>&1 | tail -1
done
