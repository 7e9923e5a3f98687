#!/bin/bash
# Environment probe for the GPU box (not part of the product).
set -o pipefail
mkdir -p gpurun_out
{
  echo "== nproc"; nproc
  echo "== mem"; free -g
  echo "== rocminfo"; timeout -k 5 60 rocminfo | grep -E "Marketing|gfx|Compute Unit|Max Clock" | head -20
  echo "== torch"; timeout -k 5 300 python -c "import torch,time; print(torch.cuda.is_available(), torch.cuda.get_device_name(0)); p=torch.cuda.get_device_properties(0); print(p.total_memory/2**30, p.multi_processor_count)"
  echo "== python pkgs"; python -c "import cffi" 2>&1 | tail -1
  ls ~/.cache/huggingface 2>&1 | head
} > gpurun_out/probe.txt 2>&1
