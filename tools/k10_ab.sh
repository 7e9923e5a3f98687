# K10 variants A/B: the E5 fp32 encode and the qkv/down GEMMs per variants/lib_k10_*.so, alternating
cd "${GRAFT_REPO_ROOT:-.}"
for rep in 1 2; do for f in variants/lib_k10_*.so; do
  CLASSMATE_HIP_LIB=$PWD/$f E5_DTYPE=float32 timeout -k 10 200 python tools/e5_probe.py 2>&1 | grep "graph unpadded=True" | sed "s/^/$(basename $f .so) /"
  for gm in qkv down; do
    CLASSMATE_HIP_LIB=$PWD/$f K10_ONLY=$gm K10_E5=0 timeout -k 10 120 python tools/k10_probe.py 2>&1 | grep "K10" | grep -v "per layer" | sed "s/^/$(basename $f .so) /"
  done
done; done
