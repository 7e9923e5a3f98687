# K10 ablation timings (variants/lib_k10_*.so): K10_ONLY GEMMs, twice each
cd "${GRAFT_REPO_ROOT:-.}"
for rep in 1 2; do for f in variants/lib_k10_*.so; do
  for gm in qkv down; do
    CLASSMATE_HIP_LIB=$PWD/$f K10_ONLY=$gm K10_E5=0 timeout -k 10 120 python tools/k10_probe.py 2>&1 | grep "K10" | sed "s/^/$(basename $f .so) /"
  done
done; done
