#!/usr/bin/env python3
"""VERDICT r3 #6 gate (GPU box, torch only -- no product kernel): how wide would K1c's certified band
be with a 1-byte coarse plane?

Data = bench.py's 10M x 768 shard (same generator, seed 1000) and bench.py's query embeddings (the
random-init fp32 E5 encode of its 256 x 24 token ids); Gaussian queries as a second set.
For every coarse format the rigorous per-query bound is the one dense_rerank_kernel uses,
  |q.c - q~.c~| <= ||e_q|| max||c~|| + ||q~|| max||e_c|| + ||e_q|| max||e_c||   (+ fp32 rounding),
and the counts reported per query are
  band  = rows with coarse_sim >= (k'-th largest coarse_sim) - 2E   (what the re-rank must read)
  cand@s = rows with coarse_sim >= (k'-th largest coarse_sim of a 1/s row sample) - 2E
           (what the scan writes with the sample seed, s = 64 today).
Formats: f16 (today), i8 rows + i8 query (one v_mfma_i32_16x16x64_i8 per product), i8 rows + query
split into two i8 planes (q = s1 q1 + s2 q2: two i8 MFMAs), fp8 e4m3 rows + query (per-row scale).
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parents[1]
for p in (str(REPO), str(REPO / "classmate-rag_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def gen_rows(n, dim, seed, dev, chunk=1 << 20):
    g = torch.Generator(device="cuda").manual_seed(seed)
    X = torch.empty(n, dim, device=dev)
    for r0 in range(0, n, chunk):
        m = min(chunk, n - r0)
        x = torch.randn(m, dim, device=dev, generator=g)
        X[r0:r0 + m] = x / x.norm(dim=1, keepdim=True)
    return X


def q_i8(x):
    """per-row symmetric int8: x ~ s * x8, s = max|x| / 127 (returned as float tensors)."""
    s = x.abs().amax(dim=1, keepdim=True) / 127.0
    x8 = torch.round(x / s).clamp_(-127, 127)
    return x8, s


def q_fp8(x):
    s = x.abs().amax(dim=1, keepdim=True) / 448.0
    return (x / s).to(torch.float8_e4m3fn).float(), s


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--pool", type=int, default=24)
    ap.add_argument("--out", default="gpurun_out/int8_band.json")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    N, D, B, P = a.rows, 768, a.batch, a.pool
    X = gen_rows(N, D, 1000, dev)
    # bench.py's query embeddings: random-init fp32 E5 over its token ids (seed 13)
    from classmate_hip.embeddings import E5MultilingualEmbedder
    g = torch.Generator(device="cuda").manual_seed(13)
    ids = torch.randint(5, 250002, (B, 24), device=dev, generator=g)
    ids[:, 0], ids[:, -1] = 0, 2
    m = E5MultilingualEmbedder.random_init(seed=0, device=str(dev), dtype="float32")
    qe = m.encode_token_ids(ids, torch.ones_like(ids)).float()
    del m
    torch.cuda.empty_cache()
    gq = torch.Generator(device="cuda").manual_seed(31)
    qg = torch.randn(B, D, device=dev, generator=gq)
    qsets = {"e5": qe / qe.norm(dim=1, keepdim=True), "gauss": qg / qg.norm(dim=1, keepdim=True)}
    res = {"rows": N, "dim": D, "batch": B, "pool": P}
    chunk = 1 << 20

    def coarse_rows(fmt, x):
        if fmt == "f16":
            xh = x.half().float()
            return xh, (x - xh)
        if fmt == "fp8":
            x8, s = q_fp8(x)
            xt = x8 * s
            return xt, x - xt
        x8, s = q_i8(x)
        xt = x8 * s
        return xt, x - xt

    def coarse_q(fmt, q):
        if fmt == "f16":
            qh = q.half().float()
            return qh
        if fmt == "fp8":
            q8, s = q_fp8(q)
            return q8 * s
        if fmt == "i8":
            q8, s = q_i8(q)
            return q8 * s
        if fmt == "i8split":
            q1, s1 = q_i8(q)
            r = q - q1 * s1
            q2, s2 = q_i8(r)
            return q1 * s1 + q2 * s2
        raise ValueError(fmt)

    # row-side statistics once per row format (max ||c~||, max ||e_c||)
    row_stats = {}
    for rf in ("f16", "i8", "fp8"):
        mx_c, mx_e, rms_e = 0.0, 0.0, 0.0
        for r0 in range(0, N, chunk):
            xt, e = coarse_rows(rf, X[r0:r0 + chunk])
            mx_c = max(mx_c, float(xt.norm(dim=1).max()))
            en = e.norm(dim=1)
            mx_e = max(mx_e, float(en.max()))
            rms_e += float((en * en).sum())
        row_stats[rf] = (mx_c, mx_e, (rms_e / N) ** 0.5)
    res["row_stats"] = {k: dict(max_norm=v[0], max_err=v[1], rms_err=v[2]) for k, v in row_stats.items()}
    print("row stats", res["row_stats"], flush=True)

    for qname, Q in qsets.items():
        for fmt, rf in (("f16", "f16"), ("i8", "i8"), ("i8split", "i8")):
            qt = coarse_q(fmt, Q)
            eq = (Q - qt).norm(dim=1)
            qn = qt.norm(dim=1)
            mx_c, mx_e, _ = row_stats[rf]
            E = (eq * mx_c + qn * mx_e + eq * mx_e) * 1.001 + 2e-6
            # per-row bound: E_r = ||e_q|| ||c~_r|| + ||q~|| ||e_c,r|| + ||e_q|| ||e_c,r|| (a row
            # test coarse - E_r; the k'-th threshold from coarse + E_r)
            def e_row(xt, e):
                cn, en = xt.norm(dim=1), e.norm(dim=1)
                return ((eq[:, None] * cn[None] + qn[:, None] * en[None] + eq[:, None] * en[None]) * 1.001 + 2e-6)
            # pass 1: k'-th largest coarse sim (full and 1/64, 1/16 samples) and the exact k'-th sim
            topc = torch.full((B, 0), -2.0, device=dev)
            topr = torch.full((B, 0), -2.0, device=dev)            # k'-th largest (coarse - E_r)
            tops = {64: torch.full((B, 0), -2.0, device=dev), 16: torch.full((B, 0), -2.0, device=dev),
                    8: torch.full((B, 0), -2.0, device=dev)}
            topsr = {s_: torch.full((B, 0), -2.0, device=dev) for s_ in tops}
            tope = torch.full((B, 0), -2.0, device=dev)
            for r0 in range(0, N, chunk):
                x = X[r0:r0 + chunk]
                xt, ex = coarse_rows(rf, x)
                cs = qt @ xt.T                                   # (B, m) coarse
                lo = cs - e_row(xt, ex)
                es = Q @ x.T
                topc = torch.cat([topc, cs], 1).topk(P, dim=1).values
                topr = torch.cat([topr, lo], 1).topk(P, dim=1).values
                tope = torch.cat([tope, es], 1).topk(P, dim=1).values
                for s in tops:
                    idx = torch.arange((-r0) % s, x.shape[0], s, device=dev)
                    tops[s] = torch.cat([tops[s], cs[:, idx]], 1).topk(P, dim=1).values
                    topsr[s] = torch.cat([topsr[s], lo[:, idx]], 1).topk(P, dim=1).values
                del lo
            kth = topc[:, -1]
            thr = {"band": kth - 2 * E, **{f"cand@{s}": tops[s][:, -1] - 2 * E for s in tops}}
            # per-row E: a row is in the band when coarse + E_r >= the k'-th largest (coarse - E_r)
            thr_r = {"band_rowE": topr[:, -1], **{f"cand_rowE@{s}": topsr[s][:, -1] for s in topsr}}
            cnt = {k: torch.zeros(B, device=dev, dtype=torch.int64) for k in list(thr) + list(thr_r)}
            for r0 in range(0, N, chunk):
                xt, ex = coarse_rows(rf, X[r0:r0 + chunk])
                cs = qt @ xt.T
                for k, t in thr.items():
                    cnt[k] += (cs >= t[:, None]).sum(1)
                hi = cs + e_row(xt, ex)
                for k, t in thr_r.items():
                    cnt[k] += (hi >= t[:, None]).sum(1)
                del hi
            out = {"E_mean": float(E.mean()), "E_max": float(E.max()),
                   "kth_exact_sim_mean": float(tope[:, -1].mean())}
            for k, c in cnt.items():
                c = c.float()
                out[k] = {"mean": float(c.mean()), "p50": float(c.median()), "max": float(c.max())}
            out["band_rerank_bytes_per_batch"] = float(cnt["band"].sum()) * D * 4
            out["band_rowE_rerank_bytes_per_batch"] = float(cnt["band_rowE"].sum()) * D * 4
            res[f"{qname}/{fmt}"] = out
            print(qname, fmt, json.dumps(out), flush=True)
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    Path(a.out).write_text(json.dumps(res, indent=1) + "\n")


if __name__ == "__main__":
    main()
