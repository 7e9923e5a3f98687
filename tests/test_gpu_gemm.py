"""K10 (cm_linear_f16x3): the E5 projections at fp32 accuracy on the f16 matrix cores.

The reference runs every XLM-R projection as an fp32 nn.Linear (rag/embeddings/__init__.py:85-105,
sentence-transformers on torch fp32).  The bar here is "as accurate as an fp32 GEMM": against an
fp64 reference of the same product, K10's error must stay within 2x the error of torch's own fp32
GEMM on the same GPU (hipBLASLt, exact fp32 MFMA) -- element-wise max and mean -- plus the GELU
epilogue against torch's F.gelu (exact erf) of the fp64 product.  The E5 forward built on it is
held to the Hugging Face fp32 module at 2e-5 (test_gpu_scale.py C3 at B = 32, S = 256, and the
query shape B = 256, S = 24 below).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _case(M, K, N, seed, xs=1.0, ws=0.02):
    import torch
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = xs * torch.randn(M, K, device="cuda", generator=g)
    w = ws * torch.randn(N, K, device="cuda", generator=g)
    b = 0.1 * torch.randn(N, device="cuda", generator=g)
    return x, w, b


@pytest.mark.parametrize("M,K,N", [(6144, 768, 2304), (6144, 768, 768), (1000, 768, 3072), (37, 3072, 768),
                                   (1, 768, 64), (129, 64, 192), (20000, 768, 3072), (8192, 3072, 768),
                                   (9216, 768, 3072), (12288, 3072, 768), (8, 768, 2304), (24, 3072, 768),
                                   (32, 768, 3072), (65536, 768, 768), (30000, 768, 2304)])
def test_linear_f16x3_fp32_accuracy(M, K, N):
    import torch
    from classmate_hip import engine
    x, w, b = _case(M, K, N, seed=M + N)
    W = engine.F16x3Weight(w, b)
    got = engine.linear_f16x3(x, W)
    torch.cuda.synchronize()
    ref = x.double() @ w.double().T + b.double()
    f32 = torch.nn.functional.linear(x, w, b).double()
    e_ours = (got.double() - ref).abs()
    e_f32 = (f32 - ref).abs()
    print(f"\nK10 {M}x{K}x{N}: max err {float(e_ours.max()):.3e} (fp32 GEMM {float(e_f32.max()):.3e}), "
          f"mean {float(e_ours.mean()):.3e} ({float(e_f32.mean()):.3e})")
    assert float(e_ours.max()) <= 2 * float(e_f32.max()) + 1e-7
    assert float(e_ours.mean()) <= 2 * float(e_f32.mean()) + 1e-9


def test_linear_f16x3_gelu_epilogue_and_scales():
    """GELU fused into the epilogue == F.gelu of the fp64 product (fp32 rounding), for activations
    of widely different magnitudes (the power-of-two a_scale keeps them in f16 range)."""
    import torch
    from classmate_hip import engine
    for xs, a_scale in ((1.0, 1.0), (1e-3, 2.0 ** 12), (3e3, 2.0 ** -4)):
        x, w, b = _case(300, 768, 3072, seed=5, xs=xs)
        W = engine.F16x3Weight(w, b)
        got = engine.linear_f16x3(x, W, a_scale=a_scale, gelu=True)
        ref64 = x.double() @ w.double().T + b.double()
        ref = torch.nn.functional.gelu(ref64)
        f32 = torch.nn.functional.gelu(torch.nn.functional.linear(x, w, b)).double()
        e_ours, e_f32 = (got.double() - ref).abs(), (f32 - ref).abs()
        assert float(e_ours.max()) <= 2 * float(e_f32.max()) + 1e-7, (xs, float(e_ours.max()), float(e_f32.max()))


def test_linear_f16x3_tile_independent_bits():
    """A single short query's rows (M <= 32: the skinny K10s kernel, one or two row blocks) are
    bit-identical to the same rows inside a batch (M = 6144: the 96 x 192 / 192 x 192 tiles) -- the
    per-element k order does not depend on the kernel, so a query embeds the same alone or batched;
    with and without GELU."""
    import torch
    from classmate_hip import engine
    for K, N in ((768, 2304), (768, 768), (3072, 768), (768, 3072)):
        x, w, b = _case(6144, K, N, seed=K + 3 * N)
        W = engine.F16x3Weight(w, b)
        for gelu in (False, True):
            big = engine.linear_f16x3(x, W, gelu=gelu)
            for m in (1, 13, 16, 17, 32, 33):
                small = engine.linear_f16x3(x[:m].contiguous(), W, gelu=gelu)
                assert torch.equal(small, big[:m]), (K, N, gelu, m)
        # the fused FFN-up epilogue (GELU -> split planes for the next projection), same bits
        bigp = engine.linear_f16x3(x, W, gelu=True, planes_out=2.0 ** -3)
        for m in (1, 17, 32):
            smallp = engine.linear_f16x3(x[:m].contiguous(), W, gelu=True, planes_out=2.0 ** -3)
            for a, b in zip(smallp.halves(), bigp.halves()):
                assert torch.equal(a, b[:m]), (K, N, m)


def test_linear_f16x3_rejects_bad_shapes():
    import torch
    from classmate_hip import engine
    with pytest.raises(ValueError):
        engine.F16x3Weight(torch.zeros(100, 768, device="cuda"))          # N % 64
    W = engine.F16x3Weight(torch.ones(64, 96, device="cuda"))
    with pytest.raises(ValueError):
        engine.linear_f16x3(torch.zeros(4, 64, device="cuda"), W)          # K mismatch


def test_e5_query_shape_f16x3_matches_hf_fp32():
    """The bench's query encode (B = 256, S = 24, 12 layers, graph-captured lean forward on K10 +
    cm_short_attention fp32 + K8 + K6) == the Hugging Face module in fp32 within 2e-5."""
    import torch
    from classmate_hip.embeddings import E5MultilingualEmbedder
    emb = E5MultilingualEmbedder.random_init(seed=0, device="cuda", dtype="float32")
    assert emb._lean_forward() is not None and emb.f16x3
    B, S = 256, 24
    g = torch.Generator(device="cuda").manual_seed(13)
    ids = torch.randint(5, 250002, (B, S), device="cuda", generator=g)
    ids[:, 0] = 0
    ids[:, -1] = 2
    mask = torch.ones_like(ids)
    u_ids, _, u_out, graph = emb.capture_graph(B, S, unpadded=True)
    u_ids.copy_(ids)
    graph.replay()
    torch.cuda.synchronize()
    ref = emb._encode_hf(ids, mask)
    err = float((u_out - ref).abs().max())
    print(f"\nE5 f16x3 query encode vs HF fp32: max abs err {err:.2e}")
    torch.testing.assert_close(u_out, ref, atol=2e-5, rtol=0)


def test_plane_producers_match_split_rows():
    """The fused producers (K8 add+LayerNorm, fp32 short attention, the GELU epilogue) write the
    same planes, bit for bit, as splitting their fp32 outputs with cm_f16x3_split_rows."""
    import torch
    from classmate_hip import engine
    torch.manual_seed(0)
    B, S, D, H = 9, 24, 768, 12
    x = torch.randn(B, S, D, device="cuda")
    r = torch.randn(S, D, device="cuda")
    g, b = 1 + 0.1 * torch.randn(D, device="cuda"), 0.1 * torch.randn(D, device="cuda")
    out, p = engine.add_layernorm_split(x, r, g, b, 1e-5, 2.0 ** 9)
    assert torch.equal(out, engine.add_layernorm(x, r, g, b, 1e-5))

    def same(p, q):
        return all(torch.equal(u, v) for u, v in zip(p.halves(), q.halves()))

    q = engine.split_rows(out, 2.0 ** 9)
    assert same(p, q)
    # the split itself: hi + lo == x * scale to 22 bits
    hi, lo = q.halves()
    rec = (hi.double() + lo.double()) / 2.0 ** 9
    assert float((rec - out.view(-1, D).double()).abs().max()) <= 2.0 ** -21 * float(out.abs().max())
    # attention: S > 32 runs the fp32 VALU kernel, whose planes are the split of its fp32 output;
    # S <= 32 runs the split-precision MFMA kernel (held to fp64 in the test below)
    qkv = torch.randn(B, 40, 3 * D, device="cuda")
    pa = engine.short_attention_split(qkv, H, 0.125, 2.0 ** 10)
    assert same(pa, engine.split_rows(engine.short_attention(qkv, H, 0.125), 2.0 ** 10))
    w = 0.02 * torch.randn(3072, D, device="cuda")
    W = engine.F16x3Weight(w, 0.1 * torch.randn(3072, device="cuda"))
    hp = engine.linear_f16x3(p, W, gelu=True, planes_out=2.0 ** 11)
    assert same(hp, engine.split_rows(engine.linear_f16x3(p, W, gelu=True), 2.0 ** 11))


@pytest.mark.parametrize("S", [1, 7, 24, 32, 40])
def test_short_attention_split_f16x3_matches_fp64(S):
    """The fp32 query-encode attention writing K10 planes (S <= 32: split-precision MFMA kernel,
    else the fp32 VALU kernel) against an fp64 softmax(q k^T / 8) v, as accurate as torch's fp32."""
    import torch
    from classmate_hip import engine
    torch.manual_seed(S)
    B, H = 37, 12
    qkv = 2 * torch.randn(B, S, 3 * H * 64, device="cuda")
    q, k, v = qkv.double().view(B, S, 3, H, 64).permute(2, 0, 3, 1, 4)
    ref = (torch.softmax(q @ k.transpose(-1, -2) / 8.0, dim=-1) @ v).transpose(1, 2).reshape(B * S, H * 64)
    q32, k32, v32 = qkv.view(B, S, 3, H, 64).permute(2, 0, 3, 1, 4)
    t32 = (torch.softmax(q32 @ k32.transpose(-1, -2) / 8.0, dim=-1) @ v32).transpose(1, 2).reshape(B * S, H * 64)
    p = engine.short_attention_split(qkv, H, 0.125, 2.0 ** 8)
    hi, lo = p.halves()
    got = (hi.double() + lo.double()) / 2.0 ** 8
    e, e32 = float((got - ref).abs().max()), float((t32.double() - ref).abs().max())
    print(f"\nattention S={S}: max err {e:.2e} (torch fp32 {e32:.2e})")
    assert e <= 2 * e32 + 2e-6


@pytest.mark.parametrize("S", [2, 13, 24, 32])
def test_short_attention_split_masked_matches_fp64(S):
    """Padded batches: cm_short_attention_split_masked (key mask, B x S int32) against an fp64
    softmax with the padded keys removed -- XLM-R's extended attention mask -- on every query row,
    padded rows included (they attend to the valid keys, as in the reference's HF forward)."""
    import torch
    from classmate_hip import engine
    torch.manual_seed(100 + S)
    B, H = 29, 12
    qkv = 2 * torch.randn(B, S, 3 * H * 64, device="cuda")
    lens = torch.randint(1, S + 1, (B,), device="cuda")
    lens[0] = S
    mask = (torch.arange(S, device="cuda")[None, :] < lens[:, None]).to(torch.int32)
    keep = mask.bool()[:, None, None, :]
    q, k, v = qkv.double().view(B, S, 3, H, 64).permute(2, 0, 3, 1, 4)
    sc = (q @ k.transpose(-1, -2) / 8.0).masked_fill(~keep, float("-inf"))
    ref = (torch.softmax(sc, dim=-1) @ v).transpose(1, 2).reshape(B * S, H * 64)
    q32, k32, v32 = qkv.view(B, S, 3, H, 64).permute(2, 0, 3, 1, 4)
    s32 = (q32 @ k32.transpose(-1, -2) / 8.0).masked_fill(~keep, float("-inf"))
    t32 = (torch.softmax(s32, dim=-1) @ v32).transpose(1, 2).reshape(B * S, H * 64)
    p = engine.short_attention_split(qkv, H, 0.125, 2.0 ** 8, key_mask=mask)
    hi, lo = p.halves()
    got = (hi.double() + lo.double()) / 2.0 ** 8
    e, e32 = float((got - ref).abs().max()), float((t32.double() - ref).abs().max())
    print(f"\nmasked attention S={S}: max err {e:.2e} (torch fp32 {e32:.2e})")
    assert e <= 2 * e32 + 2e-6
    # an all-ones mask is the unmasked kernel
    p1 = engine.short_attention_split(qkv, H, 0.125, 2.0 ** 8, key_mask=torch.ones_like(mask))
    p0 = engine.short_attention_split(qkv, H, 0.125, 2.0 ** 8)
    assert all(torch.equal(a, b) for a, b in zip(p1.halves(), p0.halves()))


@pytest.mark.parametrize("S", [1, 33, 64, 100, 256, 512])
@pytest.mark.parametrize("masked", [False, True])
def test_long_attention_split_matches_fp64(S, masked):
    """K9L (cm_long_attention_split: 64-key chunks through LDS, online softmax, split-precision
    MFMAs) -- the passage encode's attention, up to the reference's 512-token truncation -- against
    an fp64 softmax(q k^T / 8) v, padded keys removed when masked, as accurate as torch's fp32."""
    import torch
    from classmate_hip import engine
    torch.manual_seed(7 * S + masked)
    B, H = (16 if S <= 256 else 6), 12
    qkv = 2 * torch.randn(B, S, 3 * H * 64, device="cuda")
    mask = None
    keep = torch.ones(B, 1, 1, S, dtype=torch.bool, device="cuda")
    if masked:
        lens = torch.randint(1, S + 1, (B,), device="cuda")
        lens[0] = S
        mask = (torch.arange(S, device="cuda")[None, :] < lens[:, None]).to(torch.int32)
        keep = mask.bool()[:, None, None, :]
    q, k, v = qkv.double().view(B, S, 3, H, 64).permute(2, 0, 3, 1, 4)
    sc = (q @ k.transpose(-1, -2) / 8.0).masked_fill(~keep, float("-inf"))
    ref = (torch.softmax(sc, dim=-1) @ v).transpose(1, 2).reshape(B * S, H * 64)
    q32, k32, v32 = qkv.view(B, S, 3, H, 64).permute(2, 0, 3, 1, 4)
    s32 = (q32 @ k32.transpose(-1, -2) / 8.0).masked_fill(~keep, float("-inf"))
    t32 = (torch.softmax(s32, dim=-1) @ v32).transpose(1, 2).reshape(B * S, H * 64)
    p = engine.long_attention_split(qkv, H, 0.125, 2.0 ** 8, key_mask=mask)
    hi, lo = p.halves()
    got = (hi.double() + lo.double()) / 2.0 ** 8
    e, e32 = float((got - ref).abs().max()), float((t32.double() - ref).abs().max())
    print(f"\nlong attention S={S} masked={masked}: max err {e:.2e} (torch fp32 {e32:.2e})")
    assert e <= 2 * e32 + 2e-6
    if S <= 32 and not masked:          # the same math as K9s where both apply
        ps = engine.short_attention_split(qkv, H, 0.125, 2.0 ** 8)
        hs, ls = ps.halves()
        assert float(((hs.double() + ls.double()) / 2.0 ** 8 - got).abs().max()) <= 2 * e32 + 2e-6


@pytest.mark.parametrize("M", [6144, 1000, 96, 33, 30000])
def test_qkv_planes_epilogue_bits(M):
    """CM_EPI_PLANES_QKV (the fused QKV projection written for K9P) == the fp32 GEMM output split
    with cm_f16x3_split_rows, bit for bit: Q and K thirds in the standard planes, the V third in the
    transposed 32-row-unit layout (decoded by engine.qkv_planes_v)."""
    import torch
    from classmate_hip import engine
    x, w, b = _case(M, 768, 2304, seed=M + 17)
    W = engine.F16x3Weight(w, b)
    s = 2.0 ** 11
    p = engine.linear_f16x3(x, W, qkv=True, planes_out=s)
    ref = engine.split_rows(engine.linear_f16x3(x, W), s)
    for got, want in zip(p.halves(), ref.halves()):
        assert torch.equal(got[:, :1536], want[:, :1536])
    for got, want in zip(engine.qkv_planes_v(p), ref.halves()):
        assert torch.equal(got, want[:, 1536:])
    with pytest.raises(ValueError):
        engine.linear_f16x3(x, W, qkv=True)                      # planes only


def _identity_qkv_planes(qkv, s):
    """fp32 (B, S, 3*H*64) rows -> CM_EPI_PLANES_QKV planes of (hi + lo of qkv) * s, through K10 with an
    identity weight (every output is its input's 22-bit split, exactly)."""
    import torch
    from classmate_hip import engine
    F = qkv.shape[-1]
    I = engine.F16x3Weight(torch.eye(F, device="cuda"), torch.zeros(F, device="cuda"))
    return engine.linear_f16x3(qkv.reshape(-1, F), I, a_scale=2.0 ** 12, qkv=True, planes_out=s)


@pytest.mark.parametrize("S", [64, 128, 256, 320, 512])
@pytest.mark.parametrize("masked", [False, True])
def test_planes_attention_matches_fp64(S, masked):
    """K9P (cm_planes_attention: every operand an LDS-DMA'd split block of the QKV planes, one
    power-of-two scale for Q, K, V) against an fp64 softmax(q k^T / 8) v, padded keys removed when
    masked, as accurate as torch's fp32 -- and within the same bound of K9L on the fp32 rows."""
    import torch
    from classmate_hip import engine
    torch.manual_seed(11 * S + masked)
    B, H = (12 if S <= 256 else 5), 12
    qkv = 2 * torch.randn(B, S, 3 * H * 64, device="cuda")
    mask = None
    keep = torch.ones(B, 1, 1, S, dtype=torch.bool, device="cuda")
    if masked:
        lens = torch.randint(1, S + 1, (B,), device="cuda")
        lens[0] = S
        lens[1] = 1
        mask = (torch.arange(S, device="cuda")[None, :] < lens[:, None]).to(torch.int32)
        keep = mask.bool()[:, None, None, :]
    q, k, v = qkv.double().view(B, S, 3, H, 64).permute(2, 0, 3, 1, 4)
    sc = (q @ k.transpose(-1, -2) / 8.0).masked_fill(~keep, float("-inf"))
    ref = (torch.softmax(sc, dim=-1) @ v).transpose(1, 2).reshape(B * S, H * 64)
    q32, k32, v32 = qkv.view(B, S, 3, H, 64).permute(2, 0, 3, 1, 4)
    s32 = (q32 @ k32.transpose(-1, -2) / 8.0).masked_fill(~keep, float("-inf"))
    t32 = (torch.softmax(s32, dim=-1) @ v32).transpose(1, 2).reshape(B * S, H * 64)
    qp = _identity_qkv_planes(qkv, 2.0 ** 10)
    p = engine.planes_attention(qp, B, S, H, 0.125, 2.0 ** 8, key_mask=mask)
    hi, lo = p.halves()
    got = (hi.double() + lo.double()) / 2.0 ** 8
    e, e32 = float((got - ref).abs().max()), float((t32.double() - ref).abs().max())
    print(f"\nplanes attention S={S} masked={masked}: max err {e:.2e} (torch fp32 {e32:.2e})")
    assert e <= 2 * e32 + 2e-6


def test_planes_attention_rejects_bad_shapes():
    import torch
    from classmate_hip import engine
    qkv = torch.randn(2, 64, 3 * 12 * 64, device="cuda")
    qp = _identity_qkv_planes(qkv, 2.0 ** 10)
    with pytest.raises(ValueError):
        engine.planes_attention(qp, 2, 100, 12, 0.125, 1.0)       # S % 64
    with pytest.raises(ValueError):
        engine.planes_attention(qp, 4, 64, 12, 0.125, 1.0)        # M != B * S
    with pytest.raises(ValueError):
        engine.planes_attention(qp, 2, 64, 12, 0.125, 1.0, key_mask=torch.ones(2, 64, device="cuda"))


@pytest.mark.parametrize("S,cut", [(256, None), (100, 37), (320, 5), (64, 1)])
def test_e5_passage_planes_attention_matches_hf(monkeypatch, S, cut):
    """The passage encode on K9P (QKV planes; S not a multiple of 64 padded with masked pad tokens
    inside the forward) == the Hugging Face fp32 module within 2e-5, ragged rows included, and
    within 2e-5 of the K9L path on fp32 QKV rows (CM_E5_PLANES_ATTN=0)."""
    import torch
    from classmate_hip.embeddings import E5MultilingualEmbedder
    emb = E5MultilingualEmbedder.random_init(seed=5, device="cuda", num_layers=2, dtype="float32")
    B = 6
    g = torch.Generator(device="cuda").manual_seed(S)
    ids = torch.randint(5, 250002, (B, S), device="cuda", generator=g)
    ids[:, 0] = 0
    mask = torch.ones_like(ids)
    if cut is not None:
        mask[B - 1, cut:] = 0
        ids[B - 1, cut:] = 1
    got = emb.encode_token_ids(ids, mask)
    torch.testing.assert_close(got, emb._encode_hf(ids, mask), atol=2e-5, rtol=0)
    monkeypatch.setenv("CM_E5_PLANES_ATTN", "0")
    emb._lean = None
    old = emb.encode_token_ids(ids, mask)
    torch.testing.assert_close(got, old, atol=2e-5, rtol=0)


def test_e5_passage_groups_equal_reference_batches_bit_for_bit():
    """encode_passages (round 6) tokenizes 256 texts at once and runs one forward per attention path
    of sentence-transformers' 32-text batches (rag/embeddings/__init__.py:98-105); every row must get
    exactly the bits its own 32-text batch gives it (group=32: the reference's batches one by one) --
    texts from 3 to ~500 words, so batches with padding on both paths (K9s at <= 32 tokens, K9P
    above, incl. short rows inside a long batch and lengths that are not multiples of 64)."""
    import random
    from classmate_hip.embeddings import E5MultilingualEmbedder
    emb = E5MultilingualEmbedder.random_init(seed=3, device="cuda", num_layers=2, dtype="float32")
    rng = random.Random(11)
    words = [f"w{i}" for i in range(3000)]
    lens = [3, 4, 5, 7, 20, 25, 26, 27, 28, 29, 40, 60, 61, 62, 125, 126, 200, 317, 400, 507, 520]
    lens += [rng.randint(3, 520) for _ in range(280)]
    rng.shuffle(lens)
    texts = [" ".join(rng.choice(words) for _ in range(n)) for n in lens]
    grouped = emb.encode_passages(texts)
    ref = emb._encode(emb._fmt_passages(texts), batch_size=32, group=32)
    assert grouped.shape == (len(texts), 768)
    assert np.array_equal(grouped, ref)
    E5MultilingualEmbedder.release_all()
