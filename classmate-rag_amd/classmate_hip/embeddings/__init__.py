"""E5 embedder on PyTorch-ROCm with the HIP pooling epilogue.

Replaces ``rag.embeddings.E5MultilingualEmbedder`` (rag/embeddings/__init__.py:45-105):
same constructor arguments, ``query: `` / ``passage: `` prefixes, batch 32,
mean pooling over the attention mask and L2 normalisation, fp32 numpy output.

* The XLM-R (E5-base: 12 layers, d=768, 12 heads, FFN 3072, vocab 250002)
  forward runs in PyTorch-ROCm, in fp32 by default -- the reference's precision
  (sentence-transformers on torch fp32, rag/embeddings/__init__.py:87-94).
  ``dtype="bfloat16"`` (or ``CM_E5_DTYPE=bfloat16``) is the opt-in fast path;
  its drift from fp32 is bounded by tests/test_gpu_scale.py.
* Mean-pool + L2-normalise is the hand-written HIP kernel K6
  (``cm_meanpool_l2norm``), reading the hidden states in place.

Weights: ``model_name`` may be a local directory with a Hugging Face
checkpoint (config + weights + tokenizer) or a hub id already present in the
local HF cache; nothing is downloaded.  ``E5MultilingualEmbedder.random_init()``
builds the same architecture with seeded random weights and a deterministic
hashing tokenizer — what the benchmark uses offline (embedding parity with the
real E5 weights is therefore unpinned; the pooling kernel is pinned against a
torch fp32 reference).
"""
from __future__ import annotations

import contextlib
import hashlib
import math
import os
import threading
import re
import warnings
from typing import Iterable, List, Optional

import numpy as np

from .. import engine

E5_BASE_CONFIG = dict(vocab_size=250002, hidden_size=768, num_hidden_layers=12, num_attention_heads=12,
                      intermediate_size=3072, max_position_embeddings=514, type_vocab_size=1,
                      layer_norm_eps=1e-5, pad_token_id=1, bos_token_id=0, eos_token_id=2)
MAX_SEQ_LEN = 512  # sentence-transformers max_seq_length of multilingual-e5-base


_DTYPES = {"float32": "float32", "fp32": "float32", "bfloat16": "bfloat16", "bf16": "bfloat16"}


def _resolve_dtype(dtype: Optional[str]) -> str:
    """Forward dtype: the argument, else $CM_E5_DTYPE, else fp32 (the reference's precision)."""
    name = dtype or os.environ.get("CM_E5_DTYPE") or "float32"
    if name not in _DTYPES:
        raise ValueError(f"unsupported E5 dtype {name!r} (float32 or bfloat16)")
    return _DTYPES[name]


class HashTokenizer:
    """Deterministic offline stand-in for the XLM-R sentencepiece tokenizer.

    Words -> stable ids in [5, vocab) via blake2b; <s>=0, </s>=2, <pad>=1.
    Only used with random-init weights (no real vocabulary is available)."""

    _MEMO_MAX = 1 << 20   # word -> id memo (cleared when full): a query batch repeats words

    def __init__(self, vocab_size: int = 250002):
        self.vocab_size = vocab_size
        self._re = re.compile(r"\w+|[^\w\s]", re.UNICODE)
        self._memo = {}

    def _word_id(self, w: str) -> int:
        h = int.from_bytes(hashlib.blake2b(w.encode("utf-8"), digest_size=8).digest(), "little")
        i = 5 + h % (self.vocab_size - 5)
        if len(self._memo) >= self._MEMO_MAX:
            self._memo.clear()
        self._memo[w] = i
        return i

    def encode(self, text: str, max_len: int = MAX_SEQ_LEN) -> List[int]:
        memo = self._memo
        ids = [0]
        for w in self._re.findall(text or ""):
            i = memo.get(w)
            ids.append(i if i is not None else self._word_id(w))
        ids = ids[: max_len - 1] + [2]
        return ids

    def __call__(self, texts: List[str], max_len: int = MAX_SEQ_LEN):
        enc = [self.encode(t, max_len) for t in texts]
        s = max(len(e) for e in enc)
        ids = np.ones((len(enc), s), np.int64)
        mask = np.zeros((len(enc), s), np.int64)
        for i, e in enumerate(enc):
            ids[i, : len(e)] = e
            mask[i, : len(e)] = 1
        return ids, mask


def _act_scale(bound: float) -> float:
    """Power-of-two a_scale for K10 with |x| * a_scale <= 2^15 (< f16 max 65504) given |x| <= bound."""
    return (2.0 ** 15) / engine._pow2_at_most(bound) / 2.0 if bound > 0 else 1.0


def _f16x3_layers(layers, emb_ln, D: int):
    """Per layer: the four projections as K10 weights (engine.F16x3Weight) + the a_scale of each
    GEMM input, from rigorous bounds on the activations (no data needed):
      * LayerNorm output x = z * gamma + beta with sum(z^2) <= D, so |x_i| <= sqrt(D) max|gamma| +
        max|beta| and ||x||_2 <= sqrt(D) max|gamma| + ||beta||_2 (QKV and FFN-up inputs);
      * attention output: a convex combination of V rows, |o_i| <= max over tokens |v_i| with
        v = x Wv^T + bv, |v_i| <= ||x||_2 ||Wv_i||_2 + |bv_i| (O-projection input);
      * GELU output: |gelu(u)| <= max(|u|, 0.17), u = x Wi^T + bi bounded the same way
        (FFN-down input).
      * Q, K, V: |y_i| <= ||x||_2 ||W_i||_2 + |b_i| over all three thirds (the scale of the QKV planes
        that K9P reads, CM_EPI_PLANES_QKV).
    Returns tuples (wqkv, a_qkv, wo, a_o, g1, b1, wi, a_i, w2, a_2, g2, b2, s_qkv)."""
    import torch
    sq = math.sqrt(D)

    def ln_bounds(g, b):
        gm = float(g.abs().max())
        return sq * gm + float(b.abs().max()), sq * gm + float(b.norm())

    def proj_bound(l2, w, b):
        return l2 * float(w.norm(dim=1).max()) + float(b.abs().max())

    out = []
    prev_ln = (emb_ln.weight, emb_ln.bias)
    with torch.no_grad():
        for (wqkv, bqkv, wo, bo, g1, b1, wi, bi, w2, b2, g2, bb2) in layers:
            x_inf, x_l2 = ln_bounds(*prev_ln)
            o_bound = proj_bound(x_l2, wqkv[2 * D:], bqkv[2 * D:])
            y_inf, y_l2 = ln_bounds(g1, b1)
            h_bound = max(proj_bound(y_l2, wi, bi), 0.17)
            qkv_bound = proj_bound(x_l2, wqkv, bqkv)
            out.append((engine.F16x3Weight(wqkv, bqkv), _act_scale(x_inf),
                        engine.F16x3Weight(wo, bo), _act_scale(o_bound), g1, b1,
                        engine.F16x3Weight(wi, bi), _act_scale(y_inf),
                        engine.F16x3Weight(w2, b2), _act_scale(h_bound), g2, bb2, _act_scale(qkv_bound)))
            prev_ln = (g2, bb2)
    return out


# Loaded embedders by (model_name, device, dtype, normalize): the reference constructs
# E5MultilingualEmbedder on every ask / ingest call (rag/pipeline/rag.py:334,533), and loading the
# weights, splitting them into K10's planes and capturing the query graphs is seconds of work; a
# construction with a key already loaded in this process attaches to that instance's state instead
# (VERDICT r4 #3).  ``share_as`` registers an instance under another name (offline benchmarks
# register the random-init model under the production model name).
_LOADED: dict = {}
_LOADED_LOCK = threading.Lock()


class E5MultilingualEmbedder:
    def __init__(self, model_name: str = "intfloat/multilingual-e5-base", device: Optional[str] = None,
                 normalize: bool = True, dtype: Optional[str] = None, _model=None, _tokenizer=None):
        import torch
        self.normalize = bool(normalize)
        self.model_name = model_name
        self.device = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
        if self.device.type != "cuda":
            # deliberate divergence: the reference also runs on CPU; this
            # build's pooling epilogue is a HIP kernel and there is no CPU fallback
            raise RuntimeError("E5MultilingualEmbedder needs a ROCm GPU (the pooling epilogue is a HIP kernel); "
                               f"device={device!r} is not supported")
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.dtype = getattr(torch, _resolve_dtype(dtype))
        if _model is None:
            key = self._key(model_name)
            with _LOADED_LOCK:
                prim = _LOADED.get(key)
            if prim is not None:
                self.__dict__ = prim.__dict__   # the loaded model, K10 planes, graphs and caches
                return
            _model, _tokenizer = self._load(model_name)
            self.model = _model.to(self.device, self.dtype).eval()
            self.tokenizer = _tokenizer
            self._graphs = {}
            self._enc_lock = threading.RLock()
            with _LOADED_LOCK:
                _LOADED.setdefault(key, self)
            return
        self.model = _model.to(self.device, self.dtype).eval()
        self.tokenizer = _tokenizer
        self._graphs = {}
        # one encode at a time per model (instances attached by name share it): the lean forward,
        # the small-batch graphs and their input / output buffers are built once and shared
        self._enc_lock = threading.RLock()

    def _key(self, model_name: str):
        return (str(model_name), str(self.device), str(self.dtype), self.normalize)

    def share_as(self, model_name: str) -> "E5MultilingualEmbedder":
        """Later ``E5MultilingualEmbedder(model_name, device, dtype=..., normalize=...)`` calls with
        this instance's device / dtype / normalize attach to it instead of loading ``model_name``."""
        with _LOADED_LOCK:
            _LOADED[self._key(model_name)] = self
        return self

    @staticmethod
    def release_all() -> None:
        with _LOADED_LOCK:
            _LOADED.clear()

    # ------------------------------------------------------------------
    @staticmethod
    def _load(model_name: str):
        from transformers import AutoModel, AutoTokenizer
        local = os.path.isdir(model_name)
        kw = dict(local_files_only=True)
        try:
            tok = AutoTokenizer.from_pretrained(model_name, **kw)
            model = AutoModel.from_pretrained(model_name, attn_implementation="sdpa", **kw)
        except Exception as e:  # no network: only local checkpoints work
            raise RuntimeError(f"cannot load {model_name!r} from local files ({'dir' if local else 'HF cache'}): {e}."
                               " Use E5MultilingualEmbedder.random_init() for offline benchmarking.") from e
        return model, tok

    @classmethod
    def random_init(cls, seed: int = 0, device: Optional[str] = None, normalize: bool = True,
                    dtype: Optional[str] = None, num_layers: int = 12):
        """E5-base architecture with seeded random weights (no checkpoint available offline).
        The weights are drawn in fp32 and then cast, so every dtype gets the same model."""
        import torch
        from transformers import XLMRobertaConfig, XLMRobertaModel
        dtype = _resolve_dtype(dtype)
        cfg = XLMRobertaConfig(**{**E5_BASE_CONFIG, "num_hidden_layers": num_layers})
        cfg._attn_implementation = "sdpa"
        torch.manual_seed(seed)
        dev = torch.device(device or "cuda")
        with torch.device(dev):
            model = XLMRobertaModel(cfg, add_pooling_layer=False).to(getattr(torch, dtype))
        return cls(model_name="random-init:xlm-roberta-base", device=str(dev), normalize=normalize, dtype=dtype,
                   _model=model, _tokenizer=HashTokenizer(cfg.vocab_size))

    # ------------------------------------------------------------------
    @staticmethod
    def _fmt_queries(queries: Iterable[str]) -> List[str]:
        return [f"query: {q}" for q in queries]

    @staticmethod
    def _fmt_passages(texts: Iterable[str]) -> List[str]:
        return [f"passage: {t}" for t in texts]

    def _tokenize_host(self, texts: List[str]):
        """(ids, mask) int64 numpy arrays, padded to the longest text (truncation at 512 tokens)."""
        if isinstance(self.tokenizer, HashTokenizer):
            ids, mask = self.tokenizer(texts)
        else:
            enc = self.tokenizer(texts, padding=True, truncation=True, max_length=MAX_SEQ_LEN, return_tensors="np")
            ids, mask = enc["input_ids"], enc["attention_mask"]
        return np.ascontiguousarray(ids), np.ascontiguousarray(mask)

    def _to_dev(self, a: np.ndarray):
        """A host array on the device through pinned memory, stream-ordered: the host does not wait for
        the kernels already queued (a pageable copy would), so the next batch's tokenization overlaps
        the previous batch's forward."""
        import torch
        return torch.from_numpy(np.ascontiguousarray(a)).pin_memory().to(self.device, non_blocking=True)

    def _tokenize(self, texts: List[str]):
        ids, mask = self._tokenize_host(texts)
        return self._to_dev(ids), self._to_dev(mask)

    def encode_token_ids(self, input_ids, attention_mask, out=None, all_ones: Optional[bool] = None):
        """Device path: (B,S) int ids + mask on the GPU -> (B,768) fp32 unit rows on the GPU.
        Runs the lean forward (padded batches: per-row positions + key-masked SDPA); CM_E5_LEAN=0
        runs the Hugging Face module instead (``_encode_hf``, the reference's computation, which
        the GPU tests hold the lean forward to: 2e-5 in fp32).  ``all_ones``: the caller knows whether
        the mask has padding (True: none, False: some), which spares the forward its device-to-host
        check of the mask."""
        import torch
        if os.environ.get("CM_E5_LEAN", "1") == "0":
            return self._encode_hf(input_ids, attention_mask, out=out)
        with self._enc_lock, torch.inference_mode():
            fwd = self._lean_forward()
            g = self._small_batch_graph(input_ids, attention_mask)
            if g is not None:
                return g if out is None else out.copy_(g)
            if all_ones is None:
                hidden = fwd(input_ids, attention_mask)
            elif all_ones:
                hidden = fwd(input_ids, None)                       # unpadded path, no mask check
            else:
                hidden = fwd(input_ids, attention_mask, padded=True)
            return engine.meanpool_l2norm(hidden, attention_mask, self.normalize, out=out)

    _SMALL_B, _SMALL_S = (8, 32)

    def _small_batch_graph(self, ids, mask):
        """Small fp32 batches (B <= 8, S <= 32: single queries) are launch-bound (~100 kernels of a
        few us each): they replay a hipGraph of the K10 lean forward captured per (B, S bucket of
        16 / 32), the tokens right-padded into the bucket and masked (key-masked HIP attention,
        positions from the non-pad tokens, masked mean pool -- the padded batch semantics of the
        reference's HF forward).  Returns a fresh (B, 768) tensor, or None where it does not apply
        (CM_E5_SMALL_GRAPH=0 disables it)."""
        import torch
        B, S = ids.shape
        if (not getattr(self, "f16x3", False) or B > self._SMALL_B or S > self._SMALL_S
                or getattr(self, "_small_graph_failed", False)
                or os.environ.get("CM_E5_SMALL_GRAPH", "1") == "0" or torch.cuda.is_current_stream_capturing()):
            return None
        Sb = 16 if S <= 16 else 32
        cache = self.__dict__.setdefault("_small_graphs", {})
        key = (B, Sb, ids.device)
        ent = cache.get(key)
        if ent is None:
            pad = self.model.config.pad_token_id
            g_ids = torch.full((B, Sb), pad, dtype=torch.long, device=ids.device)
            g_mask = torch.zeros((B, Sb), dtype=torch.long, device=ids.device)
            g_ids[:, 0] = 0
            g_mask[:, 0] = 1
            g_out = torch.empty((B, self.model.config.hidden_size), dtype=torch.float32, device=ids.device)
            fwd = self._lean_forward()

            def run():
                hidden = fwd(g_ids, g_mask, padded=True)
                engine.meanpool_l2norm(hidden, g_mask, self.normalize, out=g_out)

            side = torch.cuda.Stream(device=ids.device)
            side.wait_stream(torch.cuda.current_stream(ids.device))
            with torch.cuda.stream(side):
                run()
            torch.cuda.current_stream(ids.device).wait_stream(side)
            graph = torch.cuda.CUDAGraph()
            try:
                # thread_local: other threads' HIP calls (another store's search) do not invalidate
                # this capture, and nothing of theirs is captured (the capture stream is private)
                with torch.cuda.graph(graph, capture_error_mode="thread_local"):
                    run()
            except RuntimeError as e:   # capture refused: the eager forward from now on, said once
                self._small_graph_failed = True
                warnings.warn(f"E5 small-batch graph capture failed ({e}); using the eager forward")
                return None
            ent = cache[key] = (g_ids, g_mask, g_out, graph, pad)
        g_ids, g_mask, g_out, graph, pad = ent
        # the graph's buffers are shared: one host thread at a time from the input fill to the output
        # copy, and each use ordered after the previous one on the device (callers on other streams)
        # 
        with self.__dict__.setdefault("_small_graph_lock", threading.Lock()):
            cur = torch.cuda.current_stream(ids.device)
            last = self.__dict__.get("_small_graph_done")
            if last is not None:
                cur.wait_event(last)
            g_ids.fill_(pad)
            g_mask.zero_()
            g_ids[:, :S].copy_(ids)
            g_mask[:, :S].copy_(mask)
            graph.replay()
            res = g_out.clone()
            done = torch.cuda.Event()
            done.record(cur)
            self._small_graph_done = done
        return res

    def _encode_hf(self, input_ids, attention_mask, out=None):
        """The Hugging Face XLM-R module forward + K6 pooling."""
        import torch
        with torch.inference_mode():
            hidden = self.model(input_ids=input_ids, attention_mask=attention_mask).last_hidden_state
            return engine.meanpool_l2norm(hidden, attention_mask, self.normalize, out=out)

    def _lean_forward(self):
        """XLM-R encoder forward for unpadded batches from this model's own weights (same math as
        the HF module: embeddings + LayerNorm, 12 x [self-attention, residual + LayerNorm, GELU
        MLP, residual + LayerNorm]) with the Q/K/V projections fused into one GEMM and attention
        through unmasked SDPA (the flash kernel).  Every "residual add + LayerNorm" (and the
        embeddings' sum + LayerNorm) is one pass of the HIP kernel cm_add_layernorm instead of
        torch's add kernel + LayerNorm kernel (CM_E5_FUSED_LN=0 restores the torch pair), and for
        S <= 64 attention is cm_short_attention reading the QKV GEMM output in place
        (CM_E5_FUSED_ATTN=0 restores permute + SDPA + transpose).
        Built once; returns fwd(ids) -> hidden."""
        import torch
        import torch.nn.functional as F
        if getattr(self, "_lean", None) is not None:
            return self._lean
        m = self.model
        cfg = m.config
        H = cfg.num_attention_heads
        D = cfg.hidden_size
        eps = cfg.layer_norm_eps
        pad = cfg.pad_token_id
        emb = m.embeddings
        layers = []
        with torch.no_grad():
            for L in m.encoder.layer:
                a = L.attention
                wqkv = torch.cat([a.self.query.weight, a.self.key.weight, a.self.value.weight], 0).contiguous()
                bqkv = torch.cat([a.self.query.bias, a.self.key.bias, a.self.value.bias], 0).contiguous()
                layers.append((wqkv, bqkv, a.output.dense.weight, a.output.dense.bias, a.output.LayerNorm.weight,
                               a.output.LayerNorm.bias, L.intermediate.dense.weight, L.intermediate.dense.bias,
                               L.output.dense.weight, L.output.dense.bias, L.output.LayerNorm.weight,
                               L.output.LayerNorm.bias))

        fused = os.environ.get("CM_E5_FUSED_LN", "1") != "0" and self.dtype in (torch.bfloat16, torch.float32)
        fused_attn = (os.environ.get("CM_E5_FUSED_ATTN", "1") != "0" and D // H == 64
                      and self.dtype in (torch.bfloat16, torch.float32))
        scale = 1.0 / math.sqrt(D // H)
        # fp32: the projections run on K10 (split-precision f16 MFMAs, fp32 accuracy) unless
        # CM_E5_F16X3=0 (then torch's fp32 GEMMs on hipBLASLt)
        self.f16x3 = (self.dtype == torch.float32 and fused and os.environ.get("CM_E5_F16X3", "1") != "0"
                      and D % 64 == 0 and cfg.intermediate_size % 64 == 0)
        if self.f16x3:
            layers = _f16x3_layers(layers, emb.LayerNorm, D)
        if fused:
            def add_ln(x, r, g, b):
                return engine.add_layernorm(x, r, g, b, eps)
        else:
            def add_ln(x, r, g, b):
                return F.layer_norm(x + r, (D,), g, b, eps)

        def embed(ids, mask, padded=False):
            """word + position/type embeddings -> (x0 input of the embedding LayerNorm, residual, keep).
            padded=True takes the padded-batch path without the host-side all-ones check (graphs)."""
            B, S = ids.shape
            keep = None
            if mask is not None and (padded or not bool(mask.all())):
                # padded rows (HF semantics): positions from the non-pad tokens
                # (create_position_ids_from_input_ids), padded keys masked out of attention
                npad = ids.ne(pad).int()
                pos = (torch.cumsum(npad, 1) * npad).long() + pad
                pt = emb.position_embeddings(pos) + emb.token_type_embeddings.weight[0]   # (B, S, D)
                keep = mask[:, None, None, :].bool()
            else:
                # unpadded rows: XLM-R position ids are padding_idx + 1 .. padding_idx + S
                pos = torch.arange(pad + 1, pad + 1 + S, device=ids.device)
                pt = emb.position_embeddings(pos) + emb.token_type_embeddings.weight[0]   # (S, D), tiled
                if not fused:
                    pt = pt[None]
            return emb.word_embeddings(ids), pt, keep

        def sdpa(qkv, B, S, keep):
            qkv = qkv.view(B, S, 3, H, D // H).permute(2, 0, 3, 1, 4)
            o = F.scaled_dot_product_attention(qkv[0], qkv[1], qkv[2], attn_mask=keep)
            return o.transpose(1, 2).reshape(B, S, D)

        # passages (32 < S <= 512): the QKV projection writes planes and K9P attends on them
        # (CM_E5_PLANES_ATTN=0: fp32 QKV rows + K9L, the round-4 path)
        planes_attn = fused_attn and os.environ.get("CM_E5_PLANES_ATTN", "1") != "0"

        def fwd_f16x3(ids, mask=None, padded=False):
            # K10 path: every GEMM operand is produced directly as split planes (K8 / attention /
            # the FFN-up epilogue write them), so the projections are pure LDS-DMA + MFMA kernels
            B, S = ids.shape
            if planes_attn and 32 < S <= 512 and S % 64 and os.environ.get("CM_E5_LONG_ATTN", "1") != "0":
                # K9P takes whole 64-key chunks: pad with masked pad tokens (HF position ids of the
                # real tokens unchanged, padded keys leave every softmax exactly) and drop the rows
                Sp = (S + 63) // 64 * 64
                ids_p = ids.new_full((B, Sp), pad)
                ids_p[:, :S] = ids
                mask_p = ids.new_zeros((B, Sp))
                mask_p[:, :S] = 1 if mask is None else mask
                return fwd_f16x3(ids_p, mask_p, padded=True)[:, :S]
            w0, pt, keep = embed(ids, mask, padded)
            x, xp = engine.add_layernorm_split(w0, pt, emb.LayerNorm.weight, emb.LayerNorm.bias, eps, layers[0][1])
            # S <= 32: K9s (one wave per (sequence, head)); longer sequences -- passages up to 512
            # tokens -- K9P on the QKV planes (K9L on fp32 QKV rows with CM_E5_PLANES_ATTN=0; 64-key
            # chunks, online softmax); all key-masked on padded batches and all write the O
            # projection's planes.  CM_E5_LONG_ATTN=0 / CM_E5_MASKED_ATTN=0 restore torch
            # SDPA + a split pass for those cases.
            short = fused_attn and S <= 32 and (keep is None or os.environ.get("CM_E5_MASKED_ATTN", "1") != "0")
            long_ = fused_attn and S > 32 and os.environ.get("CM_E5_LONG_ATTN", "1") != "0"
            km = mask.to(torch.int32).contiguous() if (short or long_) and keep is not None else None
            kp = long_ and planes_attn and S % 64 == 0 and S <= 512
            for li, (wqkv, a_qkv, wo, a_o, g1, b1, wi, a_i, w2, a_2, g2, bb2, s_qkv) in enumerate(layers):
                qkv = None if kp else engine.linear_f16x3(xp, wqkv)
                if kp:      # QKV planes -> K9P -> the O operand planes (no fp32 QKV rows)
                    qp = engine.linear_f16x3(xp, wqkv, qkv=True, planes_out=s_qkv)
                    op = engine.planes_attention(qp, B, S, H, scale, a_o, key_mask=km)
                elif short:   # HIP attention reads the QKV output in place and writes the O operand planes
                    op = engine.short_attention_split(qkv.view(B, S, 3 * D), H, scale, a_o, key_mask=km)
                elif long_:
                    op = engine.long_attention_split(qkv.view(B, S, 3 * D), H, scale, a_o, key_mask=km)
                elif fused_attn and S <= 64 and keep is None:
                    op = engine.short_attention_split(qkv.view(B, S, 3 * D), H, scale, a_o)
                else:
                    op = engine.split_rows(sdpa(qkv, B, S, keep), a_o)
                x, xp = engine.add_layernorm_split(x, engine.linear_f16x3(op, wo), g1, b1, eps, a_i)
                hp = engine.linear_f16x3(xp, wi, gelu=True, planes_out=a_2)   # GELU + split fused
                y = engine.linear_f16x3(hp, w2)
                if li + 1 < len(layers):
                    x, xp = engine.add_layernorm_split(x, y, g2, bb2, eps, layers[li + 1][1])
                else:
                    x = add_ln(x, y, g2, bb2)
            return x.view(B, S, D)

        def fwd(ids, mask=None, padded=False):
            B, S = ids.shape
            w0, pt, keep = embed(ids, mask, padded)
            x = add_ln(w0, pt, emb.LayerNorm.weight, emb.LayerNorm.bias)
            short = fused_attn and S <= 64 and keep is None
            for (wqkv, bqkv, wo, bo, g1, b1, wi, bi, w2, b2, g2, bb2) in layers:
                if short:   # HIP kernel reads the QKV GEMM output in place, writes (B, S, D)
                    o = engine.short_attention(F.linear(x, wqkv, bqkv), H, scale)
                else:
                    o = sdpa(F.linear(x, wqkv, bqkv), B, S, keep)
                x = add_ln(x, F.linear(o, wo, bo), g1, b1)
                h = F.gelu(F.linear(x, wi, bi))
                x = add_ln(x, F.linear(h, w2, b2), g2, bb2)
            return x

        if self.f16x3:
            fwd = fwd_f16x3
        self._lean = fwd
        return fwd

    @staticmethod
    @contextlib.contextmanager
    def _tuned_gemms():
        """TunableOp lookup of the hipBLASLt solutions measured on MI355X for the E5 GEMM shapes of
        a 256 x 24-token query batch (tunableop_e5_gfx950.csv; tools/tune_probe.sh regenerates it),
        scoped to a graph capture: the table is read first and lookup is switched on only if it
        loaded; no tuning, no recording of untuned shapes, results file /dev/null; the enable,
        tuning, recording and filename flags are restored on exit (the captured graph keeps the
        tuned kernels).  The table's entries stay in the process's TunableOp results table (torch
        has no way to drop them), so the table is skipped when the host application already uses
        TunableOp (enabled, or a results file set): its own results are never mixed with ours.
        Yields whether the table is in use.  CM_E5_TUNABLEOP=0 disables it."""
        import torch.cuda.tunable as tun
        table = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tunableop_e5_gfx950.csv")
        host_uses = tun.is_enabled() or bool(os.environ.get("PYTORCH_TUNABLEOP_FILENAME"))
        if os.environ.get("CM_E5_TUNABLEOP", "1") == "0" or not os.path.exists(table) or host_uses:
            yield False
            return
        prev = (tun.is_enabled(), tun.tuning_is_enabled(), tun.record_untuned_is_enabled(), tun.get_filename())
        ok = False
        try:
            tun.tuning_enable(False)
            tun.record_untuned_enable(False)
            tun.set_filename(os.devnull)
            ok = bool(tun.read_file(table))
            tun.enable(ok)
            yield ok
        finally:
            tun.enable(prev[0])
            tun.tuning_enable(prev[1])
            tun.record_untuned_enable(prev[2])
            if prev[3]:
                tun.set_filename(prev[3])

    def capture_graph(self, batch: int, seq_len: int, unpadded: bool = False):
        """HIP-graph the device encode for a fixed (batch, seq_len) (hipGraph via torch.cuda.CUDAGraph:
        one replay instead of ~200 small launches per batch).  Returns (ids, mask, out, graph): fill
        ids/mask in place, graph.replay() writes out (B, 768) fp32.  The 2-D mask becomes the 4-D
        boolean attention mask inside the graph, so no host-side all-ones check runs.  unpadded=True
        (the caller guarantees every mask entry is 1, e.g. fixed-length query batches) captures the
        lean forward instead (_lean_forward: fused QKV GEMM, unmasked flash SDPA)."""
        import torch
        dev = next(self.model.parameters()).device
        ids = torch.zeros((batch, seq_len), dtype=torch.long, device=dev)
        mask = torch.ones((batch, seq_len), dtype=torch.long, device=dev)
        out = torch.empty((batch, self.model.config.hidden_size), dtype=torch.float32, device=dev)

        lean = self._lean_forward() if unpadded else None

        def fwd():
            if lean is not None:
                hidden = lean(ids)
            else:
                m4 = mask.bool()[:, None, None, :].expand(batch, 1, seq_len, seq_len)
                hidden = self.model(input_ids=ids, attention_mask=m4).last_hidden_state
            engine.meanpool_l2norm(hidden, mask, self.normalize, out=out)

        with torch.inference_mode(), self._tuned_gemms() as tuned:
            self.tuned_gemms = tuned
            side = torch.cuda.Stream(device=dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                for _ in range(2):
                    fwd()
            torch.cuda.current_stream(dev).wait_stream(side)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                fwd()
        return ids, mask, out, graph

    def _rows_independent(self, seq_len: int) -> bool:
        """True when every kernel of the forward computes a row independently of the other rows of
        its batch and of the batch's pad length: the fp32 K10 path (fixed k order per output row,
        per-row LayerNorm) with the HIP attention -- K9s for S <= 32 and, since round 6, K9P for
        32 < S <= 512 (per sequence; padded keys leave the softmax exactly: a masked score is -inf, so
        an all-masked 64-key chunk leaves the running max, sum and output bit-unchanged).  Torch SDPA
        and hipBLASLt (bf16, the HF module, CM_E5_PLANES_ATTN=0) may pick kernels by batch shape, so
        their rows are only reproduced in sentence-transformers' own batches."""
        if os.environ.get("CM_E5_LEAN", "1") == "0" or seq_len > MAX_SEQ_LEN:
            return False
        self._lean_forward()
        env = os.environ.get
        short_ok = bool(getattr(self, "f16x3", False)) and env("CM_E5_MASKED_ATTN", "1") != "0" \
            and env("CM_E5_FUSED_ATTN", "1") != "0"
        if seq_len <= 32:
            return short_ok
        return short_ok and env("CM_E5_LONG_ATTN", "1") != "0" and env("CM_E5_PLANES_ATTN", "1") != "0"

    def _encode_dev(self, texts: List[str], batch_size: int = 32, group: Optional[int] = None):
        """(len(texts), 768) fp32 device tensor: sentence-transformers' length-sorted batches of
        ``batch_size`` (its encode() default, rag/embeddings/__init__.py:84-103), each through
        encode_token_ids, order restored.  ``group`` > batch_size tokenizes that many texts at once
        and runs them as ONE forward when the rows are provably batch-independent
        (``_rows_independent``); otherwise the group is cut back into the reference's batches
        (each trimmed to its own longest row, exactly what tokenizing that batch alone gives)."""
        with self._enc_lock:
            return self._encode_dev_locked(texts, batch_size, group)

    def _encode_dev_locked(self, texts, batch_size, group):
        import torch
        out = torch.empty((len(texts), self.model.config.hidden_size), dtype=torch.float32, device=self.device)
        if not texts:
            return out
        group = max(group or batch_size, batch_size)
        order = np.argsort([-len(t) for t in texts], kind="stable")

        def run(rows: np.ndarray, ids_h, mask_h, lens):
            """The rows (positions in the group) as one forward, trimmed to their longest; host arrays
            in, pinned stream-ordered copies: no host wait inside the loop."""
            w = int(lens[rows].max())
            m = mask_h[rows, :w]
            emb = self.encode_token_ids(self._to_dev(ids_h[rows, :w]), self._to_dev(m), all_ones=bool(m.all()))
            out[self._to_dev(idx[rows])] = emb.float()

        for s in range(0, len(texts), group):
            idx = order[s: s + group]
            ids_h, mask_h = self._tokenize_host([texts[i] for i in idx])
            lens = mask_h.sum(1)
            allr = np.arange(len(idx))
            if len(idx) <= batch_size:
                run(allr, ids_h, mask_h, lens)
            elif self._rows_independent(ids_h.shape[1]):
                # one forward per attention path the reference's own batches would take (a 32-text
                # batch whose longest row has <= 32 tokens runs K9s, a longer one K9P -- every row
                # of it): per path the rows are batch- and padding-independent, so these forwards
                # give every row the bits its 32-text batch gives it, with 8x fewer launches
                bmax = np.repeat([int(lens[t:t + batch_size].max()) for t in range(0, len(idx), batch_size)],
                                 batch_size)[:len(idx)]
                for rows in (allr[bmax > 32], allr[bmax <= 32]):
                    if rows.size:
                        run(rows, ids_h, mask_h, lens)
            else:
                for t in range(0, len(idx), batch_size):
                    run(allr[t:t + batch_size], ids_h, mask_h, lens)
        return out

    def _encode(self, texts: List[str], batch_size: int = 32, group: Optional[int] = None) -> np.ndarray:
        if not texts:
            return np.zeros((0, self.model.config.hidden_size), np.float32)
        return self._encode_dev(texts, batch_size, group).cpu().numpy()

    # Query batches: sentence-transformers encodes 32 texts per forward.  Up to 256 queries are
    # tokenized together and run as one forward when the rows are batch-independent (the fp32 K10
    # path at <= 32 tokens, _rows_independent): the same embeddings with 8x fewer launches, what a
    # 256-query retrieve_batch call needs.  Otherwise they run in the reference's 32-text batches.
    query_batch_size = 256

    def encode_queries(self, queries: Iterable[str]) -> np.ndarray:
        return self._encode(self._fmt_queries(queries), group=self.query_batch_size).astype("float32", copy=False)

    def encode_queries_dev(self, queries: Iterable[str]):
        """encode_queries, left on the device (the batched retrieval path consumes it there)."""
        return self._encode_dev(self._fmt_queries(queries), group=self.query_batch_size)

    # Passages: the same grouping (round 6) -- 256 texts tokenized together, one forward per attention
    # path of the reference's 32-text batches when the rows are batch-independent (_rows_independent:
    # the fp32 K10 path with K9s / K9P), else the reference's batches.
    passage_batch_size = 256

    def encode_passages(self, texts: Iterable[str]) -> np.ndarray:
        return self._encode(self._fmt_passages(texts), group=self.passage_batch_size).astype("float32", copy=False)


from .cache import CachingEmbedder  # noqa: E402  (rag/embeddings/cache.py drop-in)

__all__ = ["E5MultilingualEmbedder", "CachingEmbedder", "HashTokenizer", "E5_BASE_CONFIG"]
