"""Drop-in replacements for rag.retrieval (same names and signatures).

    ChromaVectorStore  -> GpuVectorStore (HBM corpus, exact cosine, K1)
    build_where_filter -> same semantics
    BM25Store          -> HBM postings, rank_bm25 semantics (K2/K3)
    rrf_fuse / HybridRetriever -> device RRF / MMR (K4/K5)
    expand_with_neighbors      -> neighbour expansion over the resident BM25 catalog
"""
from .bm25 import BM25Store
from .expand import apply_expansion_and_diversity, expand_with_neighbors, stable_chunk_id
from .filters import build_where_filter
from .fusion import HybridRetriever, _mmr_order, rrf_fuse
from .tokenize import _tokenize, detect_lang_tag
from .vector_store import ChromaVectorStore, GpuVectorStore

__all__ = ["ChromaVectorStore", "GpuVectorStore", "build_where_filter", "BM25Store", "rrf_fuse", "HybridRetriever",
           "expand_with_neighbors", "apply_expansion_and_diversity", "stable_chunk_id"]
