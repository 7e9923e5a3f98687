"""classmate_hip — MI355X-native hybrid retrieval for CLASSMATE-RAG.

Drop-in replacements for rag.retrieval (ChromaVectorStore, BM25Store,
HybridRetriever, rrf_fuse, build_where_filter) and rag.embeddings
(E5MultilingualEmbedder) over hand-written gfx950 HIP kernels behind the C ABI
in include/classmate_hip.h.
"""
__version__ = "0.1.0"
