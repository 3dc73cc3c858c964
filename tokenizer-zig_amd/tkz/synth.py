"""Synthetic bench/test inputs (libtkzsynth.so): deterministic docs and tokenizer.json
for configs C0..C4 of BASELINE.json. Not part of the encode path."""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TKZ_SYNTH_LIB") or os.path.join(_HERE, "libtkzsynth.so")
_lib = None

# config id -> short description (BASELINE.json "configs" order)
CONFIGS = {
    0: "C0 1k x 256-B ASCII docs, 8k BPE, Whitespace (examples/basic_tokenize plumbing)",
    1: "C1 1M x 512-B ASCII docs, 32k BPE, Whitespace",
    2: "C2 1M x 512-B mixed-UTF-8 docs, 32k BPE, Lowercase normalizer, Whitespace",
    3: "C3 1M x 512-B docs, 30k WordPiece, BertNormalizer + BertPreTokenizer",
    4: "C4 64M docs Zipf(64-4096 B), 50k BPE, Whitespace",
    5: "C1-disjoint: C1's docs and vocab, words from a lexicon the vocab never saw",
}
DEFAULT_DOCS = {0: 1000, 1: 1_000_000, 2: 1_000_000, 3: 1_000_000, 4: 64_000_000, 5: 1_000_000}
BENCH_SEED = 0x746F6B656E  # "token"


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: run __graft_entry__.build()")
        L = ctypes.CDLL(LIB_PATH)
        L.tkz_synth_docs.restype = ctypes.c_uint64
        L.tkz_synth_docs.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                     ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
        L.tkz_synth_tokenizer_json.restype = ctypes.c_uint64
        L.tkz_synth_tokenizer_json.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_uint64]
        _lib = L
    return _lib


def tokenizer_json(cfg: int) -> bytes:
    """tokenizer.json of config ``cfg`` (trained deterministically in C++; cached
    per process and under $TKZ_CACHE or /tmp)."""
    cache_dir = os.environ.get("TKZ_CACHE", os.path.join(os.environ.get("TMPDIR", "/tmp"), "tkz_cache"))
    cfg = {5: 1}.get(cfg, cfg)  # C5 uses C1's tokenizer.json
    path = os.path.join(cache_dir, f"tokenizer_c{cfg}.json")
    if os.path.exists(path):
        with open(path, "rb") as f:
            return f.read()
    L = lib()
    n = L.tkz_synth_tokenizer_json(cfg, None, 0)
    buf = ctypes.create_string_buffer(int(n))
    L.tkz_synth_tokenizer_json(cfg, buf, n)
    data = buf.raw[: int(n)]
    try:
        os.makedirs(cache_dir, exist_ok=True)
        tmp = path + f".{os.getpid()}"
        with open(tmp, "wb") as f:
            f.write(data)
        os.replace(tmp, path)
    except OSError:
        pass
    return data


def docs(cfg: int, n_docs: int, first_doc: int = 0, seed: int = BENCH_SEED, threads: int = 0):
    """Returns (bytes uint8[total (padded to 16)], doc_off uint64[n+1]) for docs
    [first_doc, first_doc + n_docs) of config ``cfg``."""
    L = lib()
    threads = threads or min(16, os.cpu_count() or 1)
    off = np.zeros(n_docs + 1, dtype=np.uint64)
    total = L.tkz_synth_docs(cfg, seed, first_doc, n_docs, None, off.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), 1)
    buf = np.zeros(((int(total) + 15) // 16) * 16, dtype=np.uint8)
    L.tkz_synth_docs(cfg, seed, first_doc, n_docs, buf.ctypes.data_as(ctypes.c_void_p),
                     off.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), threads)
    return buf, off
