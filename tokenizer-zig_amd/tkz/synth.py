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
    6: "C1-bytelevel: C1's docs and vocab under a ByteLevel pre_tokenizer (one pretoken per doc)",
    7: "C1-wide: C1's docs under a 106,608-id BPE vocab with 106,545 merges (wide ids and ranks)",
}
DEFAULT_DOCS = {0: 1000, 1: 1_000_000, 2: 1_000_000, 3: 1_000_000, 4: 64_000_000, 5: 1_000_000, 6: 1_000_000,
                7: 1_000_000}
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
    if os.path.exists(path) and os.path.getsize(path) > 0:
        with open(path, "rb") as f:
            return f.read()
    L = lib()
    n = L.tkz_synth_tokenizer_json(cfg, None, 0)
    if n == 0:
        raise ValueError(f"no config {cfg}")
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


# ---------------------------------------------------------------------------- device
GEN_PATH = os.path.join(_HERE, "libtkzgen.so")
_gen = None


def gen_lib():
    """libtkzgen.so (csrc/gen.hip): the device port of the generator + CSR hashes."""
    global _gen
    if _gen is None:
        if not os.path.exists(GEN_PATH):
            raise RuntimeError(f"{GEN_PATH} missing: run __graft_entry__.build()")
        import tkz  # the HIP runtime and device buffers of libtkz.so

        tkz.lib()
        G = ctypes.CDLL(GEN_PATH)
        vp, u64 = ctypes.c_void_p, ctypes.c_uint64
        G.tkz_gen_create.restype = ctypes.c_int
        G.tkz_gen_create.argtypes = [vp, vp, vp, vp, vp, ctypes.POINTER(vp)]
        G.tkz_gen_destroy.restype = None
        G.tkz_gen_destroy.argtypes = [vp]
        G.tkz_gen_offsets.restype = ctypes.c_int
        G.tkz_gen_offsets.argtypes = [vp, u64, u64, u64, vp, ctypes.POINTER(u64), vp]
        G.tkz_gen_bytes.restype = ctypes.c_int
        G.tkz_gen_bytes.argtypes = [vp, u64, u64, u64, vp, vp, vp]
        G.tkz_csr_hash_device.restype = ctypes.c_int
        G.tkz_csr_hash_device.argtypes = [vp, u64, vp, vp, u64, ctypes.POINTER(u64), vp]
        _gen = G
    return _gen


def tables(cfg: int):
    """Generator tables of config ``cfg`` (tkz_synth_tables): params {kind, fixed_len,
    zmin, n_words, n_cps, n_len}, lexicon codepoints / word offsets, word cdf, length cdf."""
    L = lib()
    L.tkz_synth_tables.restype = ctypes.c_int
    L.tkz_synth_tables.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 5
    p = np.zeros(6, dtype=np.int64)
    if L.tkz_synth_tables(cfg, p.ctypes.data, None, None, None, None):
        raise ValueError(f"no config {cfg}")
    wcp = np.zeros(max(int(p[4]), 1), dtype=np.uint32)
    woff = np.zeros(int(p[3]) + 1, dtype=np.uint32)
    wcdf = np.zeros(max(int(p[3]), 1), dtype=np.float64)
    lcdf = np.zeros(max(int(p[5]), 1), dtype=np.float64)
    L.tkz_synth_tables(cfg, p.ctypes.data, wcp.ctypes.data, woff.ctypes.data, wcdf.ctypes.data, lcdf.ctypes.data)
    return p, wcp, woff, wcdf, lcdf


class DeviceDocs:
    """Docs [first_doc, first_doc + n_docs) of config ``cfg`` generated in HBM by the
    device port of the generator (byte-identical to ``docs``): ``d_bytes`` (readable and
    zero-padded to a multiple of 16 past ``total``) and ``d_off`` (n_docs + 1 u64), as
    tkz.DeviceBuffer. No host staging: a rank generates its own shard."""

    def __init__(self, cfg: int, n_docs: int, first_doc: int = 0, seed: int = BENCH_SEED):
        import tkz

        G = gen_lib()
        p, wcp, woff, wcdf, lcdf = tables(cfg)
        h = ctypes.c_void_p()
        if G.tkz_gen_create(p.ctypes.data, wcp.ctypes.data, woff.ctypes.data, wcdf.ctypes.data, lcdf.ctypes.data,
                            ctypes.byref(h)):
            raise RuntimeError("tkz_gen_create failed")
        try:
            self.cfg, self.n_docs, self.first_doc = cfg, int(n_docs), int(first_doc)
            self.d_off = tkz.DeviceBuffer((self.n_docs + 1) * 8)
            total = ctypes.c_uint64(0)
            if G.tkz_gen_offsets(h, seed, first_doc, n_docs, self.d_off.ptr, ctypes.byref(total), None):
                raise RuntimeError("tkz_gen_offsets failed")
            self.total = int(total.value)
            padded = ((self.total + 16 + 15) // 16) * 16
            self.d_bytes = tkz.DeviceBuffer(padded)
            self.d_bytes.zero()
            if G.tkz_gen_bytes(h, seed, first_doc, n_docs, self.d_off.ptr, self.d_bytes.ptr, None):
                raise RuntimeError("tkz_gen_bytes failed")
        finally:
            G.tkz_gen_destroy(h)

    def host(self):
        """(bytes, doc_off) copied back (tests)."""
        off = np.zeros(self.n_docs + 1, dtype=np.uint64)
        self.d_off.download(off)
        buf = np.zeros(((self.total + 15) // 16) * 16, dtype=np.uint8)
        if self.total:
            self.d_bytes.download(buf, self.total)
        return buf, off

    def free(self):
        self.d_bytes.free()
        self.d_off.free()


def csr_hash_device(batch) -> dict:
    """tests/shard_hash.py's rolling hashes of a tkz.DeviceBatch's last result, on the
    device: {n_docs, n_tokens, row_ptr, ids, offsets} (hex), comparable with the committed
    oracle hashes (tests/golden/*.json)."""
    nt = batch.n_tokens()
    out = (ctypes.c_uint64 * 3)()
    if gen_lib().tkz_csr_hash_device(batch.d_row.ptr, batch.n_docs, batch.d_ids.ptr, batch.d_offs.ptr, nt, out, None):
        raise RuntimeError("tkz_csr_hash_device failed")
    return {"n_docs": batch.n_docs, "n_tokens": nt, "row_ptr": f"{out[0]:016x}", "ids": f"{out[1]:016x}",
            "offsets": f"{out[2]:016x}"}
