"""Python mirror of jrc2139/tokenizer-zig's ``Tokenizer`` API (src/lib.zig:32-224) over
the C ABI of ``include/tkz.h`` (libtkz.so, built in-tree for gfx950).

Encode always runs through the HIP kernels; if the library or a GPU is missing the
encode calls raise — there is no CPU fallback on the product path.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TKZ_LIB") or os.path.join(_HERE, "libtkz.so")

# tkz_status -> Zig error name (src/config.zig:18-30, wordpiece.zig:150,212)
ERROR_NAMES = {
    1: "InvalidJson", 2: "MissingModel", 3: "UnsupportedModelType", 4: "MissingVocab",
    5: "InvalidVocabEntry", 6: "OutOfMemory", 7: "FileNotFound", 8: "FileTooBig",
    9: "MissingUnkToken", 10: "InvalidArgument", 11: "DeviceError",
}


class TokenizerError(Exception):
    def __init__(self, code: int, msg: str = ""):
        self.code = code
        self.name = ERROR_NAMES.get(code, f"Error{code}")
        super().__init__(f"{self.name}: {msg}" if msg else self.name)


class _Offset(ctypes.Structure):
    _fields_ = [("start", ctypes.c_uint32), ("end", ctypes.c_uint32)]


class _Encoding(ctypes.Structure):
    _fields_ = [
        ("len", ctypes.c_size_t),
        ("ids", ctypes.POINTER(ctypes.c_uint32)),
        ("type_ids", ctypes.POINTER(ctypes.c_uint32)),
        ("offsets", ctypes.POINTER(_Offset)),
        ("special_token_mask", ctypes.POINTER(ctypes.c_uint32)),
        ("attention_mask", ctypes.POINTER(ctypes.c_uint32)),
        ("tokens", ctypes.POINTER(ctypes.c_char_p)),
        ("token_lens", ctypes.POINTER(ctypes.c_uint32)),
    ]


class _Batch(ctypes.Structure):
    _fields_ = [
        ("n_docs", ctypes.c_size_t),
        ("n_tokens", ctypes.c_uint64),
        ("row_ptr", ctypes.POINTER(ctypes.c_uint64)),
        ("ids", ctypes.POINTER(ctypes.c_uint32)),
        ("offsets", ctypes.POINTER(_Offset)),
        ("type_ids", ctypes.POINTER(ctypes.c_uint32)),
        ("special_token_mask", ctypes.POINTER(ctypes.c_uint32)),
        ("attention_mask", ctypes.POINTER(ctypes.c_uint32)),
    ]


class _TextBatch(ctypes.Structure):
    _fields_ = [
        ("n_docs", ctypes.c_size_t),
        ("n_bytes", ctypes.c_uint64),
        ("offsets", ctypes.POINTER(ctypes.c_uint64)),
        ("bytes", ctypes.c_void_p),
    ]


class _MemoInfo(ctypes.Structure):
    _fields_ = [("word_entries", ctypes.c_uint64), ("word_bytes", ctypes.c_uint64), ("seg_entries", ctypes.c_uint64),
                ("seg_bytes", ctypes.c_uint64), ("hot_keys", ctypes.c_uint64), ("hot_bitmap_bytes", ctypes.c_uint64),
                ("hot_build_ms", ctypes.c_double)]


class _BatchStats(ctypes.Structure):
    _fields_ = [("pretokens", ctypes.c_uint64), ("memo_hits", ctypes.c_uint64), ("deferred", ctypes.c_uint64),
                ("deferred_model", ctypes.c_uint64), ("sub_batches", ctypes.c_uint64), ("long_words", ctypes.c_uint64),
                ("long_segmented", ctypes.c_uint64), ("long_fallback_bytes", ctypes.c_uint64),
                ("seg_bound_errors", ctypes.c_uint64)]


class _Opts(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int), ("word_memo", ctypes.c_int), ("dedup", ctypes.c_int),
                ("host_chunk", ctypes.c_uint64)]


class _Info(ctypes.Structure):
    _fields_ = [
        ("model", ctypes.c_int), ("normalizer", ctypes.c_int), ("pre_tokenizer", ctypes.c_int),
        ("decoder", ctypes.c_int), ("has_post_processor", ctypes.c_int),
        ("model_vocab_size", ctypes.c_size_t), ("added_vocab_size", ctypes.c_size_t),
        ("n_merges", ctypes.c_size_t), ("unk_id", ctypes.c_uint32),
        ("max_input_chars_per_word", ctypes.c_uint64), ("compact_tables", ctypes.c_int),
        ("merges_ordered", ctypes.c_int), ("long_segments", ctypes.c_int),
    ]


_lib = None


def lib():
    """Loads libtkz.so (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} is missing: run __graft_entry__.build() (hipcc --offload-arch=gfx950)")
    L = ctypes.CDLL(LIB_PATH)
    c = ctypes
    vp, u32, u64, sz = c.c_void_p, c.c_uint32, c.c_uint64, c.c_size_t
    sig = {
        "tkz_create_from_json": (c.c_int, [c.c_char_p, sz, c.POINTER(vp)]),
        "tkz_create_from_file": (c.c_int, [c.c_char_p, c.POINTER(vp)]),
        "tkz_destroy": (None, [vp]),
        "tkz_last_error": (c.c_char_p, []),
        "tkz_get_info": (c.c_int, [vp, c.POINTER(_Info)]),
        "tkz_encode": (c.c_int, [vp, c.c_char_p, sz, c.c_int, c.POINTER(_Encoding)]),
        "tkz_encoding_free": (None, [c.POINTER(_Encoding)]),
        "tkz_encode_batch": (c.c_int, [vp, vp, c.POINTER(u64), sz, c.POINTER(_Batch)]),
        "tkz_batch_free": (None, [c.POINTER(_Batch)]),
        "tkz_encode_batch_gpus": (c.c_int, [vp, vp, c.POINTER(u64), sz, u32, c.POINTER(_Batch)]),
        "tkz_set_virtual_devices": (c.c_int, [vp, c.c_int]),
        "tkz_opts_default": (None, [c.POINTER(_Opts)]),
        "tkz_create_from_json_opts": (c.c_int, [c.c_char_p, sz, c.POINTER(_Opts), c.POINTER(vp)]),
        "tkz_device_workspace_size": (sz, [vp, u64, sz]),
        "tkz_device_workspace_size_sub": (sz, [vp, u64]),
        "tkz_device_workspace_min": (sz, [vp]),
        "tkz_device_batch_stats": (c.c_int, [vp, vp, c.POINTER(_BatchStats)]),
        "tkz_device_batch_stats_stream": (c.c_int, [vp, vp, vp, c.POINTER(_BatchStats)]),
        "tkz_encode_batch_device": (c.c_int, [vp, vp, vp, sz, u64, vp, vp, vp, vp, sz, vp, vp]),
        "tkz_decode": (c.c_int, [vp, c.POINTER(u32), sz, c.c_int, c.POINTER(c.c_void_p), c.POINTER(sz)]),
        "tkz_string_free": (None, [c.c_void_p]),
        "tkz_decode_batch": (c.c_int, [vp, c.POINTER(u64), c.POINTER(u32), sz, c.c_int, c.POINTER(_TextBatch)]),
        "tkz_text_batch_free": (None, [c.POINTER(_TextBatch)]),
        "tkz_decode_bound": (u64, [vp, u64]),
        "tkz_set_truncation": (c.c_int, [vp, c.c_int, sz, sz]),
        "tkz_set_padding": (c.c_int, [vp, c.c_int, sz, u32, u32, c.c_char_p, sz, c.c_int]),
        "tkz_pad_capacity": (u64, [vp, sz, u64]),
        "tkz_pad_workspace_size": (sz, [sz]),
        "tkz_pad_batch_device": (c.c_int, [vp, vp, vp, vp, sz, vp, vp, vp, vp, vp, vp, vp, sz, vp]),
        "tkz_decode_workspace_size": (sz, [vp, sz, u64]),
        "tkz_decode_batch_device": (c.c_int, [vp, vp, vp, sz, u64, c.c_int, vp, u64, vp, vp, sz, vp]),
        "tkz_get_vocab_size": (sz, [vp]),
        "tkz_token_to_id": (c.c_int, [vp, c.c_char_p, sz, c.POINTER(u32)]),
        "tkz_id_to_token": (c.c_void_p, [vp, u32, c.POINTER(sz)]),
        "tkz_add_special_tokens": (sz, [vp, c.POINTER(c.c_char_p), c.POINTER(sz), sz]),
        "tkz_add_special_tokens_ids": (sz, [vp, c.POINTER(c.c_char_p), c.POINTER(sz), c.POINTER(u32), sz]),
        "tkz_device_available": (c.c_int, []),
        "tkz_set_device": (c.c_int, [c.c_int]),
        "tkz_set_long_segments": (c.c_int, [vp, c.c_int]),
        "tkz_set_word_memo": (c.c_int, [vp, c.c_int]),
        "tkz_set_dedup": (c.c_int, [vp, c.c_int]),
        "tkz_get_memo_info": (c.c_int, [vp, c.POINTER(u64), c.POINTER(u64)]),
        "tkz_get_memo_info_ext": (c.c_int, [vp, c.c_void_p]),
        "tkz_set_hot_pairs": (c.c_int, [vp, c.c_int64]),
        "tkz_set_host_pipeline": (c.c_int, [vp, c.c_size_t]),
        "tkz_debug_merge_lookup": (c.c_int, [vp, u32, u32, c.POINTER(u32), c.POINTER(u32)]),
        "tkz_debug_vocab_lookup": (c.c_int, [vp, c.c_char_p, sz, c.POINTER(u32)]),
        "tkz_debug_counters_offset": (sz, [u64, sz]),
        "tkz_dev_alloc": (vp, [sz]),
        "tkz_dev_free": (None, [vp]),
        "tkz_memcpy_htod": (c.c_int, [vp, vp, sz]),
        "tkz_memcpy_dtoh": (c.c_int, [vp, vp, sz]),
        "tkz_memset_dev": (c.c_int, [vp, c.c_int, sz]),
        "tkz_dev_mem_info": (c.c_int, [c.POINTER(sz), c.POINTER(sz)]),
        "tkz_synchronize": (c.c_int, [vp]),
        "tkz_stream_create": (vp, []),
        "tkz_stream_destroy": (None, [vp]),
        "tkz_device_synchronize": (c.c_int, []),
        "tkz_profile_enable": (c.c_int, [vp, c.c_int]),
        "tkz_profile_read": (c.c_int, [vp, c.POINTER(c.c_double), c.POINTER(u64), c.c_int]),
        "tkz_host_profile_read": (c.c_int, [vp, c.POINTER(c.c_double), c.c_size_t, c.c_int]),
        "tkz_host_alloc": (vp, [c.c_size_t]),
        "tkz_host_free": (None, [vp]),
    }
    variant = bool(os.environ.get("TKZ_LIB"))  # A/B builds of older revisions may lack newer entry points
    for name, (res, args) in sig.items():
        if variant and not hasattr(L, name):
            continue
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def _err(rc: int):
    raise TokenizerError(rc, (lib().tkz_last_error() or b"").decode("utf-8", "replace"))


def _check_batch(data: np.ndarray, doc_off) -> np.ndarray:
    """doc_off as contiguous u64; rejects offsets the C ABI would read past `data` with."""
    doc_off = np.ascontiguousarray(doc_off, dtype=np.uint64)
    if doc_off.ndim != 1 or len(doc_off) == 0:
        raise ValueError("doc_off must be a 1-D array of n_docs + 1 offsets")
    if int(doc_off[-1]) > data.size:
        raise ValueError(f"doc_off[-1] = {int(doc_off[-1])} is past the end of data ({data.size} bytes)")
    return doc_off


@dataclass
class Encoding:
    """Encoding (src/encoding.zig:231-241). Offsets are pretoken-relative."""

    ids: List[int]
    type_ids: List[int]
    tokens: List[bytes]
    offsets: List[Tuple[int, int]]
    special_token_mask: List[int]
    attention_mask: List[int]
    words: Optional[List[int]] = None
    overflowing: Tuple = ()

    def __len__(self):
        return len(self.ids)


class Tokenizer:
    """Tokenizer (src/lib.zig:32-224): fromJson / fromFile / encode / decode /
    getVocabSize / tokenToId / idToToken / addSpecialTokens."""

    def __init__(self, handle: int):
        self._h = ctypes.c_void_p(handle)
        self._lib = lib()

    # Tokenizer.fromJson (lib.zig:59-85)
    @classmethod
    def from_json(cls, text, device: Optional[int] = None, word_memo: Optional[bool] = None,
                  dedup: Optional[int] = None, host_chunk: Optional[int] = None) -> "Tokenizer":
        """Any keyword given goes to tkz_create_from_json_opts (tkz_opts); the rest keep
        their defaults (device -1 = current at first GPU use)."""
        data = text.encode("utf-8") if isinstance(text, str) else bytes(text)
        h = ctypes.c_void_p()
        if device is None and word_memo is None and dedup is None and host_chunk is None:
            rc = lib().tkz_create_from_json(data, len(data), ctypes.byref(h))
        else:
            o = _Opts()
            lib().tkz_opts_default(ctypes.byref(o))
            if device is not None:
                o.device = int(device)
            if word_memo is not None:
                o.word_memo = int(bool(word_memo))
            if dedup is not None:
                o.dedup = int(dedup)
            if host_chunk is not None:
                o.host_chunk = int(host_chunk)
            rc = lib().tkz_create_from_json_opts(data, len(data), ctypes.byref(o), ctypes.byref(h))
        if rc:
            _err(rc)
        return cls(h.value)

    # Tokenizer.fromFile (lib.zig:48-56)
    @classmethod
    def from_file(cls, path: str) -> "Tokenizer":
        h = ctypes.c_void_p()
        rc = lib().tkz_create_from_file(path.encode(), ctypes.byref(h))
        if rc:
            _err(rc)
        return cls(h.value)

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            self._lib.tkz_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    def info(self) -> dict:
        inf = _Info()
        rc = self._lib.tkz_get_info(self._h, ctypes.byref(inf))
        if rc:
            _err(rc)
        return {f: getattr(inf, f) for f, _ in _Info._fields_}

    # Tokenizer.encode (lib.zig:109-160)
    def encode(self, text, add_special_tokens: bool = False) -> Encoding:
        data = text.encode("utf-8") if isinstance(text, str) else bytes(text)
        enc = _Encoding()
        rc = self._lib.tkz_encode(self._h, data, len(data), int(add_special_tokens), ctypes.byref(enc))
        if rc:
            _err(rc)
        try:
            n = enc.len
            ids = [enc.ids[i] for i in range(n)]
            offs = [(enc.offsets[i].start, enc.offsets[i].end) for i in range(n)]
            toks = [ctypes.string_at(enc.tokens[i], enc.token_lens[i]) if enc.token_lens[i] else b"" for i in range(n)]
            return Encoding(ids=ids, type_ids=[enc.type_ids[i] for i in range(n)], tokens=toks, offsets=offs,
                            special_token_mask=[enc.special_token_mask[i] for i in range(n)],
                            attention_mask=[enc.attention_mask[i] for i in range(n)])
        finally:
            self._lib.tkz_encoding_free(ctypes.byref(enc))

    # Tokenizer.truncation / Tokenizer.padding fields (lib.zig:41-42)
    def set_truncation(self, max_length: Optional[int] = 512, stride: int = 0) -> None:
        rc = self._lib.tkz_set_truncation(self._h, int(max_length is not None), max_length or 0, stride)
        if rc:
            _err(rc)

    def set_padding(self, length: Optional[int], pad_id: int = 0, pad_type_id: int = 0, pad_token=b"[PAD]",
                    direction: str = "right", enabled: bool = True) -> None:
        tokb = pad_token.encode() if isinstance(pad_token, str) else bytes(pad_token)
        rc = self._lib.tkz_set_padding(self._h, int(enabled), length or 0, pad_id, pad_type_id, tokb, len(tokb),
                                       1 if direction == "left" else 0)
        if rc:
            _err(rc)

    def _run_batch(self, data: np.ndarray, doc_off: np.ndarray, gpu_mask: Optional[int]) -> "_Batch":
        n = len(doc_off) - 1
        b = _Batch()
        dp = data.ctypes.data_as(ctypes.c_void_p)
        op = doc_off.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))
        if gpu_mask is None:
            rc = self._lib.tkz_encode_batch(self._h, dp, op, n, ctypes.byref(b))
        else:
            rc = self._lib.tkz_encode_batch_gpus(self._h, dp, op, n, int(gpu_mask), ctypes.byref(b))
        if rc:
            _err(rc)
        return b

    def set_virtual_devices(self, n: int) -> None:
        """Test hook: gpu_mask bit i -> device i % count (several replicas on one GPU)."""
        rc = self._lib.tkz_set_virtual_devices(self._h, int(n))
        if rc:
            _err(rc)

    def encode_batch_full(self, data, doc_off, gpu_mask: Optional[int] = None) -> dict:
        """encode_batch plus the Encoding masks (type_ids, special_token_mask,
        attention_mask); with truncation/padding applied when set."""
        data = np.ascontiguousarray(np.frombuffer(data, dtype=np.uint8) if isinstance(data, (bytes, bytearray)) else data, dtype=np.uint8)
        doc_off = _check_batch(data, doc_off)
        n = len(doc_off) - 1
        b = self._run_batch(data, doc_off, gpu_mask)
        try:
            T = int(b.n_tokens)
            out = {"row_ptr": np.ctypeslib.as_array(b.row_ptr, shape=(n + 1,)).copy()}

            def arr(p, shape, dflt):
                if not p or T == 0:
                    return np.full(shape, dflt, dtype=np.uint32)
                return np.ctypeslib.as_array(p, shape=shape).copy()
            out["ids"] = arr(b.ids, (T,), 0)
            out["offsets"] = arr(ctypes.cast(b.offsets, ctypes.POINTER(ctypes.c_uint32)), (T, 2), 0)
            out["type_ids"] = arr(b.type_ids, (T,), 0)
            out["special_token_mask"] = arr(b.special_token_mask, (T,), 0)
            out["attention_mask"] = arr(b.attention_mask, (T,), 1)
            return out
        finally:
            self._lib.tkz_batch_free(ctypes.byref(b))

    def encode_batch(self, data, doc_off, gpu_mask: Optional[int] = None) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        """Batched Tokenizer.encode over docs data[doc_off[i]:doc_off[i+1]] (host
        buffers). Returns CSR (row_ptr u64[n+1], ids u32[T], offsets u32[T,2]). gpu_mask:
        encode on the GPUs of the mask (bit i = device i, tkz_encode_batch_gpus)."""
        data = np.ascontiguousarray(np.frombuffer(data, dtype=np.uint8) if isinstance(data, (bytes, bytearray)) else data, dtype=np.uint8)
        doc_off = _check_batch(data, doc_off)
        n = len(doc_off) - 1
        b = self._run_batch(data, doc_off, gpu_mask)
        try:
            T = int(b.n_tokens)
            row_ptr = np.ctypeslib.as_array(b.row_ptr, shape=(n + 1,)).copy()
            if T:
                ids = np.ctypeslib.as_array(b.ids, shape=(T,)).copy()
                offs = np.ctypeslib.as_array(ctypes.cast(b.offsets, ctypes.POINTER(ctypes.c_uint32)), shape=(T, 2)).copy()
            else:
                ids = np.zeros(0, np.uint32)
                offs = np.zeros((0, 2), np.uint32)
            return row_ptr, ids, offs
        finally:
            self._lib.tkz_batch_free(ctypes.byref(b))

    # Tokenizer.decode (lib.zig:163-189)
    def decode(self, ids: Sequence[int], skip_special_tokens: bool = False) -> bytes:
        arr = (ctypes.c_uint32 * max(len(ids), 1))(*ids)
        out = ctypes.c_void_p()
        n = ctypes.c_size_t()
        rc = self._lib.tkz_decode(self._h, arr, len(ids), int(skip_special_tokens), ctypes.byref(out), ctypes.byref(n))
        if rc:
            _err(rc)
        try:
            return ctypes.string_at(out.value, n.value) if n.value else b""
        finally:
            self._lib.tkz_string_free(out)

    def decode_batch(self, row_ptr, ids, skip_special_tokens: bool = False) -> Tuple[np.ndarray, bytes]:
        """Batched Tokenizer.decode on the GPU: sequence i = ids[row_ptr[i]:row_ptr[i+1]].
        Returns (offsets u64[n+1], bytes); sequence i decodes to bytes[offsets[i]:offsets[i+1]]."""
        row_ptr = np.ascontiguousarray(row_ptr, dtype=np.uint64)
        ids = np.ascontiguousarray(ids, dtype=np.uint32)
        n = len(row_ptr) - 1
        b = _TextBatch()
        rc = self._lib.tkz_decode_batch(self._h, row_ptr.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                                        ids.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), n,
                                        int(skip_special_tokens), ctypes.byref(b))
        if rc:
            _err(rc)
        try:
            off = np.ctypeslib.as_array(b.offsets, shape=(n + 1,)).copy()
            data = ctypes.string_at(b.bytes, int(b.n_bytes)) if b.n_bytes else b""
            return off, data
        finally:
            self._lib.tkz_text_batch_free(ctypes.byref(b))

    def get_vocab_size(self) -> int:
        return int(self._lib.tkz_get_vocab_size(self._h))

    def token_to_id(self, token) -> Optional[int]:
        data = token.encode("utf-8") if isinstance(token, str) else bytes(token)
        i = ctypes.c_uint32()
        return int(i.value) if self._lib.tkz_token_to_id(self._h, data, len(data), ctypes.byref(i)) else None

    def id_to_token(self, tid: int) -> Optional[bytes]:
        n = ctypes.c_size_t()
        p = self._lib.tkz_id_to_token(self._h, tid, ctypes.byref(n))
        return None if not p else ctypes.string_at(p, n.value)

    def add_special_tokens(self, tokens: Sequence) -> int:
        """Tokenizer.addSpecialTokens (lib.zig:192-200): items are contents (AddedToken.id
        null: the next free id) or (content, id) pairs. Returns the number newly added."""
        items = [t if isinstance(t, tuple) else (t, None) for t in tokens]
        bs = [c.encode("utf-8") if isinstance(c, str) else bytes(c) for c, _ in items]
        arr = (ctypes.c_char_p * max(len(bs), 1))(*bs)
        lens = (ctypes.c_size_t * max(len(bs), 1))(*[len(b) for b in bs])
        ids = (ctypes.c_uint32 * max(len(bs), 1))(*[0xFFFFFFFF if i is None else int(i) for _, i in items])
        return int(self._lib.tkz_add_special_tokens_ids(self._h, arr, lens, ids, len(bs)))

    def set_dedup(self, mode: int) -> None:
        """Deduplicate memo-missing BPE words per batch: -1 auto, 0 off, 1 on."""
        if not hasattr(self._lib, "tkz_set_dedup"):  # an older A/B build (TKZ_LIB)
            return
        rc = self._lib.tkz_set_dedup(self._h, int(mode))
        if rc:
            _err(rc)

    def set_host_pipeline(self, chunk_bytes: int) -> None:
        """encode_batch copy/compute overlap: input bytes per chunk (0 = off)."""
        rc = self._lib.tkz_set_host_pipeline(self._h, int(chunk_bytes))
        if rc:
            _err(rc)

    def set_long_segments(self, on: bool) -> None:
        """Segmented path for long BPE pretokens (tkz_set_long_segments; same results)."""
        rc = self._lib.tkz_set_long_segments(self._h, int(bool(on)))
        if rc:
            _err(rc)

    def set_word_memo(self, on: bool) -> None:
        """BPE word memo (vocab key -> its BPE tokens, computed by the GPU path)."""
        rc = self._lib.tkz_set_word_memo(self._h, int(on))
        if rc:
            _err(rc)

    # table introspection (host copy of the GPU tables)
    def memo_info(self) -> dict:
        """tkz_get_memo_info: word-memo keys and device table bytes (0 / 0 when off)."""
        if not hasattr(self._lib, "tkz_get_memo_info"):  # an A/B build of an older revision
            return {}
        e, b = ctypes.c_uint64(0), ctypes.c_uint64(0)
        rc = self._lib.tkz_get_memo_info(self._h, ctypes.byref(e), ctypes.byref(b))
        if rc:
            _err(rc)
        out = {"entries": int(e.value), "table_bytes": int(b.value)}
        if hasattr(self._lib, "tkz_get_memo_info_ext"):
            m = _MemoInfo()
            if self._lib.tkz_get_memo_info_ext(self._h, ctypes.byref(m)) == 0:
                out.update({f: (round(getattr(m, f), 2) if f == "hot_build_ms" else int(getattr(m, f)))
                            for f, _ in _MemoInfo._fields_})
        return out

    def set_hot_pairs(self, max_keys: int) -> None:
        """Keys of the hot-pair bitmap (tkz_set_hot_pairs; -1 default, 0 none; same results)."""
        rc = self._lib.tkz_set_hot_pairs(self._h, int(max_keys))
        if rc:
            _err(rc)

    def debug_merge(self, a: int, b: int) -> Optional[Tuple[int, int]]:
        r, n = ctypes.c_uint32(), ctypes.c_uint32()
        return (r.value, n.value) if self._lib.tkz_debug_merge_lookup(self._h, a, b, ctypes.byref(r), ctypes.byref(n)) else None

    def debug_vocab(self, key) -> Optional[int]:
        data = key.encode("utf-8") if isinstance(key, str) else bytes(key)
        i = ctypes.c_uint32()
        return int(i.value) if self._lib.tkz_debug_vocab_lookup(self._h, data, len(data), ctypes.byref(i)) else None


def device_available() -> bool:
    return bool(lib().tkz_device_available())


def set_device(index: int) -> None:
    rc = lib().tkz_set_device(int(index))
    if rc:
        _err(rc)


def profile_enable(tok: "Tokenizer", on: bool = True) -> None:
    lib().tkz_profile_enable(tok.handle, int(on))


HOST_PROFILE_FIELDS = ("calls", "chunks", "bytes_in", "bytes_out", "wall_ms", "alloc_ms", "wait_ms", "fixup_ms",
                       "h2d_ms", "encode_ms", "d2h_ms", "h2d_span_ms", "encode_span_ms", "d2h_span_ms",
                       "first_chunk_ms", "last_d2h_ms", "out_pageable")


def host_profile_read(tok: "Tokenizer", reset: bool = True) -> dict:
    """tkz_host_profile_read: the host-buffer path's timeline (profiling on), summed over
    the calls since the last reset."""
    out = (ctypes.c_double * len(HOST_PROFILE_FIELDS))()
    rc = lib().tkz_host_profile_read(tok.handle, out, len(HOST_PROFILE_FIELDS), int(reset))
    if rc:
        _err(rc)
    return dict(zip(HOST_PROFILE_FIELDS, list(out)))


class _PinnedBlock:
    """Owns one tkz_host_alloc block; freed when the last view of it is gone."""

    def __init__(self, ptr: int):
        self.ptr = ptr

    def __del__(self):
        try:
            if self.ptr:
                lib().tkz_host_free(self.ptr)
                self.ptr = None
        except Exception:
            pass


class HostBuffer:
    """Page-locked host memory (tkz_host_alloc) as a numpy uint8 array: input text staged
    here is copied to the device at the full PCIe rate. The block lives as long as the
    HostBuffer or any numpy view of `array` does (the views hold the owner through their
    base chain), so a view kept after free() or after the HostBuffer is collected stays
    valid; free() only drops this object's reference."""

    def __init__(self, nbytes: int):
        self.nbytes = int(nbytes)
        ptr = lib().tkz_host_alloc(max(self.nbytes, 1))
        if not ptr:
            raise TokenizerError(6, f"page-locked allocation of {nbytes} bytes failed")
        self._block = _PinnedBlock(ptr)
        self.ptr = ptr
        raw = (ctypes.c_uint8 * max(self.nbytes, 1)).from_address(ptr)
        raw._tkz_owner = self._block  # (numpy's view keeps `raw`, which keeps the block)
        self.array = np.ctypeslib.as_array(raw)[: self.nbytes]

    def free(self):
        self.array = None
        self._block = None
        self.ptr = None


def profile_read(tok: "Tokenizer", reset: bool = True):
    """(ms_encode, ms_deferred, ms_scan, ms_compact, n_calls) summed over recorded calls."""
    ms = (ctypes.c_double * 4)()
    n = ctypes.c_uint64()
    rc = lib().tkz_profile_read(tok.handle, ms, ctypes.byref(n), int(reset))
    if rc:
        _err(rc)
    return ms[0], ms[1], ms[2], ms[3], int(n.value)


class DeviceBuffer:
    """Plain device allocation owned by libtkz's HIP runtime (bench plumbing)."""

    def __init__(self, nbytes: int):
        self.nbytes = int(nbytes)
        self.ptr = lib().tkz_dev_alloc(max(self.nbytes, 16))
        if not self.ptr:
            raise TokenizerError(6, f"device allocation of {nbytes} bytes failed")

    def upload(self, arr: np.ndarray):
        arr = np.ascontiguousarray(arr)
        assert arr.nbytes <= self.nbytes
        rc = lib().tkz_memcpy_htod(self.ptr, arr.ctypes.data_as(ctypes.c_void_p), arr.nbytes)
        if rc:
            _err(rc)

    def download(self, arr: np.ndarray, nbytes: Optional[int] = None):
        n = arr.nbytes if nbytes is None else nbytes
        rc = lib().tkz_memcpy_dtoh(arr.ctypes.data_as(ctypes.c_void_p), self.ptr, n)
        if rc:
            _err(rc)
        return arr

    def zero(self, nbytes: Optional[int] = None):
        rc = lib().tkz_memset_dev(self.ptr, 0, self.nbytes if nbytes is None else nbytes)
        if rc:
            _err(rc)

    def free(self):
        if self.ptr:
            lib().tkz_dev_free(self.ptr)
            self.ptr = None

    @property
    def freed(self) -> bool:
        return self.ptr is None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class DeviceBatch:
    """Device-resident batch: inputs uploaded once, outputs left in HBM
    (tkz_encode_batch_device). Used by bench.py and the GPU tests."""

    def __init__(self, tok: Tokenizer, data: np.ndarray, doc_off: np.ndarray, max_workspace: Optional[int] = None):
        """max_workspace: cap on the encode workspace in bytes; a batch whose one-pass
        workspace is larger runs in sub-batches (tkz_encode_batch_device). None: the
        one-pass size, capped to what the device has free after the outputs (less 2 GiB),
        so a shard larger than one pass fits (C4's 8M-doc shard)."""
        if data is None:  # from_device: inputs already in HBM
            return
        doc_off = np.ascontiguousarray(doc_off, dtype=np.uint64)
        n_docs = len(doc_off) - 1
        if n_docs < 0:
            raise ValueError("doc_off must hold at least one offset")
        total = int(doc_off[-1])
        if total > np.asarray(data).size:
            raise ValueError(f"doc_off[-1] = {total} is past the end of data ({np.asarray(data).size} bytes)")
        padded = ((total + 16 + 15) // 16) * 16
        buf = np.zeros(padded, dtype=np.uint8)
        buf[:total] = np.asarray(data, dtype=np.uint8)[:total]
        d_bytes = DeviceBuffer(padded)
        d_bytes.upload(buf)
        d_off = DeviceBuffer(doc_off.nbytes)
        d_off.upload(doc_off)
        self._setup(tok, d_bytes, d_off, n_docs, total, max_workspace)

    @classmethod
    def from_device(cls, tok: Tokenizer, d_bytes: DeviceBuffer, d_off: DeviceBuffer, n_docs: int, total: int,
                    max_workspace: Optional[int] = None, own_inputs: bool = False, owner=None) -> "DeviceBatch":
        """A batch over inputs already resident in HBM (e.g. tkz.synth.DeviceDocs): d_bytes
        readable up to a multiple of 16 bytes past `total`, d_off n_docs + 1 offsets. The
        inputs are borrowed (own_inputs=False: free() leaves them to their owner, which the
        batch keeps alive; run() refuses to launch once either buffer has been freed)."""
        b = cls(tok, None, None)
        b._setup(tok, d_bytes, d_off, int(n_docs), int(total), max_workspace, own_inputs)
        b._owner = owner
        return b

    def _setup(self, tok, d_bytes, d_off, n_docs, total, max_workspace, own_inputs=True):
        self.tok = tok
        self.n_docs = n_docs
        self.total = total
        self.d_bytes = d_bytes
        self.d_off = d_off
        self._own_inputs = own_inputs
        self.d_row = DeviceBuffer((self.n_docs + 1) * 8)
        cap = max(self.total, 1)
        self.d_ids = DeviceBuffer(cap * 4)
        self.d_offs = DeviceBuffer(cap * 8)
        self.ws_bytes = int(lib().tkz_device_workspace_size(tok.handle, self.total, self.n_docs))
        if max_workspace is None:
            free, tot = ctypes.c_size_t(0), ctypes.c_size_t(0)
            if lib().tkz_dev_mem_info(ctypes.byref(free), ctypes.byref(tot)) == 0 and free.value:
                avail = int(free.value) - (2 << 30)
                if self.ws_bytes > avail:
                    max_workspace = max(avail, 0)
        if max_workspace is not None:
            self.ws_bytes = max(min(self.ws_bytes, int(max_workspace)), int(lib().tkz_device_workspace_min(tok.handle)))
        self.d_ws = DeviceBuffer(self.ws_bytes)
        self.d_status = DeviceBuffer(16)
        self.d_status.zero()

    def run(self, stream: Optional[int] = None):
        """One encode pass, async on `stream` (a hipStream_t as int; None = the
        tokenizer's own stream)."""
        if self.d_bytes.freed or self.d_off.freed or self.d_ws.freed:
            raise TokenizerError(10, "DeviceBatch.run: an input or the workspace was freed")
        rc = lib().tkz_encode_batch_device(self.tok.handle, self.d_bytes.ptr, self.d_off.ptr, self.n_docs, self.total,
                                           self.d_row.ptr, self.d_ids.ptr, self.d_offs.ptr, self.d_ws.ptr,
                                           self.ws_bytes, self.d_status.ptr, stream)
        if rc:
            _err(rc)

    def sync(self):
        rc = lib().tkz_synchronize(self.tok.handle)
        if rc:
            _err(rc)

    def stats(self) -> dict:
        """tkz_device_batch_stats of the last run (pretokens, memo hits, deferred words,
        sub-batches)."""
        st = _BatchStats()
        rc = lib().tkz_device_batch_stats(self.tok.handle, self.d_ws.ptr, ctypes.byref(st))
        if rc:
            _err(rc)
        return {f: int(getattr(st, f)) for f, _ in _BatchStats._fields_}

    def status(self) -> int:
        s = np.zeros(4, dtype=np.uint32)
        self.d_status.download(s)
        return int(s[0])

    def results(self):
        """(row_ptr, ids, offsets) copied back to the host."""
        self.sync()
        st = self.status()
        if st:
            raise TokenizerError(st, "device-reported error")
        row = np.zeros(self.n_docs + 1, dtype=np.uint64)
        self.d_row.download(row)
        T = int(row[-1])
        ids = np.zeros(max(T, 1), dtype=np.uint32)
        offs = np.zeros((max(T, 1), 2), dtype=np.uint32)
        if T:
            self.d_ids.download(ids, T * 4)
            self.d_offs.download(offs, T * 8)
        return row, ids[:T], offs[:T]

    def results_prefix(self, n: int):
        """(row_ptr, ids, offsets) of the first n docs only (bounded host copy)."""
        self.sync()
        st = self.status()
        if st:
            raise TokenizerError(st, "device-reported error")
        n = min(int(n), self.n_docs)
        row = np.zeros(n + 1, dtype=np.uint64)
        self.d_row.download(row, (n + 1) * 8)
        T = int(row[-1])
        ids = np.zeros(max(T, 1), dtype=np.uint32)
        offs = np.zeros((max(T, 1), 2), dtype=np.uint32)
        if T:
            self.d_ids.download(ids, T * 4)
            self.d_offs.download(offs, T * 8)
        return row, ids[:T], offs[:T]

    def n_tokens(self) -> int:
        """Total tokens of the last run (row_ptr[n_docs]), after a sync."""
        self.sync()
        t = np.zeros(1, dtype=np.uint64)
        rc = lib().tkz_memcpy_dtoh(t.ctypes.data_as(ctypes.c_void_p), self.d_row.ptr + self.n_docs * 8, 8)
        if rc:
            _err(rc)
        return int(t[0])

    def free(self):
        bufs = [self.d_row, self.d_ids, self.d_offs, self.d_ws, self.d_status]
        if self._own_inputs:
            bufs += [self.d_bytes, self.d_off]
        for b in bufs:
            b.free()


from .fast import FastTokenizer, FastTokenizerOptions, SpanBatch, SpanEncoding, SpanToken  # noqa: E402,F401
