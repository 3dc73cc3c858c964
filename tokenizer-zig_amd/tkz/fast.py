"""Python mirror of jrc2139/tokenizer-zig's zero-allocation API: ``FastTokenizer``
(src/lib.zig:236-454), ``SpanEncoding`` (src/encoding.zig:16-224) and ``SpanToken``
(src/token.zig:11-70), over the C ABI (``tkz_fast_encode_batch``).

Encode runs on the GPU through the same kernels as ``Tokenizer.encode``; the two
FastTokenizer caps (``max_sequence_length / 4`` pretokens per doc, ``max_tokens`` tokens)
are applied on the device (csrc/span.hip). Intentional differences from the reference:

* token ids are those of the exact slow path ``Tokenizer.encode``; the reference's
  ``BPE.tokenizeFast`` pops merges from a heap and can give other ids (bpe.zig:285-430),
  and its per-pretoken symbol cap (``max_sequence_length`` codepoints) is not applied;
* WordPiece: when ``max_tokens`` falls inside a word that is later found to be unknown,
  the reference keeps the pieces matched so far; here the word is its ``[UNK]``.
* ``SpanEncoding.input`` is the text given to ``encode``; the reference points it at the
  normalized copy, which ``encode`` frees before returning (lib.zig:357-362).

Offsets are pretoken-relative, as the reference's fast paths write them.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np

from . import Encoding, Tokenizer, _err, _Offset, lib


class _FastOptions(ctypes.Structure):
    _fields_ = [("max_sequence_length", ctypes.c_uint32), ("max_tokens", ctypes.c_uint32)]


class _SpanBatch(ctypes.Structure):
    _fields_ = [
        ("n_docs", ctypes.c_size_t),
        ("capacity", ctypes.c_uint32),
        ("len", ctypes.POINTER(ctypes.c_uint32)),
        ("ids", ctypes.POINTER(ctypes.c_uint32)),
        ("offsets", ctypes.POINTER(_Offset)),
        ("attention_mask", ctypes.POINTER(ctypes.c_uint32)),
    ]


_bound = False


def _lib():
    global _bound
    L = lib()
    if not _bound:
        c = ctypes
        vp, u64, sz = c.c_void_p, c.c_uint64, c.c_size_t
        sig = {
            "tkz_fast_encode_batch": (c.c_int, [vp, vp, c.POINTER(u64), sz, c.POINTER(_FastOptions),
                                                c.POINTER(_SpanBatch)]),
            "tkz_span_batch_free": (None, [c.POINTER(_SpanBatch)]),
            "tkz_fast_workspace_size": (sz, [vp, u64, sz]),
            "tkz_fast_encode_batch_device": (c.c_int, [vp, vp, vp, sz, u64, u64, c.POINTER(_FastOptions), vp, vp,
                                                       vp, vp, vp, sz, vp, vp]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _bound = True
    return L


@dataclass
class FastTokenizerOptions:
    """FastTokenizerOptions (lib.zig:237-242)."""

    max_sequence_length: int = 8192
    max_tokens: int = 512

    def _c(self) -> _FastOptions:
        if not (0 <= self.max_sequence_length < 2**32 and 0 <= self.max_tokens < 2**32):
            raise ValueError("options must fit u32")
        return _FastOptions(self.max_sequence_length, self.max_tokens)


@dataclass
class SpanToken:
    """SpanToken (token.zig:20-70): id + byte span, type id and flags."""

    id: int
    start: int
    end: int
    type_id: int = 0
    is_special: bool = False
    is_continuation: bool = False
    is_padding: bool = False

    @classmethod
    def init(cls, tid: int, start: int, end: int) -> "SpanToken":
        return cls(tid, start, end)

    @classmethod
    def init_special(cls, tid: int, start: int, end: int) -> "SpanToken":
        return cls(tid, start, end, is_special=True)

    @classmethod
    def init_padding(cls, pad_id: int) -> "SpanToken":
        return cls(pad_id, 0, 0, is_padding=True)

    def len(self) -> int:
        return self.end - self.start

    def slice(self, input_: bytes) -> bytes:
        return input_[self.start:self.end]


_F_SPECIAL, _F_CONT, _F_PAD = 1, 2, 4  # SpanTokenFlags bit order (token.zig:11-16)


class SpanEncoding:
    """SpanEncoding (encoding.zig:16-224): fixed-capacity SoA arrays reused across encodes."""

    def __init__(self, capacity: int):
        self.capacity = int(capacity)
        self.input = b""
        self.len = 0
        self.ids = np.zeros(self.capacity, dtype=np.uint32)
        self.attention_mask = np.zeros(self.capacity, dtype=np.uint32)
        self.type_ids = np.zeros(self.capacity, dtype=np.uint32)
        self.offsets = np.zeros((self.capacity, 2), dtype=np.uint32)
        self.flags = np.zeros(self.capacity, dtype=np.uint8)

    def reset(self, new_input: bytes) -> None:
        self.input = new_input
        self.len = 0

    def append(self, tok: SpanToken) -> None:
        assert self.len < self.capacity
        i = self.len
        self.ids[i] = tok.id
        self.attention_mask[i] = 0 if tok.is_padding else 1
        self.type_ids[i] = tok.type_id
        self.offsets[i] = (tok.start, tok.end)
        self.flags[i] = (_F_SPECIAL if tok.is_special else 0) | (_F_CONT if tok.is_continuation else 0) | \
                        (_F_PAD if tok.is_padding else 0)
        self.len = i + 1

    def try_append(self, tok: SpanToken) -> bool:
        if self.len >= self.capacity:
            return False
        self.append(tok)
        return True

    def _fill(self, input_: bytes, ids, offsets) -> None:
        """Loads a device result row (the tokens FastTokenizer.encode appended)."""
        n = len(ids)
        self.reset(input_)
        self.ids[:n] = ids
        self.offsets[:n] = offsets
        self.attention_mask[:n] = 1
        self.type_ids[:n] = 0
        self.flags[:n] = 0
        self.len = n

    def token(self, i: int) -> SpanToken:
        f = int(self.flags[i])
        return SpanToken(int(self.ids[i]), int(self.offsets[i, 0]), int(self.offsets[i, 1]), int(self.type_ids[i]),
                         bool(f & _F_SPECIAL), bool(f & _F_CONT), bool(f & _F_PAD))

    def get_token_str(self, index: int) -> bytes:
        f = int(self.flags[index])
        if f & (_F_PAD | _F_SPECIAL):
            return b""
        return self.input[int(self.offsets[index, 0]):int(self.offsets[index, 1])]

    def length(self) -> int:
        return self.len

    def __len__(self) -> int:
        return self.len

    def is_empty(self) -> bool:
        return self.len == 0

    def get_ids(self) -> np.ndarray:
        return self.ids[:self.len]

    def get_attention_mask(self) -> np.ndarray:
        return self.attention_mask[:self.len]

    def get_type_ids(self) -> np.ndarray:
        return self.type_ids[:self.len]

    def get_offsets(self) -> np.ndarray:
        return self.offsets[:self.len]

    def get_tokens(self) -> List[SpanToken]:
        return [self.token(i) for i in range(self.len)]

    def truncate(self, max_length: int) -> None:
        if self.len > max_length:
            self.len = max_length

    def pad(self, target_length: int, pad_id: int) -> None:
        while self.len < target_length and self.len < self.capacity:
            self.append(SpanToken.init_padding(pad_id))

    def to_encoding(self) -> Encoding:
        """SpanEncoding.toEncoding (encoding.zig:165-223)."""
        n = self.len
        toks = []
        for i in range(n):
            if self.flags[i] & _F_PAD:
                toks.append(b"[PAD]")
            else:
                toks.append(self.input[int(self.offsets[i, 0]):int(self.offsets[i, 1])])
        return Encoding(ids=[int(x) for x in self.ids[:n]], type_ids=[int(x) for x in self.type_ids[:n]],
                        tokens=toks, offsets=[(int(a), int(b)) for a, b in self.offsets[:n]],
                        special_token_mask=[1 if self.flags[i] & _F_SPECIAL else 0 for i in range(n)],
                        attention_mask=[int(x) for x in self.attention_mask[:n]])


class SpanBatch:
    """A batch of SpanEncodings as dense rows (``tkz_span_batch``): doc d's tokens are
    ``ids[d, :len[d]]``; entries past ``len[d]`` are 0 and ``attention_mask`` is 0 there —
    the [n_docs, max_tokens] tensors a model consumes."""

    def __init__(self, len_, ids, offsets, attention_mask, data, doc_off):
        self.len = len_
        self.ids = ids
        self.offsets = offsets
        self.attention_mask = attention_mask
        self._data = data
        self._doc_off = doc_off

    @property
    def n_docs(self) -> int:
        return len(self.len)

    def encoding(self, d: int) -> SpanEncoding:
        enc = SpanEncoding(self.ids.shape[1])
        n = int(self.len[d])
        text = bytes(self._data[int(self._doc_off[d]):int(self._doc_off[d + 1])])
        enc._fill(text, self.ids[d, :n], self.offsets[d, :n])
        return enc


class FastTokenizer:
    """FastTokenizer (lib.zig:248-454): a base Tokenizer plus a preallocated SpanEncoding;
    ``encode`` returns that encoding, valid until the next call."""

    def __init__(self, base: Tokenizer, opts: Optional[FastTokenizerOptions] = None):
        self.base = base
        self.opts = opts or FastTokenizerOptions()
        self._copts = self.opts._c()
        self.model_type = "bpe" if base.info()["model"] == 1 else "wordpiece"  # lib.zig:290-295
        self._enc = SpanEncoding(self.opts.max_tokens)
        self._lib = _lib()

    @classmethod
    def from_json(cls, text, opts: Optional[FastTokenizerOptions] = None) -> "FastTokenizer":
        return cls(Tokenizer.from_json(text), opts)

    @classmethod
    def from_file(cls, path: str, opts: Optional[FastTokenizerOptions] = None) -> "FastTokenizer":
        return cls(Tokenizer.from_file(path), opts)

    def close(self) -> None:
        self.base.close()

    def encode_batch(self, data, doc_off) -> SpanBatch:
        """FastTokenizer.encode of every doc ``data[doc_off[d]:doc_off[d+1]]`` in one GPU call."""
        data = np.ascontiguousarray(np.frombuffer(data, dtype=np.uint8) if isinstance(data, (bytes, bytearray))
                                    else data, dtype=np.uint8)
        doc_off = np.ascontiguousarray(doc_off, dtype=np.uint64)
        n = len(doc_off) - 1
        out = _SpanBatch()
        rc = self._lib.tkz_fast_encode_batch(self.base.handle, data.ctypes.data if data.size else None,
                                             doc_off.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), n,
                                             ctypes.byref(self._copts), ctypes.byref(out))
        if rc:
            _err(rc)
        try:
            cap = int(out.capacity)
            cells = n * cap

            def u32(p, count):
                if count == 0:
                    return np.zeros(0, dtype=np.uint32)
                p = ctypes.cast(p, ctypes.POINTER(ctypes.c_uint32))
                return np.ctypeslib.as_array(p, (count,)).copy()

            lens = u32(out.len, n)
            ids = u32(out.ids, cells).reshape(n, cap)
            attn = u32(out.attention_mask, cells).reshape(n, cap)
            offs = u32(out.offsets, 2 * cells).reshape(n, cap, 2)
        finally:
            self._lib.tkz_span_batch_free(ctypes.byref(out))
        return SpanBatch(lens, ids, offs, attn, data, doc_off)

    def encode(self, text) -> SpanEncoding:
        """FastTokenizer.encode (lib.zig:352-413)."""
        data = text.encode("utf-8") if isinstance(text, str) else bytes(text)
        b = self.encode_batch(np.frombuffer(data, dtype=np.uint8), np.array([0, len(data)], dtype=np.uint64))
        n = int(b.len[0])
        self._enc._fill(data, b.ids[0, :n], b.offsets[0, :n])
        return self._enc

    def encode_owned(self, text, add_special_tokens: bool = False) -> Encoding:
        """FastTokenizer.encodeOwned (lib.zig:417-419): the base Tokenizer.encode."""
        return self.base.encode(text, add_special_tokens)

    def decode(self, ids: Sequence[int], skip_special_tokens: bool = False) -> bytes:
        return self.base.decode(ids, skip_special_tokens)

    def get_vocab_size(self) -> int:
        return self.base.get_vocab_size()

    def token_to_id(self, token) -> Optional[int]:
        return self.base.token_to_id(token)

    def id_to_token(self, tid: int) -> Optional[bytes]:
        return self.base.id_to_token(tid)

    def arena_memory_usage(self) -> int:
        """Host bytes held by the reusable SpanEncoding (arena.zig:237-244 counts its arena)."""
        e = self._enc
        return int(e.ids.nbytes + e.attention_mask.nbytes + e.type_ids.nbytes + e.offsets.nbytes + e.flags.nbytes)
