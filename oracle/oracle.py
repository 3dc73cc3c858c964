"""CPU ORACLE — test infrastructure only.

This module is the parity oracle for the MI355X tokenizer. It is imported ONLY by
``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py``,
and only as the checker / the timed CPU baseline. The product path
(``tokenizer-zig_amd/``) never imports, links or executes anything under ``oracle/``.

It restates, in plain Python, the on-path semantics of jrc2139/tokenizer-zig
(snapshot mounted at /root/reference, Zig; no Zig toolchain exists in this image, so
the reference cannot be run — see DESIGN.md "Oracle"). Every function cites the
reference file:line it follows. The heavy per-document loop also exists as a C++
restatement (``oracle/tkz_oracle.cpp``) that this module drives through ctypes for
large batches; ``RefTokenizer.encode`` (pure Python) and the C++ loop are checked
against each other and against the reference's own golden vectors
(``tests/golden/reference_vectors.json``).

Pinning: the golden vectors transcribed from the reference's inline Zig tests pin
BPE/WordPiece/normalizer/pretokenizer/decoder behaviour on small vocabularies; an
HF ``tokenizers`` cross-check (ids only, ASCII only, generated in the build container
by ``tests/golden/make_hf_vectors.py``) pins larger random cases. Behaviour that no
reference test pins (VT/FF in BertPreTokenizer, invalid UTF-8) is restated from the
Zig 0.15 std definitions and marked "unpinned" in DESIGN.md.
"""
from __future__ import annotations

import ctypes
import json
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

# ---------------------------------------------------------------------------
# Errors (src/config.zig:18-30, src/model/wordpiece.zig:150,212)
# ---------------------------------------------------------------------------


class RefError(Exception):
    """Mirror of the Zig error union names."""

    def __init__(self, name: str):
        super().__init__(name)
        self.name = name


MODEL_WORDPIECE = 0
MODEL_BPE = 1
NORM_NONE = 0
NORM_LOWER = 1  # BertNormalizer and Lowercase are the same fn in config.zig:364-379
PRETOK_NONE = 0
PRETOK_WHITESPACE = 1
PRETOK_BERT = 2
DEC_NONE = 0
DEC_WORDPIECE = 1
DEC_BYTELEVEL = 2
DEC_BPE = 3

# config.zig:452-457
PUNCT = frozenset(b"!\"#$%&'()*+,-./:;<=>?@[\\]^_`{|}~")
# std.mem.tokenizeAny(u8, input, " \t\n\r")  (config.zig:444)
WS_DELIMS = frozenset(b" \t\n\r")
# std.ascii.isWhitespace (Zig 0.15: ' ', \t, \n, \r, VT 0x0B, FF 0x0C)  (config.zig:415) — VT/FF unpinned
ASCII_WS = frozenset(b" \t\n\r\x0b\x0c")


def _string_field(obj: dict, key: str) -> Optional[str]:
    """config.zig:558-565 getStringField."""
    v = obj.get(key)
    return v if isinstance(v, str) else None


def _bool_field(obj: dict, key: str) -> Optional[bool]:
    """config.zig:567-574 getBoolField."""
    v = obj.get(key)
    return v if isinstance(v, bool) else None


def _is_int(v) -> bool:
    return isinstance(v, int) and not isinstance(v, bool)


def utf8_seq_len(b: int) -> int:
    """std.unicode.utf8ByteSequenceLength (lead-byte rule used by Utf8Iterator,
    bpe.zig:186-187). Invalid lead bytes panic/UB in the reference (``catch
    unreachable``); this build defines them as 1-byte slices (unpinned)."""
    if b < 0x80:
        return 1
    if 0xC0 <= b <= 0xDF:
        return 2
    if 0xE0 <= b <= 0xEF:
        return 3
    if 0xF0 <= b <= 0xF7:
        return 4
    return 1


def codepoint_slices(seq: bytes):
    """Utf8Iterator.nextCodepointSlice over ``seq`` (bpe.zig:186-187). A truncated
    trailing sequence (out-of-bounds slice in the reference) is clamped."""
    i = 0
    n = len(seq)
    while i < n:
        ln = utf8_seq_len(seq[i])
        j = min(n, i + ln)
        yield i, j
        i = j


@dataclass
class AddedVocab:
    """src/vocab.zig:8-102 (added/special tokens)."""

    token_to_id: Dict[bytes, int] = field(default_factory=dict)
    id_to_token: Dict[int, bytes] = field(default_factory=dict)
    special: set = field(default_factory=set)
    next_id: int = 0

    def _add(self, content: bytes, tid: Optional[int], special: bool) -> bool:
        # vocab.zig:39-58 addSpecialToken / :60-81 addToken
        if content in self.token_to_id:
            return False
        i = tid if tid is not None else self.next_id
        if i >= self.next_id:
            self.next_id = i + 1
        self.token_to_id[content] = i
        self.id_to_token[i] = content
        if special:
            self.special.add(content)
        return True

    def add_special_token(self, content: bytes, tid: Optional[int] = None) -> bool:
        return self._add(content, tid, True)

    def add_token(self, content: bytes, tid: Optional[int] = None, special: bool = False) -> bool:
        return self._add(content, tid, special)

    def __len__(self) -> int:  # vocab.zig:99-101
        return len(self.token_to_id)


def _no_dup_object(pairs):
    """std.json Value objects (Zig 0.15, config.zig:60 passes default ParseOptions):
    duplicate_field_behavior = .@"error" -> error.DuplicateField -> InvalidJson."""
    d = {}
    for k, v in pairs:
        if k in d:
            raise ValueError("duplicate field")
        d[k] = v
    return d


def _no_constant(name):
    """NaN / Infinity are not JSON (std.json.Scanner: syntax error)."""
    raise ValueError(name)


class RefTokenizer:
    """Restatement of ``Tokenizer`` (src/lib.zig:32-224) built by ``loadConfig``
    (src/config.zig:59-117)."""

    def __init__(self):
        self.model_kind = MODEL_WORDPIECE
        self.vocab: Dict[bytes, int] = {}
        self.vocab_r: Dict[int, bytes] = {}
        self.merges: Dict[Tuple[int, int], Tuple[int, int]] = {}  # (a,b) -> (rank, new_id)
        self.merge_list: List[Tuple[int, int, int, int]] = []
        self.n_accepted = 0  # rank counter after the merges loop (config.zig:230,270)
        self.unk: Optional[bytes] = None
        self.prefix: bytes = b"##"
        self.max_chars = 100
        self.norm = NORM_NONE
        self.pretok = PRETOK_NONE
        self.decoder = DEC_NONE
        self.added = AddedVocab()

    # ------------------------------------------------------------------ load
    @classmethod
    def from_json(cls, text) -> "RefTokenizer":
        """Tokenizer.fromJson (lib.zig:59-85) + config.loadConfig (config.zig:59-117)."""
        try:
            if isinstance(text, (bytes, bytearray)):
                text = bytes(text).decode("utf-8")  # std.json.Scanner rejects ill-formed UTF-8
            root = json.loads(text, object_pairs_hook=_no_dup_object, parse_constant=_no_constant)
        except (ValueError, RecursionError):
            raise RefError("InvalidJson")
        if not isinstance(root, dict):
            raise RefError("InvalidJson")
        t = cls()
        t._parse_model(root)
        # config.zig:82-86 added tokens, lib.zig:66-72 installed into the added vocab
        at = root.get("added_tokens")
        if isinstance(at, list):
            for item in at:
                if not isinstance(item, dict):
                    continue
                content = _string_field(item, "content")
                if content is None:
                    continue
                tid = item.get("id")
                tid = tid if _is_int(tid) else None
                special = _bool_field(item, "special") or False
                c = content.encode("utf-8")
                if special:
                    t.added.add_special_token(c, tid)
                else:
                    t.added.add_token(c, tid, False)
        # config.zig:339-362 normalizer: only BertNormalizer/Lowercase recognised
        nv = root.get("normalizer")
        if isinstance(nv, dict):
            ty = _string_field(nv, "type")
            if ty in ("BertNormalizer", "Lowercase"):
                t.norm = NORM_LOWER
        # config.zig:381-403 pre_tokenizer
        pv = root.get("pre_tokenizer")
        if isinstance(pv, dict):
            ty = _string_field(pv, "type")
            if ty == "BertPreTokenizer":
                t.pretok = PRETOK_BERT
            elif ty in ("Whitespace", "WhitespaceSplit"):
                t.pretok = PRETOK_WHITESPACE
        # config.zig:459-486 decoder
        dv = root.get("decoder")
        if isinstance(dv, dict):
            ty = _string_field(dv, "type")
            t.decoder = {"WordPiece": DEC_WORDPIECE, "ByteLevel": DEC_BYTELEVEL, "BPE": DEC_BPE}.get(ty, DEC_NONE)
        # post_processor (config.zig:532-555) is a no-op: nothing to record.
        return t

    def _parse_vocab(self, model: dict) -> None:
        vv = model.get("vocab")
        if not isinstance(vv, dict):
            raise RefError("MissingVocab")
        # config.zig:157-169 / :210-222 — every value must be an integer (Zig @intCast to u32)
        for k, v in vv.items():
            if not _is_int(v) or v < 0 or v > 0xFFFFFFFF:
                raise RefError("InvalidVocabEntry")
            self.vocab[k.encode("utf-8")] = v
        # bpe.zig:92-97 / wordpiece.zig:58-63 reverse map (unique ids assumed)
        for k, v in self.vocab.items():
            self.vocab_r[v] = k

    def _parse_model(self, root: dict) -> None:
        """config.zig:124-139 parseModel."""
        m = root.get("model")
        if not isinstance(m, dict):
            raise RefError("MissingModel")
        ty = _string_field(m, "type") or "WordPiece"
        if ty == "WordPiece":
            # config.zig:141-192
            self.model_kind = MODEL_WORDPIECE
            self._parse_vocab(m)
            self.unk = (_string_field(m, "unk_token") or "[UNK]").encode("utf-8")
            self.prefix = (_string_field(m, "continuing_subword_prefix") or "##").encode("utf-8")
            mc = m.get("max_input_chars_per_word")
            self.max_chars = mc if _is_int(mc) and mc >= 0 else 100
        elif ty == "BPE":
            # config.zig:194-295
            self.model_kind = MODEL_BPE
            self._parse_vocab(m)
            merges = m.get("merges")
            rank = 0
            if isinstance(merges, list):
                for item in merges:
                    if isinstance(item, str):
                        # std.mem.splitScalar(u8, s, ' '): first two segments (config.zig:238-241)
                        parts = item.split(" ")
                        if len(parts) < 2:
                            continue
                        first, second = parts[0], parts[1]
                    elif isinstance(item, list) and len(item) == 2:
                        if not (isinstance(item[0], str) and isinstance(item[1], str)):
                            continue
                        first, second = item[0], item[1]
                    else:
                        continue
                    fb, sb = first.encode("utf-8"), second.encode("utf-8")
                    a = self.vocab.get(fb)
                    if a is None:
                        continue
                    b = self.vocab.get(sb)
                    if b is None:
                        continue
                    merged = fb + sb
                    if len(merged) > 512:  # merged_buf: [512]u8 (config.zig:258-260)
                        continue
                    nid = self.vocab.get(merged)
                    if nid is None:
                        continue
                    self.merges[(a, b)] = (rank, nid)  # put: a duplicate pair overwrites
                    rank += 1
            self.n_accepted = rank
            self.merge_list = [(a, b, r, n) for (a, b), (r, n) in self.merges.items()]
            u = _string_field(m, "unk_token")
            self.unk = u.encode("utf-8") if u is not None else None
        else:
            raise RefError("UnsupportedModelType")

    # --------------------------------------------------------------- pipeline
    def normalize(self, text: bytes) -> bytes:
        """config.zig:364-379: std.ascii.toLower per byte (only A-Z)."""
        if self.norm == NORM_LOWER:
            return bytes(c | 0x20 if 0x41 <= c <= 0x5A else c for c in text)
        return text

    def pre_tokenize(self, s: bytes) -> List[Tuple[int, int]]:
        """config.zig:405-450. Returns (start, end) spans into ``s``; with no
        pretokenizer the whole text is one pretoken (lib.zig:121)."""
        if self.pretok == PRETOK_WHITESPACE:
            # std.mem.tokenizeAny(" \t\n\r"): maximal non-empty runs of non-delimiters
            out = []
            i, n = 0, len(s)
            while i < n:
                while i < n and s[i] in WS_DELIMS:
                    i += 1
                j = i
                while j < n and s[j] not in WS_DELIMS:
                    j += 1
                if j > i:
                    out.append((i, j))
                i = j
            return out
        if self.pretok == PRETOK_BERT:
            out = []
            start = 0
            for i, c in enumerate(s):
                ws = c in ASCII_WS
                p = c in PUNCT
                if ws or p:
                    if i > start:
                        out.append((start, i))
                    if p:
                        out.append((i, i + 1))
                    start = i + 1
            if start < len(s):
                out.append((start, len(s)))
            return out
        return [(0, len(s))]

    def bpe_tokenize(self, seq: bytes) -> List[Tuple[int, int, int]]:
        """BPE.tokenize (bpe.zig:173-263), the slow path Tokenizer.encode uses."""
        if len(seq) == 0:
            return []
        word: List[int] = []
        offs: List[List[int]] = []
        unk_id = self.vocab.get(self.unk) if self.unk is not None else None
        for i, j in codepoint_slices(seq):  # bpe.zig:186-211
            tid = self.vocab.get(seq[i:j])
            if tid is not None:
                word.append(tid)
                offs.append([i, j])
            elif unk_id is not None:
                word.append(unk_id)
                offs.append([i, j])
            # else: skip the char
        while len(word) > 1:  # bpe.zig:214-253
            best = None
            best_rank = 0xFFFFFFFF
            for i in range(len(word) - 1):
                pv = self.merges.get((word[i], word[i + 1]))
                if pv is not None and pv[0] < best_rank:
                    best_rank = pv[0]
                    best = (word[i], word[i + 1])
            if best is None:
                break
            new_id = self.merges[best][1]
            i = 0
            while i < len(word) - 1:
                if word[i] == best[0] and word[i + 1] == best[1]:
                    word[i] = new_id
                    del word[i + 1]
                    offs[i][1] = offs[i + 1][1]
                    del offs[i + 1]
                else:
                    i += 1
        return [(w, o[0], o[1]) for w, o in zip(word, offs)]

    def wordpiece_tokenize(self, chars: bytes) -> List[Tuple[int, int, int]]:
        """WordPiece.tokenize (wordpiece.zig:141-222)."""
        n = len(chars)
        if n > self.max_chars:
            unk_id = self.vocab.get(self.unk)
            if unk_id is None:
                raise RefError("MissingUnkToken")
            return [(unk_id, 0, n)]
        toks = []
        start = 0
        bad = False
        plen = len(self.prefix)
        while start < n:
            end = n
            cur = None
            while start < end:
                if start > 0:
                    if plen + (end - start) > 512:  # substr_buf: [512]u8
                        end -= 1
                        continue
                    sub = self.prefix + chars[start:end]
                else:
                    sub = chars[start:end]
                tid = self.vocab.get(sub)
                if tid is not None:
                    cur = tid
                    break
                end -= 1
            if cur is None:
                bad = True
                break
            toks.append((cur, start, end))
            start = end
        if bad:
            unk_id = self.vocab.get(self.unk)
            if unk_id is None:
                raise RefError("MissingUnkToken")
            return [(unk_id, 0, n)]
        return toks

    def encode(self, text: bytes, add_special_tokens: bool = False) -> List[Tuple[int, int, int]]:
        """Tokenizer.encode (lib.zig:109-160). Returns [(id, start, end)] with
        pretoken-relative offsets (lib.zig:133-137). The post-processor is a
        no-op (config.zig:551-555); truncation/padding are never set by fromJson."""
        norm = self.normalize(text)
        out = []
        for s, e in self.pre_tokenize(norm):
            piece = norm[s:e]
            if self.model_kind == MODEL_BPE:
                out.extend(self.bpe_tokenize(piece))
            else:
                out.extend(self.wordpiece_tokenize(piece))
        return out

    def encode_full(self, text: bytes, truncation: Optional[int] = None, padding: Optional[dict] = None) -> dict:
        """Tokenizer.encode with Tokenizer.truncation / .padding set (lib.zig:149-157):
        Encoding.fromTokens (encoding.zig:246-294), then Encoding.truncate(max_length)
        (encoding.zig:362-380: prefix, stride ignored) and Encoding.pad(params)
        (encoding.zig:385-437: only when shorter than params.length; pad positions get
        pad_id, pad_type_id, pad_token, offset (0,0), special 1, attention 0; right or
        left). `padding` = {length, pad_id, pad_type_id, pad_token, direction}."""
        toks = self.encode(text)
        enc = {
            "ids": [t[0] for t in toks],
            "offsets": [(t[1], t[2]) for t in toks],
            "type_ids": [0] * len(toks),
            "tokens": self.token_strings(toks),
            "special_token_mask": [0] * len(toks),
            "attention_mask": [1] * len(toks),
        }
        if truncation is not None and len(enc["ids"]) > truncation:
            for k in enc:
                enc[k] = enc[k][:truncation]
        if padding and padding.get("length") and len(enc["ids"]) < padding["length"]:
            n_pad = padding["length"] - len(enc["ids"])
            pads = {
                "ids": [padding.get("pad_id", 0)] * n_pad,
                "offsets": [(0, 0)] * n_pad,
                "type_ids": [padding.get("pad_type_id", 0)] * n_pad,
                "tokens": [padding.get("pad_token", b"[PAD]")] * n_pad,
                "special_token_mask": [1] * n_pad,
                "attention_mask": [0] * n_pad,
            }
            left = padding.get("direction", "right") == "left"
            for k in enc:
                enc[k] = pads[k] + enc[k] if left else enc[k] + pads[k]
        return enc

    def fast_encode(self, text: bytes, max_sequence_length: int = 8192,
                    max_tokens: int = 512) -> List[Tuple[int, int, int]]:
        """FastTokenizer.encode (lib.zig:352-413) with the model step of Tokenizer.encode:
        normalize, pretokenize, keep the first max_sequence_length/4 pretokens
        (TokenizerArena.addPretokenSpan, arena.zig:192,224-229), tokenize each and append
        while the max_tokens-capacity SpanEncoding has room (tryAppend, encoding.zig:95-99;
        bpe.zig:339,423, wordpiece.zig:289). WordPiece with no UNK in the vocab: an unknown
        word yields nothing (wordpiece.zig:241,297). Documented substitution: BPE uses the
        slow merge loop (bpe.zig:173-263), not the heap of tokenizeFast (bpe.zig:285-430)."""
        norm = self.normalize(text)
        spans = self.pre_tokenize(norm)[: max_sequence_length // 4]
        out: List[Tuple[int, int, int]] = []
        for s, e in spans:
            piece = norm[s:e]
            if self.model_kind == MODEL_BPE:
                toks = self.bpe_tokenize(piece)
            else:
                try:
                    toks = self.wordpiece_tokenize(piece)
                except RefError:  # MissingUnkToken: tokenizeFast returns without a token
                    toks = []
            for t in toks:
                if len(out) >= max_tokens:
                    return out
                out.append(t)
        return out

    def token_strings(self, toks) -> List[bytes]:
        """Encoding.tokens: the build defines tokens[i] = idToToken(ids[i]) (see
        DESIGN.md: the reference's WordPiece '##' values point at a dead stack
        buffer, wordpiece.zig:169,188)."""
        return [self.vocab_r.get(t[0], b"") for t in toks]

    # -------------------------------------------------------------- decode &c
    def decode(self, ids: Sequence[int], skip_special_tokens: bool = False) -> bytes:
        """Tokenizer.decode (lib.zig:163-189) + config decoders (config.zig:488-530)."""
        buf = bytearray()
        for i in ids:
            if skip_special_tokens:
                tok = self.added.id_to_token.get(i)
                if tok is not None and tok in self.added.special:
                    continue
            tok = self.vocab_r.get(i)
            if tok is not None:
                buf += tok
        b = bytes(buf)
        if self.decoder == DEC_WORDPIECE:
            out = bytearray()
            i = 0
            while i < len(b):
                if i + 1 < len(b) and b[i] == 0x23 and b[i + 1] == 0x23:
                    i += 2
                else:
                    out.append(b[i])
                    i += 1
            return bytes(out)
        if self.decoder == DEC_BPE:
            return b.replace(b"\xc4\xa0", b" ")
        return b

    def get_vocab_size(self) -> int:
        """lib.zig:203-205 (model count + added count, even if overlapping)."""
        return len(self.vocab) + len(self.added)

    def token_to_id(self, tok: bytes) -> Optional[int]:
        """lib.zig:208-214."""
        if tok in self.added.token_to_id:
            return self.added.token_to_id[tok]
        return self.vocab.get(tok)

    def id_to_token(self, i: int) -> Optional[bytes]:
        """lib.zig:217-223."""
        if i in self.added.id_to_token:
            return self.added.id_to_token[i]
        return self.vocab_r.get(i)


# ---------------------------------------------------------------------------
# C++ restatement (oracle/tkz_oracle.cpp) for large batches / the CPU baseline
# ---------------------------------------------------------------------------

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TKZ_ORACLE_LIB") or os.path.join(_HERE, "build", "liboracle.so")
_libs = {}


def build_native(out_dir: str = os.path.join(_HERE, "build", "native")) -> str:
    """Compiles tkz_oracle.cpp with -O3 -march=native for the host this runs on (the
    CPU-baseline build; the prebuilt LIB_PATH targets x86-64-v2 so it runs anywhere).
    Returns the library path; raises if the compiler fails."""
    import platform
    import subprocess

    os.makedirs(out_dir, exist_ok=True)
    src = os.path.join(_HERE, "tkz_oracle.cpp")
    tag = f"{platform.node()}_{os.path.getmtime(src):.0f}".replace(os.sep, "_")
    out = os.path.join(out_dir, f"liboracle_native_{tag}.so")
    if not os.path.exists(out):
        tmp = out + f".{os.getpid()}"
        subprocess.run(["g++", "-O3", "-march=native", "-std=c++17", "-fPIC", "-pthread", "-shared", "-o", tmp, src],
                       check=True, capture_output=True)
        os.replace(tmp, out)
    return out


def load_lib(path: str = LIB_PATH):
    if path in _libs:
        return _libs[path]
    if not os.path.exists(path):
        raise RuntimeError(f"oracle library not built: {path} (run __graft_entry__.build())")
    lib = ctypes.CDLL(path)
    u32p = ctypes.POINTER(ctypes.c_uint32)
    u64p = ctypes.POINTER(ctypes.c_uint64)
    lib.orc_create.restype = ctypes.c_void_p
    lib.orc_create.argtypes = [
        ctypes.c_int, ctypes.c_int, ctypes.c_int,
        ctypes.c_char_p, u32p, u32p, ctypes.c_size_t,
        u32p, u32p, u32p, u32p, ctypes.c_size_t,
        ctypes.c_char_p, ctypes.c_int64, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint64,
    ]
    lib.orc_destroy.argtypes = [ctypes.c_void_p]
    lib.orc_set_heap.restype = ctypes.c_int
    lib.orc_set_heap.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
    lib.orc_encode_batch.restype = ctypes.c_int
    lib.orc_encode_batch.argtypes = [
        ctypes.c_void_p, ctypes.c_void_p, u64p, ctypes.c_size_t,
        u32p, u32p, u32p, ctypes.c_int, ctypes.c_int,
    ]
    _libs[path] = lib
    return lib


class COracle:
    """ctypes driver for oracle/tkz_oracle.cpp (a C++ restatement of the same
    Tokenizer.encode loop, with the reference's per-call allocation pattern)."""

    def __init__(self, ref: RefTokenizer, lib_path: str = LIB_PATH):
        import numpy as np

        self.np = np
        lib = load_lib(lib_path)
        self.ref = ref
        keys = list(ref.vocab.keys())
        blob = b"".join(keys)
        lens = np.array([len(k) for k in keys], dtype=np.uint32)
        ids = np.array([ref.vocab[k] for k in keys], dtype=np.uint32)
        ml = ref.merge_list
        ma = np.array([m[0] for m in ml], dtype=np.uint32)
        mb = np.array([m[1] for m in ml], dtype=np.uint32)
        mr = np.array([m[2] for m in ml], dtype=np.uint32)
        mn = np.array([m[3] for m in ml], dtype=np.uint32)
        self._keep = (blob, lens, ids, ma, mb, mr, mn)
        u32p = ctypes.POINTER(ctypes.c_uint32)
        p = lambda a: a.ctypes.data_as(u32p)
        unk = ref.unk
        self.h = lib.orc_create(
            ref.model_kind, ref.norm, ref.pretok,
            blob, p(lens), p(ids), len(keys),
            p(ma), p(mb), p(mr), p(mn), len(ml),
            unk if unk is not None else b"", -1 if unk is None else len(unk),
            ref.prefix, len(ref.prefix), ref.max_chars,
        )
        self.lib = lib

    def set_heap(self, min_bytes: int) -> bool:
        """BPE pretokens of >= min_bytes bytes take the heap form of the merge loop
        (tkz_oracle.cpp bpe_tokenize_heap: the literal loop's result for ordered merge tables,
        O(n log n); 0 = never). Returns False, and keeps the literal loop, when the table does
        not allow it."""
        return bool(self.lib.orc_set_heap(self.h, int(min_bytes)))

    def __del__(self):
        try:
            if getattr(self, "h", None):
                self.lib.orc_destroy(self.h)
                self.h = None
        except Exception:
            pass

    def encode_batch(self, data, doc_off, n_threads: int = 1, full_encoding: int = 1):
        """Encode docs ``data[doc_off[i]:doc_off[i+1]]``. Returns (row_ptr u64[n+1],
        ids u32[T], offsets u32[T,2]) in CSR form. ``full_encoding`` also builds
        the Encoding arrays + token string dups per doc like Encoding.fromTokens."""
        np = self.np
        data = np.ascontiguousarray(np.frombuffer(data, dtype=np.uint8) if isinstance(data, (bytes, bytearray)) else data, dtype=np.uint8)
        doc_off = np.ascontiguousarray(doc_off, dtype=np.uint64)
        n = len(doc_off) - 1
        total = int(doc_off[-1]) if n >= 0 else 0
        counts = np.zeros(max(n, 1), dtype=np.uint32)
        ids_b = np.zeros(max(total, 1), dtype=np.uint32)
        offs_b = np.zeros((max(total, 1), 2), dtype=np.uint32)
        u32p = ctypes.POINTER(ctypes.c_uint32)
        u64p = ctypes.POINTER(ctypes.c_uint64)
        rc = self.lib.orc_encode_batch(
            self.h, data.ctypes.data_as(ctypes.c_void_p), doc_off.ctypes.data_as(u64p), n,
            counts.ctypes.data_as(u32p), ids_b.ctypes.data_as(u32p), offs_b.ctypes.data_as(u32p),
            n_threads, full_encoding,
        )
        if rc == 1:
            raise RefError("MissingUnkToken")
        if rc != 0:
            raise RuntimeError(f"orc_encode_batch failed: {rc}")
        counts = counts[:n].astype(np.uint64)
        row_ptr = np.zeros(n + 1, dtype=np.uint64)
        np.cumsum(counts, out=row_ptr[1:])
        if n == 0:
            return row_ptr, np.zeros(0, np.uint32), np.zeros((0, 2), np.uint32)
        # bound layout -> CSR (tokens of doc i live at doc_off[i] .. + counts[i])
        starts = doc_off[:-1].astype(np.int64)
        c = counts.astype(np.int64)
        T = int(c.sum())
        idx = np.repeat(starts - row_ptr[:-1].astype(np.int64), c) + np.arange(T, dtype=np.int64)
        return row_ptr, ids_b[idx], offs_b[idx]
