"""FastTokenizer / SpanEncoding / SpanToken host API (CPU): the reference's own tests of
these types (src/encoding.zig:872-1040, src/token.zig:141-200, src/lib.zig:957-1150 via
the oracle's FastTokenizer.encode restatement), the caps, and that encode fails loudly
without a GPU."""
import json

import numpy as np
import pytest

import tkz
from oracle import oracle as orc
from tkz import SpanEncoding, SpanToken


# ---- SpanEncoding (encoding.zig:872-1040) ----------------------------------------
def test_span_encoding_init():
    enc = SpanEncoding(512)
    assert enc.len == 0 and enc.capacity == 512 and enc.is_empty()


def test_span_encoding_append_get_ids():
    enc = SpanEncoding(512)
    enc.reset(b"hello world")
    enc.append(SpanToken.init(100, 0, 5))
    enc.append(SpanToken.init(200, 6, 11))
    assert enc.len == 2 and not enc.is_empty()
    assert enc.get_ids().tolist() == [100, 200]


def test_span_encoding_token_str():
    enc = SpanEncoding(512)
    enc.reset(b"hello world")
    enc.append(SpanToken.init(1, 0, 5))
    enc.append(SpanToken.init(2, 6, 11))
    assert enc.get_token_str(0) == b"hello" and enc.get_token_str(1) == b"world"
    enc.append(SpanToken.init_padding(0))
    enc.append(SpanToken.init_special(7, 0, 5))
    assert enc.get_token_str(2) == b"" and enc.get_token_str(3) == b""


def test_span_encoding_reset_reuses():
    enc = SpanEncoding(512)
    enc.reset(b"hello")
    enc.append(SpanToken.init(1, 0, 5))
    assert enc.len == 1
    enc.reset(b"world")
    assert enc.len == 0
    enc.append(SpanToken.init(2, 0, 5))
    assert enc.len == 1 and enc.get_ids().tolist() == [2]


def test_span_encoding_attention_mask():
    enc = SpanEncoding(512)
    enc.reset(b"test")
    enc.append(SpanToken.init(1, 0, 4))
    enc.append(SpanToken.init_padding(0))
    assert enc.get_attention_mask().tolist() == [1, 0]


def test_span_encoding_truncate():
    enc = SpanEncoding(512)
    enc.reset(b"abc")
    for i in range(3):
        enc.append(SpanToken.init(i + 1, i, i + 1))
    enc.truncate(2)
    assert enc.len == 2 and len(enc.get_ids()) == 2
    enc.truncate(5)
    assert enc.len == 2


def test_span_encoding_pad():
    enc = SpanEncoding(512)
    enc.reset(b"ab")
    enc.append(SpanToken.init(1, 0, 1))
    enc.append(SpanToken.init(2, 1, 2))
    enc.pad(5, 0)
    assert enc.len == 5
    assert enc.get_ids().tolist() == [1, 2, 0, 0, 0]
    assert enc.get_attention_mask().tolist() == [1, 1, 0, 0, 0]
    small = SpanEncoding(3)
    small.pad(10, 9)  # never past capacity (encoding.zig:155-159)
    assert small.len == 3 and small.get_ids().tolist() == [9, 9, 9]


def test_span_encoding_to_encoding():
    enc = SpanEncoding(512)
    enc.reset(b"hello world")
    enc.append(SpanToken.init(100, 0, 5))
    enc.append(SpanToken.init(200, 6, 11))
    enc.append(SpanToken.init_padding(0))
    e = enc.to_encoding()
    assert e.ids == [100, 200, 0]
    assert e.tokens == [b"hello", b"world", b"[PAD]"]
    assert e.attention_mask == [1, 1, 0]
    assert e.special_token_mask == [0, 0, 0]  # is_special only, not is_padding (encoding.zig:206-210)
    assert e.offsets == [(0, 5), (6, 11), (0, 0)]
    assert len(SpanEncoding(4).to_encoding()) == 0


def test_span_encoding_try_append_bounds():
    enc = SpanEncoding(2)
    enc.reset(b"abc")
    assert enc.try_append(SpanToken.init(1, 0, 1))
    assert enc.try_append(SpanToken.init(2, 1, 2))
    assert not enc.try_append(SpanToken.init(3, 2, 3))
    assert enc.len == 2


# ---- SpanToken (token.zig:141-200) -------------------------------------------------
def test_span_token():
    t = SpanToken.init(42, 10, 15)
    assert (t.id, t.start, t.end, t.type_id) == (42, 10, 15, 0)
    assert not (t.is_special or t.is_padding or t.is_continuation)
    assert t.slice(b"0123456789hello world") == b"hello" and t.len() == 5
    s = SpanToken.init_special(101, 0, 0)
    assert s.is_special and not s.is_padding
    p = SpanToken.init_padding(0)
    assert p.is_padding and (p.start, p.end) == (0, 0)
    f = SpanToken(5, 0, 3, is_continuation=True)
    enc = SpanEncoding(1)
    enc.append(f)
    assert enc.token(0) == f


# ---- FastTokenizer.encode restatement (lib.zig:957-1150) ----------------------------
def _ref(cfg):
    return orc.RefTokenizer.from_json(json.dumps(cfg))


def test_oracle_fast_reference_cases():
    bpe = {"model": {"type": "BPE", "vocab": {"h": 0, "e": 1, "l": 2, "o": 3, "he": 4, "ll": 5, "lo": 6},
                     "merges": ["h e", "l l", "l o"]}}
    assert len(_ref(bpe).fast_encode(b"hello")) >= 1  # lib.zig:957-991
    wp = {"model": {"type": "WordPiece", "vocab": {"[UNK]": 0, "hello": 1, "world": 2, "test": 3}}}
    r = _ref(wp)
    assert [t[0] for t in r.fast_encode(b"hello")] == [1]  # lib.zig:993-1017
    assert [t[0] for t in r.fast_encode(b"world")] == [2]  # lib.zig:1045-1079
    assert [t[0] for t in r.fast_encode(b"test")] == [3]
    ws = dict(wp, pre_tokenizer={"type": "Whitespace"})
    assert [t[0] for t in _ref(ws).fast_encode(b"hello world")] == [1, 2]  # lib.zig:1081-1110
    sub = {"model": {"type": "WordPiece", "vocab": {"[UNK]": 0, "play": 1, "##ing": 2, "##ed": 3, "un": 4,
                                                     "##known": 5},
                     "unk_token": "[UNK]", "continuing_subword_prefix": "##"}}
    assert _ref(sub).fast_encode(b"playing") == [(1, 0, 4), (2, 4, 7)]  # lib.zig:1112-1148
    unk = {"model": {"type": "WordPiece", "vocab": {"[UNK]": 0, "hello": 1}, "unk_token": "[UNK]"}}
    assert [t[0] for t in _ref(unk).fast_encode(b"xyz")] == [0]  # lib.zig:1150-1171


def test_oracle_fast_caps():
    cfg = {"model": {"type": "WordPiece", "vocab": {"[UNK]": 0, "a": 1, "b": 2, "##b": 3, "!": 4}},
           "pre_tokenizer": {"type": "BertPreTokenizer"}}
    r = _ref(cfg)
    text = b"a b! abb a"
    full = r.encode(text)
    assert r.fast_encode(text) == full
    assert r.fast_encode(text, max_tokens=3) == full[:3]
    # 8 // 4 = 2 pretokens: "a", "b"
    assert r.fast_encode(text, max_sequence_length=8) == [(1, 0, 1), (2, 0, 1)]
    assert r.fast_encode(text, max_sequence_length=3) == []
    assert r.fast_encode(text, max_tokens=0) == []
    whole = {"model": cfg["model"]}  # no pretokenizer: one pretoken, dropped only when the cap is 0
    assert _ref(whole).fast_encode(b"abb", max_sequence_length=4) == [(1, 0, 1), (3, 1, 2), (3, 2, 3)]
    assert _ref(whole).fast_encode(b"abb", max_sequence_length=3) == []
    no_unk = {"model": {"type": "WordPiece", "vocab": {"a": 0}}, "pre_tokenizer": {"type": "Whitespace"}}
    assert [t[0] for t in _ref(no_unk).fast_encode(b"a zz a")] == [0, 0]  # wordpiece.zig:241,297
    with pytest.raises(orc.RefError):
        _ref(no_unk).encode(b"a zz a")


def test_fast_tokenizer_host_surface():
    ft = tkz.FastTokenizer.from_json(json.dumps({"model": {"type": "WordPiece",
                                                           "vocab": {"[UNK]": 0, "hello": 1, "world": 2}}}))
    assert ft.model_type == "wordpiece"
    assert ft.get_vocab_size() == 3
    assert ft.token_to_id(b"world") == 2 and ft.id_to_token(1) == b"hello"
    assert ft.arena_memory_usage() > 0
    assert ft.opts.max_sequence_length == 8192 and ft.opts.max_tokens == 512
    bpe = tkz.FastTokenizer.from_json(json.dumps({"model": {"type": "BPE", "vocab": {"a": 0}, "merges": []}}),
                                      tkz.FastTokenizerOptions(1024, 128))
    assert bpe.model_type == "bpe" and bpe._enc.capacity == 128


def test_fast_encode_without_gpu_fails_loudly():
    if tkz.device_available():
        pytest.skip("a GPU is present")
    ft = tkz.FastTokenizer.from_json(json.dumps({"model": {"type": "WordPiece", "vocab": {"[UNK]": 0}}}))
    with pytest.raises(tkz.TokenizerError) as ei:
        ft.encode(b"hello")
    assert ei.value.name == "DeviceError"
