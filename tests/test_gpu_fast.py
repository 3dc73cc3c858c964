"""FastTokenizer API on the GPU (csrc/span.hip + the encode kernels) vs the oracle's
FastTokenizer.encode restatement: the reference's FastTokenizer tests (lib.zig:957-1150),
random configs with small pretoken / token caps (clip and fill kernels), edge cases, the
device-resident entry point, and a bench config subset. Bar: bit-exact ids and offsets."""
import ctypes
import json
import random

import numpy as np
import pytest

import tkz
from tkz import synth
from tkz.fast import _FastOptions, _lib
from oracle import oracle as orc
from test_gpu_parity import _batch, _edge_docs, _rand_cfg, _rand_text

pytestmark = pytest.mark.gpu


def _check_fast(ft, ref, docs):
    data, off = _batch(docs)
    b = ft.encode_batch(np.frombuffer(data, dtype=np.uint8), off)
    msl, mt = ft.opts.max_sequence_length, ft.opts.max_tokens
    assert b.ids.shape == (len(docs), mt)
    for i, d in enumerate(docs):
        exp = ref.fast_encode(d, msl, mt)
        n = int(b.len[i])
        assert b.ids[i, :n].tolist() == [t[0] for t in exp], (i, msl, mt, d[:80])
        assert b.offsets[i, :n].tolist() == [[t[1], t[2]] for t in exp], (i, d[:80])
        assert not b.ids[i, n:].any() and not b.offsets[i, n:].any()
        assert b.attention_mask[i, :n].all() and not b.attention_mask[i, n:].any()
    return b


def test_reference_fast_tokenizer_cases():
    wp = {"model": {"type": "WordPiece", "vocab": {"[UNK]": 0, "hello": 1, "world": 2, "test": 3}}}
    ft = tkz.FastTokenizer.from_json(json.dumps(wp))
    for text, want in ((b"hello", [1]), (b"world", [2]), (b"test", [3])):  # lib.zig:1045-1079
        enc = ft.encode(text)
        assert enc.get_ids().tolist() == want and enc.len == 1
    ws = tkz.FastTokenizer.from_json(json.dumps(dict(wp, pre_tokenizer={"type": "Whitespace"})))
    enc = ws.encode(b"hello world")  # lib.zig:1081-1110
    assert enc.get_ids().tolist() == [1, 2]
    assert enc.get_token_str(0) == b"hello" and enc.get_offsets().tolist() == [[0, 5], [0, 5]]
    sub = {"model": {"type": "WordPiece", "vocab": {"[UNK]": 0, "play": 1, "##ing": 2, "##ed": 3, "un": 4,
                                                     "##known": 5}}}
    enc = tkz.FastTokenizer.from_json(json.dumps(sub)).encode(b"playing")  # lib.zig:1112-1148
    assert enc.get_ids().tolist() == [1, 2]
    assert [(t.start, t.end) for t in enc.get_tokens()] == [(0, 4), (4, 7)]
    enc = tkz.FastTokenizer.from_json(json.dumps(sub)).encode(b"xyz")  # lib.zig:1150-1171
    assert enc.get_ids().tolist() == [0]
    bpe = {"model": {"type": "BPE", "vocab": {"h": 0, "e": 1, "l": 2, "o": 3, "he": 4, "ll": 5, "lo": 6},
                     "merges": ["h e", "l l", "l o"]}}
    ft = tkz.FastTokenizer.from_json(json.dumps(bpe))  # lib.zig:957-991
    enc = ft.encode(b"hello")
    assert enc.len >= 1 and ft.model_type == "bpe"
    assert enc.get_ids().tolist() == [t[0] for t in orc.RefTokenizer.from_json(json.dumps(bpe)).encode(b"hello")]
    # the returned encoding is the reused arena one (valid until the next encode)
    assert ft.encode(b"ll") is enc and enc.get_ids().tolist() == [5]


@pytest.mark.parametrize("model", ["BPE", "WordPiece"])
@pytest.mark.parametrize("pretok", [None, "Whitespace", "BertPreTokenizer"])
def test_random_configs_caps(model, pretok):
    rng = random.Random(f"fast-{model}-{pretok}")
    for trial in range(4):
        cfg = _rand_cfg(rng, model, pretok, rng.choice([None, "Lowercase"]))
        ref = orc.RefTokenizer.from_json(json.dumps(cfg))
        lens = [0, 1, 2, 7, 40, 63, 64, 65, 200, 513, 1100, 3000] + [rng.randint(0, 300) for _ in range(40)]
        docs = [_rand_text(rng, n) for n in lens]
        for msl, mt in ((8192, 512), (40, 7), (4, 3), (257, 64), (3, 5), (2000, 1), (100, 0)):
            ft = tkz.FastTokenizer(tkz.Tokenizer.from_json(json.dumps(cfg)), tkz.FastTokenizerOptions(msl, mt))
            _check_fast(ft, ref, docs)


@pytest.mark.parametrize("pretok", ["Whitespace", "BertPreTokenizer"])
def test_pretoken_cap_boundaries(pretok):
    """The cut lands on every position of a 64-byte scan step and past several steps."""
    vocab = {c: i for i, c in enumerate("abcdefgh!,.")}
    cfg = {"model": {"type": "BPE", "vocab": vocab, "merges": []}, "pre_tokenizer": {"type": pretok}}
    ref = orc.RefTokenizer.from_json(json.dumps(cfg))
    rng = random.Random(pretok)
    docs = []
    for _ in range(60):
        n = rng.randint(60, 900)
        docs.append(bytes(rng.choice(b"abcdefgh!,.  \t\n") for _ in range(n)))
    docs += [b"a" * 1000, b"!" * 1000, b" " * 1000, b"a " * 500, b"a!" * 500]
    for msl in (4, 8, 60, 64, 256, 400, 1024):
        ft = tkz.FastTokenizer(tkz.Tokenizer.from_json(json.dumps(cfg)), tkz.FastTokenizerOptions(msl, 4096))
        _check_fast(ft, ref, docs)


def test_edge_docs_fast():
    vocab = {"[UNK]": 0, "a": 1, "##a": 2, "b": 3, "##b": 4, "ab": 5, "##ab": 6, "hello": 7, "##llo": 8, "he": 9,
             "!": 10}
    for pretok in (None, "Whitespace", "BertPreTokenizer"):
        cfg = {"model": {"type": "WordPiece", "vocab": vocab, "max_input_chars_per_word": 40}}
        if pretok:
            cfg["pre_tokenizer"] = {"type": pretok}
        ref = orc.RefTokenizer.from_json(json.dumps(cfg))
        for opts in (tkz.FastTokenizerOptions(), tkz.FastTokenizerOptions(64, 16)):
            _check_fast(tkz.FastTokenizer(tkz.Tokenizer.from_json(json.dumps(cfg)), opts), ref, _edge_docs())


def test_missing_unk_yields_no_token():
    """WordPiece.tokenizeFast with no UNK in the vocab drops the word (wordpiece.zig:241,297),
    where Tokenizer.encode fails with MissingUnkToken."""
    cfg = {"model": {"type": "WordPiece", "vocab": {"a": 0, "##a": 1}, "max_input_chars_per_word": 6},
           "pre_tokenizer": {"type": "Whitespace"}}
    ref = orc.RefTokenizer.from_json(json.dumps(cfg))
    ft = tkz.FastTokenizer.from_json(json.dumps(cfg))
    docs = [b"a zz a", b"aaaaaaaaa a", b"b", b"", b"aa " * 200 + b"q"]
    _check_fast(ft, ref, docs)
    with pytest.raises(tkz.TokenizerError):
        ft.encode_owned(b"a zz a")


def test_device_entry_point_and_hint():
    """tkz_fast_encode_batch_device with and without the max_doc_bytes hint."""
    cfg = json.loads(synth.tokenizer_json(0))
    tok = tkz.Tokenizer.from_json(json.dumps(cfg))
    data, off = synth.docs(0, 300)
    ft = tkz.FastTokenizer(tok, tkz.FastTokenizerOptions(128, 40))
    host = ft.encode_batch(data, off)
    L = _lib()
    n, total = len(off) - 1, int(off[-1])
    cap = 40
    ws_n = int(L.tkz_fast_workspace_size(tok.handle, total, n))
    bufs = {k: tkz.DeviceBuffer(s) for k, s in (("bytes", total + 32), ("off", (n + 1) * 8), ("len", n * 4),
                                                ("ids", n * cap * 4), ("offs", n * cap * 8), ("attn", n * cap * 4),
                                                ("ws", ws_n), ("st", 4))}
    bufs["bytes"].upload(data)
    bufs["off"].upload(off)
    opts = _FastOptions(128, cap)
    for hint in (0, int(np.diff(off).max()), 1 << 40):
        bufs["st"].zero()
        bufs["ids"].zero()
        rc = L.tkz_fast_encode_batch_device(tok.handle, bufs["bytes"].ptr, bufs["off"].ptr, n, total, hint,
                                            ctypes.byref(opts), bufs["len"].ptr, bufs["ids"].ptr, bufs["offs"].ptr,
                                            bufs["attn"].ptr, bufs["ws"].ptr, ws_n, bufs["st"].ptr, None)
        assert rc == 0
        L.tkz_synchronize(tok.handle)
        lens = np.zeros(n, np.uint32)
        ids = np.zeros(n * cap, np.uint32)
        bufs["len"].download(lens)
        bufs["ids"].download(ids)
        # every hint here is above the pretoken cap (32): each call clips and equals the host API
        assert np.array_equal(lens, host.len), hint
        assert np.array_equal(ids.reshape(n, cap), host.ids), hint
    for b in bufs.values():
        b.free()


@pytest.mark.parametrize("cfg_id", [1, 3])
def test_bench_config_subset_fast(cfg_id):
    """C1 / C3 docs (512 B, below the default pretoken cap) with the default options equal
    Tokenizer.encode truncated to 512 tokens; with max_sequence_length 256 (64 pretokens)
    the clip path runs on every doc."""
    js = synth.tokenizer_json(cfg_id)
    ref = orc.RefTokenizer.from_json(js)
    data, off = synth.docs(cfg_id, 2000)
    docs = [bytes(data[int(off[i]):int(off[i + 1])]) for i in range(len(off) - 1)]
    for opts in (tkz.FastTokenizerOptions(), tkz.FastTokenizerOptions(256, 128), tkz.FastTokenizerOptions(8192, 50)):
        ft = tkz.FastTokenizer(tkz.Tokenizer.from_json(js), opts)
        b = ft.encode_batch(data, off)
        for i in range(0, len(docs), 7):
            exp = ref.fast_encode(docs[i], opts.max_sequence_length, opts.max_tokens)
            n = int(b.len[i])
            assert b.ids[i, :n].tolist() == [t[0] for t in exp], i
            assert b.offsets[i, :n].tolist() == [[t[1], t[2]] for t in exp], i
