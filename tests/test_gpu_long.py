"""Long pretokens (verdict r2 item 4): BPE words of more than 64 bytes run the
wave-cooperative k_bpe_long (one wavefront per word; LDS-resident up to 512 bytes,
word-bound scratch beyond). Such words are what a tokenizer.json with a pre_tokenizer the
reference does not recognise produces: the whole normalized text is one pretoken
(/root/reference/src/config.zig:387-402, /root/reference/src/lib.zig:121), merged by the
O(rounds x n) loop of /root/reference/src/model/bpe.zig:213-253. Every case is compared
bit-exactly (ids, offsets, row_ptr) with the C++ oracle."""
import json
import os
import time

import numpy as np
import pytest

import tkz
from tkz import synth
from oracle import oracle as orc

pytestmark = pytest.mark.gpu

NT = min(16, os.cpu_count() or 1)


def _json(cfg, pretok, **model):
    j = json.loads(synth.tokenizer_json(cfg))
    j["pre_tokenizer"] = pretok
    j["model"].update(model)
    return json.dumps(j)


def _check(js, data, off, memo=True, dedup=-1):
    tok = tkz.Tokenizer.from_json(js)
    tok.set_word_memo(memo)
    tok.set_dedup(dedup)
    row, ids, offs = tok.encode_batch(data, off)
    erow, eids, eoffs = orc.COracle(orc.RefTokenizer.from_json(js)).encode_batch(data, off, n_threads=NT)
    assert np.array_equal(row, erow)
    bad = np.nonzero(np.diff(row.astype(np.int64)) != np.diff(erow.astype(np.int64)))[0]
    assert np.array_equal(ids, eids), f"first differing doc: {bad[:3]}"
    assert np.array_equal(offs, eoffs)
    tok.close()
    return row


def _batch(docs):
    off = np.zeros(len(docs) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(d) for d in docs])
    data = np.frombuffer(b"".join(docs) + bytes(16), dtype=np.uint8).copy()
    return data, off


@pytest.mark.parametrize("pretok", [{"type": "ByteLevel", "add_prefix_space": False}, None, {"type": "Metaspace"}])
def test_whole_doc_is_one_pretoken_c1(pretok):
    """C1's docs and vocab, every doc one pretoken (C6 of the bench under ByteLevel)."""
    data, off = synth.docs(1, 4000, first_doc=12_345)
    _check(_json(1, pretok), data, off)


def test_c6_bench_config_subset():
    data, off = synth.docs(6, 5000, first_doc=999_000)
    _check(synth.tokenizer_json(6), data, off)


def test_whole_doc_mixed_utf8():
    """C2's mixed-UTF-8 docs (well-formed: the parallel slicing) under ByteLevel + Lowercase."""
    data, off = synth.docs(2, 3000, first_doc=5)
    _check(_json(2, {"type": "ByteLevel"}), data, off)


def test_zipf_docs_whole_doc():
    """C4's Zipf(64-4096 B) docs as single pretokens: LDS words up to 512 B, scratch beyond."""
    data, off = synth.docs(4, 1500, first_doc=31)
    _check(_json(4, None), data, off)


def _c1_letters(n):
    d, o = synth.docs(1, max(4, n // 300 + 4))
    w = bytes(d[: int(o[-1])]).replace(b" ", b"").replace(b"\n", b"").replace(b"\t", b"")
    assert len(w) >= n
    return w[:n]


@pytest.mark.parametrize("memo,dedup", [(True, -1), (False, 0), (True, 1)])
def test_word_lengths_around_the_thresholds(memo, dedup):
    """Whitespace-pretokenized words of 60..70, ~512 and a few KiB bytes: the register
    path below 64 B, k_bpe_long's LDS path to 512 B and its scratch path above."""
    src = _c1_letters(20_000)
    lens = list(range(56, 72)) + [127, 128, 255, 256, 500, 511, 512, 513, 600, 1023, 1024, 1025, 2048, 4097]
    docs, p = [], 0
    for i, L in enumerate(lens):
        w = src[p:p + L]
        p = (p + L) % 10_000
        docs.append(w if i % 3 else b"ab " + w + b" cd")
    docs.append(b" ".join(src[k * 70:(k + 1) * 70] for k in range(40)))  # many long words in one doc
    data, off = _batch(docs)
    _check(synth.tokenizer_json(1), data, off, memo=memo, dedup=dedup)


def test_invalid_and_truncated_utf8_long_words():
    """Ill-formed UTF-8 in long words: the sequential slicing (reference: unreachable /
    out of bounds; here 1-byte slices for invalid leads, clamped at the word end)."""
    rng = np.random.default_rng(7)
    good = "naïve café ωμέγα 中文字符 😀 ".encode() * 12
    docs = [
        good.replace(b" ", b""),
        b"\x80" + good.replace(b" ", b""),                      # starts with a continuation byte
        good.replace(b" ", b"")[:-1],                           # truncated final sequence
        good.replace(b" ", b"") + b"\xf0\x9f",                  # truncated 4-byte sequence
        b"abc\xff\xfe" * 30,                                    # invalid lead bytes
        bytes(rng.integers(1, 256, 700, dtype=np.uint8)),       # random bytes
        bytes(rng.integers(0x80, 0xC0, 90, dtype=np.uint8)),    # continuation bytes only
        b"\xc3" + b"\xa9" * 80,
        b"abc\xa9def" * 20,                                     # stray continuation bytes after ASCII
        b"xyz" * 30 + b"\xe4\xb8\xad\x80qq",                   # ... and after a complete sequence
    ]
    data, off = _batch(docs)
    for cfg, norm in ((2, {"type": "Lowercase"}), (1, None)):
        j = json.loads(_json(cfg, None))
        j["normalizer"] = norm
        _check(json.dumps(j), data, off)


def test_unknown_chars_dropped_and_unk():
    """Chars without an id are dropped (offsets keep the gap) or become the unk token."""
    w = ("héllo wörld ☃ " * 20).encode()
    data, off = _batch([w, w.replace(b" ", b""), b"\xe2\x98\x83" * 40])
    _check(_json(1, None), data, off)
    j = json.loads(_json(1, None))
    j["model"]["vocab"]["<unk>"] = len(j["model"]["vocab"])
    j["model"]["unk_token"] = "<unk>"
    _check(json.dumps(j), data, off)


def test_new_id_equals_first_long():
    """A merge with new_id == first ("a" + "" -> "a"): each merge absorbs the b's that follow
    (the reference's re-test at the same position), on long words."""
    cfg = {"model": {"type": "BPE", "vocab": {"a": 0, "": 1, "b": 2, "ab": 3, "aa": 4, "bb": 5},
                     "merges": ["a ", "b b", "a b", "a a"]}}
    js = json.dumps(cfg)
    rng = np.random.default_rng(3)
    docs = [bytes(rng.choice([97, 98], L)) for L in (65, 100, 513, 700, 3000)] + [b"ab" * 300, b"a" * 600, b"b" * 90]
    data, off = _batch(docs)
    _check(js, data, off)
    cfg2 = {"model": {"type": "BPE", "vocab": {"a": 0, "b": 1, "ab": 0}, "merges": ["a b"]}}  # "ab" -> id of "a"
    _check(json.dumps(cfg2), data, off)


def test_identical_pair_runs_long():
    """(a, a) merges: greedy left to right inside each run (bpe.zig:240-252)."""
    cfg = {"model": {"type": "BPE", "vocab": {"l": 0, "ll": 1, "llll": 2, "o": 3, "lo": 4},
                     "merges": ["l l", "ll ll", "l o"]}}
    docs = [b"l" * L for L in (65, 66, 67, 127, 513, 1031)] + [b"lo" * 40 + b"l" * 77, (b"l" * 7 + b"o") * 20]
    data, off = _batch(docs)
    _check(json.dumps(cfg), data, off)


def test_wide_tables_long():
    """Ids above 2^16 (wide merge table: new ids by a second probe per round)."""
    j = json.loads(_json(1, None))
    v = j["model"]["vocab"]
    j["model"]["vocab"] = {k: i + 70_000 for k, i in v.items()}
    data, off = synth.docs(1, 600, first_doc=3)
    tok = tkz.Tokenizer.from_json(json.dumps(j))
    assert tok.info()["compact_tables"] == 0
    tok.close()
    _check(json.dumps(j), data, off)


@pytest.mark.timeout(300)
def test_64kib_single_word():
    """A 64-KiB pretoken (verdict r2 item 4): scratch-resident, bounded time."""
    w = _c1_letters(65_536)
    data, off = _batch([w, w[:20_000], b"tail"])
    tok = tkz.Tokenizer.from_json(_json(1, None))
    t0 = time.perf_counter()
    row, ids, offs = tok.encode_batch(data, off)
    dt = time.perf_counter() - t0
    assert dt < 20.0, f"64-KiB word took {dt:.1f} s"
    erow, eids, eoffs = orc.COracle(orc.RefTokenizer.from_json(_json(1, None))).encode_batch(data, off, n_threads=NT)
    assert np.array_equal(row, erow) and np.array_equal(ids, eids) and np.array_equal(offs, eoffs)
    print(f"64-KiB word: {int(row[1])} tokens in {dt * 1e3:.1f} ms (GPU, incl. copies)")


def test_long_word_stats():
    data, off = synth.docs(6, 2000)
    tok = tkz.Tokenizer.from_json(synth.tokenizer_json(6))
    db = tkz.DeviceBatch(tok, data, off)
    db.run()
    st = db.stats()
    assert st["long_words"] == 2000 and st["pretokens"] == 2000
    db.free()
    tok.close()


@pytest.mark.parametrize("dedup", [0, 1])
def test_deferred_stats(dedup):
    """tkz_batch_stats: deferred_model counts the words k_bpe_deferred ran on -- every
    deferred word with dedup off, the distinct ones with it on (advice r2)."""
    data, off = synth.docs(5, 20000)
    tok = tkz.Tokenizer.from_json(synth.tokenizer_json(5))
    tok.set_dedup(dedup)
    db = tkz.DeviceBatch(tok, data, off)
    db.run()
    st = db.stats()
    assert st["deferred"] > 0
    if dedup:
        assert 0 < st["deferred_model"] < st["deferred"]
    else:
        assert st["deferred_model"] == st["deferred"]
    db.free()
    tok.close()
