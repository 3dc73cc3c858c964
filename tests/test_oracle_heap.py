"""The oracle's heap form of BPE.tokenize (oracle/tkz_oracle.cpp bpe_tokenize_heap), used for
the very long whole-text pretokens of the C10 bench region (4 KB - 1 MB docs, where the
literal O(rounds * n) loop of /root/reference/src/model/bpe.zig:213-253 takes minutes per
doc): equal to the literal loop on ordered merge tables, refused on others. CPU only."""
import json
import random

import numpy as np

from oracle import oracle as orc
from tests.test_segments import COUNTER_JSON, random_bpe_json, random_docs


def _both(js, docs, threads=8):
    off = np.zeros(len(docs) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(d) for d in docs])
    data = np.frombuffer(b"".join(docs) + bytes(16), dtype=np.uint8).copy()
    ref = orc.RefTokenizer.from_json(js)
    lit = orc.COracle(ref).encode_batch(data, off, n_threads=threads)
    h = orc.COracle(ref)
    assert h.set_heap(1)
    hp = h.encode_batch(data, off, n_threads=threads)
    for a, b in zip(lit, hp):
        assert np.array_equal(a, b)
    return lit


def test_heap_equals_literal_c6_docs():
    from tkz import synth

    data, off = synth.docs(6, 4000, first_doc=99)
    docs = [bytes(data[int(off[i]):int(off[i + 1])]) for i in range(4000)]
    _both(synth.tokenizer_json(6), docs)


def test_heap_equals_literal_long_pretokens():
    """C1 text cut into 2-24 KB whole-text pretokens (C6's vocab, ByteLevel)."""
    from tkz import synth

    data, off = synth.docs(1, 3000, first_doc=12345)
    text = bytes(data[: int(off[-1])])
    rng = random.Random(3)
    docs, p = [], 0
    while p < len(text) and len(docs) < 60:
        n = rng.randint(2048, 24576)
        docs.append(text[p:p + n])
        p += n
    _both(synth.tokenizer_json(6), docs)


def test_heap_equals_literal_random_ordered_tables():
    """Tiny alphabets: runs of identical pairs, unk tokens, multi-byte chars, a ' ' in merges."""
    cases = [dict(seed=1), dict(seed=3, alphabet="ab", n_merges=14), dict(seed=4, extra=("é", "中"), n_merges=80),
             dict(seed=11, unk="[UNK]"), dict(seed=13, unk="<unk>", unk_merges=True, n_merges=90),
             dict(seed=15, alphabet="ab", extra=(" ",), n_merges=20)]
    for c in cases:
        js = random_bpe_json(**c, pretok={"type": "ByteLevel"})
        docs = random_docs(c["seed"] + 7, 200, alphabet=c.get("alphabet", "abcde") + "z",
                           extra=c.get("extra", ()) + ("ü",), lo=1, hi=3000)
        _both(js, docs, threads=4)


def test_heap_refused_for_unordered_tables():
    h = orc.COracle(orc.RefTokenizer.from_json(COUNTER_JSON))
    assert not h.set_heap(1)
    js = random_bpe_json(2, n_merges=120, pretok={"type": "ByteLevel"}, ordered=False)
    assert not orc.COracle(orc.RefTokenizer.from_json(js)).set_heap(1)
    # (then the literal loop runs: same results as without the switch)
    docs = [b"abc\x00d" * 20, b"abcd " * 30]
    lit = orc.COracle(orc.RefTokenizer.from_json(COUNTER_JSON))
    off = np.array([0, 100, 250], dtype=np.uint64)
    data = np.frombuffer(b"".join(docs) + bytes(16), dtype=np.uint8).copy()
    a = lit.encode_batch(data, off)
    h.set_heap(1)
    b = h.encode_batch(data, off)
    assert all(np.array_equal(x, y) for x, y in zip(a, b))
