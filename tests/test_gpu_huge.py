"""Whole-text pretokens of 32 KB - 1 MB (verdict r5 item 1): the reference leaves the whole
normalized text as ONE pretoken under any pre_tokenizer it does not recognise
(/root/reference/src/config.zig:387-402, lib.zig:121) and its merge loop has no length cap
(bpe.zig:213-253). Round 5 segmented pretokens of <= 32,766 B only, with groups of <= 64
symbols and <= 4 join iterations; the rest ran k_bpe_long, one wave per pretoken. Here: the
segmented path takes pretokens of any length (32-bit in-pretoken offsets), groups of up to
512 symbols, up to 16 iterations -- checked against the oracle with the path on and off.
The oracle runs its heap form of the merge loop on these pretokens (tkz_oracle.cpp
bpe_tokenize_heap, equal to the literal loop on ordered tables: tests/test_oracle_heap.py)."""
import json
import random
import time

import numpy as np
import pytest

from oracle import oracle as orc
from tests.test_segments import random_bpe_json

pytestmark = pytest.mark.gpu
NT = 16


def _c1_text(n_bytes, first_doc=4242):
    from tkz import synth

    n_docs = n_bytes // 500 + 8
    data, off = synth.docs(1, n_docs, first_doc=first_doc)
    return bytes(data[: int(off[-1])])


def _run(js, docs, seg=True, memo=True, heap=4096):
    import tkz

    off = np.zeros(len(docs) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(d) for d in docs])
    data = np.frombuffer(b"".join(docs) + bytes(16), dtype=np.uint8).copy()
    tok = tkz.Tokenizer.from_json(js)
    tok.set_long_segments(seg)
    tok.set_word_memo(memo)
    db = tkz.DeviceBatch(tok, data, off)
    t0 = time.perf_counter()
    db.run()
    row, ids, offs = db.results()
    dt = time.perf_counter() - t0
    st = db.stats()
    assert st.get("seg_bound_errors", 0) == 0, st  # (-DTKZ_SEG_BOUNDS builds)
    db.free()
    tok.close()
    o = orc.COracle(orc.RefTokenizer.from_json(js))
    assert o.set_heap(heap)
    erow, eids, eoffs = o.encode_batch(data, off, n_threads=NT)
    assert np.array_equal(row, erow)
    if not np.array_equal(ids, eids):
        bad = np.nonzero(np.diff(row.astype(np.int64)) != np.diff(erow.astype(np.int64)))[0]
        raise AssertionError(f"ids differ; docs with other token counts: {bad[:5]}")
    assert np.array_equal(offs, eoffs)
    print(f"{len(docs)} docs, {int(off[-1])} B, seg={seg}: {dt * 1e3:.1f} ms, stats {st}")
    return st


def _bytelevel_c6():
    from tkz import synth

    return synth.tokenizer_json(6)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("seg", [True, False])
def test_huge_whole_text_pretokens(seg):
    """C1 text as 32 KB, 64 KB, 256 KB and 1 MB whole-doc pretokens (C6: C1's vocab under
    ByteLevel). With the path on, every one is segmented (no k_bpe_long)."""
    text = _c1_text(2_400_000)
    sizes = [32_767, 32_768, 65_536, 200_000, 262_144, 1_048_576]
    docs, p = [], 0
    for n in sizes:
        docs.append(text[p:p + n])
        p += n
    st = _run(_bytelevel_c6(), docs, seg)
    assert st["long_words"] == len(docs)
    if seg:
        assert st["long_segmented"] == len(docs) and st["long_fallback_bytes"] == 0, st
    else:
        assert st["long_fallback_bytes"] == sum(len(d) for d in docs), st


@pytest.mark.timeout(300)
def test_many_long_pretokens_memo_off():
    """120 pretokens of 4-64 KB, the segment memo off (every segment by the register BPE)."""
    text = _c1_text(4_000_000, first_doc=777)
    rng = random.Random(5)
    docs, p = [], 0
    for _ in range(120):
        n = rng.randint(4096, 65536)
        docs.append(text[p:p + n])
        p += n
    st = _run(_bytelevel_c6(), docs, True, memo=False)
    assert st["long_segmented"] == len(docs), st


@pytest.mark.timeout(300)
def test_big_groups():
    """Groups of 64-512 symbols (a run of letters with no cut: the wave path), past 512 (the
    pretoken falls back to k_bpe_long), inside whole-text pretokens of C1 text (C6's
    ByteLevel tokenizer); and a two-letter alphabet whose merges cross nearly every cut
    (joined groups past 512 symbols: fallbacks), exact either way."""
    text = _c1_text(200_000, first_doc=99)
    rng = random.Random(9)
    letters = "etaoinshrdlcumwfgypbvkjxqz"
    sizes = (65, 100, 200, 300, 400, 480, 513, 700, 1500)
    docs, p = [], 0
    for n in sizes:
        run = "".join(rng.choice(letters) for _ in range(n)).encode()
        docs.append(text[p:p + 300] + b" " + run + b" " + text[p + 300:p + 700])
        p += 700
    st = _run(_bytelevel_c6(), docs, True)
    assert st["long_segmented"] >= sum(n <= 480 for n in sizes), st
    assert st["long_segmented"] <= sum(n <= 512 for n in sizes), st
    _run(_bytelevel_c6(), docs, False)
    js = random_bpe_json(3, alphabet="ab", n_merges=14, extra=("é",), pretok={"type": "ByteLevel"})
    ab = [("".join(rng.choice("ab") for _ in range(n)) + " ").encode() * 4 for n in (20, 65, 130, 300, 600)]
    ab.append(("é".encode() * 200 + b" " + b"ab" * 75 + b" ") * 5)
    _run(js, ab, True)
