"""Vocabs past 16-bit ids / ranks (the reference's ids and ranks are u32,
/root/reference/src/model/bpe.zig:30-33, config.zig:219) and tables with a
new_id == first merge: the wide merge table, the wide word memo (id | start << 22 |
end << 27 tokens, every key in the 32-B table) and the memo for chain tables, each
checked bit-exactly against the oracle with the memo on and off."""
import json
import os

import numpy as np
import pytest

import tkz
from tkz import synth
from oracle import oracle as orc

pytestmark = pytest.mark.gpu

NT = min(16, os.cpu_count() or 1)


def _check(js, data, off, memo):
    tok = tkz.Tokenizer.from_json(js)
    tok.set_word_memo(memo)
    db = tkz.DeviceBatch(tok, data, off)
    db.run()
    row, ids, offs = db.results()
    st = db.stats()
    info = tok.memo_info()
    erow, eids, eoffs = orc.COracle(orc.RefTokenizer.from_json(js)).encode_batch(data, off, n_threads=NT)
    assert np.array_equal(row, erow)
    assert np.array_equal(ids, eids)
    assert np.array_equal(offs, eoffs)
    db.free()
    tok.close()
    return st, info


@pytest.mark.parametrize("memo", [True, False])
def test_c7_wide_vocab(memo):
    """C7: C1's docs under a 106,608-id BPE vocab with 106,545 merges (wide ids and ranks)."""
    js = synth.tokenizer_json(7)
    tok = tkz.Tokenizer.from_json(js)
    assert tok.info()["compact_tables"] == 0
    tok.close()
    data, off = synth.docs(7, 20_000, first_doc=777)
    st, info = _check(js, data, off, memo)
    if memo:
        assert info["entries"] > 100_000
        assert st["memo_hits"] > 0.8 * st["pretokens"], st
    else:
        assert st["memo_hits"] == 0


@pytest.mark.parametrize("shift", [70_000, 1_100_000])
@pytest.mark.parametrize("memo", [True, False])
def test_shifted_ids_wide_memo(memo, shift):
    """C1's vocab with every id moved past 2^16 (narrow records impossible): below 2^20
    the packed id | start << 20 | (end - 1) << 26 word tokens, past it wide tokens."""
    j = json.loads(synth.tokenizer_json(1))
    j["model"]["vocab"] = {k: i + shift for k, i in j["model"]["vocab"].items()}
    data, off = synth.docs(1, 5000, first_doc=42)
    st, _ = _check(json.dumps(j), data, off, memo)
    assert (st["memo_hits"] > 0) == memo


def test_chain_table_memo():
    """A merge with new_id == first: the memo is built by the same literal kernel path."""
    cfg = {"model": {"type": "BPE", "vocab": {"a": 0, "": 1, "b": 2, "ab": 3, "aa": 4, "bb": 5, "c": 6, "ca": 7},
                     "merges": ["a ", "b b", "a b", "a a", "c a"]},
           "pre_tokenizer": {"type": "Whitespace"}}
    js = json.dumps(cfg)
    rng = np.random.default_rng(5)
    docs = []
    for _ in range(400):
        words = [bytes(rng.choice([97, 98, 99], int(rng.integers(1, 14)))) for _ in range(int(rng.integers(1, 30)))]
        docs.append(b" ".join(words))
    off = np.zeros(len(docs) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(d) for d in docs])
    data = np.frombuffer(b"".join(docs) + bytes(16), dtype=np.uint8).copy()
    st, info = _check(js, data, off, True)
    assert info["entries"] > 0
    _check(js, data, off, False)


@pytest.mark.parametrize("seg,memo", [(True, True), (True, False), (False, True)])
def test_c9_wide_bytelevel(seg, memo):
    """C9: C7's 106k-id vocab under ByteLevel, one pretoken per doc: the segmented path with
    wide ids (merge rank -> new_id table, 20-bit symbols in the group metas, wide segment
    memo), on and off, with and without the segment memo."""
    js = synth.tokenizer_json(9)
    data, off = synth.docs(9, 8_000, first_doc=4_321)
    tok = tkz.Tokenizer.from_json(js)
    tok.set_long_segments(seg)
    tok.set_word_memo(memo)
    db = tkz.DeviceBatch(tok, data, off)
    db.run()
    row, ids, offs = db.results()
    st = db.stats()
    erow, eids, eoffs = orc.COracle(orc.RefTokenizer.from_json(js)).encode_batch(data, off, n_threads=NT)
    assert np.array_equal(row, erow) and np.array_equal(ids, eids) and np.array_equal(offs, eoffs)
    assert st["long_words"] == 8_000
    if seg:
        assert st["long_segmented"] > 0.99 * 8_000, st
    else:
        assert st["long_segmented"] == 0
    db.free()
    tok.close()


@pytest.mark.parametrize("shift", [70_000, 1_100_000])
def test_wide_segmented_shifted_ids(shift):
    """C6 (C1's vocab, ByteLevel) with every id moved past 2^16: the wide segmented path
    (below 2^20) or k_bpe_long (past it) -- the same results."""
    j = json.loads(synth.tokenizer_json(6))
    j["model"]["vocab"] = {k: i + shift for k, i in j["model"]["vocab"].items()}
    js = json.dumps(j)
    data, off = synth.docs(6, 3_000, first_doc=99)
    tok = tkz.Tokenizer.from_json(js)
    db = tkz.DeviceBatch(tok, data, off)
    db.run()
    row, ids, offs = db.results()
    st = db.stats()
    erow, eids, eoffs = orc.COracle(orc.RefTokenizer.from_json(js)).encode_batch(data, off, n_threads=NT)
    assert np.array_equal(row, erow) and np.array_equal(ids, eids) and np.array_equal(offs, eoffs)
    if shift + 32_000 < (1 << 20):
        assert st["long_segmented"] > 0.99 * 3_000, st
    db.free()
    tok.close()
