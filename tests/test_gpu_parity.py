"""Parity of the HIP encode path (through the C ABI) with the CPU oracle.

Bar: bit-exact ids AND offsets for every doc. Cases: the reference's golden vectors,
randomised small configs (Python oracle), the five bench configs C0..C4 on seeded
subsets (C++ oracle), the edge cases the reference's tests and the kernel's own
structure call for, and full-size C1 batch properties."""
import json
import os
import random

import numpy as np
import pytest

import tkz
from tkz import synth
from oracle import oracle as orc

pytestmark = pytest.mark.gpu

NT = min(16, os.cpu_count() or 1)


def _batch(docs):
    off = np.zeros(len(docs) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(d) for d in docs])
    return b"".join(docs), off


def _check_batch(tok, ref, docs, via_device=False):
    data, off = _batch(docs)
    if via_device:
        db = tkz.DeviceBatch(tok, np.frombuffer(data, dtype=np.uint8) if data else np.zeros(0, np.uint8), off)
        db.run()
        row, ids, offs = db.results()
        db.free()
    else:
        row, ids, offs = tok.encode_batch(data if data else b"\0", off)
    for i, d in enumerate(docs):
        exp = ref.encode(d)
        lo, hi = int(row[i]), int(row[i + 1])
        assert ids[lo:hi].tolist() == [t[0] for t in exp], (i, d[:80])
        assert offs[lo:hi].tolist() == [[t[1], t[2]] for t in exp], (i, d[:80])
    assert int(row[-1]) == len(ids)


def test_golden_vectors_gpu(golden):
    n = 0
    for case in golden["cases"]:
        encs = case.get("encode", [])
        if not encs:
            continue
        tok = tkz.Tokenizer.from_json(json.dumps(case["config"]))
        for e in encs:
            enc = tok.encode(e["text"])
            assert enc.ids == e["ids"], (case["name"], e["text"])
            if "offsets" in e:
                assert [list(o) for o in enc.offsets] == e["offsets"], (case["name"], e["text"])
            if "tokens" in e:
                assert [t.decode() for t in enc.tokens] == e["tokens"]
            assert enc.attention_mask == [1] * len(enc.ids)
            assert enc.type_ids == [0] * len(enc.ids)
            assert enc.special_token_mask == [0] * len(enc.ids)
            n += 1
        # the same vectors as one batch
        ref = orc.RefTokenizer.from_json(json.dumps(case["config"]))
        _check_batch(tok, ref, [e["text"].encode() for e in encs])
    assert n >= 25


def _rand_cfg(rng, model, pretok, norm):
    alpha = list("abcdeXYZ") + ["é", "Ω", "中", "😀"]
    vocab = {}
    for ch in alpha:
        if rng.random() < 0.9:
            vocab[ch] = len(vocab)
    model_obj = {}
    if model == "BPE":
        toks = list(vocab)
        merges = []
        for _ in range(60):
            a, b = rng.choice(toks), rng.choice(toks)
            m = a + b
            if m not in vocab:
                vocab[m] = len(vocab)
                toks.append(m)
            merges.append([a, b] if rng.random() < 0.3 else f"{a} {b}")
        model_obj = {"type": "BPE", "vocab": vocab, "merges": merges}
        if rng.random() < 0.5:
            vocab["<unk>"] = len(vocab)
            model_obj["unk_token"] = "<unk>"
    else:
        vocab["[UNK]"] = len(vocab)
        for _ in range(60):
            w = "".join(rng.choice(alpha) for _ in range(rng.randint(1, 6)))
            if rng.random() < 0.5:
                w = "##" + w
            vocab.setdefault(w, len(vocab))
        model_obj = {"type": "WordPiece", "vocab": vocab, "max_input_chars_per_word": rng.choice([5, 30, 100])}
    cfg = {"model": model_obj}
    if pretok:
        cfg["pre_tokenizer"] = {"type": pretok}
    if norm:
        cfg["normalizer"] = {"type": norm}
    return cfg


def _rand_text(rng, n):
    pool = list("abcdeXYZ") + ["é", "Ω", "中", "😀", "q", " ", " ", " ", "\t", "\n", "\r", ",", ".", "!", "\x0b", "\x0c"]
    return "".join(rng.choice(pool) for _ in range(n)).encode("utf-8")


@pytest.mark.parametrize("model", ["BPE", "WordPiece"])
@pytest.mark.parametrize("pretok", [None, "Whitespace", "WhitespaceSplit", "BertPreTokenizer", "Metaspace"])
def test_random_configs_gpu(model, pretok):
    rng = random.Random(f"{model}-{pretok}")
    for trial in range(5):
        cfg = _rand_cfg(rng, model, pretok, rng.choice([None, "Lowercase", "BertNormalizer", "NFC"]))
        tok = tkz.Tokenizer.from_json(json.dumps(cfg))
        if model == "BPE":
            tok.set_dedup(trial % 3 - 1)  # auto, off, on
        ref = orc.RefTokenizer.from_json(json.dumps(cfg))
        lens = [0, 1, 2, 7, 8, 9, 31, 63, 64, 65, 200, 511, 512, 513, 700, 1100] + [rng.randint(0, 90) for _ in range(60)]
        docs = [_rand_text(rng, n) for n in lens]
        _check_batch(tok, ref, docs, via_device=(trial % 2 == 1))


def _edge_docs():
    docs = [
        b"", b"a", b" ", b"  a  ", b"lllll", b"ll lll llll", b"hello world", b"Hello, World!",
        b"\t\n\r hello \r\n", b"x" * 23 + b" " + b"y" * 24 + b" " + b"z" * 25,  # around MAXB
        b"w" * 600 + b" tail",                         # long word crossing a 512-B step
        b"!" * 1030,                                   # all punct (word-ring capacity)
        b"a " * 700,                                   # many tiny words
        "é中😀Ωé".encode() * 20,                        # multi-byte, one long word
        b"\xe4\xb8",                                   # truncated codepoint
        b"\xff\xfe abc \x80",                          # invalid lead bytes
        b"ab\xe4",                                     # truncated at word end
        b"word\x0bvt\x0cff",
    ]
    # unaligned starts: prepend docs of odd length
    return docs + [b"q" * k + b" abc" for k in range(1, 17)]


@pytest.mark.parametrize("pretok", [None, "Whitespace", "BertPreTokenizer"])
def test_edge_cases_bpe(pretok):
    vocab = {c: i for i, c in enumerate(["a", "b", "c", "l", "h", "e", "o", " ", "w", "x", "y", "z", "q", "!",
                                         "é", "中", "😀", "Ω", "r", "d", "t", "i", "f", "v", "ä"])}
    merges = []
    for a, b in [("l", "l"), ("h", "e"), ("ll", "o"), ("he", "llo"), ("w", "w"), ("ww", "ww"), ("x", "x"),
                 ("é", "中"), ("😀", "Ω"), ("a", "b"), ("ab", "c"), ("!", "!"), ("q", "q")]:
        m = a + b
        vocab.setdefault(a, len(vocab)); vocab.setdefault(b, len(vocab)); vocab.setdefault(m, len(vocab))
        merges.append(f"{a} {b}")
    for unk, memo, dedup in ((None, True, -1), ("<unk>", True, 1), (None, False, 1), (None, False, 0)):
        cfg = {"model": {"type": "BPE", "vocab": dict(vocab), "merges": merges}}
        if unk:
            cfg["model"]["vocab"]["<unk>"] = len(vocab)
            cfg["model"]["unk_token"] = unk
        if pretok:
            cfg["pre_tokenizer"] = {"type": pretok}
        tok = tkz.Tokenizer.from_json(json.dumps(cfg))
        tok.set_word_memo(memo)
        tok.set_dedup(dedup)
        ref = orc.RefTokenizer.from_json(json.dumps(cfg))
        _check_batch(tok, ref, _edge_docs() + [b"abc " * 300 + b"lllll " * 200])  # repeats for dedup


@pytest.mark.parametrize("dedup", [-1, 1])
def test_bpe_new_id_equals_first(dedup):
    # pathological merge "a" + "" -> "a" (new_id == first): sequential re-test chains
    cfg = {"model": {"type": "BPE", "vocab": {"a": 0, "": 1, "b": 2}, "merges": ["a ", "a b"]}}
    tok = tkz.Tokenizer.from_json(json.dumps(cfg))
    tok.set_dedup(dedup)
    ref = orc.RefTokenizer.from_json(json.dumps(cfg))
    _check_batch(tok, ref, [b"ab", b"aab", b"abab", b"abababababab " * 40])


@pytest.mark.parametrize("pretok", [None, "Whitespace", "BertPreTokenizer"])
def test_edge_cases_wordpiece(pretok):
    vocab = {"[UNK]": 0, "a": 1, "##a": 2, "b": 3, "##b": 4, "ab": 5, "##ab": 6, "hello": 7, "##llo": 8,
             "he": 9, "!": 10, "x" * 30: 11, "##" + "x" * 30: 12, "é": 13, "##中": 14}
    for mc in (5, 40, 100):
        cfg = {"model": {"type": "WordPiece", "vocab": vocab, "max_input_chars_per_word": mc}}
        if pretok:
            cfg["pre_tokenizer"] = {"type": pretok}
        tok = tkz.Tokenizer.from_json(json.dumps(cfg))
        ref = orc.RefTokenizer.from_json(json.dumps(cfg))
        docs = _edge_docs() + [b"ab" * 15, b"x" * 60, b"x" * 90 + b"a", b"hello he llo", b"\xc3\xa9\xe4\xb8\xad"]
        _check_batch(tok, ref, docs)


def test_missing_unk_token_gpu():
    tok = tkz.Tokenizer.from_json(json.dumps({"model": {"type": "WordPiece", "vocab": {"a": 0}},
                                              "pre_tokenizer": {"type": "Whitespace"}}))
    assert tok.encode("a a").ids == [0, 0]
    with pytest.raises(tkz.TokenizerError) as ei:
        tok.encode("b")
    assert ei.value.name == "MissingUnkToken"


@pytest.mark.parametrize("cfg_id,n_docs,memo,dedup", [(0, 1000, True, -1), (1, 20000, True, -1), (2, 20000, True, -1),
                                                     (3, 20000, True, -1), (4, 4000, True, -1), (1, 20000, False, -1),
                                                     (2, 20000, False, -1), (4, 4000, False, -1), (1, 20000, True, 1),
                                                     (1, 20000, False, 1), (2, 20000, True, 0), (4, 4000, False, 1)])
def test_bench_configs_vs_oracle(cfg_id, n_docs, memo, dedup):
    js = synth.tokenizer_json(cfg_id)
    tok = tkz.Tokenizer.from_json(js)
    tok.set_word_memo(memo)
    tok.set_dedup(dedup)
    ref = orc.RefTokenizer.from_json(js)
    co = orc.COracle(ref)
    # a subset taken from the middle of the bench stream
    data, off = synth.docs(cfg_id, n_docs, first_doc=12345)
    db = tkz.DeviceBatch(tok, data, off)
    db.run()
    row, ids, offs = db.results()
    db.free()
    erow, eids, eoffs = co.encode_batch(data, off, n_threads=NT)
    assert np.array_equal(row, erow)
    assert np.array_equal(ids, eids)
    assert np.array_equal(offs, eoffs)


def test_c1_full_size_properties():
    """C1 at BASELINE size (1M x 512 B): exact parity on a seeded 50k-doc sample, and
    size-independent properties over the whole batch."""
    js = synth.tokenizer_json(1)
    tok = tkz.Tokenizer.from_json(js)
    ref = orc.RefTokenizer.from_json(js)
    n = 1_000_000
    data, off = synth.docs(1, n)
    db = tkz.DeviceBatch(tok, data, off)
    db.run()
    row, ids, offs = db.results()
    db.free()
    assert row[0] == 0 and np.all(np.diff(row.astype(np.int64)) >= 0)
    # (1) token byte lengths per doc == non-whitespace bytes per doc (every char of the
    #     synthetic alphabet is in the vocab and BPE tokens partition each word)
    klen = np.zeros(max(ref.vocab.values()) + 1, dtype=np.int64)
    for k, v in ref.vocab.items():
        klen[v] = len(k)
    tok_bytes = np.add.reduceat(klen[ids], row[:-1].astype(np.int64)) if len(ids) else np.zeros(n)
    tok_bytes[np.diff(row.astype(np.int64)) == 0] = 0
    d = data[: int(off[-1])].reshape(n, 512)
    nonws = 512 - ((d == 32) | (d == 9) | (d == 10) | (d == 13)).sum(axis=1)
    assert np.array_equal(tok_bytes, nonws)
    # (2) offsets are well-formed pretoken-relative spans
    assert np.all(offs[:, 0] < offs[:, 1])
    assert np.all(np.asarray(klen[ids]) == (offs[:, 1] - offs[:, 0]))
    # (3) exact parity on a 50k-doc seeded sample
    rng = np.random.default_rng(7)
    sample = np.sort(rng.choice(n, size=50_000, replace=False))
    docs = [bytes(d[i]) for i in sample]
    sdata, soff = _batch(docs)
    co = orc.COracle(ref)
    erow, eids, eoffs = co.encode_batch(sdata, soff, n_threads=NT)
    got_ids = np.concatenate([ids[int(row[i]):int(row[i + 1])] for i in sample])
    got_offs = np.concatenate([offs[int(row[i]):int(row[i + 1])] for i in sample])
    assert np.array_equal(got_ids, eids)
    assert np.array_equal(got_offs, eoffs)


@pytest.mark.parametrize("cfg_id", [1, 2, 3, 4])
def test_bench_shard_exact(cfg_id):
    """SURVEY.md §8(d) parity check at BASELINE size: every doc of the 1M-doc bench shard
    (C1-C3: the whole config; C4: one GPU's shard of the 64M-doc stream, ≈ 1 GB) bit-exact
    against the C++ oracle, ids, offsets and row_ptr; plus the full-batch 64-bit rolling
    hash of ids, identical on both sides."""
    js = synth.tokenizer_json(cfg_id)
    tok = tkz.Tokenizer.from_json(js)
    data, off = synth.docs(cfg_id, 1_000_000)
    db = tkz.DeviceBatch(tok, data, off)
    db.run()
    row, ids, offs = db.results()
    db.free()
    co = orc.COracle(orc.RefTokenizer.from_json(js))
    erow, eids, eoffs = co.encode_batch(data, off, n_threads=NT)
    assert np.array_equal(row, erow)
    assert np.array_equal(ids, eids)
    assert np.array_equal(offs, eoffs)

    def rolling(x):  # h = h * m + id (mod 2^64) over all ids in batch order, 1M at a time
        x = x.astype(np.uint64)
        m = np.uint64(0x100000001B3)
        h = np.uint64(0xCBF29CE484222325)
        with np.errstate(over="ignore"):
            for s0 in range(0, len(x), 1 << 20):
                blk = x[s0:s0 + (1 << 20)]
                pw = np.cumprod(np.full(len(blk), m, dtype=np.uint64))  # m^1 .. m^n
                w = np.concatenate((np.ones(1, dtype=np.uint64), pw[:-1]))[::-1]  # m^(n-1) .. m^0
                h = h * pw[-1] + np.sum(blk * w, dtype=np.uint64)
        return int(h)

    assert rolling(np.array([1, 2], np.uint64)) == ((0xCBF29CE484222325 * 0x100000001B3 + 1) * 0x100000001B3 + 2) % (1 << 64)
    print(f"C{cfg_id}: {len(ids)} tokens, id hash {rolling(ids):016x} == {rolling(eids):016x}")


@pytest.mark.parametrize("cfg_id", [1, 3])
def test_host_pipeline(cfg_id):
    """tkz_encode_batch with the PCIe copies overlapped (1-MiB chunks here, 32 MiB by
    default): the first batch runs unchunked and sets the tokens-per-byte estimate; later
    batches go in chunks, including one that outgrows the estimate (denser text), docs
    larger than a chunk and runs of empty docs. Every result equals the oracle's."""
    js = synth.tokenizer_json(cfg_id)
    tok = tkz.Tokenizer.from_json(js)
    tok.set_host_pipeline(1 << 20)
    co = orc.COracle(orc.RefTokenizer.from_json(js))

    def check(data, off):
        row, ids, offs = tok.encode_batch(data, off)
        erow, eids, eoffs = co.encode_batch(np.frombuffer(data, np.uint8), off, n_threads=NT)
        assert np.array_equal(row, erow)
        assert np.array_equal(ids, eids)
        assert np.array_equal(offs, eoffs)
        return len(ids)

    d, off = synth.docs(cfg_id, 12000, first_doc=777)
    data = d[: int(off[-1])].tobytes()
    check(data, off)  # unchunked: sets the estimate
    check(data, off)  # 6 chunks
    # denser text (1-3 byte words): more tokens per byte than the estimate
    rs = np.random.RandomState(5)
    words = [rs.choice(list(b"etaoinsrhl"), size=rs.randint(1, 4)).astype(np.uint8).tobytes() for _ in range(1_500_000)]
    dense = b" ".join(words)
    cuts = np.sort(rs.choice(len(dense), size=3000, replace=False))
    doff = np.concatenate(([0], cuts, [len(dense)])).astype(np.uint64)
    n = check(dense, doff)
    assert n > 0.3 * len(dense)  # well above the C1/C3 estimate
    check(dense, doff)  # now the estimate fits
    # a doc larger than several chunks, then runs of empty docs
    big = [data[: 3 << 20], b"", b"", data[100:5000]] + [b""] * 100 + [data[: 1 << 20]] + [b""] * 5
    bdata, boff = _batch(big)
    check(bdata, boff)


@pytest.mark.parametrize("cfg_id", [1, 6])
def test_host_pipeline_long_pretokens(cfg_id):
    """The pipelined host path (1-MiB chunks) on chunks holding pretokens of more than 255 B
    (offsets >= 256, k_bpe_long): C1 docs with 300-700-byte words in one chunk, and C6
    (ByteLevel: every doc one 512-B pretoken). Equal to the oracle, unchunked (the first
    call sets the tokens-per-byte estimate) and chunked."""
    js = synth.tokenizer_json(cfg_id)
    tok = tkz.Tokenizer.from_json(js)
    tok.set_host_pipeline(1 << 20)
    co = orc.COracle(orc.RefTokenizer.from_json(js))
    d, off = synth.docs(cfg_id, 8000 if cfg_id == 1 else 6000, first_doc=4242)
    docs = [d[int(off[i]): int(off[i + 1])].tobytes() for i in range(len(off) - 1)]
    if cfg_id == 1:
        for i, n in ((5000, 300), (5001, 700), (5003, 256)):
            docs[i] = docs[i][:40] + b" " + b"e" * n + b" " + docs[i][40:]
    data, boff = _batch(docs)
    for _ in range(2):  # unchunked (sets the tokens-per-byte estimate), then chunked
        row, ids, offs = tok.encode_batch(data, boff)
        erow, eids, eoffs = co.encode_batch(np.frombuffer(data, np.uint8), boff, n_threads=NT)
        assert np.array_equal(row, erow)
        assert np.array_equal(ids, eids)
        assert np.array_equal(offs, eoffs)
    if cfg_id == 1:
        assert int(np.max(offs)) >= 256  # the long words' offsets made it through


def _np_stream(seed, total, max_doc, tiny_frac=0.3):
    """Byte stream + doc offsets for the chunked scan: ASCII letters, delimiters, punct
    and stray UTF-8 lead/continuation bytes; word lengths vary per 4-KiB block (short,
    medium, a few hundred to thousands of bytes); docs are empty/tiny or long."""
    rs = np.random.RandomState(seed)
    pool = np.frombuffer(b"abcdeXYZqlmnop" * 4 + b"!,.\t\n\r\x0b\x0c" + b"\xc3\xa9\xe4\xb8\xad\xf0\x9f\x98\x80", np.uint8)
    data = pool[rs.randint(0, len(pool), size=total)]
    blk = 4096
    p = rs.choice([0.25, 0.08, 0.002, 0.0], size=(total + blk - 1) // blk, p=[0.5, 0.3, 0.15, 0.05])
    space = rs.random_sample(total) < np.repeat(p, blk)[:total]
    data[space] = ord(" ")
    lens = []
    s = 0
    while s < total:
        r = rs.random_sample()
        n = rs.randint(0, 4) if r < tiny_frac else rs.randint(4, max_doc)
        n = min(n, total - s)
        lens.append(n)
        s += n
    off = np.zeros(len(lens) + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    return data, off


def _check_stream(tok, co, data, off):
    db = tkz.DeviceBatch(tok, data, off)
    db.run()
    row, ids, offs = db.results()
    db.free()
    erow, eids, eoffs = co.encode_batch(data, off, n_threads=NT)
    lo = int(off[0])
    assert np.array_equal(row - row[0], erow - erow[0]) and int(row[0]) == 0
    assert np.array_equal(ids, eids)
    assert np.array_equal(offs, eoffs)
    return len(ids), lo


@pytest.mark.parametrize("model", ["BPE", "WordPiece"])
@pytest.mark.parametrize("pretok", [None, "Whitespace", "BertPreTokenizer"])
def test_chunked_stream(model, pretok):
    """24 MiB batches: words and documents crossing 512-B steps and chunk boundaries,
    runs of empty/tiny docs (more than 64 doc boundaries per step)."""
    rng = random.Random(f"stream-{model}-{pretok}")
    cfg = _rand_cfg(rng, model, pretok, rng.choice([None, "Lowercase"]))
    tok = tkz.Tokenizer.from_json(json.dumps(cfg))
    co = orc.COracle(orc.RefTokenizer.from_json(json.dumps(cfg)))
    data, off = _np_stream(hash((model, pretok)) & 0xFFFF, 24 << 20, 3000 if pretok is None else 40000)
    n_tok, _ = _check_stream(tok, co, data, off)
    assert n_tok > 0


def test_chunked_stream_large_chunks():
    """~110 MB BPE/Whitespace batch: the chunk size reaches its 8-KiB maximum."""
    rng = random.Random("stream-large")
    cfg = _rand_cfg(rng, "BPE", "Whitespace", None)
    tok = tkz.Tokenizer.from_json(json.dumps(cfg))
    co = orc.COracle(orc.RefTokenizer.from_json(json.dumps(cfg)))
    data, off = _np_stream(7, 110 << 20, 60000, tiny_frac=0.5)
    _check_stream(tok, co, data, off)


def test_doc_offsets_not_starting_at_zero():
    """tkz_encode_batch_device with doc_off[0] > 0 (bytes before the first doc ignored)."""
    rng = random.Random("offset")
    cfg = _rand_cfg(rng, "BPE", "Whitespace", None)
    tok = tkz.Tokenizer.from_json(json.dumps(cfg))
    co = orc.COracle(orc.RefTokenizer.from_json(json.dumps(cfg)))
    data, off = _np_stream(11, 3 << 20, 5000)
    for shift in (1, 100, 8192 + 3):
        off2 = off + np.uint64(shift)
        data2 = np.concatenate([np.frombuffer(b"zz zz" * (shift // 5 + 1), np.uint8)[:shift], data])
        db = tkz.DeviceBatch(tok, data2, off2)
        db.run()
        row, ids, offs = db.results()
        db.free()
        erow, eids, eoffs = co.encode_batch(data, off, n_threads=NT)
        assert np.array_equal(row, erow) and np.array_equal(ids, eids) and np.array_equal(offs, eoffs)


def test_all_empty_docs():
    cfg = {"model": {"type": "BPE", "vocab": {"a": 0}, "merges": []}, "pre_tokenizer": {"type": "Whitespace"}}
    tok = tkz.Tokenizer.from_json(json.dumps(cfg))
    for n in (1, 5, 1000):
        off = np.zeros(n + 1, dtype=np.uint64)
        db = tkz.DeviceBatch(tok, np.zeros(0, np.uint8), off)
        db.run()
        row, ids, offs = db.results()
        db.free()
        assert row.tolist() == [0] * (n + 1) and len(ids) == 0


@pytest.mark.parametrize("max_len", [0, 8, 40, 70])
def test_dense_doc_boundaries(max_len):
    """Many doc boundaries per 1-KiB scan step (k_encode takes up to 15 from one vector load
    of doc_off, more through the scalar walk): docs of 0..max_len bytes, empty runs and
    docs of exactly 64 bytes in between, C1's vocab; row_ptr, ids and offsets exact."""
    from tkz import synth

    js = synth.tokenizer_json(1)
    tok = tkz.Tokenizer.from_json(js)
    rng = np.random.default_rng(max_len)
    words = [b"the", b"of", b"tokenizer", b"a", b"zig", b"gpu", b"\n", b"  "]
    docs = []
    for i in range(30_000):
        r = rng.random()
        if r < 0.05:
            docs.append(b"x" * 64)
        elif r < 0.10:
            docs.extend([b""] * int(rng.integers(1, 40)))
        else:
            n = int(rng.integers(0, max_len + 1))
            d = b""
            while len(d) < n:
                d += words[int(rng.integers(len(words)))] + b" "
            docs.append(d[:n])
    data, off = _batch(docs)
    data = np.frombuffer(data + bytes(16), dtype=np.uint8).copy()
    db = tkz.DeviceBatch(tok, data, off)
    db.run()
    row, ids, offs = db.results()
    db.free()
    erow, eids, eoffs = orc.COracle(orc.RefTokenizer.from_json(js)).encode_batch(data, off, n_threads=NT)
    assert np.array_equal(row, erow) and np.array_equal(ids, eids) and np.array_equal(offs, eoffs)
