"""Segmented long pretokens (encode.hip, the k_seg_* kernels): a long BPE pretoken
(the whole text under ByteLevel / Metaspace / no pre_tokenizer, /root/reference/src/
config.zig:387-402 and lib.zig:121) is cut at the ASCII chars BPE.tokenize skips
(/root/reference/src/model/bpe.zig:192-208); boundaries are checked against the merge
order (bpe.zig:214-253) and crossed ones joined. CPU: the algorithm's Python model
(tests/segment_model.py) equals the reference loop on random vocabs chosen so that merges
cross the cuts often. GPU: the kernel equals the oracle, with the path on and off."""
import json
import os
import random

import numpy as np
import pytest

from oracle import oracle as orc
from tests.segment_model import segmented_bpe

NT = min(16, os.cpu_count() or 1)


def random_bpe_json(seed, alphabet="abcde", n_merges=60, extra=(), unk=None, pretok=None, max_len=6,
                    unk_merges=False, ordered=True):
    """A BPE tokenizer.json over a tiny alphabet: merges of random token pairs, so merges
    across dropped spaces and runs of identical pairs are common. `extra`: more chars in
    the vocab (multi-byte ones and ' ' too: a whitespace with a mergeable id). `unk`: an
    unk token, at the end of the vocab (in no merge: inert), or among the merged tokens
    (unk_merges). `ordered`: skip a merge whose result is a token some earlier merge already
    used as a part (it would rank after that use: tokenizer.cpp merges_ordered), as in a
    trained table; False keeps such tables, which never take the segmented path."""
    rng = random.Random(seed)
    parts = set()
    vocab = {}
    for c in list(alphabet) + list(extra):
        vocab.setdefault(c, len(vocab))
    if unk is not None and unk_merges:
        vocab.setdefault(unk, len(vocab))
    toks = list(vocab)
    merges, seen = [], set()
    tries = 0
    while len(merges) < n_merges and tries < 100 * n_merges:
        tries += 1
        # short tokens merge first (more frequent in a trained vocab)
        pool = sorted(toks, key=len)[: max(4, len(toks) // 2)] if rng.random() < 0.7 else toks
        a, b = rng.choice(pool), rng.choice(pool)
        m = a + b
        if len(m.encode()) > max_len or (a, b) in seen or (ordered and m in parts):
            continue
        seen.add((a, b))
        parts.update((a, b))
        if m not in vocab:
            vocab[m] = len(vocab)
            toks.append(m)
        merges.append([a, b] if " " in a + b else f"{a} {b}")  # (tokens with a space: the list form)
    if unk is not None:
        vocab.setdefault(unk, len(vocab))
    model = {"type": "BPE", "vocab": vocab, "merges": merges, "unk_token": unk}
    return json.dumps({"model": model, "normalizer": None, "pre_tokenizer": pretok, "decoder": None})


def random_docs(seed, n, alphabet="abcde", lo=65, hi=512, seps=(" ", "\n", "  ", "\t"), extra=(), wmax=10):
    rng = random.Random(seed)
    chars = list(alphabet) + list(extra)
    docs = []
    for _ in range(n):
        target = rng.randint(lo, hi)
        s = ""
        while len(s.encode()) < target:
            s += "".join(rng.choice(chars) for _ in range(rng.randint(1, wmax)))
            s += rng.choice(seps)
        b = s.encode()[:target]
        while b and (b[-1] & 0xC0) == 0x80:  # no truncated multi-byte char at the end
            b = b[:-1]
        docs.append(b)
    return docs


CASES = [
    dict(seed=1),
    dict(seed=2, n_merges=120),
    dict(seed=3, alphabet="ab", n_merges=14),  # runs of identical pairs, long groups
    dict(seed=4, extra=("é", "中"), n_merges=80),
    dict(seed=5, alphabet="abcdefgh", n_merges=200, max_len=8),
]
# round 5: unk tokens (every char a symbol; spaces and unknown chars are the inert unk),
# an unk that merges (no inert cut: the whitespace cuts are checked), a ' ' with a
# mergeable id (a checked cut before it) next to a dropped '\n'
CASES_CUT = [
    dict(seed=11, unk="[UNK]"),
    dict(seed=12, unk="[UNK]", extra=("é",), n_merges=100),
    dict(seed=13, unk="<unk>", unk_merges=True, n_merges=90),
    dict(seed=14, extra=(" ",), n_merges=90),
    dict(seed=15, alphabet="ab", extra=(" ",), n_merges=20),
    dict(seed=16, unk="[UNK]", extra=(" ",), n_merges=90),
]


@pytest.mark.parametrize("case", CASES, ids=[str(c["seed"]) for c in CASES])
def test_model_equals_reference_loop(case):
    """The segment / profile / boundary-replay algorithm == BPE.tokenize on the whole
    pretoken (CPU model of the kernel)."""
    tok = orc.RefTokenizer.from_json(random_bpe_json(**case))
    docs = random_docs(case["seed"] + 100, 60, alphabet=case.get("alphabet", "abcde"),
                       extra=case.get("extra", ()) + (("ü",) if case.get("extra") else ()))
    taken = 0
    for d in docs:
        seg = segmented_bpe(tok, d)
        if seg is not None:
            taken += 1
            assert seg == tok.bpe_tokenize(d), d
            assert segmented_bpe(tok, d, edges=True) == seg, d
    assert taken >= len(docs) // 2


def _cut_docs(case, seed, n):
    # chars outside the vocab ('z', 'ü') map to unk (or are dropped without one)
    return random_docs(seed, n, alphabet=case.get("alphabet", "abcde") + "z",
                       extra=case.get("extra", ()) + ("ü",))


@pytest.mark.parametrize("case", CASES_CUT, ids=[str(c["seed"]) for c in CASES_CUT])
def test_model_cut_classes_equal_reference_loop(case):
    """Inert cuts (a symbol in no merge) and checked whitespace cuts: the segmented
    algorithm == BPE.tokenize on the whole pretoken."""
    tok = orc.RefTokenizer.from_json(random_bpe_json(**case))
    from tests.segment_model import cut_classes

    cls, _ = cut_classes(tok)
    if case.get("unk") and not case.get("unk_merges"):
        assert cls[ord(" ")] == "inert" or " " in case.get("extra", ())
    if " " in case.get("extra", ()):
        assert cls[ord(" ")] == "cut"
    taken = 0
    for d in _cut_docs(case, case["seed"] + 100, 80):
        seg = segmented_bpe(tok, d)
        if seg is not None:
            taken += 1
            assert seg == tok.bpe_tokenize(d), d
            assert segmented_bpe(tok, d, edges=True) == seg, d
    assert taken >= 40


def test_model_c6_docs():
    from tkz import synth

    tok = orc.RefTokenizer.from_json(synth.tokenizer_json(6))
    data, off = synth.docs(6, 40, first_doc=77)
    for i in range(40):
        d = bytes(data[int(off[i]):int(off[i + 1])])
        assert segmented_bpe(tok, d) == tok.bpe_tokenize(d)


def _random_merge_table(rng, ordered):
    """merges {(a, b): (rank, new_id)} over symbols 0..nsym-1. ordered: each merge makes a new
    symbol from existing ones (a trained table); else the ranks are shuffled, and a merge may
    make a symbol that already exists, so parts can be created after their use."""
    nsym = rng.randint(2, 7)
    merges, syms, nid = {}, list(range(nsym)), nsym
    for _ in range(rng.randint(2, 24)):
        a, b = rng.choice(syms), rng.choice(syms)
        if (a, b) in merges:
            continue
        new = nid if ordered or rng.random() < 0.7 else rng.choice(syms[nsym:] or [nid])
        if not ordered and new in (a, b):
            new = nid
        merges[(a, b)] = new
        if new == nid:
            syms.append(nid)
            nid += 1
    keys = list(merges)
    ranks = list(range(len(keys)))
    if ordered:
        rank, ranks = 0, []
        for _ in keys:
            ranks.append(rank)
            rank += rng.randint(1, 2)
    else:
        rng.shuffle(ranks)
    return {k: (r, merges[k]) for k, r in zip(keys, ranks)}, nsym


def test_edge_list_walk_equals_replay():
    """The kernel's boundary check walks only the edge lists (the rounds that changed the
    left group's last symbol and the right group's first): the same verdict as the replay of
    both whole profiles, on random ordered merge tables (ties and runs of equal pairs
    included) -- and on shuffled tables, wherever the two differ, the table is one the
    library keeps off the segmented path (merges_ordered False)."""
    from tests.segment_model import bpe_profile, crossed, crossed_edges, merges_ordered

    rng = random.Random(11)
    n_cross = n_diff = n_unordered = 0
    for it in range(3000):
        ordered = it % 2 == 0
        merges, nsym = _random_merge_table(rng, ordered)
        mo = merges_ordered(merges)
        assert mo or not ordered
        n_unordered += not mo
        for _ in range(6):
            A = [rng.randrange(nsym) for _ in range(rng.randint(1, 9))]
            B = [rng.randrange(nsym) for _ in range(rng.randint(1, 9))]
            left = (A, bpe_profile(merges, A)[1])
            right = (B, bpe_profile(merges, B)[1])
            c = crossed(merges, left, right)
            e = crossed_edges(merges, left, right)
            if mo:
                assert e == c, (merges, A, B)
            n_diff += e != c
            n_cross += c
    assert n_cross > 1000
    assert n_unordered > 300
    assert n_diff > 0  # (the shuffled tables do break the edge walk: the rule is needed)


# merges (ab,c), (c,d), (a,b) -- "ab" ranks after "abc" uses it. Whole
# pretoken "abcd": the reference merges (c,d) before (a,b) and gives [ab, cd]; the groups
# abc | d (a dropped char between them) each encode alone, and the edge walk judges their
# boundary uncrossed ([abc, d]).
COUNTER_JSON = json.dumps({
    "model": {"type": "BPE", "vocab": {"a": 0, "b": 1, "c": 2, "d": 3, "ab": 4, "abc": 5, "cd": 6},
              "merges": ["ab c", "c d", "a b"]},
    "normalizer": None, "pre_tokenizer": {"type": "ByteLevel"}, "decoder": None})


def test_unordered_table_counterexample():
    from tests.segment_model import bpe_profile, crossed, crossed_edges, merges_ordered

    tok = orc.RefTokenizer.from_json(COUNTER_JSON)
    assert not merges_ordered(tok.merges)
    A, B = [0, 1, 2], [3]
    left, right = (A, bpe_profile(tok.merges, A)[1]), (B, bpe_profile(tok.merges, B)[1])
    assert crossed(tok.merges, left, right) and not crossed_edges(tok.merges, left, right)
    assert [t[0] for t in tok.bpe_tokenize(b"abcd")] == [4, 6]
    d = b"abc\x00d" * 20  # (NUL has no id: a dropped cut between abc and d)
    assert segmented_bpe(tok, d) == tok.bpe_tokenize(d)
    assert segmented_bpe(tok, d, edges=True) != tok.bpe_tokenize(d)


def test_library_reports_unordered_tables():
    """The host library finds the same property (tkz_info.merges_ordered) and keeps such a
    table off the segmented path whatever tkz_set_long_segments says; trained tables and
    the random test vocabs take it."""
    import tkz
    from tkz import synth

    t = tkz.Tokenizer.from_json(COUNTER_JSON)
    inf = t.info()
    assert inf["merges_ordered"] == 0 and inf["long_segments"] == 0
    t.set_long_segments(True)
    assert t.info()["long_segments"] == 0
    t.close()
    for js in (synth.tokenizer_json(6), random_bpe_json(2, n_merges=120, pretok={"type": "ByteLevel"})):
        t = tkz.Tokenizer.from_json(js)
        assert t.info()["merges_ordered"] == 1 and t.info()["long_segments"] == 1
        t.set_long_segments(False)
        assert t.info()["long_segments"] == 0
        t.close()
    t = tkz.Tokenizer.from_json(random_bpe_json(2, n_merges=120, pretok={"type": "ByteLevel"}, ordered=False))
    assert t.info()["merges_ordered"] == 0 and t.info()["long_segments"] == 0
    t.close()


# ------------------------------------------------------------------------------ GPU
def _gpu_check(js, docs, seg=True, min_segmented=None, memo=True):
    import tkz

    off = np.zeros(len(docs) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(d) for d in docs])
    data = np.frombuffer(b"".join(docs) + bytes(16), dtype=np.uint8).copy()
    tok = tkz.Tokenizer.from_json(js)
    tok.set_long_segments(seg)
    tok.set_word_memo(memo)
    db = tkz.DeviceBatch(tok, data, off)
    db.run()
    row, ids, offs = db.results()
    st = db.stats()
    assert st.get("seg_bound_errors", 0) == 0, st  # (-DTKZ_SEG_BOUNDS builds)
    erow, eids, eoffs = orc.COracle(orc.RefTokenizer.from_json(js)).encode_batch(data, off, n_threads=NT)
    assert np.array_equal(row, erow)
    bad = np.nonzero(np.diff(row.astype(np.int64)) != np.diff(erow.astype(np.int64)))[0]
    assert np.array_equal(ids, eids), f"first differing docs: {bad[:3]}"
    assert np.array_equal(offs, eoffs)
    if not seg:
        assert st["long_segmented"] == 0
    elif min_segmented is not None:
        assert st["long_segmented"] >= min_segmented, st
    db.free()
    tok.close()
    return st


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=[str(c["seed"]) for c in CASES])
@pytest.mark.parametrize("seg", [True, False])
def test_gpu_random_vocabs(case, seg):
    js = random_bpe_json(**case, pretok={"type": "ByteLevel"})
    docs = random_docs(case["seed"] + 200, 400, alphabet=case.get("alphabet", "abcde"),
                       extra=case.get("extra", ()) + (("ü",) if case.get("extra") else ()))
    _gpu_check(js, docs, seg)


@pytest.mark.gpu
@pytest.mark.parametrize("memo", [True, False])
def test_gpu_c6_segmented_path_taken(memo):
    """C6 docs: (nearly) every doc takes the segmented path, with the segment memo (its
    single segments from the table) and without it (all by the register BPE)."""
    from tkz import synth

    data, off = synth.docs(6, 3000, first_doc=424_242)
    docs = [bytes(data[int(off[i]):int(off[i + 1])]) for i in range(3000)]
    st = _gpu_check(synth.tokenizer_json(6), docs, True, min_segmented=2900, memo=memo)
    assert st["long_words"] == 3000


@pytest.mark.gpu
def test_gpu_long_pretokens_past_512_bytes():
    """Zipf(64-4096 B) docs as whole pretokens (segmented beyond the 512-B LDS words too)."""
    from tkz import synth

    data, off = synth.docs(4, 1500, first_doc=31)
    docs = [bytes(data[int(off[i]):int(off[i + 1])]) for i in range(1500)]
    j = json.loads(synth.tokenizer_json(4))
    j["pre_tokenizer"] = {"type": "ByteLevel"}
    st = _gpu_check(json.dumps(j), docs, True, min_segmented=1000)
    assert st["long_words"] > 1000


@pytest.mark.gpu
def test_gpu_edge_docs():
    """Runs of identical pairs across cuts, groups past 16 / 32 / 64 symbols (W = 32 lanes,
    wave path, then the whole-pretoken fallback), groups of > 32 bytes, segments whose only char has no id (fallback), multi-byte
    chars, docs at 65 and 512 bytes, leading / trailing / repeated separators, words at the
    doc edges, one doc past 512 bytes (not segmented)."""
    js = random_bpe_json(3, alphabet="ab", n_merges=14, extra=("é",), pretok=None)
    docs = [
        b"a" * 30 + b" " + b"a" * 40 + b"\n" + b"ab" * 20,
        (b"ab " * 40)[:120],
        (b"ba " * 100)[:300],
        (b"a b " * 128)[:512],
        b" " * 3 + b"ab" * 40 + b" " * 5,
        "é a é ü b ab ü".encode() * 6,
        "üüü".encode() + b" " + b"ab" * 40,
        b"a" * 65,
        b"ab\n\n\n" * 30,
        (b"abba " * 120)[:600],
        (b"b" * 17 + b" ") * 10,
        (b"ab" * 40 + b" ") * 5,
        # groups of 17..32 symbols over more than 32 bytes (the W = 32 lane encode)
        ("é".encode() * 25 + b" ") * 4,
        ("éa".encode() * 12 + b" " + b"ab" * 5 + b"\n") * 3,
    ]
    _gpu_check(js, docs, True)
    _gpu_check(js, docs, False)


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES_CUT, ids=[str(c["seed"]) for c in CASES_CUT])
@pytest.mark.parametrize("seg", [True, False])
def test_gpu_cut_classes(case, seg):
    """Unk tokens (inert spaces and unknown chars), an unk in merges, whitespace with a
    mergeable id: the kernel == the oracle, the path on and off, and (on) most docs take
    it."""
    js = random_bpe_json(**case, pretok={"type": "Metaspace"})
    docs = _cut_docs(case, case["seed"] + 200, 400)
    # (a doc cut inside a multi-byte char ends in a truncated codepoint: not segmented)
    _gpu_check(js, docs, seg, min_segmented=200 if seg else None)


@pytest.mark.gpu
def test_gpu_unk_inert_segments():
    """An unk token makes every space a symbol; the unk is in no merge, so the spaces are
    inert cuts and the docs take the segmented path (round 4: no segmented path with unk)."""
    js = random_bpe_json(1, unk="[UNK]", pretok={"type": "ByteLevel"})
    docs = random_docs(9, 50)
    st = _gpu_check(js, docs, True)
    assert st["long_segmented"] >= 45, st


@pytest.mark.gpu
@pytest.mark.parametrize("seg", [True, False])
def test_gpu_c2_docs_lowercase_bytelevel(seg):
    """C2's mixed-UTF-8 docs and vocab with its Lowercase normalizer, every doc one pretoken
    (ByteLevel): segments with multi-byte chars, normalized bytes in the segment memo keys."""
    from tkz import synth

    data, off = synth.docs(2, 2000, first_doc=777)
    docs = [bytes(data[int(off[i]):int(off[i + 1])]) for i in range(2000)]
    j = json.loads(synth.tokenizer_json(2))
    j["pre_tokenizer"] = {"type": "ByteLevel"}
    st = _gpu_check(json.dumps(j), docs, seg, min_segmented=1000 if seg else None)
    assert st["long_words"] > 1000


@pytest.mark.gpu
def test_gpu_very_long_pretokens():
    """Whole-doc pretokens of 8..32 KB (thousands of segments each: k_seg_init's rounds,
    k_seg_out's 128-segment rounds, 16-bit token offsets near the 32,766-byte limit) and
    one just past it (not segmented), C1 text under ByteLevel."""
    from tkz import synth

    data, off = synth.docs(1, 12_000, first_doc=4242)
    text = bytes(data[: int(off[-1])])
    rng = random.Random(7)
    docs, p = [], 0
    for n in [32_766, 32_767] + [rng.randint(8_000, 32_000) for _ in range(150)]:
        if p + n > len(text):
            p = 0
        docs.append(text[p:p + n])
        p += n
    j = json.loads(synth.tokenizer_json(1))
    j["pre_tokenizer"] = {"type": "ByteLevel"}
    st = _gpu_check(json.dumps(j), docs, True, min_segmented=140)
    assert st["long_words"] == len(docs)


@pytest.mark.gpu
@pytest.mark.parametrize("seg,memo", [(True, True), (True, False), (False, True)])
def test_gpu_c8_metaspace_unk(seg, memo):
    """C8: C1's docs and vocab + an unk token under Metaspace (one pretoken per doc): every
    space, newline and tab is the unk symbol, which is in no merge -- inert cuts, no
    boundary checks. The path on and off, with and without the segment memo."""
    from tkz import synth

    data, off = synth.docs(8, 3000, first_doc=31_337)
    docs = [bytes(data[int(off[i]):int(off[i + 1])]) for i in range(3000)]
    st = _gpu_check(synth.tokenizer_json(8), docs, seg, min_segmented=2990 if seg else None, memo=memo)
    assert st["long_words"] == 3000


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [2, 4, 13])
def test_gpu_unordered_tables_exact(seed):
    """merge tables whose parts are created after their use (and the fixed
    counterexample) -- the GPU equals the oracle, and no doc takes the segmented path."""
    case = dict(next(c for c in CASES + CASES_CUT if c["seed"] == seed))
    js = random_bpe_json(**case, pretok={"type": "ByteLevel"}, ordered=False)
    docs = _cut_docs(case, seed + 300, 300)
    st = _gpu_check(js, docs, True)
    assert st["long_words"] > 100 and st["long_segmented"] == 0, st
    docs = [b"abc\x00d" * k for k in (20, 40, 70)] + [b"abcd " * 30, b"xabcdab\x00cd" * 10]
    st = _gpu_check(COUNTER_JSON, docs, True)
    assert st["long_segmented"] == 0, st


@pytest.mark.gpu
@pytest.mark.parametrize("hot", [0, 64, 1000])
def test_gpu_small_hot_bitmap(hot):
    """Verdict r5 item 6: the hot-pair bitmap at a forced small key count (set before the
    tables' first GPU use, and changed after it: rebuilt at once) gives the oracle's result;
    memo_info reports its keys and bytes."""
    import tkz
    from tkz import synth

    js = synth.tokenizer_json(6)
    data, off = synth.docs(6, 3000, first_doc=5150)
    erow, eids, eoffs = orc.COracle(orc.RefTokenizer.from_json(js)).encode_batch(data, off, n_threads=NT)
    tok = tkz.Tokenizer.from_json(js)
    tok.set_hot_pairs(hot)
    for k in (hot, 4096 if hot else 17):
        if k != hot:
            tok.set_hot_pairs(k)
        db = tkz.DeviceBatch(tok, data, off)
        db.run()
        row, ids, offs = db.results()
        assert np.array_equal(row, erow) and np.array_equal(ids, eids) and np.array_equal(offs, eoffs)
        assert db.stats()["long_segmented"] >= 2900
        mi = tok.memo_info()
        assert mi["hot_keys"] == k and mi["hot_bitmap_bytes"] == (k * k + 31) // 32 * 4, mi
        assert mi["table_bytes"] == mi["word_bytes"] + mi["seg_bytes"] + mi["hot_bitmap_bytes"]
        db.free()
    tok.close()
