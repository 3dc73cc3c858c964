"""Pins the CPU oracle (pure-Python restatement + C++ restatement) to the reference's
own known-answer tests (tests/golden/reference_vectors.json) and cross-checks the two
restatements against each other. CPU only."""
import json
import random

import numpy as np
import pytest

from oracle import oracle as orc


def _cases(golden):
    return golden["cases"]


def test_golden_encode_python(golden):
    n = 0
    for case in _cases(golden):
        tk = orc.RefTokenizer.from_json(json.dumps(case["config"]))
        for e in case.get("encode", []):
            toks = tk.encode(e["text"].encode("utf-8"))
            assert [t[0] for t in toks] == e["ids"], (case["name"], e["text"])
            if "offsets" in e:
                assert [[t[1], t[2]] for t in toks] == e["offsets"], (case["name"], e["text"])
            if "tokens" in e:
                assert [s.decode() for s in tk.token_strings(toks)] == e["tokens"]
            n += 1
    assert n >= 25


def test_golden_host_functions(golden):
    for case in _cases(golden):
        tk = orc.RefTokenizer.from_json(json.dumps(case["config"]))
        if "vocab_size" in case:
            assert tk.get_vocab_size() == case["vocab_size"], case["name"]
        for tok, tid in case.get("token_to_id", []):
            assert tk.token_to_id(tok.encode()) == tid, case["name"]
        for tid, tok in case.get("id_to_token", []):
            got = tk.id_to_token(tid)
            assert (got.decode() if got is not None else None) == tok, case["name"]
        for d in case.get("decode", []):
            assert tk.decode(d["ids"], d["skip_special"]).decode() == d["text"], case["name"]
        for nz in case.get("normalize", []):
            assert tk.normalize(nz["text"].encode()).decode() == nz["out"], case["name"]
        for pt in case.get("pretokenize", []):
            s = pt["text"].encode()
            assert [s[a:b].decode() for a, b in tk.pre_tokenize(s)] == pt["out"], case["name"]
        for a in case.get("add_special", []):
            added = sum(tk.added.add_special_token(t.encode()) for t in a["tokens"])
            assert added == a["added"]
            assert tk.get_vocab_size() == a["vocab_size_after"]


def test_golden_errors(golden):
    for e in golden["errors"]:
        with pytest.raises(orc.RefError) as ei:
            orc.RefTokenizer.from_json(e["json"])
        assert ei.value.name == e["error"], e["name"]


def test_missing_unk_token_error():
    # wordpiece.zig:150,212: UNK absent from the vocab -> error.MissingUnkToken
    tk = orc.RefTokenizer.from_json(json.dumps({"model": {"type": "WordPiece", "vocab": {"a": 0}}}))
    with pytest.raises(orc.RefError) as ei:
        tk.encode(b"b")
    assert ei.value.name == "MissingUnkToken"


def test_slow_path_identical_pair_runs():
    # with the single merge 'l l', "lllll" -> [ll, ll, l] on the slow path
    cfg = {"model": {"type": "BPE", "vocab": {"l": 0, "ll": 1}, "merges": ["l l"]}}
    tk = orc.RefTokenizer.from_json(json.dumps(cfg))
    assert [t[0] for t in tk.encode(b"lllll")] == [1, 1, 0]
    assert [(t[1], t[2]) for t in tk.encode(b"lllll")] == [(0, 2), (2, 4), (4, 5)]


def test_merge_table_rules():
    # config.zig:228-273: rank counts accepted merges only; duplicate pair overwrites;
    # 'a' (no second part) skipped; unknown parts skipped; merged string must exist.
    cfg = {"model": {"type": "BPE", "vocab": {"a": 0, "b": 1, "ab": 2, "c": 3, "bc": 4},
                     "merges": ["a", "x b", "a c", "a b", ["b", "c"], "a b extra"]}}
    tk = orc.RefTokenizer.from_json(json.dumps(cfg))
    assert tk.merges == {(0, 1): (2, 2), (1, 3): (1, 4)}


def _rand_cfg(rng, model, pretok, norm):
    alpha = list("abcdeXYZ") + ["é", "Ω", "中"]
    vocab = {}
    for ch in alpha:
        vocab[ch] = len(vocab)
    merges = []
    if model == "BPE":
        toks = list(alpha)
        for _ in range(40):
            a, b = rng.choice(toks), rng.choice(toks)
            m = a + b
            if m not in vocab:
                vocab[m] = len(vocab)
                toks.append(m)
            merges.append(f"{a} {b}")
        model_obj = {"type": "BPE", "vocab": vocab, "merges": merges}
        if rng.random() < 0.5:
            vocab["<unk>"] = len(vocab)
            model_obj["unk_token"] = "<unk>"
    else:
        vocab["[UNK]"] = len(vocab)
        for _ in range(40):
            w = "".join(rng.choice(alpha) for _ in range(rng.randint(1, 5)))
            if rng.random() < 0.5:
                w = "##" + w
            vocab.setdefault(w, len(vocab))
        model_obj = {"type": "WordPiece", "vocab": vocab, "max_input_chars_per_word": rng.choice([5, 100])}
    cfg = {"model": model_obj}
    if pretok:
        cfg["pre_tokenizer"] = {"type": pretok}
    if norm:
        cfg["normalizer"] = {"type": norm}
    return cfg


def _rand_text(rng, n):
    pool = list("abcdeXYZ") + ["é", "Ω", "中", "😀", " ", " ", "\t", "\n", ",", ".", "!", "\x0b"]
    return "".join(rng.choice(pool) for _ in range(n)).encode("utf-8")


@pytest.mark.parametrize("model", ["BPE", "WordPiece"])
@pytest.mark.parametrize("pretok", [None, "Whitespace", "BertPreTokenizer"])
def test_python_vs_cpp_oracle(model, pretok):
    rng = random.Random(hash((model, pretok)) & 0xFFFF)
    for trial in range(4):
        cfg = _rand_cfg(rng, model, pretok, rng.choice([None, "Lowercase", "BertNormalizer"]))
        tk = orc.RefTokenizer.from_json(json.dumps(cfg))
        docs = [_rand_text(rng, rng.randint(0, 60)) for _ in range(60)]
        off = np.zeros(len(docs) + 1, dtype=np.uint64)
        off[1:] = np.cumsum([len(d) for d in docs])
        data = b"".join(docs)
        co = orc.COracle(tk)
        row_ptr, ids, offs = co.encode_batch(data, off, n_threads=2)
        for i, d in enumerate(docs):
            exp = tk.encode(d)
            lo, hi = int(row_ptr[i]), int(row_ptr[i + 1])
            assert ids[lo:hi].tolist() == [t[0] for t in exp], (cfg, d)
            assert offs[lo:hi].tolist() == [[t[1], t[2]] for t in exp], (cfg, d)
