"""Truncation / padding (Tokenizer.encode steps 6-7, lib.zig:149-157; Encoding.truncate /
Encoding.pad, encoding.zig:362-437). CPU: the oracle restatement against the reference's
own truncate/pad rules on hand-made cases. GPU: the batch path (pad.hip) and the single
Encoding API against the oracle, including the dense [n, L] case (max_length == length)."""
import json
import random

import numpy as np
import pytest

from oracle import oracle as orc

CFG = {"model": {"type": "WordPiece", "vocab": {"[UNK]": 0, "a": 1, "b": 2, "##b": 3, "ab": 4, "[PAD]": 5}},
       "pre_tokenizer": {"type": "Whitespace"}}


def test_oracle_truncate_pad_rules():
    ref = orc.RefTokenizer.from_json(json.dumps(CFG))
    e = ref.encode_full(b"a b ab a", truncation=2)
    assert e["ids"] == [1, 2] and e["attention_mask"] == [1, 1]
    e = ref.encode_full(b"a b", padding={"length": 5, "pad_id": 5, "pad_type_id": 1})
    assert e["ids"] == [1, 2, 5, 5, 5]
    assert e["type_ids"] == [0, 0, 1, 1, 1]
    assert e["special_token_mask"] == [0, 0, 1, 1, 1]
    assert e["attention_mask"] == [1, 1, 0, 0, 0]
    assert e["offsets"][2:] == [(0, 0)] * 3
    assert e["tokens"][2:] == [b"[PAD]"] * 3
    e = ref.encode_full(b"a b", padding={"length": 4, "pad_id": 9, "direction": "left"})
    assert e["ids"] == [9, 9, 1, 2] and e["attention_mask"] == [0, 0, 1, 1]
    # longer than the padding length: untouched (encoding.zig:387-389)
    e = ref.encode_full(b"a b a b", padding={"length": 2})
    assert e["ids"] == [1, 2, 1, 2]
    # truncate then pad
    e = ref.encode_full(b"a b a b a", truncation=3, padding={"length": 3})
    assert e["ids"] == [1, 2, 1]


def _random_docs(rng, n):
    words = [b"a", b"b", b"ab", b"abb", b"ba", b"x"]
    return [b" ".join(rng.choice(words) for _ in range(rng.randint(0, 30))) for _ in range(n)]


@pytest.mark.gpu
@pytest.mark.parametrize("trunc,pad", [(None, {"length": 40, "pad_id": 5, "pad_type_id": 2}),
                                       (7, None),
                                       (16, {"length": 16, "pad_id": 5}),
                                       (12, {"length": 20, "pad_id": 5, "direction": "left", "pad_token": b"<p>"}),
                                       (0, {"length": 3})])
def test_gpu_truncate_pad(trunc, pad):
    import tkz
    tok = tkz.Tokenizer.from_json(json.dumps(CFG))
    ref = orc.RefTokenizer.from_json(json.dumps(CFG))
    if trunc is not None:
        tok.set_truncation(trunc)
    if pad:
        tok.set_padding(pad["length"], pad.get("pad_id", 0), pad.get("pad_type_id", 0),
                        pad.get("pad_token", b"[PAD]"), pad.get("direction", "right"))
    rng = random.Random(f"{trunc}-{pad}")
    docs = _random_docs(rng, 3000) + [b"", b"a"]
    off = np.zeros(len(docs) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(d) for d in docs])
    out = tok.encode_batch_full(b"".join(docs), off)
    row = out["row_ptr"]
    for i, d in enumerate(docs):
        e = ref.encode_full(d, trunc, pad)
        lo, hi = int(row[i]), int(row[i + 1])
        assert out["ids"][lo:hi].tolist() == e["ids"], i
        assert [tuple(x) for x in out["offsets"][lo:hi].tolist()] == e["offsets"], i
        for k in ("type_ids", "special_token_mask", "attention_mask"):
            assert out[k][lo:hi].tolist() == e[k], (i, k)
    if trunc is not None and pad and trunc == pad["length"]:
        assert np.array_equal(row, np.arange(len(docs) + 1, dtype=np.uint64) * trunc)  # dense [n, L]
    # the single-document API (Tokenizer.encode -> Encoding)
    for d in docs[:50]:
        e = ref.encode_full(d, trunc, pad)
        enc = tok.encode(d)
        assert enc.ids == e["ids"] and enc.attention_mask == e["attention_mask"]
        assert enc.type_ids == e["type_ids"] and enc.special_token_mask == e["special_token_mask"]
        assert list(enc.tokens) == e["tokens"]
