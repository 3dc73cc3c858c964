"""Parity of the batched GPU decode (tkz_decode_batch, decode.hip) with the oracle's
Tokenizer.decode restatement (oracle/oracle.py, lib.zig:163-189 + config.zig:488-530).

Bar: every decoded sequence byte-identical to the oracle's. Cases: each decoder type
(none, WordPiece "##" removal, ByteLevel copy, BPE "\\xC4\\xA0" -> " "), skip_special on
and off with added special tokens, ids outside every vocab, "#" runs and C4|A0 pairs that
straddle token and sequence boundaries, empty sequences, and an encode -> decode pass
over a bench config."""
import json
import random

import numpy as np
import pytest

import tkz
from tkz import synth
from oracle import oracle as orc

pytestmark = pytest.mark.gpu


def _cfg(decoder):
    toks = ["a", "b", "#", "##", "###", "#a", "a#", "##b", "Ġ", "Ġx", "x", "Ä", " ", "hello", "é",
            "Ä", "ab", "[CLS]", "[SEP]"]
    vocab = {}
    for t in toks:
        vocab.setdefault(t, len(vocab))
    cfg = {
        "model": {"type": "WordPiece", "vocab": vocab, "unk_token": "[CLS]"},
        "added_tokens": [
            {"id": vocab["[CLS]"], "content": "[CLS]", "special": True},
            {"id": vocab["[SEP]"], "content": "[SEP]", "special": True},
            {"id": len(vocab) + 5, "content": "<extra>", "special": True},
            {"id": len(vocab) + 6, "content": "<plain>", "special": False},
        ],
    }
    if decoder:
        cfg["decoder"] = {"type": decoder}
    return cfg, len(vocab) + 10


def _check(tok, ref, seqs, skip):
    row = np.zeros(len(seqs) + 1, dtype=np.uint64)
    row[1:] = np.cumsum([len(s) for s in seqs])
    ids = np.array([i for s in seqs for i in s], dtype=np.uint32)
    off, data = tok.decode_batch(row, ids, skip)
    assert len(off) == len(seqs) + 1 and int(off[0]) == 0
    for k, s in enumerate(seqs):
        exp = ref.decode(s, skip)
        got = data[int(off[k]):int(off[k + 1])]
        assert got == exp, (k, s[:20], got[:60], exp[:60])
        # the single-sequence host API agrees as well
        assert tok.decode(s, skip) == exp


@pytest.mark.parametrize("decoder", [None, "WordPiece", "ByteLevel", "BPE"])
def test_decode_batch_decoders(decoder):
    cfg, id_range = _cfg(decoder)
    js = json.dumps(cfg)
    tok = tkz.Tokenizer.from_json(js)
    ref = orc.RefTokenizer.from_json(js)
    rng = random.Random(f"dec-{decoder}")
    seqs = [[], [0], [2, 2, 2], [3, 3], [4, 2], [2, 3, 2], [6, 5, 7], [8, 9], [11, 8], [15, 8, 8]]
    seqs += [[rng.randrange(id_range) for _ in range(rng.randint(0, 40))] for _ in range(3000)]
    seqs += [[rng.choice([2, 3, 4, 5, 6, 8, 15]) for _ in range(rng.randint(0, 2000))] for _ in range(20)]
    seqs += [[] for _ in range(50)]
    for skip in (False, True):
        _check(tok, ref, seqs, skip)


def test_decode_batch_empty_batch():
    cfg, _ = _cfg("WordPiece")
    tok = tkz.Tokenizer.from_json(json.dumps(cfg))
    off, data = tok.decode_batch(np.zeros(6, dtype=np.uint64), np.zeros(0, dtype=np.uint32))
    assert off.tolist() == [0] * 6 and data == b""


@pytest.mark.parametrize("cfg_id,decoder", [(1, "BPE"), (3, "WordPiece"), (2, None)])
def test_encode_decode_bench_config(cfg_id, decoder):
    """encode (GPU) -> decode (GPU) over 5000 docs of a bench config, checked per doc
    against the oracle's decode of the same ids."""
    cfg = json.loads(synth.tokenizer_json(cfg_id))
    if decoder:
        cfg["decoder"] = {"type": decoder}
    js = json.dumps(cfg)
    tok = tkz.Tokenizer.from_json(js)
    ref = orc.RefTokenizer.from_json(js)
    data, off = synth.docs(cfg_id, 5000, first_doc=4242)
    row, ids, _ = tok.encode_batch(data[: int(off[-1])].tobytes(), off)
    doff, text = tok.decode_batch(row, ids)
    for k in range(len(off) - 1):
        seq = ids[int(row[k]):int(row[k + 1])].tolist()
        assert text[int(doff[k]):int(doff[k + 1])] == ref.decode(seq), k
