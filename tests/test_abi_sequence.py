"""The reference API's call sequence through the C ABI (verdict r2 item 6):
tests/c/abi_sequence.c makes the calls integration/zig/gpu.zig makes -- fromJson,
fromFile, getVocabSize, tokenToId, idToToken, decode, addSpecialTokens, encode,
encodeBatch, decodeBatch, the error paths, deinit (/root/reference/src/lib.zig:48-223) --
as a C program linked against libtkz.so. Its output is checked against the reference's
own test vectors (tests/golden/reference_vectors.json) and the oracle. Host-side calls
run here; encode / batch calls run on the GPU (and fail loudly without one)."""
import json
import os
import subprocess

import pytest

from oracle import oracle as orc

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(REPO, "tokenizer-zig_amd", "tkz", "abi_sequence")
GOLDEN = json.load(open(os.path.join(REPO, "tests", "golden", "reference_vectors.json"), encoding="utf-8"))
CASES = [c for c in GOLDEN["cases"] if c.get("config") and ("encode" in c or "decode" in c or "token_to_id" in c)]


def _run(case, mode, tmp_path):
    path = tmp_path / "tokenizer.json"
    path.write_text(json.dumps(case["config"]), encoding="utf-8")
    text = next((e["text"] for e in case.get("encode", []) if e["text"]), "hello")
    toks = [t for t, _ in case.get("token_to_id", [])] or ["hello"]
    ids = [i for i, _ in case.get("id_to_token", [])]
    dec = case.get("decode", [])
    if dec and dec[0]["ids"]:
        ids = dec[0]["ids"]
    ids = ids or [0, 1]
    r = subprocess.run([BIN, str(path), mode, text, ",".join(toks), ",".join(map(str, ids))], capture_output=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr.decode(errors="replace")[-2000:]
    return json.loads(r.stdout), text, toks, ids


def _expect_common(out, case, toks, ids):
    ref = orc.RefTokenizer.from_json(json.dumps(case["config"]))
    assert out["from_json"] == 0 and out["from_file"] == 0
    assert out["vocab_size"] == out["from_file_vocab_size"] == ref.get_vocab_size()
    if "vocab_size" in case:
        assert out["vocab_size"] == case["vocab_size"]
    assert out["token_to_id"] == [ref.token_to_id(t.encode()) for t in toks]
    for t, want in case.get("token_to_id", []):
        assert out["token_to_id"][toks.index(t)] == want
    got_i2t = [None if x is None else bytes(x) for x in out["id_to_token"]]
    assert got_i2t == [ref.id_to_token(i) for i in ids]
    for i, want in case.get("id_to_token", []):
        if i in ids:
            assert got_i2t[ids.index(i)] == (None if want is None else want.encode())
    assert bytes(out["decode"]) == ref.decode(ids, False)
    assert bytes(out["decode_skip"]) == ref.decode(ids, True)
    for d in case.get("decode", []):
        if d["ids"] == ids:
            assert bytes(out["decode_skip" if d["skip_special"] else "decode"]) == d["text"].encode()
    # addSpecialTokens([<x1>, <x2> with id 500, <x1> again]) (vocab.zig:39-57)
    n_before = ref.get_vocab_size()
    added = sum(ref.added.add_special_token(c, i) for c, i in ((b"<x1>", None), (b"<x2>", 500), (b"<x1>", None)))
    assert out["added"] == added == 2
    assert out["x2_id"] == 500
    assert out["vocab_size_after"] == n_before + 2 == ref.get_vocab_size()
    assert bytes(out["decode_x2"]) == ref.decode(ids + [500], False)
    assert bytes(out["decode_x2_skip"]) == ref.decode(ids + [500], True)
    # error names (config.zig:18-30; std.json duplicate field; std.fs)
    assert (out["err_invalid_json"], out["err_duplicate_key"], out["err_missing_model"], out["err_unsupported"],
            out["err_file"]) == (1, 1, 2, 3, 7)
    assert out["done"] is True
    return ref


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_host_call_sequence(case, tmp_path):
    out, text, toks, ids = _run(case, "host", tmp_path)
    _expect_common(out, case, toks, ids)
    if not _gpu_visible():
        assert out["encode"] == 11  # TKZ_ERR_DEVICE: no CPU fallback


def _gpu_visible():
    import tkz

    return tkz.device_available()


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_gpu_call_sequence(case, tmp_path):
    out, text, toks, ids = _run(case, "gpu", tmp_path)
    ref = _expect_common(out, case, toks, ids)
    exp = orc.RefTokenizer.from_json(json.dumps(case["config"])).encode(text.encode())
    assert out["encode"] == 0
    assert out["ids"] == [t[0] for t in exp]
    assert out["offsets"] == [[t[1], t[2]] for t in exp]
    n = len(exp)
    assert out["type_ids"] == [0] * n and out["special_token_mask"] == [0] * n and out["attention_mask"] == [1] * n
    # Token.value is the MODEL vocab's string (bpe.zig:255-262, wordpiece.zig), whatever
    # the added vocab maps the id to
    assert [bytes(t) for t in out["tokens"]] == [ref.vocab_r.get(t[0], b"") for t in exp]
    for e in case.get("encode", []):
        if e["text"] == text:
            assert out["ids"] == e["ids"]
            if "offsets" in e:
                assert out["offsets"] == e["offsets"]
    assert out["encode_batch"] == 0
    assert out["batch_row_ptr"] == [0, n, 2 * n, 2 * n]
    assert out["batch_ids"] == out["ids"] * 2
    assert out["decode_batch"] == 0
    assert bytes(out["decode_batch_row0"]) == ref.decode(out["ids"], False)
    assert out["decode_batch_row2_len"] == 0
