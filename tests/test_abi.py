"""CPU-only tests of the product library: the C ABI loads and exports every symbol
declared in include/tkz.h, and the host side (tokenizer.json loader, GPU table images,
decode, vocab queries, added tokens) matches the oracle. No compute is launched."""
import json
import os
import re

import pytest

import tkz
from oracle import oracle as orc
from tests.conftest import REPO


def _header_functions():
    src = open(os.path.join(REPO, "include", "tkz.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"\b(tkz_\w+)\s*\(", src)
    return sorted(set(names))


def test_library_exports_every_header_symbol():
    names = _header_functions()
    assert len(names) >= 25
    L = tkz.lib()
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing


def test_golden_host_side(golden):
    for case in golden["cases"]:
        t = tkz.Tokenizer.from_json(json.dumps(case["config"]))
        r = orc.RefTokenizer.from_json(json.dumps(case["config"]))
        assert t.get_vocab_size() == r.get_vocab_size(), case["name"]
        if "vocab_size" in case:
            assert t.get_vocab_size() == case["vocab_size"], case["name"]
        for tok, tid in case.get("token_to_id", []):
            assert t.token_to_id(tok) == tid, case["name"]
        for tid, tok in case.get("id_to_token", []):
            got = t.id_to_token(tid)
            assert (got.decode() if got is not None else None) == tok, case["name"]
        for d in case.get("decode", []):
            assert t.decode(d["ids"], d["skip_special"]).decode() == d["text"], case["name"]
        for a in case.get("add_special", []):
            assert t.add_special_tokens(a["tokens"]) == a["added"]
            assert t.get_vocab_size() == a["vocab_size_after"]
        info = t.info()
        assert info["model"] == r.model_kind
        assert info["normalizer"] == r.norm
        assert info["pre_tokenizer"] == r.pretok
        assert info["decoder"] == r.decoder
        assert info["n_merges"] == r.n_accepted, case["name"]


def test_golden_errors(golden):
    for e in golden["errors"]:
        with pytest.raises(tkz.TokenizerError) as ei:
            tkz.Tokenizer.from_json(e["json"])
        assert ei.value.name == e["error"], e["name"]


def test_more_config_errors():
    bad = [
        ('{"model": {"type": "BPE", "vocab": {"a": 1.5}}}', "InvalidVocabEntry"),
        ('{"model": {"type": "BPE", "vocab": {"a": "x"}}}', "InvalidVocabEntry"),
        ('{"model": {"type": "BPE", "vocab": {"a": true}}}', "InvalidVocabEntry"),
        ('{"model": {"type": "BPE", "vocab": []}}', "MissingVocab"),
        ('{"model": 3}', "MissingModel"),
        ("[1, 2]", "InvalidJson"),
        ('{"model": {"type": "WordPiece", "vocab": {}},}', "InvalidJson"),
    ]
    for js, name in bad:
        with pytest.raises(tkz.TokenizerError) as ei:
            tkz.Tokenizer.from_json(js)
        assert ei.value.name == name, js
        with pytest.raises(orc.RefError) as eo:
            orc.RefTokenizer.from_json(js)
        assert eo.value.name == name, js


def test_json_duplicate_keys_and_utf8_are_invalid():
    """Zig 0.15 std.json (config.zig:60, default ParseOptions): a duplicate key in any
    object is error.DuplicateField and ill-formed UTF-8 in a string a syntax error, both
    InvalidJson. Restated from the std library (no reference test pins them)."""
    bad = [
        b'{"model": {"type": "BPE", "vocab": {"a": 0, "a": 1}}}',                 # vocab key
        b'{"model": {"type": "BPE", "vocab": {"a": 0}}, "model": {"type": "BPE", "vocab": {"b": 0}}}',
        b'{"model": {"type": "BPE", "type": "WordPiece", "vocab": {"a": 0}}}',
        b'{"model": {"type": "BPE", "vocab": {"\\u00e9": 0, "\xc3\xa9": 1}}}',    # equal after unescaping
        b'{"model": {"type": "BPE", "vocab": {"\xc3": 0}}}',                       # truncated sequence
        b'{"model": {"type": "BPE", "vocab": {"\xc0\xaf": 0}}}',                   # overlong
        b'{"model": {"type": "BPE", "vocab": {"\xed\xa0\x80": 0}}}',               # encoded surrogate
        b'{"model": {"type": "BPE", "vocab": {"\xf4\x90\x80\x80": 0}}}',           # above U+10FFFF
        b'{"model": {"type": "BPE", "vocab": {"a": NaN}}}',
    ]
    for js in bad:
        with pytest.raises(tkz.TokenizerError) as ei:
            tkz.Tokenizer.from_json(js)
        assert ei.value.name == "InvalidJson", js
        with pytest.raises(orc.RefError) as eo:
            orc.RefTokenizer.from_json(js)
        assert eo.value.name == "InvalidJson", js
    ok = b'{"model": {"type": "BPE", "vocab": {"\xc3\xa9": 0, "\xf0\x9f\x98\x80": 1, "\xe4\xb8\x80": 2}}}'
    assert tkz.Tokenizer.from_json(ok).get_vocab_size() == 3
    assert len(orc.RefTokenizer.from_json(ok).vocab) == 3


def test_json_escapes_and_unicode_keys():
    cfg = '{"model": {"type": "BPE", "vocab": {"\\u00e9": 0, "\\ud83d\\ude00": 1, "a\\"b": 2, "\\u00e9\\ud83d\\ude00": 3}, "merges": [["\\u00e9", "\\ud83d\\ude00"]]}}'
    t = tkz.Tokenizer.from_json(cfg)
    assert t.token_to_id("é") == 0
    assert t.token_to_id("😀") == 1
    assert t.token_to_id('a"b') == 2
    assert t.debug_merge(0, 1) == (0, 3)


def test_missing_file():
    with pytest.raises(tkz.TokenizerError) as ei:
        tkz.Tokenizer.from_file("/nonexistent/tokenizer.json")
    assert ei.value.name == "FileNotFound"


def test_merge_rules_match_oracle():
    cfg = {"model": {"type": "BPE", "vocab": {"a": 0, "b": 1, "ab": 2, "c": 3, "bc": 4},
                     "merges": ["a", "x b", "a c", "a b", ["b", "c"], "a b extra", "", " b"]}}
    t = tkz.Tokenizer.from_json(json.dumps(cfg))
    r = orc.RefTokenizer.from_json(json.dumps(cfg))
    for a in range(5):
        for b in range(5):
            assert t.debug_merge(a, b) == r.merges.get((a, b)), (a, b)


@pytest.mark.parametrize("cfg_id", [0, 1, 3])
def test_synthetic_tables_match_oracle(cfg_id):
    from tkz import synth
    js = synth.tokenizer_json(cfg_id)
    t = tkz.Tokenizer.from_json(js)
    r = orc.RefTokenizer.from_json(js)
    assert t.get_vocab_size() == r.get_vocab_size()
    for (a, b), v in list(r.merges.items())[:5000]:
        assert t.debug_merge(a, b) == v
    for k, v in list(r.vocab.items())[:5000]:
        assert t.debug_vocab(k) == v
    assert t.debug_vocab(b"\x00never-a-key") is None


def test_wide_ids_use_wide_tables():
    cfg = {"model": {"type": "BPE", "vocab": {"a": 70000, "b": 1, "ab": 80000}, "merges": ["a b"]}}
    t = tkz.Tokenizer.from_json(json.dumps(cfg))
    assert t.info()["compact_tables"] == 0
    assert t.debug_merge(70000, 1) == (0, 80000)
    cfg["model"]["vocab"] = {"a": 7, "b": 1, "ab": 8}
    t2 = tkz.Tokenizer.from_json(json.dumps(cfg))
    assert t2.info()["compact_tables"] == 1


def test_encode_without_gpu_fails_loudly():
    if tkz.device_available():
        pytest.skip("a GPU is present")
    t = tkz.Tokenizer.from_json(json.dumps({"model": {"type": "WordPiece", "vocab": {"[UNK]": 0, "a": 1}}}))
    with pytest.raises(tkz.TokenizerError) as ei:
        t.encode("a")
    assert ei.value.name == "DeviceError"


def test_tuning_switches_host_side():
    """tkz_set_dedup / tkz_set_word_memo / tkz_set_host_pipeline only record a mode (no
    compute); a null handle is InvalidArgument."""
    from tkz import synth

    t = tkz.Tokenizer.from_json(synth.tokenizer_json(2))
    for mode in (-1, 0, 1, 7):
        t.set_dedup(mode)
    t.set_word_memo(False)
    t.set_word_memo(True)
    for chunk in (0, 1 << 20, 32 << 20):
        t.set_host_pipeline(chunk)
    lib = tkz.lib()
    assert lib.tkz_set_dedup(None, 1) != 0
    assert lib.tkz_set_word_memo(None, 1) != 0
    assert lib.tkz_set_host_pipeline(None, 1) != 0


def test_create_opts_host_side():
    """tkz_create_from_json_opts (tkz_opts) records its options without touching a GPU;
    invalid options are InvalidArgument; defaults equal tkz_create_from_json's."""
    import ctypes

    from tkz import synth

    js = synth.tokenizer_json(1)
    t = tkz.Tokenizer.from_json(js, device=0, word_memo=False, dedup=1, host_chunk=4 << 20)
    assert t.info()["model"] == 1
    o = tkz._Opts()
    tkz.lib().tkz_opts_default(ctypes.byref(o))
    assert (o.device, o.word_memo, o.dedup, o.host_chunk) == (-1, 1, -1, 32 << 20)
    o.device = -2
    h = ctypes.c_void_p()
    assert tkz.lib().tkz_create_from_json_opts(js, len(js), ctypes.byref(o), ctypes.byref(h)) != 0
    assert not h.value


def test_encode_batch_gpus_without_gpu_fails_loudly():
    """tkz_encode_batch_gpus has no CPU fallback either."""
    if tkz.device_available():
        pytest.skip("a GPU is present")
    import numpy as np

    t = tkz.Tokenizer.from_json(json.dumps({"model": {"type": "WordPiece", "vocab": {"[UNK]": 0, "a": 1}}}))
    with pytest.raises(tkz.TokenizerError) as ei:
        t.encode_batch(b"a a", np.array([0, 1, 3], dtype=np.uint64), gpu_mask=0b11)
    assert ei.value.name == "DeviceError"
