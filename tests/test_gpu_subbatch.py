"""Workspace-bounded device encode (doc-aligned sub-batches), the batch statistics, the
C4 shard at its BASELINE size, and the multi-rank bench on one GPU.

A batch whose one-pass workspace exceeds the caller's runs in sub-batches; the outputs
must be identical to the oracle's (and so to a one-pass run) whatever the cut points."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import tkz
from tkz import synth
from oracle import oracle as orc
from shard_hash import CsrHash

pytestmark = pytest.mark.gpu

NT = min(16, os.cpu_count() or 1)
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _device(tok, data, off, max_ws=None):
    db = tkz.DeviceBatch(tok, data, off, max_workspace=max_ws)
    db.run()
    res = db.results()
    st = db.stats()
    db.free()
    return res, st


def _exact(res, exp):
    for a, b in zip(res, exp):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("cfg_id", [1, 2, 3, 4, 6, 7, 8, 9])
def test_sub_batches_exact(cfg_id):
    """~30-60 MB batches through a workspace for 1-2 MiB sub-batches: every doc equal to
    the oracle, and more than one pass ran (C6 / C8 / C9: the segmented path's arrays in
    every sub-batch's workspace; C7 / C9: wide tables)."""
    js = synth.tokenizer_json(cfg_id)
    tok = tkz.Tokenizer.from_json(js)
    n = 60_000 if cfg_id in (4, 6, 8, 9) else 80_000
    data, off = synth.docs(cfg_id, n, first_doc=12345)
    ws = int(tkz.lib().tkz_device_workspace_size_sub(tok.handle, 2 << 20))
    res, st = _device(tok, data, off, max_ws=ws)
    exp = orc.COracle(orc.RefTokenizer.from_json(js)).encode_batch(data, off, n_threads=NT)
    _exact(res, exp)
    assert st["sub_batches"] > 10, st
    res1, st1 = _device(tok, data, off)  # one pass: the same outputs and statistics
    _exact(res1, exp)
    assert st1["sub_batches"] == 1
    assert st1["pretokens"] == st["pretokens"] and st1["memo_hits"] == st["memo_hits"]
    if cfg_id in (6, 8, 9):  # the segmented path's outcome is deterministic (k_seg_check
        # reads the flags of the iterations before only): the same docs take it either way
        assert st["long_segmented"] == st1["long_segmented"], (st, st1)
        assert st1["long_segmented"] > 0.99 * n, st1


def test_sub_batches_edge_docs():
    """Sub-batch cuts among empty docs, 1-byte docs, docs of nearly a whole sub-batch and
    a first offset > 0 (the batch starts inside the buffer)."""
    js = synth.tokenizer_json(1)
    tok = tkz.Tokenizer.from_json(js)
    rs = np.random.RandomState(7)
    body, boff = synth.docs(1, 9000, first_doc=99)
    docs = []
    for i in range(9000):
        d = bytes(body[int(boff[i]):int(boff[i + 1])])
        k = rs.randint(10)
        if k == 0:
            d = b""
        elif k == 1:
            d = d[:1]
        docs.append(d)
    big = b" ".join([b"lorem"] * 170_000)[: (1 << 20) - 700]  # ~1 MiB: nearly a whole sub-batch
    docs[100:100] = [big, b"", b"", big]
    docs += [b""] * 5000
    lead = b"x" * 1000  # doc_off[0] = 1000: bytes before the first doc are not encoded
    data = lead + b"".join(docs)
    off = np.zeros(len(docs) + 1, np.uint64)
    off[0] = len(lead)
    off[1:] = len(lead) + np.cumsum([len(d) for d in docs])
    arr = np.frombuffer(data, np.uint8)
    ws = int(tkz.lib().tkz_device_workspace_size_sub(tok.handle, 1 << 20))
    res, st = _device(tok, arr, off, max_ws=ws)
    co = orc.COracle(orc.RefTokenizer.from_json(js))
    rel = off - off[0]
    exp = co.encode_batch(arr[len(lead):], rel, n_threads=NT)
    _exact(res, exp)
    assert st["sub_batches"] >= 4


def test_sub_batch_doc_too_large():
    """A doc larger than the workspace's sub-batch is InvalidArgument (not a wrong result)."""
    js = synth.tokenizer_json(1)
    tok = tkz.Tokenizer.from_json(js)
    doc = (b"abc " * 700_000)  # 2.8 MB
    off = np.array([0, 10, len(doc)], np.uint64)
    ws = int(tkz.lib().tkz_device_workspace_size_sub(tok.handle, 1 << 20))
    db = tkz.DeviceBatch(tok, np.frombuffer(doc, np.uint8), off, max_workspace=ws)
    with pytest.raises(tkz.TokenizerError) as ei:
        db.run()
    db.free()
    assert ei.value.name == "InvalidArgument"


def test_batch_stats_pretokens():
    """tkz_device_batch_stats: pretokens = the Whitespace pretokens of the batch (counted
    here on the host), memo hits <= pretokens; the memo off gives no hits."""
    js = synth.tokenizer_json(1)
    tok = tkz.Tokenizer.from_json(js)
    data, off = synth.docs(1, 20_000)
    b = np.asarray(data[: int(off[-1])])
    delim = np.isin(b, np.frombuffer(b" \t\n\r", np.uint8))
    starts = ~delim & np.concatenate(([True], delim[:-1]))
    starts[off[:-1].astype(np.int64)] |= ~delim[off[:-1].astype(np.int64)]  # every doc start is a break
    _, st = _device(tok, data, off)
    assert st["pretokens"] == int(starts.sum())
    assert 0 < st["memo_hits"] <= st["pretokens"]
    tok.set_word_memo(False)
    _, st0 = _device(tok, data, off)
    assert st0["memo_hits"] == 0 and st0["pretokens"] == st["pretokens"]


@pytest.mark.timeout(900)
def test_c4_shard_8M():
    """SURVEY.md 8(d) C4 rule at the stated size: one GPU's shard of the 64M-doc stream
    (docs [0, 8M), ~7.7 GB) through a 32-GiB workspace (the one-pass workspace would be
    ~210 GB): the rolling hashes of row_ptr, ids and offsets of the whole shard equal the
    oracle's (tests/golden/c4_shard_8M.json), and a 1M-doc subset in the middle is
    checked doc by doc."""
    gold = json.load(open(os.path.join(REPO, "tests", "golden", "c4_shard_8M.json")))
    n = gold["n_docs"]
    js = synth.tokenizer_json(4)
    tok = tkz.Tokenizer.from_json(js)
    data, off = synth.docs(4, n)
    assert int(off[-1]) == gold["bytes"]
    (row, ids, offs), st = _device(tok, data, off, max_ws=32 << 30)
    assert st["sub_batches"] > 1
    h = CsrHash()
    h.add(row, ids, offs)
    got = h.result()
    assert got["n_tokens"] == gold["n_tokens"]
    assert (got["row_ptr"], got["ids"], got["offsets"]) == (gold["row_ptr"], gold["ids"], gold["offsets"])
    d0, d1 = 3_500_000, 4_500_000
    sub = off[d0:d1 + 1] - off[d0]
    erow, eids, eoffs = orc.COracle(orc.RefTokenizer.from_json(js)).encode_batch(
        data[int(off[d0]):int(off[d1])], sub, n_threads=NT)
    t0, t1 = int(row[d0]), int(row[d1])
    assert np.array_equal(row[d0:d1 + 1] - row[d0], erow)
    assert np.array_equal(ids[t0:t1], eids)
    assert np.array_equal(offs[t0:t1], eoffs)
    print(f"C4 8M shard: {got['n_tokens']} tokens in {st['sub_batches']} sub-batches, hashes match")


@pytest.mark.timeout(900)
def test_c4_shard_8M_auto_workspace():
    """The same shard through DeviceBatch's default workspace (the one-pass size capped to
    the device's free memory after the outputs: what `bench.py --config 4 --docs 8000000`
    uses, 2 sub-batches on a 288-GB MI355X): the whole-shard hashes equal the oracle's."""
    gold = json.load(open(os.path.join(REPO, "tests", "golden", "c4_shard_8M.json")))
    js = synth.tokenizer_json(4)
    tok = tkz.Tokenizer.from_json(js)
    data, off = synth.docs(4, gold["n_docs"])
    (row, ids, offs), st = _device(tok, data, off)
    h = CsrHash()
    h.add(row, ids, offs)
    got = h.result()
    assert got["n_tokens"] == gold["n_tokens"]
    assert (got["row_ptr"], got["ids"], got["offsets"]) == (gold["row_ptr"], gold["ids"], gold["offsets"])
    print(f"C4 8M shard, default workspace: {st['sub_batches']} sub-batches, hashes match")


_STREAM = {}  # shard -> CsrHash result of the device encode (test_c4_stream_shard)
_STREAM_GOLD = os.path.join(REPO, "tests", "golden", "c4_stream_64M.json")


@pytest.mark.skipif(not os.path.exists(_STREAM_GOLD), reason="c4_stream_64M.json not generated")
@pytest.mark.timeout(900)
@pytest.mark.parametrize("shard", range(8))
def test_c4_stream_shard(shard):
    """SURVEY.md 8(d) C4 rule over the WHOLE BASELINE stream: 64M Zipf docs (62 GB) as the
    8 shards of 8M docs that 8 GPUs get; each shard runs on this GPU through a 32-GiB
    workspace and its row_ptr / ids / offsets hashes must equal the oracle's
    (tests/golden/c4_stream_64M.json, make_c4_stream_hash.py)."""
    gold = json.load(open(_STREAM_GOLD))["shards"][shard]
    tok = tkz.Tokenizer.from_json(synth.tokenizer_json(4))
    data, off = synth.docs(4, gold["n_docs"], first_doc=gold["first_doc"])
    assert int(off[-1]) == gold["bytes"]
    (row, ids, offs), st = _device(tok, data, off, max_ws=32 << 30)
    del data
    h = CsrHash()
    h.add(row, ids, offs)
    got = h.result()
    _STREAM[shard] = got
    assert {k: got[k] for k in ("n_docs", "n_tokens", "row_ptr", "ids", "offsets")} == \
        {k: gold[k] for k in ("n_docs", "n_tokens", "row_ptr", "ids", "offsets")}
    print(f"C4 shard {shard}: {got['n_tokens']} tokens, {st['sub_batches']} sub-batches, hashes match")


@pytest.mark.skipif(not os.path.exists(_STREAM_GOLD), reason="c4_stream_64M.json not generated")
def test_c4_stream_whole():
    """The full-batch hashes of the 64M-doc stream (the 8 shards concatenated in doc order,
    row_ptr continued across shards), composed from the device shard results."""
    from shard_hash import combine

    if len(_STREAM) < 8:
        pytest.skip("needs every test_c4_stream_shard result in this session")
    gold = json.load(open(_STREAM_GOLD))["stream"]
    got = combine([_STREAM[s] for s in range(8)])
    assert got == {k: gold[k] for k in got}
    print(f"C4 64M-doc stream: {got['n_tokens']} tokens, full-batch hashes match")


def test_bench_two_ranks_share_gpu():
    """bench.py --gpus 2 (no torchrun) on one GPU: two HIP ranks, each encoding and
    verifying its own shard against the oracle; one JSON line with both shards."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--share-gpu",
                        "--docs", "50000", "--steps", "2", "--warmup", "1", "--verify", "--verify-docs", "50000",
                        "--no-cpu-baseline", "--no-memo-off-run", "--primary-only"], capture_output=True, text=True,
                       timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert out["n_gpus"] == 2
    v = out["verified"]
    assert (v["docs_per_rank"], v["sample_match"], v["ranks_failed"]) == (50000, True, 0)
    assert out["config"]["parallelism"] == "doc-shard x2"
    assert out["config"]["bytes_per_gpu"] == 50000 * 512
