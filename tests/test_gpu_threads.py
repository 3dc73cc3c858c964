"""Concurrent callers (SURVEY §8(b) Threading): the reference's Tokenizer.encode is
read-only on self, so callers may share a tokenizer across threads
(/root/reference/src/lib.zig:109-160). Here several host threads encode different batches
through one tokenizer, and through two tokenizers, at the same time (ctypes releases the
GIL for the calls); every result must equal the same batch encoded alone, and the oracle's."""
import threading

import numpy as np
import pytest

import tkz
from tkz import synth
from oracle import oracle as orc

pytestmark = pytest.mark.gpu


def _same(a, b):
    for x, y in zip(a, b):
        assert np.array_equal(x, y)


def _run_threads(jobs):
    """jobs: list of callables; runs them together, returns results in order (re-raises)."""
    out = [None] * len(jobs)
    err = []

    def work(i):
        try:
            out[i] = jobs[i]()
        except BaseException as e:  # noqa: BLE001 - re-raised in the main thread
            err.append(e)

    ts = [threading.Thread(target=work, args=(i,)) for i in range(len(jobs))]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in ts), "a thread did not finish"
    if err:
        raise err[0]
    return out


def test_threads_share_one_tokenizer():
    js = synth.tokenizer_json(1)
    tok = tkz.Tokenizer.from_json(js)
    batches = [synth.docs(1, 3000 + 500 * i, first_doc=10_000 * i) for i in range(4)]
    alone = [tok.encode_batch(d, o) for d, o in batches]
    co = orc.COracle(orc.RefTokenizer.from_json(js))
    for (d, o), a in zip(batches, alone):
        _same(a, co.encode_batch(d, o, n_threads=8))
    for _ in range(3):
        got = _run_threads([lambda d=d, o=o: tok.encode_batch(d, o) for d, o in batches])
        for g, a in zip(got, alone):
            _same(g, a)


def test_threads_two_tokenizers_and_single_docs():
    """BPE and WordPiece tokenizers side by side, batch and single-doc calls mixed."""
    js1, js3 = synth.tokenizer_json(1), synth.tokenizer_json(3)
    t1, t3 = tkz.Tokenizer.from_json(js1), tkz.Tokenizer.from_json(js3)
    d1, o1 = synth.docs(1, 4000, first_doc=3)
    d3, o3 = synth.docs(3, 4000, first_doc=3)
    a1, a3 = t1.encode_batch(d1, o1), t3.encode_batch(d3, o3)
    docs = [bytes(np.asarray(d1[int(o1[i]):int(o1[i + 1])])) for i in range(8)]
    singles = [t1.encode(x).ids for x in docs]
    jobs = [lambda: t1.encode_batch(d1, o1), lambda: t3.encode_batch(d3, o3),
            lambda: [t1.encode(x).ids for x in docs], lambda: t3.encode_batch(d3, o3)]
    for _ in range(2):
        g1, g3, gs, g3b = _run_threads(jobs)
        _same(g1, a1)
        _same(g3, a3)
        _same(g3b, a3)
        assert [list(x) for x in gs] == [list(x) for x in singles]


def test_threads_gpu_mask_with_settings_changes():
    """Two threads encode through gpu_mask (per-device replicas) while the main thread
    toggles the word memo between rounds (advice r2: replica settings are applied under the
    replica's lock); every result equals the single-device one."""
    js = synth.tokenizer_json(1)
    tok = tkz.Tokenizer.from_json(js)
    tok.set_virtual_devices(4)
    batches = [synth.docs(1, 6000, first_doc=40_000 * (i + 1)) for i in range(2)]
    alone = [tok.encode_batch(d, o) for d, o in batches]
    for rnd in range(4):
        tok.set_word_memo(rnd % 2 == 1)
        got = _run_threads([lambda d=d, o=o, m=m: tok.encode_batch(d, o, gpu_mask=m)
                            for (d, o), m in zip(batches, (0b11, 0b1111))])
        for g, a in zip(got, alone):
            _same(g, a)
    tok.set_word_memo(True)
