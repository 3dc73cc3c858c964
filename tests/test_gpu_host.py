"""The host-buffer batch path (tkz_encode_batch: host text in, host CSR out, the shape of
/root/reference/src/lib.zig:109-160 Tokenizer.encode over a batch): pipelined chunks with
the CSR slices queued from a helper thread, page-locked input (tkz_host_alloc), and the
timeline recorded while profiling is on (tkz_host_profile_read)."""
import os

import numpy as np
import pytest

import tkz
from tkz import synth
from oracle import oracle as orc

pytestmark = pytest.mark.gpu

NT = min(16, os.cpu_count() or 1)


def test_pipelined_pageable_and_pinned_inputs():
    js = synth.tokenizer_json(1)
    tok = tkz.Tokenizer.from_json(js)
    tok.set_host_pipeline(1 << 20)  # many chunks
    data, off = synth.docs(1, 20_000, first_doc=11)
    erow, eids, eoffs = orc.COracle(orc.RefTokenizer.from_json(js)).encode_batch(data, off, n_threads=NT)
    for _ in range(2):  # the first call sizes the pipeline (tokens per byte), the second pipelines
        row, ids, offs = tok.encode_batch(data, off)
        assert np.array_equal(row, erow) and np.array_equal(ids, eids) and np.array_equal(offs, eoffs)
    pin = tkz.HostBuffer(len(data))
    pin.array[:] = data
    tkz.profile_enable(tok, True)
    tkz.host_profile_read(tok, reset=True)
    row, ids, offs = tok.encode_batch(pin.array, off)
    hp = tkz.host_profile_read(tok, reset=True)
    tkz.profile_enable(tok, False)
    assert np.array_equal(row, erow) and np.array_equal(ids, eids) and np.array_equal(offs, eoffs)
    assert hp["calls"] == 1 and hp["chunks"] >= 8
    assert hp["bytes_in"] == int(off[-1]) and hp["bytes_out"] == 8 * (len(off)) + 12 * len(ids)
    for k in ("h2d_ms", "encode_ms", "d2h_ms", "wall_ms"):
        assert hp[k] > 0, hp
    assert hp["d2h_span_ms"] <= hp["wall_ms"] * 1.5
    pin.free()
    tok.close()
