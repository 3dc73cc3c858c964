"""The device port of the synthetic generator (tokenizer-zig_amd/csrc/gen.hip) against
the host generator (synth.cpp), byte for byte, and the device CSR hashes against
tests/shard_hash.py on the same result. Both are measurement infrastructure: bench.py
generates every rank's shard in HBM and verifies it with these hashes."""
import numpy as np
import pytest

import tkz
from tkz import synth
from shard_hash import CsrHash

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cfg,n,first", [(0, 1000, 0), (1, 20000, 0), (1, 3000, 999_000), (2, 20000, 5),
                                         (3, 20000, 123), (4, 20000, 0), (4, 5000, 63_995_000), (5, 20000, 7),
                                         (6, 2000, 1_000_000)])
def test_device_docs_match_host(cfg, n, first):
    dd = synth.DeviceDocs(cfg, n, first)
    try:
        data, off = dd.host()
        hd, ho = synth.docs(cfg, n, first_doc=first)
        assert np.array_equal(off, ho)
        assert dd.total == int(ho[-1])
        assert np.array_equal(data[: dd.total], hd[: dd.total])
    finally:
        dd.free()


@pytest.mark.parametrize("cfg", [1, 3, 4])
def test_device_batch_from_device_and_hash(cfg):
    """A batch over device-generated inputs equals the host-input batch, and the device
    rolling hashes equal CsrHash over the downloaded CSR."""
    js = synth.tokenizer_json(cfg)
    tok = tkz.Tokenizer.from_json(js)
    dd = synth.DeviceDocs(cfg, 30000, 1000)
    db = tkz.DeviceBatch.from_device(tok, dd.d_bytes, dd.d_off, dd.n_docs, dd.total, owner=dd)
    try:
        db.run()
        row, ids, offs = db.results()
        data, off = synth.docs(cfg, 30000, first_doc=1000)
        erow, eids, eoffs = tok.encode_batch(data, off)
        assert np.array_equal(row, erow) and np.array_equal(ids, eids) and np.array_equal(offs, eoffs)
        h = CsrHash()
        h.add(row, ids, offs)
        assert synth.csr_hash_device(db) == h.result()
        prow, pids, poffs = db.results_prefix(777)
        assert np.array_equal(prow, row[:778])
        assert np.array_equal(pids, ids[: int(row[777])]) and np.array_equal(poffs, offs[: int(row[777])])
    finally:
        db.free()
        dd.free()
        tok.close()


def test_hash_of_empty_and_tiny():
    tok = tkz.Tokenizer.from_json(synth.tokenizer_json(0))
    for data, off in ((np.zeros(16, np.uint8), np.zeros(1, np.uint64)),
                      (np.frombuffer(b"a b\0" + bytes(12), np.uint8).copy(), np.array([0, 3], np.uint64))):
        db = tkz.DeviceBatch(tok, data, off)
        try:
            db.run()
            row, ids, offs = db.results()
            h = CsrHash()
            h.add(row, ids, offs)
            assert synth.csr_hash_device(db) == h.result()
        finally:
            db.free()
    tok.close()
