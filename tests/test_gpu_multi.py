"""tkz_encode_batch_gpus (SURVEY §8(b) gpu_mask): one process fanning a host batch out
over several GPUs. On a one-GPU box the split / replica / merge path runs with virtual
devices (gpu_mask bit i -> device i % count); the result must equal tkz_encode_batch's and
the C++ oracle's for any number of parts, including truncation / padding and docs far
larger than the rest (empty parts)."""
import numpy as np
import pytest

import tkz
from tkz import synth
from oracle import oracle as orc

pytestmark = pytest.mark.gpu


def _same(a, b):
    for x, y in zip(a, b):
        assert np.array_equal(x, y)


@pytest.mark.parametrize("cfg_id", [1, 2, 3, 4])
def test_gpus_match_single_device_and_oracle(cfg_id):
    js = synth.tokenizer_json(cfg_id)
    tok = tkz.Tokenizer.from_json(js)
    tok.set_virtual_devices(8)
    data, off = synth.docs(cfg_id, 20000, first_doc=777)
    one = tok.encode_batch(data, off)
    co = orc.COracle(orc.RefTokenizer.from_json(js))
    _same(one, co.encode_batch(data, off, n_threads=8))
    for mask in (0b1, 0b11, 0b1011, 0xFF):
        _same(tok.encode_batch(data, off, gpu_mask=mask), one)


def test_gpus_uneven_docs_and_padding():
    js = synth.tokenizer_json(1)
    tok = tkz.Tokenizer.from_json(js)
    tok.set_virtual_devices(4)
    data, off = synth.docs(1, 64, first_doc=5)
    # one doc holding most of the bytes: the byte-balanced cuts leave parts empty
    head = np.frombuffer(b"word " * 20000, np.uint8)
    big = np.concatenate([head, np.asarray(data, np.uint8)[: int(off[-1])]])
    off2 = np.concatenate([[0], np.asarray(off, np.uint64) + head.size]).astype(np.uint64)
    assert big.size == int(off2[-1])
    _same(tok.encode_batch(big, off2, gpu_mask=0xF), tok.encode_batch(big, off2))
    tok.set_truncation(16)
    tok.set_padding(16, pad_id=3)
    full1 = tok.encode_batch_full(data, off)
    full4 = tok.encode_batch_full(data, off, gpu_mask=0xF)
    for k in full1:
        assert np.array_equal(full1[k], full4[k]), k
    assert int(full4["row_ptr"][-1]) == 16 * 64


def test_gpus_empty_batch_and_bad_mask():
    tok = tkz.Tokenizer.from_json(synth.tokenizer_json(1))
    row, ids, offs = tok.encode_batch(np.zeros(0, np.uint8), np.zeros(1, np.uint64), gpu_mask=0b1)
    assert row.tolist() == [0] and ids.size == 0
    with pytest.raises(tkz.TokenizerError) as ei:  # no virtual devices: bit 31 names no device
        tok.encode_batch(b"a b", np.array([0, 3], np.uint64), gpu_mask=1 << 31)
    assert ei.value.name == "InvalidArgument"
    with pytest.raises(tkz.TokenizerError):
        tok.encode_batch(b"a b", np.array([0, 3], np.uint64), gpu_mask=0)


def test_opts_device_and_memo_off():
    """tkz_opts: the tokenizer binds to device 0; memo off gives the same ids."""
    js = synth.tokenizer_json(1)
    data, off = synth.docs(1, 3000, first_doc=9)
    a = tkz.Tokenizer.from_json(js).encode_batch(data, off)
    b = tkz.Tokenizer.from_json(js, device=0, word_memo=False, dedup=1, host_chunk=0).encode_batch(data, off)
    _same(a, b)
    with pytest.raises(tkz.TokenizerError):
        tkz.Tokenizer.from_json(js, device=999).encode_batch(data, off)
