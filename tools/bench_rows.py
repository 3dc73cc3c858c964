"""Device-resident throughput of the SURVEY 8(f) rows beside encode, on C1 (1M x 512-B
docs, 32k BPE): truncation + padding to a dense [n_docs, 128] batch
(tkz_pad_batch_device, from the encode CSR) and the FastTokenizer batch
(tkz_fast_encode_batch_device: encode + clip + span fill into [n_docs, max_tokens]).
One JSON line per row; inputs and outputs resident in HBM, HIP stream synchronised
around K timed calls."""
import ctypes
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tokenizer-zig_amd")]
import tkz  # noqa: E402
from tkz import fast, synth  # noqa: E402

K = 5
L = fast._lib()
tok = tkz.Tokenizer.from_json(synth.tokenizer_json(1))
data, off = synth.docs(1, 1_000_000)
db = tkz.DeviceBatch(tok, data, off)
db.run()
db.sync()
n = db.n_docs
row = np.zeros(n + 1, dtype=np.uint64)
db.d_row.download(row)
T = int(row[-1])


def timed(fn):
    fn()
    L.tkz_synchronize(tok.handle)
    t0 = time.perf_counter()
    for _ in range(K):
        fn()
    L.tkz_synchronize(tok.handle)
    return (time.perf_counter() - t0) / K


# truncation + padding to a dense [n, 128] batch
LEN = 128
tok.set_truncation(LEN)
tok.set_padding(LEN)
cap = int(L.tkz_pad_capacity(tok.handle, n, T))
wsb = int(L.tkz_pad_workspace_size(n))
bufs = [tkz.DeviceBuffer(x) for x in ((n + 1) * 8, cap * 4, cap * 8, cap * 4, cap * 4, cap * 4, wsb)]


def pad():
    rc = L.tkz_pad_batch_device(tok.handle, db.d_row.ptr, db.d_ids.ptr, db.d_offs.ptr, n, *[b.ptr for b in bufs[:6]],
                                bufs[6].ptr, wsb, None)
    if rc:
        raise RuntimeError(rc)


dt = timed(pad)
out_bytes = n * LEN * (4 + 8 + 4 * 3) + (n + 1) * 8
print(json.dumps({"row": "truncate+pad to [n, 128] (tkz_pad_batch_device)", "docs": n, "tokens_in": T,
                  "ms": round(dt * 1e3, 4), "docs_per_s": round(n / dt), "out_GB_per_s": round(out_bytes / dt / 1e9, 1)}))
for b in bufs:
    b.free()
tok.set_truncation(None)
tok.set_padding(None, enabled=False)

# FastTokenizer batch: encode + clip + span fill into [n, max_tokens]
MT = 256
opts = fast._FastOptions(2048, MT)
fws = int(L.tkz_fast_workspace_size(tok.handle, db.total, n))
d_len, d_ids, d_offs, d_attn, d_ws, d_st = (tkz.DeviceBuffer(x) for x in (n * 4, n * MT * 4, n * MT * 8, n * MT * 4,
                                                                          fws, 16))
d_st.zero()


def fast_batch():
    rc = L.tkz_fast_encode_batch_device(tok.handle, db.d_bytes.ptr, db.d_off.ptr, n, db.total, 512,
                                        ctypes.byref(opts), d_len.ptr, d_ids.ptr, d_offs.ptr, d_attn.ptr, d_ws.ptr,
                                        fws, d_st.ptr, None)
    if rc:
        raise RuntimeError(rc)


dt = timed(fast_batch)
print(json.dumps({"row": "FastTokenizer batch, max_tokens 256 (tkz_fast_encode_batch_device)", "docs": n,
                  "bytes": db.total, "ms": round(dt * 1e3, 4), "input_GB_per_s": round(db.total / dt / 1e9, 1)}))
