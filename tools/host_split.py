"""Debug: where the host-buffer encode time goes (C1): pageable H2D of the input, the GPU
encode, D2H of the CSR into pre-touched vs freshly allocated host arrays."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tokenizer-zig_amd")]
import tkz  # noqa: E402
from tkz import synth  # noqa: E402

tok = tkz.Tokenizer.from_json(synth.tokenizer_json(1))
data, off = synth.docs(1, 1_000_000)
db = tkz.DeviceBatch(tok, data, off)
db.run()
db.sync()
src = np.zeros(db.d_bytes.nbytes, dtype=np.uint8)
src[: db.total] = np.asarray(data, dtype=np.uint8)[: db.total]
for rep in range(3):
    t0 = time.perf_counter()
    db.d_bytes.upload(src)
    t1 = time.perf_counter()
    db.run()
    db.sync()
    t2 = time.perf_counter()
    row = np.zeros(db.n_docs + 1, np.uint64)
    db.d_row.download(row)
    T = int(row[-1])
    ids = np.zeros(T, np.uint32)
    offs = np.zeros((T, 2), np.uint32)
    t3 = time.perf_counter()
    db.d_ids.download(ids, T * 4)
    db.d_offs.download(offs, T * 8)
    t4 = time.perf_counter()
    ids2 = np.empty(T, np.uint32)
    offs2 = np.empty((T, 2), np.uint32)
    t5 = time.perf_counter()
    db.d_ids.download(ids2, T * 4)
    db.d_offs.download(offs2, T * 8)
    t6 = time.perf_counter()
    print(f"H2D {1e3 * (t1 - t0):.1f} ms  encode {1e3 * (t2 - t1):.1f} ms  D2H pre-touched "
          f"{1e3 * (t4 - t3):.1f} ms  D2H fresh {1e3 * (t6 - t5):.1f} ms")
