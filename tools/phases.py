"""Debug: k_encode cycles per phase (library built with -DTKZ_PHASES), C1 workload.

Phases: 0 deferred-list flush, 1 bucket run (model), 2 dispatch (+ word memo),
3 scan step, 4 batch-end closure, 5 next chunk."""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tokenizer-zig_amd")]
import tkz  # noqa: E402
from tkz import synth  # noqa: E402

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 1
tok = tkz.Tokenizer.from_json(synth.tokenizer_json(cfg))
data, off = synth.docs(cfg, 1_000_000 if cfg else 1000)
db = tkz.DeviceBatch(tok, data, off)
db.run()
db.sync()
o = tkz.lib().tkz_debug_counters_offset(db.total, db.n_docs)
ph = np.zeros(8, dtype=np.uint64)
tkz.lib().tkz_memcpy_dtoh(ph.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(db.d_ws.ptr + o + 32), 64)
names = ["defer_flush", "bucket_run", "dispatch_memo", "scan", "close", "next_chunk"]
tot = float(ph[:6].sum())
for n, v in zip(names, ph[:6]):
    print(f"{n:14s} {int(v):16d}  {100 * v / tot:5.1f} %")
