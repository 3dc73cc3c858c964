"""Debug: k_encode cycles per phase (library built with -DTKZ_PHASES), C1 workload.

Phases: deferred-list flush, bucket run (model), dispatch (state reads / word memo /
enqueue), scan step (load + doc bounds / classify + ring / tail), batch-end closure,
next chunk."""
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
ph = np.zeros(10, dtype=np.uint64)
tkz.lib().tkz_memcpy_dtoh(ph.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(db.d_ws.ptr + o), 80)
names_blk = ["chunk loads", "barriers", "classes+stage", "starts/ends+scan", "scatter+doc_word", "open word",
             "words", "tail", "-", "-"]
names = names_blk if os.environ.get("TKZ_BLK_PHASES") else ["defer_flush", "bucket_run", "dispatch:enqueue", "scan:tail", "close", "next_chunk",
         "dispatch:state", "dispatch:memo", "scan:load+bounds", "scan:classify+ring"]
tot = float(ph[:10].sum())
for n, v in zip(names, ph[:10]):
    print(f"{n:14s} {int(v):16d}  {100 * v / tot:5.1f} %")
