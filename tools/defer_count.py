"""Debug: deferred-list counts (short <= 8 B, long) after one encode of a bench config."""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tokenizer-zig_amd")]
import tkz  # noqa: E402
from tkz import synth  # noqa: E402

for cfg in [int(a) for a in sys.argv[1:]] or [1]:
    tok = tkz.Tokenizer.from_json(synth.tokenizer_json(cfg))
    data, off = synth.docs(cfg, 1_000_000)
    db = tkz.DeviceBatch(tok, data, off)
    db.run()
    db.sync()
    o = tkz.lib().tkz_debug_counters_offset(db.total, db.n_docs)
    c = np.zeros(2, dtype=np.uint32)
    tkz.lib().tkz_memcpy_dtoh(c.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(db.d_ws.ptr + o + 8), 8)
    print(f"C{cfg}: bytes {db.total} deferred short {c[0]} long {c[1]}")
