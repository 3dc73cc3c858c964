"""Debug: the segmented path's list sizes per iteration (library built with -DTKZ_SEG_STATS,
TKZ_LIB=<that .so>): segments, pending groups of iterations 0-3, crossed boundaries
listed for joining in 0-2, groups of > 16 symbols in 0-2, wave-path groups in 1.
usage: TKZ_LIB=... python tools/seg_stats.py [cfg ...] (default 6 11)"""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tokenizer-zig_amd")]
import tkz  # noqa: E402
from tkz import synth  # noqa: E402

names = ["segments", "pend0", "pend1", "pend2", "pend3", "join0", "join1", "join2", "big0", "big1", "big2", "wave1"]
for cfg in [int(a) for a in sys.argv[1:]] or [6, 11]:
    tok = tkz.Tokenizer.from_json(synth.tokenizer_json(cfg))
    data, off = synth.docs(cfg, 1_000_000)
    db = tkz.DeviceBatch(tok, data, off)
    db.run()
    db.sync()
    o = tkz.lib().tkz_debug_counters_offset(db.total, db.n_docs)
    v = np.zeros(12, dtype=np.uint64)
    tkz.lib().tkz_memcpy_dtoh(v.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(db.d_ws.ptr + o), 96)
    print(f"C{cfg}", " ".join(f"{n}={int(x)}" for n, x in zip(names, v)), flush=True)
    db.free()
    tok.close()
