"""Diagnostic: why bench.py's host_e2e_region runs at half the D2H rate of
tools/bench_host.py: the tool's loop repeated in one process, with variations.
usage: python tools/host_replica.py"""
import ctypes
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tokenizer-zig_amd")]
import numpy as np  # noqa: E402

import tkz  # noqa: E402
from tkz import synth  # noqa: E402


def tool_loop(tag, close=True, reuse_batch=False, warm=1, tok=None):
    own = tok is None
    tok = tok or tkz.Tokenizer.from_json(synth.tokenizer_json(1))
    data, off = synth.docs(1, 1_000_000)
    lib = tkz.lib()
    b0 = tkz._Batch()

    def once():
        b = b0 if reuse_batch else tkz._Batch()
        t0 = time.perf_counter()
        rc = lib.tkz_encode_batch(tok.handle, data.ctypes.data_as(ctypes.c_void_p),
                                  off.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), 1_000_000, ctypes.byref(b))
        dt = time.perf_counter() - t0
        lib.tkz_batch_free(ctypes.byref(b))
        assert rc == 0
        return dt
    for _ in range(warm):
        once()
    ts = sorted(once() for _ in range(5))
    tkz.profile_enable(tok, True)
    tkz.host_profile_read(tok, reset=True)
    once()
    tl = tkz.host_profile_read(tok, reset=True)
    tkz.profile_enable(tok, False)
    print(tag, "median ms", round(ts[2] * 1e3, 2), "d2h_span", round(tl["d2h_span_ms"], 2),
          "out_pageable", tl["out_pageable"], flush=True)
    if own and close:
        tok.close()
    return tok


tkz.set_device(0)
tool_loop("A first tokenizer")
tool_loop("B second tokenizer (first closed)")
t = tool_loop("C third, kept open", close=False)
tool_loop("D same tokenizer again", tok=t)
tool_loop("E fresh tokenizer, batch struct reused, 2 warm-ups", reuse_batch=True, warm=2)
t.close()
time.sleep(1.0)
tool_loop("F fresh tokenizer 1 s after the previous one closed")
