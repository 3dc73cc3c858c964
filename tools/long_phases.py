"""Debug: k_bpe_long's LDS path per word (library built with -DTKZ_LONG_STATS): s_memtime
cycles of the setup and the merge rounds, of the rounds' probe sections, the rounds per
word and the accepted speculative ranks. usage: TKZ_LIB=... python tools/long_phases.py [docs]"""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tokenizer-zig_amd")]
import tkz  # noqa: E402
from tkz import synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
tok = tkz.Tokenizer.from_json(synth.tokenizer_json(6))
data, off = synth.docs(6, n)
db = tkz.DeviceBatch(tok, data, off)
db.run()
db.sync()
o = tkz.lib().tkz_debug_counters_offset(db.total, db.n_docs)
c = np.zeros(12, dtype=np.uint64)
tkz.lib().tkz_memcpy_dtoh(c.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(db.d_ws.ptr + o), 96)
words = max(int(c[5]), 1)
print(f"words {words}: cycles/word setup {c[0] / words:.0f}, rounds {c[1] / words:.0f} "
      f"(probe sections {c[2] / words:.0f}), rounds/word {c[3] / words:.1f}, "
      f"speculative ranks accepted/word {c[4] / words:.1f}, cycles/round {c[1] / max(int(c[3]), 1):.0f}")
