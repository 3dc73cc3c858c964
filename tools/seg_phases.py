"""Debug: the segmented long-pretoken path per doc (library built with -DTKZ_SEG_STATS):
s_memtime cycles of its phases (segments, lane-per-group encodes, whole-wave groups,
boundary checks, joins, output), iterations, passes and whole-wave groups per doc.
usage: TKZ_LIB=... python tools/seg_phases.py [docs]"""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tokenizer-zig_amd")]
import tkz  # noqa: E402
from tkz import synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 200000
tok = tkz.Tokenizer.from_json(synth.tokenizer_json(6))
dd = synth.DeviceDocs(6, n)
db = tkz.DeviceBatch.from_device(tok, dd.d_bytes, dd.d_off, dd.n_docs, dd.total, owner=dd)
for _ in range(2):
    db.run()
db.sync()
o = tkz.lib().tkz_debug_counters_offset(db.total, db.n_docs)
c = np.zeros(12, dtype=np.uint64)
tkz.lib().tkz_memcpy_dtoh(c.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(db.d_ws.ptr + o), 96)
docs = max(int(c[10]), 1)
names = ["segments", "lane encodes", "wave groups", "checks", "joins", "output"]
tot = sum(int(c[k]) for k in range(6))
print(f"docs {docs} (of {n}), segments/doc {c[11] / docs:.1f}, cycles/doc {tot / docs:.0f}")
for k, nm in enumerate(names):
    print(f"  {nm:13s} {c[k] / docs:9.0f} cycles/doc ({c[k] / max(tot, 1):.1%})")
print(f"  iterations/doc {c[6] / docs:.2f}, lane passes/doc {c[8] / docs:.2f}, whole-wave groups/doc {c[7] / docs:.2f}, "
      f"check passes/doc {c[9] / docs:.2f}")
