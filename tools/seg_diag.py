"""Diagnostic run of the segmented long-pretoken path (k_seg_* kernels), off and on
(tkz_set_long_segments): saves each mode's CSR result of a test_segments.py case for
offline comparison with tests/segment_model.py. usage: python tools/seg_diag.py [cases]"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tokenizer-zig_amd")]
import tkz  # noqa: E402
from tests.test_segments import CASES, random_bpe_json, random_docs  # noqa: E402

out = os.path.join(REPO, "gpurun_out", "segdiag")
os.makedirs(out, exist_ok=True)
for ci in (int(a) for a in (sys.argv[1:] or ["0"])):
    case = CASES[ci]
    js = random_bpe_json(**case, pretok={"type": "ByteLevel"})
    docs = random_docs(case["seed"] + 200, 400, alphabet=case.get("alphabet", "abcde"),
                       extra=case.get("extra", ()) + (("ü",) if case.get("extra") else ()))
    off = np.zeros(len(docs) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(d) for d in docs])
    data = np.frombuffer(b"".join(docs) + bytes(16), dtype=np.uint8).copy()
    for mode in (0, 1):
        tok = tkz.Tokenizer.from_json(js)
        tok.set_long_segments(mode)
        db = tkz.DeviceBatch(tok, data, off)
        db.run()
        row, ids, offs = db.results()
        st = db.stats()
        np.savez(os.path.join(out, f"case{ci}_mode{mode}.npz"), row=row, ids=ids, offs=offs,
                 seg=st["long_segmented"], long=st["long_words"])
        print(ci, mode, int(row[-1]), st["long_segmented"], st["long_words"], flush=True)
        db.free()
        tok.close()
