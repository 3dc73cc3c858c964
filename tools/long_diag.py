"""Diagnostic: C1 docs under ByteLevel (tests/test_gpu_long.py's first case) through the
segmented path, memo on / off, against the oracle; prints the first differing docs.
usage: python tools/long_diag.py"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tokenizer-zig_amd")]
import tkz  # noqa: E402
from tkz import synth  # noqa: E402
from oracle import oracle as orc  # noqa: E402

j = json.loads(synth.tokenizer_json(1))
j["pre_tokenizer"] = {"type": "ByteLevel", "add_prefix_space": False}
js = json.dumps(j)
data, off = synth.docs(1, 4000, first_doc=12_345)
erow, eids, eoffs = orc.COracle(orc.RefTokenizer.from_json(js)).encode_batch(data, off, n_threads=16)
for seg, memo in ((True, True), (True, False), (False, True)):
    tok = tkz.Tokenizer.from_json(js)
    tok.set_long_segments(seg)
    tok.set_word_memo(memo)
    row, ids, offs = tok.encode_batch(data, off)
    cnt = np.diff(row.astype(np.int64)) - np.diff(erow.astype(np.int64))
    bad = np.nonzero(cnt)[0]
    print(f"seg {seg} memo {memo}: docs with another token count {len(bad)}, extra tokens {int(cnt.sum())}", flush=True)
    for i in bad[:3]:
        d = bytes(data[int(off[i]):int(off[i + 1])])
        g = ids[int(row[i]):int(row[i + 1])].tolist()
        e = eids[int(erow[i]):int(erow[i + 1])].tolist()
        go = offs[int(row[i]):int(row[i + 1])].tolist()
        k = next((x for x in range(min(len(g), len(e))) if g[x] != e[x]), min(len(g), len(e)))
        a = int(go[k][0]) if k < len(go) else 0
        print(f"  doc {i}: first difference at token {k}, byte {a}: {d[max(0, a - 30):a + 30]!r}")
        print("   exp", e[max(0, k - 3):k + 6], "\n   got", g[max(0, k - 3):k + 6])
    tok.close()
