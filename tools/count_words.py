"""Debug: words dispatched / processed per stage (library built with -DTKZ_COUNT_WORDS)
vs the number of pretokens counted on the host, for C1."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tokenizer-zig_amd")]
import tkz  # noqa: E402
from tkz import synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
tok = tkz.Tokenizer.from_json(synth.tokenizer_json(1))
data, off = synth.docs(1, n)
db = tkz.DeviceBatch(tok, data, off)
db.run()  # first call builds the word memo (its own launches count too)
db.sync()
db.d_status.zero()
db.run()
db.sync()
st = np.zeros(4, dtype=np.uint32)
db.d_status.download(st)
d = data[: int(off[-1])].reshape(n, 512)
ws = (d == 32) | (d == 9) | (d == 10) | (d == 13)
starts = (~ws) & np.concatenate([np.ones((n, 1), bool), ws[:, :-1]], axis=1)
print("host words", int(starts.sum()), "dispatched", int(st[1]), "dispatch batches", int(st[2]),
      "steps", int(off[-1]) // 512)
