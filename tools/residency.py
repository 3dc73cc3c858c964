"""Debug: max co-resident k_encode waves (library built with -DTKZ_RESIDENCY) on C1."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tokenizer-zig_amd")]
import tkz  # noqa: E402
from tkz import synth  # noqa: E402

tok = tkz.Tokenizer.from_json(synth.tokenizer_json(1))
data, off = synth.docs(1, 200000)
db = tkz.DeviceBatch(tok, data, off)
db.run()
db.sync()
db.d_status.zero()
db.run()
db.sync()
st = np.zeros(4, dtype=np.uint32)
db.d_status.download(st)
print(os.environ.get("TKZ_LIB"), "max resident waves", int(st[2]))
