"""Diagnostic: the random configs of test_gpu_fast.test_random_configs_caps through the
plain batch encode (DeviceBatch), segmented path and memo on / off, against the oracle;
prints the docs that differ. usage: python tools/fast_diag.py [pretok] [model] [seg memo modes, e.g. 11,10,01]"""
import json
import os
import random
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tokenizer-zig_amd"), os.path.join(REPO, "tests")]
import tkz  # noqa: E402
from oracle import oracle as orc  # noqa: E402
from test_gpu_parity import _batch, _rand_cfg, _rand_text  # noqa: E402

pretok = None if len(sys.argv) < 2 or sys.argv[1] == "None" else sys.argv[1]
model = sys.argv[2] if len(sys.argv) > 2 else "BPE"
modes = ((True, True), (True, False), (False, True)) if len(sys.argv) < 4 else \
    tuple((m[0] == "1", m[1] == "1") for m in sys.argv[3].split(","))  # e.g. 11,10
rng = random.Random(f"fast-{model}-{pretok}")
for trial in range(4):
    cfg = _rand_cfg(rng, model, pretok, rng.choice([None, "Lowercase"]))
    lens = [0, 1, 2, 7, 40, 63, 64, 65, 200, 513, 1100, 3000] + [rng.randint(0, 300) for _ in range(40)]
    docs = [_rand_text(rng, n) for n in lens]
    js = json.dumps(cfg)
    ref = orc.RefTokenizer.from_json(js)
    data, off = _batch(docs)
    data = np.frombuffer(data, dtype=np.uint8)
    for seg, memo in modes:
        tok = tkz.Tokenizer.from_json(js)
        tok.set_long_segments(seg)
        tok.set_word_memo(memo)
        db = tkz.DeviceBatch(tok, data, off)
        db.run()
        row, ids, offs = db.results()
        st = db.stats()
        bad = []
        for i, d in enumerate(docs):
            exp = ref.encode(d)
            got = ids[int(row[i]):int(row[i + 1])].tolist()
            if got != [t[0] for t in exp]:
                bad.append(i)
        print(f"trial {trial} seg {seg} memo {memo} unk {cfg['model'].get('unk_token')} norm {cfg.get('normalizer')}"
              f" segmented {st['long_segmented']} long {st['long_words']} bad {bad}", flush=True)
        for i in bad[:2]:
            exp = ref.encode(docs[i])
            got = ids[int(row[i]):int(row[i + 1])].tolist()
            print("  doc", i, docs[i][:120], "\n   exp", [t[0] for t in exp][:60], "\n   got", got[:60], len(got), len(exp))
        db.free()
        tok.close()
