"""Secondary cross-check against third-party HF `tokenizers` ids (fixtures generated
in the build container by tests/golden/make_hf_vectors.py; HF itself is not imported
here). The oracle must match them on CPU; the HIP path must match them on the GPU."""
import hashlib
import json
import os

import numpy as np
import pytest

import tkz
from tkz import synth
from oracle import oracle as orc
from tests.conftest import GOLDEN


def _cases():
    with open(os.path.join(GOLDEN, "hf_vectors.json")) as f:
        return json.load(f)["cases"]


def _inputs(case):
    js = synth.tokenizer_json(case["config"])
    assert hashlib.sha256(js).hexdigest() == case["tokenizer_sha256"], "tokenizer generator changed: regenerate fixture"
    data, off = synth.docs(case["config"], case["n_docs"], first_doc=case["first_doc"])
    assert hashlib.sha256(bytes(data[: int(off[-1])])).hexdigest() == case["docs_sha256"], "doc generator changed"
    return js, data, off


N_CASES = 9  # configs 0, 1, 3, 4, 5, 2, 6, 8, 9 (make_hf_vectors.py; 6, 8, 9: one pretoken per doc)


def _docs_of(case):
    return case.get("doc_idx", range(len(case["ids"])))


@pytest.mark.parametrize("idx", range(N_CASES))
def test_oracle_matches_hf(idx):
    case = _cases()[idx]
    js, data, off = _inputs(case)
    ref = orc.RefTokenizer.from_json(js)
    for i, exp in zip(_docs_of(case), case["ids"]):
        got = [t[0] for t in ref.encode(bytes(data[int(off[i]):int(off[i + 1])]))]
        assert got == exp, (case["config"], i)


@pytest.mark.gpu
@pytest.mark.parametrize("idx", range(N_CASES))
def test_gpu_matches_hf(idx):
    case = _cases()[idx]
    js, data, off = _inputs(case)
    tok = tkz.Tokenizer.from_json(js)
    row, ids, _ = tok.encode_batch(data, off)
    for i, exp in zip(_docs_of(case), case["ids"]):
        assert ids[int(row[i]):int(row[i + 1])].tolist() == exp, (case["config"], i)
