"""Generates tests/golden/hf_vectors.json — a SECONDARY, third-party cross-check.

The reference (Zig) cannot run in this image. HF `tokenizers` (0.22.2, local wheel,
offline `Tokenizer.from_str`) reproduces the reference's golden ids on ASCII inputs
(SURVEY.md §0.9): for vocabularies whose merges were learned in order (every merge's
parts exist before it), HF's heap BPE and the reference's slow BPE agree; HF's
`WhitespaceSplit` == the reference's Whitespace/WhitespaceSplit; HF's
BertNormalizer/BertPreTokenizer == the reference's on ASCII text without VT/FF.
Only ids are compared (HF offsets are document-absolute).

Run in the build container only (HF is not used on the GPU box):
    python tests/golden/make_hf_vectors.py
The docs and tokenizer.json are regenerated deterministically by libtkzsynth.so; the
fixture stores their sha256 so a generator change is detected instead of silently
passing.
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "tokenizer-zig_amd"))

from tkz import synth  # noqa: E402

N_DOCS = 120
N_DOCS_LONG = 40  # whole-doc pretokens (the Python oracle's O(rounds x n) loop in the CPU test)
FIRST = 777


def main():
    from tokenizers import Tokenizer as HFTokenizer

    out = {"about": __doc__.strip().splitlines()[0], "hf_tokenizers_version": None, "cases": []}
    import tokenizers

    out["hf_tokenizers_version"] = tokenizers.__version__
    # C0, C1, C3 (ASCII), C4 (50k vocab, Zipf lengths), C5 (C1's vocab on words it never
    # saw: the general BPE path), and C2 (mixed UTF-8 + Lowercase) on the docs whose only
    # uppercase letters are ASCII (HF's Lowercase is Unicode-wide, the reference's ASCII-only)
    # (round 5) C6, C8, C9: every doc ONE pretoken under the reference (ByteLevel / Metaspace
    # are not recognised, config.zig:387-402): HF with no pre_tokenizer takes the whole text
    # too -- an independent check of the segmented whole-text path at full vocab sizes,
    # C8 with an unk token for the spaces
    for cfg in (0, 1, 3, 4, 5, 2, 6, 8, 9):
        js = synth.tokenizer_json(cfg)
        d = json.loads(js)
        if d["pre_tokenizer"] and d["pre_tokenizer"]["type"] == "Whitespace":
            d["pre_tokenizer"] = {"type": "WhitespaceSplit"}
        if cfg in (6, 8, 9):
            d["pre_tokenizer"] = None
        d["decoder"] = None  # decode is not compared
        d["post_processor"] = None
        hf = HFTokenizer.from_str(json.dumps(d))
        pool = N_DOCS_LONG if cfg in (6, 8, 9) else N_DOCS * (8 if cfg == 2 else 1)
        data, off = synth.docs(cfg, pool, first_doc=FIRST)
        ids, idx = [], []
        for i in range(pool):
            raw = bytes(data[int(off[i]):int(off[i + 1])])
            text = raw.decode("utf-8")
            if cfg == 2:
                ascii_lower = bytes(b | 0x20 if 65 <= b <= 90 else b for b in raw).decode("utf-8")
                if text.lower() != ascii_lower:
                    continue
            ids.append(hf.encode(text, add_special_tokens=False).ids)
            idx.append(i)
            if len(idx) == min(N_DOCS, pool):
                break
        case = {
            "config": cfg, "first_doc": FIRST, "n_docs": pool,
            "tokenizer_sha256": hashlib.sha256(js).hexdigest(),
            "docs_sha256": hashlib.sha256(bytes(data[: int(off[-1])])).hexdigest(),
            "ids": ids,
        }
        if cfg == 2:
            case["doc_idx"] = idx
        out["cases"].append(case)
    with open(os.path.join(HERE, "hf_vectors.json"), "w") as f:
        json.dump(out, f, separators=(",", ":"))


if __name__ == "__main__":
    main()
