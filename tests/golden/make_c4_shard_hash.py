"""Builds tests/golden/c4_shard_8M.json: rolling hashes (tests/shard_hash.py) of the C++
oracle's encoding of one GPU's C4 shard at its BASELINE size, docs [0, 8M) of the 64M-doc
Zipf(64-4096 B) stream (64M docs over 8 GPUs), 50k BPE. Run in the build container
(about 3 minutes on 8 cores); the GPU test compares the device result of the whole
shard against it. The synthetic stream is deterministic (tokenizer-zig_amd/csrc/synth.cpp).

usage: python tests/golden/make_c4_shard_hash.py [n_docs] [threads]
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
for p in (REPO, os.path.join(REPO, "tokenizer-zig_amd"), os.path.join(REPO, "tests")):
    sys.path.insert(0, p)

from oracle import oracle as orc  # noqa: E402
from shard_hash import CsrHash  # noqa: E402
from tkz import synth  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8_000_000
    th = int(sys.argv[2]) if len(sys.argv) > 2 else (os.cpu_count() or 1)
    js = synth.tokenizer_json(4)
    co = orc.COracle(orc.RefTokenizer.from_json(js))
    h = CsrHash()
    blk = 250_000
    t0 = time.time()
    total = 0
    for d0 in range(0, n, blk):
        m = min(blk, n - d0)
        data, off = synth.docs(4, m, first_doc=d0, threads=th)
        row, ids, offs = co.encode_batch(data, off, n_threads=th)
        h.add(row, ids, offs)
        total += int(off[-1])
        print(f"{d0 + m} docs, {total / 1e9:.2f} GB, {h.n_tokens} tokens, {time.time() - t0:.0f} s", flush=True)
    res = dict(h.result(), config=4, first_doc=0, bytes=total,
               source="oracle/tkz_oracle.cpp (C++ restatement of Tokenizer.encode), tests/golden/make_c4_shard_hash.py")
    out = os.path.join(HERE, f"c4_shard_{n // 1_000_000}M.json" if n % 1_000_000 == 0 else f"c4_shard_{n}.json")
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
