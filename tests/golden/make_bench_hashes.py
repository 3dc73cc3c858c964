"""Builds tests/golden/bench_shards.json: rolling hashes (tests/shard_hash.py) of the C++
oracle's encoding of every bench shard bench.py can time, so the driver's own bench run
verifies its result in full (verdict r2 item 1a). Shard r of config c = docs
[r * n, (r + 1) * n) of the config's deterministic stream (tokenizer-zig_amd/csrc/synth.cpp),
n = 1M docs (C10: 2,700 docs of 4 KB - 1 MB, about 0.5 GB), ranks 0..7 (the 8-GPU node).
C4's 8M-doc shards are in c4_stream_64M.json. C10's whole-doc pretokens of up to 1 MB run the
oracle's heap form of the merge loop (tkz_oracle.cpp bpe_tokenize_heap, equal to the literal
loop on its ordered merge table: tests/test_oracle_heap.py); the literal loop would take
hours per shard.
Run in the build container (C6, one pretoken per doc, is the slow one: ~2 min per shard
on 8 cores).

usage: python tests/golden/make_bench_hashes.py [configs (comma list)] [ranks] [threads]
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

SHARD_DOCS = 1_000_000
SHARD_DOCS_BY_CONFIG = {10: 2_700}
HEAP_BYTES = {10: 4096}  # pretokens of >= this many bytes: the heap form
OUT = os.path.join(HERE, "bench_shards.json")


def shard_hash(co, cfg, rank, n, th):
    h = CsrHash()
    blk = 125_000 if n >= 125_000 else 300
    total = 0
    for d0 in range(0, n, blk):
        m = min(blk, n - d0)
        data, off = synth.docs(cfg, m, first_doc=rank * n + d0, threads=th)
        row, ids, offs = co.encode_batch(data, off, n_threads=th)
        h.add(row, ids, offs)
        total += int(off[-1])
    return dict(h.result(), bytes=total, first_doc=rank * n)


def main():
    cfgs = [int(c) for c in (sys.argv[1] if len(sys.argv) > 1 else "1,2,3,5,6").split(",")]
    ranks = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    th = int(sys.argv[3]) if len(sys.argv) > 3 else (os.cpu_count() or 1)
    res = json.load(open(OUT)) if os.path.exists(OUT) else {
        "shard_docs": SHARD_DOCS, "configs": {},
        "source": "oracle/tkz_oracle.cpp (C++ restatement of Tokenizer.encode), tests/golden/make_bench_hashes.py"}
    for cfg in cfgs:
        co = orc.COracle(orc.RefTokenizer.from_json(synth.tokenizer_json(cfg)))
        if cfg in HEAP_BYTES:
            assert co.set_heap(HEAP_BYTES[cfg])
        n = SHARD_DOCS_BY_CONFIG.get(cfg, SHARD_DOCS)
        if n != SHARD_DOCS:
            res.setdefault("shard_docs_by_config", {})[str(cfg)] = n
        out = res["configs"].setdefault(str(cfg), [])
        for r in range(len(out), ranks):
            t0 = time.time()
            out.append(shard_hash(co, cfg, r, n, th))
            print(f"C{cfg} rank {r}: {out[-1]['n_tokens']} tokens, {time.time() - t0:.0f} s", flush=True)
            with open(OUT, "w") as f:  # progress survives an interruption
                json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
