"""Builds tests/golden/c4_stream_64M.json: rolling hashes (tests/shard_hash.py) of the C++
oracle's encoding of the whole C4 stream at its BASELINE size: 64M Zipf(64-4096 B) docs,
50k BPE, as 8 shards of 8M docs (one GPU's share each, 64M docs over 8 GPUs). Per shard:
the hashes of its own CSR (row_ptr from 0); for the stream: the hashes continued across
the shards in doc order, i.e. of the concatenated batch. Run in the build container (about
3 minutes per shard on 8 cores); tests/test_gpu_subbatch.py::test_c4_stream_64M compares
the device results against it. The synthetic stream is deterministic
(tokenizer-zig_amd/csrc/synth.cpp).

usage: python tests/golden/make_c4_stream_hash.py [threads]
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

SHARDS, PER = 8, 8_000_000


def main():
    th = int(sys.argv[1]) if len(sys.argv) > 1 else (os.cpu_count() or 1)
    js = synth.tokenizer_json(4)
    co = orc.COracle(orc.RefTokenizer.from_json(js))
    whole = CsrHash()
    shards = []
    blk = 250_000
    t0 = time.time()
    total = 0
    for s in range(SHARDS):
        h = CsrHash()
        nbytes = 0
        for d0 in range(s * PER, (s + 1) * PER, blk):
            data, off = synth.docs(4, blk, first_doc=d0, threads=th)
            row, ids, offs = co.encode_batch(data, off, n_threads=th)
            h.add(row, ids, offs)
            whole.add(row, ids, offs)
            nbytes += int(off[-1])
        total += nbytes
        shards.append(dict(h.result(), first_doc=s * PER, bytes=nbytes))
        print(f"shard {s}: {shards[-1]}  ({time.time() - t0:.0f} s)", flush=True)
    res = {"config": 4, "n_docs": SHARDS * PER, "shards": shards, "stream": dict(whole.result(), bytes=total),
           "source": "oracle/tkz_oracle.cpp (C++ restatement of Tokenizer.encode), tests/golden/make_c4_stream_hash.py"}
    with open(os.path.join(HERE, "c4_stream_64M.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res["stream"]))


if __name__ == "__main__":
    main()
