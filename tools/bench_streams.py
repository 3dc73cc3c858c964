"""Experiment: N independent device batches in flight on N HIP streams (each a full
encode pass of its own workspace/outputs), against the same batches run back to back on
one stream. Prints GB/s of input for both. usage: python tools/bench_streams.py [cfg] [nstreams] [steps]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tokenizer-zig_amd")]
import torch  # noqa: E402

import tkz  # noqa: E402
from tkz import synth  # noqa: E402


def main():
    cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    ns = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    tkz.set_device(0)
    js = synth.tokenizer_json(cfg)
    tok = tkz.Tokenizer.from_json(js)
    data, off = synth.docs(cfg, 1_000_000, first_doc=0)
    total = int(off[-1])
    dbs = [tkz.DeviceBatch(tok, data, off) for _ in range(ns)]
    streams = [torch.cuda.Stream() for _ in range(ns)]
    L = tkz.lib()

    def launch(i, st):
        db = dbs[i]
        rc = L.tkz_encode_batch_device(tok.handle, db.d_bytes.ptr, db.d_off.ptr, db.n_docs, db.total, db.d_row.ptr,
                                       db.d_ids.ptr, db.d_offs.ptr, db.d_ws.ptr, db.ws_bytes, db.d_status.ptr,
                                       st)
        assert rc == 0

    for mode in ("serial", "streams", "serial", "streams"):
        for i in range(ns):  # warm-up
            launch(i, streams[i].cuda_stream)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(steps):
            i = k % ns
            launch(i, streams[i].cuda_stream if mode == "streams" else streams[0].cuda_stream)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(f"C{cfg} {mode:8s} x{ns}: {total * steps / dt / 1e9:.1f} GB/s  {dt / steps * 1e3:.3f} ms/batch", flush=True)
    ref = dbs[0].results()
    for db in dbs[1:]:
        r = db.results()
        assert all((a == b).all() for a, b in zip(ref, r)), "stream results differ"
    print("results identical across streams")


if __name__ == "__main__":
    main()
