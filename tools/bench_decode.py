"""Batched GPU decode throughput: C1 encoded on the GPU, then the
device-resident CSR ids decoded K times with tkz_decode_batch_device. Prints one JSON
line: tokens/s and output MB/s (ids and outputs resident in HBM)."""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tokenizer-zig_amd")]
import tkz  # noqa: E402
from tkz import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=1)
    ap.add_argument("--docs", type=int, default=1_000_000)
    ap.add_argument("--decoder", default="BPE")
    ap.add_argument("--steps", type=int, default=5)
    args = ap.parse_args()
    cfg = json.loads(synth.tokenizer_json(args.config))
    if args.decoder:
        cfg["decoder"] = {"type": args.decoder}
    tok = tkz.Tokenizer.from_json(json.dumps(cfg))
    data, off = synth.docs(args.config, args.docs)
    db = tkz.DeviceBatch(tok, data, off)
    db.run()
    db.sync()
    n = db.n_docs
    row = np.zeros(n + 1, dtype=np.uint64)
    db.d_row.download(row)
    T = int(row[-1])
    L = tkz.lib()
    bound = int(L.tkz_decode_bound(tok.handle, T))
    wsb = int(L.tkz_decode_workspace_size(tok.handle, n, T))
    d_out = tkz.DeviceBuffer(bound)
    d_off = tkz.DeviceBuffer((n + 1) * 8)
    d_ws = tkz.DeviceBuffer(wsb)

    def step():
        rc = L.tkz_decode_batch_device(tok.handle, db.d_row.ptr, db.d_ids.ptr, n, T, 0, d_out.ptr, bound,
                                       d_off.ptr, d_ws.ptr, wsb, None)
        if rc:
            raise RuntimeError(rc)

    step()
    tok_sync = L.tkz_synchronize
    tok_sync(tok.handle)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    tok_sync(tok.handle)
    dt = (time.perf_counter() - t0) / args.steps
    outoff = np.zeros(n + 1, dtype=np.uint64)
    d_off.download(outoff)
    nbytes = int(outoff[-1])
    print(json.dumps({"metric": "GPU batched decode", "config": args.config, "decoder": args.decoder,
                      "docs": n, "tokens": T, "out_bytes": nbytes, "ms_per_step": round(dt * 1e3, 3),
                      "tokens_per_s": round(T / dt, 1), "out_MB_per_s": round(nbytes / dt / 1e6, 1)}))
    for b in (d_out, d_off, d_ws):
        b.free()
    db.free()


if __name__ == "__main__":
    main()
