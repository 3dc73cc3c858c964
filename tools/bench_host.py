"""Host-buffer encode rate (PCIe-inclusive, not the bench metric): tkz_encode_batch on C1
(1M x 512-B docs) from pageable host memory, output CSR back in host memory.

usage: python tools/bench_host.py [config] [docs] [chunk_bytes (tkz_set_host_pipeline; default: the
library's 32 MiB, 0 = unchunked)]; TKZ_SET_DEVICE=<i>: tkz.set_device(i) first (as bench.py)"""
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

if os.environ.get("TKZ_SET_DEVICE"):
    tkz.set_device(int(os.environ["TKZ_SET_DEVICE"]))
cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 1
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
chunk = int(sys.argv[3]) if len(sys.argv) > 3 else None
tok = tkz.Tokenizer.from_json(synth.tokenizer_json(cfg))
if chunk is not None:
    tok.set_host_pipeline(chunk)
data, off = synth.docs(cfg, n)
data = np.ascontiguousarray(data, dtype=np.uint8)
off = np.ascontiguousarray(off, dtype=np.uint64)
lib = tkz.lib()


def once():
    b = tkz._Batch()
    t0 = time.perf_counter()
    rc = lib.tkz_encode_batch(tok.handle, data.ctypes.data_as(ctypes.c_void_p),
                              off.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), n, ctypes.byref(b))
    dt = time.perf_counter() - t0
    T = int(b.n_tokens)
    lib.tkz_batch_free(ctypes.byref(b))
    assert rc == 0
    return dt, T


once()
times = []
for _ in range(5):
    dt, T = once()
    times.append(dt)
total = int(off[-1])
med = sorted(times)[2]
tkz.profile_enable(tok, True)  # one more call with the library's timeline
tkz.host_profile_read(tok, reset=True)
once()
tl = {k: round(v, 3) for k, v in tkz.host_profile_read(tok, reset=True).items()}
tkz.profile_enable(tok, False)
print(json.dumps({"workload": f"C{cfg} {n} docs", "chunk_bytes": 32 << 20 if chunk is None else chunk, "bytes": total, "tokens": T, "s_median": round(med, 4),
                  "input_MB_per_s_pcie_inclusive": round(total / med / 1e6, 1),
                  "output_bytes": 12 * T + 8 * (n + 1), "timeline": tl}))
