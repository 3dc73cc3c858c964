"""Multi-rank harness of bench.py on CPU (gloo, world_size 2): shard assignment, the
barrier-bracketed timing with max over ranks, and the sum of per-rank work. The per-rank
'step' here is the CPU oracle encoding the rank's shard (no GPU in this container); on
the GPU box bench.py runs the same harness with the HIP path."""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.multiprocessing as mp  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import sys
    from tests.conftest import REPO, PKG  # noqa: F401
    for p in (REPO, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    import bench
    from tkz import synth
    from oracle import oracle as orc

    d = bench.Dist()
    n = 300
    first = bench.shard_first_doc(d.rank, n)
    js = synth.tokenizer_json(1)
    co = orc.COracle(orc.RefTokenizer.from_json(js))
    data, off = synth.docs(1, n, first_doc=first)
    out = {}

    def step():
        out["r"] = co.encode_batch(data, off, n_threads=1)

    el = bench.run_timed(step, lambda: None, d, steps=2, warmup=1)
    tot = d.sum(float(off[-1]))
    q.put((rank, first, el, tot, int(out["r"][0][-1])))
    d.close()


def test_two_rank_gloo_harness():
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    assert [r[1] for r in res] == [0, 300]            # disjoint contiguous doc shards
    assert res[0][2] == res[1][2]                       # max over ranks is shared
    assert res[0][3] == res[1][3] == 2 * 300 * 512      # sum of per-rank bytes
    assert all(r[4] > 0 for r in res)


def test_bench_spawns_ranks():
    """`bench.py --gpus 2` without torchrun: the parent spawns two rank processes (it never
    imports tkz), they run the gloo harness (here with the CPU oracle as the step) and rank
    0's single JSON line reports both shards."""
    import json
    import subprocess
    import sys

    from tests.conftest import REPO

    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--simulate-cpu",
                        "--docs", "300", "--steps", "2", "--warmup", "1"],
                       capture_output=True, text=True, timeout=600, env={k: v for k, v in os.environ.items()
                                                                         if k not in ("WORLD_SIZE", "RANK")})
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2
    assert out["config"]["bytes_all"] == 2 * 300 * 512
    assert out["config"]["shard_first_docs"] == [0, 300]
    assert out["config"]["parallelism"] == "doc-shard x2"


def test_bench_rank_failure_propagates():
    """A failing rank makes the parent exit non-zero (here: an invalid config on every rank)."""
    import subprocess
    import sys

    from tests.conftest import REPO

    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--simulate-cpu",
                        "--config", "99", "--docs", "10"], capture_output=True, text=True, timeout=300,
                       env={k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK")})
    assert r.returncode != 0
    assert not [x for x in r.stdout.splitlines() if x.startswith("{")]
