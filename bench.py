"""Encode throughput bench (BASELINE.json metric: input MB/s, bit-exact ids).

One step = one pass of the encode hot path (normalize -> pretokenize -> BPE/WordPiece
-> vocab lookup -> CSR ids/offsets) over one batch of synthetic docs already resident
in HBM. Default workload: C1 (configs[1]) = 1M x 512-B ASCII docs, 32k BPE, Whitespace.
The docs are generated in HBM by the device port of the deterministic generator
(tokenizer-zig_amd/csrc/gen.hip, byte-identical to synth.cpp): a rank stages nothing on
the host.

Every region is verified in the same run (verdict r2 item 1a): the rolling hashes of
the whole device result (row_ptr, ids, offsets; computed on the device) against the C++
oracle's hashes of the same shard committed under tests/golden/, plus a doc-by-doc
comparison of a bounded sample with the oracle run here. Any mismatch on any rank makes
the run exit non-zero.

N GPUs (`--gpus N`): one process per GPU, each encoding its own contiguous doc shard of
the synthetic stream (weak scaling; docs are independent, `Tokenizer.encode` reads only
immutable tables, /root/reference/src/lib.zig:109-160, so there is no data-path
collective). Started by torchrun (WORLD_SIZE set) or, without it, by this script: the
parent spawns N fresh child processes before anything touches HIP, relays rank 0's JSON
line and exits non-zero if any rank fails. A gloo barrier brackets each timed region and
the max time over ranks is reported. rank 0 prints one JSON line: the C1 value with its
roofline (algorithmic bytes of the step / step time, HIP events on the
encode stream), the memo-off and two-stream rates, the secondary regions (C2, C3, C5,
C6 at 1M docs per rank, C4 at its BASELINE per-GPU shard of 8M docs), and `cpu_baseline`
(the C++ restatement of the reference's CPU algorithm on a bounded sample; N=1 only).
"""
import argparse
import ctypes
import hashlib
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
for p in (REPO, os.path.join(REPO, "tokenizer-zig_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
HBM_COPY_GBS = 6300.0  # measured copy bandwidth (same guide, HBM section)
N_SIMDS = 256 * 4  # 256 CUs x 4 SIMDs
VALU_PEAK_FAST, VALU_PEAK_SLOW = 0.90, 0.55  # wave64 VALU instructions per SIMD per ns (tools/valu_mix.hip)
METRIC = "input MB/s encode (bit-exact ids) at 1/2/4/8 MI355X vs Zig CPU baseline"
WORKLOADS = {
    0: "C0: 1k x 256-B ASCII docs, 8k BPE, Whitespace",
    1: "C1: 1M x 512-B ASCII docs, 32k BPE, Whitespace",
    2: "C2: 1M x 512-B mixed-UTF-8 docs, 32k BPE, Lowercase, Whitespace",
    3: "C3: 1M x 512-B docs, 30k WordPiece, BertNormalizer + BertPreTokenizer",
    4: "C4 shard: Zipf(64-4096 B) docs, 50k BPE, Whitespace",
    5: "C1-disjoint: 1M x 512-B ASCII docs from a lexicon disjoint from the vocab's, C1's 32k BPE, Whitespace",
    6: "C1-bytelevel: C1's docs and 32k BPE under a ByteLevel pre_tokenizer (one pretoken per doc, config.zig:387-402)",
    7: "C1-wide: C1's docs under a 106,608-id BPE vocab with 106,545 merges (ids and ranks past 16 bits), Whitespace",
    8: "C1-metaspace-unk: C1's docs, C1's 32k BPE + an unk token, Metaspace (one pretoken per doc; spaces are the "
       "unk symbol, bpe.zig:198-205)",
    9: "C7-bytelevel: C1's docs under C7's 106,608-id BPE, ByteLevel (one pretoken per doc, wide ids)",
    10: "C10: C1's text in Zipf(4 KB - 1 MB) docs, C1's 32k BPE under ByteLevel (whole-doc pretokens of up to 1 MB)",
    11: "C5-bytelevel: C5's docs (a lexicon disjoint from the vocab's) under C6's ByteLevel tokenizer (one pretoken "
        "per doc)",
}
# secondary regions of the default run: (config, docs per rank); C4 at its BASELINE
# 8-GPU config's per-GPU share (64M docs / 8)
SECONDARY = [(2, 1_000_000), (3, 1_000_000), (5, 1_000_000), (4, 8_000_000), (6, 1_000_000), (7, 1_000_000),
             (8, 1_000_000), (9, 1_000_000), (10, 2_700), (11, 1_000_000)]
LONG_CFGS = (6, 8, 9, 10, 11)  # one pretoken per doc (smaller oracle samples: O(rounds x n) per doc on the CPU)
# configs whose oracle check runs the heap form of the merge loop on pretokens of >= this many
# bytes (oracle/tkz_oracle.cpp bpe_tokenize_heap; the literal loop takes minutes per 1-MB doc)
HEAP_CFGS = {10: 4096}
# kernels of one encode step (PMC step sums)
STEP_KERNELS = ("k_chunk_docs", "k_encode", "k_encode_blk", "k_bpe_short", "k_dedup", "k_bpe_deferred", "k_bpe_long", "k_dedup_copy",
                "k_scan_partials", "k_scan_top", "k_scan_final", "k_compact", "k_compact_long",
                "__amd_rocclr_fillBufferAligned")
# files that determine the encode kernels' binaries (PMC summaries are stamped with their hash)
KERNEL_SOURCES = ["tokenizer-zig_amd/csrc/encode.hip", "tokenizer-zig_amd/csrc/encode.hpp",
                  "tokenizer-zig_amd/csrc/tables.hpp", "tokenizer-zig_amd/Makefile"]
GOLDEN = os.path.join(REPO, "tests", "golden")


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", type=int, default=1,
                    help="0..4 = BASELINE.json configs, 5 = C1 on a disjoint lexicon, 6 = C1 under ByteLevel, "
                         "7 = C1 under a 106k-id vocab, 8 = C1 + unk under Metaspace, 9 = C7 under ByteLevel")
    ap.add_argument("--docs", type=int, default=0, help="docs per rank (default: the config's size)")
    ap.add_argument("--max-workspace-gb", type=float, default=0.0,
                    help="cap on every region's encode workspace (sub-batched above it); 0 = one pass when it fits")
    ap.add_argument("--cpu-sample-docs", type=int, default=200_000)
    ap.add_argument("--cpu-min-seconds", type=float, default=8.0, help="repeat the all-threads sample until this long")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-memo-off-run", action="store_true", help="skip the memo-off timed region")
    ap.add_argument("--no-pipelined-run", action="store_true", help="skip the two-stream timed region")
    ap.add_argument("--primary-only", action="store_true", help="skip the secondary regions (PMC passes)")
    ap.add_argument("--secondary", default="",
                    help="secondary regions as cfg:docs[,cfg:docs...] or none (default: C2, C3, C5, C6-C9 at 1M, C4 at 8M)")
    ap.add_argument("--secondary-steps", type=int, default=3)
    ap.add_argument("--host-e2e-first", action="store_true",
                    help="diagnostic: run the host-buffer region before the others")
    ap.add_argument("--no-host-e2e", action="store_true",
                    help="skip the host-buffer region (tkz_encode_batch, PCIe copies included)")
    ap.add_argument("--no-single-doc", action="store_true",
                    help="skip the single-doc latency region (tkz_encode, the reference's call shape)")
    ap.add_argument("--no-decode-pad", action="store_true",
                    help="skip the device decode and truncate/pad regions over the primary result")
    ap.add_argument("--streams", type=int, default=1,
                    help="batches in flight: step k runs batch k %% S on HIP stream k %% S (each batch its own "
                         "workspace and outputs over the same resident input); 0 = 2 when two one-pass batches "
                         "fit in free HBM, else 1")
    ap.add_argument("--verify", action="store_true", help="(default; kept for older command lines)")
    ap.add_argument("--no-verify", action="store_true", help="skip the oracle sample and the hash check")
    ap.add_argument("--verify-docs", type=int, default=100_000, help="oracle sample of the primary region")
    ap.add_argument("--no-memo", action="store_true", help="disable the BPE word memo (vocab-key results)")
    ap.add_argument("--no-long-segments", action="store_true",
                    help="disable the segmented path of long BPE pretokens (k_seg_* kernels; same results)")
    ap.add_argument("--host-inputs", action="store_true",
                    help="generate the docs on the host and upload them (default: on the device)")
    ap.add_argument("--share-gpu", action="store_true",
                    help="rehearsal only: every rank uses GPU 0 (multi-rank path on a 1-GPU box)")
    ap.add_argument("--simulate-cpu", action="store_true",
                    help="test only: each rank runs the C++ oracle as its step (no GPU; the multi-rank harness on CPU)")
    return ap.parse_args(argv)


def default_docs(cfg):
    return {0: 1000, 1: 1_000_000, 2: 1_000_000, 3: 1_000_000, 4: 1_000_000, 5: 1_000_000, 6: 1_000_000,
            7: 1_000_000, 8: 1_000_000, 9: 1_000_000, 10: 2_700, 11: 1_000_000}[cfg]


def secondary_regions(args):
    if args.primary_only:
        return []
    if not args.secondary:
        return list(SECONDARY)
    if args.secondary == "none":
        return []
    out = []
    for item in args.secondary.split(","):
        c, n = item.split(":")
        out.append((int(c), int(n)))
    return out


def kernel_src_hash() -> str:
    h = hashlib.sha256()
    for f in KERNEL_SOURCES:
        with open(os.path.join(REPO, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


# --------------------------------------------------------------------------- launcher
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch(argv, n: int) -> int:
    """Parent of an N-rank run started without torchrun: spawns N fresh `python bench.py`
    children (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*), relays rank 0's stdout, and
    returns the first non-zero exit code (the remaining ranks are then stopped: they would
    wait at the next barrier forever). Never imports tkz or touches the GPU."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL))
    rc = 0
    live = list(range(n))
    while live:
        for r in list(live):
            code = procs[r].poll()
            if code is None:
                continue
            live.remove(r)
            if code != 0 and rc == 0:
                rc = code
                print(f"bench.py: rank {r} exited with {code}; stopping the other ranks", file=sys.stderr, flush=True)
                for q in live:
                    procs[q].kill()
        time.sleep(0.05)
    out = procs[0].stdout.read().decode() if procs[0].stdout else ""
    if rc == 0:
        sys.stdout.write(out)
        sys.stdout.flush()
    return rc


# --------------------------------------------------------------------------- ranks
class Dist:
    """Barrier / max / sum over ranks (gloo; measurement only, not on the data path)."""

    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        if self.world > 1:
            import torch.distributed as dist

            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            # gloo prints its connection report on stdout; send it to stderr, so that
            # rank 0's JSON line is the only thing on stdout
            sys.stdout.flush()
            saved = os.dup(1)
            os.dup2(2, 1)
            try:
                dist.init_process_group("gloo", rank=self.rank, world_size=self.world)
                dist.barrier()
            finally:
                sys.stdout.flush()
                os.dup2(saved, 1)
                os.close(saved)
            self.dist = dist

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()

    def _reduce(self, x: float, op) -> float:
        if self.world == 1:
            return x
        import torch

        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t, op=op)
        return float(t.item())

    def max(self, x: float) -> float:
        return self._reduce(x, self.dist.ReduceOp.MAX if self.world > 1 else None)

    def sum(self, x: float) -> float:
        return self._reduce(x, self.dist.ReduceOp.SUM if self.world > 1 else None)

    def close(self):
        if self.world > 1:
            self.dist.destroy_process_group()


def shard_first_doc(rank: int, n_docs: int) -> int:
    """Doc index of this rank's shard in the global synthetic stream."""
    return rank * n_docs


def run_timed(step_fn, sync_fn, dist: Dist, steps: int, warmup: int):
    for _ in range(warmup):
        step_fn()
    sync_fn()
    dist.barrier()
    sync_fn()
    t0 = time.perf_counter()
    for _ in range(steps):
        step_fn()
    sync_fn()
    dist.barrier()
    t1 = time.perf_counter()
    return dist.max(t1 - t0)


# --------------------------------------------------------------------------- evidence
def pmc_summary(src_hash=None):
    """(file, summary) of the newest committed rocprofv3 PMC summary (profiles/*_pmc.json,
    tools/pmc_summary.py) of the primary workload (C1: its command has no other --config)
    whose kernel-source hash equals `src_hash` (the build being measured); (None, {}) when
    none matches."""
    pdir = os.path.join(REPO, "profiles")
    if not os.path.isdir(pdir):
        return None, {}
    for f in sorted((f for f in os.listdir(pdir) if f.endswith("_pmc.json")), reverse=True):
        try:
            d = json.load(open(os.path.join(pdir, f)))
        except Exception:
            continue
        cmd = str(d.get("cmd", "")).split()
        cfg = cmd[cmd.index("--config") + 1] if "--config" in cmd[:-1] else "1"
        # the primary workload's passes only (other configs' summaries share the hash)
        if d.get("src_hash") == src_hash and ("k_encode" in d or "k_encode_blk" in d) and cfg == "1":
            return f, merge_encode_stage(d)
    return None, {}


ENCODE_STAGE = ("k_encode", "k_encode_blk", "k_bpe_short")  # the kernels between HIP events 0 and 1


def merge_encode_stage(d):
    """A PMC summary with the encode stage's kernels (k_encode_blk + k_bpe_short since round
    6; k_encode before) summed into one "k_encode" entry: bytes and counters per step."""
    parts = [d[k] for k in ENCODE_STAGE if isinstance(d.get(k), dict)]
    if not parts or (len(parts) == 1 and "k_encode" in d):
        return d
    out = dict(d)
    m = {"kernels": [k for k in ENCODE_STAGE if k in d], "counters": {}}
    for p in parts:
        lps = p.get("launches_per_step", 1.0) or 1.0
        for key in ("bytes", "read_bytes", "write_bytes", "fetch_size_bytes"):
            if p.get(key) is not None:
                m[key] = m.get(key, 0) + int(p[key] * lps)
        for c, v in (p.get("counters") or {}).items():
            m["counters"][c] = m["counters"].get(c, 0) + v * lps
    out["k_encode"] = m
    return out


def trace_summary(src_hash=None):
    """(file, k_encode ms) of the newest committed rocprofv3 --kernel-trace summary of the
    primary workload (profiles/*_kernel_trace_summary.txt, tools/trace_summary.py, first
    line "# src_hash <hash> ...") whose kernel-source hash equals `src_hash`; the k_encode
    average is over its bench-sized launches (the largest grid). (None, None) if none."""
    pdir = os.path.join(REPO, "profiles")
    if not os.path.isdir(pdir):
        return None, None
    for f in sorted((f for f in os.listdir(pdir) if f.endswith("_kernel_trace_summary.txt")), reverse=True):
        try:
            lines = open(os.path.join(pdir, f)).read().splitlines()
        except OSError:
            continue
        if not lines or not lines[0].startswith("# src_hash ") or lines[0].split()[2] != src_hash:
            continue
        best = None  # (grid, avg ms) of the largest-grid k_encode / k_encode_blk
        short = 0.0  # k_bpe_short (the encode stage's second kernel since round 6)
        for ln in lines[1:]:
            t = ln.split()
            if len(t) >= 4 and (t[0].startswith("tkz::k_encode") or t[0].startswith("tkz::k_bpe_short")):
                try:
                    grid, ms = int(t[-3]), float(t[-1])
                except ValueError:
                    continue
                if t[0].startswith("tkz::k_bpe_short"):
                    short = max(short, ms)
                elif best is None or grid > best[0]:
                    best = (grid, ms)
        return f, (round(best[1] + short, 4) if best else None)
    return None, None


def host_cpus():
    """(os.cpu_count(), CPUs in this process's affinity mask, the cgroup CPU quota or None)."""
    total = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = total
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    return total, aff, quota


def oracle_threads(world: int = 1):
    """Host threads for one rank's oracle work: the CPUs this process may use (affinity,
    capped by the cgroup quota), shared by the `world` ranks of the node (eight ranks
    verifying at once must not each start a thread per CPU)."""
    _, aff, quota = host_cpus()
    cpus = min(aff, quota) if quota else aff
    return max(1, cpus // max(1, world))


def cpu_baseline(cfg, js, n_sample, threads, min_seconds):
    """The C++ restatement of Tokenizer.encode (oracle/tkz_oracle.cpp, per-doc loop with
    the reference's allocation pattern; the Zig reference cannot be built here) built
    -O3 -march=native on this host: `threads` threads over a bounded sample of the same
    workload until `min_seconds`, then 1 thread over 1/16 of it."""
    from oracle import oracle as orc
    from tkz import synth

    build = "-O3 -march=native"
    try:
        path = orc.build_native()
    except Exception as e:  # no compiler: the portable prebuilt library
        path, build = orc.LIB_PATH, f"-O3 -march=x86-64-v2 (native build failed: {type(e).__name__})"
    ref = orc.RefTokenizer.from_json(js)
    co = orc.COracle(ref, lib_path=path)
    data, off = synth.docs(cfg, n_sample, first_doc=0)

    def timed(d, o, th, min_s, max_passes):
        passes, t0 = 0, time.perf_counter()
        while passes < 1 or (time.perf_counter() - t0 < min_s and passes < max_passes):
            co.encode_batch(d, o, n_threads=th)
            passes += 1
        return passes, time.perf_counter() - t0

    p_all, dt_all = timed(data, off, threads, min_seconds, 8)
    n1 = max(1, n_sample // 16)
    off1 = off[: n1 + 1]
    p_1, dt_1 = timed(data[: int(off1[-1])], off1, 1, min_seconds / 2, 4)
    total, aff, quota = host_cpus()
    return {"value": round(float(off[-1]) * p_all / dt_all / 1e6, 3), "unit": "MB/s", "cores": threads,
            "kind": "port", "threads": threads, "host_cores": total, "affinity_cores": aff, "cgroup_cpus": quota,
            "value_1thread": round(float(off1[-1]) * p_1 / dt_1 / 1e6, 3), "build": build,
            "sample": f"{p_all} pass(es) over {n_sample} docs ({int(off[-1])} B) of the same workload on {threads} "
                      f"threads in {dt_all:.2f} s; 1 thread: {p_1} pass(es) over {n1} docs ({int(off1[-1])} B) in "
                      f"{dt_1:.2f} s. C++ restatement of Tokenizer.encode (oracle/tkz_oracle.cpp, {build}), "
                      f"contiguous doc ranges per thread"}


def stream_steps(tkz, dbs):
    """(step, sync) over len(dbs) batches: step k runs batch k % S on HIP stream k % S, so
    a step's kernels start while the previous step's last kernels drain (each step is
    still one full pass over the batch). One batch: its own tokenizer stream."""
    if len(dbs) == 1:
        return dbs[0].run, dbs[0].sync
    streams = [tkz.lib().tkz_stream_create() for _ in dbs]
    if not all(streams):
        raise RuntimeError("tkz_stream_create failed")
    k_step = [0]

    def step_fn():
        i = k_step[0] % len(dbs)
        k_step[0] += 1
        dbs[i].run(streams[i])

    def sync_fn():
        if tkz.lib().tkz_device_synchronize():
            raise RuntimeError("tkz_device_synchronize failed")

    return step_fn, sync_fn


def two_batches_fit(tok, total: int, n_docs: int) -> bool:
    """True when two one-pass batches (workspace, input, worst-case outputs) fit in 90 % of
    the device's free memory."""
    import tkz

    free, tot = ctypes.c_size_t(0), ctypes.c_size_t(0)
    if tkz.lib().tkz_dev_mem_info(ctypes.byref(free), ctypes.byref(tot)) != 0:
        return False
    one = int(tkz.lib().tkz_device_workspace_size(tok.handle, total, n_docs)) + 13 * total + 16 * (n_docs + 2) + 64
    return 2 * one <= 0.9 * free.value


# --------------------------------------------------------------------------- verification
def golden_hashes(cfg: int, n_docs: int, first_doc: int):
    """The oracle's committed hashes of docs [first_doc, first_doc + n_docs) of config
    cfg, or None when no golden file holds that shard."""
    try:
        if cfg == 4 and n_docs == 8_000_000 and first_doc % n_docs == 0:
            g = json.load(open(os.path.join(GOLDEN, "c4_stream_64M.json")))
            s = first_doc // n_docs
            return g["shards"][s] if s < len(g["shards"]) else None
        if cfg == 4 and n_docs == 8_000_000:
            return None
        g = json.load(open(os.path.join(GOLDEN, "bench_shards.json")))
        shards = g["configs"].get(str(cfg), [])
        shard_docs = g.get("shard_docs_by_config", {}).get(str(cfg), g["shard_docs"])
        if n_docs == shard_docs and first_doc % n_docs == 0 and first_doc // n_docs < len(shards):
            return shards[first_doc // n_docs]
        if cfg == 4 and n_docs == 1_000_000 and first_doc == 0:  # the first 1M docs of the C4 stream
            return json.load(open(os.path.join(GOLDEN, "c4_shard_1M.json"))) if os.path.exists(
                os.path.join(GOLDEN, "c4_shard_1M.json")) else None
    except (OSError, ValueError, KeyError):
        return None
    return None


def verify_region(cfg, js, db, first_doc, n_sample, world=1, require_hash=False):
    """(1) the device-computed rolling hashes of the whole result vs the oracle's committed
    hashes of this shard (None when none is committed); (2) the first n_sample docs
    doc by doc (row_ptr, ids, offsets) vs the C++ oracle run now on this host. `full`: the
    whole result was checked (hash match), not only the sample; with require_hash a region
    whose shard has no committed hash fails."""
    from oracle import oracle as orc
    from tkz import synth

    got = synth.csr_hash_device(db)
    gold = golden_hashes(cfg, db.n_docs, first_doc)
    keys = ("n_docs", "n_tokens", "row_ptr", "ids", "offsets")
    hash_ok = None if gold is None else all(got[k] == gold[k] for k in keys)
    n = min(n_sample, db.n_docs)
    t0 = time.perf_counter()
    data, off = synth.docs(cfg, n, first_doc=first_doc)
    co = orc.COracle(orc.RefTokenizer.from_json(js))
    heap = cfg in HEAP_CFGS and co.set_heap(HEAP_CFGS[cfg])
    th = oracle_threads(world)
    t1 = time.perf_counter()
    erow, eids, eoffs = co.encode_batch(data, off, n_threads=th)
    t_cpu = time.perf_counter() - t1
    row, ids, offs = db.results_prefix(n)
    sample_ok = bool(np.array_equal(row, erow) and np.array_equal(ids, eids) and np.array_equal(offs, eoffs))
    nbytes = int(off[-1] - off[0]) if n else 0
    # the same oracle call timed: the reference algorithm's CPU rate on this config (the
    # C++ restatement, oracle/tkz_oracle.cpp, on the host threads; tables built before)
    cpu = {"value": round(nbytes / max(t_cpu, 1e-9) / 1e6, 3), "unit": "MB/s", "threads": th,
           "kind": "port-heap" if heap else "port",
           "sample": f"{n} docs ({nbytes} B) of this region in {t_cpu:.2f} s" +
                     (f" (pretokens of >= {HEAP_CFGS[cfg]} B by the heap form of the merge loop)" if heap else "")}
    if heap:  # the literal loop (the reference's algorithm) on the sample's shorter docs
        lens = np.diff(off.astype(np.int64))
        pick = [i for i in range(n) if lens[i] <= 16384][:64]
        if pick:
            sub = [bytes(data[int(off[i]):int(off[i + 1])]) for i in pick]
            so = np.zeros(len(sub) + 1, dtype=np.uint64)
            so[1:] = np.cumsum([len(x) for x in sub])
            sd = np.frombuffer(b"".join(sub) + bytes(16), dtype=np.uint8).copy()
            lit = orc.COracle(orc.RefTokenizer.from_json(js))
            t1 = time.perf_counter()
            lit.encode_batch(sd, so, n_threads=th)
            t_lit = time.perf_counter() - t1
            cpu["literal"] = {"value": round(int(so[-1]) / max(t_lit, 1e-9) / 1e6, 3), "unit": "MB/s", "threads": th,
                              "kind": "port", "sample": f"the sample's {len(sub)} docs of <= 16 KB ({int(so[-1])} B) "
                                                        f"by the literal loop in {t_lit:.2f} s (longer docs cost more "
                                                        f"per byte: O(rounds x n) per pretoken)"}
    return {"hash_match": hash_ok, "hash": got, "golden": "committed" if gold is not None else None,
            "sample_docs": n, "sample_match": sample_ok, "verify_s": round(time.perf_counter() - t0, 2),
            "cpu": cpu, "full": hash_ok is True,
            "ok": bool(sample_ok and (hash_ok is True if require_hash else hash_ok is not False))}


# --------------------------------------------------------------------------- regions
def make_batch(tkz, synth, tok, cfg, n_docs, first_doc, args, max_ws):
    """Inputs of the region in HBM (device generator, or host + upload) and one batch."""
    if args.host_inputs:
        data, off = synth.docs(cfg, n_docs, first_doc=first_doc)
        return None, tkz.DeviceBatch(tok, data, off, max_workspace=max_ws)
    dd = synth.DeviceDocs(cfg, n_docs, first_doc)
    return dd, tkz.DeviceBatch.from_device(tok, dd.d_bytes, dd.d_off, dd.n_docs, dd.total, max_workspace=max_ws, owner=dd)


def secondary_region(tkz, synth, dist, cfg, n_docs, args):
    """A few timed steps of another config on this rank's shard, verified."""
    js = synth.tokenizer_json(cfg)
    t_tab = time.perf_counter()
    tok = tkz.Tokenizer.from_json(js)  # host parse + device tables + the word / segment memos + hot pairs
    table_build_ms = (time.perf_counter() - t_tab) * 1e3
    tok.set_word_memo(not args.no_memo)
    tok.set_long_segments(not args.no_long_segments)
    first = shard_first_doc(dist.rank, n_docs)
    max_ws = int(args.max_workspace_gb * (1 << 30)) if args.max_workspace_gb > 0 else None
    dd, db = make_batch(tkz, synth, tok, cfg, n_docs, first, args, max_ws)
    tkz.profile_enable(tok, True)
    el = run_timed(db.run, db.sync, dist, args.secondary_steps, 1)
    ms = tkz.profile_read(tok)
    tkz.profile_enable(tok, False)
    stats = db.stats()
    n_sample = 40 if cfg in HEAP_CFGS else 10_000 if cfg in LONG_CFGS else 20_000
    ver = None if args.no_verify else verify_region(cfg, js, db, first, n_sample, dist.world,
                                                    require_hash=not args.secondary)
    n_bad = int(dist.sum(0.0 if ver is None or ver["ok"] else 1.0))
    total = db.total
    calls = args.secondary_steps + 1
    res = {"workload": WORKLOADS[cfg], "docs_per_gpu": n_docs, "bytes_per_gpu": total,
           "value": round(dist.sum(float(total)) * args.secondary_steps / el / 1e6, 2), "unit": "MB/s",
           "steps": args.secondary_steps, "ms_per_step": round(el / args.secondary_steps * 1e3, 3),
           "kernel_ms": {"k_encode": round(ms[0] / calls, 4), "deferred": round(ms[1] / calls, 4),
                         "scan": round(ms[2] / calls, 4), "compact": round(ms[3] / calls, 4)},
           "sub_batches": stats["sub_batches"],
           "long_words": stats["long_words"], "long_segmented": stats["long_segmented"],
           "long_fallback_bytes": stats["long_fallback_bytes"],
           "long_fallback_frac": round(stats["long_fallback_bytes"] / max(total, 1), 6),
           "memo_hit_rate": round(stats["memo_hits"] / max(stats["pretokens"], 1), 4),
           "table_build_ms": round(table_build_ms, 1), "memo_info": tok.memo_info(),
           "verified": None if ver is None else {k: ver[k] for k in ("hash_match", "full", "sample_docs", "sample_match")},
           "cpu_sample": None if ver is None else ver["cpu"],
           "ranks_failed": n_bad}
    if ver is not None and ver["cpu"]["value"] > 0:  # this GPU's rate over the host threads' rate
        res["vs_cpu_sample"] = round(float(total) * args.secondary_steps / el / 1e6 / ver["cpu"]["value"], 1)
    db.free()
    if dd is not None:
        dd.free()
    tok.close()
    return res, n_bad


def single_doc_region(tkz, synth, cfg, n_docs):
    """The reference's own call shape, timed per call (verdict r5 item 7): Tokenizer.encode of
    ONE doc from a host buffer to a host Encoding (/root/reference/src/lib.zig:109-160,
    examples/basic_tokenize.zig:34) = tkz_encode, which runs the whole device pipeline for
    the doc (copy in, the encode kernels, copy out). p50 / p90 / p99 latency over n_docs
    512-B docs, each call's ids checked against the oracle; beside it the oracle's per-doc
    time on one host thread (the C++ restatement of the reference's loop)."""
    from oracle import oracle as orc

    js = synth.tokenizer_json(cfg)
    tok = tkz.Tokenizer.from_json(js)
    L = tkz.lib()
    data, off = synth.docs(cfg, n_docs, first_doc=0)
    docs = [bytes(data[int(off[i]):int(off[i + 1])]) for i in range(n_docs)]
    erow, eids, _ = orc.COracle(orc.RefTokenizer.from_json(js)).encode_batch(data, off, n_threads=oracle_threads(1))
    enc = tkz._Encoding()
    for d in docs[:200]:  # warm-up: staging buffers grown, kernels loaded
        if L.tkz_encode(tok.handle, d, len(d), 0, ctypes.byref(enc)):
            raise RuntimeError("tkz_encode failed")
        L.tkz_encoding_free(ctypes.byref(enc))
    lat, bad = [], 0
    for i, d in enumerate(docs):
        t0 = time.perf_counter_ns()
        rc = L.tkz_encode(tok.handle, d, len(d), 0, ctypes.byref(enc))
        t1 = time.perf_counter_ns()
        if rc:
            raise RuntimeError("tkz_encode failed")
        n = int(enc.len)
        got = np.ctypeslib.as_array(enc.ids, shape=(n,)) if n else np.zeros(0, np.uint32)
        bad += int(not np.array_equal(got, eids[int(erow[i]):int(erow[i + 1])]))
        L.tkz_encoding_free(ctypes.byref(enc))
        lat.append((t1 - t0) / 1e3)
    tok.close()
    lat = np.array(lat)
    co = orc.COracle(orc.RefTokenizer.from_json(js))
    t0 = time.perf_counter()
    co.encode_batch(data, off, n_threads=1)
    cpu_us = (time.perf_counter() - t0) / n_docs * 1e6
    return {"workload": WORKLOADS[cfg] + "; one doc per tkz_encode call (host buffer in, host Encoding out)",
            "calls": n_docs, "unit": "us", "p50": round(float(np.percentile(lat, 50)), 1),
            "p90": round(float(np.percentile(lat, 90)), 1), "p99": round(float(np.percentile(lat, 99)), 1),
            "mean": round(float(lat.mean()), 1), "min": round(float(lat.min()), 1),
            "cpu_oracle_us_per_doc_1thread": round(cpu_us, 2), "mismatches": bad}, int(bad != 0)


def decode_region(tkz, tok, js, db, dist, steps):
    """Batched Tokenizer.decode on the device over the primary region's CSR result (SURVEY
    8(f) row 1: /root/reference/src/lib.zig:163-189 + the config decoders,
    config.zig:488-530; tkz_decode_batch_device, csrc/decode.hip): tokens/s and bytes/s, a
    sample checked against the oracle's decode."""
    from oracle import oracle as orc

    L = tkz.lib()
    n, T = db.n_docs, db.n_tokens()
    cap = int(L.tkz_decode_bound(tok.handle, T))
    wsz = int(L.tkz_decode_workspace_size(tok.handle, n, T))
    d_out, d_off, d_ws = tkz.DeviceBuffer(cap + 16), tkz.DeviceBuffer((n + 1) * 8), tkz.DeviceBuffer(wsz)

    def step():
        rc = L.tkz_decode_batch_device(tok.handle, db.d_row.ptr, db.d_ids.ptr, n, T, 0, d_out.ptr, cap, d_off.ptr,
                                       d_ws.ptr, wsz, None)
        if rc:
            tkz._err(rc)

    el = run_timed(step, lambda: L.tkz_synchronize(tok.handle), dist, steps, 1)
    offs = np.zeros(n + 1, dtype=np.uint64)
    d_off.download(offs)
    k = min(2000, n)
    row, ids, _ = db.results_prefix(k)
    out = np.zeros(int(offs[k]) + 1, dtype=np.uint8)
    d_out.download(out, int(offs[k]))
    ref = orc.RefTokenizer.from_json(js)
    ok = all(bytes(out[int(offs[i]):int(offs[i + 1])]) == ref.decode(ids[int(row[i]):int(row[i + 1])].tolist())
             for i in range(k))
    out_bytes = int(offs[n])
    alg = 4 * T + 8 * (n + 1) + out_bytes + 8 * (n + 1)  # ids + row_ptr read, text + its offsets written
    ms = el / steps * 1e3
    for b in (d_out, d_off, d_ws):
        b.free()
    return {"workload": "tkz_decode_batch_device over the primary region's result (C1: 32k BPE, BPE decoder)",
            "docs": n, "tokens": T, "out_bytes": out_bytes, "ms_per_step": round(ms, 3),
            "tokens_per_s": round(dist.sum(float(T)) / (ms / 1e3), 1),
            "value": round(dist.sum(float(out_bytes)) / (ms / 1e3) / 1e6, 2), "unit": "MB/s (decoded text)",
            "roofline": {"bound": "hbm", "alg_bytes": alg, "achieved": round(alg / (ms / 1e3) / 1e9, 2),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(alg / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                         "bytes": "4 B/token ids + 8 B/doc row_ptr read; decoded bytes + 8 B/doc offsets written"},
            "verified": {"sample_docs": k, "sample_match": ok}}, int(not ok)


def pad_region(tkz, tok, db, dist, steps, length=128):
    """Truncation + padding to a dense [n_docs, length] batch on the device over the primary
    region's CSR (Encoding.truncate / Encoding.pad,
    /root/reference/src/encoding.zig:362-437; tkz_pad_batch_device, csrc/pad.hip), a
    sample checked against the reference's rules restated in numpy."""
    L = tkz.lib()
    n, T = db.n_docs, db.n_tokens()
    tok.set_truncation(length)
    tok.set_padding(length, 0, 0, b"[PAD]", "right")
    cap = int(L.tkz_pad_capacity(tok.handle, n, T))
    wsz = int(L.tkz_pad_workspace_size(n))
    row2, ids2, offs2 = tkz.DeviceBuffer((n + 1) * 8), tkz.DeviceBuffer(cap * 4), tkz.DeviceBuffer(cap * 8)
    ty, sp, at, ws = tkz.DeviceBuffer(cap * 4), tkz.DeviceBuffer(cap * 4), tkz.DeviceBuffer(cap * 4), tkz.DeviceBuffer(wsz)

    def step():
        rc = L.tkz_pad_batch_device(tok.handle, db.d_row.ptr, db.d_ids.ptr, db.d_offs.ptr, n, row2.ptr, ids2.ptr,
                                    offs2.ptr, ty.ptr, sp.ptr, at.ptr, ws.ptr, wsz, None)
        if rc:
            tkz._err(rc)

    el = run_timed(step, lambda: L.tkz_synchronize(tok.handle), dist, steps, 1)
    k = min(2000, n)
    row, ids, offs = db.results_prefix(k)
    r2 = np.zeros(n + 1, dtype=np.uint64)
    row2.download(r2)
    got_ids = np.zeros(k * length, dtype=np.uint32)
    ids2.download(got_ids, k * length * 4)
    got_at = np.zeros(k * length, dtype=np.uint32)
    at.download(got_at, k * length * 4)
    exp_ids = np.zeros((k, length), dtype=np.uint32)
    exp_at = np.zeros((k, length), dtype=np.uint32)
    for i in range(k):  # encoding.zig:362-380 (keep the first max_length), 385-437 (pad right)
        t = ids[int(row[i]):int(row[i + 1])][:length]
        exp_ids[i, :len(t)] = t
        exp_at[i, :len(t)] = 1
    ok = bool(np.array_equal(r2[:k + 1], np.arange(k + 1, dtype=np.uint64) * length) and
              np.array_equal(got_ids.reshape(k, length), exp_ids) and np.array_equal(got_at.reshape(k, length), exp_at))
    tok.set_truncation(None)
    tok.set_padding(None, enabled=False)
    for b in (row2, ids2, offs2, ty, sp, at, ws):
        b.free()
    ms = el / steps * 1e3
    alg_in = 4 * T + 8 * T + 8 * (n + 1)  # (upper bound: every token read; truncated ones need not be)
    alg_out = n * length * (4 + 8 + 4 + 4 + 4) + 8 * (n + 1)
    return {"workload": f"tkz_pad_batch_device: truncate + pad the primary result to a dense [{n}, {length}] batch",
            "docs": n, "tokens_in": T, "ms_per_step": round(ms, 3), "out_bytes": alg_out,
            "value": round(dist.sum(float(alg_out)) / (ms / 1e3) / 1e6, 2), "unit": "MB/s (dense output written)",
            "roofline": {"bound": "hbm", "alg_bytes": alg_in + alg_out,
                         "achieved": round((alg_in + alg_out) / (ms / 1e3) / 1e9, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round((alg_in + alg_out) / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                         "bytes": "CSR ids + offsets + row_ptr read; ids, offsets, type ids, special and attention "
                                  "masks of the dense batch written"},
            "verified": {"sample_docs": k, "sample_match": ok}}, int(not ok)


def host_e2e_region(tkz, synth, dist, cfg, n_docs, args):
    """The reference's own call shape (Tokenizer.encode: host text in, host Encoding out,
    /root/reference/src/lib.zig:109-160), batched: tkz_encode_batch from host input to host
    CSR, PCIe copies included (never the bench `value`). Timed twice, from pageable input
    (what a caller's []const u8 is) and from page-locked input (tkz_host_alloc), with the
    library's timeline of the pipelined path (HIP events per chunk + host timers) and the
    raw link rates of the same box (a hipMemcpy of the same sizes), so the split shows what
    bounds it. Verified: host CSR hashes vs the oracle's committed shard hashes."""
    from tests.shard_hash import CsrHash

    js = synth.tokenizer_json(cfg)
    tok = tkz.Tokenizer.from_json(js)
    L = tkz.lib()
    first = shard_first_doc(dist.rank, n_docs)
    data, off = synth.docs(cfg, n_docs, first_doc=first, threads=oracle_threads(dist.world))
    total = int(off[-1])
    op = off.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))

    def timed(ptr):
        b = tkz._Batch()
        for _ in range(2):  # warm-up: sizes the pipeline's output arrays, page-locks the pool
            rc = L.tkz_encode_batch(tok.handle, ptr, op, n_docs, ctypes.byref(b))
            if rc:
                tkz._err(rc)
            L.tkz_batch_free(ctypes.byref(b))
        # device memory freed before this point (the earlier regions' buffers, the warm-up's
        # resized staging) is cleared by the driver on the DMA engines in the background,
        # which halves the device-to-host copy rate for the next few hundred ms
        # (profiles/r04n_host_dma_settle.txt): time the steady state
        time.sleep(1.0)
        dist.barrier()
        t0 = time.perf_counter()
        for k in range(args.secondary_steps):
            rc = L.tkz_encode_batch(tok.handle, ptr, op, n_docs, ctypes.byref(b))
            if rc:
                tkz._err(rc)
            L.tkz_batch_free(ctypes.byref(b))
        el = time.perf_counter() - t0
        dist.barrier()
        el = dist.max(el)
        # one more call with the timeline recorded (HIP timing events on both streams; the
        # timed calls above run without them), its result verified
        tkz.profile_enable(tok, True)
        tkz.host_profile_read(tok, reset=True)
        t0 = time.perf_counter()
        rc = L.tkz_encode_batch(tok.handle, ptr, op, n_docs, ctypes.byref(b))
        if rc:
            tkz._err(rc)
        el_prof = time.perf_counter() - t0
        hp = tkz.host_profile_read(tok, reset=True)
        tkz.profile_read(tok, reset=True)
        tkz.profile_enable(tok, False)
        hp["profiled_call_ms"] = el_prof * 1e3
        nt = int(b.n_tokens)
        h = CsrHash()
        h.add(np.ctypeslib.as_array(b.row_ptr, shape=(n_docs + 1,)), np.ctypeslib.as_array(b.ids, shape=(nt,)),
              np.ctypeslib.as_array(ctypes.cast(b.offsets, ctypes.POINTER(ctypes.c_uint32)), shape=(nt, 2)))
        L.tkz_batch_free(ctypes.byref(b))
        calls = max(hp["calls"], 1.0)
        per = {k: round(v / calls, 3) for k, v in hp.items() if k.endswith("_ms") and k != "profiled_call_ms"}
        per["profiled_call_ms"] = round(hp["profiled_call_ms"], 3)
        per["chunks"] = hp["chunks"] / calls
        per["out_pageable"] = hp["out_pageable"] / calls  # output arrays the pinned pool could not serve
        return el, per, h.result(), nt

    el_p, tl_p, hash_p, nt = timed(data.ctypes.data_as(ctypes.c_void_p))
    pin = tkz.HostBuffer(len(data))
    pin.array[:] = data
    el_q, tl_q, hash_q, _ = timed(ctypes.c_void_p(pin.ptr))

    # raw link rates on this box, the same sizes: input H2D (pageable / page-locked), CSR D2H
    out_bytes = (n_docs + 1) * 8 + 12 * nt
    dbuf = tkz.DeviceBuffer(max(total, out_bytes))
    hout = tkz.HostBuffer(out_bytes)

    def rate(fn, nbytes, reps=3):
        fn()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        return round(nbytes * reps / (time.perf_counter() - t0) / 1e9, 2)

    link = {"h2d_pageable_gbs": rate(lambda: L.tkz_memcpy_htod(dbuf.ptr, data.ctypes.data_as(ctypes.c_void_p), total),
                                     total),
            "h2d_pinned_gbs": rate(lambda: L.tkz_memcpy_htod(dbuf.ptr, ctypes.c_void_p(pin.ptr), total), total),
            "d2h_pinned_gbs": rate(lambda: L.tkz_memcpy_dtoh(ctypes.c_void_p(hout.ptr), dbuf.ptr, out_bytes), out_bytes)}
    dbuf.free()
    hout.free()
    pin.free()
    gold = golden_hashes(cfg, n_docs, first)
    keys = ("n_docs", "n_tokens", "row_ptr", "ids", "offsets")
    ok = gold is not None and all(hash_p[k] == gold[k] and hash_q[k] == gold[k] for k in keys)
    n_bad = int(dist.sum(0.0 if ok or args.no_verify else 1.0))
    d2h_floor_ms = out_bytes / (link["d2h_pinned_gbs"] * 1e9) * 1e3
    res = {"workload": WORKLOADS[cfg] + "; host buffers in and out (tkz_encode_batch, PCIe copies included)",
           "docs_per_gpu": n_docs, "bytes_per_gpu": total, "out_bytes_per_gpu": out_bytes, "unit": "MB/s",
           "steps": args.secondary_steps,
           "value": round(dist.sum(float(total)) * args.secondary_steps / el_p / 1e6, 2),
           "ms_per_call": round(el_p / args.secondary_steps * 1e3, 3),
           "value_pinned_input": round(dist.sum(float(total)) * args.secondary_steps / el_q / 1e6, 2),
           "ms_per_call_pinned_input": round(el_q / args.secondary_steps * 1e3, 3),
           "timeline_pageable_ms": tl_p, "timeline_pinned_ms": tl_q, "link": link,
           "d2h_floor_ms": round(d2h_floor_ms, 3),
           "frac_of_d2h_floor": round(d2h_floor_ms / (el_q / args.secondary_steps * 1e3), 3),
           "verified": {"hash_match": ok, "full": ok}, "ranks_failed": n_bad}
    tok.close()
    return res, n_bad


# --------------------------------------------------------------------------- main
def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch(argv, args.gpus))
    if args.simulate_cpu:
        return main_simulated(args)
    import tkz
    from tkz import synth

    dist = Dist()
    if args.gpus != dist.world and dist.rank == 0:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={dist.world}; using {dist.world} ranks",
              file=sys.stderr, flush=True)
    tkz.set_device(0 if args.share_gpu else dist.local_rank)
    n_bad = 0
    host_e2e = None
    if args.host_e2e_first and not args.no_host_e2e:  # (diagnostic: before any other region)
        host_e2e, bad = host_e2e_region(tkz, synth, dist, 1, default_docs(1), args)
        n_bad += bad
    cfg = args.config
    n_docs = args.docs or default_docs(cfg)
    js = synth.tokenizer_json(cfg)
    t_tab = time.perf_counter()
    tok = tkz.Tokenizer.from_json(js)  # host parse + device tables + the word memo (GPU encode of the vocab keys)
    table_build_ms = (time.perf_counter() - t_tab) * 1e3
    bpe = tok.info()["model"] == 1
    tok.set_word_memo(not args.no_memo)
    tok.set_long_segments(not args.no_long_segments)
    first = shard_first_doc(dist.rank, n_docs)
    max_ws = int(args.max_workspace_gb * (1 << 30)) if args.max_workspace_gb > 0 else None
    t_in = time.perf_counter()
    dd, db = make_batch(tkz, synth, tok, cfg, n_docs, first, args, max_ws)
    inputs_s = time.perf_counter() - t_in
    total = db.total
    n_streams = args.streams or (2 if max_ws is None and two_batches_fit(tok, total, n_docs) else 1)
    dbs = [db] + [tkz.DeviceBatch.from_device(tok, db.d_bytes, db.d_off, n_docs, total, max_workspace=max_ws, owner=dd)
                  for _ in range(n_streams - 1)]
    step_fn, sync_fn = stream_steps(tkz, dbs)

    # timed region: K full passes, inputs resident, kernel timers on the encode streams
    tkz.profile_enable(tok, True)
    elapsed = run_timed(step_fn, sync_fn, dist, args.steps, args.warmup)
    ms_enc, ms_def, ms_scan, ms_comp, npass = tkz.profile_read(tok)
    tkz.profile_enable(tok, False)
    stats = db.stats()
    n_tokens = db.n_tokens()
    ver = None
    if not args.no_verify:
        ver = verify_region(cfg, js, db, first, args.verify_docs, dist.world,
                            require_hash=cfg == 1 and n_docs == default_docs(cfg))
        if len(dbs) > 1:  # every stream's batch holds the same result
            h0 = ver["hash"]
            ver["streams_identical"] = all(synth.csr_hash_device(b) == h0 for b in dbs[1:])
            ver["ok"] = ver["ok"] and ver["streams_identical"]
    n_bad += int(dist.sum(0.0 if ver is None or ver["ok"] else 1.0))

    # memo-off rate on the same shard (BPE: the memo is a vocab-derived shortcut; this is the
    # general path's rate)
    memo_off = None
    if bpe and not args.no_memo and not args.no_memo_off_run:
        tok.set_word_memo(False)
        el_off = run_timed(step_fn, sync_fn, dist, args.steps, 1)
        same_off = None
        if not args.no_verify:
            same_off = synth.csr_hash_device(db) == ver["hash"]
            n_bad += int(dist.sum(0.0 if same_off else 1.0))
        tok.set_word_memo(True)
        memo_off = {"value": round(dist.sum(float(total)) * args.steps / el_off / 1e6, 2),
                    "ms_per_step": round(el_off / args.steps * 1e3, 3), "results_identical": same_off}
    # the same steps with two batches in flight on two streams (secondary: `value` and the
    # kernel rooflines stay single-stream, where HIP event durations are per kernel)
    pipelined = None
    fits = n_streams == 1 and not args.no_pipelined_run and max_ws is None and two_batches_fit(tok, total, n_docs)
    if dist.sum(0.0 if fits else 1.0) == 0:  # every rank or none (the region has barriers)
        db2 = tkz.DeviceBatch.from_device(tok, db.d_bytes, db.d_off, n_docs, total)
        st2, sy2 = stream_steps(tkz, [db, db2])
        el2 = run_timed(st2, sy2, dist, args.steps, args.warmup)
        same = None
        if not args.no_verify:
            same = synth.csr_hash_device(db2) == ver["hash"] and synth.csr_hash_device(db) == ver["hash"]
            n_bad += int(dist.sum(0.0 if same else 1.0))
        pipelined = {"streams": 2, "value": round(dist.sum(float(total)) * args.steps / el2 / 1e6, 2),
                     "ms_per_step": round(el2 / args.steps * 1e3, 3), "results_identical": same}
        db2.free()
    total_all = dist.sum(float(total))
    tokens_all = dist.sum(float(n_tokens))
    value = total_all * args.steps / elapsed / 1e6
    ms_step = elapsed / args.steps * 1e3

    # roofline: the path's algorithmic bytes per batch = input bytes + 12 B
    # per token (u32 id + 2 x u32 offset) + 8 B per row_ptr entry, over the step's time
    # (all kernels, barrier to barrier). Per-kernel figures are sub-fields, each with its
    # own byte definition; kernel times are HIP events on the encode stream.
    calls = args.steps + args.warmup
    npass = max(npass, 1)
    per_call = lambda ms: ms / calls  # noqa: E731  (ms per step, all passes of a call)
    alg_step = total + 12 * n_tokens + 8 * (n_docs + 1)
    alg_out = 12 * n_tokens + 8 * (n_docs + 1)
    enc_s = per_call(ms_enc) / 1e3
    comp_s = per_call(ms_comp) / 1e3
    src_hash = kernel_src_hash()
    default_cmd = cfg == 1 and not args.no_memo and n_docs == default_docs(cfg) and max_ws is None
    pmc_file, pmc = pmc_summary(src_hash) if default_cmd else (None, {})
    trace_file, trace_ms = trace_summary(src_hash) if default_cmd else (None, None)
    step_pmc = pmc.get("step", {})
    gbs = lambda b, s: round(b / s / 1e9, 2) if s > 0 else None  # noqa: E731
    frac = lambda b, s: round(b / s / 1e9 / HBM_PEAK_GBS, 5) if s > 0 else None  # noqa: E731
    roof = {
        "bound": "hbm", "scope": "step",
        "definition": "SURVEY 8(d): (input bytes + 12 B/token + 8 B/row_ptr entry) per step / step time",
        "achieved": gbs(alg_step, ms_step / 1e3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": frac(alg_step, ms_step / 1e3),
        "frac_of_measured_copy": round(alg_step / (ms_step / 1e3) / 1e9 / HBM_COPY_GBS, 5),
        "alg_bytes": alg_step, "ms": round(ms_step, 4),
        # PMC HBM bytes of the whole step (every kernel; rocprofv3 at this source hash):
        # read bytes from the memory-side request sizes (32/64/128 B), writes from WRITE_SIZE
        "traffic": step_pmc.get("bytes"),
        "traffic_ratio": round(step_pmc["bytes"] / alg_step, 3) if step_pmc.get("bytes") else None,
        "traffic_detail": step_pmc or None, "traffic_source": pmc_file, "src_hash": src_hash,
        # the rocprofv3 kernel trace of this command at this source hash (k_encode's average
        # launch there, to set beside avg_launch_ms below)
        "trace_source": trace_file, "trace_k_encode_ms": trace_ms,
        # the path is probe bound; one word-memo / vocab probe per pretoken
        "pretokens_per_s": round(stats["pretokens"] / (ms_step / 1e3), 1),
        "kernels": {
            "k_encode": {"bytes": "input bytes (reads the docs; its per-word results are scratch)",
                         "alg_bytes": total, "ms": round(enc_s * 1e3, 4), "achieved": gbs(total, enc_s),
                         "frac": frac(total, enc_s), "frac_step_bytes": frac(alg_step, enc_s),
                         "avg_launch_ms": round(enc_s * 1e3 * calls / npass, 4),
                         "passes_per_step": round(npass / calls, 3),
                         "traffic": (pmc.get("k_encode") or {}).get("bytes")},
            "k_compact": {"bytes": "CSR written (12 B/token + 8 B/row_ptr entry)", "alg_bytes": alg_out,
                          "ms": round(comp_s * 1e3, 4), "achieved": gbs(alg_out, comp_s),
                          "frac": frac(alg_out, comp_s), "traffic": (pmc.get("k_compact") or {}).get("bytes")},
            "other_ms": {"deferred_and_long": round(per_call(ms_def), 4), "chunk_scan": round(per_call(ms_scan), 4)},
        },
    }
    # k_encode is bound by instruction issue, not bytes: its VALU / SALU per
    # launch from the same PMC summary, as a rate per SIMD against the measured issue
    # rates of tools/valu_mix.hip (profiles/r02bg_valu_mix.jsonl, 5 waves/SIMD: two-source
    # 32-bit ops 0.90 per SIMD per ns, three-source / 64-bit / DPP / mul 0.55)
    cnt = (pmc.get("k_encode") or {}).get("counters", {})
    if cnt.get("SQ_INSTS_VALU") and enc_s > 0:
        launch_ns = enc_s * 1e9 * calls / npass
        rate = cnt["SQ_INSTS_VALU"] / N_SIMDS / launch_ns
        roof["kernels"]["k_encode"]["issue"] = {
            "valu_per_launch": cnt["SQ_INSTS_VALU"], "salu_per_launch": cnt.get("SQ_INSTS_SALU"),
            "valu_per_simd_per_ns": round(rate, 4), "peak_fast": VALU_PEAK_FAST, "peak_slow": VALU_PEAK_SLOW,
            "frac_fast": round(rate / VALU_PEAK_FAST, 4), "frac_slow": round(rate / VALU_PEAK_SLOW, 4),
            "wait_frac": round(cnt["SQ_WAIT_ANY"] / cnt["SQ_WAVE_CYCLES"], 4) if cnt.get("SQ_WAVE_CYCLES") else None}
    memo = {"hit_rate": round(stats["memo_hits"] / max(stats["pretokens"], 1), 4), "pretokens": stats["pretokens"],
            "deferred_words": stats["deferred"], "memo_off": memo_off, **tok.memo_info()} if not args.no_memo else None
    # SURVEY 8(f) rows 1 and 3 on the primary result: device decode, truncate + pad
    decode = pad = None
    if bpe and not args.no_decode_pad and not args.primary_only:
        decode, bad = decode_region(tkz, tok, js, db, dist, args.secondary_steps)
        n_bad += int(dist.sum(float(bad)))
        pad, bad = pad_region(tkz, tok, db, dist, args.secondary_steps)
        n_bad += int(dist.sum(float(bad)))
    for b in dbs:
        b.free()
    if dd is not None:
        dd.free()

    # the host-buffer region before the secondary regions: the driver clears device memory
    # freed by a region on the DMA engines in the background, and after the large
    # secondary regions (C4 8M, C6) that takes longer than the region's 1-s settle
    if not args.primary_only and not args.no_host_e2e and not args.host_e2e_first:
        host_e2e, bad = host_e2e_region(tkz, synth, dist, 1, default_docs(1), args)
        n_bad += bad
    # the reference's call shape: one doc per call, latency (rank 0's device only)
    single = None
    if not args.primary_only and not args.no_single_doc and dist.rank == 0:
        single, bad = single_doc_region(tkz, synth, 1, 3000)
        n_bad += bad
    # secondary regions: other configs on this rank's shard, a few steps each, verified
    secondary = {}
    for c2, n2 in secondary_regions(args):
        res, bad = secondary_region(tkz, synth, dist, c2, n2, args)
        secondary[f"C{c2}" + ("" if n2 == default_docs(c2) else f"_{n2 // 1_000_000}M")] = res
        n_bad += bad
    out = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "MB/s",
        "n_gpus": dist.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (deterministic generator, generated in HBM by tokenizer-zig_amd/csrc/gen.hip = "
                "synth.cpp; vocab trained in-repo)",
        "config": {"workload": WORKLOADS[cfg], "docs_per_gpu": n_docs, "bytes_per_gpu": total,
                   "tokens_per_gpu": n_tokens, "tokens_all": int(tokens_all), "parallelism": f"doc-shard x{dist.world}",
                   "word_memo": not args.no_memo, "sub_batches": stats["sub_batches"],
                   "shared_gpu": bool(args.share_gpu and dist.world > 1), "inputs": "host" if args.host_inputs
                   else "device-generated", "inputs_s": round(inputs_s, 3),
                   "table_build_ms": round(table_build_ms, 1), "streams": n_streams},
        "roofline": roof,
        "memo": memo,
        "pipelined": pipelined,
        "verified": None if ver is None else {
            "docs_per_rank": ver["sample_docs"], "sample_match": ver["sample_match"],
            "hash_match": ver["hash_match"], "full": ver["full"], "hash": ver["hash"], "ranks_failed": n_bad},
        "secondary": secondary or None,
        "host_e2e": host_e2e,
        "single_doc": single,
        "decode": decode,
        "pad": pad,
    }
    if dist.rank == 0 and dist.world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(cfg, js, min(args.cpu_sample_docs, n_docs), oracle_threads(1)
                                           if not args.cpu_threads else args.cpu_threads, args.cpu_min_seconds)
    else:
        out["cpu_baseline"] = None
    dist.close()
    if dist.rank == 0:
        print(json.dumps(out), flush=True)
    if n_bad:
        print(f"bench.py: verification FAILED on {n_bad} region-rank(s)", file=sys.stderr, flush=True)
        sys.exit(3)
    return out


def main_simulated(args):
    """The multi-rank harness with the C++ oracle as each rank's step (CPU tests)."""
    from oracle import oracle as orc
    from tkz import synth

    dist = Dist()
    n_docs = args.docs or default_docs(args.config)
    js = synth.tokenizer_json(args.config)
    co = orc.COracle(orc.RefTokenizer.from_json(js))
    data, off = synth.docs(args.config, n_docs, first_doc=shard_first_doc(dist.rank, n_docs))
    res = {}
    el = run_timed(lambda: res.setdefault("r", co.encode_batch(data, off, n_threads=1)), lambda: None, dist,
                   args.steps, args.warmup)
    total_all = dist.sum(float(off[-1]))
    tokens_all = dist.sum(float(res["r"][0][-1]))
    first_all = [dist.sum(float(shard_first_doc(dist.rank, n_docs)) if r == dist.rank else 0.0)
                 for r in range(dist.world)]
    out = {"metric": METRIC, "value": round(total_all * args.steps / el / 1e6, 3), "unit": "MB/s",
           "n_gpus": dist.world, "steps": args.steps, "warmup": args.warmup, "simulated_cpu": True,
           "config": {"bytes_all": int(total_all), "tokens_all": int(tokens_all), "shard_first_docs": first_all,
                      "parallelism": f"doc-shard x{dist.world}"}}
    dist.close()
    if dist.rank == 0:
        print(json.dumps(out), flush=True)
    return out


if __name__ == "__main__":
    main()
