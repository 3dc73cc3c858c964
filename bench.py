"""Encode throughput bench (BASELINE.json metric: input MB/s, bit-exact ids).

One step = one pass of the encode hot path (normalize -> pretokenize -> BPE/WordPiece
-> vocab lookup -> CSR ids/offsets) over one batch of synthetic docs already resident
in HBM. Default workload: C1 (configs[1]) = 1M x 512-B ASCII docs, 32k BPE, Whitespace.

N GPUs: one process per GPU (torchrun), each rank encodes its own 1M-doc shard (weak
scaling; docs are independent, so there is no data-path collective). A gloo barrier
brackets the timed region and the max time over ranks is reported. rank 0 prints one
JSON line with `roofline` (k_encode, HIP events on the encode stream) and
`cpu_baseline` (the C++ oracle restatement timed on a bounded sample, rank 0 only).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
for p in (REPO, os.path.join(REPO, "tokenizer-zig_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
HBM_COPY_GBS = 6300.0  # measured copy bandwidth (same guide, HBM section)
WORKLOADS = {
    0: "C0: 1k x 256-B ASCII docs, 8k BPE, Whitespace",
    1: "C1: 1M x 512-B ASCII docs, 32k BPE, Whitespace",
    2: "C2: 1M x 512-B mixed-UTF-8 docs, 32k BPE, Lowercase, Whitespace",
    3: "C3: 1M x 512-B docs, 30k WordPiece, BertNormalizer + BertPreTokenizer",
    4: "C4 shard: Zipf(64-4096 B) docs, 50k BPE, Whitespace",
}


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", type=int, default=1, help="0..4 = BASELINE.json configs")
    ap.add_argument("--docs", type=int, default=0, help="docs per rank (default: the config's size)")
    ap.add_argument("--cpu-sample-docs", type=int, default=1_000_000)
    ap.add_argument("--cpu-min-seconds", type=float, default=10.0, help="repeat the CPU sample until this long")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--verify", action="store_true", help="check the batch against the oracle (sample)")
    ap.add_argument("--no-memo", action="store_true", help="disable the BPE word memo (vocab-key results)")
    ap.add_argument("--share-gpu", action="store_true",
                    help="rehearsal only: every rank uses GPU 0 (multi-rank path on a 1-GPU box)")
    return ap.parse_args(argv)


def default_docs(cfg):
    return {0: 1000, 1: 1_000_000, 2: 1_000_000, 3: 1_000_000, 4: 1_000_000}[cfg]


class Dist:
    """Barrier / max-reduce over ranks (gloo; measurement only, not on the data path)."""

    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self.pg = None
        if self.world > 1:
            import torch.distributed as dist

            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("gloo", rank=self.rank, world_size=self.world)
            self.dist = dist

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()

    def max(self, x: float) -> float:
        if self.world == 1:
            return x
        import torch

        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum(self, x: float) -> float:
        if self.world == 1:
            return x
        import torch

        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return float(t.item())

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


def latest_pmc_entry(kernel="k_encode"):
    """(file, entry) of k_encode in the newest committed rocprofv3 PMC summary
    (profiles/*_pmc.json, written by tools/pmc_summary.py), else (None, {})."""
    pdir = os.path.join(REPO, "profiles")
    if not os.path.isdir(pdir):
        return None, {}
    cands = sorted(f for f in os.listdir(pdir) if f.endswith("_pmc.json"))
    for f in reversed(cands):
        try:
            d = json.load(open(os.path.join(pdir, f)))
            if kernel in d:
                return f, d[kernel]
        except Exception:
            continue
    return None, {}


def latest_pmc(kernel="k_encode"):
    """HBM traffic per k_encode launch from the newest committed PMC summary, else None."""
    return latest_pmc_entry(kernel)[1].get("hbm_bytes_per_launch")


def valu_issue(avg_launch_s):
    """k_encode's VALU issue rate against the measured gfx950 issue peak: SQ_INSTS_VALU per
    launch (newest committed PMC summary of the default C1 command) / this run's average
    launch time, over tools/valu_peak's wave-instructions/s at 5 waves per SIMD (k_encode's
    occupancy; profiles/*_valu_peak.jsonl). None when either file is missing."""
    f, e = latest_pmc_entry()
    valu = e.get("counters", {}).get("SQ_INSTS_VALU")
    pdir = os.path.join(REPO, "profiles")
    peaks = sorted(x for x in os.listdir(pdir) if x.endswith("_valu_peak.jsonl")) if os.path.isdir(pdir) else []
    if not valu or not peaks:
        return None
    peak = None
    for line in open(os.path.join(pdir, peaks[-1])):
        r = json.loads(line)
        if r.get("waves_per_simd") == 5:
            peak = r["valu_wave_instr_per_s"]
    if not peak:
        return None
    ach = valu / avg_launch_s
    return {"bound": "valu-issue", "achieved": float(f"{ach:.4e}"), "peak": peak, "unit": "wave-instr/s",
            "frac": round(ach / peak, 4), "valu_per_launch": valu, "pmc": f, "peak_source": peaks[-1]}


def cpu_baseline(cfg, js, n_sample, threads, min_seconds=10.0):
    """The C++ restatement of Tokenizer.encode (oracle/tkz_oracle.cpp) on the host cores:
    passes over a bounded sample of the same workload until `min_seconds` of CPU work."""
    from oracle import oracle as orc
    from tkz import synth

    ref = orc.RefTokenizer.from_json(js)
    co = orc.COracle(ref)
    data, off = synth.docs(cfg, n_sample, first_doc=0)
    passes, dt = 0, 0.0
    t0 = time.perf_counter()
    while passes < 1 or (dt < min_seconds and passes < 8):
        co.encode_batch(data, off, n_threads=threads)
        passes += 1
        dt = time.perf_counter() - t0
    nbytes = float(off[-1]) * passes
    return {"value": round(nbytes / dt / 1e6, 3), "unit": "MB/s", "cores": threads, "kind": "port",
            "sample": f"{passes} pass(es) over {n_sample} docs ({int(off[-1])} B) of the same workload, C++ "
                      f"restatement of Tokenizer.encode (oracle/tkz_oracle.cpp, -O3), {threads} threads, {dt:.2f} s"}


def main(argv=None):
    args = parse_args(argv)
    import tkz
    from tkz import synth

    dist = Dist()
    tkz.set_device(0 if args.share_gpu else dist.local_rank)
    cfg = args.config
    n_docs = args.docs or default_docs(cfg)
    js = synth.tokenizer_json(cfg)
    tok = tkz.Tokenizer.from_json(js)
    tok.set_word_memo(not args.no_memo)
    data, off = synth.docs(cfg, n_docs, first_doc=shard_first_doc(dist.rank, n_docs))
    total = int(off[-1])
    db = tkz.DeviceBatch(tok, data, off)

    # timed region: K full passes, inputs resident, kernel timers on the encode stream
    tkz.profile_enable(tok, True)
    elapsed = run_timed(db.run, db.sync, dist, args.steps, args.warmup)
    ms_enc, ms_def, ms_scan, ms_comp, ncalls = tkz.profile_read(tok)
    tkz.profile_enable(tok, False)
    row, ids, offs = db.results()
    n_tokens = int(row[-1])
    if args.verify and dist.rank == 0:
        from oracle import oracle as orc
        sel = slice(0, min(n_docs, 20000))
        co = orc.COracle(orc.RefTokenizer.from_json(js))
        sub_off = off[: sel.stop + 1]
        erow, eids, _ = co.encode_batch(data[: int(sub_off[-1])], sub_off, n_threads=8)
        assert np.array_equal(ids[: int(erow[-1])], eids), "parity failure"
    total_all = dist.sum(float(total))
    tokens_all = dist.sum(float(n_tokens))
    value = total_all * args.steps / elapsed / 1e6
    # roofline of the dominant kernel (k_encode), SURVEY.md 8(d): algorithmic bytes per
    # launch = input bytes + 12 B per token (u32 id + 2 x u32 offset) + 8 B per row_ptr entry
    avg_enc_s = (ms_enc / max(ncalls, 1)) / 1e3
    alg = total + 12 * n_tokens + 8 * (n_docs + 1)
    achieved = alg / avg_enc_s / 1e9
    # the committed PMC summaries are of the default C1 command; other workloads report null
    default_cmd = cfg == 1 and not args.no_memo and n_docs == default_docs(cfg)
    traffic = latest_pmc() if default_cmd else None
    out = {
        "metric": "input MB/s encode (bit-exact ids) at 1/2/4/8 MI355X vs Zig CPU baseline",
        "value": round(value, 2),
        "unit": "MB/s",
        "n_gpus": dist.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (deterministic generator, tokenizer-zig_amd/csrc/synth.cpp; vocab trained in-repo)",
        "config": {"workload": WORKLOADS[cfg], "docs_per_gpu": n_docs, "bytes_per_gpu": total,
                   "tokens_per_gpu": n_tokens, "tokens_all": int(tokens_all), "parallelism": f"doc-shard x{dist.world}",
                   "word_memo": not args.no_memo},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                     "frac_vs_measured_copy": round(achieved / HBM_COPY_GBS, 5),
                     "kernel": "k_encode", "avg_launch_ms": round(avg_enc_s * 1e3, 4),
                     "alg_bytes_per_launch": alg,
                     "other_kernels_ms": {"bpe_deferred": round(ms_def / max(ncalls, 1), 4),
                                          "count_scan": round(ms_scan / max(ncalls, 1), 4),
                                          "compact": round(ms_comp / max(ncalls, 1), 4)}},
        # k_encode is integer/indexing work bound by VALU issue, not HBM
        "issue_roofline": valu_issue(avg_enc_s) if default_cmd else None,
    }
    if dist.rank == 0 and dist.world == 1 and not args.no_cpu_baseline:
        th = args.cpu_threads or min(16, os.cpu_count() or 1)
        out["cpu_baseline"] = cpu_baseline(cfg, js, min(args.cpu_sample_docs, n_docs), th, args.cpu_min_seconds)
    elif dist.rank == 0:
        out["cpu_baseline"] = None
    db.free()
    dist.close()
    if dist.rank == 0:
        print(json.dumps(out), flush=True)
    return out


if __name__ == "__main__":
    main()
