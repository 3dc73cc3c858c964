"""Summarise rocprofv3 --pmc counter CSVs (tools/pmc.sh) per kernel and per encode step.

usage: python tools/pmc_summary.py gpurun_out/pmc_<name> [profiles/<tag>_pmc.json] [--calib]

Bench mode (default): the encode calls of the timed steps are the dispatches from the
k_chunk_docs before the first bench-sized k_encode (largest grid; the word-memo build at
table upload runs the same kernels on a small batch) to the last k_compact. Per kernel:
the mean counter value per dispatch; per step: the sum over the step's kernels of mean x
dispatches per step.

HBM bytes (MI355X_MICROARCH.md §HBM; counter_defs.yaml for gfx950):
  FETCH_SIZE = (BUBBLE*128 + (RDREQ - BUBBLE - RDREQ_32B)*64 + RDREQ_32B*32) / 1024 KiB
counts a 128-B request as 64 B (the guide's "exactly 1/2 of a wide streaming read").
The request-size counters give the read bytes without a blanket factor:
  read_bytes = 32*RDREQ_32B + 64*RDREQ_64B + 128*RDREQ_128B
  write_bytes = WRITE_SIZE*1024 = 32*(WRREQ - WRREQ_64B) + 64*WRREQ_64B
and `bytes` = read_bytes + write_bytes. tools/fetch_calib.hip checks both against known
byte counts on the encode kernels' access patterns (--calib mode: one row per kernel,
last dispatch of each name, with the nominal bytes from the program's stdout log).
"""
import collections
import csv
import glob
import json
import os
import re
import sys

STEP_KERNELS = ("k_chunk_docs", "k_encode", "k_encode_blk", "k_bpe_short", "k_dedup", "k_bpe_deferred", "k_bpe_long", "k_dedup_copy",
                "k_scan_partials", "k_scan_top", "k_scan_final", "k_compact", "k_compact_long",
                "__amd_rocclr_fillBufferAligned")


def short(name: str) -> str:
    n = name.split("(")[0].replace("void ", "").strip()
    n = n.split("::")[-1] if "::" in n else n
    return n.split("<")[0] if not n.startswith("rand_rd") else n.replace(" ", "")


def derive(cs: dict) -> dict:
    """HBM bytes of one dispatch from its counters (whatever subset was collected)."""
    out = {}
    if "FETCH_SIZE" in cs:
        out["fetch_size_bytes"] = cs["FETCH_SIZE"] * 1024
    if "WRITE_SIZE" in cs:
        out["write_bytes"] = cs["WRITE_SIZE"] * 1024
    if all(k in cs for k in ("TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum")):
        out["read_bytes"] = (32 * cs["TCC_EA0_RDREQ_32B_sum"] + 64 * cs["TCC_EA0_RDREQ_64B_sum"] +
                             128 * cs["TCC_EA0_RDREQ_128B_sum"])
        if "TCC_EA0_RDREQ_sum" in cs:
            out["rdreq_unsized"] = cs["TCC_EA0_RDREQ_sum"] - (cs["TCC_EA0_RDREQ_32B_sum"] + cs["TCC_EA0_RDREQ_64B_sum"] +
                                                               cs["TCC_EA0_RDREQ_128B_sum"])
    if "read_bytes" in out and "write_bytes" in out:
        out["bytes"] = out["read_bytes"] + out["write_bytes"]
    if "fetch_size_bytes" in out and "write_bytes" in out:
        out["raw_fetch_plus_write"] = out["fetch_size_bytes"] + out["write_bytes"]
    return {k: int(v) for k, v in out.items()}


def load_passes(d):
    """[(rows of one pass sorted by dispatch), ...]; a row = (dispatch, kernel, grid, {counter: value}, ns)."""
    passes = []
    for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
        disp = {}
        for row in csv.DictReader(open(f)):
            did = int(row.get("Dispatch_Id") or row.get("Correlation_Id") or 0)
            e = disp.setdefault(did, [did, short(row["Kernel_Name"]), int(row["Grid_Size"]), {},
                                      int(row["End_Timestamp"]) - int(row["Start_Timestamp"])])
            e[3][row["Counter_Name"]] = e[3].get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
        passes.append(sorted(disp.values()))
    return passes


def bench_window(rows):
    """The dispatches of the timed encode calls and the number of calls."""
    enc = [r for r in rows if r[1] in ("k_encode", "k_encode_blk")]
    if not enc:
        return [], 0
    gmax = max(r[2] for r in enc)
    big = [r for r in enc if r[2] == gmax]
    first = big[0][0]
    chunk_docs = [r[0] for r in rows if r[1] == "k_chunk_docs" and r[0] < first]
    lo = chunk_docs[-1] if chunk_docs else first
    hi = max(r[0] for r in rows if r[1] == "k_compact")
    return [r for r in rows if lo <= r[0] <= hi], len(big)


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    calib = "--calib" in sys.argv
    d = args[0]
    out = args[1] if len(args) > 1 else None
    passes = load_passes(d)
    summary = {}
    for extra in ("src_hash", "cmd"):
        f = os.path.join(d, f"{extra}.txt")
        if os.path.exists(f):
            summary[extra] = open(f).read().strip()
    if calib:
        # the measured dispatches of the last repetition, in launch order (the evictions and
        # the MALL warm-up rand_rd<1> excluded), matched to the program's lines in order
        nominal = []
        for line in open(sorted(glob.glob(os.path.join(d, "p*.log")))[0]):
            if line.startswith("{"):
                j = json.loads(line)
                nominal.append((j["kernel"], j["bytes"]))
        merged = [dict() for _ in nominal]
        for rows in passes:
            meas = [r for r in rows if r[1] not in ("evict", "rand_rd<1>")][-len(nominal):]
            for m, r in zip(merged, meas):
                m.update(r[3])
        for (k, b), cs in zip(nominal, merged):
            dv = derive(cs)
            row = {"nominal_bytes": b, **dv, "counters": {c: v for c, v in cs.items() if not c.startswith("_")}}
            for key in ("fetch_size_bytes", "read_bytes", "write_bytes"):
                if key in dv and b:
                    row[key.replace("_bytes", "") + "_ratio"] = round(dv[key] / b, 4)
            summary[k] = row
            print(k, json.dumps({x: row.get(x) for x in ("nominal_bytes", "fetch_size_ratio", "read_ratio",
                                                          "write_ratio")}))
    else:
        per = collections.defaultdict(lambda: collections.defaultdict(list))
        cnt = collections.defaultdict(list)
        ns = collections.defaultdict(list)
        n_calls = 0
        for rows in passes:
            win, calls = bench_window(rows)
            n_calls = max(n_calls, calls)
            c = collections.Counter(r[1] for r in win)
            for r in win:
                for k, v in r[3].items():
                    per[r[1]][k].append(v)
                ns[r[1]].append(r[4])
            for k, v in c.items():
                cnt[k].append(v / max(calls, 1))
        step = collections.defaultdict(float)
        for k in per:
            cs = {c: sum(v) / len(v) for c, v in per[k].items()}
            launches = sum(cnt[k]) / max(len(cnt[k]), 1)
            dv = derive(cs)
            summary[k] = {**dv, "launches_per_step": launches, "avg_ns": sum(ns[k]) / max(len(ns[k]), 1),
                          "counters": cs}
            if k in STEP_KERNELS:
                for key, v in dv.items():
                    step[key] += v * launches
        summary["step"] = {k: int(v) for k, v in step.items()}
        summary["step"]["calls"] = n_calls
        for k in sorted(summary, key=lambda k: -summary[k].get("bytes", 0) if isinstance(summary[k], dict) else 0):
            if isinstance(summary[k], dict):
                print(k, {x: summary[k].get(x) for x in ("bytes", "read_bytes", "fetch_size_bytes", "write_bytes",
                                                        "launches_per_step")})
    if out:
        json.dump(summary, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
