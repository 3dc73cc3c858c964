"""Summarise rocprofv3 --pmc counter CSVs per kernel.

usage: python tools/pmc_summary.py gpurun_out/pmc_<tag> [profiles/<tag>_pmc.json]

Per kernel: mean counter value per dispatch over all passes (p1..pN), bench-sized
launches only (largest grid). For k_encode the
HBM traffic per launch is derived as the MI355X_MICROARCH.md §HBM recipe prescribes:
FETCH_SIZE and WRITE_SIZE are KiB; gfx950 FETCH_SIZE counts half of the bytes of a wide
coalesced streaming read, so the read side is doubled (hbm = (2*FETCH_SIZE +
WRITE_SIZE) * 1024). The raw undoubled sum is reported beside it.
"""
import collections
import csv
import glob
import json
import os
import sys


def short(name: str) -> str:
    n = name.split("(")[0].replace("void ", "")
    return n.split("::")[-1].split("<")[0] if "::" in n else n


def main():
    d = sys.argv[1]
    out = sys.argv[2] if len(sys.argv) > 2 else None
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    durs = collections.defaultdict(list)
    rows = []
    for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
        rows += list(csv.DictReader(open(f)))
    # only the bench-sized launches of each kernel (the word-memo build at table upload
    # launches the same kernels on a small grid)
    gmax = collections.defaultdict(int)
    for row in rows:
        gmax[short(row["Kernel_Name"])] = max(gmax[short(row["Kernel_Name"])], int(row["Grid_Size"]))
    for row in rows:
        k = short(row["Kernel_Name"])
        if int(row["Grid_Size"]) != gmax[k]:
            continue
        vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
        durs[k].append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    res = {}
    for k, cs in vals.items():
        res[k] = {c: sum(v) / len(v) for c, v in cs.items()}
    for k in sorted(res, key=lambda k: -sum(durs[k])):
        print(f"== {k}")
        for c, v in sorted(res[k].items()):
            print(f"   {c:28s} {v:18.1f}")
    enc = res.get("k_encode", {})
    summary = {}
    for extra in ("src_hash", "cmd"):
        f = os.path.join(d, f"{extra}.txt")
        if os.path.exists(f):
            summary[extra] = open(f).read().strip()
    for k, cs in res.items():  # HBM bytes of every kernel with both counters
        if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs and k != "k_encode":
            summary[k] = {"hbm_bytes_per_launch": int((2 * cs["FETCH_SIZE"] + cs["WRITE_SIZE"]) * 1024),
                          "FETCH_SIZE_KiB": cs["FETCH_SIZE"], "WRITE_SIZE_KiB": cs["WRITE_SIZE"], "counters": cs,
                          "avg_ns": sum(durs[k]) / max(len(durs[k]), 1)}
    if "FETCH_SIZE" in enc and "WRITE_SIZE" in enc:
        summary["k_encode"] = {
            "hbm_bytes_per_launch": int((2 * enc["FETCH_SIZE"] + enc["WRITE_SIZE"]) * 1024),
            "raw_fetch_plus_write_bytes": int((enc["FETCH_SIZE"] + enc["WRITE_SIZE"]) * 1024),
            "FETCH_SIZE_KiB": enc["FETCH_SIZE"],
            "WRITE_SIZE_KiB": enc["WRITE_SIZE"],
            "counters": enc,
        }
        print(json.dumps(summary["k_encode"], indent=1)[:400])
    if out:
        json.dump(summary, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
