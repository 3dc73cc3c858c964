"""Per-launch averages of the counters tools/bisect_pmc.sh collected, per library and kernel.
usage: python tools/bisect_summary.py gpurun_out/bisect [kernel-substring ...]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    root = sys.argv[1]
    pats = sys.argv[2:] or ["k_encode", "k_bpe_deferred", "k_compact", "k_dedup"]
    for d in sorted(glob.glob(os.path.join(root, "c*_*"))):
        if not os.path.isdir(d):
            continue
        files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        if not files:
            continue
        acc = defaultdict(lambda: defaultdict(float))
        disp = defaultdict(set)
        dur = defaultdict(dict)
        for f in files:
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"].split("(")[0].split("<")[0].replace("(anonymous namespace)::", "")
                k = k.split("::")[-1]
                if not any(p in k for p in pats):
                    continue
                acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[k].add(r["Dispatch_Id"])
                dur[k][r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        for k in sorted(acc):
            n = len(disp[k])
            c = {x: v / n for x, v in acc[k].items()}
            wc = c.get("SQ_WAVE_CYCLES", 0.0)
            if "SQ_INSTS_VALU" in c:
                print(f"{os.path.basename(d):24s} {k:16s} n={n:2d} ms={sum(dur[k].values()) / n:7.4f} "
                      f"VALU={c.get('SQ_INSTS_VALU', 0) / 1e6:8.2f}M SALU={c.get('SQ_INSTS_SALU', 0) / 1e6:8.2f}M "
                      f"LDS={c.get('SQ_INSTS_LDS', 0) / 1e6:6.2f}M wait={c.get('SQ_WAIT_ANY', 0) / wc if wc else 0:5.3f}")
            else:
                print(f"{os.path.basename(d):24s} {k:16s} n={n:2d} ms={sum(dur[k].values()) / n:7.4f} " +
                      " ".join(f"{x}={v / 1e6:.2f}M" for x, v in sorted(c.items())))


if __name__ == "__main__":
    main()
