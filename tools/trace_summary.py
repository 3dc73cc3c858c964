"""Per-kernel, per-grid average durations from a rocprofv3 --kernel-trace CSV.

usage: python tools/trace_summary.py <run_kernel_trace.csv>
The word-memo build at table upload launches the encode kernels on a small grid; the
bench-sized launches are the largest grid of each kernel (compare with bench.py's
HIP-event averages)."""
import collections
import csv
import sys

d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"].split("(")[0].replace("void ", "")
    d[(n, int(r["Grid_Size_X"]))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
print(f"{'kernel':40s} {'grid':>9s} {'calls':>5s} {'avg ms':>9s}")
for (n, g), v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    print(f"{n:40s} {g:9d} {len(v):5d} {sum(v) / len(v):9.4f}")
