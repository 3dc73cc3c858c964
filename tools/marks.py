"""Static instruction counts of k_encode<BPE, compact> per phase marker (-DTKZ_MARKS asm
listing): VALU / SALU / LDS / VMEM / SMEM instructions between consecutive markers, in
listing order. Compares the working tree with a git revision.
usage: python tools/marks.py [REV]"""
import os
import re
import subprocess
import sys
import tempfile
from collections import Counter, OrderedDict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def asm(src_dir, inc_dir):
    out = tempfile.mktemp(suffix=".s")
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S",
                    "-DTKZ_MAXB=24", "-DTKZ_MARKS", "-Wno-unused-result", "-Wno-unused-value", "-I", inc_dir,
                    os.path.join(src_dir, "encode.hip"), "-o", out], check=True, stderr=subprocess.DEVNULL)
    return open(out).read()


def classify(ins):
    if ins.startswith("v_readlane") or ins.startswith("v_readfirstlane") or ins.startswith("v_writelane"):
        return "XLANE"
    if ins.startswith("v_"):
        return "VALU"
    if ins.startswith("s_load") or ins.startswith("s_buffer"):
        return "SMEM"
    if ins.startswith("s_waitcnt") or ins.startswith("s_nop"):
        return "WAIT"
    if ins.startswith("s_"):
        return "SALU"
    if ins.startswith("ds_"):
        return "LDS"
    if ins.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "VMEM"
    return None


def phases(text, kernel="_ZN3tkz8k_encodeILi1ELb1E"):
    starts = [(m.start(), m.group(1)) for m in re.finditer(r"^(_ZN3tkz\w+):", text, re.M)]
    body = ""
    for i, (p, n) in enumerate(starts):
        if n.startswith(kernel):
            body = text[p:starts[i + 1][0] if i + 1 < len(starts) else len(text)]
    res = OrderedDict()
    cur = "prologue"
    for line in body.split("\n"):
        m = re.search(r"TKZ_MARK (.*)$", line)
        if m:
            cur = m.group(1).strip()
            continue
        t = line.strip().split()
        if not t or t[0].startswith((".", ";")) or t[0].endswith(":"):
            continue
        c = classify(t[0])
        if c:
            res.setdefault(cur, Counter())[c] += 1
    return res


def main():
    cur = phases(asm(os.path.join(REPO, "tokenizer-zig_amd", "csrc"), os.path.join(REPO, "include")))
    old = None
    if len(sys.argv) > 1:
        d = tempfile.mkdtemp()
        os.makedirs(os.path.join(d, "csrc"))
        os.makedirs(os.path.join(d, "include"))
        for f in ("encode.hip", "encode.hpp", "tables.hpp"):
            r = subprocess.run(["git", "-C", REPO, "show", f"{sys.argv[1]}:tokenizer-zig_amd/csrc/{f}"], capture_output=True)
            if r.returncode == 0:
                open(os.path.join(d, "csrc", f), "wb").write(r.stdout)
        r = subprocess.run(["git", "-C", REPO, "show", f"{sys.argv[1]}:include/tkz.h"], capture_output=True)
        open(os.path.join(d, "include", "tkz.h"), "wb").write(r.stdout)
        old = phases(asm(os.path.join(d, "csrc"), os.path.join(d, "include")))
    keys = list(cur) + [k for k in (old or {}) if k not in cur]
    for k in keys:
        a = cur.get(k, Counter())
        line = f"{k:14s} " + " ".join(f"{c}={a[c]:5d}" for c in ("VALU", "SALU", "XLANE", "LDS", "VMEM", "SMEM"))
        if old is not None:
            b = old.get(k, Counter())
            line += "   | old " + " ".join(f"{c}={b[c]:5d}" for c in ("VALU", "SALU", "XLANE", "LDS", "VMEM"))
        print(line)


if __name__ == "__main__":
    main()
