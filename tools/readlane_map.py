#!/usr/bin/env python3
"""Where a kernel's SGPR spill reloads are: v_readlane / v_writelane instructions of one
kernel in the gfx950 assembly (built with -g), counted per source line.

usage: python tools/readlane_map.py [kernel-symbol-substring] (default: k_encode<1,true>)"""
import collections
import re
import subprocess
import sys

SRC = "tokenizer-zig_amd/csrc/encode.hip"
sym = sys.argv[1] if len(sys.argv) > 1 else "_ZN3tkz8k_encodeILi1ELb1EE"
subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-g", "-std=c++17", "--offload-arch=gfx950", "-DTKZ_MAXB=24",
                "--cuda-device-only", "-S", SRC, "-o", "/tmp/readlane_map.s"], check=True, capture_output=True)
s = open("/tmp/readlane_map.s").read()
files = {m.group(1): m.group(2) for m in re.finditer(r'\.file\s+(\d+)\s+"[^"]*"\s+"([^"]+)"', s)}
i = next(m.start() for m in re.finditer(r"^(\S+):", s, re.M) if sym in m.group(1))
body = s[i:s.index(".Lfunc_end", i)].split("\n")
cur, rl, wl, total = None, collections.Counter(), collections.Counter(), 0
for line in body:
    t = line.strip()
    m = re.match(r"\.loc\s+(\d+)\s+(\d+)", t)
    if m:
        cur = (files.get(m.group(1), m.group(1)).split("/")[-1], int(m.group(2)))
        continue
    if line.startswith("\t") and t and not t.startswith((";", ".")):
        total += 1
    if t.startswith("v_readlane_b32"):
        rl[cur] += 1
    if t.startswith("v_writelane_b32"):
        wl[cur] += 1
src = open(SRC).read().split("\n")
print(f"{total} instructions, {sum(rl.values())} v_readlane, {sum(wl.values())} v_writelane")
for (f, ln), n in rl.most_common(20):
    text = src[ln - 1].strip()[:90] if f == SRC.split("/")[-1] and ln > 0 else ""
    print(f"{n:4d}  {f}:{ln}  {text}")
