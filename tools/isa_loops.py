#!/usr/bin/env python3
"""Instruction mix of every loop of one kernel in a gfx950 .s file (hipcc --save-temps):
    python3 tools/isa_loops.py <file.s> <kernel-name-substring>"""
import re
import sys

s = open(sys.argv[1]).read()
names = re.findall(r"^(\S*" + re.escape(sys.argv[2]) + r"\S*):", s, re.M)
name = names[0]
body = s[s.index(name + ":"):]
body = body[:body.index(".Lfunc_end")]
lines = body.splitlines()
labels = {}
for i, ln in enumerate(lines):
    m = re.match(r"^(\.LBB\S+):", ln)
    if m:
        labels[m.group(1)] = i
PAT = {"fma64": r"v_fma_f64|v_fmac_f64", "mul64": r"v_mul_f64", "add64": r"v_add_f64",
       "ds_read": r"ds_read", "ds_write": r"ds_write", "waitcnt": r"s_waitcnt", "vmem": r"buffer_|global_",
       "lane": r"v_readlane|v_writelane|v_readfirstlane", "valu": r"^\s+v_", "salu": r"^\s+s_"}
print(name, len(lines), "lines")
for i, ln in enumerate(lines):
    m = re.search(r"s_cbranch_\w+\s+(\.LBB\S+)|s_branch\s+(\.LBB\S+)", ln)
    if not m:
        continue
    t = m.group(1) or m.group(2)
    if t in labels and labels[t] < i:
        seg = lines[labels[t]:i + 1]
        cnt = {k: sum(1 for x in seg if re.search(p, x)) for k, p in PAT.items()}
        print(f"loop {t} [{labels[t]}-{i}] n={len(seg)} " + " ".join(f"{k}={v}" for k, v in cnt.items()))
