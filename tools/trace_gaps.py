#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace of bench.py's sweep leg: per-stream launch pattern of one
interval group, the gap between steps and what fills it.
    python tools/trace_gaps.py gpurun_out/.../bench_kernel_trace.csv"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
rows.sort(key=lambda r: r["s"])
iv = [r for r in rows if "k_interval" in r["Kernel_Name"]]
streams = collections.Counter(r["Stream_Id"] for r in iv)
crit = max(streams, key=lambda s: sum(r["e"] - r["s"] for r in iv if r["Stream_Id"] == s))
civ = [r for r in iv if r["Stream_Id"] == crit]
gaps = [i for i in range(1, len(civ)) if civ[i]["s"] - civ[i - 1]["e"] > 300000]
print("interval launches per stream", dict(streams), "critical stream", crit)
per = collections.defaultdict(list)
for r in rows:
    per[(r["Stream_Id"], r["Kernel_Name"][:40])].append(r["e"] - r["s"])
for k, v in sorted(per.items()):
    print(f"  stream {k[0]} {k[1]:40s} n={len(v):5d} avg={sum(v)/len(v)/1e3:9.1f} us")
for gi in gaps:
    a, b = civ[gi - 1]["e"], civ[gi]["s"]
    print(f"step gap before launch {gi}: {(b - a)/1e3:.1f} us; GPU ops inside (stream, name, start, duration in us after the last launch):")
    for r in rows:
        if a <= r["s"] <= b:
            print(f"    {r['Stream_Id']} {r['Kernel_Name'][:30]:30s} {(r['s'] - a)/1e3:9.1f} {(r['e'] - r['s'])/1e3:8.1f}")
if len(gaps) >= 2:
    spans = [(civ[gaps[j + 1] - 1]["e"] - civ[gaps[j]]["s"]) / 1e3 for j in range(len(gaps) - 1)]
    print("first-to-last launch span per step (us):", [round(x) for x in spans])
    busy = sum(r["e"] - r["s"] for r in civ[gaps[0]:gaps[1]]) / 1e3
    print(f"critical-stream interval kernel time in one step: {busy:.0f} us")
