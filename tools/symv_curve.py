#!/usr/bin/env python3
"""Per-column time of k_trd_symv / k_trd_colref / k_trd_wfin against the trailing size m, from a
rocprofv3 kernel trace of `probe_sytrd <n> split` (three sytrd_lower runs; the last one is used):
bytes 8 m^2 / 2 per symv launch, GB/s by m band.   symv_curve.py <kernel_trace.csv> <n>"""
import csv
import sys

path, n = sys.argv[1], int(sys.argv[2])
rows = [r for r in csv.DictReader(open(path))]
key = "Kernel_Name" if "Kernel_Name" in rows[0] else "Name"
def pick(sub):
    xs = [r for r in rows if sub in r[key]]
    xs.sort(key=lambda r: int(r["Start_Timestamp"]))
    return xs
sym = pick("k_trd_symv")
per = len(sym) // 5  # split mode: warm-up eig_sym_lower, 3 timed sytrd_lower, 1 before dstedc
last = sym[-per:] if per else sym
cols = len(last)
print(f"symv launches {len(sym)}, per run {per}")
bands = [(0, 1024), (1024, 2048), (2048, 4096), (4096, 8192), (8192, 12288), (12288, 16385)]
tot_b = tot_t = 0.0
# column index c: launches in order, skipping the panel structure (every column has one symv)
for lo, hi in bands:
    b = t = 0.0
    k = 0
    for idx, r in enumerate(last):
        m = n - 1 - idx  # trailing size of the idx-th reduced column, approximately (panels are in order)
        if lo <= m < hi:
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
            b += 8.0 * m * m / 2
            t += d
            k += 1
    if k:
        print(f"m in [{lo},{hi}): {k} launches, avg {t / k * 1e6:.1f} us, {b / t / 1e9:.0f} GB/s")
        tot_b += b
        tot_t += t
print(f"all: {tot_t * 1e3:.1f} ms, {tot_b / tot_t / 1e9:.0f} GB/s")
for name in ("k_trd_colref", "k_trd_wfin"):
    xs = pick(name)[-per:]
    if xs:
        ds = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3 for r in xs]
        print(f"{name}: {len(xs)} launches, avg {sum(ds) / len(ds):.1f} us, first {sum(ds[:256]) / 256:.1f} us, last {sum(ds[-256:]) / 256:.1f} us")
# gaps between consecutive kernels of the last run on the stream
allk = [r for r in rows if int(r["Start_Timestamp"]) >= int(last[0]["Start_Timestamp"]) and
        int(r["End_Timestamp"]) <= int(last[-1]["End_Timestamp"]) + 10**6]
allk.sort(key=lambda r: int(r["Start_Timestamp"]))
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in allk) * 1e-6
span = (int(allk[-1]["End_Timestamp"]) - int(allk[0]["Start_Timestamp"])) * 1e-6
print(f"last run: span {span:.1f} ms, kernels busy {busy:.1f} ms, gaps {span - busy:.1f} ms over {len(allk)} launches")
