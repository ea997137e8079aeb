#!/usr/bin/env python3
"""Per-kernel HBM-side traffic from the FETCH_SIZE / WRITE_SIZE counter passes of
tools/gpu_profile.sh (gpurun_out/prof/{fetch,write}/*_counter_collection.csv) -> JSON.

    python tools/pmc_summary.py gpurun_out/prof profiles/r01/v7_pmc_traffic.json ["<profiled command>"]

rocprofv3 reports kB per dispatch.  FETCH_SIZE is doubled: on gfx950 it counts 1/2 of a wide
(16 B per lane) streaming read (MI355X_MICROARCH.md, HBM section); WRITE_SIZE as reported.
bench.py reads "traffic_bytes_per_launch" of its dominant kernel from the committed file.
"""
import collections
import csv
import glob
import json
import re
import sys


def per_kernel(path):
    d = collections.defaultdict(list)
    for f in glob.glob(path):
        for r in csv.DictReader(open(f)):
            name = re.sub(r"^void dse::\(anonymous namespace\)::", "", r["Kernel_Name"])
            name = re.sub(r"\(.*$", "", name)
            d[name].append(float(r["Counter_Value"]) * 1024.0)
    return d


def main():
    root, out = sys.argv[1], sys.argv[2]
    cmd = sys.argv[3] if len(sys.argv) > 3 else "python3 bench.py --no-cpu-baseline --steps 1 --warmup 0"
    fe = per_kernel(root + "/fetch/*counter_collection.csv")
    wr = per_kernel(root + "/write/*counter_collection.csv")
    kernels = {}
    for k in sorted(set(fe) | set(wr)):
        f = sum(fe.get(k, [0.0])) / max(len(fe.get(k, [])), 1)
        w = sum(wr.get(k, [0.0])) / max(len(wr.get(k, [])), 1)
        kernels[k] = {"launches": len(fe.get(k, [])), "fetch_bytes_raw": f, "fetch_bytes_corrected": 2 * f,
                      "write_bytes": w, "traffic_bytes_per_launch": 2 * f + w}
    rec = {
        "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes, over "
                  f"`{cmd}` (tools/gpu.sh traffic / traffic_large)",
        "units": "bytes per launch (rocprofv3 reports kB)",
        "gfx950_correction": "FETCH_SIZE doubled: it counts 1/2 of a wide (16 B/lane) streaming read on "
                             "gfx950 (MI355X_MICROARCH.md, HBM section); WRITE_SIZE as reported",
        "note": "L2 <-> fabric bytes (Infinity Cache hits included). k_interval: dominated by the per-term "
                "sc1 hand-off of the 2-tile problems, not by the H terms, which stay on chip",
        "kernels": kernels,
    }
    with open(out, "w") as fh:
        json.dump(rec, fh, indent=1)
    for k, v in kernels.items():
        print(f"{k:40s} {v['launches']:6d} {v['traffic_bytes_per_launch'] / 1e6:12.1f} MB/launch")


if __name__ == "__main__":
    main()
