"""Summarise gpurun_out/whtvar: ms per H application and per-pass kernel averages."""
import csv
import glob
import json
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/whtvar"
for d in sorted(glob.glob(root + "/n*")):
    if d.endswith((".json", ".err")):
        continue
    f = glob.glob(d + "/*kernel_stats.csv")
    if not f:
        print(d, "missing")
        continue
    j = json.load(open(d + ".json"))
    print(d.split("/")[-1], "ms/H", round(j["ms_per_h_application"], 3))
    for r in csv.DictReader(open(f[0])):
        if "k_wht<" in r["Name"]:
            print("   ", r["Name"].split("<")[1][:5], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1))
