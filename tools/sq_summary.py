#!/usr/bin/env python3
"""Per-kernel SQ counter summary of the three `sq` passes of tools/gpu.sh
(<dir>/pmc/<set>_p{1,2,3}/**/*counter_collection.csv) -> JSON.

    python tools/sq_summary.py gpurun_out/r04/<tag> singles_real_0_span_tile_0_ profiles/r04/sq_k_interval.json

Counters are summed over the dispatches of a kernel, then divided by the dispatch count.
SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles summed over waves
(MI355X_MICROARCH.md, PMC table); WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES.
GRBM_GUI_ACTIVE is summed over the 8 XCDs: / 8 = the dispatch's duration in cycles (checked
against the HIP-event time of the same launches at ~2.1 GHz).  Derived (per wave, then per SIMD):
  issue_frac         ACTIVE_INST_ANY / WAVE_CYCLES   (a wave's life spent issuing)
  wait_frac          WAIT_ANY / WAVE_CYCLES          (parked on s_waitcnt / barrier)
  stall_frac         WAIT_INST_ANY / WAVE_CYCLES     (issue stalls: dependency, pipe busy)
  lds_stall_frac     WAIT_INST_LDS / WAVE_CYCLES
  valu_frac          ACTIVE_INST_VALU / WAVE_CYCLES
  cycles             GRBM_GUI_ACTIVE / 8
  waves_per_simd_counter  4 WAVE_CYCLES / (cycles x SIMDs holding the kernel's workgroups) (reads
                     ~0.7 x the resident waves for persistent kernels: a counter-unit caveat, use
                     the launch configuration for occupancy)
  fp64_busy          4 cycles x (FMA_F64 + ADD_F64 + MUL_F64) / (4 SIMDs x CUs in use x cycles)
  lds_busy           SQ_LDS_IDX_ACTIVE / (CUs in use x cycles)  (LDS-array cycles per CU cycle)
  lds_conflict_frac  SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  fp64_flop          64 x (2 FMA_F64 + ADD_F64 + MUL_F64) per dispatch (all lanes active assumed)
"""
import collections
import csv
import glob
import json
import re
import sys

N_CU = 256


def load(root, prefix):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    meta = {}
    for p in ("p1", "p2", "p3"):
        for f in glob.glob(f"{root}/pmc/{prefix}{p}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                name = re.sub(r"^void dse::\(anonymous namespace\)::", "", r["Kernel_Name"])
                name = re.sub(r"\(.*$", "", name)
                acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
                meta.setdefault(name, {"grid": int(r.get("Grid_Size", 0) or 0),
                                       "wg": int(r.get("Workgroup_Size", 0) or 0),
                                       "lds": int(r.get("LDS_Block_Size", 0) or 0),
                                       "vgpr": int(r.get("VGPR_Count", 0) or 0)})
    return acc, meta


def main():
    root, prefix, out = sys.argv[1], sys.argv[2], sys.argv[3]
    acc, meta = load(root, prefix)
    res = {}
    for k, cs in acc.items():
        c = {n: sum(v) / len(v) for n, v in cs.items()}
        m = meta[k]
        wgs = m["grid"] // max(m["wg"], 1) if m["wg"] else 0
        cus = min(max(wgs, 1), N_CU)
        simds = min(max(wgs, 1) * max(1, (m["wg"] + 63) // 64), 4 * cus)
        d = {"dispatches": max(len(v) for v in cs.values()), "workgroups": wgs, **m, "counters": c}
        wc = c.get("SQ_WAVE_CYCLES")
        gui = c.get("GRBM_GUI_ACTIVE")
        cyc = gui / 8.0 if gui else None
        if cyc:
            d["cycles"] = cyc
        if wc:
            for key, num in (("issue_frac", "SQ_ACTIVE_INST_ANY"), ("wait_frac", "SQ_WAIT_ANY"),
                             ("stall_frac", "SQ_WAIT_INST_ANY"), ("lds_stall_frac", "SQ_WAIT_INST_LDS"),
                             ("valu_frac", "SQ_ACTIVE_INST_VALU")):
                if num in c:
                    d[key] = c[num] / wc
        if wc and cyc:
            d["waves_per_simd_counter"] = 4.0 * wc / (cyc * simds)
        if cyc and "SQ_LDS_IDX_ACTIVE" in c:
            d["lds_busy"] = c["SQ_LDS_IDX_ACTIVE"] / (cus * cyc)
        if c.get("SQ_LDS_IDX_ACTIVE"):
            d["lds_conflict_frac"] = c.get("SQ_LDS_BANK_CONFLICT", 0.0) / c["SQ_LDS_IDX_ACTIVE"]
        if "SQ_INSTS_VALU_FMA_F64" in c:
            n64 = c["SQ_INSTS_VALU_FMA_F64"] + c.get("SQ_INSTS_VALU_ADD_F64", 0.0) + c.get("SQ_INSTS_VALU_MUL_F64", 0.0)
            d["fp64_flop"] = 64.0 * (n64 + c["SQ_INSTS_VALU_FMA_F64"])
            if cyc:
                d["fp64_busy"] = 4.0 * n64 / (4.0 * cus * cyc)
        res[k] = d
    rec = {"source": f"rocprofv3 --pmc, three SQ passes over tools/probe_one.py ({prefix.rstrip('_')})",
           "definitions": __doc__.split("Derived")[1].strip(), "kernels": res}
    with open(out, "w") as f:
        json.dump(rec, f, indent=1)
    for k, d in sorted(res.items(), key=lambda kv: -kv[1]["counters"].get("GRBM_GUI_ACTIVE", 0))[:3]:
        print(k, {x: round(d[x], 3) for x in ("waves_per_simd_counter", "issue_frac", "wait_frac", "stall_frac",
                                            "fp64_busy", "lds_busy", "lds_conflict_frac") if x in d})


if __name__ == "__main__":
    main()
