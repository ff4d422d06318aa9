"""Aggregate rocprofv3 --pmc CSV output per kernel.

Usage: python -m dash_amd.utils.pmcsum <counter_collection.csv> [more.csv ...]
Prints per kernel: dispatches, summed time, and per-counter totals; with the
SQ counters it derives VALU-active / wait / issue-stall fractions of wave
cycles and (with FETCH_SIZE) the achieved fetch bandwidth.
"""
from __future__ import annotations

import csv
import re
import sys
from collections import defaultdict


def load(paths):
    agg = defaultdict(lambda: defaultdict(float))
    times = defaultdict(dict)
    cpass = defaultdict(dict)  # kernel -> counter -> pass (file) it was collected in
    for p in paths:
        with open(p) as f:
            for r in csv.DictReader(f):
                k = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")
                agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
                cpass[k][r["Counter_Name"]] = p
                times[k][(p, r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    return agg, times, cpass


def main(paths):
    agg, times, cpass = load(paths)
    rows = []
    for k, c in agg.items():
        # time per pass: counters of different passes come from different dispatches
        ms_by_pass = defaultdict(float)
        for (p, _), ms in times[k].items():
            ms_by_pass[p] += ms
        ms = max(ms_by_pass.values()) if ms_by_pass else 0.0
        wc = c.get("SQ_WAVE_CYCLES", 0.0)
        d = {"kernel": k, "ms": ms, "dispatch": len(times[k]) // max(1, len(ms_by_pass))}
        if wc:
            d["valu%"] = 100 * c.get("SQ_ACTIVE_INST_VALU", 0) / wc
            d["active%"] = 100 * c.get("SQ_ACTIVE_INST_ANY", 0) / wc
            d["wait%"] = 100 * c.get("SQ_WAIT_ANY", 0) / wc
            d["stall%"] = 100 * c.get("SQ_WAIT_INST_ANY", 0) / wc
        if c.get("SQ_WAVES"):
            d["valu_insts/wave"] = c.get("SQ_INSTS_VALU", 0) / c["SQ_WAVES"]
            d["vmem_rd/wave"] = c.get("SQ_INSTS_VMEM_RD", 0) / c["SQ_WAVES"]
            for ctr, name in (("SQ_INSTS_VMEM_WR", "vmem_wr/wave"), ("SQ_INSTS_LDS", "lds/wave"),
                              ("SQ_INSTS_SALU", "salu/wave")):
                if ctr in c:
                    d[name] = c[ctr] / c["SQ_WAVES"]
            for ctr, name in (("SQ_ACTIVE_INST_LDS", "lds_act%"), ("SQ_ACTIVE_INST_SCA", "salu_act%"),
                              ("SQ_INST_CYCLES_VMEM", "vmem_cyc%"), ("SQ_WAIT_INST_LDS", "wait_lds%")):
                if ctr in c:
                    d[name] = 100 * c[ctr] / wc
        if c.get("SQ_WAVES") and "SQ_IFETCH" in c:
            d["ifetch/wave"] = c["SQ_IFETCH"] / c["SQ_WAVES"]
        if c.get("SQ_ACTIVE_INST_LDS"):
            d["lds_conf%"] = 100 * c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_ACTIVE_INST_LDS"]
        for ctr, name in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
            if ctr in c and ms_by_pass:
                pms = ms_by_pass.get(cpass[k][ctr], ms)  # time of the pass that collected this counter
                d[f"{name}_GB"] = c[ctr] * 1024 / 1e9
                d[f"{name}_TB/s"] = d[f"{name}_GB"] / max(pms, 1e-9)
        rows.append(d)
    rows.sort(key=lambda r: -r["ms"])
    cols = ["kernel", "ms", "dispatch", "valu%", "active%", "wait%", "stall%", "valu_insts/wave", "vmem_rd/wave",
            "vmem_wr/wave", "lds/wave", "salu/wave", "lds_conf%", "lds_act%", "salu_act%", "vmem_cyc%", "wait_lds%",
            "ifetch/wave", "fetch_GB", "fetch_TB/s", "write_GB", "write_TB/s"]
    cols = [c for c in cols if c == "kernel" or any(c in r for r in rows)]
    print(" ".join(f"{c:>14s}" if c != "kernel" else f"{c:40s}" for c in cols))
    for r in rows[:25]:
        out = []
        for c in cols:
            v = r.get(c, "")
            out.append(f"{v[:40]:40s}" if c == "kernel" else (f"{v:14.2f}" if isinstance(v, float) else f"{str(v):>14s}"))
        print(" ".join(out))


if __name__ == "__main__":
    main(sys.argv[1:])
