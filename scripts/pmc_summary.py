"""Per-kernel summary of rocprofv3 --pmc counter CSVs: python scripts/pmc_summary.py OUT (passes under OUT/*/).
PMC_AFTER=<regex>: only dispatches after the last one whose kernel matches (e.g. 'gg::' drops the GPU garbler's
dispatches of kernels it shares with the evaluator, such as k_conv_img2; the collection regex must include it)."""
import csv, glob, os, sys, re
from collections import defaultdict
N_SIMD = 256 * 4   # MI355X: 256 CUs x 4 SIMDs
CLOCK_HZ = 2.4e9   # peak engine clock (MI355X_MICROARCH.md)
out = sys.argv[1]
agg = defaultdict(lambda: defaultdict(float))
ms = defaultdict(float)
nd = defaultdict(int)
for f in glob.glob(f"{out}/*/**/*counter_collection.csv", recursive=True):
    seen = set()
    pas = f[len(out) + 1:].split("/")[0]
    rows = list(csv.DictReader(open(f)))
    after = os.environ.get("PMC_AFTER")
    cut = max((int(r["Dispatch_Id"]) for r in rows if after and re.search(after, r["Kernel_Name"])), default=-1)
    for r in rows:
        if after and (int(r["Dispatch_Id"]) <= cut or re.search(after, r["Kernel_Name"])):
            continue
        k = re.sub(r"\(.*", "", r["Kernel_Name"])
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        key = r["Dispatch_Id"]
        if key not in seen:
            seen.add(key)
            ms[(k, pas)] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            nd[(k, pas)] += 1
for k, c in sorted(agg.items()):
    print(k)
    for n, v in sorted(c.items()):
        print(f"   {n:28s} {v:18.0f}")
    g = c.get
    if g("SQ_INSTS_LDS"):
        print(f"   {'lds_bank_conflict_per_lds':28s} {g('SQ_LDS_BANK_CONFLICT', 0) / max(1, g('SQ_ACTIVE_INST_LDS', 1)):18.3f}")
    if g("SQ_VALU_MFMA_BUSY_CYCLES") is not None:
        # SQ_VALU_MFMA_BUSY_CYCLES is summed over every SIMD of the chip (cycles, not quad-cycles), so it is
        # normalised by the SIMD count times the kernel's elapsed cycles (dispatch time x engine clock). The
        # round-5 form divided it by SQ_BUSY_CYCLES (one sequencer's busy cycles) and reported up to 352 %.
        dur_s = sum(v for (kk, _), v in ms.items() if kk == k) / 1e3 / max(1, len({p for (kk, p) in ms if kk == k}))
        if dur_s > 0:
            util = g("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (N_SIMD * dur_s * CLOCK_HZ)
            print(f"   {'mfma_util_pct':28s} {100 * util:18.2f}")
            if g("SQ_INSTS_VALU_MFMA_MOPS_I8"):
                # MOPS counters count in units of 512 operations; dense int8 peak = 2x the bf16 rate, ~5.0 P/s
                tops = g("SQ_INSTS_VALU_MFMA_MOPS_I8") * 512 / dur_s / 1e12
                print(f"   {'int8_tops':28s} {tops:18.2f}")
                print(f"   {'int8_pct_of_dense_peak':28s} {100 * tops / 5000:18.2f}")
    if g("SQ_WAVE_CYCLES"):
        print(f"   {'wait_any_pct':28s} {100 * g('SQ_WAIT_ANY', 0) / g('SQ_WAVE_CYCLES'):18.2f}")
        print(f"   {'wait_lds_pct':28s} {100 * g('SQ_WAIT_INST_LDS', 0) / g('SQ_WAVE_CYCLES'):18.2f}")
for (k, p), v in sorted(ms.items()):
    print(f"{k} pass={p} {v:.3f} ms {nd[(k, p)]} dispatches")
