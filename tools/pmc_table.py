"""Per-kernel table from a kernel-trace pass and a PMC pass of the same
command (rocprofv3 csv output): average duration, every counter's average per
dispatch, the effective shader clock (GRBM_GUI_ACTIVE / 8 XCDs / duration)
and the SQ breakdown as fractions of SQ_WAVE_CYCLES.
Usage: python tools/pmc_table.py <kt_dir> <pmc_dir> <kernel-substring>"""
import csv
import glob
import json
import sys
from collections import defaultdict


def main():
    kt, pmc, sub = sys.argv[1:4]
    durs = []
    for f in glob.glob(f"{kt}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if sub in r["Kernel_Name"]:
                durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    acc = defaultdict(list)
    meta = {}
    for f in glob.glob(f"{pmc}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if sub in r["Kernel_Name"]:
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
                meta = {k: r.get(k) for k in ("VGPR_Count", "Accum_VGPR_Count", "SGPR_Count", "LDS_Block_Size")}
    c = {k: sum(v) / len(v) for k, v in acc.items()}
    us = sum(durs) / len(durs)
    out = {"kernel": sub, "avg_us": round(us, 2), "n": len(durs), "regs": meta,
           "counters": {k: round(v, 1) for k, v in sorted(c.items())}}
    if "GRBM_GUI_ACTIVE" in c:
        out["eff_clock_ghz"] = round(c["GRBM_GUI_ACTIVE"] / 8 / (us * 1e3), 3)
    if "SQ_WAVE_CYCLES" in c:
        w = c["SQ_WAVE_CYCLES"]
        out["frac_of_wave_cycles"] = {k: round(c[k] / w, 3) for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                                                                       "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU")
                                      if k in c}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
