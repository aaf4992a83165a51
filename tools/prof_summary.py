"""Condense rocprofv3 outputs from gpurun_out/ into profiles/<round>/.

    python tools/prof_summary.py r01

Reads
  gpurun_out/prof_kt/bench_kernel_stats.csv      (--kernel-trace --stats)
  gpurun_out/prof_kt/bench_kernel_trace.csv
  gpurun_out/prof_fetch/bench_counter_collection.csv   (--pmc FETCH_SIZE)
  gpurun_out/prof_write/bench_counter_collection.csv   (--pmc WRITE_SIZE)
and writes profiles/<round>/kernel_stats.csv (names shortened) and
profiles/<round>/pmc_summary.json.  HBM bytes per launch follow
MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE reports exactly half of a wide streaming read, so it is doubled.
"""

import csv
import json
import os
import re
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")

KERNELS = {
    "shuffle_enc": "k_shuffle_enc<",
    "shuffle_dec": ("k_shuffle_dec<", "k_shuffle4_dec_pair<"),
    "shuffle_f32_enc": "k_shuffle_f32_enc<",
    "f32_unshuffle": "k_f32_unshuffle<",
    "map": "k_map<",
    "bitround": "k_bitround<",
    "delta_enc": "k_delta_enc<",
    "scan_reduce": "k_scan_reduce<",
    "scan_apply": "k_scan_apply<",
    "f32_partial": "k_f32_partial<",
    "shuffle8_enc_pair": "k_shuffle8_enc_pair<",
    "shuffle8_dec_pair": "k_shuffle8_dec_pair<",
    "c4_enc": "k_c4_enc<",
    "c4_reduce2": "k_c4_reduce2<",
    "c4_apply": "k_c4_apply<",
    "scan_sums": "k_scan_sums<",
}
ALGO_BYTES = {"shuffle_enc": 2 * 256 * 2**20, "shuffle_dec": 2 * 256 * 2**20}


def _match(pat, name: str) -> bool:
    return any(p in name for p in ((pat,) if isinstance(pat, str) else pat))


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    name = re.sub(r"\(.*$", "", name)  # drop the parameter list
    return name[:120]


def main():
    rnd = sys.argv[1] if len(sys.argv) > 1 else "r01"
    tag = sys.argv[2] if len(sys.argv) > 2 else ""  # "" = headline, "_extra" = bench.py --extra
    dst = os.path.join(ROOT, "profiles", rnd)
    os.makedirs(dst, exist_ok=True)
    summary = {"round": rnd, "kernels": {}}
    stats_fn = os.path.join(OUT, "prof_kt" + tag, "bench_kernel_stats.csv")
    if os.path.exists(stats_fn):
        rows = list(csv.DictReader(open(stats_fn)))
        with open(os.path.join(dst, f"kernel_stats{tag}.csv"), "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
            for r in rows:
                w.writerow([short(r["Name"]), r["Calls"], r["TotalDurationNs"], r["AverageNs"],
                            r["Percentage"], r["MinNs"], r["MaxNs"]])
        for key, pat in KERNELS.items():
            for r in rows:
                if _match(pat, r["Name"]):
                    k = summary["kernels"].setdefault(key, {})
                    k["name"] = short(r["Name"])
                    k["calls"] = int(r["Calls"])
                    k["avg_ns"] = float(r["AverageNs"])
                    if key in ALGO_BYTES:
                        k["algorithmic_bytes_per_launch"] = ALGO_BYTES[key]
                        k["achieved_GBps"] = round(ALGO_BYTES[key] / float(r["AverageNs"]), 1)
    for sub, counter in (("prof_fetch", "FETCH_SIZE"), ("prof_write", "WRITE_SIZE")):
        fn = os.path.join(OUT, sub + tag, "bench_counter_collection.csv")
        if not os.path.exists(fn):
            continue
        rows = list(csv.DictReader(open(fn)))
        for key, pat in KERNELS.items():
            vals = [float(r["Counter_Value"]) for r in rows
                    if _match(pat, r["Kernel_Name"]) and r["Counter_Name"] == counter]
            if vals:
                k = summary["kernels"].setdefault(key, {})
                k[counter + "_KiB_median"] = statistics.median(vals)
                k[counter + "_dispatches"] = len(vals)
    for key, k in summary["kernels"].items():
        if "FETCH_SIZE_KiB_median" in k and "WRITE_SIZE_KiB_median" in k:
            fetch = 2 * k["FETCH_SIZE_KiB_median"] * 1024  # gfx950: FETCH_SIZE reads half
            write = k["WRITE_SIZE_KiB_median"] * 1024
            k["hbm_bytes_per_launch"] = int(fetch + write)
            if key in ALGO_BYTES:
                k["traffic_over_algorithmic"] = round((fetch + write) / ALGO_BYTES[key], 4)
    summary["correction"] = "hbm = 2*FETCH_SIZE + WRITE_SIZE (KiB*1024), MI355X_MICROARCH.md HBM section"
    with open(os.path.join(dst, f"pmc_summary{tag}.json"), "w") as f:
        json.dump(summary, f, indent=1, sort_keys=True)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
