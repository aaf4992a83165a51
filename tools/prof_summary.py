"""Condense per-config rocprofv3 runs (tools/prof_all.sh) into
profiles/<round>/config_profile.json.

    python tools/prof_summary.py r02

For every CONFIG/direction directory gpurun_out/prof/<CONFIG>_<dir>_{kt,fetch,write}
(tools/prof_configs.py under --kernel-trace, --pmc FETCH_SIZE, --pmc WRITE_SIZE):

* the measured dispatches are those between the two "spin_kernel" markers
  (by dispatch id), i.e. exactly `reps` calls of the operation;
* kernels are keyed by their FULL name (template arguments included), never
  by a prefix; each kernel's dispatch count must be a multiple of `reps`
  (else the entry is marked invalid);
* time per call = the sum of the measured kernel durations / reps; achieved
  GB/s = the config's algorithmic bytes per call / that time (an entry above
  the 8 TB/s peak is marked invalid);
* HBM bytes per call = (2 * FETCH_SIZE + WRITE_SIZE) summed over the measured
  dispatches / reps (KiB counters; gfx950 FETCH_SIZE counts half of a wide
  streaming read -- MI355X_MICROARCH.md, HBM), and traffic_over_algorithmic.
"""

import csv
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out", "prof")
PEAK_GBPS = 8000.0


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return re.sub(r"\(.*$", "", name)[:140]


def _find(d, suffix):
    f = glob.glob(os.path.join(d, "**", "*" + suffix), recursive=True)
    return f[0] if f else None


def measured(rows, name_key, id_key):
    """Rows strictly between the two spin_kernel markers (by dispatch id)."""
    rows = sorted(rows, key=lambda r: int(r[id_key]))
    marks = [int(r[id_key]) for r in rows if "spin_kernel" in r[name_key]]
    if len(set(marks)) < 2:
        return None
    lo, hi = sorted(set(marks))[0], sorted(set(marks))[-1]
    return [r for r in rows if lo < int(r[id_key]) < hi and "spin_kernel" not in r[name_key]]


def one(cfg_dir_prefix, meta):
    res = {"reps": meta["reps"], "alg_bytes_per_call": meta["alg_bytes_per_call"],
           "event_us_per_call": meta["event_us_per_call"], "kernels": {}, "valid": True, "notes": []}
    reps = meta["reps"]
    kt = _find(cfg_dir_prefix + "_kt", "kernel_trace.csv")
    if kt:
        rows = measured(list(csv.DictReader(open(kt))), "Kernel_Name", "Dispatch_Id")
        if rows is None:
            res["valid"] = False
            res["notes"].append("markers not found in the kernel trace")
            rows = []
        total = 0
        for r in rows:
            k = res["kernels"].setdefault(short(r["Kernel_Name"]), {"dispatches": 0, "total_ns": 0})
            dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            k["dispatches"] += 1
            k["total_ns"] += dur
            total += dur
        for name, k in res["kernels"].items():
            k["avg_ns"] = round(k["total_ns"] / k["dispatches"], 1)
            if k["dispatches"] % reps:
                res["valid"] = False
                res["notes"].append(f"{name}: {k['dispatches']} dispatches for {reps} calls")
        if rows:
            us = total / reps / 1e3
            res["kernel_us_per_call"] = round(us, 2)
            res["achieved_GBps"] = round(meta["alg_bytes_per_call"] / (us * 1e3), 1)
            res["frac_of_peak"] = round(res["achieved_GBps"] / PEAK_GBPS, 4)
            if res["achieved_GBps"] > PEAK_GBPS:
                res["valid"] = False
                res["notes"].append("achieved above the 8 TB/s peak")
    hbm = 0.0
    have = 0
    for sub, counter, mult in (("_fetch", "FETCH_SIZE", 2.0), ("_write", "WRITE_SIZE", 1.0)):
        f = _find(cfg_dir_prefix + sub, "counter_collection.csv")
        if not f:
            continue
        rows = list(csv.DictReader(open(f)))
        id_key = "Dispatch_Id" if rows and "Dispatch_Id" in rows[0] else "Correlation_Id"
        rows = measured(rows, "Kernel_Name", id_key)
        if rows is None:
            res["notes"].append(f"markers not found in the {counter} pass")
            continue
        vals = [float(r["Counter_Value"]) for r in rows if r["Counter_Name"] == counter]
        res[counter + "_KiB_per_call"] = round(sum(vals) / reps, 1)
        hbm += mult * sum(vals) * 1024 / reps
        have += 1
    if have == 2:
        res["hbm_bytes_per_call"] = int(hbm)
        res["traffic_over_algorithmic"] = round(hbm / meta["alg_bytes_per_call"], 4)
    return res


def main():
    rnd = sys.argv[1] if len(sys.argv) > 1 else "r02"
    summary = {"round": rnd, "peak_GBps": PEAK_GBPS,
               "correction": "hbm = 2*FETCH_SIZE + WRITE_SIZE (KiB*1024) over the marked dispatches; "
                             "MI355X_MICROARCH.md HBM section",
               "configs": {}}
    for meta_fn in sorted(glob.glob(os.path.join(OUT, "*_meta.json"))):
        meta = json.load(open(meta_fn))
        key = f"{meta['config']}_{meta['direction']}"
        summary["configs"][key] = one(os.path.join(OUT, key), meta)
    dst = os.path.join(ROOT, "profiles", rnd)
    os.makedirs(dst, exist_ok=True)
    with open(os.path.join(dst, "config_profile.json"), "w") as f:
        json.dump(summary, f, indent=1, sort_keys=True)
    # the headline's PMC record for bench.py (roofline.traffic): configs[1]'s
    # Shuffle(4) encode and decode kernels, one launch per call
    head = {}
    for key, name in (("C2_f32_enc", "shuffle_enc"), ("C2_f32_dec", "shuffle_dec")):
        c = summary["configs"].get(key)
        if not c or not c.get("valid") or "hbm_bytes_per_call" not in c or len(c["kernels"]) != 1:
            continue
        kname, k = next(iter(c["kernels"].items()))
        head[name] = {"name": kname, "avg_ns": k["avg_ns"], "calls": c["reps"],
                      "algorithmic_bytes_per_launch": c["alg_bytes_per_call"],
                      "hbm_bytes_per_launch": c["hbm_bytes_per_call"],
                      "FETCH_SIZE_KiB_per_launch": c["FETCH_SIZE_KiB_per_call"],
                      "WRITE_SIZE_KiB_per_launch": c["WRITE_SIZE_KiB_per_call"],
                      "achieved_GBps": c["achieved_GBps"],
                      "traffic_over_algorithmic": c["traffic_over_algorithmic"]}
    if len(head) == 2:
        with open(os.path.join(dst, "pmc_summary.json"), "w") as f:
            json.dump({"round": rnd, "source": "config_profile.json (tools/prof_all.sh C2_f32)",
                       "correction": summary["correction"], "kernels": head}, f, indent=1, sort_keys=True)
    for k, v in summary["configs"].items():
        print(f"{k:12s} {v.get('kernel_us_per_call', '-'):>9} us  {v.get('achieved_GBps', '-'):>8} GB/s  "
              f"frac {v.get('frac_of_peak', '-'):>7}  traffic/alg {v.get('traffic_over_algorithmic', '-'):>7}  "
              f"valid {v['valid']} {'; '.join(v['notes'])}")


if __name__ == "__main__":
    main()
