"""Per-kernel summary of a rocprofv3 SQLite output (run_results.db): average
duration (kernel trace) or average counter values per dispatch (--pmc).
Usage: python tools/rocpd_summary.py <db> [kernel-substring]"""
import sqlite3
import sys
from collections import defaultdict


def main():
    db = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    c = sqlite3.connect(db)
    names = {r[0] for r in c.execute("select name from sqlite_master")}
    rows = list(c.execute("select kernel_name, counter_name, dispatch_id, value, vgpr_count, accum_vgpr_count, "
                          "sgpr_count, lds_block_size from counters_collection")) if "counters_collection" in names else []
    if rows:
        acc = defaultdict(lambda: defaultdict(list))
        meta = {}
        for k, cn, d, v, vg, ag, sg, lds in rows:
            if sub in k:
                acc[k][cn].append(v)
                meta[k] = (vg, ag, sg, lds)
        for k, cs in acc.items():
            print(k[:90], "vgpr/agpr/sgpr/lds", meta[k])
            for cn, vs in sorted(cs.items()):
                print(f"   {cn:28s} {sum(vs) / len(vs):16.1f}  (n={len(vs)})")
        return
    acc = defaultdict(list)
    for k, s, e in c.execute("select name, start, end from kernels"):
        if sub in k:
            acc[k].append(e - s)
    for k, ds in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
        print(f"{sum(ds) / len(ds) / 1e3:10.2f} us  n={len(ds):3d}  {k[:110]}")


if __name__ == "__main__":
    main()
