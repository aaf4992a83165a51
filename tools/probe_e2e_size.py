"""Why the host->host line moved from round 1's 42.9 GiB/s (its separate end-to-end mode, 2 GiB
of 4 MiB chunks) to ~41 GiB/s (cfg_e2e, 1 GiB): bench.end_to_end at 1, 2 and
4 GiB on one box, alternating, with the duplex PCIe rate beside each.  The
pipeline's fill (first slice's H2D) and drain (last slice's D2H) do not
overlap anything; with 64 MiB slices they are 2 of 16 slice-times at 1 GiB
and 2 of 32 at 2 GiB.

    python tools/probe_e2e_size.py  -> one JSON line per size and round
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    rows = []
    for rnd in range(2):
        for g in (1, 2, 4):
            r = bench.end_to_end(dev, None, total_gib=g)
            row = {"round": rnd, "GiB": g, "GiBps": r["GiBps"], "enc": r["enc_GiBps"], "dec": r["dec_GiBps"],
                   "duplex_each_way": r["pcie_duplex_GiBps_each_way"], "frac_of_duplex": r["frac_of_duplex"]}
            rows.append(row)
            print(json.dumps(row), flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/probe_e2e_size.json", "w") as f:
        json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
