#!/usr/bin/env python3
"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes of the l4 correlation kernel into the
JSON bench.py reads for roofline.traffic (profiles/<round>_l4corr_pmc.json).

    python tools/pmc_summary.py <fetch_csv> <write_csv> <out_json> [kernel-substring]

Correction (MI355X_MICROARCH.md, HBM section): on gfx950 FETCH_SIZE counts half the bytes of a
16-B-per-lane streaming read (LDS-DMA included) -> x2; WRITE_SIZE is exact for 16-B stores.
Both are reported in KB (1024 B)."""
import csv
import json
import sys

ALG = (2 * 32 * 96 * 112 + 81 * 96 * 112) * 4 * 8


def mean_kb(path, sub):
    vals, name = [], None
    for r in csv.DictReader(open(path)):
        if sub in r["Kernel_Name"]:
            vals.append(float(r["Counter_Value"]))
            name = r["Kernel_Name"]
    return sum(vals) / len(vals), len(vals), name


def main():
    fetch, write, out = sys.argv[1:4]
    sub = sys.argv[4] if len(sys.argv) > 4 else "corr_fwd_stream"
    f, n, name = mean_kb(fetch, sub)
    w, _, _ = mean_kb(write, sub)
    rd = int(f * 1024 * 2)
    wr = int(w * 1024)
    d = {
        "kernel": name,
        "workload": "l4 Correlation(9,1,9,1,2), B=8, C=32, 96x112 fp32 (tools/kbench.py --levels 4)",
        "dispatches": n,
        "fetch_size_kb_mean": round(f, 3),
        "write_size_kb_mean": round(w, 3),
        "correction": "MI355X_MICROARCH.md HBM section: FETCH_SIZE counts 1/2 of the bytes of "
                      "16-B-per-lane streaming reads on gfx950 -> x2; WRITE_SIZE exact for 16-B "
                      "stores; KB = 1024 B",
        "hbm_read_bytes_per_launch": rd,
        "hbm_write_bytes_per_launch": wr,
        "hbm_bytes_per_launch": rd + wr,
        "algorithmic_bytes_per_launch": ALG,
        "traffic_over_algorithmic": round((rd + wr) / ALG, 4),
        "collected_with": "rocprofv3 --pmc FETCH_SIZE (and separately WRITE_SIZE) "
                          f"--kernel-include-regex {sub} -- python tools/kbench.py --levels 4 "
                          "--ops corr --iters 20 (tools/gpu_profile_r02.sh)",
    }
    json.dump(d, open(out, "w"), indent=1)
    print(json.dumps(d))


if __name__ == "__main__":
    main()
