#!/usr/bin/env python3
"""Aggregate a rocprofv3 --pmc counter_collection.csv per kernel name: mean counter value per
dispatch (summed over the dimensions rocprofv3 splits a counter into).  Prints JSON lines.

    python tools/pmc_agg.py <dir with *_counter_collection.csv> [--delete]
"""
import collections
import csv
import glob
import json
import os
import sys


def main():
    root = sys.argv[1]
    files = glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)  # (kernel, counter) -> dispatches that report it
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row.get("Kernel_Name", "?")[:90]
                c = row["Counter_Name"]
                disp[(k, c)].add((f, row.get("Dispatch_Id")))
                per[k][c] += float(row["Counter_Value"])
    for k, cs in per.items():
        n = max(len(disp[(k, c)]) for c in cs)
        print(json.dumps(dict(kernel=k, dispatches=n, **{
            c: round(v / max(1, len(disp[(k, c)])), 1) for c, v in sorted(cs.items())})))
    if "--delete" in sys.argv:
        for f in files:
            os.remove(f)


if __name__ == "__main__":
    main()
