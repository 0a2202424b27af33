#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes (tools/gpu_prof.sh output): per kernel,
mean counter values per dispatch, plus derived HBM bytes (FETCH_SIZE x 2 per
MI355X_MICROARCH.md's gfx950 correction, + WRITE_SIZE; both in KiB)."""
import collections
import csv
import glob
import json
import sys


def load(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(d + "/pmc*/run_counter_collection.csv")):
        for row in csv.DictReader(open(f)):
            agg[row["Kernel_Name"]][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in agg.items()}


if __name__ == "__main__":
    out = load(sys.argv[1])
    keys = [k for k in out if "bqsr_" in k]
    for k in keys:
        d = out[k]
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            d["hbm_bytes"] = (2 * d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024
        print(k)
        for c in sorted(d):
            print("   %-22s %14.4g" % (c, d[c]))
    if len(sys.argv) > 2:
        json.dump({k: out[k] for k in keys}, open(sys.argv[2], "w"), indent=1)
