#!/usr/bin/env python3
"""pmc_traffic.json (what bench.py's roofline `traffic` reads) from a
tools/pmc_summary.py json of the separate FETCH_SIZE / WRITE_SIZE passes:
python tools/make_traffic.py SUMMARY.json OUT.json CONFIG SOURCE [READS]"""
import json
import sys

STAGES = (("prep_complex", "bqsr_prep_complex"), ("prep", "bqsr_prep_kernel"), ("observe", "bqsr_observe"),
          ("apply", "bqsr_apply_kernel"), ("fold_hist", "bqsr_fold_hist"), ("gather", "bqsr_bucket_gather"))

summ = json.load(open(sys.argv[1]))
kernels = {}
for stage, pat in STAGES:
    for name, d in summ.items():
        if pat in name and stage not in kernels and "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            if stage == "prep" and "complex" in name:
                continue
            kernels[stage] = {"kernel": name, "hbm_bytes_per_launch": (2 * d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024,
                              "fetch_kib": d["FETCH_SIZE"], "write_kib": d["WRITE_SIZE"]}
json.dump({"config": sys.argv[3], "reads_per_gpu": int(sys.argv[5]) if len(sys.argv) > 5 else 10_000_000, "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; "
           "hbm_bytes = (2*FETCH_SIZE + WRITE_SIZE) KiB * 1024 (MI355X_MICROARCH.md gfx950 FETCH_SIZE correction), "
           "mean over dispatches", "source": sys.argv[4], "kernels": kernels}, open(sys.argv[2], "w"), indent=1)
print(json.dumps(kernels, indent=1))
