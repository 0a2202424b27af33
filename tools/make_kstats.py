#!/usr/bin/env python3
"""profiles/kernel_stats_<config>.json (what bench.py's roofline.kernels
reads) from a `rocprofv3 --kernel-trace --stats` kernel_stats.csv of a bench
run: per stage the kernel's average duration.

    python tools/make_kstats.py STATS.csv OUT.json CONFIG READS_PER_GPU SOURCE [COMMIT]
"""
import csv
import json
import sys

STAGES = (("observe", ("bqsr_observe_lean", "bqsr_observe_chunks")), ("apply", ("bqsr_apply_kernel",)),
          ("prep", ("bqsr_prep_kernel",)), ("prep_complex", ("bqsr_prep_complex",)),
          ("fold_hist", ("bqsr_fold_hist",)), ("window_reduce", ("bqsr_window_reduce",)),
          ("apply_chars", ("bqsr_apply_chars",)), ("fold_plan", ("bqsr_fold_plan",)),
          ("fold_tiles", ("bqsr_fold_tiles",)), ("fold_segs", ("bqsr_fold_segs",)),
          ("fold_chain", ("bqsr_fold_chain",)))


def main():
    path, out, config, reads, source = sys.argv[1:6]
    commit = sys.argv[6] if len(sys.argv) > 6 else None
    kernels = {}
    with open(path) as fh:
        for row in csv.DictReader(fh):
            name = row["Name"]
            for stage, pats in STAGES:
                if stage not in kernels and any(p in name for p in pats):
                    if stage == "prep" and "complex" in name:
                        continue
                    kernels[stage] = {"kernel": name, "avg_ms": float(row["AverageNs"]) / 1e6,
                                      "calls": int(row["Calls"]), "min_ms": float(row["MinNs"]) / 1e6,
                                      "max_ms": float(row["MaxNs"]) / 1e6}
    doc = {"config": config, "reads_per_gpu": int(reads), "commit": commit, "source": source,
           "method": "rocprofv3 --kernel-trace --stats of bench.py (kernel-only durations, mean over dispatches)",
           "kernels": kernels}
    with open(out, "w") as fh:
        json.dump(doc, fh, indent=1)
    print(json.dumps({k: round(v["avg_ms"], 4) for k, v in kernels.items()}))


if __name__ == "__main__":
    main()
