"""Average kernel durations (us) from rocprofv3 --stats csv files:
python tools/kstat_summary.py DIR... (each DIR searched for *kernel_stats.csv)."""
import csv
import glob
import sys

for d in sys.argv[1:]:
    for f in sorted(glob.glob(d + "/**/*kernel_stats.csv", recursive=True)):
        rows = list(csv.DictReader(open(f)))
        print("==", f)
        for r in rows:
            name = r["Name"]
            if any(s in name for s in ("prep", "observe", "apply", "fold", "final", "reduce", "hist", "bgzf", "bam_chain")):
                print("  %-60s %10.1f us  x%s" % (name[:60], float(r["AverageNs"]) / 1e3, r["Calls"]))
