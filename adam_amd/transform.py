"""`adam transform` for SAM in, SAM out: the CLI harness around the device
path (adam-cli/.../cli/Transform.scala:38-110).

    python -m adam_amd.transform INPUT.sam OUTPUT.sam [-mark_duplicate_reads]
        [-recalibrate_base_qualities] [-dbsnp_sites SITES.vcf]

Steps in Transform.run's order (:66-90): load (the SAM text parsed on the
device, SAMRecordConverter semantics), MarkDuplicates (`adamMarkDuplicates`),
BQSR (`adamBQSR(loadSnpTable)`: an empty SnpTable without -dbsnp_sites,
:96-105), save.  The output is SAM text -- the input records with their QUAL
fields replaced by the recalibrated strings (and FLAG 0x400 by MarkDuplicates'
result) -- where the reference writes ADAM/Parquet (adamSave,
core/rdd/AdamRDDFunctions.scala:37-56).  The input is one partition (one
Hadoop split of a small file).  -sort_reads, -coalesce and -realignIndels are
outside this build and are refused.
"""
from __future__ import annotations

import argparse
import sys
import time
from typing import Dict, Optional

from . import bqsr
from .sam import SamText


def transform(inp: str, out: str, mark_duplicates: bool = False, recalibrate: bool = False,
              dbsnp: Optional[str] = None, device: int = 0) -> Dict[str, float]:
    t0 = time.perf_counter()
    ctx = bqsr.Context.get(device)
    with open(inp, "rb") as fh:
        data = fh.read()
    sam = SamText(data, ctx)
    stats: Dict[str, float] = {"reads": sam.counts().n_reads}
    try:
        if mark_duplicates:
            stats["duplicates"] = sam.mark_duplicates()
        job = None
        if recalibrate:
            from .job import ResidentJob
            snp = bqsr.SnpTable.from_vcf(dbsnp) if dbsnp else bqsr.SnpTable()
            batch = sam.batch()
            job = ResidentJob(batch, bqsr.dims_of([batch]), snp if snp.table else None, device)
            try:
                job.step()
                sam.rewrite(job)
            finally:
                job.close()
        elif mark_duplicates:
            sam.rewrite(None)
        text = sam.text()
    finally:
        sam.close()
    with open(out, "wb") as fh:
        fh.write(text)
    stats["seconds"] = time.perf_counter() - t0
    return stats


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="adam_amd.transform", description=__doc__.split("\n\n")[0])
    ap.add_argument("input")
    ap.add_argument("output")
    ap.add_argument("-mark_duplicate_reads", action="store_true")
    ap.add_argument("-recalibrate_base_qualities", action="store_true")
    ap.add_argument("-dbsnp_sites", default=None)
    for flag in ("-sort_reads", "-realignIndels"):
        ap.add_argument(flag, action="store_true")
    ap.add_argument("-coalesce", type=int, default=-1)
    a = ap.parse_args(argv)
    if a.sort_reads or a.realignIndels or a.coalesce != -1:
        ap.error("-sort_reads / -coalesce / -realignIndels are outside this build")
    st = transform(a.input, a.output, a.mark_duplicate_reads, a.recalibrate_base_qualities, a.dbsnp_sites)
    print(" ".join("%s=%s" % kv for kv in st.items()), file=sys.stderr)
    return 0


if __name__ == "__main__":
    sys.exit(main())
