"""SAM text from a RecordBatch (synthetic inputs for the ingest tests and the
ingest throughput line).  Header: @SQ per reference name, @RG per read
group id ("rg<i>", LB "lib<i % 2>").  FLAG is rebuilt from the flag bits (a
read with none of them set gets FLAG 0, which SAMRecordConverter reads back
as unmapped, quirk Q2 -- the text is an input, not a round trip)."""
from __future__ import annotations

from typing import List

import numpy as np

from . import records as R


def sam_text(b: R.RecordBatch, n_rg: int = 1, qname: str = "r") -> bytes:
    out: List[bytes] = [b"@HD\tVN:1.4\tSO:unsorted\n"]
    for name in b.ref_names:
        out.append(b"@SQ\tSN:%s\tLN:100000000\n" % name.encode("latin-1"))
    for i in range(n_rg):
        out.append(b"@RG\tID:rg%d\tLB:lib%d\tSM:s\n" % (i, i % 2))
    so, qo, co, mo = b.seq_offset, b.qual_offset, b.cigar_offset, b.md_offset
    seq, qual, md = b.seq.tobytes(), b.qual.tobytes(), b.md.tobytes()
    for r in range(b.n_reads):
        f = int(b.flags[r])
        flag = 0
        if f & R.F_PAIRED:
            flag |= 0x1
            if f & R.F_SECOND_OF_PAIR:
                flag |= 0x80
            else:
                flag |= 0x40
        if f & R.F_DUPLICATE:
            flag |= 0x400
        if f & R.F_NEG_STRAND:
            flag |= 0x10
        if not f & R.F_PRIMARY:
            flag |= 0x100
        if not f & R.F_MAPPED:
            flag |= 0x4
        rname = b.ref_names[b.ref_index[r]].encode("latin-1") if f & R.F_HAS_REFNAME else b"*"
        pos = int(b.start[r]) + 1 if f & R.F_HAS_START else 0
        cig = R.cigar_to_text(b.cigar[int(co[r]):int(co[r + 1])]).encode() if f & R.F_HAS_CIGAR else b"*"
        s = seq[int(so[r]):int(so[r + 1])] if f & R.F_HAS_SEQ else b"*"
        q = qual[int(qo[r]):int(qo[r + 1])] if f & R.F_HAS_QUAL else b"*"
        tags = b""
        if f & R.F_HAS_MD:
            tags += b"\tMD:Z:" + md[int(mo[r]):int(mo[r + 1])]
        if f & R.F_HAS_RG:
            tags += b"\tRG:Z:rg%d" % int(b.rg_id[r])
        out.append(b"%s%d\t%d\t%s\t%d\t60\t%s\t*\t0\t0\t%s\t%s%s\n" % (qname.encode(), r, flag, rname, pos, cig, s or b"*",
                                                                    q or b"*", tags))
    return b"".join(out)
