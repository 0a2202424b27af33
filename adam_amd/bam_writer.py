"""SAM text -> BAM bytes (BGZF), for the BAM ingest tests and tools: the
reference loads BAM through Hadoop-BAM (core/rdd/AdamContext.scala:122-137),
so its SAM fixtures are converted here, record by record, as samtools would
write them (SAM v1 BAM encoding: 4-bit SEQ codes, QUAL - 33 or 0xFF, CIGAR
words, typed optional fields; integers in the smallest fitting type).
Pure Python (zlib): test and tool infrastructure, not the ingest path."""
from __future__ import annotations

import struct
import zlib
from typing import Dict, List, Tuple

_SEQ = {c: i for i, c in enumerate("=ACMGRSVTWYHKDBN")}
_CIG = {c: i for i, c in enumerate("MIDNSHP=X")}


def _int_tag(v: int) -> Tuple[bytes, bytes]:
    for t, fmt, lo, hi in (("c", "<b", -128, 127), ("C", "<B", 0, 255), ("s", "<h", -32768, 32767),
                           ("S", "<H", 0, 65535), ("i", "<i", -2 ** 31, 2 ** 31 - 1), ("I", "<I", 0, 2 ** 32 - 1)):
        if lo <= v <= hi:
            return t.encode(), struct.pack(fmt, v)
    raise ValueError("integer tag out of range")


def _reg2bin(beg: int, end: int) -> int:
    end -= 1
    if beg >> 14 == end >> 14:
        return ((1 << 15) - 1) // 7 + (beg >> 14)
    if beg >> 17 == end >> 17:
        return ((1 << 12) - 1) // 7 + (beg >> 17)
    if beg >> 20 == end >> 20:
        return ((1 << 9) - 1) // 7 + (beg >> 20)
    if beg >> 23 == end >> 23:
        return ((1 << 6) - 1) // 7 + (beg >> 23)
    if beg >> 26 == end >> 26:
        return ((1 << 3) - 1) // 7 + (beg >> 26)
    return 0


def _record(f: List[bytes], ref_id: Dict[bytes, int]) -> bytes:
    qname, flag, rname, pos, mapq, cigar, rnext, pnext, tlen, seq, qual = f[:11]
    flag, pos, mapq, pnext, tlen = int(flag), int(pos), int(mapq), int(pnext), int(tlen)
    rid = ref_id.get(rname, -1) if rname != b"*" else -1
    nid = rid if rnext == b"=" else (ref_id.get(rnext, -1) if rnext != b"*" else -1)
    ops = []
    if cigar != b"*":
        n = 0
        for ch in cigar.decode():
            if ch.isdigit():
                n = 10 * n + int(ch)
            else:
                ops.append((n << 4) | _CIG[ch])
                n = 0
    l_seq = 0 if seq == b"*" else len(seq)
    s = seq.decode("latin-1") if l_seq else ""
    packed = bytearray((l_seq + 1) // 2)
    for i, c in enumerate(s):
        packed[i >> 1] |= _SEQ.get(c.upper(), 15) << (0 if i & 1 else 4)
    if qual == b"*" or l_seq == 0:
        q = b"\xff" * l_seq
    else:
        q = bytes((b - 33) & 0xFF for b in qual)
    tags = b""
    for t in f[11:]:
        tag, typ, val = t.split(b":", 2)
        if typ == b"i":
            tt, vv = _int_tag(int(val))
            tags += tag + tt + vv
        elif typ == b"A":
            tags += tag + b"A" + val[:1]
        elif typ == b"f":
            tags += tag + b"f" + struct.pack("<f", float(val))
        else:  # Z, H (and anything else kept as text)
            tags += tag + (typ if typ in (b"Z", b"H") else b"Z") + val + b"\0"
    name = qname + b"\0"
    end = pos + sum(o >> 4 for o in ops if (o & 15) in (0, 2, 3, 7, 8)) if ops else pos + 1
    body = struct.pack("<iiBBHHHiiii", rid, pos - 1, len(name), mapq, _reg2bin(max(pos - 1, 0), max(end - 1, pos)),
                       len(ops), flag, l_seq, nid, pnext - 1, tlen)
    body += name + b"".join(struct.pack("<I", o) for o in ops) + bytes(packed) + q + tags
    return struct.pack("<i", len(body)) + body


def _bgzf(data: bytes, block: int = 65280) -> bytes:
    out = []
    for i in range(0, len(data), block):
        chunk = data[i:i + block]
        c = zlib.compressobj(6, zlib.DEFLATED, -15)
        comp = c.compress(chunk) + c.flush()
        bsize = 18 + len(comp) + 8 - 1
        out.append(struct.pack("<BBBBIBBHBBHH", 31, 139, 8, 4, 0, 0, 255, 6, 66, 67, 2, bsize) + comp +
                   struct.pack("<II", zlib.crc32(chunk) & 0xFFFFFFFF, len(chunk)))
    # the empty EOF block
    out.append(bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000"))
    return b"".join(out)


def _bam_header(head: List[bytes]) -> Tuple[bytes, Dict[bytes, int]]:
    refs = []
    for l in head:
        if l.startswith(b"@SQ"):
            f = dict(x.split(b":", 1) for x in l.split(b"\t")[1:] if b":" in x)
            refs.append((f[b"SN"], int(f.get(b"LN", b"0"))))
    ref_id: Dict[bytes, int] = {}
    for i, (n, _) in enumerate(refs):
        ref_id.setdefault(n, i)
    htext = b"".join(l + b"\n" for l in head)
    raw = b"BAM\1" + struct.pack("<i", len(htext)) + htext + struct.pack("<i", len(refs))
    for n, ln in refs:
        raw += struct.pack("<i", len(n) + 1) + n + b"\0" + struct.pack("<i", ln)
    return raw, ref_id


_EOF = bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")


def _chunk_blocks(args) -> bytes:
    lines, ref_id = args
    return _bgzf(b"".join(_record(l.split(b"\t"), ref_id) for l in lines))[:-len(_EOF)]


def sam_to_bam_parallel(text: bytes, workers: int = 16, progress=None) -> bytes:
    """sam_to_bam with the records encoded and compressed by a process pool
    (BGZF blocks are independent: the header's blocks, each slice's blocks,
    one EOF block).  Fork before the GPU is touched."""
    from multiprocessing import get_context
    lines = [l[:-1] if l.endswith(b"\r") else l for l in text.split(b"\n")]
    head = [l for l in lines if l.startswith(b"@")]
    body = [l for l in lines if l and not l.startswith(b"@")]
    raw, ref_id = _bam_header(head)
    step = max(1, (len(body) + 4 * workers - 1) // (4 * workers))
    jobs = [(body[i:i + step], ref_id) for i in range(0, len(body), step)]
    out = [_bgzf(raw)[:-len(_EOF)]]
    # close() + join() rather than the context manager's terminate(), which
    # SIGTERMs workers that are still unwinding
    pool = get_context("fork").Pool(workers)
    try:
        for i, b in enumerate(pool.imap(_chunk_blocks, jobs)):
            out.append(b)
            if progress:
                progress(i + 1, len(jobs))
        pool.close()
    except BaseException:
        pool.terminate()
        raise
    finally:
        pool.join()
    out.append(_EOF)
    return b"".join(out)


def sam_to_bam(text: bytes) -> bytes:
    """BAM bytes of a SAM text: header text kept, @SQ lines as the reference list."""
    lines = [l[:-1] if l.endswith(b"\r") else l for l in text.split(b"\n")]
    head = [l for l in lines if l.startswith(b"@")]
    refs = []
    for l in head:
        if l.startswith(b"@SQ"):
            f = dict(x.split(b":", 1) for x in l.split(b"\t")[1:] if b":" in x)
            refs.append((f[b"SN"], int(f.get(b"LN", b"0"))))
    ref_id = {}
    for i, (n, _) in enumerate(refs):
        ref_id.setdefault(n, i)
    htext = b"".join(l + b"\n" for l in head)
    raw = b"BAM\1" + struct.pack("<i", len(htext)) + htext + struct.pack("<i", len(refs))
    for n, ln in refs:
        raw += struct.pack("<i", len(n) + 1) + n + b"\0" + struct.pack("<i", ln)
    raw += b"".join(_record(l.split(b"\t"), ref_id) for l in lines if l and not l.startswith(b"@"))
    return _bgzf(raw)
