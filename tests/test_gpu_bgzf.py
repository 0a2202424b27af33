"""BGZF inflated on the device (bgzf_inflate.hip, BQSR_TUNE_BGZF 1) against
the host form (libdeflate / zlib threads, BQSR_TUNE_BGZF 0, the default):
the same BAM recompressed with every DEFLATE block form -- stored (level 0),
fixed Huffman codes (Z_FIXED), dynamic codes at levels 1, 6, 9, Huffman-only
and run-length strategies -- and with members of 100 B to 64 KiB (records
spanning several members, members without a record start) parses to the
same columns.  The records' offsets are found on the device and checked as a
chain; a damaged file takes the host form and fails as before
(test_gpu_sam.py::test_bam_ingest_rejects_damaged_bgzf)."""
import os
import struct
import zlib

import pytest

from adam_amd import bqsr
from adam_amd.bam_writer import sam_to_bam
from adam_amd.sam import SamText
from test_gpu_sam import FIXTURES, GOLD, _dup_sam, assert_same_columns

pytestmark = pytest.mark.gpu

EOF_BLOCK = bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")


def _inflate(bam: bytes) -> bytes:
    out, p = [], 0
    while p < len(bam):
        xlen = bam[p + 10] | (bam[p + 11] << 8)
        bsize = bam[p + 16] | (bam[p + 17] << 8)
        out.append(zlib.decompress(bam[p + 12 + xlen:p + bsize + 1 - 8], -15))
        p += bsize + 1
    return b"".join(out)


def _reblock(raw: bytes, block: int, level: int, strategy: int) -> bytes:
    out = []
    for i in range(0, len(raw), block):
        chunk = raw[i:i + block]
        c = zlib.compressobj(level, zlib.DEFLATED, -15, 9, strategy)
        comp = c.compress(chunk) + c.flush()
        bsize = 18 + len(comp) + 8 - 1
        out.append(struct.pack("<BBBBIBBHBBHH", 31, 139, 8, 4, 0, 0, 255, 6, 66, 67, 2, bsize) + comp +
                   struct.pack("<II", zlib.crc32(chunk) & 0xFFFFFFFF, len(chunk)))
    out.append(EOF_BLOCK)
    return b"".join(out)


def _columns(data: bytes, bgzf: int):
    with bqsr.Context.get(0).tuned(bgzf=bgzf):
        s = SamText(data, bam=True)
        try:
            return s.batch()
        finally:
            s.close()


@pytest.fixture(scope="module")
def raw_bam():
    return _inflate(sam_to_bam(_dup_sam(20000, 4243, 30000)))


@pytest.mark.parametrize("block,level,strategy", [
    (65280, 6, zlib.Z_DEFAULT_STRATEGY),
    (65536, 9, zlib.Z_DEFAULT_STRATEGY),
    (65280, 1, zlib.Z_DEFAULT_STRATEGY),
    (65280, 0, zlib.Z_DEFAULT_STRATEGY),   # stored blocks
    (20000, 6, zlib.Z_FIXED),              # fixed Huffman codes
    (65280, 6, zlib.Z_HUFFMAN_ONLY),       # literals only
    (65280, 6, zlib.Z_RLE),                # distance-1 matches
    (1000, 6, zlib.Z_DEFAULT_STRATEGY),    # records across members
    (100, 6, zlib.Z_DEFAULT_STRATEGY),     # members without a record start
])
def test_device_inflate_equals_host(raw_bam, block, level, strategy):
    data = _reblock(raw_bam, block, level, strategy)
    assert_same_columns(_columns(data, 1), _columns(data, 0))


@pytest.mark.parametrize("name", FIXTURES)
def test_device_inflate_reference_fixtures(name):
    with open(os.path.join(GOLD, name), "rb") as fh:
        data = sam_to_bam(fh.read())
    assert_same_columns(_columns(data, 1), _columns(data, 0))


def test_device_inflate_long_records():
    # records longer than a member (4000-base reads, 600-B members): record
    # starts several members apart, most members without one
    from adam_amd import synth
    from adam_amd.samgen import sam_text
    b = synth.generate(300, (4000,), 1, seed=99)
    data = _reblock(_inflate(sam_to_bam(sam_text(b))), 600, 6, zlib.Z_DEFAULT_STRATEGY)
    assert_same_columns(_columns(data, 1), _columns(data, 0))


@pytest.mark.parametrize("run,block", [(150000, 65280), (100000, 20000), (1, 1000)])
def test_device_inflate_in_runs(raw_bam, monkeypatch, run, block):
    # the symbol buffer reused over runs of whole blocks (ADAM_BQSR_BGZF_RUN
    # bytes of output a run; 1: a block a run)
    data = _reblock(raw_bam, block, 6, zlib.Z_DEFAULT_STRATEGY)
    want = _columns(data, 0)
    monkeypatch.setenv("ADAM_BQSR_BGZF_RUN", str(run))
    assert_same_columns(_columns(data, 1), want)


def test_device_inflate_many_blocks(raw_bam):
    # more blocks than the device holds at once at 16 a workgroup (n_cu * 32):
    # the 12-a-workgroup decode (bam_ingest.hip)
    data = _reblock(raw_bam, 250, 6, zlib.Z_DEFAULT_STRATEGY)
    assert len(raw_bam) // 250 > 256 * 32
    assert_same_columns(_columns(data, 1), _columns(data, 0))
