"""adamSave's GZIP part files (AdamRDDFunctions.scala:37-48; ParquetArgs.scala:27
default codec GZIP) written by the library's page recompressor
(adam_amd/csrc/parquet_gzip.cpp, bqsr_parquet_gzip): host code, no GPU.

Every page must be a gzip member any inflater reads (zlib here, Arrow's reader
below), and the rewritten file must read back as the same table Arrow's own
GZIP writer produces, with GZIP as every column chunk's codec."""
import ctypes
import io
import zlib

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq
import pytest

from adam_amd.adam_save import DICT_COLS, HUFFMAN_COLS, STATS_COLS, AdamWriter, _lib


def gz(data: bytes, huffman: bool, level: int = 6) -> bytes:
    L = _lib()
    n = ctypes.c_int64()
    src = ctypes.create_string_buffer(data, len(data)) if data else None
    assert L.bqsr_gzip_bytes(src, len(data), int(huffman), level, None, 0, ctypes.byref(n)) == 0
    out = ctypes.create_string_buffer(n.value)
    assert L.bqsr_gzip_bytes(src, len(data), int(huffman), level, out, n.value, ctypes.byref(n)) == 0
    return out.raw[:n.value]


@pytest.mark.parametrize("kind", ["empty", "one_byte", "one_symbol", "two_symbols", "all_256", "quals", "bases",
                                  "skewed_long_codes"])
def test_huffman_member_inflates(kind):
    rng = np.random.default_rng(3)
    data = {
        "empty": b"",
        "one_byte": b"A",
        "one_symbol": b"#" * 100000,
        "two_symbols": bytes(rng.choice([65, 67], 5000).astype(np.uint8)),
        "all_256": bytes(rng.integers(0, 256, 300000).astype(np.uint8)),
        "quals": bytes(np.clip(np.round(rng.normal(38, 3, 1 << 20)), 3, 41).astype(np.uint8) + 33),
        "bases": bytes(rng.choice(np.frombuffer(b"ACGTN", np.uint8), 1 << 20, p=[.3, .2, .2, .29, .01])),
        # Fibonacci-like frequencies force Huffman depths past 15: the length limit must hold
        "skewed_long_codes": b"".join(bytes([i]) * int(1.6 ** i + 1) for i in range(30)),
    }[kind]
    c = gz(data, True)
    assert c[:2] == b"\x1f\x8b"
    assert zlib.decompress(c, 31) == data
    if kind in ("quals", "bases"):  # compresses as zlib's Huffman-only strategy does
        zc = zlib.compressobj(6, zlib.DEFLATED, 31, 8, zlib.Z_HUFFMAN_ONLY)
        ref = zc.compress(data) + zc.flush()
        assert len(c) <= len(ref) * 1.01 + 300


def test_level_member_inflates():
    data = b"c0_12345\tRG:Z:rg1\tNM:i:0" * 4000
    c = gz(data, False, 6)
    assert zlib.decompress(c, 31) == data
    assert len(c) < len(data) // 10


def adam_like_table(n=5000, seed=1):
    rng = np.random.default_rng(seed)
    quals = ["".join(chr(33 + int(q)) for q in np.clip(rng.normal(35, 4, 100), 2, 41)) for _ in range(n)]
    seqs = ["".join(rng.choice(list("ACGT"), 100)) for _ in range(n)]
    return pa.table({
        "referenceName": pa.array(rng.choice(["chr1", "chr2", None], n)),
        "start": pa.array(rng.integers(0, 1 << 30, n), pa.int64()),
        "readName": pa.array(["r%07d" % i for i in range(n)]),
        "sequence": pa.array(seqs),
        "qual": pa.array([q if i % 97 else None for i, q in enumerate(quals)]),
        "cigar": pa.array(rng.choice(["100M", "50M2I48M", "10S90M"], n)),
        "readMapped": pa.array(rng.random(n) < 0.99),
        "recordGroupId": pa.array(rng.integers(0, 3, n).astype(np.int32)),
        "mapq": pa.array(rng.integers(0, 60, n).astype(np.int32)),
        "attributes": pa.array(["NM:i:%d\tAS:i:%d" % (i % 5, i % 100) for i in range(n)]),
    })


def rewrite(table, path, **kw):
    buf = pa.BufferOutputStream()
    pq.write_table(table, buf, compression="none", **kw)
    data = buf.getvalue()
    n = ctypes.c_int64()
    st = _lib().bqsr_parquet_gzip(ctypes.c_void_p(data.address), data.size, str(path).encode(), 6,
                                  b"qual,sequence", 3, ctypes.byref(n))
    return st, n.value


@pytest.mark.parametrize("kw", [{}, {"use_dictionary": False}, {"row_group_size": 1234, "data_page_size": 20000},
                                {"write_statistics": False}])
def test_rewritten_file_reads_back(tmp_path, kw):
    t = adam_like_table()
    st, n = rewrite(t, tmp_path / "a.parquet", **kw)
    assert st == 0
    f = pq.ParquetFile(tmp_path / "a.parquet")
    assert f.metadata.num_row_groups >= 1
    for rg in range(f.metadata.num_row_groups):
        for c in range(f.metadata.num_columns):
            assert f.metadata.row_group(rg).column(c).compression == "GZIP"
    assert pq.read_table(tmp_path / "a.parquet").equals(t)
    # Arrow's own GZIP writer: the same table
    pq.write_table(t, tmp_path / "b.parquet", compression="gzip", **kw)
    assert pq.read_table(tmp_path / "b.parquet").equals(pq.read_table(tmp_path / "a.parquet"))
    assert n == (tmp_path / "a.parquet").stat().st_size


def test_empty_table(tmp_path):
    t = adam_like_table(0)
    st, _ = rewrite(t, tmp_path / "e.parquet")
    assert st == 0
    assert pq.read_table(tmp_path / "e.parquet").equals(t)


def test_rejects_compressed_or_foreign_input(tmp_path):
    t = adam_like_table(100)
    buf = pa.BufferOutputStream()
    pq.write_table(t, buf, compression="snappy")
    data = buf.getvalue()
    n = ctypes.c_int64()
    L = _lib()
    assert L.bqsr_parquet_gzip(ctypes.c_void_p(data.address), data.size, str(tmp_path / "x").encode(), 6, b"",
                               1, ctypes.byref(n)) != 0
    junk = ctypes.create_string_buffer(b"PAR1 not a parquet file PAR1")
    assert L.bqsr_parquet_gzip(junk, 28, str(tmp_path / "y").encode(), 6, b"", 1, ctypes.byref(n)) != 0


def test_adam_writer_gzip_parts(tmp_path):
    t = adam_like_table(3000)
    out = str(tmp_path / "o.adam")
    w = AdamWriter(out, "gzip")
    w.add(t.slice(0, 2000))
    w.add(t.slice(2000))
    w.close(True)
    got = pq.read_table(out)
    assert got.equals(t)
    md = pq.ParquetFile(out + "/part-r-00000.parquet").metadata
    assert md.row_group(0).column(0).compression == "GZIP"
    assert set(HUFFMAN_COLS) <= set(t.column_names)
