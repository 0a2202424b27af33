"""The JNI shim (adam_amd/csrc/bqsr_jni.c): the C core the JNI entry points
run is built and exported; the HAVE_JNI branch type-checks against the JNI
calls it makes (tests/jni_stub/jni.h: no JDK in this image); on the GPU the
shim's observe -> merge -> finalize -> apply sequence equals the oracle."""
import ctypes
import os
import shutil
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM = os.path.join(ROOT, "adam_amd", "libadam_bqsr_jni.so")
SRC = os.path.join(ROOT, "adam_amd", "csrc", "bqsr_jni.c")

# status -> the exception the Scala reference raises (adam_bqsr.h cites each)
EXPECTED = {
    0: None,
    1: b"java/lang/NullPointerException",           # NULL_RG
    2: b"java/lang/IllegalArgumentException",       # MD_PARSE
    3: b"java/lang/IndexOutOfBoundsException",      # CIGAR_SHORT
    4: b"java/util/NoSuchElementException",         # BAD_REVCOMP_BASE
    5: b"java/lang/UnsupportedOperationException",  # EMPTY_TABLE
    6: b"java/util/NoSuchElementException",         # MISSING_KEY
    7: b"java/lang/ArrayIndexOutOfBoundsException", # QUAL_RANGE
    8: b"java/lang/NullPointerException",           # NULL_FIELD
    9: b"java/lang/ArrayIndexOutOfBoundsException", # SEQ_SHORT
    10: b"java/util/NoSuchElementException",        # CIGAR_INVALID
}


def _shim():
    if not os.path.exists(SHIM):
        pytest.skip("libadam_bqsr_jni.so not built (__graft_entry__.build())")
    L = ctypes.CDLL(SHIM)
    L.bqsr_jni_exception_class.restype = ctypes.c_char_p
    L.bqsr_jni_exception_class.argtypes = [ctypes.c_int]
    L.bqsr_jni_eligible.argtypes = [ctypes.c_uint32]
    return L


def test_exports_and_exception_classes():
    L = _shim()
    for name in ("bqsr_jni_observe", "bqsr_jni_finalize", "bqsr_jni_apply"):
        assert hasattr(L, name)
    for st, cls in EXPECTED.items():
        assert L.bqsr_jni_exception_class(st) == cls, st
    for st in (11, 12, 13, 14):
        assert L.bqsr_jni_exception_class(st) is not None


def test_eligible_matches_apply_table_filter():
    from adam_amd.records import F_DUPLICATE, F_MAPPED, F_PRIMARY
    L = _shim()
    for f in range(64):
        fl = (F_MAPPED if f & 1 else 0) | (F_PRIMARY if f & 2 else 0) | (F_DUPLICATE if f & 4 else 0) | (f & ~7) << 8
        assert bool(L.bqsr_jni_eligible(fl)) == bool((f & 1) and (f & 2) and not (f & 4))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="no gcc")
def test_jni_branch_type_checks():
    r = subprocess.run(["gcc", "-fsyntax-only", "-Wall", "-Wextra", "-Werror", "-std=c99", "-DHAVE_JNI",
                        "-I", os.path.join(ROOT, "tests", "jni_stub"), SRC], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


@pytest.mark.gpu
def test_shim_sequence_matches_oracle():
    """What HipBqsr.observe / finalizeTable / apply do per partition (the
    driver's ++ between them), against the oracle on the same partitions."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from adam_amd import _capi, bqsr, synth
    L = _shim()
    ctx = bqsr.Context.get(0)
    batch = synth.generate(6000, lens=(100, 150), n_rg=2, seed=11)
    parts = [batch.slice(0, 2500), batch.slice(2500, 6000)]
    d = bqsr.dims_of(parts)
    nw = _capi.lib().bqsr_table_words(d)
    words = np.zeros(nw, dtype=np.int64)
    em = 0.0
    for p in parts:
        s, _ = p.c_struct(p.contig_ids_for(None))
        w = np.zeros(nw, dtype=np.int64)
        e = ctypes.c_double()
        assert L.bqsr_jni_observe(ctx.handle, None, ctypes.byref(s), d, w.ctypes.data_as(ctypes.c_void_p),
                                  ctypes.byref(e)) == 0
        words += w
        em = em + e.value
    lut = ctypes.c_void_p()
    assert L.bqsr_jni_finalize(ctx.handle, words.ctypes.data_as(ctypes.c_void_p), d, ctypes.c_double(em),
                               ctypes.byref(lut)) == 0
    od = O.Dims(d.n_rg, d.max_len)
    owords = np.zeros(O.table_words(od), dtype=np.int64)
    oem = 0.0
    for p in parts:
        w, e = O.observe(p, O.Sites({}), od)
        owords += w
        oem = oem + e
    assert np.array_equal(words, owords) and em == oem
    fin = O.Final(od, owords, oem)
    try:
        for p in parts:
            s, _ = p.c_struct(p.contig_ids_for(None))
            chars = np.zeros(max(1, int(p.qual_offset[-1])), dtype=np.uint16)
            ln = np.zeros(max(1, p.n_reads), dtype=np.int32)
            assert L.bqsr_jni_apply(ctx.handle, lut, ctypes.byref(s), chars.ctypes.data_as(ctypes.c_void_p),
                                    ln.ctypes.data_as(ctypes.c_void_p)) == 0
            ref, ref_len = O.apply(p, fin)
            elig = np.array([bool(L.bqsr_jni_eligible(int(f))) for f in p.flags[:p.n_reads]])
            assert np.array_equal(ln[:p.n_reads][elig], ref_len[:p.n_reads][elig].astype(np.int32))
            assert (ln[:p.n_reads][~elig] == -1).all()
            for r in np.flatnonzero(elig)[:2000]:
                o = int(p.qual_offset[r])
                assert np.array_equal(chars[o:o + ln[r]], ref[o:o + ln[r]]), r
    finally:
        _capi.lib().bqsr_lut_destroy(lut)
