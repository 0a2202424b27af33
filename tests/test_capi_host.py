"""The C-ABI library on a host without a GPU: it loads, exports every function
include/*.h declare, and its host-only tables agree with the oracle.
No call here touches a HIP device."""
import ctypes
import math
import os
import re

import numpy as np

import oracle as O
from adam_amd import _capi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    names = set()
    for h in sorted(os.listdir(os.path.join(ROOT, "include"))):
        if h.endswith(".h"):
            text = open(os.path.join(ROOT, "include", h)).read()
            text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
            names |= set(re.findall(r"\b(bqsr_[a-z0-9_]+)\s*\(", text))
    return sorted(names)


def test_library_exports_every_declared_function():
    lib = ctypes.CDLL(_capi.LIB_PATH)
    names = header_functions()
    assert len(names) >= 40
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert set(_capi.EXPORTS) <= set(names)


def test_abi_version_and_status_names():
    L = _capi.lib()
    assert L.bqsr_abi_version() >= 1
    for code, name in enumerate(_capi.STATUS_NAMES):
        assert L.bqsr_status_name(code).decode() == name


def test_phred_threshold_table_matches_oracle():
    # errorProbabilityToPhred as the apply kernel evaluates it (thresholds of a
    # step function) vs the oracle's javaD2I(-10 * log10(p)) (PhredUtils.scala:36-38)
    L = _capi.lib()
    qmin = ctypes.c_int32()
    n = L.bqsr_phred_threshold_table(None, 0, ctypes.byref(qmin))
    thr = np.zeros(n, dtype=np.float64)
    L.bqsr_phred_threshold_table(thr.ctypes.data_as(ctypes.c_void_p), n, ctypes.byref(qmin))

    def q_of(p):  # largest i with p <= thr[i]
        i = int(np.searchsorted(-thr, -p, side="right")) - 1
        return qmin.value + i

    rng = np.random.default_rng(5)
    ps = list(10.0 ** rng.uniform(-30, 0.5, 20000)) + [O.pow10cache(q) for q in range(256)]
    ps += [math.nextafter(O.pow10cache(q), 0.0) for q in range(1, 120)]
    ps += [math.nextafter(O.pow10cache(q), 1.0) for q in range(1, 120)]
    ps += [1e-6, 1.0, 1.5, 2.0, 1e-300, 5e-324]
    for p in ps:
        assert q_of(p) == O.error_prob_to_phred(p), p
