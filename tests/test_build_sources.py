"""build()'s staleness stamp covers every source the library compiles: each
file bqsr_capi.cpp pulls in through local #includes (transitively) is listed in
__graft_entry__.LIB_SRC, so an edit to any of them rebuilds the library."""
import os
import re

import __graft_entry__ as ge

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _includes(path, seen):
    if path in seen:
        return
    seen.add(path)
    with open(os.path.join(ROOT, path)) as fh:
        for m in re.finditer(r'^#include "([^"]+)"', fh.read(), re.M):
            inc = os.path.normpath(os.path.join(os.path.dirname(path), m.group(1)))
            _includes(inc, seen)


def test_lib_sources_cover_includes():
    seen = set()
    _includes("adam_amd/csrc/bqsr_capi.cpp", seen)
    missing = sorted(seen - set(os.path.normpath(f) for f in ge.LIB_SRC))
    assert not missing, missing
