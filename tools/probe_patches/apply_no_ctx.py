# timing probe: bqsr_apply_kernel with every context taken as slot 4 (no base
# loads, no context-table lookups)
import os, sys
p = sys.argv[1] + "/bqsr_kernels.hip"
s = open(p).read()
old = "    chunk_ctx(P.rd, x.fl & kInfoNeg, chunk_n0(x, o0), ld.cr, j, pc.tb, xo);"
assert old in s
s = s.replace(old, "", 1)
old = "    if (!(x.fl & kInfoPass)) v.cr = chunk_raw(P.rd, chunk_n0(x, o0));"
assert old in s
s = s.replace(old, "", 1)
open(p, "w").write(s)
sys.path.insert(0, os.path.dirname(__file__))
import _no_errors
_no_errors.apply(sys.argv[1])
