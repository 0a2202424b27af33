# timing probe (wrong counts): the lean observe takes every read of a cfg2
# batch (10M x 100 bp, one read group, 112-slot spans) from its index alone --
# slot 112 r, [st, en) = [0, 100), strand and mate from r's low bits -- so a
# wavefront iteration has no dependent round trip before its chunk loads
# (record + info -> trim quals -> chunks): the ceiling of prefetching them
import os, sys
p = sys.argv[1] + "/bqsr_observe_lean.hip"
s = open(p).read()
old = "      x = lane_read(P.rd, P.info, r, live, L);"
assert old in s
new = ("      {\n"
       "        ReadMeta m{(uint64_t)r * 112u, 100, 100, 0, 0};\n"
       "        ReadInfo inf{0, 100, (uint16_t)(kInfoObs | ((r & 1) ? kInfoNeg : 0) | ((r & 2) ? kInfoSecond : 0)), 0};\n"
       "        x = lane_decode(live ? r : P.rd.n_reads, m, inf, m.slot, L);\n"
       "        x.trimmed = false;\n"
       "        if (!live) x.fl = 0;\n"
       "      }")
s = s.replace(old, new, 1)
open(p, "w").write(s)
sys.path.insert(0, os.path.dirname(__file__))
import _no_errors
_no_errors.apply(sys.argv[1])
