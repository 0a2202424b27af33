# timing probe (wrong counts): the lean observe resolves a read's deferred
# trimming (kInfoTrim) without loading its first and last 16 quals -- the
# range taken as [0, lq) -- so each wavefront iteration has one dependent
# memory round trip less (record -> trim quals -> chunks)
import os, sys
p = sys.argv[1] + "/bqsr_observe_lean.hip"
s = open(p).read()
old = "      x = lane_read(P.rd, P.info, r, live, L);"
assert old in s
new = ("      {\n"
       "        ReadMeta m{0, 0, 0, 0, 0};\n"
       "        ReadInfo inf{0, 0, 0, 0};\n"
       "        if (live) { m = P.rd.meta[r]; inf = P.info[r]; }\n"
       "        const bool tr = inf.fl & kInfoTrim;\n"
       "        if (tr) { inf.st = 0; inf.en = m.lq; inf.fl &= (uint16_t)~kInfoTrim; }\n"
       "        x = lane_decode(live ? r : P.rd.n_reads, m, inf, m.slot, L);\n"
       "        x.trimmed = tr;\n"
       "      }")
s = s.replace(old, new, 1)
open(p, "w").write(s)
sys.path.insert(0, os.path.dirname(__file__))
import _no_errors
_no_errors.apply(sys.argv[1])
