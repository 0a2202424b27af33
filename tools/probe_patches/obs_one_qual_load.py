# timing probe (wrong counts): bqsr_observe_lean's 8 chunks of a step all take
# the first chunk's quals (one qual load a step instead of 8)
import os, sys
p = sys.argv[1] + "/bqsr_observe_lean.hip"
s = open(p).read()
old = "        qs[i] = lv ? *(const uint4*)(qp + o0) : make_uint4(0, 0, 0, 0);"
assert old in s
s = s.replace(old, "        qs[i] = lv ? (i == 0 ? *(const uint4*)(qp + o0) : qs[0]) : make_uint4(0, 0, 0, 0);", 1)
open(p, "w").write(s)
sys.path.insert(0, os.path.dirname(__file__))
import _no_errors
_no_errors.apply(sys.argv[1])
