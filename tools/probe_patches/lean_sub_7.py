# A/B build (correct results): the lean observe walks 7 chunks (112 offsets)
# per step instead of 8 -- a 100-bp read's whole span, fewer registers
import sys
p = sys.argv[1] + "/bqsr_observe_lean.hip"
s = open(p).read()
old = "constexpr int kLeanSub = 8;"
assert old in s
s = s.replace(old, "constexpr int kLeanSub = 7;", 1)
open(p, "w").write(s)
