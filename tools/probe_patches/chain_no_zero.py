# the bitmap cleared by the apply kernel only (not by the fold chain's spare workgroups)
import sys
p = sys.argv[1] + "/bqsr_capi.cpp"
s = open(p).read()
old = "const bool zero = !fork && b->sbits_atomic && !b->sbits_zero;"
assert s.count(old) == 1
s = s.replace(old, "const bool zero = false;")
open(p, "w").write(s)
