# timing probe (wrong counts): bqsr_observe_lean's clean chunks without the
# masked / mismatch fix-up loop
import sys
p = sys.argv[1] + "/bqsr_observe_lean.hip"
s = open(p).read()
old = "  uint32_t mk = bm | bx;\n  if (__builtin_amdgcn_ballot_w64(mk != 0)) {"
assert old in s
s = s.replace(old, "  uint32_t mk = 0;\n  if (__builtin_amdgcn_ballot_w64(mk != 0)) {", 1)
open(p, "w").write(s)
