# A/B build: bqsr_apply_kernel with the clean-row test in every piece (one walk instance)
import sys
p = sys.argv[1] + "/bqsr_kernels.hip"
s = open(p).read()
old = "    if (pc.folded_clean) {\n      const auto fchunk"
assert old in s
s = s.replace(old, "    if (false) {\n      const auto fchunk", 1)
open(p, "w").write(s)
