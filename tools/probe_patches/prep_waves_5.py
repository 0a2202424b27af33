# A/B build: the atomic-form prep kernel at 5 waves per SIMD (launch bounds; 6 by default: 80 VGPRs)
import sys
p = sys.argv[1] + "/bqsr_kernels.hip"
s = open(p).read()
old = "__launch_bounds__(kPrepThreads, kStore ? 1 : 6)"
assert old in s
s = s.replace(old, "__launch_bounds__(kPrepThreads, kStore ? 1 : 5)", 1)
open(p, "w").write(s)
