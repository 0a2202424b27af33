# listed reads straight to prep_one (no long form first)
import sys
p = sys.argv[1] + "/bqsr_kernels.hip"
s = open(p).read()
n = s.count("if (!prep_long(P, ")
assert n == 2, n
s = s.replace("if (!prep_long(P, (int64_t)list[i]))", "").replace("if (!prep_long(P, (int64_t)P.work[c0 + i]))", "")
open(p, "w").write(s)
