# A/B build: reads per bqsr_prep_kernel workgroup (kPrepChunk; 2048 = 8 per thread, pipelined two ahead)
import sys
p = sys.argv[1] + "/bqsr_kernels.hip"
s = open(p).read()
old = "constexpr int kPrepChunk = 2048;"
assert old in s
s = s.replace(old, "constexpr int kPrepChunk = 4096;", 1)
open(p, "w").write(s)
