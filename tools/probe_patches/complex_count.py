# diagnostic build: bqsr_prep_complex prints its blocks' listed-read counts above 8 (device printf)
import sys
p = sys.argv[1] + "/bqsr_kernels.hip"
s = open(p).read()
old = """  const uint32_t k = P.n_work[blockIdx.x];
  const int64_t c0 = (int64_t)blockIdx.x * kPrepChunk;"""
assert old in s
s = s.replace(old, old + """
  if (threadIdx.x == 0 && (k > 8 || blockIdx.x < 4)) printf("COMPLEX block %u k %u\\n", blockIdx.x, k);""", 1)
open(p, "w").write(s)
