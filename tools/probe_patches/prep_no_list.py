# timing probe (wrong results): bqsr_prep_kernel<false> without its listed reads (prep_one)
import os, sys
p = sys.argv[1] + "/bqsr_kernels.hip"
s = open(p).read()
old = """  if (!kStore) {
    for (uint32_t i = threadIdx.x; i < k; i += kPrepThreads)
      prep_one(P, (int64_t)list[i], &s_cig[threadIdx.x * kPrepCigStride], &s_md[threadIdx.x * kPrepMdStride]);
    return;
  }"""
assert old in s
s = s.replace(old, """  if (!kStore) {
    if (k == 0xFFFFFFFFu)
      prep_one(P, (int64_t)list[0], &s_cig[threadIdx.x * kPrepCigStride], &s_md[threadIdx.x * kPrepMdStride]);
    return;
  }""", 1)
open(p, "w").write(s)
sys.path.insert(0, os.path.dirname(__file__))
import _no_errors
_no_errors.apply(sys.argv[1])
