# prep_one forced inline (the tree lets the compiler outline it once prep_long sits beside it)
import sys
p = sys.argv[1] + "/bqsr_kernels.hip"
s = open(p).read()
old = "__device__ void prep_one(const PrepParams& P, int64_t r, uint32_t* s_cig, uint32_t* s_md) {"
assert s.count(old) == 1
s = s.replace(old, old.replace("__device__ void", "__device__ __forceinline__ void"))
open(p, "w").write(s)
