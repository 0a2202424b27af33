# bqsr_window_reduce: slabs per thread (kRedSlabs) from the environment of the build: RED_SLABS=N
import os, sys
p = sys.argv[1] + "/bqsr_internal.h"
s = open(p).read()
old = "constexpr int kRedSlabs = 16;"
assert s.count(old) == 1
s = s.replace(old, "constexpr int kRedSlabs = %d;" % int(os.environ["RED_SLABS"]))
open(p, "w").write(s)
