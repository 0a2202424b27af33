# prep's word-store form (known sites) leaves indel reads to bqsr_prep_complex, as in round 4
import sys
p = sys.argv[1] + "/bqsr_kernels.hip"
s = open(p).read()
old = "  if (!fast_cigar(cw, a.n_cigar, m, a.start, c)) return false;\n"
assert s.count(old) == 1
s = s.replace(old, old + "  if (kStore && c.x > 0) return false;\n")
open(p, "w").write(s)
