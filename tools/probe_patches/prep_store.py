# A/B build: prep's word-store form (every sbits word stored, no zero fill) without known sites too
import sys
p = sys.argv[1] + "/bqsr_capi.cpp"
s = open(p).read()
old = "    P.store_words = b->dims.max_len <= 128 && P.sites.n_contigs > 0;"
assert old in s
s = s.replace(old, "    P.store_words = b->dims.max_len <= 128;", 1)
open(p, "w").write(s)
