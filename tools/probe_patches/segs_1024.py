# A/B build: bqsr_fold_segs with 1024 threads (tiles in chunks of 1024: 2 chunks of a cfg2 candidate block's 1085 tiles, not 3)
import sys
p = sys.argv[1] + "/bqsr_fold.hip"
s = open(p).read()
old = "constexpr int kSegThreads = 512, kSegWaves = kSegThreads / 64;"
assert old in s
s = s.replace(old, "constexpr int kSegThreads = 1024, kSegWaves = kSegThreads / 64;", 1)
open(p, "w").write(s)
