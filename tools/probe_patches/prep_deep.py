# A/B build: bqsr_prep_kernel's software pipeline one read deeper (records
# three iterations ahead, CIGAR / MD two) at 5 waves per SIMD
import sys
p = sys.argv[1] + "/bqsr_kernels.hip"
s = open(p).read()
old = """  PrepRec x0 = prep_rec(P, rt), x1 = prep_rec(P, rt + kPrepThreads);
  PrepCols k0 = prep_cols(P, x0);
  for (int i = 0; i < kPrepChunk; i += kPrepThreads) {
    const int64_t r = rt + i;
    const PrepRec x2 = i + 2 * kPrepThreads < kPrepChunk ? prep_rec(P, r + 2 * kPrepThreads) : PrepRec{};
    const PrepCols k1 = i + kPrepThreads < kPrepChunk ? prep_cols(P, x1) : PrepCols{};"""
new = """  PrepRec x0 = prep_rec(P, rt), x1 = prep_rec(P, rt + kPrepThreads), x2 = prep_rec(P, rt + 2 * kPrepThreads);
  PrepCols k0 = prep_cols(P, x0), k1 = prep_cols(P, x1);
  for (int i = 0; i < kPrepChunk; i += kPrepThreads) {
    const int64_t r = rt + i;
    const PrepRec x3 = i + 3 * kPrepThreads < kPrepChunk ? prep_rec(P, r + 3 * kPrepThreads) : PrepRec{};
    const PrepCols k2 = i + 2 * kPrepThreads < kPrepChunk ? prep_cols(P, x2) : PrepCols{};"""
assert old in s
s = s.replace(old, new, 1)
old = """    x0 = x1;
    x1 = x2;
    k0 = k1;"""
new = """    x0 = x1;
    x1 = x2;
    x2 = x3;
    k0 = k1;
    k1 = k2;"""
assert old in s
s = s.replace(old, new, 1)
old = "__launch_bounds__(kPrepThreads, kStore ? 1 : 6) bqsr_prep_kernel"
assert old in s
s = s.replace(old, "__launch_bounds__(kPrepThreads, kStore ? 1 : 5) bqsr_prep_kernel", 1)
open(p, "w").write(s)
