# diagnostic build: clock stamps (s_memtime) through prep_one for the listed reads of
# the first prep workgroups, printed at the end (device printf)
import sys
p = sys.argv[1] + "/bqsr_kernels.hip"
s = open(p).read()
def rep(old, new):
    global s
    assert s.count(old) == 1, old[:60]
    s = s.replace(old, new, 1)
rep("""__device__ void prep_one(const PrepParams& P, int64_t r, uint32_t* s_cig, uint32_t* s_md) {
  const ReadMeta m = P.rd.meta[r];""", """__device__ uint64_t g_clk[8];
__device__ void prep_one(const PrepParams& P, int64_t r, uint32_t* s_cig, uint32_t* s_md) {
  g_clk[0] = __builtin_amdgcn_s_memtime();
  const ReadMeta m = P.rd.meta[r];""")
rep("""  int st, en;
  trim_quals(P.rd.qual + m.slot, m.lq, st, en);  // isLowQualityBase, minQuality = 2
  inf.st = (uint16_t)min(st, 0xFFFF);""", """  int st, en;
  g_clk[1] = __builtin_amdgcn_s_memtime() + (uint64_t)(m.lq & 0);
  trim_quals(P.rd.qual + m.slot, m.lq, st, en);  // isLowQualityBase, minQuality = 2
  g_clk[2] = __builtin_amdgcn_s_memtime() + (uint64_t)(st & 0);
  inf.st = (uint16_t)min(st, 0xFFFF);""")
rep("""  // walk the CIGAR once: clip, read-consuming and reference-consuming lengths
  const int ncig = a.n_cigar;""", """  g_clk[3] = __builtin_amdgcn_s_memtime() + (uint64_t)(cig[0] & 0);
  // walk the CIGAR once: clip, read-consuming and reference-consuming lengths
  const int ncig = a.n_cigar;""")
rep("""  // ---- masked / mismatch bits over [st, en) ----""", """  g_clk[4] = __builtin_amdgcn_s_memtime();
  // ---- masked / mismatch bits over [st, en) ----""")
rep("""  // positions past the MD span but before `end` are not matches either""", """  g_clk[5] = __builtin_amdgcn_s_memtime() + (uint64_t)(md_total & 0);
  // positions past the MD span but before `end` are not matches either""")
rep("""  if (!kStore) {
    for (uint32_t i = threadIdx.x; i < k; i += kPrepThreads)
      prep_one(P, (int64_t)list[i], &s_cig[threadIdx.x * kPrepCigStride], &s_md[threadIdx.x * kPrepMdStride]);
    return;
  }""", """  if (!kStore) {
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (uint32_t i = threadIdx.x; i < k; i += kPrepThreads)
      prep_one(P, (int64_t)list[i], &s_cig[threadIdx.x * kPrepCigStride], &s_md[threadIdx.x * kPrepMdStride]);
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (blockIdx.x < 6 && threadIdx.x == 0 && k > 0)
      printf("PCLK blk %u k %u total %lu meta %lu trim %lu stage %lu check %lu bits %lu rest %lu\\n", blockIdx.x, k,
             (unsigned long)(t1 - t0), (unsigned long)(g_clk[1] - g_clk[0]), (unsigned long)(g_clk[2] - g_clk[1]),
             (unsigned long)(g_clk[3] - g_clk[2]), (unsigned long)(g_clk[4] - g_clk[3]), (unsigned long)(g_clk[5] - g_clk[4]),
             (unsigned long)(t1 - g_clk[5]));
    return;
  }""")
open(p, "w").write(s)
