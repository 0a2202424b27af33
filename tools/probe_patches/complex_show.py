# diagnostic build: bqsr_prep_complex prints the listed reads of its first 8 blocks (device printf)
import sys
p = sys.argv[1] + "/bqsr_kernels.hip"
s = open(p).read()
old = """  const uint32_t k = P.n_work[blockIdx.x];
  const int64_t c0 = (int64_t)blockIdx.x * kPrepChunk;"""
assert old in s
s = s.replace(old, old + """
  if (blockIdx.x < 8 && threadIdx.x < k) {
    const int64_t rr = (int64_t)P.work[c0 + threadIdx.x];
    const ReadMeta m = P.rd.meta[rr];
    const ReadAlign a = P.rd.align[rr];
    const uint32_t* cg = P.rd.cigar + a.cigar_off;
    printf("LISTED r %ld flags %x lq %d ls %d ncig %d mdlen %d start %ld cig %x %x %x md %.16s\\n", (long)rr, (unsigned)m.flags,
           (int)m.lq, (int)m.ls, (int)a.n_cigar, (int)a.md_len, (long)a.start, a.n_cigar > 0 ? cg[0] : 0u,
           a.n_cigar > 1 ? cg[1] : 0u, a.n_cigar > 2 ? cg[2] : 0u, (const char*)(P.rd.md + a.md_off));
  }""", 1)
open(p, "w").write(s)
