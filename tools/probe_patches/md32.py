# A/B build: prep's lock-step form (and the fused observe's) takes MD tags up
# to 32 bytes: one unrolled 16-byte parse run over bytes 16..31 as well, the
# second 16 bytes loaded only for such a tag
import sys
p = sys.argv[1] + "/bqsr_kernels.hip"
s = open(p).read()
def rep(old, new):
    global s
    assert s.count(old) == 1, old[:60]
    s = s.replace(old, new, 1)
rep("constexpr int kFastCigOps = 5;  // CIGAR elements of a common read: S? M ((I|D) M)? S?",
    "constexpr int kFastCigOps = 5;  // CIGAR elements of a common read: S? M ((I|D) M)? S?\nconstexpr int kFastMd = 32;     // MD bytes of a common read (fast_md)")
rep("    if (usable_read(f) && a.md_len > 0 && a.md_len <= 16) c.md4 = *(const uint4*)(rd.md + a.md_off);",
    "    if (usable_read(f) && a.md_len > 0 && a.md_len <= kFastMd) c.md4 = *(const uint4*)(rd.md + a.md_off);")
i = s.index("__device__ __forceinline__ FastMd fast_md(const uint4 md4, int n, const FastCig& cg, int st, int en) {")
j = s.index("  r.ok &= prev == 1 && !over;  // ends with digits", i)
body = '''__device__ __forceinline__ FastMd fast_md(const uint4 md4, const uint4 md4b, int n, const FastCig& cg, int st, int en) {
  uint32_t num = 0, pos = 0;
  bool over = false;
  int prev = 0;
  FastMd r{n > 0, en < 256, 0ull, 0};
  uint32_t lsh = 0;
  uint4 cur = md4;
#pragma nounroll
  for (int part = 0; part < 2; ++part) {
    const uint32_t w[4] = {cur.x, cur.y, cur.z, cur.w};
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const uint32_t c = __builtin_amdgcn_ubfe(w[i >> 2], 8 * (i & 3), 8);
      if (16 * part + i < n) {
        const uint32_t d = c - '0';
        if (d < 10u) {
          r.ok &= prev != 3;
          over |= num > 214748364u;
          num = num * 10u + d;
          over |= num > 0x7FFFFFFFu;
          prev = 1;
        } else {
          if (prev == 1) {
            r.ok &= !over;
            pos = min(pos + num, 0x7FFFFFFFu);
            num = 0;
            over = false;
          }
          if (c == '^') {
            r.ok &= prev == 1;
            prev = 3;
          } else {
            r.ok &= md_base((uint8_t)c) && prev != 0;
            if (pos < (uint32_t)cg.span) {
              const int32_t o = fc_offset(cg, (int32_t)pos);
              if (o >= st && o < en) {
                r.listed &= lsh < 64;
                r.lst |= lsh < 64 ? (uint64_t)(o + 1) << lsh : 0ull;
                lsh += 8;
              }
            }
            pos = min(pos + 1u, 0x7FFFFFFFu);
            prev = 2;
          }
        }
      }
    }
    if (!__builtin_amdgcn_ballot_w64(n > 16)) break;
    cur = md4b;
  }
'''
s = s[:i] + body + s[j:]
rep("  if (usable && (a.md_len == 0 || a.md_len > 16)) return false;", "  if (usable && (a.md_len == 0 || a.md_len > kFastMd)) return false;")
rep("    const FastMd md = fast_md(cols.md4, a.md_len, c, st, en);",
    "    const uint4 md4b = a.md_len > 16 ? *(const uint4*)(P.rd.md + a.md_off + 16) : make_uint4(0, 0, 0, 0);\n    const FastMd md = fast_md(cols.md4, md4b, a.md_len, c, st, en);")
rep("""      if (!md.listed) {  // more than 8 non-matching positions: the tag's per-byte walk
        if (c.x > 0) return false;""", """      if (!md.listed) {  // more than 8 non-matching positions: the tag's per-byte walk
        if (c.x > 0 || a.md_len > 16) return false;""")
open(p, "w").write(s)
p = sys.argv[1] + "/bqsr_observe_lean.hip"
s = open(p).read()
rep("!(usable && (a.md_len == 0 || a.md_len > 16));", "!(usable && (a.md_len == 0 || a.md_len > kFastMd));")
rep("    md = fast_md(cols.md4, a.md_len, c, 0, m.lq);",
    "    md = fast_md(cols.md4, a.md_len > 16 ? *(const uint4*)(P.rd.md + a.md_off + 16) : make_uint4(0, 0, 0, 0), a.md_len, c, 0, m.lq);")
open(p, "w").write(s)
