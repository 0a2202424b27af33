// bqsr_kernels.hip -- gfx950 kernels of the BQSR path.
//
//   bqsr_prep_kernel / _complex  per read: ReadCovariates' constructor + the
//                         per-read parts of next() (trimming, CIGAR, MD, known
//                         sites) -> ReadInfo + the 2-bit slot bitmap
//   bqsr_observe_chunks   RecalTable.+= over bucketed batches (several read
//                         groups): a lane per 16-offset chunk (chunk_walk)
//                         (read order: bqsr_observe_lean.hip)
//   bqsr_window_reduce    the workgroups' LDS windows -> the int64 table
//   bqsr_key_*            counting sort of reads by (front, read group, mate)
//   bqsr_fold_hist        the expectedMismatch fold's per-block quality
//                         histograms of bucketed batches (bqsr_fold.hip folds)
//   bqsr_final_*          RecalTable.finalizeTable + the apply tables
//   bqsr_apply_chars / bqsr_apply_kernel  RecalUtil.recalibrate over every
//                         eligible read (char tables, then the chunk walk)
//   bqsr_table_add        RecalTable.++ (int64 counts)
//   staged expand / copies / job status  the streamed path's plumbing
//
// DESIGN.md section 3 has the account of each kernel and its measurements.
// Compiled with -ffp-contract=off: the double arithmetic must round exactly
// as the JVM's.
#include <hip/hip_runtime.h>

#include "bqsr_internal.h"

namespace bqsr {

// ---------------------------------------------------------------- helpers --

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ bool usable_read(uint16_t f) {  // RecalibrateBaseQualities.scala:29-32
  return (f & BQSR_F_MAPPED) && (f & BQSR_F_PRIMARY) && !(f & BQSR_F_DUPLICATE) && (f & BQSR_F_HAS_MD);
}
__device__ __forceinline__ bool eligible_read(uint16_t f) {  // RecalibrateBaseQualities.scala:69
  return (f & BQSR_F_MAPPED) && (f & BQSR_F_PRIMARY) && !(f & BQSR_F_DUPLICATE);
}

__device__ __forceinline__ void report(unsigned long long* err, uint64_t key) { atomicMin(err, (unsigned long long)key); }

__device__ __forceinline__ uint32_t cig_op(uint32_t e) { return e & 0xFu; }
__device__ __forceinline__ uint32_t cig_len(uint32_t e) { return e >> 4; }
__device__ __forceinline__ bool is_seg_op(uint32_t op) {  // emits reference positions
  return op == BQSR_CIGAR_M || op == BQSR_CIGAR_X || op == BQSR_CIGAR_EQ || op == BQSR_CIGAR_S;
}
__device__ __forceinline__ bool consumes_ref(uint32_t op) {
  return op == BQSR_CIGAR_M || op == BQSR_CIGAR_D || op == BQSR_CIGAR_N || op == BQSR_CIGAR_EQ || op == BQSR_CIGAR_X;
}

// MdTag basesPattern after toUpperCase (MdTag.scala:36)
__device__ __forceinline__ bool md_base(uint8_t c) {
  if (c >= 'a' && c <= 'z') c = (uint8_t)(c - 32);
  switch (c) {
    case 'A': case 'G': case 'C': case 'T': case 'N': case 'U': case 'K': case 'M': case 'R':
    case 'S': case 'W': case 'B': case 'V': case 'H': case 'D': case 'X': case 'Y':
      return true;
    default:
      return false;
  }
}

// MdTag.apply (MdTag.scala:38-98): validates the tag and calls nonmatch(p) for
// every mismatch / deleted position p (relative to start) in order; *total =
// the reference span the tag describes.  isMatch(p) == p in [0,total) && p
// was not reported.
// (MdPtr / CigPtr below: LDS-typed pointers for the staged copies -- a
// generic pointer made every byte a flat load, each waited for alone: the
// per-read path took ~60 us a read)
template <class MdPtr, class F>
__device__ bool md_scan(MdPtr md, int n, int64_t* total, F&& nonmatch) {
  int off = 0;
  int64_t pos = 0;
  *total = 0;
  if (n == 0) return true;
  auto digits = [&]() -> bool {
    int b = off;
    int64_t v = 0;
    while (off < n && md[off] >= '0' && md[off] <= '9') {
      v = v * 10 + (md[off] - '0');
      if (v > 2147483647LL) return false;  // Integer.parseInt overflow
      ++off;
    }
    if (off == b) return false;
    pos += v;
    return true;
  };
  if (!digits()) return false;
  while (off < n) {
    if (md[off] == '^') ++off;
    int b = off;
    while (off < n && md_base(md[off])) {
      nonmatch(pos + (off - b));
      ++off;
    }
    if (off == b) return false;
    pos += off - b;
    if (!digits()) return false;
  }
  *total = pos;
  return true;
}

// read offset holding reference position p, or -1 (position in no M/X/=/S element)
template <class CigPtr>
__device__ int refpos_to_offset(CigPtr cig, int ncig, int64_t unclipped, int64_t p) {
  int ro = 0;
  int64_t pos = unclipped;
  for (int i = 0; i < ncig; ++i) {
    uint32_t e = cig[i], op = cig_op(e), len = cig_len(e);
    if (is_seg_op(op)) {
      if (p < pos) return -1;
      if (p < pos + (int64_t)len) return ro + (int)(p - pos);
      ro += len;
      pos += len;
    } else if (op == BQSR_CIGAR_I) {
      ro += len;
    } else if (op != BQSR_CIGAR_H) {
      pos += len;
    }
  }
  return -1;
}

// set bits [lo, hi) (absolute base slots) of the batch's slot bitmap: word i
// holds slots 32i..32i+31 at bit `half` (0 masked, 32 mismatch).  Two reads
// can share a word, hence the atomics (few per read: most reads have no
// masked base and a handful of mismatches).
__device__ void set_sbits(uint64_t* sb, uint64_t lo, uint64_t hi, int half) {
  while (lo < hi) {
    const uint64_t i = lo >> 5;
    const int b = (int)(lo & 31);
    const int n = (int)min((uint64_t)(32 - b), hi - lo);
    const uint32_t m = (n == 32) ? 0xFFFFFFFFu : (((1u << n) - 1u) << b);
    atomicOr((unsigned long long*)&sb[i], (unsigned long long)m << half);
    lo += (uint64_t)n;
  }
}

// ---------------------------------------------------------------- prep -----
//
// One thread per read.  Eligible reads (mapped, primary, not duplicate) get
// trimmed and validated in the order ReadCovariates would throw; usable reads
// (eligible + MD) also get their masked / mismatch bitmaps:
//   masked   = refPos None, refPos outside [start, end), or a known site
//              (ReadCovariates.scala:56: snp(o) || mismatch(o).isEmpty);
//   mismatch = !MdTag.isMatch(refPos)  (RichADAMRecord.scala:138-154).
// Errors of usable reads are errors of observe; those of every eligible read
// are errors of apply (observe runs first).
// First index k < n (n <= 16) of the 16 bytes w whose qual is above 2
// (isLowQualityBase: qual <= minQuality = 2, Java signed byte), or 16; with
// `rev` the bytes are scanned from byte 15 down.
__device__ __forceinline__ int first_good(const uint4 v, int n, bool rev) {
  // SWAR: bit 7 of byte b set iff the byte is a qual in [3, 127] ((x & 0x7F) + 0x7D carries into bit 7
  // from 3 on, never past the byte; a set high bit is a negative Java byte)
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  uint32_t g[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) g[i] = ((w[i] & 0x7F7F7F7Fu) + 0x7D7D7D7Du) & ~w[i] & 0x80808080u;
  uint64_t lo = ((uint64_t)g[1] << 32) | g[0], hi = ((uint64_t)g[3] << 32) | g[2];
  if (n < 16) {  // bytes k >= n (scan order) do not count
    const int keep = n <= 0 ? 0 : n;
    if (!rev) {
      lo &= keep >= 8 ? ~0ull : ((1ull << (8 * keep)) - 1ull);
      hi &= keep <= 8 ? 0ull : ((1ull << (8 * (keep - 8))) - 1ull);
    } else {
      hi &= keep >= 8 ? ~0ull : ~((1ull << (8 * (8 - keep))) - 1ull);
      lo &= keep <= 8 ? 0ull : ~((1ull << (8 * (16 - keep))) - 1ull);
    }
  }
  if (!rev) return lo ? (__builtin_ctzll(lo) >> 3) : hi ? 8 + (__builtin_ctzll(hi) >> 3) : 16;
  return hi ? (__builtin_clzll(hi) >> 3) : lo ? 8 + (__builtin_clzll(lo) >> 3) : 16;
}

// ReadCovariates' quality trimming (ReadCovariates.scala:31-39): st = the
// number of leading quals <= minQuality (2, Java signed byte), en = lq minus
// the trailing ones.  The first and last 16 quals come in with one load each.
__device__ __forceinline__ void trim_quals(const uint8_t* q, int lq, int& st, int& en) {
  int s = 0, tail = 0;
  bool more_st = true, more_tail = true;
  if (lq >= 16) {
    const uint4 head = *(const uint4*)q, back = *(const uint4*)(q + lq - 16);
    s = first_good(head, 16, false);
    tail = first_good(back, 16, true);
    more_st = s == 16;
    more_tail = tail == 16;
  }
  if (more_st)
    while (s < lq && (int8_t)q[s] <= 2) ++s;
  if (more_tail)
    while (tail < lq && (int8_t)q[lq - 1 - tail] <= 2) ++tail;
  st = s;
  en = lq - tail;
}

// A read's ReadInfo with the trimmed range filled in when prep left it to
// the first pass over the quals (kInfoTrim); what prep_one writes for the
// same read: {st, en, flags}, or {st, 0, 0} when no base is left.
__device__ __forceinline__ ReadInfo resolve_info(const ReadsDev& rd, ReadInfo inf, uint64_t slot, int lq) {
  if (inf.fl & kInfoTrim) {
    int st, en;
    trim_quals(rd.qual + slot, lq, st, en);
    inf.st = (uint16_t)st;
    if (st >= en) {
      inf.en = 0;
      inf.fl = 0;
    } else {
      inf.en = (uint16_t)en;
      inf.fl &= (uint16_t)~kInfoTrim;
    }
  }
  return inf;
}

// Per-thread LDS copies of a read's CIGAR (<= kPrepCig ops) and MD (<= kPrepMd
// bytes): the parsers below then walk LDS instead of issuing one dependent
// global load per element.  Strides of 5 and 9 dwords keep the 64 lanes'
// slots in distinct banks.
constexpr int kPrepThreads = 256;
constexpr int kComplexThreads = 128;  // bqsr_prep_complex: a segment holds a few % of its 2048 reads
constexpr int kPrepCig = 4, kPrepCigStride = 5;
constexpr int kPrepMd = 32, kPrepMdStride = 9;
constexpr int kPrepChunk = 2048;  // reads per workgroup of bqsr_prep_kernel (8 per thread)

template <class CigPtr, class MdPtr>
__device__ void prep_one_rest(const PrepParams& P, int64_t r, const ReadMeta& m, const ReadAlign& a, ReadInfo inf,
                              int st, int en, bool usable, CigPtr cig, MdPtr md);

__device__ __forceinline__ void prep_one(const PrepParams& P, int64_t r, uint32_t* s_cig, uint32_t* s_md) {  // (inline: see bqsr_prep_kernel)
  const ReadMeta m = P.rd.meta[r];
  const ReadAlign a = P.rd.align[r];  // issued with the meta load: one round trip for both
  ReadInfo inf{0, 0, 0, 0};
  const uint16_t f = m.flags;
  if (!eligible_read(f)) {
    inf.fl = kInfoPass;
    P.info[r] = inf;
    return;
  }
  const bool usable = usable_read(f);
  auto fail = [&](uint64_t key) {
    if (usable) report(&P.err[kErrObs], key);
    report(&P.err[kErrAppPrep], key);
  };
  if (!(f & BQSR_F_HAS_QUAL)) {  // qualityScores: getQual.toString
    fail(err_key(r, 0, kRankCtor, BQSR_ERR_NULL_FIELD));
    P.info[r] = inf;
    return;
  }
  int st, en;
  trim_quals(P.rd.qual + m.slot, m.lq, st, en);  // isLowQualityBase, minQuality = 2
  inf.st = (uint16_t)min(st, 0xFFFF);
  if (!(f & BQSR_F_HAS_RG)) {  // QualByRG: 60 * getRecordGroupId
    fail(err_key(r, 0, kRankCtor, BQSR_ERR_NULL_RG));
    P.info[r] = inf;
    return;
  }
  if (!(f & BQSR_F_HAS_SEQ)) {  // DiscreteCycle: getSequence.toString
    fail(err_key(r, 0, kRankCtor, BQSR_ERR_NULL_FIELD));
    P.info[r] = inf;
    return;
  }
  if ((f & BQSR_F_NEG_STRAND) && (f & kSeqOther)) {  // BaseContext reverse complement
    fail(err_key(r, 0, kRankCtor, BQSR_ERR_BAD_REVCOMP_BASE));
    P.info[r] = inf;
    return;
  }
  if (st >= en) {  // no base is iterated: an empty recalibrated quality string
    P.info[r] = inf;
    return;
  }
  const uint16_t check_fl = (usable ? kInfoObsCheck : 0) | kInfoAppCheck;
  if (!(f & BQSR_F_HAS_CIGAR) || !(f & BQSR_F_HAS_START)) {  // referencePositions
    fail(err_key(r, st, kRankCigar, BQSR_ERR_NULL_FIELD));
    inf.en = (uint16_t)st;
    inf.fl = check_fl;
    P.info[r] = inf;
    return;
  }
  const uint32_t* gcig = P.rd.cigar + a.cigar_off;
  const uint8_t* gmd = P.rd.md + a.md_off;
  // short CIGAR / MD (the common case): staged into this thread's LDS slots
  // and read through LDS-typed pointers; otherwise straight from the columns
  const bool sc = a.n_cigar <= kPrepCig, sm = !(f & BQSR_F_HAS_MD) || a.md_len <= kPrepMd;
  typedef __attribute__((address_space(3))) uint32_t* LdsW;
  typedef const __attribute__((address_space(3))) uint32_t* LdsCW;
  typedef const __attribute__((address_space(3))) uint8_t* LdsCB;
  if (sc && sm) {
    const uint4 c4 = *(const uint4*)gcig;
    uint4 m0 = make_uint4(0, 0, 0, 0), m1 = m0;
    if (f & BQSR_F_HAS_MD) {
      m0 = *(const uint4*)gmd;
      m1 = *(const uint4*)(gmd + 16);
    }
    LdsW lc = (LdsW)s_cig, lm = (LdsW)s_md;
    lc[0] = c4.x;
    lc[1] = c4.y;
    lc[2] = c4.z;
    lc[3] = c4.w;
    lm[0] = m0.x;
    lm[1] = m0.y;
    lm[2] = m0.z;
    lm[3] = m0.w;
    lm[4] = m1.x;
    lm[5] = m1.y;
    lm[6] = m1.z;
    lm[7] = m1.w;
    prep_one_rest(P, r, m, a, inf, st, en, usable, (LdsCW)lc, (LdsCB)lm);
  } else {
    prep_one_rest(P, r, m, a, inf, st, en, usable, gcig, gmd);
  }
}

// prep_one after its checks of the record: the CIGAR / MD walks, errors, the
// ReadInfo and the bits (cig / md: LDS-typed or global pointers)
template <class CigPtr, class MdPtr>
__device__ void prep_one_rest(const PrepParams& P, int64_t r, const ReadMeta& m, const ReadAlign& a, ReadInfo inf,
                              int st, int en, bool usable, CigPtr cig, MdPtr md) {
  const uint16_t f = m.flags;
  auto fail = [&](uint64_t key) {
    if (usable) report(&P.err[kErrObs], key);
    report(&P.err[kErrAppPrep], key);
  };
  const uint16_t check_fl = (usable ? kInfoObsCheck : 0) | kInfoAppCheck;
  // walk the CIGAR once: clip, read-consuming and reference-consuming lengths
  const int ncig = a.n_cigar;
  int64_t lead = 0, rp_len = 0, ref_len = 0;
  bool leading = true, zero = false;
  for (int i = 0; i < ncig; ++i) {
    uint32_t e = cig[i], op = cig_op(e), len = cig_len(e);
    if (leading && (op == BQSR_CIGAR_S || op == BQSR_CIGAR_H)) lead += len; else leading = false;
    if (is_seg_op(op) || op == BQSR_CIGAR_I) rp_len += len;
    if (is_seg_op(op) && len == 0) zero = true;
    if (consumes_ref(op)) ref_len += len;
  }
  const int64_t start = a.start;
  const int64_t unclipped = start - lead;
  const int64_t ref_end = start + ref_len;
  uint64_t best = kNoError;
  if (zero) {
    best = err_key(r, st, kRankCigar, BQSR_ERR_CIGAR_INVALID);  // Range(a, a).last
  } else if (unclipped < -2147483648LL || unclipped + rp_len + ref_len > 2147483647LL) {
    // the reference does this arithmetic in Int; positions that wrap are not supported here
    best = err_key(r, st, kRankCigar, BQSR_ERR_UNSUPPORTED);
  } else {
    // first trimmed base that has a reference position
    const int e1 = (int)min((int64_t)en, rp_len);
    int o_first = -1;
    {
      int ro = 0;
      for (int i = 0; i < ncig && o_first < 0; ++i) {
        uint32_t e = cig[i], op = cig_op(e), len = cig_len(e);
        if (is_seg_op(op)) {
          int lo = max(ro, st), hi = min(ro + (int)len, e1);
          if (lo < hi) o_first = lo;
          ro += len;
        } else if (op == BQSR_CIGAR_I) {
          ro += len;
        }
      }
    }
    if (o_first >= 0) {
      int64_t tot;
      if ((f & BQSR_F_HAS_MD) && !md_scan(md, a.md_len, &tot, [](int64_t) {}))
        best = min(best, err_key(r, o_first, kRankMd, BQSR_ERR_MD_PARSE));
      if (!(f & BQSR_F_HAS_REFNAME)) best = min(best, err_key(r, o_first, kRankSnp, BQSR_ERR_NULL_FIELD));
    }
    if ((int64_t)en > rp_len)
      best = min(best, err_key(r, (uint32_t)max((int64_t)st, rp_len), kRankCigar, BQSR_ERR_CIGAR_SHORT));
    if (en > (int)m.ls) best = min(best, err_key(r, (uint32_t)max(st, (int)m.ls), kRankCov, BQSR_ERR_SEQ_SHORT));
  }
  if (best != kNoError) {
    fail(best);
    inf.en = (uint16_t)((best >> 8) & 0xFFFFF);  // bases before the failing one are still checked
    inf.fl = check_fl;
    P.info[r] = inf;
    return;
  }
  inf.en = (uint16_t)en;
  inf.fl = kInfoApp | (usable ? kInfoObs : 0) | ((f & BQSR_F_NEG_STRAND) ? kInfoNeg : 0) |
           (((f & BQSR_F_PAIRED) && (f & BQSR_F_SECOND_OF_PAIR)) ? kInfoSecond : 0);
  P.info[r] = inf;
  if (!usable) return;

  // ---- masked / mismatch bits over [st, en) ----
  uint64_t* bw = P.sbits;
  const uint64_t rs = m.slot;
  {
    int ro = 0;
    int64_t pos = unclipped;
    for (int i = 0; i < ncig; ++i) {
      uint32_t e = cig[i], op = cig_op(e), len = cig_len(e);
      if (is_seg_op(op)) {
        int lo = max(ro, st), hi = min(ro + (int)len, en);
        if (lo < hi) {
          // refPos in [start, ref_end) <=> o in [ro + start - pos, ro + ref_end - pos)
          int64_t w0 = (int64_t)ro + (start - pos), w1 = (int64_t)ro + (ref_end - pos);
          int a0 = (int)min(max(w0, (int64_t)lo), (int64_t)hi);
          int a1 = (int)min(max(w1, (int64_t)lo), (int64_t)hi);
          set_sbits(bw, rs + (uint64_t)(lo), rs + (uint64_t)(a0), 0);
          set_sbits(bw, rs + (uint64_t)(max(a1, a0)), rs + (uint64_t)(hi), 0);
        }
        ro += len;
        pos += len;
      } else if (op == BQSR_CIGAR_I) {  // insertion: refPos None
        int lo = max(ro, st), hi = min(ro + (int)len, en);
        set_sbits(bw, rs + (uint64_t)(lo), rs + (uint64_t)(max(lo, hi)), 0);
        ro += len;
      } else if (op != BQSR_CIGAR_H) {
        pos += len;
      }
    }
  }
  // MD non-match positions inside the overlap window
  int64_t md_total = 0;
  md_scan(md, a.md_len, &md_total, [&](int64_t prel) {
    int64_t p = start + prel;
    if (p >= ref_end) return;
    int o = refpos_to_offset(cig, ncig, unclipped, p);
    if (o >= st && o < en) set_sbits(bw, rs + (uint64_t)(o), rs + (uint64_t)(o + 1), 32);
  });
  // positions past the MD span but before `end` are not matches either
  if (start + md_total < ref_end) {
    int ro = 0;
    int64_t pos = unclipped;
    const int64_t t0 = start + md_total;
    for (int i = 0; i < ncig; ++i) {
      uint32_t e = cig[i], op = cig_op(e), len = cig_len(e);
      if (is_seg_op(op)) {
        int64_t p0 = max(pos, t0), p1 = min(pos + (int64_t)len, ref_end);
        if (p0 < p1) {
          int lo = max(ro + (int)(p0 - pos), st), hi = min(ro + (int)(p1 - pos), en);
          if (lo < hi) set_sbits(bw, rs + (uint64_t)(lo), rs + (uint64_t)(hi), 32);
        }
        ro += len;
        pos += len;
      } else if (op == BQSR_CIGAR_I) {
        ro += len;
      } else if (op != BQSR_CIGAR_H) {
        pos += len;
      }
    }
  }
  // known sites (SnpTable.isMaskedAtReadOffset): raw VCF POS vs 0-based refPos (Q7)
  if (a.contig >= 0 && a.contig < P.sites.n_contigs) {
    const SitesDev& S = P.sites;
    const int64_t* sp = S.pos + S.off[a.contig];
    const int64_t ns = (int64_t)(S.off[a.contig + 1] - S.off[a.contig]);
    if (ns > 0) {
      // reference span of the read: refPos increases along the read
      const int64_t lo_p = unclipped, hi_p = unclipped + rp_len + ref_len;
      const uint32_t* bk = S.bucket + S.bucket_off[a.contig];
      const int64_t nb = (int64_t)(S.bucket_off[a.contig + 1] - S.bucket_off[a.contig]);
      const int64_t base = S.bucket_base[a.contig];
      int64_t j;
      const int64_t bi = (lo_p - base) >> S.shift;
      if (bi < 0) j = 0;
      else if (bi >= nb) j = ns;
      else j = bk[bi];
      while (j < ns && sp[j] < lo_p) ++j;
      for (; j < ns && sp[j] < hi_p; ++j) {
        int o = refpos_to_offset(cig, ncig, unclipped, sp[j]);
        if (o >= st && o < en) set_sbits(bw, rs + (uint64_t)(o), rs + (uint64_t)(o + 1), 0);
      }
    }
  }
}

// Known sites of a read whose reference position at offset o is
// unclipped + o for every offset (CIGAR [S]M[S]): mask the trimmed offsets
// [st, en) holding a site (SnpTable.isMaskedAtReadOffset, raw VCF POS vs
// 0-based refPos, Q7).
__device__ void mask_sites_linear(const PrepParams& P, int32_t contig, int64_t unclipped, int st, int en,
                                  uint64_t rs) {
  if (contig < 0 || contig >= P.sites.n_contigs) return;
  const SitesDev& S = P.sites;
  const int64_t* sp = S.pos + S.off[contig];
  const int64_t ns = (int64_t)(S.off[contig + 1] - S.off[contig]);
  if (ns == 0) return;
  const int64_t lo_p = unclipped + st, hi_p = unclipped + en;
  const uint32_t* bk = S.bucket + S.bucket_off[contig];
  const int64_t nb = (int64_t)(S.bucket_off[contig + 1] - S.bucket_off[contig]);
  const int64_t bi = (lo_p - S.bucket_base[contig]) >> S.shift;
  int64_t j = bi < 0 ? 0 : (bi >= nb ? ns : (int64_t)bk[bi]);
  while (j < ns && sp[j] < lo_p) ++j;
  for (; j < ns && sp[j] < hi_p; ++j) {
    const uint64_t o = (uint64_t)(sp[j] - unclipped);
    set_sbits(P.sbits, rs + o, rs + o + 1, 0);
  }
}

// The same from the contig's position bitmap: 64 offsets per step, one
// funnel shift of two bitmap words (the next step reuses the second), an
// atomic OR per sbits word only where a site falls.  False when the contig
// has no bitmap.
__device__ __forceinline__ bool mask_sites_bitmap(const PrepParams& P, int32_t contig, int64_t unclipped, int lq,
                                                  uint64_t rs) {
  const SitesDev& S = P.sites;
  const int64_t nw = (int64_t)(S.bm_off[contig + 1] - S.bm_off[contig]);
  if (nw == 0) return false;
  const uint64_t* w = S.bm + S.bm_off[contig];
  const int64_t b0 = unclipped - S.bm_base[contig];  // bit of offset 0
  int64_t wi = b0 >> 6;                               // floor
  const uint32_t sh = (uint32_t)(b0 & 63);
  uint64_t lo = (wi >= 0 && wi < nw) ? w[wi] : 0ull;
  for (int o = 0; o < lq; o += 64) {
    ++wi;
    const uint64_t hi = (wi >= 0 && wi < nw) ? w[wi] : 0ull;
    uint64_t m = sh ? (lo >> sh) | (hi << (64 - sh)) : lo;  // bits of offsets o .. o + 63
    lo = hi;
    if (lq - o < 64) m &= (1ull << (lq - o)) - 1ull;
    if (!m) continue;
    // slots s .. s + 63 span sbits words s >> 5 .. (s >> 5) + 2 (masked half: the low 32 bits)
    const uint64_t s = rs + (uint64_t)o;
    const uint32_t sb = (uint32_t)(s & 31);
    const uint64_t lo64 = m << sb, hi64 = sb ? m >> (64 - sb) : 0ull;  // bit k of (hi64:lo64): slot (s & ~31) + k
    const uint32_t p0 = (uint32_t)lo64, p1 = (uint32_t)(lo64 >> 32), p2 = (uint32_t)hi64;
    unsigned long long* sw = (unsigned long long*)&P.sbits[s >> 5];
    if (p0) atomicOr(sw, (unsigned long long)p0);
    if (p1) atomicOr(sw + 1, (unsigned long long)p1);
    if (p2) atomicOr(sw + 2, (unsigned long long)p2);
  }
  return true;
}

constexpr int kFastCigOps = 5;  // CIGAR elements of a common read: S? M ((I|D) M)? S?
struct PrepRec {
  ReadMeta m;
  ReadAlign a;
  uint64_t nslot;  // store_words, last lane of a wavefront: the next read's slot (n_slots past the batch)
};
struct PrepCols {
  uint4 c4, md4;
  uint32_t c5;  // the fifth CIGAR word
};
// A read's sbits words in registers (prep_fast, reads whose bits fit in
// kAccWords words): bit b of the accumulator = slot (rs & ~31) + b; static
// indices only (a dynamic one would put the array in scratch).
constexpr int kAccWords = 5;
__device__ __forceinline__ void acc_range(uint64_t acc[kAccWords], uint32_t lo, uint32_t hi, int half) {
#pragma unroll
  for (int j = 0; j < kAccWords; ++j) {
    const uint32_t a = max(lo, 32u * j), b = min(hi, 32u * j + 32u);
    const uint32_t n = b > a ? b - a : 0u;
    const uint32_t m = n >= 32u ? 0xFFFFFFFFu : (((1u << n) - 1u) << (a - 32u * j));
    acc[j] |= n ? (uint64_t)m << half : 0ull;
  }
}
__device__ __forceinline__ void acc_bit(uint64_t acc[kAccWords], uint32_t b, int half) {
#pragma unroll
  for (int j = 0; j < kAccWords; ++j) acc[j] |= (b >> 5) == (uint32_t)j ? 1ull << ((b & 31) + half) : 0ull;
}
// mask_sites_bitmap into the accumulator (offsets 0 .. lq-1 at bits r0 + o)
__device__ __forceinline__ bool sites_bitmap_acc(const SitesDev& S, int32_t contig, int64_t unclipped, int lq,
                                                 uint32_t r0, uint64_t acc[kAccWords]) {
  const int64_t nw = (int64_t)(S.bm_off[contig + 1] - S.bm_off[contig]);
  if (nw == 0) return false;
  const uint64_t* w = S.bm + S.bm_off[contig];
  const int64_t b0 = unclipped - S.bm_base[contig];
  int64_t wi = b0 >> 6;
  const uint32_t sh = (uint32_t)(b0 & 63);
  uint64_t lo = (wi >= 0 && wi < nw) ? w[wi] : 0ull;
#pragma unroll
  for (int step = 0; step < 2; ++step) {  // offsets 64 step .. 64 step + 63 (lq <= 160 - r0 <= 160)
    const int o = 64 * step;
    if (o >= lq) break;
    ++wi;
    const uint64_t hi = (wi >= 0 && wi < nw) ? w[wi] : 0ull;
    uint64_t m = sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
    lo = hi;
    if (lq - o < 64) m &= (1ull << (lq - o)) - 1ull;
    // bits r0 + o .. : word 2 step + ((r0 + o) >> 5 - 2 step) = 2 step, at bit r0
    const uint64_t lo64 = m << r0, hi64 = r0 ? m >> (64 - r0) : 0ull;
    acc[2 * step] |= (uint64_t)(uint32_t)lo64;
    acc[2 * step + 1] |= (uint64_t)(uint32_t)(lo64 >> 32);
    if (2 * step + 2 < kAccWords) acc[2 * step + 2] |= (uint64_t)(uint32_t)hi64;
  }
  if (lq > 128) {  // offsets 128 .. lq-1 (lq <= 160 - r0 <= 160: at most 32 more)
    ++wi;
    const uint64_t hi = (wi >= 0 && wi < nw) ? w[wi] : 0ull;
    uint64_t m = sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
    m &= (1ull << (lq - 128)) - 1ull;
    const uint64_t lo64 = m << r0;
    acc[4] |= (uint64_t)(uint32_t)lo64;
  }
  return true;
}

// The common read, prepared in lock step (no data-dependent loop) and
// without touching its quals: eligible, every field present, a CIGAR of the
// form [S]M[S] covering the whole read (so the trimmed range, whatever it is,
// has reference positions and no CIGAR_SHORT / SEQ_SHORT can arise), and
// (usable reads) an MD tag of at most 16 bytes without deletions, parsed in
// a fixed 16-step loop.  With that CIGAR the reference position of offset o
// is unclipped + o (RichADAMRecord.scala:101-109,156-187): the clips fall
// outside [start, end) and are masked, and MD position p (MdTag.scala:38-98,
// relative to start) is offset lead + p.  Bits are set over the whole read:
// the per-base passes only read those of the trimmed range.  The trimming
// itself is left to the first pass over the quals (kInfoTrim, resolve_info).
// Returns false for anything else: the read goes to bqsr_prep_complex, which
// runs prep_one with the full exception order.
// A read's columns as prep_fast reads them, loaded an iteration or two
// ahead by bqsr_prep_kernel (the three dependent loads of a read -- record,
// then its CIGAR / MD, then the site bitmap -- were a chain of memory round
// trips per iteration): PrepRec first, PrepCols once the record is in.
__device__ __forceinline__ PrepRec prep_rec(const PrepParams& P, int64_t r) {
  PrepRec x{};
  if (r < P.rd.n_reads) {
    x.m = P.rd.meta[r];
    x.a = P.rd.align[r];
  }
  if (P.store_words && (threadIdx.x & 63) == 63)
    x.nslot = r + 1 < P.rd.n_reads ? P.rd.meta[r + 1].slot : (uint64_t)P.rd.n_slots;
  return x;
}
// (the columns have 32 B of padding; only reads prep_fast may take load)
__device__ __forceinline__ PrepCols prep_cols(const ReadsDev& rd, const ReadMeta& m, const ReadAlign& a) {
  PrepCols c{make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0), 0u};
  const uint16_t f = m.flags;
  if (eligible_read(f) && a.n_cigar > 0 && a.n_cigar <= kFastCigOps) {
    c.c4 = *(const uint4*)(rd.cigar + a.cigar_off);
    if (a.n_cigar > 4) c.c5 = rd.cigar[a.cigar_off + 4];
    if (usable_read(f) && a.md_len > 0 && a.md_len <= 16) c.md4 = *(const uint4*)(rd.md + a.md_off);
  }
  return c;
}
__device__ __forceinline__ PrepCols prep_cols(const PrepParams& P, const PrepRec& x) { return prep_cols(P.rd, x.m, x.a); }


// The common read's CIGAR: S? M ((I|D) M)? S? -- one insertion or deletion
// at most -- covering the whole read, no zero-length element (prep_one's
// CIGAR_INVALID for M / S; a zero I / D is left to prep_one too), the read and
// sequence no longer than the CIGAR's read span (else CIGAR_SHORT / SEQ_SHORT
// may arise), positions inside Int (the reference does this arithmetic in
// Int).  Offsets and reference positions (RichADAMRecord.scala:101-109,
// 156-187): the leading clip and M1 at unclipped + o; an insertion's offsets
// have none; M2 (and the trailing clip) continue after the indel.
struct FastCig {
  int32_t lead, m1, x, m2;  // leading clip, first M, indel length (0: none), second M
  bool del;                 // the indel is a deletion
  int32_t span;             // reference span [start, end): m1 + (del ? x : 0) + m2
  int32_t o_end;            // first offset past M2: the trailing clip starts here
  int64_t unclipped;
};
__device__ __forceinline__ bool fast_cigar(const uint32_t cw[kFastCigOps], int nc, const ReadMeta& m, int64_t start,
                                           FastCig& c) {
  int i = 0;
  int64_t trail = 0;
  c.lead = c.m1 = c.x = c.m2 = 0;
  c.del = false;
  bool ok = nc >= 1 && nc <= kFastCigOps;
  // (static indices: a dynamic one would put cw in scratch)
  auto op = [&](int k) { return cig_op(k == 0 ? cw[0] : k == 1 ? cw[1] : k == 2 ? cw[2] : k == 3 ? cw[3] : cw[4]); };
  auto len = [&](int k) {
    return (int64_t)cig_len(k == 0 ? cw[0] : k == 1 ? cw[1] : k == 2 ? cw[2] : k == 3 ? cw[3] : cw[4]);
  };
  int64_t lead = 0, m1 = 0, x = 0, m2 = 0;
  if (ok && op(0) == BQSR_CIGAR_S) {
    lead = len(0);
    i = 1;
  }
  ok &= i < nc && op(i) == BQSR_CIGAR_M;
  if (ok) m1 = len(i++);
  if (ok && i < nc && (op(i) == BQSR_CIGAR_I || op(i) == BQSR_CIGAR_D)) {
    c.del = op(i) == BQSR_CIGAR_D;
    x = len(i++);
    ok &= x > 0 && i < nc && op(i) == BQSR_CIGAR_M;
    if (ok) m2 = len(i++);
    ok &= m2 > 0;
  }
  if (ok && i < nc && op(i) == BQSR_CIGAR_S) {
    trail = len(i++);
    ok &= trail > 0;
  }
  ok &= i == nc && m1 > 0 && (lead > 0 || op(0) != BQSR_CIGAR_S);
  if (!ok) return false;
  const int64_t rp_len = lead + m1 + (c.del ? 0 : x) + m2 + trail;
  const int64_t ref_len = m1 + (c.del ? x : 0) + m2;
  if (rp_len < m.lq || m.ls < m.lq) return false;
  const int64_t unclipped = start - lead;
  if (unclipped < 0 || unclipped + rp_len + ref_len > 2147483647LL || rp_len > 65535 || ref_len > 65535) return false;
  c.lead = (int32_t)lead;
  c.m1 = (int32_t)m1;
  c.x = (int32_t)x;
  c.m2 = (int32_t)m2;
  c.span = (int32_t)ref_len;
  c.o_end = (int32_t)(lead + m1 + (c.del ? 0 : x) + m2);
  c.unclipped = unclipped;
  return true;
}
// read offset of reference position start + rel (0 <= rel < span), -1 in a deletion
__device__ __forceinline__ int32_t fc_offset(const FastCig& c, int32_t rel) {
  if (rel < c.m1) return c.lead + rel;
  if (c.del) return rel < c.m1 + c.x ? -1 : c.lead + rel - c.x;
  return c.lead + rel + c.x;
}

// MD (MdTag.scala:38-98, md_scan) of at most 16 bytes: digits ('^'? letters
// digits)*, the digit runs <= 2^31 - 1 (Integer.parseInt).  One pass:
// validity, the tag's span, and (reads of < 256 bases) the offsets inside
// [st, en) of its non-matching positions -- mismatch letters and deleted
// bases alike (md_scan reports both) -- as a list of bytes o + 1 (at most 8).
struct FastMd {
  bool ok, listed;
  uint64_t lst;
  int64_t md_total;
};
template <int kN>
__device__ __forceinline__ FastMd fast_md_n(const uint32_t (&w)[kN / 4], int n, const FastCig& cg, int st, int en) {
  // 32-bit arithmetic: `over` marks a digit run past 2^31 - 1 (the tag is
  // then invalid), and the running position saturates at 2^31 - 1, beyond
  // any read's reference span, so the comparisons against it keep their outcome
  uint32_t num = 0, pos = 0;
  bool over = false;
  int prev = 0;  // class of the previous byte: 0 none, 1 digit, 2 letter, 3 '^'
  FastMd r{n > 0, en < 256, 0ull, 0};
  uint32_t lsh = 0;
#pragma unroll
  for (int i = 0; i < kN; ++i) {
    const uint32_t c = __builtin_amdgcn_ubfe(w[i >> 2], 8 * (i & 3), 8);
    if (i < n) {
      const uint32_t d = c - '0';
      if (d < 10u) {
        r.ok &= prev != 3;  // '^' is followed by a letter
        over |= num > 214748364u;
        num = num * 10u + d;
        over |= num > 0x7FFFFFFFu;
        prev = 1;
      } else {
        if (prev == 1) {  // a digit run ends: the matches it counts
          r.ok &= !over;
          pos = min(pos + num, 0x7FFFFFFFu);
          num = 0;
          over = false;
        }
        if (c == '^') {
          r.ok &= prev == 1;  // after a digit run, before letters
          prev = 3;
        } else {
          r.ok &= md_base((uint8_t)c) && prev != 0;
          if (pos < (uint32_t)cg.span) {
            const int32_t o = fc_offset(cg, (int32_t)pos);  // reference position start + pos
            if (o >= st && o < en) {
              r.listed &= lsh < 64;  // (more than 8: adjacent letters, e.g. "5AC5")
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
  r.ok &= prev == 1 && !over;  // ends with digits
  r.md_total = (int64_t)min(pos + num, 0x7FFFFFFFu);
  return r;
}
__device__ __forceinline__ FastMd fast_md(const uint4 md4, int n, const FastCig& cg, int st, int en) {
  const uint32_t w[4] = {md4.x, md4.y, md4.z, md4.w};
  return fast_md_n<16>(w, n, cg, st, en);
}

// The bits of a common read over [st, en): emit(lo, hi, half) for each range
// of offsets -- masked (half 0): the clips and an insertion's offsets
// (reference positions None or outside [start, end)); mismatch (half 32): the
// MD's non-matching positions and every position past the tag's span.
template <class Emit>
__device__ __forceinline__ void fast_emit(const FastCig& c, const FastMd& md, int st, int en, Emit&& emit) {
  if (c.lead > st) emit(st, min(c.lead, en), 0);
  if (!c.del && c.x > 0) {
    const int lo = max(st, c.lead + c.m1), hi = min(en, c.lead + c.m1 + c.x);
    if (lo < hi) emit(lo, hi, 0);
  }
  if (c.o_end < en) emit(max(st, c.o_end), en, 0);
  for (uint64_t l = md.lst; l; l >>= 8) {
    const int o = (int)(l & 0xFFu) - 1;
    emit(o, o + 1, 32);
  }
  if (md.md_total < c.span) {
    const int32_t t = (int32_t)md.md_total;
    if (t < c.m1) {  // reference [t, m1) -> offsets lead + t ..
      const int lo = max(st, c.lead + t), hi = min(en, c.lead + c.m1);
      if (lo < hi) emit(lo, hi, 32);
    }
    const int32_t r2 = max(t, c.m1 + (c.del ? c.x : 0));  // the part after the indel
    if (c.x > 0 && r2 < c.span) {
      const int lo = max(st, fc_offset(c, r2)), hi = min(en, c.o_end);
      if (lo < hi) emit(lo, hi, 32);
    }
  }
}

// OR a 64-bit run of masked bits into the accumulator at bit b (< 32 kAccWords)
__device__ __forceinline__ void acc_or64(uint64_t acc[kAccWords], uint64_t m, uint32_t b) {
  const uint32_t wi = b >> 5, sh = b & 31;
  const uint64_t lo64 = m << sh;
  const uint32_t w0 = (uint32_t)lo64, w1 = (uint32_t)(lo64 >> 32), w2 = sh ? (uint32_t)(m >> (64 - sh)) : 0u;
#pragma unroll
  for (int j = 0; j < kAccWords; ++j)
    acc[j] |= (uint64_t)(((uint32_t)j == wi ? w0 : 0u) | ((uint32_t)j == wi + 1 ? w1 : 0u) |
                         ((uint32_t)j == wi + 2 ? w2 : 0u));
}
// known sites of offsets [o_lo, o_hi) whose reference position is u + o,
// from the contig's position bitmap, into the accumulator at bit r0 + o
__device__ __forceinline__ void sites_seg_acc(const SitesDev& S, int32_t contig, int64_t u, int o_lo, int o_hi,
                                              uint32_t r0, uint64_t acc[kAccWords]) {
  const int64_t nw = (int64_t)(S.bm_off[contig + 1] - S.bm_off[contig]);
  const uint64_t* w = S.bm + S.bm_off[contig];
  for (int o = o_lo; o < o_hi; o += 64) {
    const int64_t b0 = u + o - S.bm_base[contig];
    const int64_t wi = b0 >> 6;
    const uint32_t sh = (uint32_t)(b0 & 63);
    const uint64_t lo = (wi >= 0 && wi < nw) ? w[wi] : 0ull, hi = (wi + 1 >= 0 && wi + 1 < nw) ? w[wi + 1] : 0ull;
    uint64_t m = sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
    if (o_hi - o < 64) m &= (1ull << (o_hi - o)) - 1ull;
    if (m) acc_or64(acc, m, r0 + (uint32_t)o);
  }
}

// The bits of a common read in registers (offset o at bit r0 + o of acc,
// r0 + en <= 32 kAccWords), known sites from the contig's position bitmap;
// *linear when the contig has none (its sorted list must be searched).
__device__ __forceinline__ void fast_bits(const SitesDev& S, int32_t contig, const FastCig& c, const FastMd& md,
                                          int st, int en, uint32_t r0, uint64_t acc[kAccWords], bool* linear) {
  fast_emit(c, md, st, en, [&](int lo, int hi, int half) { acc_range(acc, r0 + (uint32_t)lo, r0 + (uint32_t)hi, half); });
  *linear = false;
  if (contig < 0 || contig >= S.n_contigs) return;
  if (S.bm_off[contig + 1] == S.bm_off[contig]) {
    *linear = true;
  } else if (c.x == 0) {
    sites_bitmap_acc(S, contig, c.unclipped, en, r0, acc);
  } else {  // the two reference segments either side of the indel
    sites_seg_acc(S, contig, c.unclipped, 0, min(en, c.lead + c.m1), r0, acc);
    const int ob = c.lead + c.m1 + (c.del ? 0 : c.x);
    sites_seg_acc(S, contig, c.unclipped + (c.del ? c.x : -c.x), ob, en, r0, acc);
  }
}

// ReadInfo flags of an eligible read that prep finds valid
__device__ __forceinline__ uint16_t valid_flags(uint16_t f) {
  return (uint16_t)(kInfoApp | (usable_read(f) ? kInfoObs : 0) | ((f & BQSR_F_NEG_STRAND) ? kInfoNeg : 0) |
                    (((f & BQSR_F_PAIRED) && (f & BQSR_F_SECOND_OF_PAIR)) ? kInfoSecond : 0));
}
constexpr uint16_t kFastNeed = BQSR_F_HAS_QUAL | BQSR_F_HAS_RG | BQSR_F_HAS_SEQ | BQSR_F_HAS_CIGAR | BQSR_F_HAS_START |
                               BQSR_F_HAS_REFNAME;

// kLong (the listed reads, after pass 1): MD tags up to 32 bytes (md4b: bytes
// 16..31) and the read's trim resolved here, so only the mismatch letters
// inside [st, en) are listed -- a read ending in a Q2 run has every trimmed
// base in its MD as a mismatch (cfg2's listed reads: ~10 of 2048, prep_one
// 66 us of the launch)
template <bool kStore, bool kLong = false>
__device__ __forceinline__ bool prep_fast(const PrepParams& P, int64_t r, const PrepRec& x, const PrepCols& cols,
                          uint64_t acc_out[kAccWords], uint4 md4b = make_uint4(0, 0, 0, 0)) {
  const ReadMeta m = x.m;
  const ReadAlign a = x.a;
  const uint16_t f = m.flags;
  if (!eligible_read(f)) {
    P.info[r] = ReadInfo{0, 0, kInfoPass, 0};
    return true;
  }
  if ((f & kFastNeed) != kFastNeed || ((f & BQSR_F_NEG_STRAND) && (f & kSeqOther)) || m.lq == 0 || a.n_cigar == 0 ||
      a.n_cigar > kFastCigOps)
    return false;
  const bool usable = usable_read(f);
  if (usable && (a.md_len == 0 || a.md_len > (kLong ? 32 : 16))) return false;
  int st = 0, en = m.lq;  // bits over the whole read (see above)
  if (kLong) {
    trim_quals(P.rd.qual + m.slot, m.lq, st, en);  // isLowQualityBase, minQuality = 2
    if (st >= en) return false;
  }
  const uint32_t cw[kFastCigOps] = {cols.c4.x, cols.c4.y, cols.c4.z, cols.c4.w, cols.c5};
  FastCig c;
  if (!fast_cigar(cw, a.n_cigar, m, a.start, c)) return false;
  const uint64_t rs = m.slot;
  bool nobits = false;  // (kStore false) the read sets no bit: kInfoNoBits, the passes skip its words
  if (usable) {
    FastMd md;
    if (kLong) {
      const uint32_t w[8] = {cols.md4.x, cols.md4.y, cols.md4.z, cols.md4.w, md4b.x, md4b.y, md4b.z, md4b.w};
      md = fast_md_n<32>(w, a.md_len, c, st, en);
    } else {
      md = fast_md(cols.md4, a.md_len, c, st, en);
    }
    if (!md.ok) return false;  // prep_one raises MD_PARSE at the right offset
    // with known sites (several bits per read, from three sources) the bits
    // are gathered per word first; without, the few bits go straight out
    // (measured: the gathering costs more than it saves on cfg2's reads)
    if (kStore && (int64_t)(rs & 31) + en > 32 * kAccWords) return false;  // (not with <= 128 bases)
    if ((kStore || P.sites.n_contigs > 0) && (int64_t)(rs & 31) + en <= 32 * kAccWords) {
      // the read's sbits words in registers, one atomic OR per word with bits
      // (measured: plain stores of the words a read owns alone, mixed with
      // the neighbours' atomics on the same lines, were 2x slower)
      if (!md.listed) return false;  // (en <= 160: only a list overflow)
      uint64_t acc[kAccWords] = {0, 0, 0, 0, 0};
      const uint32_t r0 = (uint32_t)(rs & 31);  // bit of offset 0 in acc
      bool linear;
      fast_bits(P.sites, a.contig, c, md, st, en, r0, acc, &linear);
      if (kStore) {
        // the words go out with the wavefront's stores (prep_store_words); a
        // contig without a bitmap goes to pass 2, whose atomics land on them
        if (linear) return false;
#pragma unroll
        for (int j = 0; j < kAccWords; ++j) acc_out[j] = acc[j];
      } else {
        if (linear && c.x > 0) return false;  // (mask_sites_linear maps offsets as unclipped + o)
        nobits = !linear && !(acc[0] | acc[1] | acc[2] | acc[3] | acc[4]);
        const uint64_t wb = rs >> 5;
#pragma unroll
        for (int j = 0; j < kAccWords; ++j) {
          if (!acc[j]) continue;
          const uint64_t wi = wb + (uint64_t)j;
          atomicOr((unsigned long long*)&P.sbits[wi], (unsigned long long)acc[j]);
        }
        if (linear) mask_sites_linear(P, a.contig, c.unclipped, st, en, rs);
      }
    } else {
      if (a.contig >= 0 && a.contig < P.sites.n_contigs && c.x > 0) return false;  // (sites as unclipped + o)
      // bits: clips, an insertion, a tag shorter than the span, MD letters, sites
      nobits = c.lead <= st && (c.del || c.x == 0) && c.o_end >= en && md.listed && md.lst == 0 &&
               md.md_total >= c.span && !(a.contig >= 0 && a.contig < P.sites.n_contigs);
      if (!md.listed) {  // more than 8 non-matching positions: the tag's per-byte walk
        if (kLong || c.x > 0) return false;
        const uint32_t w[4] = {cols.md4.x, cols.md4.y, cols.md4.z, cols.md4.w};
        int64_t num = 0, pos = 0;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const uint32_t ch = (w[i >> 2] >> (8 * (i & 3))) & 0xFFu;
          if (i < a.md_len) {
            if (ch >= '0' && ch <= '9') {
              num = num * 10 + (int64_t)(ch - '0');
            } else if (ch != '^') {
              pos += num;
              num = 0;
              const int64_t o = c.lead + pos;  // reference position start + pos
              if (pos < c.m1 && o >= st && o < en) set_sbits(P.sbits, rs + (uint64_t)o, rs + (uint64_t)o + 1, 32);
              pos += 1;
            }
          }
        }
      }
      FastMd me = md;
      if (!md.listed) me.lst = 0;  // (its letters: the walk above)
      fast_emit(c, me, st, en,
                [&](int lo, int hi, int half) { set_sbits(P.sbits, rs + (uint64_t)lo, rs + (uint64_t)hi, half); });
      if (a.contig >= 0 && a.contig < P.sites.n_contigs && !mask_sites_bitmap(P, a.contig, c.unclipped, en, rs))
        mask_sites_linear(P, a.contig, c.unclipped, st, en, rs);
    }
  }
  const uint16_t nb = nobits ? kInfoNoBits : 0;
  P.info[r] = kLong ? ReadInfo{(uint16_t)st, (uint16_t)en, (uint16_t)(valid_flags(f) | nb), 0}
                    : ReadInfo{0, 0, (uint16_t)(kInfoTrim | valid_flags(f) | nb), 0};
  return true;
}

// a listed read through prep_fast's long form (own loads, no pipeline); false:
// prep_one decides
__device__ __forceinline__ bool prep_long(const PrepParams& P, int64_t r) {
  PrepRec x{};
  x.m = P.rd.meta[r];
  x.a = P.rd.align[r];
  const uint16_t f = x.m.flags;
  if (!eligible_read(f) || x.a.n_cigar == 0 || x.a.n_cigar > kFastCigOps || x.a.md_len > 32) return false;
  PrepCols c{*(const uint4*)(P.rd.cigar + x.a.cigar_off), make_uint4(0, 0, 0, 0), P.rd.cigar[x.a.cigar_off + 4]};
  uint4 md4b = make_uint4(0, 0, 0, 0);
  if (usable_read(f) && x.a.md_len > 0) {  // (the columns have 32 B of padding)
    c.md4 = *(const uint4*)(P.rd.md + x.a.md_off);
    md4b = *(const uint4*)(P.rd.md + x.a.md_off + 16);
  }
  uint64_t acc[kAccWords] = {0, 0, 0, 0, 0};
  return prep_fast<false, true>(P, r, x, c, acc, md4b);
}

// store_words: the wavefront's sbits words as plain stores (no zeroing
// pass, no read-modify-write atomics at the memory side: measured 1 ms of
// cfg3's 3 ms prep).  Lane l (read r, first slot s_l) owns the words whose
// first slot lies in [s_l, s_l+1) -- every word once, gaps included -- and
// stores its read's bits there.  A read starting inside a word owns neither
// that word nor its bits in it: those go down the wavefront to the owner by a
// segmented OR scan keyed by the word (keys are nondecreasing along the
// lanes); lane 0's go to bnd for pass 2 (the owner is in an earlier
// wavefront).  Read 0 owns its first word outright.
__device__ __forceinline__ uint64_t shfl_down_u64(uint64_t v, int d) {
  const uint32_t lo = (uint32_t)__shfl_down((int)(uint32_t)v, d), hi = (uint32_t)__shfl_down((int)(uint32_t)(v >> 32), d);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ void prep_store_words(const PrepParams& P, int64_t r, const PrepRec& x,
                                                 const uint64_t acc[kAccWords]) {
  const int lane = threadIdx.x & 63;
  const int64_t n = P.rd.n_reads;
  const uint64_t slot = r < n ? x.m.slot : (uint64_t)P.rd.n_slots;
  uint64_t nslot = shfl_down_u64(slot, 1);
  if (lane == 63) nslot = r < n ? x.nslot : (uint64_t)P.rd.n_slots;
  const uint64_t fw = slot >> 5;
  const bool mid = (slot & 31) != 0 && r != 0;  // starts inside a word it does not own
  const uint64_t own_lo = mid ? fw + 1 : fw, own_hi = (nslot + 31) >> 5;
  uint64_t S = mid ? acc[0] : 0ull;
  const uint32_t key = (uint32_t)fw;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t So = shfl_down_u64(S, d);
    const uint32_t ko = (uint32_t)__shfl_down((int)key, d);
    if (lane + d < 64 && ko == key) S |= So;
  }
  const uint64_t Sn = shfl_down_u64(S, 1);
  const uint32_t kn = (uint32_t)__shfl_down((int)key, 1);
  const uint64_t extra = (lane < 63 && own_hi > own_lo && kn == (uint32_t)(own_hi - 1)) ? Sn : 0ull;
  for (uint64_t w = own_lo; w < own_hi; ++w) {
    const uint64_t j = w - fw;
    uint64_t v = 0;
#pragma unroll
    for (int k = 0; k < kAccWords; ++k) v = j == (uint64_t)k ? acc[k] : v;
    P.sbits[w] = v | (w + 1 == own_hi ? extra : 0ull);
  }
  if (lane == 0) {
    const int64_t g = r >> 6;
    P.bnd[2 * g] = mid ? S : 0ull;
    P.bnd[2 * g + 1] = fw;
  }
}

// Pass 1: workgroup w takes reads [w * kPrepChunk, (w + 1) * kPrepChunk); the
// common ones are finished in lock step, the others listed (in read order)
// in the workgroup's own segment of the worklist -- LDS-compacted, no global
// atomics (one counter shared by every wavefront serialised at the memory
// side: measured 1.8 ms for 10M reads).
// (kStore = PrepParams::store_words, a template so each form gets its own registers)
// Without word stores (kStore false: a zeroed bitmap, bits OR-ed atomically)
// the workgroup then finishes its listed reads itself (prep_one, a thread a
// read): no second launch waiting for every workgroup of this one, and the
// listed reads' latency chains overlap other workgroups' lock-step work
// (round 5, cfg2: the listed reads -- ~10 of 2048, the reads ending in a Q2
// run, whose MD lists every trimmed base as a mismatch -- cost 66 us here
// and 74 us as bqsr_prep_complex after the pass, 251 + 74 against 317 us).
// Each listed read first tries prep_fast's long form (prep_long: MD up to 32
// bytes, the trim resolved so only the letters inside it are listed), which
// takes those reads without prep_one's per-byte walks; prep_one is forced
// inline (outlined, the call cost more than the long form saved: 308 -> 465
// us; inline 267 us, profiles/r05ae_prep_long_ab.txt).
// With word stores they wait for bqsr_prep_complex, whose atomics must land
// on words every workgroup has stored.  The atomic form asks for 5 waves per
// SIMD (round 5, with the indel fast path's registers: 329.5 -> 317.6 us
// cfg2 against 6 waves; round 4 had 6 against 5); the store form keeps its
// 104 VGPRs (at 6 waves it ran 2.08 -> 3.08 ms on cfg3).
template <bool kStore>
__global__ void __launch_bounds__(kPrepThreads, kStore ? 1 : 5) bqsr_prep_kernel(PrepParams P) {
  __shared__ uint32_t list[kPrepChunk];
  __shared__ uint32_t cnt;
  __shared__ uint32_t s_cig[kStore ? 1 : kPrepThreads * kPrepCigStride];
  __shared__ uint32_t s_md[kStore ? 1 : kPrepThreads * kPrepMdStride];
  __shared__ uint64_t s_rng[2];
  const int64_t n = P.rd.n_reads;
  const int64_t c0 = (int64_t)blockIdx.x * kPrepChunk;
  if (threadIdx.x == 0) {
    cnt = 0;
    if (!kStore) {  // the slots of this workgroup's reads: [slot of c0, slot of the next workgroup's first)
      s_rng[0] = c0 < n ? P.rd.meta[c0].slot : P.rd.n_slots;
      s_rng[1] = c0 + kPrepChunk < n ? P.rd.meta[c0 + kPrepChunk].slot : P.rd.n_slots;
    }
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  // software pipeline: the record of the read two iterations ahead and the
  // CIGAR / MD of the next one load while this one is worked
  const int64_t rt = c0 + threadIdx.x;
  PrepRec x0 = prep_rec(P, rt), x1 = prep_rec(P, rt + kPrepThreads);
  PrepCols k0 = prep_cols(P, x0);
  if (!kStore) {
    // the bitmap words of this workgroup's slots cleared before its ORs, so
    // no fill pass precedes the launch: whole words by plain stores, the two
    // shared with the neighbours' ranges by an AND of this range's bits (a
    // neighbour's own bits are never cleared, whatever the order).  (The
    // words' writes cost ~55 us on cfg2 wherever they go -- fill kernel,
    // apply kernel -- here they overlap the pass's loads.)
    const uint64_t sa = s_rng[0], sb = s_rng[1];
    const uint64_t wa = (sa + 31) >> 5, wb = sb >> 5;
    for (uint64_t w = wa + threadIdx.x; w < wb; w += kPrepThreads) P.sbits[w] = 0ull;
    if (threadIdx.x < 2 && sa < sb) {
      const uint64_t w = threadIdx.x == 0 ? sa >> 5 : (sb - 1) >> 5;  // the first / last word
      const uint64_t lo = max(sa, w << 5) - (w << 5), hi = min(sb, (w << 5) + 32) - (w << 5);
      const bool part = lo > 0 || hi < 32;  // (a whole word was stored above)
      const bool mine = threadIdx.x == 0 || (sb - 1) >> 5 != sa >> 5;  // (one word: thread 0's)
      if (part && mine) {
        const uint64_t m = (uint64_t)((hi >= 32 ? 0xFFFFFFFFu : ((1u << hi) - 1u)) & ~((1u << lo) - 1u));
        atomicAnd((unsigned long long*)&P.sbits[w], (unsigned long long)~(m | (m << 32)));
      }
    }
    __syncthreads();
  }
  for (int i = 0; i < kPrepChunk; i += kPrepThreads) {
    const int64_t r = rt + i;
    const PrepRec x2 = i + 2 * kPrepThreads < kPrepChunk ? prep_rec(P, r + 2 * kPrepThreads) : PrepRec{};
    const PrepCols k1 = i + kPrepThreads < kPrepChunk ? prep_cols(P, x1) : PrepCols{};
    uint64_t acc[kAccWords] = {0, 0, 0, 0, 0};
    const bool todo = r < n && !prep_fast<kStore>(P, r, x0, k0, acc);
    if (kStore) {
      if (todo) {
#pragma unroll
        for (int k = 0; k < kAccWords; ++k) acc[k] = 0;
      }
      prep_store_words(P, r, x0, acc);
    }
    x0 = x1;
    x1 = x2;
    k0 = k1;
    const uint64_t mask = __builtin_amdgcn_ballot_w64(todo);
    if (mask) {
      uint32_t base = 0;
      if (lane == (int)__builtin_ctzll(mask)) base = atomicAdd(&cnt, (uint32_t)__popcll(mask));
      base = __shfl(base, (int)__builtin_ctzll(mask));
      if (todo) list[base + (uint32_t)__popcll(mask & ((1ull << lane) - 1ull))] = (uint32_t)r;
    }
  }
  __syncthreads();
  const uint32_t k = cnt;
  if (!kStore) {
    for (uint32_t i = threadIdx.x; i < k; i += kPrepThreads)
      if (!prep_long(P, (int64_t)list[i]))
        prep_one(P, (int64_t)list[i], &s_cig[threadIdx.x * kPrepCigStride], &s_md[threadIdx.x * kPrepMdStride]);
    return;
  }
  for (uint32_t i = threadIdx.x; i < k; i += kPrepThreads) P.work[c0 + i] = list[i];
  if (threadIdx.x == 0) P.n_work[blockIdx.x] = k;
}

// Pass 2 (word stores only): workgroup w takes the reads pass 1's workgroup w
// listed, one thread per read, the full per-read path (prep_one).
extern "C" __global__ void __launch_bounds__(kComplexThreads) bqsr_prep_complex(PrepParams P) {
  __shared__ uint32_t s_cig[kComplexThreads * kPrepCigStride];
  __shared__ uint32_t s_md[kComplexThreads * kPrepMdStride];
  const uint32_t k = P.n_work[blockIdx.x];
  const int64_t c0 = (int64_t)blockIdx.x * kPrepChunk;
  if (P.store_words && threadIdx.x < kPrepChunk / 64) {  // pass 1's wavefront-boundary shares
    const int64_t g = (c0 >> 6) + threadIdx.x;
    if (g * 64 < P.rd.n_reads && P.bnd[2 * g])
      atomicOr((unsigned long long*)&P.sbits[P.bnd[2 * g + 1]], (unsigned long long)P.bnd[2 * g]);
  }
  for (uint32_t i = threadIdx.x; i < k; i += kComplexThreads)
    if (!prep_long(P, (int64_t)P.work[c0 + i]))
      prep_one(P, (int64_t)P.work[c0 + i], &s_cig[threadIdx.x * kPrepCigStride], &s_md[threadIdx.x * kPrepMdStride]);
}

// ------------------------------------------------------- lane-per-read ----
//
// The per-base passes give each lane one read: a wavefront takes 64
// consecutive reads and every lane walks its own read's offsets in chunks of
// 16, holding the chunk's quals (one 16-B load), its 17 base codes (one 16-B
// load, reverse-complemented in registers for reverse-strand reads) and its
// masked / mismatch bits (two 8-B loads) in registers.  Everything that is
// per read (trimming, strand, cycle direction, read group, window row test)
// is decoded once per read, so the per-base work is a few bit-field extracts
// and the table update.  Loads are unaligned 16-B accesses: the columns need
// 32 B of readable padding past their ends (bqsr_device_reads).

constexpr int kChunk = 16;

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}



// the same window for the batch's first bases, where n0 < 0 (nibble k of the
// result = code(n0 + k) for n0 + k >= 0, else 0); rare, byte by byte
__device__ __forceinline__ void load_window_head(const uint8_t* bases, int64_t n0, int64_t n_slots, uint64_t& lo,
                                              uint32_t& hi) {
  lo = 0;
  hi = 0;
  for (int k = 0; k <= 16; ++k) {
    const int64_t n = n0 + k;
    if (n < 0 || n >= n_slots) continue;
    const uint64_t c = (bases[n >> 1] >> ((n & 1) * 4)) & 0xFu;
    if (k < 16) lo |= c << (4 * k); else hi = (uint32_t)c;
  }
}

// Per-lane read decode shared by observe and apply.
struct LaneRead {
  int64_t r;      // record index (into rd.meta / info)
  int64_t ro;     // the read's index in the batch (errors, per-read outputs): r
  uint64_t slot;  // first base slot of rd's qual / base columns
  uint64_t oslot; // its slot in the batch (slot bitmap, output): slot
  int st, en;     // visited offsets [st, en)
  int fl;         // kInfo* bits
  bool trimmed;   // st / en computed here (kInfoTrim): observe writes the ReadInfo back
  ReadInfo inf;   // the resolved ReadInfo
  int rg;
  int lq, ls;
  int cell0, dir; // cycle cell of offset o = cell0 + dir * o (DiscreteCycle + L)
  int aux;        // a pass's own per-read value (set by its fread, carried to the read's chunks)
};

// A lane's read from its record and resolved ReadInfo (qs: the read's slot
// in rd's qual / base columns)
__device__ __forceinline__ LaneRead lane_decode(int64_t r, const ReadMeta& m, const ReadInfo& inf, uint64_t qs, int L) {
  LaneRead x;
  x.r = r;
  x.ro = r;
  x.aux = 0;
  x.trimmed = false;
  x.inf = inf;
  x.slot = qs;
  x.oslot = m.slot;
  x.fl = inf.fl;
  x.rg = m.rg;
  x.lq = m.lq;
  x.ls = m.ls;
  const bool pass = inf.fl & kInfoPass;
  x.st = pass ? 0 : inf.st;
  x.en = pass ? ((m.flags & BQSR_F_HAS_QUAL) ? m.lq : 0) : inf.en;
  // DiscreteCycle (StandardCovariate.scala:39-48): cyc = neg ? ls - o : o + 1,
  // negated for the second read of a pair
  const bool neg = inf.fl & kInfoNeg, sec = inf.fl & kInfoSecond;
  if (!neg) {
    x.cell0 = sec ? L - 1 : L + 1;
    x.dir = sec ? -1 : 1;
  } else {
    x.cell0 = sec ? L - (int)m.ls : L + (int)m.ls;
    x.dir = sec ? 1 : -1;
  }
  return x;
}

// ks: the read's slot in rd's qual / base columns when they are the
// key-major copy (OrderDev::kslot), ~0 for its own slot
__device__ __forceinline__ LaneRead lane_read(const ReadsDev& rd, const ReadInfo* info, int64_t r, bool live, int L,
                                              uint64_t ks = ~0ull) {
  ReadMeta m{0, 0, 0, 0, 0};
  ReadInfo inf{0, 0, 0, 0};
  if (live) {
    m = rd.meta[r];
    inf = info_load(info + r);
  }
  const bool trimmed = inf.fl & kInfoTrim;
  const uint64_t qs = ks == ~0ull ? m.slot : ks;
  inf = resolve_info(rd, inf, qs, m.lq);
  LaneRead x = lane_decode(live ? r : rd.n_reads, m, inf, qs, L);
  x.trimmed = trimmed;
  return x;
}

// ---- read order and pieces (OrderDev) ----
// first sorted position of workgroup w's range: whole tiles, as the fold's
// blocks (identity order: workgroup w's range IS fold block w)
__device__ __forceinline__ int64_t wg_begin(const ReadsDev& rd, int64_t w, int G) {
  return min(rd.n_tiles * w / G * (int64_t)rd.reads_per_tile, rd.n_reads);
}
// the workgroup whose range holds sorted position p (the largest w with wg_begin(w) <= p)
__device__ __forceinline__ int64_t wg_of(const ReadsDev& rd, int64_t p, int G) {
  const int64_t t = p / rd.reads_per_tile;
  return min((int64_t)G - 1, ((t + 1) * G - 1) / rd.n_tiles);
}
__device__ __forceinline__ int order_keys(const OrderDev& o) { return o.perm ? o.n_keys : 1; }
__device__ __forceinline__ int64_t key_begin(const OrderDev& o, int64_t n, int g) {
  return o.perm ? o.key_off[g] : (g == 0 ? 0 : n);
}
// the key holding sorted position p: the largest g with key_off[g] <= p
__device__ __forceinline__ int key_at(const OrderDev& o, int64_t p) {
  if (!o.perm) return 0;
  int lo = 0, hi = o.n_keys - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (o.key_off[mid] <= p) lo = mid; else hi = mid - 1;
  }
  return lo;
}
// the chunk-walk passes' workgroup ranges: piece w itself with fronts, else wg_begin
__device__ __forceinline__ int64_t pass_begin(const ReadsDev& rd, const OrderDev& o, int64_t w, int G) {
  return o.n_base ? o.key_off[min((int64_t)o.n_keys, w)] : wg_begin(rd, w, G);
}
__device__ __forceinline__ int64_t order_read(const OrderDev& o, int64_t i) { return o.perm ? (int64_t)o.perm[i] : i; }
// the read group of a key's window rows
__device__ __forceinline__ int key_rg(const OrderDev& o, int key, int rg_lo) {
  return o.perm ? (o.n_base ? key % o.n_base : key) >> 1 : rg_lo;
}
// the base key (read group, mate class) of a key: what the apply char tables are per
__device__ __forceinline__ int base_key(const OrderDev& o, int key) { return o.n_base ? key % o.n_base : key; }
__device__ __forceinline__ int order_base_keys(const OrderDev& o) { return o.perm ? (o.n_base ? o.n_base : o.n_keys) : 1; }
// the cycle cells a piece's windows hold: all of them in read order, the
// key's mate-class half when bucketed (OrderDev)
struct WinGeom {
  int c_lo, cw;
};
__device__ __forceinline__ WinGeom win_geom(const OrderDev& o, const TableGeom& g, int key) {
  if (!o.perm) return WinGeom{0, g.C};
  return (key & 1) ? WinGeom{0, g.L} : WinGeom{g.L + 1, g.L};  // (n_base is even: key & 1 is the mate class)
}


// The 17-code window of chunk o0 of a read (forward: codes o0-1 .. o0+15;
// reverse: the mirrored codes, o0's mirror + 1 down to o0+15's -- quirk Q9).
// Split so a super-chunk's loads all issue before any is used: chunk_n0 /
// chunk_raw issue the 16-B load, chunk_ctx turns it into context slots.
__device__ __forceinline__ int64_t chunk_n0(const LaneRead& x, int o0) {
  const bool neg = x.fl & kInfoNeg;
  return (int64_t)x.slot + (neg ? (int64_t)(x.en + x.st - o0 - 16) : (int64_t)(o0 - 1));
}
__device__ __forceinline__ uint4 chunk_raw(const ReadsDev& rd, int64_t n0) {
  return n0 >= 0 ? *(const uint4*)(rd.bases + (n0 >> 1)) : make_uint4(0, 0, 0, 0);
}
// Offsets per super-chunk: the loads of kSub chunks of one read are issued
// together, so the few cache lines a read spans are fetched once while hot
// instead of once per chunk.
constexpr int kSub = 4;
constexpr int kSuper = kSub * kChunk;

// 16 masked / mismatch bits of sub-chunk i from a step's NW bitmap words
// (w[0] holds the slot of the step's first offset at bit b0)
template <int NW>
__device__ __forceinline__ void sub_bits(const uint64_t* w, uint32_t b0, int i, uint32_t& masked, uint32_t& mism) {
  const uint32_t b = b0 + 16u * (uint32_t)i;
  const uint32_t wi = b >> 5, sh = b & 31;
  uint64_t lo = w[0], hi = w[1];
#pragma unroll
  for (int k = 1; k < NW; ++k) {  // a chunk starting in the last word ends in it
    lo = wi == (uint32_t)k ? w[k] : lo;
    hi = wi == (uint32_t)k ? w[k + 1 < NW ? k + 1 : k] : hi;
  }
  masked = __builtin_amdgcn_alignbit((uint32_t)hi, (uint32_t)lo, sh);
  mism = __builtin_amdgcn_alignbit((uint32_t)(hi >> 32), (uint32_t)(lo >> 32), sh);
}

// The same bits when the step's first slot sits at bit 16 h of w[0] (h = 0
// or 1: 16-aligned slots, ReadsDev::slots_aligned): chunk i's bits are one
// half of word (h + i) >> 1 -- a select for odd i instead of a scan.
template <int NW>
__device__ __forceinline__ void sub_bits16(const uint64_t* w, uint32_t h, int i, uint32_t& masked, uint32_t& mism) {
  const int a = i >> 1, b = (i + 1) >> 1 < NW ? (i + 1) >> 1 : NW - 1;
  const uint64_t v = (i & 1) ? (h ? w[b] : w[a]) : w[a];
  const uint32_t sh = 16u * ((h + (uint32_t)i) & 1u);
  masked = (uint32_t)v >> sh;
  mism = (uint32_t)(v >> 32) >> sh;
}

// the read's first visited offset k has context 0 (slot 4): its predecessor
// in the 17-code window (nibble k, after any reverse complement) read as N
__device__ __forceinline__ uint64_t window_first(uint64_t lo, int k) {
  const uint32_t sh = 4u * (uint32_t)k;
  return (lo & ~(0xFull << sh)) | ((uint64_t)kCodeN << sh);
}

// ---- context table (LDS, kCtxTabBytes) ----
// The context slots of two neighbouring offsets from three codes of the raw
// (forward) window: entry c0 | c1 << 4 | c2 << 8 of the forward half holds
// slot(c0, c1) | slot(c1, c2) << 8, so a chunk's 16 slots are 8 u16 reads
// instead of spreading the codes to bytes and two lookups per offset.  The
// reverse half holds what the reverse-complemented window gives (quirk Q9,
// BaseContext.simpleReverseComplement): lookup m of the raw window yields the
// slots of offsets 15 - m and 14 - m, so the 16 bytes come out mirrored and
// one byte permute per dword restores them -- no reverse complement of the
// window.  Slot (ctx + 4) of the pair (a, b) = (previous, current) code:
// 4 (context 0) when either is N, else 4 (idx(a) + 1) + (idx(b) + 1) with
// idx 0..3 for ACGT and -1 for any other byte (BaseContext.scala).
__device__ __forceinline__ uint32_t ctx_slot(uint32_t a, uint32_t b) {
  if (a == kCodeN || b == kCodeN) return 4u;
  return 4u * (a < 4u ? a + 1u : 0u) + (b < 4u ? b + 1u : 0u);
}
__device__ __forceinline__ uint32_t comp_code(uint32_t c) { return c < 4u ? c ^ 3u : c; }
__device__ __forceinline__ void ctx_table_fill(uint16_t* t, int tid, int nthreads) {
  for (int i = tid; i < (int)(2 * kCtxTab); i += nthreads) {
    const uint32_t e = (uint32_t)i & (kCtxTab - 1u);
    const uint32_t c0 = e & 15u, c1 = (e >> 4) & 15u, c2 = e >> 8;
    t[i] = (uint16_t)((uint32_t)i < kCtxTab ? ctx_slot(c0, c1) | ctx_slot(c1, c2) << 8
                                  : ctx_slot(comp_code(c1), comp_code(c0)) |
                                        ctx_slot(comp_code(c2), comp_code(c1)) << 8);
  }
}
typedef unsigned short u16x2v __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) const uint16_t* LdsHalves;
// tb + 2 x in one instruction (the compiler's form of the same sum was a
// shift, a mask and an add: 8 VALU a chunk more)
__device__ __forceinline__ uint32_t lshl1_add(uint32_t x, uint32_t tb) {
  uint32_t r;
  asm("v_lshl_add_u32 %0, %1, 1, %2" : "=v"(r) : "v"(x), "v"(tb));
  return r;
}
// raw window (lo: codes 0..15, hi: code 16) of a chunk -> its 16 slots;
// tb = LDS address of the table half (forward, or reverse for neg reads)
__device__ __forceinline__ void ctx_lookup(uint64_t lo, uint32_t hi, uint32_t tb, bool neg, uint32_t xo[4]) {
  const uint32_t d0 = (uint32_t)lo, d1 = (uint32_t)(lo >> 32);
  const uint32_t ix[8] = {__builtin_amdgcn_ubfe(d0, 0, 12),  __builtin_amdgcn_ubfe(d0, 8, 12),
                          __builtin_amdgcn_ubfe(d0, 16, 12), __builtin_amdgcn_alignbit(d1, d0, 24) & 0xFFFu,
                          __builtin_amdgcn_ubfe(d1, 0, 12),  __builtin_amdgcn_ubfe(d1, 8, 12),
                          __builtin_amdgcn_ubfe(d1, 16, 12), __builtin_amdgcn_alignbit(hi, d1, 24) & 0xFFFu};
  uint32_t X[4];
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    u16x2v v;
    v.x = *(LdsHalves)(uintptr_t)lshl1_add(ix[2 * w], tb);
    v.y = *(LdsHalves)(uintptr_t)lshl1_add(ix[2 * w + 1], tb);
    X[w] = __builtin_bit_cast(uint32_t, v);
  }
  const uint32_t sel = neg ? 0x04050607u : 0x03020100u;  // bytes of X[3 - w] reversed, or X[w]
#pragma unroll
  for (int w = 0; w < 4; ++w) xo[w] = __builtin_amdgcn_perm(X[3 - w], X[w], sel);
}
// Context slots by byte tables (bqsr_observe_lean, the arithmetic apply
// form): byte m of h = U1[code m] + U2[code m + 1] of a window (lo: codes
// 0..15, hi: code 16); U = v_perm tables {lo: codes 0..3, hi: codes 4..7}
__device__ __forceinline__ void lean_ctx(uint64_t lo, uint32_t hi, uint32_t u1lo, uint32_t u1hi, uint32_t u2lo,
                                         uint32_t u2hi, uint32_t h[4]) {
  uint32_t s[5];
#pragma unroll
  for (int d = 0; d < 2; ++d) {
    const uint32_t x = (uint32_t)(lo >> (32 * d));
    const uint32_t e = x & 0x07070707u, o = (x >> 4) & 0x07070707u;
    s[2 * d] = __builtin_amdgcn_perm(o, e, 0x05010400u);
    s[2 * d + 1] = __builtin_amdgcn_perm(o, e, 0x07030602u);
  }
  s[4] = hi & 7u;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const uint32_t b = __builtin_amdgcn_alignbit(s[w + 1], s[w], 8);
    h[w] = __builtin_amdgcn_perm(u1hi, u1lo, s[w]) + __builtin_amdgcn_perm(u2hi, u2lo, b);
  }
}

// T[code] for codes 0..7 (A C G T N other), unscaled: slot = T1[a] + T2[b]
constexpr uint32_t kA1lo = 0x100C0804u, kA1hi = 0x00000015u;  // 4 (idx + 1); N 21
constexpr uint32_t kA2lo = 0x04030201u, kA2hi = 0x00000015u;  // idx + 1
constexpr uint32_t kA1clo = 0x04080C10u, kA2clo = 0x01020304u;  // complemented

// a chunk's 16 context slots from its raw 16-B bases load: the 17-code window
// (forward), the read's first offset given context 0, the table lookups
__device__ __forceinline__ void chunk_ctx(const ReadsDev& rd, bool neg, int64_t n0, uint4 v, int j, uint32_t tb,
                                          uint32_t xo[4]) {
  uint64_t lo;
  uint32_t hi;
  if (__builtin_expect(n0 >= 0, 1)) {
    const uint32_t sh = (uint32_t)(n0 & 1) * 4u;
    lo = ((uint64_t)__builtin_amdgcn_alignbit(v.z, v.y, sh) << 32) | __builtin_amdgcn_alignbit(v.y, v.x, sh);
    hi = __builtin_amdgcn_alignbit(v.w, v.z, sh) & 0xFu;
  } else {
    load_window_head(rd.bases, n0, rd.n_slots, lo, hi);
  }
  if (j <= 0) {  // the first visited offset -j: its predecessor (raw nibble -j, or 16 + j mirrored) read as N
    const int t = neg ? 16 + j : -j;
    if (t < 16) lo = window_first(lo, t); else hi = kCodeN;
  }
  // (the byte-table form of bqsr_observe_lean here, junk slots fixed to 4 in
  // SWAR: cfg2 apply 793 -> 825 us, cfg4 5948 -> 6011 us; not taken)
  ctx_lookup(lo, hi, neg ? tb + 2u * kCtxTab : tb, neg, xo);
}

// the low 16 bits of x mirrored (bit p <- bit 15 - p) when rev
__device__ __forceinline__ uint32_t mirror_bits16(uint32_t x, bool rev) {
  return rev ? (__builtin_bitreverse32(x & 0xFFFFu) >> 16) : (x & 0xFFFFu);
}
// 16 bytes of x mirrored (byte k <- byte 15 - k) when sel = 0x04050607 (0x03020100: as is)
__device__ __forceinline__ void mirror16(uint32_t x[4], uint32_t sel) {
  const uint32_t y0 = __builtin_amdgcn_perm(x[3], x[0], sel), y1 = __builtin_amdgcn_perm(x[2], x[1], sel);
  const uint32_t y2 = __builtin_amdgcn_perm(x[1], x[2], sel), y3 = __builtin_amdgcn_perm(x[0], x[3], sel);
  x[0] = y0;
  x[1] = y1;
  x[2] = y2;
  x[3] = y3;
}

// ------------------------------------------------------- lane per chunk ----
//
// The per-base passes' wavefront walk: every lane takes one 16-offset chunk
// per step, the chunks of consecutive reads laid end to end over the 64
// lanes, so a step's loads and stores are consecutive 16-B pieces of the
// columns (read order, 16-aligned slots: one contiguous kilobyte) and no lane
// idles while another finishes a longer read.
//
// Windows of 64 sorted positions: lane j first decodes the window's read j
// (`read lane`: lane_read, the per-read callback), and a scan of the reads'
// chunk counts gives read j its first chunk ps_j.  The window's chunks are
// then taken 64 at a time: lane l takes chunk g0 + l, whose read is the last
// read with a chunk and ps <= g0 + l -- a per-wavefront LDS word per lane
// takes the largest such read starting at each lane (LDS max), a DPP max-scan
// carries it to the lanes after it -- and fetches that read's packed fields
// from its read lane with ds_bpermute.

template <int kCtrl, int kRowMask = 0xF>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, kCtrl, kRowMask, 0xF, false);  // 0 where no source lane
}
__device__ __forceinline__ uint32_t wave_incl_add(uint32_t x) {
  x += dpp_u32<0x111>(x);
  x += dpp_u32<0x112>(x);
  x += dpp_u32<0x114>(x);
  x += dpp_u32<0x118>(x);
  x += dpp_u32<0x142, 0xA>(x);
  x += dpp_u32<0x143, 0xC>(x);
  return x;
}
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t x) {
  x = max(x, dpp_u32<0x111>(x));
  x = max(x, dpp_u32<0x112>(x));
  x = max(x, dpp_u32<0x114>(x));
  x = max(x, dpp_u32<0x118>(x));
  x = max(x, dpp_u32<0x142, 0xA>(x));
  x = max(x, dpp_u32<0x143, 0xC>(x));
  return x;
}
__device__ __forceinline__ uint32_t bperm(int src_lane, uint32_t v) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute(src_lane << 2, (int)v);
}

constexpr uint32_t kPkRev = 0x8000u;  // packed flags: cycle direction -1

// kAct: the kInfo bits of reads whose [st, en) the pass visits.  Chunk k of a
// read covers offsets st + jb + 16k .. +15 (jb = -(st & 15) in the aligned
// layout, else 0).  fread(x, live) runs once per read (on its read lane).  A
// step takes kU groups of 64 chunks: every group's chunk is mapped and its
// loads issued (fload(x, j, on) -> LD) before the first is used
// (fchunk(x, j, n, on, ld)), so a lane has kU chunks' loads in flight; x
// holds r, slot, st, en, fl, rg, cell0 and dir of the chunk's read, j = jb +
// 16k, n = en - st.
template <uint32_t kAct, int kU, class LD, bool kAux, class FRead, class FLoad, class FChunk>
__device__ __forceinline__ void chunk_walk(const ReadsDev& rd, const ReadInfo* info, const OrderDev& ord, int64_t q0,
                                           int64_t q1, int64_t qstep, int L, int lane, uint32_t* mk, FRead&& fread,
                                           FLoad&& fload, FChunk&& fchunk) {
  for (int64_t wb = q0; wb < q1; wb += qstep) {
    const bool live = wb + lane < q1;
    LaneRead x = lane_read(rd, info, live ? order_read(ord, wb + lane) : 0, live, L,
                           live && ord.kslot ? ord.kslot[wb + lane] : ~0ull);
    fread(x, live);
    const int n = (live && (x.fl & kAct)) ? x.en - x.st : 0;
    const int jb = rd.slots_aligned ? -(x.st & 15) : 0;
    const uint32_t nch = n > 0 ? (uint32_t)((n - jb + 15) >> 4) : 0u;
    const uint32_t pe = wave_incl_add(nch), ps = pe - nch;
    const uint32_t total = __builtin_amdgcn_readlane(pe, 63);
    const uint32_t p_r = (uint32_t)x.r, p_slo = (uint32_t)x.slot, p_shi = (uint32_t)(x.slot >> 32);
    const uint32_t p_olo = (uint32_t)x.oslot, p_ohi = (uint32_t)(x.oslot >> 32);
    const uint32_t p_se = (uint32_t)x.st | ((uint32_t)x.en << 16);
    const uint32_t p_fl = (uint32_t)x.fl | (x.dir < 0 ? kPkRev : 0u) | ((uint32_t)x.cell0 << 16);
    const uint32_t p_rg = (uint32_t)x.rg, p_aux = (uint32_t)x.aux;
    for (uint32_t g00 = 0; g00 < total; g00 += 64 * kU) {
      LaneRead c[kU];
      int jj[kU];
      bool on[kU];
      LD ld[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const uint32_t g0 = g00 + 64 * u;
        mk[lane] = 0;
        __builtin_amdgcn_wave_barrier();
        if (nch && ps > g0 && ps < g0 + 64) atomicMax(&mk[ps - g0], (uint32_t)lane);
        __builtin_amdgcn_wave_barrier();
        // chunk g0's read: the last read with chunks whose first is <= g0
        const uint64_t below = __builtin_amdgcn_ballot_w64(nch && ps <= g0);
        uint32_t v = mk[lane];
        __builtin_amdgcn_wave_barrier();
        if (lane == 0) v = 63u - (uint32_t)__builtin_clzll(below);
        const int ri = (int)wave_incl_max(v);
        c[u].r = bperm(ri, p_r);
        c[u].slot = ((uint64_t)bperm(ri, p_shi) << 32) | bperm(ri, p_slo);
        c[u].ro = c[u].r;
        c[u].oslot = ord.kslot ? ((uint64_t)bperm(ri, p_ohi) << 32) | bperm(ri, p_olo) : c[u].slot;
        const uint32_t se = bperm(ri, p_se), fl = bperm(ri, p_fl);
        c[u].st = (int)(se & 0xFFFFu);
        c[u].en = (int)(se >> 16);
        c[u].fl = (int)(fl & 0x7FFFu);
        c[u].dir = (fl & kPkRev) ? -1 : 1;
        c[u].cell0 = (int)(fl >> 16);
        c[u].rg = (int)bperm(ri, p_rg);
        c[u].aux = kAux ? (int)bperm(ri, p_aux) : 0;
        const uint32_t ps_c = bperm(ri, ps);
        const int jb_c = rd.slots_aligned ? -(c[u].st & 15) : 0;
        jj[u] = jb_c + 16 * (int)(g0 + lane - ps_c);
        on[u] = g0 + lane < total;
        ld[u] = fload(c[u], jj[u], on[u]);
      }
#pragma unroll
      for (int u = 0; u < kU; ++u) fchunk(c[u], jj[u], c[u].en - c[u].st, on[u], ld[u]);
    }
  }
}

// ------------------------------------------------------------ observe ------

typedef __attribute__((address_space(3))) uint32_t* LdsWords;
typedef __attribute__((address_space(3))) const uint8_t* LdsBytes;
__device__ __forceinline__ void lds_add(uint32_t addr, uint32_t v) {
  __hip_atomic_fetch_add((LdsWords)(uintptr_t)addr, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}


// Lane per chunk (chunk_walk): the same counts, each lane one 16-offset
// chunk of the wavefront's reads laid end to end.  LDS: the window as in
// bqsr_observe_lean's slab layout, then the walk's kMkWords markers.
struct ObsChunkLoads {
  uint4 qs, cr;
  uint64_t bw0, bw1;  // sbits words of the chunk's first slot and the next
};

__device__ __forceinline__ ObsChunkLoads observe_load(const ObserveParams& P, const LaneRead& x, int j, bool on) {
  ObsChunkLoads v{make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0), 0, 0};
  if (!on) return v;
  const int o0 = x.st + j;
  v.qs = *(const uint4*)(P.rd.qual + x.slot + o0);
  if (x.fl & kInfoObs) {
    v.cr = chunk_raw(P.rd, chunk_n0(x, o0));
    const uint64_t s0 = x.oslot + (uint64_t)o0;
    if (!(x.fl & kInfoNoBits)) {  // (a read without bits: nothing to load)
      v.bw0 = P.sbits[s0 >> 5];
      if ((s0 & 31) > 16) v.bw1 = P.sbits[(s0 >> 5) + 1];  // an unaligned layout's chunk across two words
    }
  }
  return v;
}

struct ObsPiece {
  uint32_t *w_obs, *w_mm, *w_masked, *blk_hist;
  int rg_w, c_lo, cw, q_lo, qw, wcells;
  bool ident;
  uint32_t tb;  // LDS address of the context table
};

__device__ __forceinline__ void observe_chunk(const ObserveParams& P, const ObsPiece& pc, const LaneRead& x, int j,
                                              int n, bool on, const ObsChunkLoads& ld) {
  if (!on) return;
  const bool full = x.fl & kInfoObs;
  const int o0 = x.st + j;
  const int C = P.g.C, cells = P.g.cells;
  const uint32_t qd[4] = {ld.qs.x, ld.qs.y, ld.qs.z, ld.qs.w};
  uint32_t bm = 0, bx = 0;
  uint32_t xo[4] = {4u, 4u, 4u, 4u};
  if (full) {
    const uint32_t sb = (uint32_t)((x.oslot + (uint64_t)o0) & 31);
    bm = __builtin_amdgcn_alignbit((uint32_t)ld.bw1, (uint32_t)ld.bw0, sb);
    bx = __builtin_amdgcn_alignbit((uint32_t)(ld.bw1 >> 32), (uint32_t)(ld.bw0 >> 32), sb);
    chunk_ctx(P.rd, x.fl & kInfoNeg, chunk_n0(x, o0), ld.cr, j, pc.tb, xo);
  }
  const int cc0 = x.cell0 + __mul24(x.dir, o0);  // table cycle cell of offset k: cc0 + dir * k
  const int wc0 = cc0 - pc.c_lo;                 // ... and window cycle cell
  const uint32_t nv = (uint32_t)min(kChunk, n - j);
  const int klo = j < 0 ? -j : 0;
  const bool cok = full && x.rg == pc.rg_w && (unsigned)(wc0 + __mul24(klo, x.dir)) < (unsigned)pc.cw &&
                   (unsigned)(wc0 + __mul24((int)nv - 1, x.dir)) < (unsigned)pc.cw;
  const uint32_t vmask = (nv >= 16u ? 0xFFFFu : ((1u << nv) - 1u)) & (0xFFFFu << klo);
  uint32_t fastm = 0;
  if (cok) {
#pragma unroll
    for (int k = 0; k < kChunk; ++k) {
      const int q = (int)__builtin_amdgcn_ubfe(qd[k >> 2], 8 * (k & 3), 8);
      const int row = q - pc.q_lo;
      const bool f = (unsigned)row < (unsigned)pc.qw && ((vmask >> k) & 1u);
      const bool m = (bm >> k) & 1u;
      const int base = __mul24(row, pc.wcells);
      if (f) {
        atomicAdd(m ? &pc.w_masked[row] : &pc.w_obs[base + wc0 + x.dir * k], 1u);
        if (!m) atomicAdd(&pc.w_obs[base + pc.cw + (int)__builtin_amdgcn_ubfe(xo[k >> 2], 8 * (k & 3), 8)], 1u);
      }
      fastm |= (uint32_t)f << k;
    }
  }
  uint32_t slow = vmask & ~fastm;
  uint32_t mmk = fastm & ~bm & bx;
  if (__builtin_amdgcn_ballot_w64(mmk != 0)) {  // mismatches (about 1 base in 100)
    const uint64_t x01 = ((uint64_t)xo[1] << 32) | xo[0], x23 = ((uint64_t)xo[3] << 32) | xo[2];
    while (mmk) {
      const int k = __builtin_ctz(mmk);
      mmk &= mmk - 1;
      const int q = (int)__builtin_amdgcn_ubfe(qd[k >> 2], 8 * (k & 3), 8);
      const int base = __mul24(q - pc.q_lo, pc.wcells);
      atomicAdd(&pc.w_mm[base + wc0 + __mul24(x.dir, k)], 1u);
      atomicAdd(&pc.w_mm[base + pc.cw + (int)(((k < 8 ? x01 : x23) >> (8 * (k & 7))) & 0xFFu)], 1u);
    }
  }
  if (__builtin_amdgcn_ballot_w64(slow != 0)) {
    const uint64_t x01 = ((uint64_t)xo[1] << 32) | xo[0], x23 = ((uint64_t)xo[3] << 32) | xo[2];
    while (slow) {
      const int k = __builtin_ctz(slow);
      slow &= slow - 1;
      const int o = o0 + k;
      const int q = (int)(int8_t)__builtin_amdgcn_ubfe(qd[k >> 2], 8 * (k & 3), 8);
      if (q < 0) {  // RecalTable.+= : phredToErrorProbabilityCache(qual)
        report(P.err, err_key((uint64_t)x.ro, (uint32_t)o, kRankTable, BQSR_ERR_QUAL_RANGE));
      } else if (full) {  // outside the LDS window: straight to the int64 table
        const bool masked = (bm >> k) & 1u, mism = (bx >> k) & 1u;
        const int ccell = cc0 + __mul24(x.dir, k);
        const int xcell = C + (int)(((k < 8 ? x01 : x23) >> (8 * (k & 7))) & 0xFFu);
        if (pc.ident) atomicAdd(&pc.blk_hist[q], 1u);
        const int64_t key = (int64_t)q + (int64_t)kMaxQ * x.rg;
        atomicAdd((unsigned long long*)&P.touched[key], 1ull);
        if (!masked) {
          atomicAdd((unsigned long long*)&P.obs[key * cells + ccell], 1ull);
          atomicAdd((unsigned long long*)&P.obs[key * cells + xcell], 1ull);
          if (mism) {
            atomicAdd((unsigned long long*)&P.mm[key * cells + ccell], 1ull);
            atomicAdd((unsigned long long*)&P.mm[key * cells + xcell], 1ull);
          }
        }
      }
    }
  }
}

constexpr int kObserveU = 2;  // chunks in flight per lane

extern "C" __global__ void __launch_bounds__(kBlockThreads) bqsr_observe_chunks(ObserveParams P) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int qw = P.w.qw, L = P.g.L;
  const int wcells = P.wcells;
  uint16_t* ctab = (uint16_t*)smem;
  uint32_t* w_obs = (uint32_t*)(smem + kCtxTabBytes);
  uint32_t* w_mm = w_obs + qw * wcells;
  uint32_t* w_masked = w_mm + qw * wcells;
  uint32_t* blk_hist = w_masked + qw;
  uint32_t* mk_all = blk_hist + kQBins;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  uint32_t* mk = mk_all + wave * 64;
  const int G = P.n_blocks;
  const bool ident = P.ord.perm == nullptr;
  for (int i = tid; i < kQBins; i += blockDim.x) blk_hist[i] = 0;
  ctx_table_fill(ctab, tid, blockDim.x);  // ready at the piece loop's first barrier
  const int64_t wa = pass_begin(P.rd, P.ord, blockIdx.x, G), wb = pass_begin(P.rd, P.ord, blockIdx.x + 1, G);
  const int nk = order_keys(P.ord);
  for (int key = wa < wb ? key_at(P.ord, wa) : nk; key < nk; ++key) {
    const int64_t p0 = max(wa, key_begin(P.ord, P.rd.n_reads, key));
    const int64_t p1 = min(wb, key_begin(P.ord, P.rd.n_reads, key + 1));
    if (p0 >= wb) break;
    if (p0 >= p1) continue;
    const WinGeom gm = win_geom(P.ord, P.g, key);
    const ObsPiece pc{w_obs, w_mm, w_masked, blk_hist, key_rg(P.ord, key, P.w.rg_lo), gm.c_lo, gm.cw, P.w.q_lo, qw,
                      wcells, ident, (uint32_t)(uintptr_t)(LdsHalves)ctab};
    for (int i = tid; i < 2 * qw * wcells + qw; i += blockDim.x) w_obs[i] = 0;
    __syncthreads();
    const auto fread = [&](LaneRead& x, bool live) {
      if (live && x.trimmed) info_store(P.info + x.r, x.inf);  // fold and apply read the trimmed range
    };
    const auto fload = [&](const LaneRead& x, int j, bool on) { return observe_load(P, x, j, on); };
    const auto fchunk = [&](const LaneRead& x, int j, int n, bool on, const ObsChunkLoads& ld) {
      observe_chunk(P, pc, x, j, n, on, ld);
    };
    chunk_walk<kInfoObs | kInfoObsCheck, kObserveU, ObsChunkLoads, false>(P.rd, P.info, P.ord, p0 + 64 * wave, p1,
                                                                          64 * kWaves, L, lane, mk, fread, fload, fchunk);
    __syncthreads();
    // ---- the piece's window -> its slab; window rows into the block histogram ----
    uint32_t* pb = P.part + (int64_t)(blockIdx.x + (ident ? 0 : key)) * P.part_stride;
    for (int i = tid; i < 2 * qw * wcells; i += blockDim.x) pb[i] = w_obs[i];
    for (int slot = wave; slot < qw; slot += kWaves) {
      uint32_t v = 0;
      for (int c = lane; c < gm.cw; c += 64) v += w_obs[slot * wcells + c];  // every unmasked base hits one cycle cell
      v = wave_sum(v);
      if (lane == 0) {
        const uint32_t tot = v + w_masked[slot];
        pb[2 * qw * wcells + slot] = tot;
        if (ident && tot && P.w.q_lo + slot < kQBins) atomicAdd(&blk_hist[P.w.q_lo + slot], tot);
      }
    }
    __syncthreads();
  }
  if (ident)
    for (int k = tid; k < kQBins; k += blockDim.x) P.hq_block[(int64_t)blockIdx.x * kQBins + k] = blk_hist[k];
}

// Sum the pieces' window counts into the int64 table: one thread per (key,
// window cell, slab group), over the slabs (w + key) of the workgroups whose
// range meets the key's positions (the observe kernel's direct atomics have
// all landed).
extern "C" __global__ void bqsr_window_reduce(const uint32_t* part, ReadsDev rd, OrderDev ord, int32_t n_blocks,
                                              int32_t stride, int32_t wcells, Window w, TableGeom g, int64_t* touched,
                                              int64_t* obs, int64_t* mm, int32_t junk) {
  // fronts: a thread per (base key, word) sums the base key's pieces (slab
  // 2 key of workgroup key), one atomic per table word as without fronts
  const int nk = order_base_keys(ord);
  const int nc = w.qw * wcells;
  const int64_t total = (int64_t)nk * stride;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int key = (int)(t / stride);
    const int i = (int)(t - (int64_t)key * stride);
    uint64_t s = 0;
    if (ord.n_base) {
#pragma unroll 4
      for (int kf = key; kf < ord.n_keys; kf += ord.n_base) {
        const uint32_t v = part[2 * (int64_t)kf * stride + i];
        if (ord.key_off[kf] < ord.key_off[kf + 1]) s += v;
      }
    } else {
      const int64_t k0 = key_begin(ord, rd.n_reads, key), k1 = key_begin(ord, rd.n_reads, key + 1);
      if (k0 >= k1) continue;
      // grid y: thread y takes the groups y, y + gridDim.y, ... of kRedSlabs
      // slabs of the key's range
      const int64_t wk1 = wg_of(rd, k1 - 1, n_blocks);
      for (int64_t w0 = wg_of(rd, k0, n_blocks) + (int64_t)blockIdx.y * kRedSlabs; w0 <= wk1;
           w0 += (int64_t)gridDim.y * kRedSlabs) {
        const int64_t w1 = min(wk1, w0 + kRedSlabs - 1);
#pragma unroll 8
        for (int64_t b = w0; b <= w1; ++b) {
          // a workgroup with an empty range in between wrote no slab (its words
          // are read but not added: the loads stay independent)
          uint32_t v = part[(b + (ord.perm ? key : 0)) * stride + i];
          if (max(k0, wg_begin(rd, b, n_blocks)) < min(k1, wg_begin(rd, b + 1, n_blocks))) s += v;
        }
      }
    }
    if (!s) continue;
    const int rg = key_rg(ord, key, w.rg_lo);
    const WinGeom gm = win_geom(ord, g, key);
    const int64_t key0 = (int64_t)w.q_lo + (int64_t)kMaxQ * rg;
    if (i < 2 * nc) {
      const int j = i < nc ? i : i - nc;
      const int slot = j / wcells, wc = j - slot * wcells;
      // context cells past the 21 slots: bqsr_observe_lean's `junk` cells of
      // windows with an N, context 0 (slot 4); then the row's pad words
      const int xw = wc - gm.cw;
      const int cell = wc < gm.cw ? gm.c_lo + wc : g.C + (xw < kCtxSlots ? xw : 4);
      if (key0 + slot >= g.K || xw >= kCtxSlots + junk) continue;
      // atomics: two read groups' rows can alias one key (q >= 60, quirk Q3)
      int64_t* dst = i < nc ? obs : mm;
      atomicAdd((unsigned long long*)&dst[(key0 + slot) * g.cells + cell], (unsigned long long)s);
    } else {
      const int slot = i - 2 * nc;
      if (key0 + slot >= g.K) continue;
      atomicAdd((unsigned long long*)&touched[key0 + slot], (unsigned long long)s);
    }
  }
}

// ------------------------------------------------------ read-group buckets --
//
// Bucketed batches (several read groups) walk their reads grouped by read
// group so that a workgroup's LDS window always holds the rows of the group it
// is counting (OrderDev).  A counting sort on the device: per-key counts, an
// exclusive scan, then a scatter in which each workgroup reserves one range
// per key it holds (one global atomic per workgroup and key) and ranks its
// reads inside it with LDS atomics.  The order inside a key is immaterial:
// counts commute, apply writes by read, errors are reduced by read index.

constexpr int kSortThreads = 256;
constexpr int kSortPer = 16;             // reads per thread in the scatter
constexpr int kSortLdsKeys = 4096;       // keys kept in LDS; more go straight to global atomics

// key = front * n_base + 2 * read group + mate class (OrderDev); n_base = 2 *
// n_rg, front = read r's share of [0, n) when there are `fronts` of them
__device__ __forceinline__ int sort_key(const ReadMeta& m, int64_t r, int64_t n, int n_base, int fronts) {
  const int cls = ((m.flags & BQSR_F_PAIRED) && (m.flags & BQSR_F_SECOND_OF_PAIR)) ? 1 : 0;
  const int f = fronts > 1 ? (int)((r * fronts) / n) : 0;
  return f * n_base + 2 * min((int)m.rg, n_base / 2 - 1) + cls;
}

// ---- key-major copy (OrderDev::kslot; bqsr_capi.cpp layout_build) ----
// kKmLanes lanes per sorted position: the read's 16-slot pieces (16-B qual,
// 8-B code) to its key-major slots, a piece per lane (pieces beyond kKmLanes
// looped), kKmPer positions per lane group at once with every load of the
// group issued before the first store.  cfg4 (6.2 GB of quals and codes):
// a wavefront per read (10-16 of its 64 lanes busy) 8.4 ms a build, a
// position per lane group 4.1 ms, four 4.4 ms.  Off by default (BQSR_TUNE_KEYMAJOR):
// it saves 0.27 ms a cfg4 job, so it pays only after ~17 jobs on one batch.
constexpr int kKmLanes = 16;
constexpr int kKmPer = 1;
extern "C" __global__ void __launch_bounds__(256) bqsr_km_gather(ReadsDev rd, const uint32_t* perm, const uint64_t* kslot,
                                                                uint8_t* kqual, uint8_t* kbases) {
  const int sub = threadIdx.x & (kKmLanes - 1);
  const int64_t g0 = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / kKmLanes;
  const int64_t ng = ((int64_t)gridDim.x * blockDim.x) / kKmLanes;
  const int64_t n = rd.n_reads;
  for (int64_t p0 = g0 * kKmPer; p0 < n; p0 += ng * kKmPer) {
    uint64_t src[kKmPer], dst[kKmPer];
    uint32_t pieces[kKmPer];
#pragma unroll
    for (int u = 0; u < kKmPer; ++u) {
      const bool on = p0 + u < n;
      const ReadMeta m = on ? rd.meta[perm[p0 + u]] : ReadMeta{};
      src[u] = m.slot;
      pieces[u] = on ? (uint32_t)(slot_span(m.lq, m.ls) / 16) : 0u;
      dst[u] = on ? kslot[p0 + u] : 0ull;
    }
    for (uint32_t i = sub;; i += kKmLanes) {
      uint4 q[kKmPer];
      uint64_t c[kKmPer];
      bool any = false;
#pragma unroll
      for (int u = 0; u < kKmPer; ++u) {
        const bool on = i < pieces[u];
        any |= on;
        q[u] = on ? ((const uint4*)(rd.qual + src[u]))[i] : make_uint4(0, 0, 0, 0);
        c[u] = on ? ((const uint64_t*)(rd.bases + src[u] / 2))[i] : 0ull;
      }
#pragma unroll
      for (int u = 0; u < kKmPer; ++u)
        if (i < pieces[u]) {
          ((uint4*)(kqual + dst[u]))[i] = q[u];
          ((uint64_t*)(kbases + dst[u] / 2))[i] = c[u];
        }
      if (!__builtin_amdgcn_ballot_w64(any)) break;
    }
  }
}

extern "C" __global__ void __launch_bounds__(kSortThreads) bqsr_key_count(const ReadMeta* meta, int64_t n,
                                                                            int32_t n_keys, int32_t n_base,
                                                                            int32_t fronts, uint32_t* counts) {
  __shared__ uint32_t h[kSortLdsKeys];
  const bool lds = n_keys <= kSortLdsKeys;
  if (lds)
    for (int i = threadIdx.x; i < n_keys; i += blockDim.x) h[i] = 0;
  __syncthreads();
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    const int k = sort_key(meta[r], r, n, n_base, fronts);
    if (lds) atomicAdd(&h[k], 1u); else atomicAdd(&counts[k], 1u);
  }
  __syncthreads();
  if (lds)
    for (int i = threadIdx.x; i < n_keys; i += blockDim.x)
      if (h[i]) atomicAdd(&counts[i], h[i]);
}

// one workgroup: key_off = exclusive scan of counts (key_off[n_keys] = n), cursor = key_off
extern "C" __global__ void __launch_bounds__(1024) bqsr_key_scan(const uint32_t* counts, int32_t n_keys,
                                                                   int64_t* key_off, uint32_t* cursor) {
  __shared__ int64_t part[1024];
  const int tid = threadIdx.x;
  const int per = (n_keys + 1023) / 1024;
  const int k0 = min(n_keys, tid * per), k1 = min(n_keys, k0 + per);
  int64_t s = 0;
  for (int k = k0; k < k1; ++k) s += counts[k];
  part[tid] = s;
  __syncthreads();
  if (tid == 0) {
    int64_t acc = 0;
    for (int i = 0; i < 1024; ++i) {
      const int64_t v = part[i];
      part[i] = acc;
      acc += v;
    }
    key_off[n_keys] = acc;
  }
  __syncthreads();
  int64_t acc = part[tid];
  for (int k = k0; k < k1; ++k) {
    key_off[k] = acc;
    cursor[k] = (uint32_t)acc;
    acc += counts[k];
  }
}

extern "C" __global__ void __launch_bounds__(kSortThreads) bqsr_key_scatter(const ReadMeta* meta, int64_t n,
                                                                              int32_t n_keys, int32_t n_base,
                                                                              int32_t fronts, uint32_t* cursor,
                                                                              uint32_t* perm, uint64_t* span) {
  // span (optional): each sorted position's slot span, for the key-major copy's scan
  __shared__ uint32_t h[kSortLdsKeys];
  const bool lds = n_keys <= kSortLdsKeys;
  const int tid = threadIdx.x;
  for (int64_t c0 = (int64_t)blockIdx.x * kSortThreads * kSortPer; c0 < n;
       c0 += (int64_t)gridDim.x * kSortThreads * kSortPer) {
    if (!lds) {
      for (int i = 0; i < kSortPer; ++i) {
        const int64_t r = c0 + (int64_t)i * kSortThreads + tid;
        if (r < n) {
          const ReadMeta m = meta[r];
          const uint32_t pos = atomicAdd(&cursor[sort_key(m, r, n, n_base, fronts)], 1u);
          perm[pos] = (uint32_t)r;
          if (span) span[pos] = slot_span(m.lq, m.ls);
        }
      }
      continue;
    }
    for (int i = tid; i < n_keys; i += kSortThreads) h[i] = 0;
    __syncthreads();
    int key[kSortPer];
    uint32_t rank[kSortPer];
    uint16_t sp[kSortPer];
#pragma unroll
    for (int i = 0; i < kSortPer; ++i) {
      const int64_t r = c0 + (int64_t)i * kSortThreads + tid;
      const ReadMeta m = r < n ? meta[r] : ReadMeta{};
      key[i] = r < n ? sort_key(m, r, n, n_base, fronts) : -1;
      sp[i] = (uint16_t)(slot_span(m.lq, m.ls) >> 4);
    }
#pragma unroll
    for (int i = 0; i < kSortPer; ++i) rank[i] = key[i] >= 0 ? atomicAdd(&h[key[i]], 1u) : 0u;
    __syncthreads();
    for (int i = tid; i < n_keys; i += kSortThreads)
      if (h[i]) h[i] = atomicAdd(&cursor[i], h[i]);  // the workgroup's range of key i
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kSortPer; ++i)
      if (key[i] >= 0) {
        const uint32_t pos = h[key[i]] + rank[i];
        perm[pos] = (uint32_t)(c0 + (int64_t)i * kSortThreads + tid);
        if (span) span[pos] = (uint64_t)sp[i] << 4;
      }
    __syncthreads();
  }
}

// Per-block qual histograms of the folded bases (usable valid reads, trimmed
// ranges) in read order, for bucketed batches whose observe kernel does not
// walk the fold's blocks.  kFhSplit workgroups per block, each adding its
// part into hq_block (zeroed first); lanes as in the lane-per-super-chunk
// passes (2^ls lanes per read, 64 offsets each, 16-B loads).  The kernel is
// bound by its LDS atomics (one per base: 8 / 16 / 32 copies per wavefront
// against same-bin conflicts ran 1.70 / 1.43 / 1.46 ms on cfg4), so a full
// chunk counts its bases in PAIRS: one atomic on the cell (q[2k], q[2k+1]) of
// a 64 x 64 pair table (rows 65 words apart, so a cell's bank is qa + qb mod
// 32, spread over the banks though the quals crowd a few values; a copy per
// lane parity), half the atomics; the tables are expanded (row sums plus
// column sums) once per workgroup.  Partial chunks (a read's last) and pairs
// with a qual >= 64 add single bases to the wavefront's own 128-bin row.
constexpr int kFhWaves = 8;
constexpr int kFhSplit = 4;
constexpr int kFhPairStride = 65;
constexpr int kFhPairWords = 64 * kFhPairStride;
constexpr int kFhPairCopies = 2;
constexpr int kFhStride = kQBins + 1;
constexpr size_t fold_hist_lds() { return ((size_t)kFhPairCopies * kFhPairWords + (size_t)kFhWaves * kFhStride) * 4; }
extern "C" __global__ void __launch_bounds__(kFhWaves * 64) bqsr_fold_hist(ReadsDev rd, const ReadInfo* info,
                                                                             int32_t n_blocks, int32_t ls,
                                                                             uint32_t* hq_block) {
  extern __shared__ uint32_t fh_smem[];
  uint32_t* pairs = fh_smem;
  uint32_t* singles = fh_smem + kFhPairCopies * kFhPairWords;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < kFhPairCopies * kFhPairWords + kFhWaves * kFhStride; i += blockDim.x) fh_smem[i] = 0;
  __syncthreads();
  const int blk = blockIdx.x / kFhSplit, part = blockIdx.x - blk * kFhSplit;
  const int64_t b0 = wg_begin(rd, blk, n_blocks), b1 = wg_begin(rd, blk + 1, n_blocks);
  const int64_t r0 = b0 + (b1 - b0) * part / kFhSplit, r1 = b0 + (b1 - b0) * (part + 1) / kFhSplit;
  uint32_t* pw = pairs + (lane & (kFhPairCopies - 1)) * kFhPairWords;
  uint32_t* sw = singles + wv * kFhStride;
  const int sub = lane & ((1 << ls) - 1), rl = lane >> ls, rpw = 64 >> ls;
  for (int64_t g0 = r0 + (int64_t)rpw * wv; g0 < r1; g0 += (int64_t)rpw * kFhWaves) {
    const int64_t r = g0 + rl;
    int n = 0;
    const uint8_t* qp = rd.qual;
    if (r < r1) {
      const ReadMeta m = rd.meta[r];
      const ReadInfo inf = resolve_info(rd, info_load(info + r), m.slot, m.lq);
      if ((inf.fl & kInfoObs) && inf.en > inf.st) {
        n = inf.en - inf.st;
        qp = rd.qual + m.slot + inf.st;
      }
    }
    for (int j0 = kSuper * sub; __builtin_amdgcn_ballot_w64(j0 < n); j0 += kSuper << ls) {
      if (j0 >= n) continue;
      uint4 v[kSub];
#pragma unroll
      for (int i = 0; i < kSub; ++i) v[i] = j0 + kChunk * i < n ? *(const uint4*)(qp + j0 + kChunk * i) : make_uint4(0, 0, 0, 0);
#pragma unroll
      for (int i = 0; i < kSub; ++i) {
        const int m = n - j0 - kChunk * i;  // valid bytes of chunk i (all when >= 16)
        const uint32_t w[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
        if (m >= kChunk) {
          const bool low = (((w[0] | w[1] | w[2] | w[3]) & 0xC0C0C0C0u) == 0u);  // every qual < 64
          if (low) {
#pragma unroll
            for (int k = 0; k < kChunk; k += 2) {
              const uint32_t qa = __builtin_amdgcn_ubfe(w[k >> 2], 8 * (k & 3), 6);
              const uint32_t qb = __builtin_amdgcn_ubfe(w[k >> 2], 8 * (k & 3) + 8, 6);
              atomicAdd(&pw[__mul24(qa, (uint32_t)kFhPairStride) + qb], 1u);
            }
          } else {
#pragma unroll
            for (int k = 0; k < kChunk; ++k) atomicAdd(&sw[__builtin_amdgcn_ubfe(w[k >> 2], 8 * (k & 3), 7)], 1u);
          }
        } else if (m > 0) {
#pragma unroll
          for (int k = 0; k < kChunk; ++k)  // (a byte past the end adds 0: no branch per byte)
            atomicAdd(&sw[__builtin_amdgcn_ubfe(w[k >> 2], 8 * (k & 3), 7)], k < m ? 1u : 0u);
        }
      }
    }
  }
  __syncthreads();
  for (int q = threadIdx.x; q < kQBins; q += blockDim.x) {
    uint32_t s = 0;
    for (int i = 0; i < kFhWaves; ++i) s += singles[i * kFhStride + q];
    if (q < 64)
      for (int c = 0; c < kFhPairCopies; ++c) {
        const uint32_t* pc = pairs + c * kFhPairWords;
        for (int o = 0; o < 64; ++o) s += pc[q * kFhPairStride + o] + pc[o * kFhPairStride + q];  // q first, q second
      }
    if (s) atomicAdd(&hq_block[(int64_t)blk * kQBins + q], s);
  }
}

// -------------------------------------------------------------- finalize ----
//
// RecalTable.finalizeTable (RecalTable.scala:117-126) and the per-(rg, q)
// apply tables.  Key-level sums first (one wavefront per key), then one
// workgroup for groups / average, then the tables.

extern "C" __global__ void bqsr_final_keys(const int64_t* touched, const int64_t* obs, const int64_t* mm, TableGeom g,
                                           int64_t* qk_obs, int64_t* qk_mm) {
  const int key = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (key >= g.K) return;
  int64_t so = 0, sm = 0;
  if (touched[key]) {
    // qualByRGCounts(k) = cycle covariate's errorsByVariate.values.reduce(_ ++ _)
    for (int c = lane; c < g.C; c += 64) {
      so += obs[(int64_t)key * g.cells + c];
      sm += mm[(int64_t)key * g.cells + c];
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    so += __shfl_down(so, off);
    sm += __shfl_down(sm, off);
  }
  if (lane == 0) {
    qk_obs[key] = so;
    qk_mm[key] = sm;
  }
}

// ErrorCount.getErrorProb (RecalTable.scala:210-214)
__device__ __forceinline__ bool err_prob(int64_t obs, int64_t mm, double mre, double* v) {
  if (obs == 0) return false;
  const double x = (double)mm / (double)obs;
  *v = x > mre ? x : mre;  // math.max(MIN_REASONABLE_ERROR, x); x is never NaN here
  return true;
}

// one workgroup: groups, globals, average, then a2 per (rg, q)
extern "C" __global__ void __launch_bounds__(256) bqsr_final_groups(const int64_t* touched, const int64_t* qk_obs,
                                                                      const int64_t* qk_mm, TableGeom g, int32_t n_rg,
                                                                      double em_host, const double* em_dev,
                                                                      const double* pow10, int32_t n_groups,
                                                                      int64_t* grp_obs, int64_t* grp_mm, uint8_t* grp_ok,
                                                                      uint8_t* key_ok, double* a2, uint8_t* rq_ok,
                                                                      FinalOut* out) {
  const int tid = threadIdx.x;
  __shared__ int64_t s_go[256], s_gm[256];
  __shared__ int s_any[256];
  // readgroups = keys.sorted.groupBy((t - 1) / 60) (Java division): group r
  // (index r + 1) holds keys 0..60 for r = 0 and 60r+1 .. 60r+60 above; one
  // wavefront per group, a lane per key (a thread walking a group's keys was
  // a chain of dependent loads: 14 us of cfg2's job)
  const int lane = tid & 63;
  int64_t go = 0, gm = 0;
  int any = 0;
  for (int i = tid >> 6; i < n_groups; i += blockDim.x >> 6) {
    const int r = i - 1;
    int64_t so = 0, sm = 0;
    int ok = 0;
    if (r >= 0) {
      const int k0 = r == 0 ? 0 : kMaxQ * r + 1, k1 = min(g.K - 1, kMaxQ * r + kMaxQ);  // at most 61 keys
      const int k = k0 + lane;
      if (k <= k1 && touched[k]) {
        ok = 1;
        so = qk_obs[k];
        sm = qk_mm[k];
      }
    }
    for (int off = 32; off > 0; off >>= 1) {
      so += __shfl_xor(so, off);
      sm += __shfl_xor(sm, off);
      ok |= __shfl_xor(ok, off);
    }
    if (lane == 0) {
      grp_obs[i] = so;
      grp_mm[i] = sm;
      grp_ok[i] = (uint8_t)ok;
      go += so;
      gm += sm;
      any |= ok;
    }
  }
  for (int k = tid; k < g.K; k += blockDim.x) key_ok[k] = touched[k] != 0;
  // integer sums: the order is immaterial (wavefront sums, then the four)
  for (int off = 32; off > 0; off >>= 1) {
    go += __shfl_xor(go, off);
    gm += __shfl_xor(gm, off);
    any |= __shfl_xor(any, off);
  }
  if ((tid & 63) == 0) {
    s_go[tid >> 6] = go;
    s_gm[tid >> 6] = gm;
    s_any[tid >> 6] = any;
  }
  __syncthreads();
  if (tid == 0) {
    go = gm = 0;
    any = 0;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) {
      go += s_go[i];
      gm += s_gm[i];
      any |= s_any[i];
    }
    out->g_obs = go;
    out->g_mm = gm;
    out->any_key = any;
    const double em = em_dev ? *em_dev : em_host;
    const double avg = em / (double)go;  // averageReportedError
    out->avg = avg;
    double ge;
    out->global_error = err_prob(go, gm, pow10[kMaxQ], &ge) ? ge : avg;
  }
  __syncthreads();
  const double avg = out->avg;
  const double mre = pow10[kMaxQ];
  // a2 = (e + readGroupDelta) + qualScoreDelta for every (rg, q), q in 0..127
  for (int i = tid; i < n_rg * kQBins; i += blockDim.x) {
    const int rg = i / kQBins, q = i - rg * kQBins;
    const int key = q + kMaxQ * rg;
    const int r = (key - 1) / kMaxQ;
    const bool ok = key < g.K && touched[key] != 0 && grp_ok[r + 1];
    rq_ok[i] = ok;
    if (!ok) {
      a2[i] = 0.0;
      continue;
    }
    double v;
    const double rg_delta = (err_prob(grp_obs[r + 1], grp_mm[r + 1], mre, &v) ? v : avg) - avg;
    const double e = pow10[q];
    const double a1 = e + rg_delta;
    const double q_delta = (err_prob(qk_obs[key], qk_mm[key], mre, &v) ? v : a1) - a1;
    a2[i] = a1 + q_delta;
  }
}

// s1[rq][c] = a2 + cycleDelta, d2[rq][x] = contextDelta (RecalTable.scala:141-145)
extern "C" __global__ void bqsr_final_tables(const int64_t* obs, const int64_t* mm, TableGeom g, int32_t n_rg,
                                             const double* a2, const uint8_t* rq_ok, double mre, double* s1,
                                             double* d2) {
  const int64_t n1 = (int64_t)n_rg * kQBins * g.C, n2 = (int64_t)n_rg * kQBins * kCtxSlots;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n1 + n2; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t rq, cell;
    if (i < n1) {
      rq = i / g.C;
      cell = i - rq * g.C;
    } else {
      rq = (i - n1) / kCtxSlots;
      cell = g.C + (i - n1 - rq * kCtxSlots);
    }
    if (!rq_ok[rq]) {
      if (i < n1) s1[i] = 0.0; else d2[i - n1] = 0.0;
      continue;
    }
    const int rg = (int)(rq / kQBins), q = (int)(rq - (int64_t)rg * kQBins);
    const int64_t key = q + (int64_t)kMaxQ * rg;
    const double x = a2[rq];
    double v;
    const int64_t gi = key * g.cells + cell;
    const double delta = (err_prob(obs[gi], mm[gi], mre, &v) ? v : x) - x;
    if (i < n1) s1[i] = x + delta; else d2[i - n1] = delta;
  }
}

// ----------------------------------------------------------------- apply ----

// errorProbabilityToPhred(p) = javaD2I(-10 * log10(p)) from the bucketed
// threshold table (PhredThresholds / PhredBuckets in bqsr_capi.cpp).
__device__ __forceinline__ int32_t phred_q(double p, const double* qb_thr, const int16_t* qb_q, const double* thr,
                                           int qmin, int nthr) {
  const uint64_t b = (uint64_t)__double_as_longlong(p);
  if (b - 1ull < 0x7FEFFFFFFFFFFFFFull) {  // 0 < p < inf
    const int e = (int)(b >> 52) - 1023;
    if (e >= kQbElo && e <= kQbEhi) {
      const int idx = ((e - kQbElo) << kQbBits) | (int)((b >> (52 - kQbBits)) & ((1u << kQbBits) - 1u));
      const int q = qb_q[idx];
      if (q != -32768) return p <= qb_thr[idx] ? q : q - 1;
    }
    int lo = 0, hi = nthr - 1;  // largest i with p <= thr[i]; thr[0] = DBL_MAX
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (p <= thr[mid]) lo = mid; else hi = mid - 1;
    }
    return qmin + lo;
  }
  if (p != p) return 0;                // NaN: (int)NaN = 0
  if (p == 0.0) return 2147483647;     // log10(0) = -inf
  if (p < 0.0) return 0;               // log10(p < 0) = NaN
  return (int32_t)0x80000000;          // log10(inf) = inf
}

// LDS: the wavefronts' chunk-walk markers (kMkWords u32), then the piece's
// char table [qw rows][cw cycle cells][21 contexts] u8, built once per piece
// from the exact LUT: char = (errorProbabilityToPhred(s1[c] + d2[x]) + 33)
// for every (qual row, cycle cell, context) of the piece's read group, 0
// where the checked path must decide (key not in the table, a char above
// 0xFF, or a genuine 0).  A lane per chunk (chunk_walk); per offset the fast
// path is one LDS byte read.  Offsets it cannot finish (qual outside the
// rows, entry 0, the read only being checked) set a bit of `slow` and are
// redone after the chunk by the exact checked path.  Chunks leave as 16-B
// stores (an unaligned layout's last chunk of a read byte-wise).
struct ApplyPiece {
  const uint8_t* lut;
  int rg_lo, c_lo, cw, cw21, q_lo, qw;
  uint32_t tb;         // LDS address of the context table
  int clean_lo, clean_hi;  // quals whose rows hold no 0 entry
  bool all_cycles;     // the window holds every cycle cell (read order)
  bool folded_clean;   // every qual of every folded base lies in [clean_lo, clean_hi): a folded
                       // (kInfoObs) read's chunks skip the clean-row test
};

struct ChunkLoads {
  uint4 qs, cr;
};
__device__ __forceinline__ ChunkLoads apply_load(const ApplyParams& P, const LaneRead& x, int j, bool on) {
  ChunkLoads v{make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0)};
  if (on) {
    const int o0 = x.st + j;
    v.qs = *(const uint4*)(P.rd.qual + x.slot + o0);
    if (!(x.fl & kInfoPass)) v.cr = chunk_raw(P.rd, chunk_n0(x, o0));
  }
  return v;
}

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));


// The checked path of a chunk's flagged offsets (RecalUtil.recalibrate with
// the table's key checks), out of line: its table pointers stay out of the
// fast path's registers.
__device__ __forceinline__ uint4 apply_slow(const ApplyParams* Pp, LaneRead x, int o0, uint32_t slow, uint64_t x01,
                                         uint64_t x23, uint4 outv) {
  const ApplyParams& P = *Pp;
  const bool app = x.fl & kInfoApp;
  const uint8_t* qp = P.rd.qual + x.slot;
  uint64_t lo = ((uint64_t)outv.y << 32) | outv.x, hi = ((uint64_t)outv.w << 32) | outv.z;
  while (slow) {
    const int k = __builtin_ctz(slow);
    slow &= slow - 1;
    const int o = o0 + k;
    const int q = (int)(int8_t)qp[o];
    const int xs = (int)(((k < 8 ? x01 : x23) >> (8 * (k & 7))) & 0xFFu);
    // key validity as getReadGroupDelta / getQualScoreDelta see it
    const int64_t key = (int64_t)q + (int64_t)kMaxQ * x.rg;
    const int64_t gr = (key - 1) / kMaxQ;
    const bool grp = (gr + 1) >= 0 && (gr + 1) < P.n_groups && P.grp_ok[gr + 1];
    const bool kok = key >= 0 && key < P.g.K && P.key_ok[key];
    if (!grp || !kok) {
      report(P.err, err_key((uint64_t)x.ro, (uint32_t)o, kRankTable, BQSR_ERR_MISSING_KEY));
      continue;
    }
    if (q < 0) {
      report(P.err, err_key((uint64_t)x.ro, (uint32_t)o, kRankTable, BQSR_ERR_QUAL_RANGE));
      continue;
    }
    if (!app) continue;
    const int64_t rq = (int64_t)x.rg * kQBins + q;
    const int ccell = x.cell0 + __mul24(x.dir, o);
    const double p = P.s1[rq * P.g.C + ccell] + P.d2[rq * kCtxSlots + xs];
    const int32_t Q = phred_q(p, P.qb_thr, P.qb_q, P.thr, P.thr_qmin, P.thr_n);
    const uint32_t code = ((uint32_t)Q + 33u) & 0xFFFFu;  // (Q + 33).toChar
    if (code > 0xFFu) {
      const unsigned long long e = atomicAdd(P.n_exc, 1ull);
      if ((int64_t)e < P.max_exc) P.exc[e] = ((x.oslot + (uint64_t)o) << 16) | code;
    }
    // byte k := code
    const uint64_t m = 0xFFull << (8 * (k & 7)), v = (uint64_t)(code & 0xFFu) << (8 * (k & 7));
    if (k < 8) lo = (lo & ~m) | v; else hi = (hi & ~m) | v;
  }
  return make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
}

// kTest: the per-chunk clean-row test.  Without it (the piece's folded_clean:
// every folded base's qual in the clean rows) a folded read's offsets need
// none, and any other read (eligible without an MD tag: its quals are in no
// histogram) takes the checked path for every offset.
template <bool kTest>
__device__ __forceinline__ void apply_chunk(const ApplyParams& P, const ApplyParams* Pp, const ApplyPiece& pc,
                                            const LaneRead& x, int j, int n, bool on, const ChunkLoads& ld) {
  if (!on) return;
  const bool app = x.fl & kInfoApp, pass = x.fl & kInfoPass;
  const int o0 = x.st + j;
  const uint4 qs = ld.qs;
  const uint32_t qd[4] = {qs.x, qs.y, qs.z, qs.w};
  uint32_t out[4];
  uint32_t slow = 0;
  uint32_t xo[4] = {4u, 4u, 4u, 4u};
  if (pass) {  // the original chars: (qual + 33) byte-wise
#pragma unroll
    for (int i2 = 0; i2 < 4; ++i2) out[i2] = ((qd[i2] & 0x7F7F7F7Fu) + 0x21212121u) ^ (qd[i2] & 0x80808080u);
  } else {
    chunk_ctx(P.rd, x.fl & kInfoNeg, chunk_n0(x, o0), ld.cr, j, pc.tb, xo);
    const int wc0 = x.cell0 + __mul24(x.dir, o0) - pc.c_lo;  // window cycle cell of offset k: wc0 + dir * k
    // the cycle cells of the chunk's valid offsets inside the table
    // (monotone in k: both ends)
    const uint32_t nv = (uint32_t)min(kChunk, n - j);
    const int klo = j < 0 ? -j : 0;  // chunk offsets klo .. nv-1 are visited
    const bool cok = app && x.rg == pc.rg_lo &&
                     (pc.all_cycles || ((unsigned)(wc0 + __mul24(klo, x.dir)) < (unsigned)pc.cw &&
                                        (unsigned)(wc0 + __mul24((int)nv - 1, x.dir)) < (unsigned)pc.cw));
    const uint32_t vmask = (nv >= 16u ? 0xFFFFu : ((1u << nv) - 1u)) & (0xFFFFu << klo);
    const int dx = x.dir * kCtxSlots;
    // LDS address of offset k: lut + (q - q_lo) * cw21 + wc0 * 21 + dx * k +
    // xs, clamped to the table's last byte; an offset whose row or cycle
    // cell lies outside the window reads some other entry and is flagged
    // below.  The 16 addresses first (a negative table index wraps far above
    // the table and clamps), then the 16 byte reads into 16-bit halves, two
    // halves per register, merged by byte permutes.  (Reads in processing
    // order with the cycle step as the ds_read's immediate offset -- 8 byte
    // permutes against 16 multiply-adds -- measured equal: cfg2 763 vs 753
    // us, cfg4 3756 vs 3749, round 5.)
    const uint32_t lbase = (uint32_t)(uintptr_t)(LdsBytes)pc.lut;
    const uint32_t amax = lbase + (uint32_t)(pc.qw * pc.cw21 - 1);
    uint32_t ei[kChunk];
    uint32_t ek = lbase + (uint32_t)(wc0 * kCtxSlots - pc.q_lo * pc.cw21);
#pragma unroll
    for (int k = 0; k < kChunk; ++k) {
      const uint32_t q = __builtin_amdgcn_ubfe(qd[k >> 2], 8 * (k & 3), 8);
      const uint32_t xs = __builtin_amdgcn_ubfe(xo[k >> 2], 8 * (k & 3), 8);
      ei[k] = min((uint32_t)__mul24((int)q, pc.cw21) + ek + xs, amax);
      ek += (uint32_t)dx;
    }
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      u16x2 a, b;  // a: bytes 0 and 2 of the word, b: bytes 1 and 3
      a.x = *(LdsBytes)(uintptr_t)ei[4 * w];
      b.x = *(LdsBytes)(uintptr_t)ei[4 * w + 1];
      a.y = *(LdsBytes)(uintptr_t)ei[4 * w + 2];
      b.y = *(LdsBytes)(uintptr_t)ei[4 * w + 3];
      out[w] = __builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, b), __builtin_bit_cast(uint32_t, a), 0x06020400u);
    }
    // per word: bytes whose qual is outside the clean rows (SWAR, per byte
    // no borrow; q >= 128 never is in them) -- entries 0 (key not in the
    // table, a char above 0xFF: the checked path decides) lie only in other
    // rows -- gathered to one bit per offset.  Skipped (kTest false) when a
    // folded read's quals are known to be in the clean rows: cfg2 51 us of
    // the 0.80 ms launch (profiles/r05p_apply_probes.txt)
    uint32_t badm = kTest ? 0u : ((x.fl & kInfoObs) ? 0u : 0xFFFFu);
    if (kTest) {
      const uint32_t lo4 = (uint32_t)pc.clean_lo * 0x01010101u, hi4 = (uint32_t)pc.clean_hi * 0x01010101u;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const uint32_t v = qd[w] | 0x80808080u;
        const uint32_t bad = ((qd[w] | ~(v - lo4) | (v - hi4)) & 0x80808080u) >> 7;  // bit 8i: byte i
        badm |= ((bad | (bad >> 7) | (bad >> 14) | (bad >> 21)) & 0xFu) << (4 * w);  // offsets 4w .. 4w + 3
      }
    }
    slow = vmask & (cok ? badm : 0xFFFFu);
  }
  // ---- the checked path ----
  if (__builtin_amdgcn_ballot_w64(slow != 0)) {
    if (slow) {
      const uint4 r = apply_slow(Pp, x, o0, slow, ((uint64_t)xo[1] << 32) | xo[0], ((uint64_t)xo[3] << 32) | xo[2],
                                 make_uint4(out[0], out[1], out[2], out[3]));
      out[0] = r.x;
      out[1] = r.y;
      out[2] = r.z;
      out[3] = r.w;
    }
  }
  if (app || pass) {
    uint8_t* op = P.out_qual + x.oslot;
    if (j + kChunk <= n || P.rd.slots_aligned) {  // aligned: the chunk's other bytes are this read's scratch
      *(uint4*)(op + o0) = make_uint4(out[0], out[1], out[2], out[3]);
    } else {
#pragma unroll
      for (int k = 0; k < kChunk; ++k)
        if (k < n - j) op[o0 + k] = (uint8_t)(out[k >> 2] >> (8 * (k & 3)));
    }
  }
}

constexpr int kApplyU = 4;  // chunks in flight per lane

// Every piece's char table, once per apply launch: entry (row, cycle cell,
// context) of piece `key` = errorProbabilityToPhred(s1 + d2) + 33, 0 where
// the checked path must decide (key not in the table, a char above 0xFF).
// A thread per entry; each workgroup of bqsr_apply_kernel then copies its
// piece's table into LDS (it used to compute it itself: 65 us of a 0.87 ms
// cfg2 launch with every workgroup repeating the same 156K entries).
// The per-read outputs in read order (bucketed batches, ApplyParams::
// outs_apart): the walk visits a piece's reads scattered over the batch, and
// its two 4-B stores per read each cost a partial line; here a thread per
// read, the stores coalesced.  Same values as the walk's fread.
extern "C" __global__ void bqsr_apply_outs(ApplyParams P) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < P.rd.n_reads; r += (int64_t)gridDim.x * blockDim.x) {
    const LaneRead x = lane_read(P.rd, P.info, r, true, P.g.L);
    if (x.fl & kInfoPass) {  // quality string passed through
      P.out_start[r] = 0;
      P.out_len[r] = (uint32_t)x.en;
    } else {
      P.out_start[r] = (uint32_t)x.st;
      P.out_len[r] = (x.fl & kInfoApp) ? (uint32_t)(x.en - x.st) : 0u;
    }
  }
}

extern "C" __global__ void bqsr_apply_chars(ApplyParams P, uint8_t* chars) {
  const int nk = order_base_keys(P.ord), qw = P.w.qw, q_lo = P.w.q_lo;
  const int64_t total = (int64_t)nk * P.piece_stride;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int key = (int)(t / P.piece_stride);
    const int64_t e = t - (int64_t)key * P.piece_stride;
    const WinGeom gm = win_geom(P.ord, P.g, key);
    const int64_t cw21 = (int64_t)gm.cw * kCtxSlots;
    const bool pad = e >= (int64_t)qw * cw21;  // the piece's padding
    const int row = pad ? 0 : (int)(e / cw21);
    const int rem = (int)(e - row * cw21), c = rem / kCtxSlots, x = rem - c * kCtxSlots;
    const int rg = key_rg(P.ord, key, P.w.rg_lo);
    const int64_t rq = (int64_t)rg * kQBins + q_lo + row;
    uint8_t v = 0;
    if (!pad && rg < P.n_rg && q_lo + row < kQBins && P.rq_ok[rq]) {
      // RecalUtil.recalibrate: (((e + rgD) + qD) + cycD) + ctxD = (a2 + cycD) + ctxD
      const int32_t Q = phred_q(P.s1[rq * P.g.C + gm.c_lo + c] + P.d2[rq * kCtxSlots + x], P.qb_thr, P.qb_q, P.thr,
                                P.thr_qmin, P.thr_n);
      const uint32_t code = ((uint32_t)Q + 33u) & 0xFFFFu;  // (Q + 33).toChar
      v = code <= 0xFFu ? (uint8_t)code : 0;
    }
    if (!pad) chars[t] = v;
    // rows holding a 0 entry: one atomic per run of such entries in the
    // wavefront (a run is one row's; its first lane reports it)
    const int zr = (!pad && v == 0) ? key * kQBins + row : -1;
    const int prev = __shfl_up(zr, 1);
    if (zr >= 0 && ((threadIdx.x & 63) == 0 || prev != zr))
      atomicOr(&P.rowbad[(zr >> 7) * 4 + ((zr & 127) >> 5)], 1u << (zr & 31));
  }
}

extern "C" __global__ void __launch_bounds__(kBlockThreads) bqsr_apply_kernel(ApplyParams P) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int qw = P.w.qw, C = P.g.C, L = P.g.L;
  // LDS: [clean rows 16 B][walk markers][context table][char table]
  uint32_t* clean_rows = (uint32_t*)smem;  // [lo, hi): quals whose char-table rows hold no 0 entry; [2] folded_clean
  uint32_t* mk_all = (uint32_t*)(smem + 16);
  uint16_t* ctab = (uint16_t*)(smem + 16 + kMkWords * 4);
  uint8_t* lut = smem + 16 + kMkWords * 4 + kCtxTabBytes;
  const uint32_t tb = (uint32_t)(uintptr_t)(LdsHalves)ctab;

  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63;
  uint32_t* mk = mk_all + wave * 64;
  const int q_lo = P.w.q_lo;
  const int G = gridDim.x;
  const int64_t wa = pass_begin(P.rd, P.ord, blockIdx.x, G), wb = pass_begin(P.rd, P.ord, blockIdx.x + 1, G);
  const int nk = order_keys(P.ord);
  ctx_table_fill(ctab, tid, blockDim.x);  // ready at the piece loop's first barrier

  for (int key = wa < wb ? key_at(P.ord, wa) : nk; key < nk; ++key) {
    const int64_t p0 = max(wa, key_begin(P.ord, P.rd.n_reads, key));
    const int64_t p1 = min(wb, key_begin(P.ord, P.rd.n_reads, key + 1));
    if (p0 >= wb) break;
    if (p0 >= p1) continue;
    const int rg_lo = key_rg(P.ord, key, P.w.rg_lo);
    const WinGeom gm = win_geom(P.ord, P.g, key);
    __syncthreads();  // the previous piece is done with the table
    // ---- the piece's char table (bqsr_apply_chars) into LDS, 16 B a thread ----
    {
      const uint4* src = (const uint4*)(P.chars + (int64_t)base_key(P.ord, key) * P.piece_stride);
      uint4* dst = (uint4*)lut;
      const int n16 = (int)(P.piece_stride >> 4);
      for (int i = tid; i < n16; i += blockDim.x) dst[i] = src[i];
    }
    if (tid == 0) {  // the longest run of rows without a 0 entry: quals there need no per-entry check
      const uint4 rb = *(const uint4*)(P.rowbad + base_key(P.ord, key) * 4);  // one load, not one per row
      const uint32_t rw[4] = {rb.x, rb.y, rb.z, rb.w};
      int best_lo = 0, best_n = 0, run = 0;
      for (int r = 0; r < qw; ++r) {
        const bool bad = (rw[r >> 5] >> (r & 31)) & 1u;
        run = bad ? 0 : run + 1;
        if (run > best_n) {
          best_n = run;
          best_lo = r - run + 1;
        }
      }
      clean_rows[0] = (uint32_t)(q_lo + best_lo);
      clean_rows[1] = (uint32_t)(q_lo + best_lo + best_n);
      // the batch's folded quals (bins of the fold histograms) all in the clean rows?
      uint32_t fc = 0;
      if (P.qmask) {
        const uint4 qm = *(const uint4*)P.qmask;
        const uint32_t qw4[4] = {qm.x, qm.y, qm.z, qm.w};
        fc = 1;
        for (int q = 0; q < kQBins; ++q)
          if (((qw4[q >> 5] >> (q & 31)) & 1u) && (q < q_lo + best_lo || q >= q_lo + best_lo + best_n)) fc = 0;
      }
      clean_rows[2] = fc;
    }
    __syncthreads();
    const ApplyPiece pc{lut, rg_lo, gm.c_lo, gm.cw, gm.cw * kCtxSlots, q_lo, qw, tb, (int)clean_rows[0],
                        (int)clean_rows[1], gm.c_lo == 0 && gm.cw == C, clean_rows[2] != 0};
    const auto fread = [&](LaneRead& x, bool live) {
      if (!live || P.outs_apart) return;
      if (x.fl & kInfoPass) {  // quality string passed through
        P.out_start[x.ro] = 0;
        P.out_len[x.ro] = (uint32_t)x.en;
      } else {
        P.out_start[x.ro] = (uint32_t)x.st;
        P.out_len[x.ro] = (x.fl & kInfoApp) ? (uint32_t)(x.en - x.st) : 0u;
      }
    };
    const auto fload = [&](const LaneRead& x, int j, bool on) { return apply_load(P, x, j, on); };
    // two instances of the walk, picked per piece (uniform): with and
    // without the clean-row test (a per-lane branch around it cost spills)
    if (pc.folded_clean) {
      const auto fchunk = [&](const LaneRead& x, int j, int n, bool on, const ChunkLoads& ld) {
        apply_chunk<false>(P, &P, pc, x, j, n, on, ld);
      };
      chunk_walk<kInfoApp | kInfoAppCheck | kInfoPass, kApplyU, ChunkLoads, false>(
          P.rd, P.info, P.ord, p0 + 64 * wave, p1, 64 * kWaves, L, lane, mk, fread, fload, fchunk);
    } else {
      const auto fchunk = [&](const LaneRead& x, int j, int n, bool on, const ChunkLoads& ld) {
        apply_chunk<true>(P, &P, pc, x, j, n, on, ld);
      };
      chunk_walk<kInfoApp | kInfoAppCheck | kInfoPass, kApplyU, ChunkLoads, false>(
          P.rd, P.info, P.ord, p0 + 64 * wave, p1, 64 * kWaves, L, lane, mk, fread, fload, fchunk);
    }
  }  // pieces
}


// RecalTable.++ over partitions in a declared order (RecalTable.scala:90-108):
// expectedMismatch = ((0.0 + e_0) + e_1) + ... -- one lane, each `+` one IEEE
// double addition as on the JVM's driver
extern "C" __global__ void bqsr_em_fold(const double* ems, int64_t n, double* out) {
  if (threadIdx.x != 0) return;
  double s = 0.0;
  for (int64_t i = 0; i < n; ++i) s = s + ems[i];
  *out = s;
}

// ------------------------------------------------------- job reset / status --
extern "C" __global__ void bqsr_job_reset_kernel(int64_t* words, int64_t n, unsigned long long* err) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    words[i] = 0;
  if (blockIdx.x == 0 && threadIdx.x < kErrWords) err[threadIdx.x] = threadIdx.x == kNExc ? 0ull : ~0ull;
}
// [0, kErrWords) error words, [kErrWords] expectedMismatch bits, then FinalOut
extern "C" __global__ void bqsr_job_status_kernel(const unsigned long long* err, const double* em, const FinalOut* fo,
                                                  uint64_t* host) {
  const int t = threadIdx.x;
  if (t < kErrWords) host[t] = err[t];
  else if (t == kErrWords) host[t] = (uint64_t)__double_as_longlong(*em);
  else if (t < kErrWords + 1 + (int)(sizeof(FinalOut) / 8)) host[t] = ((const uint64_t*)fo)[t - kErrWords - 1];
}

// Multi-rank error exchange (every rank raises the job's first error in global
// read order, as the reference's one job fails on its first failing
// partition): the batch's observe and apply error keys rebased to global read
// indices (read_base << 28 added) as signed int64, no error = INT64_MAX, for
// an all-reduce MIN; then the reduced keys written back as the batch's own.
extern "C" __global__ void bqsr_job_err_export(const unsigned long long* err, int64_t read_base, int64_t* out) {
  const int t = threadIdx.x;
  if (t >= 2) return;
  const unsigned long long k = t == 0 ? err[kErrObs] : min(err[kErrAppPrep], err[kErrAppKern]);
  out[t] = k == kNoError ? INT64_MAX : (int64_t)(k + ((unsigned long long)read_base << 28));
}
extern "C" __global__ void bqsr_job_err_import(unsigned long long* err, const int64_t* in) {
  const int t = threadIdx.x;
  if (t == 0) err[kErrObs] = in[0] == INT64_MAX ? kNoError : (unsigned long long)in[0];
  if (t == 1) err[kErrAppPrep] = in[1] == INT64_MAX ? kNoError : (unsigned long long)in[1];
  if (t == 2) err[kErrAppKern] = kNoError;
}

// --------------------------------------------------------- table merge -----
extern "C" __global__ void bqsr_table_add(int64_t* acc, const int64_t* part, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    acc[i] += part[i];
}

}  // namespace bqsr
