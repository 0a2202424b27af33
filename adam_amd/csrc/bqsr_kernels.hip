// bqsr_kernels.hip -- gfx950 kernels of the BQSR path.
//
//   bqsr_observe_kernel   RecalibrateBaseQualities.computeTable, one partition
//   bqsr_fold_kernel      expectedMismatch: the partition's sequential fold
//   bqsr_final_*          RecalTable.finalizeTable + the apply tables
//   bqsr_apply_kernel     RecalUtil.recalibrate over every eligible read
//   bqsr_table_add        RecalTable.++ (int64 counts)
//
// Structure (DESIGN.md has the full account): one 512-thread workgroup per CU,
// each owning a contiguous range of read tiles; each wavefront processes one
// tile (<= 64 reads, <= 2048 base slots) at a time:
//   1. stage the tile's packed bases / MD / CIGAR into LDS (coalesced),
//   2. per-read prep, one lane per read: quality trimming, CIGAR walk, MD
//      parse, known-site lookup -> two LDS bitmasks {masked, mismatch} over
//      the tile's slots (the "2-bit structural mask" of SURVEY.md 8d),
//   3. per-base pass, 16 slots per lane per step (one 16-B qual load):
//      covariates -> LDS-privatised u32 histogram of the workgroup's window
//      of the table; bases outside the window go to global int64 atomics,
//   4. at the end the workgroup flushes its window with int64 atomics.
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

// set bits [lo, hi) of an LDS bitmap (ranges of different reads may share a word)
__device__ void lds_set_bits(uint32_t* bits, int lo, int hi) {
  while (lo < hi) {
    int w = lo >> 5, b = lo & 31;
    int n = min(32 - b, hi - lo);
    uint32_t m = (n == 32) ? 0xFFFFFFFFu : (((1u << n) - 1u) << b);
    atomicOr(&bits[w], m);
    lo += n;
  }
}

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
template <class F>
__device__ bool md_scan(const uint8_t* md, int n, int64_t* total, F&& nonmatch) {
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
__device__ int refpos_to_offset(const uint32_t* cig, int ncig, int64_t unclipped, int64_t p) {
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

__device__ __forceinline__ int64_t lower_bound_i64(const int64_t* a, int64_t n, int64_t v) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    int64_t mid = (lo + hi) >> 1;
    if (a[mid] < v) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// per-read results of the prep step, kept in LDS for the per-base pass
struct ReadRow {
  uint16_t st, en, ls, fl, rg;
};
constexpr uint16_t kRowActive = 1, kRowNeg = 2, kRowSecond = 4, kRowQualCheck = 8;

// Per-read prep, one lane per read (ReadCovariates' constructor plus the
// per-read parts of next(), ReadCovariates.scala:30-60):
//   quality trimming, the error checks in the order the JVM would hit them,
//   and (observe) the masked / mismatch bits of every trimmed base:
//   masked   = refPos None, refPos outside [start, end), or a known site
//              (ReadCovariates.scala:56: snp(o) || mismatch(o).isEmpty);
//   mismatch = !MdTag.isMatch(refPos)  (RichADAMRecord.scala:138-154).
template <bool kObserve>
__device__ ReadRow prep_read(const ReadsDev& rd, const SitesDev& sites, uint64_t r, const ReadMeta& m,
                             const ReadAlign& a, int rslot, const uint32_t* cig, const uint8_t* md, uint32_t* mmbits,
                             uint32_t* maskbits, unsigned long long* err) {
  ReadRow row{0, 0, m.ls, 0, m.rg};
  const uint16_t f = m.flags;
  if (!(kObserve ? usable_read(f) : eligible_read(f))) return row;
  if (!(f & BQSR_F_HAS_QUAL)) {  // qualityScores: getQual.toString
    report(err, err_key(r, 0, kRankCtor, BQSR_ERR_NULL_FIELD));
    return row;
  }
  const uint8_t* q = rd.qual + m.slot;
  const int lq = m.lq;
  int st = 0;
  while (st < lq && (int8_t)q[st] <= 2) ++st;  // isLowQualityBase, minQuality = 2
  int tail = 0;
  while (tail < lq && (int8_t)q[lq - 1 - tail] <= 2) ++tail;
  const int en = lq - tail;
  if (!(f & BQSR_F_HAS_RG)) {  // QualByRG: 60 * getRecordGroupId
    report(err, err_key(r, 0, kRankCtor, BQSR_ERR_NULL_RG));
    return row;
  }
  if (!(f & BQSR_F_HAS_SEQ)) {  // DiscreteCycle: getSequence.toString
    report(err, err_key(r, 0, kRankCtor, BQSR_ERR_NULL_FIELD));
    return row;
  }
  if ((f & BQSR_F_NEG_STRAND) && (f & kSeqOther)) {  // BaseContext reverse complement
    report(err, err_key(r, 0, kRankCtor, BQSR_ERR_BAD_REVCOMP_BASE));
    return row;
  }
  if (st >= en) return row;  // no base is iterated
  row.st = (uint16_t)st;
  if (!(f & BQSR_F_HAS_CIGAR) || !(f & BQSR_F_HAS_START)) {  // referencePositions
    report(err, err_key(r, st, kRankCigar, BQSR_ERR_NULL_FIELD));
    return row;
  }
  // walk the CIGAR once: clip, read-consuming and reference-consuming lengths
  const int ncig = a.n_cigar;
  int64_t lead = 0;
  bool leading = true, zero = false;
  int64_t rp_len = 0, ref_len = 0;
  for (int i = 0; i < ncig; ++i) {
    uint32_t e = cig[i], op = cig_op(e), len = cig_len(e);
    if (leading && (op == BQSR_CIGAR_S || op == BQSR_CIGAR_H)) lead += len; else leading = false;
    if (is_seg_op(op) || op == BQSR_CIGAR_I) rp_len += len;
    if (is_seg_op(op) && len == 0) zero = true;
    if (consumes_ref(op)) ref_len += len;
  }
  if (zero) {  // Range(a, a).last
    report(err, err_key(r, st, kRankCigar, BQSR_ERR_CIGAR_INVALID));
    return row;
  }
  const int64_t start = a.start;
  const int64_t unclipped = start - lead;
  const int64_t ref_end = start + ref_len;
  if (unclipped < -2147483648LL || unclipped + rp_len + ref_len > 2147483647LL) {
    // the reference does this arithmetic in Int; positions that wrap are not supported here
    report(err, err_key(r, st, kRankCigar, BQSR_ERR_UNSUPPORTED));
    return row;
  }
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
  uint64_t best = kNoError;
  int64_t md_total = 0;
  if (o_first >= 0) {
    if (f & BQSR_F_HAS_MD) {
      if (!md_scan(md, a.md_len, &md_total, [](int64_t) {}))
        best = min(best, err_key(r, o_first, kRankMd, BQSR_ERR_MD_PARSE));
    }
    if (!(f & BQSR_F_HAS_REFNAME)) best = min(best, err_key(r, o_first, kRankSnp, BQSR_ERR_NULL_FIELD));
  }
  if ((int64_t)en > rp_len) best = min(best, err_key(r, (uint32_t)max((int64_t)st, rp_len), kRankCigar, BQSR_ERR_CIGAR_SHORT));
  if (en > (int)m.ls) best = min(best, err_key(r, (uint32_t)max(st, (int)m.ls), kRankCov, BQSR_ERR_SEQ_SHORT));
  if (best != kNoError) {
    report(err, best);
    // bases before the failing one are still checked for negative quals
    row.en = (uint16_t)((best >> 8) & 0xFFFFF);
    row.fl = kRowQualCheck;
    return row;
  }
  row.en = (uint16_t)en;
  row.fl = kRowActive | ((f & BQSR_F_NEG_STRAND) ? kRowNeg : 0) |
           (((f & BQSR_F_PAIRED) && (f & BQSR_F_SECOND_OF_PAIR)) ? kRowSecond : 0);
  if (!kObserve) return row;

  // ---- masked / mismatch bits over [st, en) ----
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
          lds_set_bits(maskbits, rslot + lo, rslot + a0);
          lds_set_bits(maskbits, rslot + max(a1, a0), rslot + hi);
        }
        ro += len;
        pos += len;
      } else if (op == BQSR_CIGAR_I) {  // insertion: refPos None
        int lo = max(ro, st), hi = min(ro + (int)len, en);
        lds_set_bits(maskbits, rslot + lo, rslot + max(lo, hi));
        ro += len;
      } else if (op != BQSR_CIGAR_H) {
        pos += len;
      }
    }
  }
  // MD non-match positions inside the overlap window
  md_scan(md, a.md_len, &md_total, [&](int64_t prel) {
    int64_t p = start + prel;
    if (p >= ref_end) return;
    int o = refpos_to_offset(cig, ncig, unclipped, p);
    if (o >= st && o < en) lds_set_bits(mmbits, rslot + o, rslot + o + 1);
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
          if (lo < hi) lds_set_bits(mmbits, rslot + lo, rslot + hi);
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
  if (a.contig >= 0 && a.contig < sites.n_contigs) {
    const int64_t* sp = sites.pos + sites.off[a.contig];
    const int64_t ns = (int64_t)(sites.off[a.contig + 1] - sites.off[a.contig]);
    if (ns > 0) {
      // reference span of the trimmed bases: refPos is increasing along the read
      int64_t lo_p = unclipped, hi_p = unclipped + rp_len + ref_len;
      const uint32_t* bk = sites.bucket + sites.bucket_off[a.contig];
      const int64_t nb = (int64_t)(sites.bucket_off[a.contig + 1] - sites.bucket_off[a.contig]);
      const int64_t base = sites.bucket_base[a.contig];
      int64_t j;
      int64_t bi = (lo_p - base) >> sites.shift;
      if (bi < 0) j = 0;
      else if (bi >= nb) j = ns;
      else j = bk[bi];
      while (j < ns && sp[j] < lo_p) ++j;
      for (; j < ns && sp[j] < hi_p; ++j) {
        int o = refpos_to_offset(cig, ncig, unclipped, sp[j]);
        if (o >= st && o < en) lds_set_bits(maskbits, rslot + o, rslot + o + 1);
      }
    }
  }
  return row;
}

// base code at tile-relative slot s (bases staged from absolute slot ts0 & ~1)
__device__ __forceinline__ uint32_t base_code(const uint8_t* st_bases, int s_abs_rel) {
  uint8_t b = st_bases[s_abs_rel >> 1];
  return (s_abs_rel & 1) ? (b >> 4) : (b & 0xF);
}

// BaseContext(2) value of read offset o (StandardCovariate.scala:59-90),
// including the mirrored reverse-strand indexing (quirk Q9).
__device__ __forceinline__ int context_of(const uint8_t* stb, int bshift, int rslot, int o, int st, int en, bool neg) {
  const int k = o - st;
  if (k == 0) return 0;
  uint32_t ca, cb;
  if (!neg) {
    ca = base_code(stb, bshift + rslot + o - 1);
    cb = base_code(stb, bshift + rslot + o);
    if (ca == kCodeN || cb == kCodeN) return 0;
    int ia = ca < 4 ? (int)ca : -1, ib = cb < 4 ? (int)cb : -1;
    return 1 + 4 * ia + ib;
  }
  const int ia_o = en + st - o;  // complement of s[end - k], s[end - 1 - k]
  ca = base_code(stb, bshift + rslot + ia_o);
  cb = base_code(stb, bshift + rslot + ia_o - 1);
  if (ca == kCodeN || cb == kCodeN) return 0;
  return 1 + 4 * (3 - (int)ca) + (3 - (int)cb);
}

// ----------------------------------------------------------- tile staging --

struct WaveStage {
  uint8_t bases[kTileSlots / 2 + 16];
  uint32_t mmbits[kTileSlots / 32 + 1];
  uint32_t maskbits[kTileSlots / 32 + 1];
  uint16_t rslot[kMaxTileReads + 1];
  ReadRow rows[kMaxTileReads];
  uint32_t hist[kQBins];
  uint8_t md[kMdStage];
  uint32_t cigar[kCigarStage];
};

struct TileInfo {
  int64_t r0;
  int nr;
  uint64_t ts0;  // absolute slot of the tile start
  int nslots;
  int bshift;    // ts0 & 1 (the staged bases start at ts0 & ~1)
  bool md_staged, cig_staged;
  uint32_t md0, cig0;
};

// Load the tile's per-read records, stage bases / MD / CIGAR, and clear the
// per-tile LDS state.  Returns this lane's read records.
__device__ TileInfo stage_tile(const ReadsDev& rd, int64_t tile, WaveStage& ws, int lane, ReadMeta& m, ReadAlign& a,
                               bool stage_bases) {
  TileInfo ti;
  ti.r0 = tile * (int64_t)rd.reads_per_tile;
  ti.nr = (int)min((int64_t)rd.reads_per_tile, rd.n_reads - ti.r0);
  if (lane < ti.nr) {
    m = rd.meta[ti.r0 + lane];
    a = rd.align[ti.r0 + lane];
  } else {
    m = ReadMeta{0, 0, 0, 0, 0};
    a = ReadAlign{0, 0, 0, -1, 0, 0};
  }
  const int last = ti.nr - 1;
  ti.ts0 = __shfl(m.slot, 0);
  const uint64_t last_slot = __shfl(m.slot, last);
  const uint32_t last_len = __shfl((uint32_t)max(m.lq, m.ls), last);
  const uint64_t ts1 = last_slot + last_len;
  ti.nslots = (int)(ts1 - ti.ts0);
  ti.bshift = (int)(ti.ts0 & 1);
  if (lane < ti.nr) ws.rslot[lane] = (uint16_t)(m.slot - ti.ts0);
  if (lane == 0) ws.rslot[ti.nr] = (uint16_t)ti.nslots;
  // MD / CIGAR ranges of the tile are contiguous
  ti.md0 = __shfl(a.md_off, 0);
  const uint32_t md1 = __shfl(a.md_off + (uint32_t)a.md_len, last);
  ti.cig0 = __shfl(a.cigar_off, 0);
  const uint32_t cig1 = __shfl(a.cigar_off + (uint32_t)a.n_cigar, last);
  ti.md_staged = (md1 - ti.md0) <= (uint32_t)kMdStage;
  ti.cig_staged = (cig1 - ti.cig0) <= (uint32_t)kCigarStage;
  if (ti.md_staged)
    for (uint32_t i = lane; i < md1 - ti.md0; i += 64) ws.md[i] = rd.md[ti.md0 + i];
  if (ti.cig_staged)
    for (uint32_t i = lane; i < cig1 - ti.cig0; i += 64) ws.cigar[i] = rd.cigar[ti.cig0 + i];
  if (stage_bases) {
    const uint64_t b0 = ti.ts0 >> 1, b1 = (ts1 + 1) >> 1;
    for (uint64_t i = lane; i < b1 - b0; i += 64) ws.bases[i] = rd.bases[b0 + i];
  }
  for (int i = lane; i < kTileSlots / 32 + 1; i += 64) {
    ws.mmbits[i] = 0;
    ws.maskbits[i] = 0;
  }
  for (int i = lane; i < kQBins; i += 64) ws.hist[i] = 0;
  return ti;
}

__device__ __forceinline__ int find_row(const uint16_t* rslot, int nr, int s) {
  int lo = 0, hi = nr;  // last i with rslot[i] <= s
  while (hi - lo > 1) {
    int mid = (lo + hi) >> 1;
    if (rslot[mid] <= s) lo = mid; else hi = mid;
  }
  return lo;
}

// ------------------------------------------------------------ observe ------

// LDS: [obs window qw*cells u32][mm window qw*cells u32][masked qw u32]
//      [block hist 128 u32][tile counter] [WaveStage x 8]
extern "C" __global__ void __launch_bounds__(kBlockThreads) bqsr_observe_kernel(ObserveParams P) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int qw = P.w.qw, cells = P.g.cells, C = P.g.C, L = P.g.L;
  uint32_t* w_obs = (uint32_t*)smem;
  uint32_t* w_mm = w_obs + qw * cells;
  uint32_t* w_masked = w_mm + qw * cells;
  uint32_t* blk_hist = w_masked + qw;
  uint32_t* blk_next = blk_hist + kQBins;
  uintptr_t stage_off = ((uintptr_t)(blk_next + 4) - (uintptr_t)smem + 15) & ~(uintptr_t)15;
  WaveStage* stages = (WaveStage*)(smem + stage_off);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < 2 * qw * cells + qw; i += blockDim.x) w_obs[i] = 0;
  for (int i = tid; i < kQBins; i += blockDim.x) blk_hist[i] = 0;
  const int64_t nt = P.rd.n_tiles;
  const int64_t tb0 = nt * blockIdx.x / P.n_blocks, tb1 = nt * (blockIdx.x + 1) / P.n_blocks;
  if (tid == 0) blk_next[0] = 0;
  __syncthreads();

  WaveStage& ws = stages[wave];
  for (;;) {
    int64_t t;
    {
      uint32_t ti = 0;
      if (lane == 0) ti = atomicAdd(&blk_next[0], 1u);
      ti = __shfl(ti, 0);
      t = tb0 + ti;
    }
    if (t >= tb1) break;
    ReadMeta m;
    ReadAlign a;
    TileInfo T = stage_tile(P.rd, t, ws, lane, m, a, true);
    wave_sync();
    if (lane < T.nr) {
      const uint32_t* cig = T.cig_staged ? ws.cigar + (a.cigar_off - T.cig0) : P.rd.cigar + a.cigar_off;
      const uint8_t* md = T.md_staged ? ws.md + (a.md_off - T.md0) : P.rd.md + a.md_off;
      ws.rows[lane] = prep_read<true>(P.rd, P.sites, (uint64_t)(T.r0 + lane), m, a, (int)(m.slot - T.ts0), cig, md,
                                      ws.mmbits, ws.maskbits, P.err);
    }
    wave_sync();
    // ---- per-base pass: 16-slot chunks, one 16-B qual load per lane ----
    const uint64_t c0 = T.ts0 >> 4, c1 = (T.ts0 + T.nslots + 15) >> 4;
    for (uint64_t c = c0 + lane; c < c1; c += 64) {
      const uint4 qv = *(const uint4*)(P.rd.qual + (c << 4));
      const uint32_t qw4[4] = {qv.x, qv.y, qv.z, qv.w};
      int s = (int)((int64_t)(c << 4) - (int64_t)T.ts0);  // tile-relative slot of the chunk's first byte
      int i = find_row(ws.rslot, T.nr, max(s, 0));
      int nexts = ws.rslot[i + 1];
      ReadRow row = ws.rows[i];
      int rs = ws.rslot[i];
#pragma unroll 4
      for (int j = 0; j < 16; ++j, ++s) {
        if (s < 0 || s >= T.nslots) continue;
        while (s >= nexts) {
          ++i;
          nexts = ws.rslot[i + 1];
          row = ws.rows[i];
          rs = ws.rslot[i];
        }
        if (!(row.fl & (kRowActive | kRowQualCheck))) continue;
        const int o = s - rs;
        if (o < row.st || o >= row.en) continue;
        const int q = (int)(int8_t)((qw4[j >> 2] >> ((j & 3) * 8)) & 0xFF);
        if (q < 0) {  // RecalTable.+= : phredToErrorProbabilityCache(qual)
          report(P.err, err_key((uint64_t)(T.r0 + i), o, kRankTable, BQSR_ERR_QUAL_RANGE));
          continue;
        }
        if (!(row.fl & kRowActive)) continue;
        const bool neg = row.fl & kRowNeg;
        const bool masked = (ws.maskbits[s >> 5] >> (s & 31)) & 1u;
        const bool mism = (ws.mmbits[s >> 5] >> (s & 31)) & 1u;
        int cyc = neg ? ((int)row.ls - o) : (o + 1);  // DiscreteCycle
        if (row.fl & kRowSecond) cyc = -cyc;
        const int ctx = context_of(ws.bases, T.bshift, rs, o, row.st, row.en, neg);
        atomicAdd(&ws.hist[q], 1u);
        const int slot = q - P.w.q_lo;
        if ((int)row.rg == P.w.rg_lo && (unsigned)slot < (unsigned)qw) {
          if (masked) {
            atomicAdd(&w_masked[slot], 1u);
          } else {
            const int c_cyc = slot * cells + (cyc + L), c_ctx = slot * cells + C + (ctx + 4);
            atomicAdd(&w_obs[c_cyc], 1u);
            atomicAdd(&w_obs[c_ctx], 1u);
            if (mism) {
              atomicAdd(&w_mm[c_cyc], 1u);
              atomicAdd(&w_mm[c_ctx], 1u);
            }
          }
        } else {  // outside the LDS window: straight to the int64 table
          const int64_t key = (int64_t)q + (int64_t)kMaxQ * row.rg;
          atomicAdd((unsigned long long*)&P.touched[key], 1ull);
          if (!masked) {
            const int64_t c_cyc = key * cells + (cyc + L), c_ctx = key * cells + C + (ctx + 4);
            atomicAdd((unsigned long long*)&P.obs[c_cyc], 1ull);
            atomicAdd((unsigned long long*)&P.obs[c_ctx], 1ull);
            if (mism) {
              atomicAdd((unsigned long long*)&P.mm[c_cyc], 1ull);
              atomicAdd((unsigned long long*)&P.mm[c_ctx], 1ull);
            }
          }
        }
      }
    }
    wave_sync();
    // per-tile histogram of folded quals (input of the exact expectedMismatch fold)
    for (int k = lane; k < kQBins; k += 64) {
      const uint32_t h = ws.hist[k];
      P.h2[t * kQBins + k] = (uint16_t)h;
      if (h) atomicAdd(&blk_hist[k], h);
    }
    wave_sync();
  }
  __syncthreads();
  // ---- flush the window (int64 atomics) ----
  const int64_t key0 = (int64_t)P.w.q_lo + (int64_t)kMaxQ * P.w.rg_lo;
  for (int i = tid; i < qw * cells; i += blockDim.x) {
    const int slot = i / cells, cell = i - slot * cells;
    if (key0 + slot >= P.g.K) continue;
    const uint32_t o = w_obs[i], mmv = w_mm[i];
    const int64_t g = (key0 + slot) * cells + cell;
    if (o) atomicAdd((unsigned long long*)&P.obs[g], (unsigned long long)o);
    if (mmv) atomicAdd((unsigned long long*)&P.mm[g], (unsigned long long)mmv);
  }
  for (int slot = tid; slot < qw; slot += blockDim.x) {
    if (key0 + slot >= P.g.K) continue;
    uint64_t tot = w_masked[slot];
    for (int c = 0; c < C; ++c) tot += w_obs[slot * cells + c];  // every unmasked base hits one cycle cell
    if (tot) atomicAdd((unsigned long long*)&P.touched[key0 + slot], (unsigned long long)tot);
  }
  for (int k = tid; k < kQBins; k += blockDim.x) P.hq_block[(int64_t)blockIdx.x * kQBins + k] = blk_hist[k];
}

// ------------------------------------------------------ expectedMismatch --
//
// The reference folds expectedMismatch += pow10cache[q] sequentially over the
// partition (RecalTable.scala:61) and the low bits of that double decide
// Q59 vs Q60, so the fold is replayed exactly.  While the sum
// S stays inside one binade [2^e, 2^(e+1)), fl(S + t) = S + u*round(t/u)
// with u = 2^(e-52) (no ties), so a run of additions is an integer sum of
// per-qual increments: the per-block and per-tile qual histograms written by
// the observe kernel give that sum for whole blocks / tiles at once.  Only the
// additions that leave the binade (about log2(S_end/S_0) of them) or hit a
// rounding tie are done one by one, in double arithmetic, exactly as the JVM
// does.  One workgroup of 256 threads.

constexpr int kFoldThreads = 256;

struct FoldShared {
  double t[kQBins];        // phredToErrorProbabilityCache
  double inc[kQBins];      // round(t / u) at the current binade
  uint8_t tie[kQBins];     // t / u is exactly a half-integer at the current binade
  double red[kFoldThreads];
  uint8_t stream[kTileSlots];
  int32_t lens[kMaxTileReads + 1];
  int32_t sts[kMaxTileReads];
  double S;
  int32_t e;
  int32_t mode_seq;
  int32_t found;
  int32_t ntot;
  double cut_sum;
};

__device__ __forceinline__ double two_pow(int k) { return ldexp(1.0, k); }

// (re)derive the binade state of S and the increment table
__device__ void fold_set_binade(FoldShared& F, int tid, double Sv) {
  __syncthreads();
  if (tid == 0) {
    F.S = Sv;
    int e = ilogb(Sv);
    F.e = e;
  }
  __syncthreads();
  const int e = F.e;
  for (int q = tid; q < kQBins; q += kFoldThreads) {
    double x = ldexp(F.t[q], 52 - e);
    double fl = floor(x);
    F.tie[q] = (x - fl) == 0.5;
    F.inc[q] = rint(x);
  }
  __syncthreads();
}

// Materialise a tile's fold-order qual stream (usable reads, trimmed bases)
// into LDS; returns its length.
__device__ int fold_stream(const ReadsDev& rd, int64_t tile, FoldShared& F, int tid) {
  const int64_t r0 = tile * (int64_t)rd.reads_per_tile;
  const int nr = (int)min((int64_t)rd.reads_per_tile, rd.n_reads - r0);
  if (tid < nr) {
    const ReadMeta m = rd.meta[r0 + tid];
    int st = 0, en = 0;
    if (usable_read(m.flags) && (m.flags & BQSR_F_HAS_QUAL)) {
      const uint8_t* q = rd.qual + m.slot;
      const int lq = m.lq;
      while (st < lq && (int8_t)q[st] <= 2) ++st;
      int tail = 0;
      while (tail < lq && (int8_t)q[lq - 1 - tail] <= 2) ++tail;
      en = lq - tail;
      if (en < st) en = st;
    }
    F.lens[tid] = en - st;
    F.sts[tid] = st;
  }
  __syncthreads();
  if (tid == 0) {
    int acc = 0;
    for (int i = 0; i < nr; ++i) {
      int l = F.lens[i];
      F.lens[i] = acc;
      acc += l;
    }
    F.lens[nr] = acc;
    F.ntot = acc;
  }
  __syncthreads();
  for (int i = 0; i < nr; ++i) {
    const int b = F.lens[i], n = F.lens[i + 1] - b;
    if (n == 0) continue;
    const uint8_t* q = rd.qual + rd.meta[r0 + i].slot + F.sts[i];
    for (int k = tid; k < n; k += kFoldThreads) F.stream[b + k] = q[k];
  }
  __syncthreads();
  return F.ntot;
}

// block-wide inclusive scan of doubles (exact for integer values < 2^53)
__device__ double block_scan(FoldShared& F, int tid, double v) {
  F.red[tid] = v;
  __syncthreads();
  for (int off = 1; off < kFoldThreads; off <<= 1) {
    double x = (tid >= off) ? F.red[tid - off] : 0.0;
    __syncthreads();
    F.red[tid] += x;
    __syncthreads();
  }
  double r = F.red[tid];
  __syncthreads();
  return r;
}

// Fold one tile's stream exactly, starting from F.S.
__device__ void fold_tile_exact(const ReadsDev& rd, int64_t tile, FoldShared& F, int tid, double seq_limit) {
  const int n = fold_stream(rd, tile, F, tid);
  int pos = 0;
  while (pos < n) {
    if (F.S < seq_limit) {
      // small S: the binade changes every few additions -- plain sequential fold
      if (tid == 0) {
        double S = F.S;
        int p = pos;
        for (; p < n && S < seq_limit; ++p) S = S + F.t[F.stream[p]];
        F.S = S;
        F.ntot = p;
      }
      __syncthreads();
      pos = F.ntot;
      if (F.S >= seq_limit) fold_set_binade(F, tid, F.S);
      continue;
    }
    // binade mode: per-thread contiguous runs of the remaining stream
    const double N0 = ldexp(F.S, 52 - F.e);  // S / u, an integer < 2^53
    const double head = 9007199254740992.0 - N0;  // additions allowed before leaving the binade
    const int rem = n - pos;
    const int per = (rem + kFoldThreads - 1) / kFoldThreads;
    const int a = pos + tid * per, b = min(a + per, n);
    double mine = 0.0;
    int stop = -1;
    for (int k = a; k < b; ++k) {
      const int q = F.stream[k];
      if (F.tie[q]) { stop = k; break; }
      mine += F.inc[q];
    }
    // prefix over threads of the sums before each thread's stop (or whole run)
    double incl = block_scan(F, tid, mine);
    double excl = incl - mine;
    // first element where the running count reaches `head` or a tie sits
    if (tid == 0) F.found = 0x7FFFFFFF;
    __syncthreads();
    {
      int cand = 0x7FFFFFFF;
      if (a < b) {
        if (excl + mine >= head || stop >= 0) {
          // locate inside this run
          double run = excl;
          for (int k = a; k < b; ++k) {
            const int q = F.stream[k];
            if (F.tie[q] || run + F.inc[q] >= head) { cand = k; break; }
            run += F.inc[q];
          }
        }
      }
      if (cand != 0x7FFFFFFF) atomicMin(&F.found, cand);
    }
    __syncthreads();
    const int found = F.found;
    if (found == 0x7FFFFFFF) {
      // whole remainder stays in the binade
      if (tid == kFoldThreads - 1) F.cut_sum = incl;
      __syncthreads();
      if (tid == 0) F.S = ldexp(N0 + F.cut_sum, F.e - 52);
      __syncthreads();
      pos = n;
      break;
    }
    // sum of increments strictly before `found`
    {
      double part = 0.0;
      if (a < b && a < found) {
        const int hi = min(b, found);
        for (int k = a; k < hi; ++k) part += F.inc[F.stream[k]];
      }
      double tot = block_scan(F, tid, part);
      if (tid == kFoldThreads - 1) F.cut_sum = tot;
      __syncthreads();
    }
    double Snew = 0.0;
    if (tid == 0) {
      double S = ldexp(N0 + F.cut_sum, F.e - 52);
      S = S + F.t[F.stream[found]];  // the exact IEEE addition the JVM performs
      F.S = S;
    }
    __syncthreads();
    Snew = F.S;
    pos = found + 1;
    fold_set_binade(F, tid, Snew);
  }
}

// Advance over `count` consecutive units (blocks or tiles) whose qual
// histograms are hist(unit) while no unit leaves the binade; returns the index
// of the first unit that would (or count).
template <class H>
__device__ int64_t fold_units(FoldShared& F, int tid, int64_t first, int64_t count, H&& hist) {
  int64_t u = 0;
  while (u < count) {
    const int64_t my = first + u + tid;
    const bool have = (u + tid) < count;
    double d = 0.0;
    bool tie = false;
    if (have) {
      for (int q = 0; q < kQBins; ++q) {
        const uint32_t h = hist(my, q);
        if (h) {
          d += (double)h * F.inc[q];
          tie |= F.tie[q] != 0;
        }
      }
    }
    const double N0 = ldexp(F.S, 52 - F.e);
    const double head = 9007199254740992.0 - N0;
    if (d >= head) d = head;  // saturate: it crosses anyway
    double incl = block_scan(F, tid, d);
    if (tid == 0) F.found = 0x7FFFFFFF;
    __syncthreads();
    if (have && (tie || incl >= head)) atomicMin(&F.found, tid);
    __syncthreads();
    const int found = F.found;
    const int take = (found == 0x7FFFFFFF) ? (int)min((int64_t)kFoldThreads, count - u) : found;
    // commit the units before `found`
    if (take > 0) {
      if (tid == take - 1) F.cut_sum = incl;
      __syncthreads();
      if (tid == 0) F.S = ldexp(N0 + F.cut_sum, F.e - 52);
      __syncthreads();
      // S may have become exactly 2^(e+1) only if a unit reached head; not here
    }
    u += take;
    if (found != 0x7FFFFFFF) return u;
  }
  return count;
}

extern "C" __global__ void __launch_bounds__(kFoldThreads) bqsr_fold_kernel(FoldParams P) {
  __shared__ FoldShared F;
  const int tid = threadIdx.x;
  for (int q = tid; q < kQBins; q += kFoldThreads) F.t[q] = P.pow10[q];
  if (tid == 0) {
    F.S = 0.0;
    F.e = 0;
  }
  __syncthreads();
  // Binade mode needs S >= 2^1: every q >= 1 has t < 1 <= S/2 there, so no
  // tie at that binade except q = 0's (t = 1, a tie only at 2^53); ties are
  // still detected and added one by one, this is only where the fast path
  // starts.
  const double seq_limit = 2.0;
  const int64_t nt = P.rd.n_tiles;
  for (int64_t b = 0; b < P.n_blocks; ++b) {
    const int64_t tb0 = nt * b / P.n_blocks, tb1 = nt * (b + 1) / P.n_blocks;
    if (tb0 == tb1) continue;
    if (F.S >= seq_limit) {
      // whole blocks at once
      const int64_t k = fold_units(F, tid, b, P.n_blocks - b,
                                   [&](int64_t blk, int q) { return P.hq_block[blk * kQBins + q]; });
      b += k;
      if (b >= P.n_blocks) break;
    }
    // block b leaves the binade somewhere (or S is still small): tile level
    const int64_t c0 = nt * b / P.n_blocks, c1 = nt * (b + 1) / P.n_blocks;
    int64_t t = c0;
    while (t < c1) {
      if (F.S >= seq_limit) {
        const int64_t k = fold_units(F, tid, t, c1 - t, [&](int64_t tile, int q) { return (uint32_t)P.h2[tile * kQBins + q]; });
        t += k;
        if (t >= c1) break;
      }
      fold_tile_exact(P.rd, t, F, tid, seq_limit);
      ++t;
    }
  }
  __syncthreads();
  if (tid == 0) P.em_out[0] = F.S;
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
                                                                      double em, const double* pow10, int32_t n_groups,
                                                                      int64_t* grp_obs, int64_t* grp_mm, uint8_t* grp_ok,
                                                                      uint8_t* key_ok, double* a2, uint8_t* rq_ok,
                                                                      FinalOut* out) {
  const int tid = threadIdx.x;
  for (int i = tid; i < n_groups; i += blockDim.x) {
    grp_obs[i] = 0;
    grp_mm[i] = 0;
    grp_ok[i] = 0;
  }
  __syncthreads();
  if (tid == 0) {
    // readgroups = keys.sorted.groupBy((t - 1) / 60) (Java division)
    int64_t go = 0, gm = 0;
    int any = 0;
    for (int k = 0; k < g.K; ++k) {
      key_ok[k] = touched[k] != 0;
      if (!touched[k]) continue;
      any = 1;
      const int r = (k - 1) / kMaxQ;  // C++ division truncates like Java's
      grp_obs[r + 1] += qk_obs[k];
      grp_mm[r + 1] += qk_mm[k];
      grp_ok[r + 1] = 1;
    }
    for (int i = 0; i < n_groups; ++i) {
      go += grp_obs[i];
      gm += grp_mm[i];
    }
    out->g_obs = go;
    out->g_mm = gm;
    out->any_key = any;
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

// errorProbabilityToPhred(p) = javaD2I(-10 * log10(p)) by the threshold table
// (see PhredThresholds in bqsr_capi.cpp): the float estimate is within one of
// the answer, the two double comparisons make it exact.
__device__ __forceinline__ int32_t phred_of(double p, const double* thr_lds, const double* thr, int32_t qmin, int32_t nthr) {
  if (p != p) return 0;  // NaN
  if (p <= 0.0) return p == 0.0 ? 2147483647 : 0;  // log10(0) = -inf; log10(<0) = NaN
  if (p == __builtin_inf()) return (int32_t)0x80000000;
  int E;
  const double mant = frexp(p, &E);
  const float gf = -10.0f * ((float)E + __log2f((float)mant)) * 0.30102999566398120f;
  int n = (int)gf;  // trunc, the candidate
  auto th = [&](int k) -> double {  // thr for Q = k (p <= thr(k)  <=>  Q >= k)
    const int i = k - kThrLdsLo;
    if ((unsigned)i < (unsigned)kThrLdsN) return thr_lds[i];
    const int j = k - qmin;
    if (j < 0) return __builtin_inf();
    if (j >= nthr) return 0.0;
    return thr[j];
  };
  for (int it = 0; it < 4 && p > th(n); ++it) --n;
  for (int it = 0; it < 4 && p <= th(n + 1); ++it) ++n;
  return n;
}

extern "C" __global__ void __launch_bounds__(kBlockThreads) bqsr_apply_kernel(ApplyParams P) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int qw = P.w.qw, C = P.g.C;
  double* w_s1 = (double*)smem;        // [qw][C]
  double* w_d2 = w_s1 + qw * C;        // [qw][21]
  double* thr_l = w_d2 + qw * kCtxSlots;  // [256]
  uint8_t* w_ok = (uint8_t*)(thr_l + kThrLdsN);  // [qw]
  uint32_t* blk_next = (uint32_t*)(w_ok + ((qw + 15) & ~15));
  uintptr_t stage_off = ((uintptr_t)(blk_next + 4) - (uintptr_t)smem + 15) & ~(uintptr_t)15;
  WaveStage* stages = (WaveStage*)(smem + stage_off);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t rq0 = (int64_t)P.w.rg_lo * kQBins + P.w.q_lo;
  for (int i = tid; i < qw * C; i += blockDim.x) {
    const int slot = i / C;
    w_s1[i] = (P.w.rg_lo < P.n_rg && P.w.q_lo + slot < kQBins) ? P.s1[(rq0 + slot) * C + (i - slot * C)] : 0.0;
  }
  for (int i = tid; i < qw * kCtxSlots; i += blockDim.x) {
    const int slot = i / kCtxSlots;
    w_d2[i] = (P.w.rg_lo < P.n_rg && P.w.q_lo + slot < kQBins) ? P.d2[(rq0 + slot) * kCtxSlots + (i - slot * kCtxSlots)]
                                                                : 0.0;
  }
  for (int i = tid; i < kThrLdsN; i += blockDim.x) {
    const int j = i + kThrLdsLo - P.thr_qmin;
    thr_l[i] = (j >= 0 && j < P.thr_n) ? P.thr[j] : 0.0;
  }
  for (int i = tid; i < qw; i += blockDim.x)
    w_ok[i] = (P.w.rg_lo < P.n_rg && P.w.q_lo + i < kQBins) ? P.rq_ok[rq0 + i] : 0;
  const int64_t nt = P.rd.n_tiles;
  const int64_t tb0 = nt * blockIdx.x / gridDim.x, tb1 = nt * (blockIdx.x + 1) / gridDim.x;
  if (tid == 0) blk_next[0] = 0;
  __syncthreads();
  WaveStage& ws = stages[wave];
  const SitesDev no_sites{nullptr, nullptr, nullptr, nullptr, nullptr, 0, 0};
  for (;;) {
    int64_t t;
    {
      uint32_t ti = 0;
      if (lane == 0) ti = atomicAdd(&blk_next[0], 1u);
      ti = __shfl(ti, 0);
      t = tb0 + ti;
    }
    if (t >= tb1) break;
    ReadMeta m;
    ReadAlign a;
    TileInfo T = stage_tile(P.rd, t, ws, lane, m, a, true);
    wave_sync();
    if (lane < T.nr) {
      const uint32_t* cig = T.cig_staged ? ws.cigar + (a.cigar_off - T.cig0) : P.rd.cigar + a.cigar_off;
      const uint8_t* md = T.md_staged ? ws.md + (a.md_off - T.md0) : P.rd.md + a.md_off;
      const uint64_t r = (uint64_t)(T.r0 + lane);
      ReadRow row = prep_read<false>(P.rd, no_sites, r, m, a, (int)(m.slot - T.ts0), cig, md, ws.mmbits, ws.maskbits,
                                     P.err);
      // pass-through reads keep their quality string
      if (!eligible_read(m.flags)) {
        row.fl = 0x100;
        P.out_start[r] = 0;
        P.out_len[r] = (m.flags & BQSR_F_HAS_QUAL) ? m.lq : 0;
      } else {
        P.out_start[r] = row.st;
        P.out_len[r] = (row.fl & kRowActive) ? (uint32_t)(row.en - row.st) : 0;
      }
      ws.rows[lane] = row;
    }
    wave_sync();
    const uint64_t c0 = T.ts0 >> 4, c1 = (T.ts0 + T.nslots + 15) >> 4;
    for (uint64_t c = c0 + lane; c < c1; c += 64) {
      const uint4 qv = *(const uint4*)(P.rd.qual + (c << 4));
      const uint32_t qin[4] = {qv.x, qv.y, qv.z, qv.w};
      uint32_t qo[4] = {qv.x, qv.y, qv.z, qv.w};
      uint32_t keep = 0;  // bit j: byte j of the chunk is written
      int s = (int)((int64_t)(c << 4) - (int64_t)T.ts0);
      int i = find_row(ws.rslot, T.nr, max(s, 0));
      int nexts = ws.rslot[i + 1];
      ReadRow row = ws.rows[i];
      int rs = ws.rslot[i];
      for (int j = 0; j < 16; ++j, ++s) {
        if (s < 0 || s >= T.nslots) continue;
        while (s >= nexts) {
          ++i;
          nexts = ws.rslot[i + 1];
          row = ws.rows[i];
          rs = ws.rslot[i];
        }
        const int o = s - rs;
        const uint32_t qb = (qin[j >> 2] >> ((j & 3) * 8)) & 0xFF;
        uint32_t code;
        if (row.fl == 0x100) {  // pass-through: original char
          if (o >= (int)P.rd.meta[T.r0 + i].lq) continue;
          code = (qb + 33u) & 0xFFu;
        } else {
          if (!(row.fl & (kRowActive | kRowQualCheck)) || o < row.st || o >= row.en) continue;
          const int q = (int)(int8_t)qb;
          const int64_t key = (int64_t)q + (int64_t)kMaxQ * row.rg;
          double p;
          bool ok;
          const int slot = q - P.w.q_lo;
          if ((int)row.rg == P.w.rg_lo && (unsigned)slot < (unsigned)qw) {
            ok = w_ok[slot];
            if (!ok || !(row.fl & kRowActive)) {
              if (!ok) report(P.err, err_key((uint64_t)(T.r0 + i), o, kRankTable, BQSR_ERR_MISSING_KEY));
              continue;
            }
            const bool neg = row.fl & kRowNeg;
            int cyc = neg ? ((int)row.ls - o) : (o + 1);
            if (row.fl & kRowSecond) cyc = -cyc;
            const int ctx = context_of(ws.bases, T.bshift, rs, o, row.st, row.en, neg);
            p = w_s1[slot * C + cyc + P.g.L] + w_d2[slot * kCtxSlots + ctx + 4];
          } else {
            // outside the window: validity as getReadGroupDelta / getQualScoreDelta see it
            const int64_t r = (key - 1) / kMaxQ;
            const bool grp = (r + 1) >= 0 && (r + 1) < P.n_groups && P.grp_ok[r + 1];
            const bool kok = key >= 0 && key < P.g.K && P.key_ok[key];
            if (!grp || !kok) {
              report(P.err, err_key((uint64_t)(T.r0 + i), o, kRankTable, BQSR_ERR_MISSING_KEY));
              continue;
            }
            if (q < 0) {
              report(P.err, err_key((uint64_t)(T.r0 + i), o, kRankTable, BQSR_ERR_QUAL_RANGE));
              continue;
            }
            if (!(row.fl & kRowActive)) continue;
            const bool neg = row.fl & kRowNeg;
            int cyc = neg ? ((int)row.ls - o) : (o + 1);
            if (row.fl & kRowSecond) cyc = -cyc;
            const int ctx = context_of(ws.bases, T.bshift, rs, o, row.st, row.en, neg);
            const int64_t rq = (int64_t)row.rg * kQBins + q;
            p = P.s1[rq * C + cyc + P.g.L] + P.d2[rq * kCtxSlots + ctx + 4];
          }
          const int32_t Q = phred_of(p, thr_l, P.thr, P.thr_qmin, P.thr_n);
          code = ((uint32_t)Q + 33u) & 0xFFFFu;  // (Q + 33).toChar
          if (code > 0xFFu) {
            const unsigned long long k = atomicAdd(P.n_exc, 1ull);
            if ((int64_t)k < P.max_exc) P.exc[k] = ((unsigned long long)((c << 4) + j) << 16) | code;
            code &= 0xFFu;
          }
        }
        qo[j >> 2] = (qo[j >> 2] & ~(0xFFu << ((j & 3) * 8))) | (code << ((j & 3) * 8));
        keep |= 1u << j;
      }
      uint8_t* dst = P.out_qual + (c << 4);
      if (keep == 0xFFFFu) {
        *(uint4*)dst = make_uint4(qo[0], qo[1], qo[2], qo[3]);
      } else if (keep) {
        for (int j = 0; j < 16; ++j)
          if (keep & (1u << j)) dst[j] = (uint8_t)(qo[j >> 2] >> ((j & 3) * 8));
      }
    }
    wave_sync();
  }
}

// --------------------------------------------------------- table merge -----
extern "C" __global__ void bqsr_table_add(int64_t* acc, const int64_t* part, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    acc[i] += part[i];
}

}  // namespace bqsr
