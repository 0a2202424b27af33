// bqsr_oracle.cpp -- TEST INFRASTRUCTURE ONLY.
//
// A plain, per-read / per-base CPU restatement of ADAM's BQSR (fnothaft/adam
// @ 0.6.1-SNAPSHOT), used as the parity oracle for the HIP path and as the
// "port" CPU baseline in bench.py.  Only tests/, __graft_entry__.smoke() and
// bench.py's cpu_baseline leg may load it; the product (adam_amd/) never does.
//
// Every function follows one reference function and cites it.  Paths are
// relative to adam-core/src/main/scala/edu/berkeley/cs/amplab/adam/.
//
// The reference is Scala 2.9.3 / Spark 0.8.1 and cannot be built or run in
// this image (no JVM), so parity is pinned by the reference's own test
// vectors (tests/test_oracle_*.py port ReadCovariatesSuite, RichADAMRecordSuite,
// MdTagSuite, RecalibrateBaseQualitiesSuite, AdamContextSuite) and by the
// hand-derived goldens G1/G2 of SURVEY.md Appendix B (tests/golden/).  The
// JVM's Math.log10 is not reproducible here; errorProbabilityToPhred uses a
// log10 correctly rounded to double (long double log10l, then one rounding),
// see DESIGN.md "Parity".
//
// Build: oracle/Makefile  (g++ -O2 -ffp-contract=off: Java doubles never fuse)

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../include/adam_bqsr.h"

namespace {

constexpr int kMaxReasonableQ = 60;  // RecalUtil.Constants.MAX_REASONABLE_QSCORE, recalibration/RecalUtil.scala:26
constexpr int kCtxSlots = 21;        // BaseContext(2) values -4..16, recalibration/StandardCovariate.scala:84-88

// PhredUtils.phredToErrorProbabilityCache: pow(10.0, -p / 10.0), p in 0..255
// (util/PhredUtils.scala:22-24).  Note -p is an Int, then divided by 10.0.
struct Pow10Cache {
  double v[256];
  Pow10Cache() {
    for (int p = 0; p < 256; ++p) v[p] = std::pow(10.0, (double)(-p) / 10.0);
  }
};
const Pow10Cache& pow10c() {
  static Pow10Cache c;
  return c;
}

// log10 correctly rounded to double (see header note).
double cr_log10(double x) { return (double)log10l((long double)x); }

// Java (int)(double): NaN -> 0, saturating, truncation toward zero (JLS 5.1.3).
int32_t java_d2i(double d) {
  if (std::isnan(d)) return 0;
  if (d >= 2147483647.0) return INT32_MAX;
  if (d <= -2147483648.0) return INT32_MIN;
  return (int32_t)d;
}

// PhredUtils.errorProbabilityToPhred: (-10.0 * log10(p)).toInt (PhredUtils.scala:34-38).
int32_t error_prob_to_phred(double p) { return java_d2i(-10.0 * cr_log10(p)); }

struct Dims {
  int64_t K, C, X, L;
  explicit Dims(bqsr_dims d) : K(60LL * (d.n_rg - 1) + 128), C(2LL * d.max_len + 1), X(kCtxSlots), L(d.max_len) {}
  int64_t cells() const { return C + X; }
  int64_t words() const { return K + 2 * K * cells(); }
};

struct Fail {
  int code;
};

// ---- CIGAR / reference positions -------------------------------------------

inline int cig_op(uint32_t e) { return (int)(e & 0xF); }
inline uint32_t cig_len(uint32_t e) { return e >> 4; }
inline bool consumes_ref(int op) {  // samtools CigarOperator.consumesReferenceBases
  return op == BQSR_CIGAR_M || op == BQSR_CIGAR_D || op == BQSR_CIGAR_N || op == BQSR_CIGAR_EQ || op == BQSR_CIGAR_X;
}

// Option[Long] as (valid, value).
struct OptPos {
  bool some;
  int64_t v;
};

// RichADAMRecord.referencePositions (rich/RichADAMRecord.scala:156-187) with
// unclippedStart (:101-109): fold from start - sum(leading S/H lengths); M/X/=/S
// emit Range(pos.toInt, pos.toInt + len) (Int arithmetic, `.last` throws on an
// empty range); H emits nothing; D/P/N advance; I emits None.
void reference_positions(const uint32_t* cig, size_t n, int64_t start, std::vector<OptPos>& out) {
  out.clear();
  int64_t pos = start;
  for (size_t i = 0; i < n; ++i) {  // unclippedStart: takeWhile(isClipped)
    int op = cig_op(cig[i]);
    if (op != BQSR_CIGAR_S && op != BQSR_CIGAR_H) break;
    pos -= cig_len(cig[i]);
  }
  for (size_t i = 0; i < n; ++i) {
    int op = cig_op(cig[i]);
    uint32_t len = cig_len(cig[i]);
    switch (op) {
      case BQSR_CIGAR_M:
      case BQSR_CIGAR_X:
      case BQSR_CIGAR_EQ:
      case BQSR_CIGAR_S: {
        int32_t a = (int32_t)(uint32_t)(uint64_t)pos;             // posAtCigar.toInt
        int32_t b = (int32_t)((uint32_t)a + len);                  // Int addition (wraps)
        if (len == 0 || b <= a) throw Fail{BQSR_ERR_CIGAR_INVALID};  // empty Range: positions.last
        for (int32_t t = a; t != b; ++t) out.push_back({true, (int64_t)t});
        pos = (int64_t)(int32_t)((uint32_t)b - 1u + 1u);           // positions.last + 1 (Int)
        break;
      }
      case BQSR_CIGAR_H:
        break;
      case BQSR_CIGAR_D:
      case BQSR_CIGAR_P:
      case BQSR_CIGAR_N:
        pos += len;
        break;
      case BQSR_CIGAR_I:
        for (uint32_t t = 0; t < len; ++t) out.push_back({false, 0});
        break;
      default:
        throw Fail{BQSR_ERR_CIGAR_INVALID};
    }
  }
}

// RichADAMRecord.end (RichADAMRecord.scala:77-87): start + sum of reference-consuming lengths.
int64_t reference_end(const uint32_t* cig, size_t n, int64_t start) {
  int64_t e = start;
  for (size_t i = 0; i < n; ++i)
    if (consumes_ref(cig_op(cig[i]))) e += cig_len(cig[i]);
  return e;
}

// ---- MD tag -----------------------------------------------------------------

// MdTag.apply(String, Long) (util/MdTag.scala:38-98): keeps only the match
// ranges (isMatch, :247-249 tests membership in any of them).
struct MdRuns {
  std::vector<std::pair<int64_t, int64_t>> runs;  // [lo, hi)
  bool is_match(int64_t p) const {
    for (auto& r : runs)
      if (p >= r.first && p < r.second) return true;
    return false;
  }
};

bool md_base_char(uint8_t c) {  // basesPattern "[AaGgCcTtNnUuKkMmRrSsWwBbVvHhDdXxYy]" after toUpperCase
  if (c >= 'a' && c <= 'z') c = (uint8_t)(c - 32);
  switch (c) {
    case 'A': case 'G': case 'C': case 'T': case 'N': case 'U': case 'K': case 'M': case 'R':
    case 'S': case 'W': case 'B': case 'V': case 'H': case 'D': case 'X': case 'Y':
      return true;
    default:
      return false;
  }
}

void parse_md(const uint8_t* s, size_t n, int64_t ref_start, MdRuns& out) {
  out.runs.clear();
  if (n == 0) return;  // "" parses to an MdTag with no runs (MdTagSuite "zero length md tag")
  size_t off = 0;
  int64_t pos = ref_start;
  auto read_matches = [&]() {  // digitPattern.findPrefixOf + s.toInt (Integer.parseInt, overflow throws)
    size_t b = off;
    int64_t v = 0;
    while (off < n && s[off] >= '0' && s[off] <= '9') {
      v = v * 10 + (s[off] - '0');
      if (v > INT32_MAX) throw Fail{BQSR_ERR_MD_PARSE};  // NumberFormatException <: IllegalArgumentException
      ++off;
    }
    if (off == b) throw Fail{BQSR_ERR_MD_PARSE};
    if (v > 0) out.runs.push_back({pos, pos + v});
    pos += v;
  };
  read_matches();
  while (off < n) {
    if (s[off] == '^') ++off;  // deletion; positions advance exactly like mismatches
    size_t b = off;
    while (off < n && md_base_char(s[off])) ++off;
    if (off == b) throw Fail{BQSR_ERR_MD_PARSE};
    pos += (int64_t)(off - b);
    read_matches();
  }
}

// ---- known sites --------------------------------------------------------------

struct Sites {
  std::vector<std::vector<int64_t>> pos;  // sorted unique per contig
  bool contains(int32_t contig, int64_t p) const {
    if (contig < 0 || contig >= (int32_t)pos.size()) return false;  // unknown contig: caught -> false
    auto& v = pos[contig];
    return std::binary_search(v.begin(), v.end(), p);
  }
};

// ---- per-read covariates -----------------------------------------------------

int base_idx(uint8_t b) {  // BASES.indexOf (StandardCovariate.scala:54,89)
  switch (b) {
    case 'A': return 0;
    case 'C': return 1;
    case 'G': return 2;
    case 'T': return 3;
    default: return -1;
  }
}
uint8_t compl_base(uint8_t b) {  // COMPL_MP (StandardCovariate.scala:55-57)
  switch (b) {
    case 'A': return 'T';
    case 'C': return 'G';
    case 'G': return 'C';
    case 'T': return 'A';
    case 'N': return 'N';
    default: throw Fail{BQSR_ERR_BAD_REVCOMP_BASE};
  }
}
// BaseContext.encode of a sliding window (StandardCovariate.scala:86-90); a
// window can be the partial last window of length 1 (Scala sliding semantics).
int encode_window(const uint8_t* w, size_t n) {
  for (size_t i = 0; i < n; ++i)
    if (w[i] == 'N') return 0;
  int acc = base_idx(w[0]);
  for (size_t i = 1; i < n; ++i) acc = acc * 4 + base_idx(w[i]);
  return 1 + acc;
}
// BaseContext.getContext (StandardCovariate.scala:81-84): (1 to size-1).map(0) ++ bases.sliding(2).map(encode)
void get_context(const uint8_t* b, size_t n, std::vector<int>& out) {
  out.assign(1, 0);
  if (n == 1) out.push_back(encode_window(b, 1));
  for (size_t i = 1; i < n; ++i) out.push_back(encode_window(b + i - 1, 2));
}

struct ReadView {
  const bqsr_records* R;
  int64_t r;
  uint32_t flags;
  bool has(uint32_t f) const { return (flags & f) != 0; }
  const uint8_t* qual() const { return R->qual + R->qual_offset[r]; }
  size_t lq() const { return (size_t)(R->qual_offset[r + 1] - R->qual_offset[r]); }
  const uint8_t* seq() const { return R->seq + R->seq_offset[r]; }
  size_t ls() const { return (size_t)(R->seq_offset[r + 1] - R->seq_offset[r]); }
  const uint32_t* cig() const { return R->cigar + R->cigar_offset[r]; }
  size_t ncig() const { return (size_t)(R->cigar_offset[r + 1] - R->cigar_offset[r]); }
  const uint8_t* md() const { return R->md + R->md_offset[r]; }
  size_t nmd() const { return (size_t)(R->md_offset[r + 1] - R->md_offset[r]); }
};

struct BaseCov {  // BaseCovariates (recalibration/ReadCovariates.scala:64)
  int32_t qual_by_rg;
  int32_t cycle;
  int32_t context;
  int8_t qual;
  bool is_mismatch;
  bool is_masked;
};

// ReadCovariates (recalibration/ReadCovariates.scala:30-60): the eager
// constructor (quality trimming, QualByRG, DiscreteCycle, BaseContext) plus
// iteration of `next`.  Calls f(BaseCov) per base; throws Fail on the first
// exception the reference would raise for this read.
template <class F>
void read_covariates(const ReadView& rv, const Sites* snp, std::vector<OptPos>& rp, MdRuns& md,
                     std::vector<int>& ctx, std::vector<uint8_t>& rc, F&& f) {
  // RichADAMRecord.qualityScores (RichADAMRecord.scala:43): (char - 33).toByte
  if (!rv.has(BQSR_F_HAS_QUAL)) throw Fail{BQSR_ERR_NULL_FIELD};
  const size_t lq = rv.lq();
  const uint8_t* qc = rv.qual();
  auto qs = [&](size_t i) -> int8_t { return (int8_t)(uint8_t)(qc[i] - 33); };
  // qualityStartOffset / qualityEndOffset, minQuality = 2 (ReadCovariates.scala:31-39)
  size_t st = 0;
  while (st < lq && qs(st) <= 2) ++st;
  size_t tail = 0;
  while (tail < lq && qs(lq - 1 - tail) <= 2) ++tail;
  const int64_t end = (int64_t)lq - (int64_t)tail;
  // QualByRG (StandardCovariate.scala:25-32): 60 * getRecordGroupId (NPE when null)
  if (!rv.has(BQSR_F_HAS_RG)) throw Fail{BQSR_ERR_NULL_RG};
  const int64_t rg_off = (int64_t)kMaxReasonableQ * rv.R->rg_id[rv.r];
  // DiscreteCycle (StandardCovariate.scala:39-48): getSequence.toString.size
  if (!rv.has(BQSR_F_HAS_SEQ)) throw Fail{BQSR_ERR_NULL_FIELD};
  const int64_t ls = (int64_t)rv.ls();
  const bool neg = rv.has(BQSR_F_NEG_STRAND);
  const bool second = rv.has(BQSR_F_PAIRED) && rv.has(BQSR_F_SECOND_OF_PAIR);
  const int64_t c_lo = std::min<int64_t>((int64_t)st, ls), c_hi = std::min<int64_t>(end, ls);
  const int64_t cyc_len = std::max<int64_t>(0, c_hi - c_lo);  // cycles.slice(st, end)
  // BaseContext(2) (StandardCovariate.scala:59-79)
  const uint8_t* s = rv.seq();
  if (neg) {
    rc.resize((size_t)ls);
    for (int64_t i = 0; i < ls; ++i) rc[(size_t)i] = compl_base(s[ls - 1 - i]);  // simpleReverseComplement
    int64_t lo = std::max<int64_t>(0, ls - end), hi = std::min<int64_t>(ls, ls - (int64_t)st);
    get_context(rc.data() + lo, (size_t)std::max<int64_t>(0, hi - lo), ctx);
  } else {
    int64_t lo = std::min<int64_t>((int64_t)st, ls), hi = std::min<int64_t>(end, ls);
    get_context(s + lo, (size_t)std::max<int64_t>(0, hi - lo), ctx);
  }
  bool rp_done = false, md_done = false;
  int64_t ref_end = 0;
  for (int64_t o = (int64_t)st; o < end; ++o) {
    const int64_t k = o - (int64_t)st;
    // RichADAMRecord.isMismatchAtReadOffset (RichADAMRecord.scala:147-154)
    if (!rp_done) {
      if (!rv.has(BQSR_F_HAS_CIGAR) || !rv.has(BQSR_F_HAS_START)) throw Fail{BQSR_ERR_NULL_FIELD};
      reference_positions(rv.cig(), rv.ncig(), rv.R->start[rv.r], rp);
      ref_end = reference_end(rv.cig(), rv.ncig(), rv.R->start[rv.r]);
      rp_done = true;
    }
    // both isMismatchAtReadOffset (non-empty list) and SnpTable's
    // readOffsetToReferencePosition index the List: IndexOutOfBounds past its end
    if ((size_t)o >= rp.size()) throw Fail{BQSR_ERR_CIGAR_SHORT};
    const OptPos ref = rp[(size_t)o];
    int mism = -1;  // None
    if (ref.some) {
      // isMismatchAtReferencePosition (:138-144): mdEvent first (lazy parse), then overlap
      if (rv.has(BQSR_F_HAS_MD)) {
        if (!md_done) {
          parse_md(rv.md(), rv.nmd(), rv.R->start[rv.r], md);
          md_done = true;
        }
        const int64_t st_ref = rv.R->start[rv.r];
        if (st_ref <= ref.v && ref.v < ref_end) mism = md.is_match(ref.v) ? 0 : 1;
      }
    }
    // SnpTable.isMaskedAtReadOffset (models/SnpTable.scala:15-23), evaluated first in `||`
    bool masked;
    if (!ref.some) {
      masked = true;
    } else {
      if (!rv.has(BQSR_F_HAS_REFNAME)) throw Fail{BQSR_ERR_NULL_FIELD};
      masked = snp != nullptr && snp->contains(rv.R->contig_id[rv.r], ref.v);
    }
    masked = masked || mism < 0;
    const int8_t q = qs((size_t)o);
    // new BaseCovariates(qualCovar(k), requestedCovars.map(v => v(k)), ...)
    if (k >= cyc_len) throw Fail{BQSR_ERR_SEQ_SHORT};
    int64_t cyc = neg ? (ls - o) : (o + 1);
    if (second) cyc = -cyc;
    if (k >= (int64_t)ctx.size()) throw Fail{BQSR_ERR_SEQ_SHORT};
    BaseCov b;
    b.qual_by_rg = (int32_t)((int64_t)q + rg_off);
    b.cycle = (int32_t)cyc;
    b.context = ctx[(size_t)k];
    b.qual = q;
    b.is_mismatch = mism == 1;
    b.is_masked = masked;
    f(b);
  }
}

struct Table {  // dense RecalTable: [touched K][obs K*(C+X)][mm K*(C+X)]
  Dims d;
  int64_t* w;
  int64_t* touched() { return w; }
  int64_t* obs() { return w + d.K; }
  int64_t* mm() { return w + d.K + d.K * d.cells(); }
  int64_t cyc_cell(int64_t key, int64_t cyc) const { return key * d.cells() + (cyc + d.L); }
  int64_t ctx_cell(int64_t key, int64_t ctx) const { return key * d.cells() + d.C + (ctx + 4); }
};

}  // namespace

extern "C" {

double oracle_pow10cache(int q) { return pow10c().v[q & 255]; }
double oracle_log10(double x) { return cr_log10(x); }
int32_t oracle_error_prob_to_phred(double p) { return error_prob_to_phred(p); }
int64_t oracle_table_words(bqsr_dims d) { return Dims(d).words(); }

// Opaque known-site table (SnpTable.apply(File), SnpTable.scala:32-47).
void* oracle_sites_create(const int64_t* const* pos, const uint64_t* n, int32_t n_contigs) {
  Sites* s = new Sites;
  s->pos.resize((size_t)n_contigs);
  for (int32_t c = 0; c < n_contigs; ++c) {
    s->pos[(size_t)c].assign(pos[c], pos[c] + n[c]);
    std::sort(s->pos[(size_t)c].begin(), s->pos[(size_t)c].end());
    s->pos[(size_t)c].erase(std::unique(s->pos[(size_t)c].begin(), s->pos[(size_t)c].end()), s->pos[(size_t)c].end());
  }
  return s;
}
void oracle_sites_destroy(void* s) { delete (Sites*)s; }

// usableRead (RecalibrateBaseQualities.scala:29-32)
static bool usable(uint32_t f) {
  return (f & BQSR_F_MAPPED) && (f & BQSR_F_PRIMARY) && !(f & BQSR_F_DUPLICATE) && (f & BQSR_F_HAS_MD);
}

// One partition of computeTable (RecalibrateBaseQualities.scala:52-64):
// rdd.filter(usableRead).map(ReadCovariates(...)).aggregate(new RecalTable)(table + covar, ...)
// foldLeft within the partition, folding into `words` and continuing `*em`
// (the caller starts a partition at 0.0).  RecalTable.+= (RecalTable.scala:55-62):
// lookup touches the key; ErrorCount.+= counts unmasked bases; expectedMismatch
// always adds phredToErrorProbability(qual).
int oracle_observe(const bqsr_records* R, int64_t r0, int64_t r1, const void* sites, bqsr_dims dims,
                   int64_t* words, double* em, int64_t* err_read) {
  Table t{Dims(dims), words};
  const Sites* snp = (const Sites*)sites;
  std::vector<OptPos> rp;
  MdRuns md;
  std::vector<int> ctx;
  std::vector<uint8_t> rc;
  double acc = *em;
  const double* p10 = pow10c().v;
  for (int64_t r = r0; r < r1; ++r) {
    const uint32_t f = R->flags[r];
    if (!usable(f)) continue;
    ReadView rv{R, r, f};
    if ((f & BQSR_F_HAS_SEQ) && (int64_t)rv.ls() > dims.max_len) {
      *err_read = r;
      return BQSR_ERR_INVALID_ARG;
    }
    if ((f & BQSR_F_HAS_RG) && (R->rg_id[r] < 0 || R->rg_id[r] >= dims.n_rg)) {
      *err_read = r;
      return BQSR_ERR_INVALID_ARG;
    }
    try {
      read_covariates(rv, snp, rp, md, ctx, rc, [&](const BaseCov& b) {
        // the table update precedes the failing cache lookup, but the job dies
        // either way; checking first keeps negative keys out of the dense array
        if (b.qual < 0) throw Fail{BQSR_ERR_QUAL_RANGE};  // phredToErrorProbabilityCache(qual)
        t.touched()[b.qual_by_rg] += 1;
        if (!b.is_masked) {
          int64_t c1 = t.cyc_cell(b.qual_by_rg, b.cycle), c2 = t.ctx_cell(b.qual_by_rg, b.context);
          t.obs()[c1] += 1;
          t.obs()[c2] += 1;
          if (b.is_mismatch) {
            t.mm()[c1] += 1;
            t.mm()[c2] += 1;
          }
        }
        acc = acc + p10[b.qual];
      });
    } catch (Fail e) {
      *em = acc;
      *err_read = r;
      return e.code;
    }
  }
  *em = acc;
  return BQSR_OK;
}

// Finalized table (RecalTable.finalizeTable, RecalTable.scala:117-126).
struct OracleFinal {
  bqsr_dims dims;
  std::vector<int64_t> words;
  std::vector<int64_t> qk_obs, qk_mm;  // per key (touched keys only meaningful)
  std::vector<int64_t> rg_obs, rg_mm;  // per group r, index r + 1 (r >= -1)
  std::vector<uint8_t> rg_exists;
  int64_t g_obs = 0, g_mm = 0;
  double avg = 0.0, global_error = 0.0;
};

// ErrorCount.getErrorProb (RecalTable.scala:210-214): None when no observation.
static bool error_prob(int64_t obs, int64_t mm, double* out) {
  if (obs == 0) return false;
  double v = (double)mm / (double)obs;
  const double mre = pow10c().v[kMaxReasonableQ];  // MIN_REASONABLE_ERROR
  *out = std::max(mre, v);                          // math.max
  return true;
}

void* oracle_finalize(bqsr_dims dims, const int64_t* words, double em, int* status) {
  OracleFinal* F = new OracleFinal;
  Dims d(dims);
  F->dims = dims;
  F->words.assign(words, words + d.words());
  Table t{d, F->words.data()};
  F->qk_obs.assign((size_t)d.K, 0);
  F->qk_mm.assign((size_t)d.K, 0);
  const int64_t n_groups = (d.K - 1) / kMaxReasonableQ + 2;
  F->rg_obs.assign((size_t)n_groups, 0);
  F->rg_mm.assign((size_t)n_groups, 0);
  F->rg_exists.assign((size_t)n_groups, 0);
  bool any = false;
  for (int64_t k = 0; k < d.K; ++k) {
    if (t.touched()[k] == 0) continue;
    any = true;
    // qualByRGCounts(k) = counts(k)(0).errorsByVariate.values.reduce(_ ++ _)  (cycle covariate)
    for (int64_t c = 0; c < d.C; ++c) {
      F->qk_obs[(size_t)k] += t.obs()[k * d.cells() + c];
      F->qk_mm[(size_t)k] += t.mm()[k * d.cells() + c];
    }
    // readgroups: groupBy((t - 1) / MAX_REASONABLE_QSCORE) (Java int division)
    int64_t r = (k - 1) / kMaxReasonableQ;
    F->rg_exists[(size_t)(r + 1)] = 1;
    F->rg_obs[(size_t)(r + 1)] += F->qk_obs[(size_t)k];
    F->rg_mm[(size_t)(r + 1)] += F->qk_mm[(size_t)k];
  }
  if (!any) {  // readGroupCounts.values.reduce on an empty collection
    delete F;
    *status = BQSR_ERR_EMPTY_TABLE;
    return nullptr;
  }
  for (size_t i = 0; i < F->rg_obs.size(); ++i) {
    F->g_obs += F->rg_obs[i];
    F->g_mm += F->rg_mm[i];
  }
  F->avg = em / (double)F->g_obs;  // averageReportedError
  double ge;
  F->global_error = error_prob(F->g_obs, F->g_mm, &ge) ? ge : F->avg;
  *status = BQSR_OK;
  return F;
}
void oracle_final_destroy(void* f) { delete (OracleFinal*)f; }
double oracle_final_avg(const void* f) { return ((const OracleFinal*)f)->avg; }
void oracle_final_global(const void* f, int64_t* obs, int64_t* mm) {
  *obs = ((const OracleFinal*)f)->g_obs;
  *mm = ((const OracleFinal*)f)->g_mm;
}
// read-group counts for group r (>= -1); returns 0 when the group does not exist
int oracle_final_group(const void* fp, int32_t r, int64_t* obs, int64_t* mm) {
  const OracleFinal* F = (const OracleFinal*)fp;
  if (r + 1 < 0 || r + 1 >= (int32_t)F->rg_exists.size() || !F->rg_exists[(size_t)(r + 1)]) return 0;
  *obs = F->rg_obs[(size_t)(r + 1)];
  *mm = F->rg_mm[(size_t)(r + 1)];
  return 1;
}

// RecalTable.getErrorRateShifts (RecalTable.scala:128-152) and the fold of
// RecalUtil.recalibrate (RecalUtil.scala:37): returns a status (MISSING_KEY /
// QUAL_RANGE), the four shifts and the new phred score.
static int shifts_for(const OracleFinal* F, int64_t key, int32_t qual, int64_t cyc, int64_t ctx, double sh[4],
                      int32_t* newq) {
  Dims d(F->dims);
  // getReadGroupDelta: readGroupCounts((key - 1) / 60)
  int64_t r = (key - 1) / kMaxReasonableQ;
  if (r + 1 < 0 || r + 1 >= (int64_t)F->rg_exists.size() || !F->rg_exists[(size_t)(r + 1)])
    return BQSR_ERR_MISSING_KEY;
  double v;
  const double avg = F->avg;
  const double rg_delta = (error_prob(F->rg_obs[(size_t)(r + 1)], F->rg_mm[(size_t)(r + 1)], &v) ? v : avg) - avg;
  // getQualScoreDelta: qualByRGCounts(key), then reportedErr = pow10cache(qual)
  if (key < 0 || key >= d.K || F->words[(size_t)key] == 0) return BQSR_ERR_MISSING_KEY;
  if (qual < 0 || qual > 255) return BQSR_ERR_QUAL_RANGE;
  const double e = pow10c().v[qual];
  const double a1 = e + rg_delta;
  const double q_delta = (error_prob(F->qk_obs[(size_t)key], F->qk_mm[(size_t)key], &v) ? v : a1) - a1;
  // getCovariateDelta: errAdjusted = reportedErr + readGroupDelta + qualScoreDelta
  const double a2 = a1 + q_delta;
  const int64_t* obs = F->words.data() + d.K;
  const int64_t* mm = obs + d.K * d.cells();
  const int64_t c1 = key * d.cells() + (cyc + d.L), c2 = key * d.cells() + d.C + (ctx + 4);
  const double cyc_delta = (error_prob(obs[c1], mm[c1], &v) ? v : a2) - a2;
  const double ctx_delta = (error_prob(obs[c2], mm[c2], &v) ? v : a2) - a2;
  sh[0] = rg_delta;
  sh[1] = q_delta;
  sh[2] = cyc_delta;
  sh[3] = ctx_delta;
  // shifts.foldLeft(toErr(qual))(_ + _)
  double p = e;
  for (int i = 0; i < 4; ++i) p = p + sh[i];
  *newq = error_prob_to_phred(p);
  return BQSR_OK;
}

int oracle_shifts(const void* f, int32_t key, int32_t qual, int32_t cyc, int32_t ctx, double* sh, int32_t* newq) {
  const OracleFinal* F = (const OracleFinal*)f;
  Dims d(F->dims);
  if (cyc < -d.L || cyc > d.L || ctx < -4 || ctx > 16) return BQSR_ERR_INVALID_ARG;
  return shifts_for(F, key, qual, cyc, ctx, sh, newq);
}

// One partition of applyTable (RecalibrateBaseQualities.scala:66-76) with
// RecalUtil.recalibrate (RecalUtil.scala:31-42).  Recalibrated reads get
// out_len = end - st chars at out_qual[qual_offset[r]...]; other reads are
// passed through (their qual chars copied, out_len = Lq; a null qual gives 0).
int oracle_apply(const bqsr_records* R, int64_t r0, int64_t r1, const void* fp, uint16_t* out_qual,
                 uint32_t* out_len, int64_t* err_read) {
  const OracleFinal* F = (const OracleFinal*)fp;
  std::vector<OptPos> rp;
  MdRuns md;
  std::vector<int> ctx;
  std::vector<uint8_t> rc;
  for (int64_t r = r0; r < r1; ++r) {
    const uint32_t f = R->flags[r];
    uint16_t* out = out_qual + R->qual_offset[r];
    const bool eligible = (f & BQSR_F_MAPPED) && (f & BQSR_F_PRIMARY) && !(f & BQSR_F_DUPLICATE);
    if (!eligible) {
      size_t lq = (f & BQSR_F_HAS_QUAL) ? (size_t)(R->qual_offset[r + 1] - R->qual_offset[r]) : 0;
      for (size_t i = 0; i < lq; ++i) out[i] = R->qual[R->qual_offset[r] + i];
      out_len[r] = (uint32_t)lq;
      continue;
    }
    ReadView rv{R, r, f};
    if ((f & BQSR_F_HAS_SEQ) && (int64_t)rv.ls() > F->dims.max_len) {
      *err_read = r;
      return BQSR_ERR_INVALID_ARG;
    }
    uint32_t n = 0;
    try {
      // RecalUtil.recalibrate uses ReadCovariates(read, qualByRG, covars) with SnpTable()
      Sites empty;
      read_covariates(rv, &empty, rp, md, ctx, rc, [&](const BaseCov& b) {
        double sh[4];
        int32_t q;
        int st = shifts_for(F, b.qual_by_rg, b.qual, b.cycle, b.context, sh, &q);
        if (st != BQSR_OK) throw Fail{st};
        out[n++] = (uint16_t)(uint32_t)((int32_t)((uint32_t)q + 33u));  // (b + 33).toChar
      });
    } catch (Fail e) {
      *err_read = r;
      return e.code;
    }
    out_len[r] = n;
  }
  return BQSR_OK;
}

// Whole BQSR on `nthreads` std::threads: the CPU baseline ("C++ restatement of
// ADAM BQSR").  Reads are cut into n_parts contiguous partitions (Spark
// partitions); partition i folds from a zero table / 0.0; tables are merged in
// partition order (RecalTable.++, expectedMismatch = acc + part); finalize;
// apply per partition.  Outputs like oracle_apply.  Returns a status;
// *err_read = first failing read of the first failing partition.
// expectedMismatch of reads [r0, r1) as ONE partition's foldLeft from *em
// (RecalTable.scala:61 over ReadCovariates' trimmed ranges of usable reads,
// masked bases included, Q15) -- without the covariates: the sequential part
// of observe, for the single-partition check of the benchmark's job.  Assumes
// error-free input (observe reports errors).
void oracle_em_fold(const bqsr_records* R, int64_t r0, int64_t r1, double* em) {
  const double* p10 = pow10c().v;
  double acc = *em;
  for (int64_t r = r0; r < r1; ++r) {
    const uint32_t f = R->flags[r];
    if (!usable(f) || !(f & BQSR_F_HAS_QUAL)) continue;
    const uint8_t* qc = R->qual + R->qual_offset[r];
    const size_t lq = (size_t)(R->qual_offset[r + 1] - R->qual_offset[r]);
    auto qs = [&](size_t i) -> int8_t { return (int8_t)(uint8_t)(qc[i] - 33); };
    size_t st = 0;
    while (st < lq && qs(st) <= 2) ++st;  // ReadCovariates.scala:31-39
    size_t tail = 0;
    while (tail < lq && qs(lq - 1 - tail) <= 2) ++tail;
    for (size_t o = st; o + tail < lq; ++o) {
      const int8_t q = qs(o);
      if (q < 0) break;  // QUAL_RANGE: observe reports it
      acc = acc + p10[q];
    }
  }
  *em = acc;
}

static int bqsr_impl(const bqsr_records* R, int32_t n_parts, const void* sites, bqsr_dims dims, int32_t nthreads,
                     bool fold1, uint16_t* out_qual, uint32_t* out_len, int64_t* words_out, double* em_out,
                     int64_t* err_read);

int oracle_bqsr(const bqsr_records* R, int32_t n_parts, const void* sites, bqsr_dims dims, int32_t nthreads,
                uint16_t* out_qual, uint32_t* out_len, int64_t* words_out, double* em_out, int64_t* err_read) {
  return bqsr_impl(R, n_parts, sites, dims, nthreads, false, out_qual, out_len, words_out, em_out, err_read);
}

// The same job as ONE partition (the table -- partition-order free -- still
// built by n_parts threads; expectedMismatch folded over all reads in order
// by one more thread running beside them): what one GPU's benchmark job
// computes over its shard.
int oracle_bqsr_fold1(const bqsr_records* R, int32_t n_parts, const void* sites, bqsr_dims dims, int32_t nthreads,
                      uint16_t* out_qual, uint32_t* out_len, int64_t* words_out, double* em_out, int64_t* err_read) {
  return bqsr_impl(R, n_parts, sites, dims, nthreads, true, out_qual, out_len, words_out, em_out, err_read);
}

// Compare the oracle's output (qual_offset layout, Java chars) with the HIP
// apply output in the packed device layout: read r's chars at
// got[slot(r) + got_start[r] ...] (slot = running sum of max(Lq, Ls) rounded
// up to 16 when `aligned`), chars above 0xFF in the (slot << 16 | code) list.
// Returns the number of reads that differ; *first_bad = the first one (-1).
int64_t oracle_compare_device_output(const bqsr_records* R, const uint16_t* ref, const uint32_t* ref_len,
                                     const uint8_t* got, const uint32_t* got_start, const uint32_t* got_len,
                                     const uint64_t* exc, int64_t n_exc, int32_t aligned, int32_t nthreads,
                                     int64_t* first_bad) {
  const int64_t n = R->n_reads;
  std::vector<uint64_t> slot((size_t)n + 1, 0);
  for (int64_t r = 0; r < n; ++r) {
    const uint32_t f = R->flags[r];
    const uint64_t lq = (f & BQSR_F_HAS_QUAL) ? R->qual_offset[r + 1] - R->qual_offset[r] : 0;
    const uint64_t ls = (f & BQSR_F_HAS_SEQ) ? R->seq_offset[r + 1] - R->seq_offset[r] : 0;
    const uint64_t sl = std::max(lq, ls);
    slot[(size_t)r + 1] = slot[(size_t)r] + (aligned ? (sl + 15) / 16 * 16 : sl);
  }
  std::vector<std::pair<uint64_t, uint16_t>> ex;
  for (int64_t i = 0; i < n_exc; ++i) ex.push_back({exc[i] >> 16, (uint16_t)(exc[i] & 0xFFFF)});
  std::sort(ex.begin(), ex.end());
  std::atomic<int64_t> bad{0}, first{INT64_MAX};
  const int nt = std::max(1, nthreads);
  auto work = [&](int t) {
    int64_t b = 0, fb = INT64_MAX;
    for (int64_t r = n * t / nt; r < n * (t + 1) / nt; ++r) {
      bool ok = got_len[r] == ref_len[r];
      const uint16_t* rq = ref + R->qual_offset[r];
      const uint64_t s0 = slot[(size_t)r] + got_start[r];
      for (uint32_t k = 0; ok && k < ref_len[r]; ++k) {
        uint16_t v = got[s0 + k];
        if (rq[k] > 0xFF) {
          auto it = std::lower_bound(ex.begin(), ex.end(), std::make_pair(s0 + k, (uint16_t)0));
          v = (it != ex.end() && it->first == s0 + k) ? it->second : v;
        }
        ok = v == rq[k];
      }
      if (!ok) {
        ++b;
        fb = std::min(fb, r);
      }
    }
    bad += b;
    int64_t cur = first.load();
    while (fb < cur && !first.compare_exchange_weak(cur, fb)) {
    }
  };
  std::vector<std::thread> th;
  for (int t = 0; t < nt; ++t) th.emplace_back(work, t);
  for (auto& x : th) x.join();
  *first_bad = bad.load() ? first.load() : -1;
  return bad.load();
}

// The same check against the compacted form (bqsr_compact_outputs_async):
// read r's chars at got[off[r] .. off[r + 1]), exceptions keyed by position.
int64_t oracle_compare_compact_output(const bqsr_records* R, const uint16_t* ref, const uint32_t* ref_len,
                                      const uint8_t* got, const uint32_t* off, const uint64_t* exc, int64_t n_exc,
                                      int32_t nthreads, int64_t* first_bad) {
  const int64_t n = R->n_reads;
  std::vector<std::pair<uint64_t, uint16_t>> ex;
  for (int64_t i = 0; i < n_exc; ++i) ex.push_back({exc[i] >> 16, (uint16_t)(exc[i] & 0xFFFF)});
  std::sort(ex.begin(), ex.end());
  std::atomic<int64_t> bad{0}, first{INT64_MAX};
  const int nt = std::max(1, nthreads);
  auto work = [&](int t) {
    int64_t b = 0, fb = INT64_MAX;
    for (int64_t r = n * t / nt; r < n * (t + 1) / nt; ++r) {
      bool ok = off[r + 1] - off[r] == ref_len[r];
      const uint16_t* rq = ref + R->qual_offset[r];
      for (uint32_t k = 0; ok && k < ref_len[r]; ++k) {
        const uint64_t p = (uint64_t)off[r] + k;
        uint16_t v = got[p];
        if (rq[k] > 0xFF) {
          auto it = std::lower_bound(ex.begin(), ex.end(), std::make_pair(p, (uint16_t)0));
          v = (it != ex.end() && it->first == p) ? it->second : v;
        }
        ok = v == rq[k];
      }
      if (!ok) {
        ++b;
        fb = std::min(fb, r);
      }
    }
    bad += b;
    int64_t cur = first.load();
    while (fb < cur && !first.compare_exchange_weak(cur, fb)) {
    }
  };
  std::vector<std::thread> th;
  for (int t = 0; t < nt; ++t) th.emplace_back(work, t);
  for (auto& x : th) x.join();
  *first_bad = bad.load() ? first.load() : -1;
  return bad.load();
}

// computeTable over the batch split into n_parts partitions (observe per
// partition on nthreads threads, RecalTable.++ in partition order,
// RecalibrateBaseQualities.scala:52-64).  fold1: expectedMismatch folded as if
// the batch were ONE partition (one more thread, sequential over all reads).
int oracle_observe_mt(const bqsr_records* R, int32_t n_parts, const void* sites, bqsr_dims dims, int32_t nthreads,
                      int32_t fold1, int64_t* words_out, double* em_out, int64_t* err_read) {
  if (n_parts < 1 || nthreads < 1) return BQSR_ERR_INVALID_ARG;
  Dims d(dims);
  const int64_t n = R->n_reads;
  std::vector<int64_t> bounds((size_t)n_parts + 1);
  for (int32_t i = 0; i <= n_parts; ++i) bounds[(size_t)i] = n * i / n_parts;
  std::vector<std::vector<int64_t>> tabs((size_t)n_parts);
  std::vector<double> ems((size_t)n_parts, 0.0);
  std::vector<int> st((size_t)n_parts, BQSR_OK);
  std::vector<int64_t> er((size_t)n_parts, -1);
  std::atomic<int32_t> next{0};
  auto work_obs = [&]() {
    for (int32_t p; (p = next.fetch_add(1)) < n_parts;) {
      tabs[(size_t)p].assign((size_t)d.words(), 0);
      st[(size_t)p] = oracle_observe(R, bounds[(size_t)p], bounds[(size_t)p + 1], sites, dims, tabs[(size_t)p].data(),
                                     &ems[(size_t)p], &er[(size_t)p]);
    }
  };
  std::vector<std::thread> th;
  double em1 = 0.0;
  if (fold1) th.emplace_back([&]() { oracle_em_fold(R, 0, n, &em1); });
  for (int32_t i = 0; i < nthreads; ++i) th.emplace_back(work_obs);
  for (auto& t : th) t.join();
  for (int32_t p = 0; p < n_parts; ++p)
    if (st[(size_t)p] != BQSR_OK) {
      *err_read = er[(size_t)p];
      return st[(size_t)p];
    }
  std::vector<int64_t> acc((size_t)d.words(), 0);
  double em = 0.0;  // new RecalTable: expectedMismatch 0.0, then ++ in partition order
  for (int32_t p = 0; p < n_parts; ++p) {
    for (size_t i = 0; i < acc.size(); ++i) acc[i] += tabs[(size_t)p][i];
    em = em + ems[(size_t)p];
  }
  if (fold1) em = em1;
  if (words_out) std::memcpy(words_out, acc.data(), acc.size() * sizeof(int64_t));
  if (em_out) *em_out = em;
  return BQSR_OK;
}

// finalizeTable of (words, em) then applyTable over the batch, n_parts
// partitions on nthreads threads (RecalibrateBaseQualities.scala:66-76).
// Outputs like oracle_apply.
int oracle_apply_mt(const bqsr_records* R, int32_t n_parts, bqsr_dims dims, int32_t nthreads, const int64_t* words,
                    double em, uint16_t* out_qual, uint32_t* out_len, int64_t* err_read) {
  if (n_parts < 1 || nthreads < 1) return BQSR_ERR_INVALID_ARG;
  const int64_t n = R->n_reads;
  std::vector<int64_t> bounds((size_t)n_parts + 1);
  for (int32_t i = 0; i <= n_parts; ++i) bounds[(size_t)i] = n * i / n_parts;
  std::vector<int> st((size_t)n_parts, BQSR_OK);
  std::vector<int64_t> er((size_t)n_parts, -1);
  int fst;
  void* F = oracle_finalize(dims, words, em, &fst);
  if (!F) return fst;
  std::atomic<int32_t> next{0};
  auto work_apply = [&]() {
    for (int32_t p; (p = next.fetch_add(1)) < n_parts;)
      st[(size_t)p] = oracle_apply(R, bounds[(size_t)p], bounds[(size_t)p + 1], F, out_qual, out_len, &er[(size_t)p]);
  };
  std::vector<std::thread> th;
  for (int32_t i = 0; i < nthreads; ++i) th.emplace_back(work_apply);
  for (auto& t : th) t.join();
  oracle_final_destroy(F);
  for (int32_t p = 0; p < n_parts; ++p)
    if (st[(size_t)p] != BQSR_OK) {
      *err_read = er[(size_t)p];
      return st[(size_t)p];
    }
  return BQSR_OK;
}

static int bqsr_impl(const bqsr_records* R, int32_t n_parts, const void* sites, bqsr_dims dims, int32_t nthreads,
                     bool fold1, uint16_t* out_qual, uint32_t* out_len, int64_t* words_out, double* em_out,
                     int64_t* err_read) {
  if (n_parts < 1 || nthreads < 1) return BQSR_ERR_INVALID_ARG;
  std::vector<int64_t> acc((size_t)Dims(dims).words(), 0);
  double em = 0.0;
  int st = oracle_observe_mt(R, n_parts, sites, dims, nthreads, fold1 ? 1 : 0, acc.data(), &em, err_read);
  if (st != BQSR_OK) return st;
  if (words_out) std::memcpy(words_out, acc.data(), acc.size() * sizeof(int64_t));
  if (em_out) *em_out = em;
  return oracle_apply_mt(R, n_parts, dims, nthreads, acc.data(), em, out_qual, out_len, err_read);
}

// Exposed for the reference-suite ports (RichADAMRecordSuite / MdTagSuite).
// Returns count of positions written (or -code on error); pos_out[i] = value
// or INT64_MIN for None.
int64_t oracle_reference_positions(const uint32_t* cig, uint64_t n, int64_t start, int64_t* pos_out, int64_t cap) {
  std::vector<OptPos> rp;
  try {
    reference_positions(cig, (size_t)n, start, rp);
  } catch (Fail e) {
    return -e.code;
  }
  for (size_t i = 0; i < rp.size() && (int64_t)i < cap; ++i) pos_out[i] = rp[i].some ? rp[i].v : INT64_MIN;
  return (int64_t)rp.size();
}
int64_t oracle_reference_end(const uint32_t* cig, uint64_t n, int64_t start) { return reference_end(cig, (size_t)n, start); }
// MD: returns number of runs (or -code); runs_out = [lo, hi) pairs
int64_t oracle_md_runs(const uint8_t* s, uint64_t n, int64_t ref_start, int64_t* runs_out, int64_t cap) {
  MdRuns md;
  try {
    parse_md(s, (size_t)n, ref_start, md);
  } catch (Fail e) {
    return -e.code;
  }
  for (size_t i = 0; i < md.runs.size() && (int64_t)(2 * i + 1) < cap; ++i) {
    runs_out[2 * i] = md.runs[i].first;
    runs_out[2 * i + 1] = md.runs[i].second;
  }
  return (int64_t)md.runs.size();
}

// Per-base covariates of one read (ReadCovariates iteration), for the
// ReadCovariatesSuite port: writes up to cap entries of
// {qual_by_rg, cycle, context, qual, is_mismatch, is_masked} (6 int32 each).
int64_t oracle_read_covariates(const bqsr_records* R, int64_t r, const void* sites, int32_t* out, int64_t cap) {
  std::vector<OptPos> rp;
  MdRuns md;
  std::vector<int> ctx;
  std::vector<uint8_t> rc;
  int64_t n = 0;
  try {
    read_covariates(ReadView{R, r, R->flags[r]}, (const Sites*)sites, rp, md, ctx, rc, [&](const BaseCov& b) {
      if (n < cap) {
        int32_t* o = out + 6 * n;
        o[0] = b.qual_by_rg;
        o[1] = b.cycle;
        o[2] = b.context;
        o[3] = b.qual;
        o[4] = b.is_mismatch;
        o[5] = b.is_masked;
      }
      ++n;
    });
  } catch (Fail e) {
    return -e.code;
  }
  return n;
}

}  // extern "C"
