// ADAMRecord columns from a parse's SAM lines (`transform`
// ends in adamSave, adam-cli/.../cli/Transform.scala:95-96 ->
// core/rdd/AdamRDDFunctions.scala:37-56, of records built by
// core/converters/SAMRecordConverter.scala:26-144).
//
// After bqsr_sam_rewrite_quals the parse's device text holds every record's
// line with its recalibrated QUAL (UTF-8) and MarkDuplicates' FLAG, so the
// ADAMRecord fields are a function of the text alone: a thread per record
// splits its line and writes the Arrow buffers of the record-level columns
// -- six strings (offsets + bytes + validity bits), six integers, eleven
// flags as bitmaps.  Columns that are a function of the read group or of the
// @SQ entry only (recordGroup*, reference{Length,Url}, the names) are taken
// from the header by index on the host.  Two passes: lengths (with every
// fixed-width column and bitmap), a scan, the bytes.
//
// Included by bqsr_capi.cpp after sam_ingest.hip / bam_ingest.hip.

namespace adamk {

constexpr int kStr = 6;    // readName, sequence, cigar, qual, mismatchingPositions, attributes
constexpr int kI32 = 4;    // referenceId, mapq, mateReferenceId, recordGroupId
constexpr int kI64 = 2;    // start, mateAlignmentStart
constexpr int kBools = 11; // readPaired .. duplicateRead (adam.avdl order)
constexpr int kMaxTags = 48;

// error word: (read << 8) | code, the smallest wins
enum : uint32_t {
  kAdamOk = 0,
  kAdamTagType = 1,   // an H or B tag: AttributeUtils.convertSAMTagAndValue casts its array to
                      // Array[java.lang.Byte] -- ClassCastException in the reference
  kAdamIntRange = 2,  // an 'i' value outside Int: a Long, which convertSAMTagAndValue does not match
  kAdamTagValue = 3,  // an 'i' / 'f' value that does not parse (htsjdk's TextTagCodec throws)
  kAdamTags = 4,      // more than kMaxTags tags on one record (not supported here)
};

struct AdamParams {
  const uint8_t* text;
  const uint64_t* line_span;  // [2 n_all]: line start, end (no newline)
  const uint64_t* cig_off;    // the parse's CIGAR elements (getCigarString re-encodes them)
  const uint32_t* cig;
  int64_t r0, n;              // records [r0, r0 + n)
  samk::NameTable sq, rg;
  uint64_t* len;              // [kStr][n] string bytes (pass 1)
  const uint64_t* off;        // [kStr][n + 1] exclusive scans (pass 2)
  int32_t* soff;              // [kStr][n + 1] Arrow offsets (pass 2)
  uint8_t* sbytes[kStr];      // string bytes (pass 2)
  uint64_t* svalid;           // [kStr][W] validity bitmaps, W = n / 64 + 1
  int32_t* i32;               // [kI32][n]
  int64_t* i64;               // [kI64][n]
  uint64_t* ivalid;           // [kI32 + kI64][W] referenceId, mapq, mateReferenceId, recordGroupId, start, mateAlignmentStart
  uint64_t* bools;            // [kBools][W]
  int64_t W;
  unsigned long long* err;
  // the apply's outputs in place of the text's QUAL (bqsr_sam_adam_set_quals;
  // out_qual null: the text's), and MarkDuplicates' bits in place of FLAG 0x400
  const ReadMeta* meta;
  const ReadInfo* info;
  const uint8_t* out_qual;
  const uint32_t* out_start;
  const uint32_t* out_len;
  const uint64_t* exc;  // sorted (slot << 16 | char)
  int64_t n_exc;
  const uint32_t* dup_flags;
};

// the recalibrated char at slot (u8 column, exceptions above 0xFF)
__device__ __forceinline__ uint32_t apply_char(const AdamParams& P, uint64_t slot) {
  uint32_t c = P.out_qual[slot];
  int64_t lo = 0, hi = P.n_exc - 1;
  while (lo <= hi) {
    const int64_t mid = (lo + hi) >> 1;
    const uint64_t v = P.exc[mid], s = v >> 16;
    if (s == slot) return (uint32_t)(v & 0xFFFFull);
    if (s < slot) lo = mid + 1;
    else hi = mid - 1;
  }
  return c;
}
// record r's QUAL from the apply (not a pass-through read)
__device__ __forceinline__ bool new_qual(const AdamParams& P, int64_t r) {
  return P.out_qual && !(P.info[r].fl & kInfoPass);
}

__device__ __forceinline__ void adam_error(const AdamParams& P, int64_t i, uint32_t code) {
  atomicMin(P.err, (unsigned long long)(((uint64_t)i << 8) | code));
}

// Long.valueOf of t[a, b): optional sign, decimal digits
__device__ bool parse_long(const uint8_t* t, int64_t a, int64_t b, int64_t* v) {
  bool neg = false;
  if (a < b && (t[a] == '+' || t[a] == '-')) {
    neg = t[a] == '-';
    ++a;
  }
  if (a >= b || b - a > 18) return false;
  int64_t x = 0;
  for (int64_t i = a; i < b; ++i) {
    if (t[i] < '0' || t[i] > '9') return false;
    x = x * 10 + (t[i] - '0');
  }
  *v = neg ? -x : x;
  return true;
}

struct Tag {
  uint32_t id;      // htsjdk's binary tag: second char << 8 | first char
  int64_t a, b;     // the value's bytes
  uint8_t type;
};

// The attributes string: SAMRecordConverter.scala:110-121 folds
// getAttributes -- htsjdk keeps them sorted by binary tag, a repeated tag
// replacing the earlier value -- into `tags ::= attr` (so, descending) and
// joins Attribute.toString ("%s:%s:%s", tag, type abbreviation, value) with
// tabs; MD is left out (mismatchingPositions).  Returns the byte count
// (out == nullptr: count only), or -1 with *code set.
__device__ int64_t attributes_text(const uint8_t* t, const Tag* tg, int nt, uint8_t* out, uint32_t* code) {
  int64_t n = 0;
  auto put = [&](uint8_t c) {
    if (out) out[n] = c;
    ++n;
  };
  bool first = true;
  for (int k = nt - 1; k >= 0; --k) {
    const Tag& g = tg[k];
    if (g.id == ((uint32_t)'D' << 8 | 'M')) continue;
    if (!first) put('\t');
    first = false;
    put((uint8_t)(g.id & 0xFF));
    put((uint8_t)(g.id >> 8));
    put(':');
    switch (g.type) {
      case 'A':
      case 'Z':
        put(g.type);
        put(':');
        for (int64_t i = g.a; i < g.b; ++i) put(t[i]);
        break;
      case 'i': {
        int64_t v;
        if (!parse_long(t, g.a, g.b, &v)) {
          *code = kAdamTagValue;
          return -1;
        }
        if (v < INT32_MIN || v > INT32_MAX) {
          *code = kAdamIntRange;
          return -1;
        }
        put('i');
        put(':');
        bamk::Put p{out ? out + n : nullptr, 0};
        p.integer(v);
        n += p.n;
        break;
      }
      case 'f': {
        float f;
        if (!samk::java_parse_float(t, g.a, g.b, &f)) {
          *code = kAdamTagValue;
          return -1;
        }
        put('f');
        put(':');
        n += samk::java_float_text(f, out ? out + n : nullptr);
        break;
      }
      default:
        *code = kAdamTagType;
        return -1;
    }
  }
  return n;
}

// getCigarString: the elements re-encoded (TextCigarCodec.encode), "*" when none
__device__ int64_t cigar_text(const uint32_t* e, int64_t ne, uint8_t* out) {
  if (ne == 0) {
    if (out) out[0] = '*';
    return 1;
  }
  const char kOps[] = "MIDNSHP=X";
  bamk::Put p{out, 0};
  for (int64_t k = 0; k < ne; ++k) {
    p.integer(e[k] >> 4);
    p.c((e[k] & 15u) < 9u ? (uint8_t)kOps[e[k] & 15u] : (uint8_t)'?');
  }
  return p.n;
}

struct AdamRec {
  int64_t sa[kStr], sb[kStr];  // string spans in the text (attributes / cigar: formatted instead)
  bool sv[kStr];
  int64_t attr_n, cig_n;
  int32_t i32[kI32];
  int64_t i64[kI64];
  bool iv[kI32 + kI64];
  uint32_t flag;
  int nt;
  uint32_t code;
};

// fields of record r (index in the parse); tags into tg (sorted, deduplicated)
__device__ void adam_record(const AdamParams& P, int64_t r, AdamRec& x, Tag* tg) {
  const uint8_t* t = P.text;
  const int64_t s = (int64_t)P.line_span[2 * r], e = (int64_t)P.line_span[2 * r + 1];
  int64_t fa[11], fb[11];
  int64_t p = s;
  for (int f = 0; f < 11; ++f) {
    fa[f] = p;
    while (p < e && t[p] != '\t') ++p;
    fb[f] = p;
    if (p < e) ++p;
  }
  bool more = fb[10] < e;
  // tags: htsjdk's sorted list (insertion by binary tag, a repeat replacing)
  x.nt = 0;
  x.code = kAdamOk;
  int64_t md_a = -1, md_b = -1, rg_a = -1, rg_b = -1;
  while (more) {
    const int64_t ta = p;
    while (p < e && t[p] != '\t') ++p;
    const int64_t tb = p;
    more = p < e;
    if (more) ++p;
    if (tb - ta < 5 || t[ta + 2] != ':' || t[ta + 4] != ':') {  // htsjdk: a two-char tag and a one-char type
      x.code = kAdamTagValue;
      continue;
    }
    Tag g{(uint32_t)t[ta] | ((uint32_t)t[ta + 1] << 8), ta + 5, tb, t[ta + 3]};  // "TG:T:value"
    if (g.id == ((uint32_t)'D' << 8 | 'M')) {
      md_a = g.a;
      md_b = g.b;
    } else if (g.id == ((uint32_t)'G' << 8 | 'R')) {
      rg_a = g.a;
      rg_b = g.b;
    }
    int k = 0;
    while (k < x.nt && tg[k].id < g.id) ++k;
    if (k < x.nt && tg[k].id == g.id) {
      tg[k] = g;
    } else if (x.nt == kMaxTags) {
      x.code = kAdamTags;
    } else {
      for (int j = x.nt; j > k; --j) tg[j] = tg[j - 1];
      tg[k] = g;
      ++x.nt;
    }
  }
  int64_t flag = 0, pos = 0, mapq = 255, pnext = 0;
  (void)samk::parse_int(t, fa[1], fb[1], &flag);  // (the parse accepted FLAG; POS when the reference is known)
  x.flag = (uint32_t)flag;
  if (P.dup_flags)  // FLAG 0x400 following duplicateRead, as bqsr_sam_rewrite_quals writes it
    x.flag = (P.dup_flags[r] & BQSR_F_DUPLICATE) ? (x.flag | 0x400u) : (x.flag & ~0x400u);
  int32_t sq = -1;
  if (!(fb[2] - fa[2] == 1 && t[fa[2]] == '*')) sq = samk::name_lookup(P.sq, t + fa[2], fb[2] - fa[2]);
  // referenceId / referenceName / start / mapq only when the read has a reference (:36-54)
  x.i32[0] = sq;
  x.iv[0] = sq >= 0;
  const bool has_pos = sq >= 0 && samk::parse_int(t, fa[3], fb[3], &pos) && pos != 0;
  x.i64[0] = has_pos ? pos - 1 : 0;
  x.iv[4] = has_pos;
  const bool has_mapq = sq >= 0 && samk::parse_int(t, fa[4], fb[4], &mapq) && mapq != 255;
  x.i32[1] = has_mapq ? (int32_t)mapq : 0;
  x.iv[1] = has_mapq;
  // the mate (:56-71): RNEXT "=" is RNAME's reference
  int32_t msq = -1;
  if (fb[6] - fa[6] == 1 && t[fa[6]] == '=') msq = sq;
  else if (!(fb[6] - fa[6] == 1 && t[fa[6]] == '*')) msq = samk::name_lookup(P.sq, t + fa[6], fb[6] - fa[6]);
  x.i32[2] = msq;
  x.iv[2] = msq >= 0;
  const bool has_mpos = msq >= 0 && samk::parse_int(t, fa[7], fb[7], &pnext) && pnext > 0;
  x.i64[1] = has_mpos ? pnext - 1 : 0;
  x.iv[5] = has_mpos;
  const int32_t rg = rg_a >= 0 ? samk::name_lookup(P.rg, t + rg_a, rg_b - rg_a) : -1;
  x.i32[3] = rg;
  x.iv[3] = rg >= 0;
  // strings: readName, sequence, cigar, qual, mismatchingPositions, attributes
  const int fi[4] = {0, 9, 5, 10};
  for (int c = 0; c < 4; ++c) {
    x.sa[c] = fa[fi[c]];
    x.sb[c] = fb[fi[c]];
    x.sv[c] = true;
  }
  x.sa[4] = md_a;
  x.sb[4] = md_b;
  x.sv[4] = md_a >= 0;
  x.sa[5] = x.sb[5] = 0;
  x.sv[5] = true;  // getAttributes is never null: "" without tags
  x.cig_n = cigar_text(P.cig + P.cig_off[r], (int64_t)(P.cig_off[r + 1] - P.cig_off[r]), nullptr);
  x.attr_n = 0;
  if (x.code == kAdamOk) {
    uint32_t code = kAdamOk;
    x.attr_n = attributes_text(t, tg, x.nt, nullptr, &code);
    if (x.attr_n < 0) {
      x.code = code;
      x.attr_n = 0;
    }
  }
}

// SAMRecordConverter.scala:72-108: every flag false when the FLAG word is 0;
// the pair flags only for paired reads
__device__ __forceinline__ bool flag_bit(uint32_t f, int k) {
  if (f == 0) return false;
  const bool paired = f & 0x1;
  switch (k) {
    case 0: return paired;                       // readPaired
    case 1: return paired && (f & 0x2);          // properPair
    case 2: return !(f & 0x4);                   // readMapped
    case 3: return paired && !(f & 0x8);         // mateMapped
    case 4: return f & 0x10;                     // readNegativeStrand
    case 5: return paired && (f & 0x20);         // mateNegativeStrand
    case 6: return paired && (f & 0x40);         // firstOfPair
    case 7: return paired && (f & 0x80);         // secondOfPair
    case 8: return !(f & 0x100);                 // primaryAlignment
    case 9: return f & 0x200;                    // failedVendorQualityChecks
    default: return f & 0x400;                   // duplicateRead
  }
}

// pass 1: fixed-width columns, bitmaps, string lengths.  Lanes of a
// wavefront take 64 consecutive records, so a ballot is one bitmap word.
extern "C" __global__ void __launch_bounds__(256) adam_len(AdamParams P) {
  const int lane = threadIdx.x & 63;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  Tag tg[kMaxTags];
  for (int64_t i0 = blockIdx.x * (int64_t)blockDim.x + (threadIdx.x & ~63); i0 < P.n; i0 += stride) {
    const int64_t i = i0 + lane;
    const bool live = i < P.n;
    AdamRec x;
    if (live) {
      adam_record(P, P.r0 + i, x, tg);
      if (x.code != kAdamOk) adam_error(P, i, x.code);
      for (int c = 0; c < kI32; ++c) P.i32[(int64_t)c * P.n + i] = x.i32[c];
      for (int c = 0; c < kI64; ++c) P.i64[(int64_t)c * P.n + i] = x.i64[c];
      for (int c = 0; c < kStr; ++c)
        P.len[(int64_t)c * P.n + i] = c == 5 ? (uint64_t)x.attr_n : c == 2 ? (uint64_t)x.cig_n
                                               : x.sv[c] ? (uint64_t)(x.sb[c] - x.sa[c]) : 0ull;
      const int64_t r = P.r0 + i;
      if (new_qual(P, r)) {  // the recalibrated chars as UTF-8
        const uint64_t slot = P.meta[r].slot + P.out_start[r];
        uint64_t q = 0;
        for (uint32_t k = 0; k < P.out_len[r]; ++k) q += (uint64_t)samk::utf8_len(apply_char(P, slot + k));
        P.len[3 * P.n + i] = q;
      }
    } else {
      x.flag = 0;
      for (int c = 0; c < kStr; ++c) x.sv[c] = false;
      for (int c = 0; c < kI32 + kI64; ++c) x.iv[c] = false;
    }
    const int64_t w = i0 >> 6;
    for (int c = 0; c < kStr; ++c) {
      const uint64_t m = __builtin_amdgcn_ballot_w64(x.sv[c]);
      if (lane == 0) P.svalid[(int64_t)c * P.W + w] = m;
    }
    for (int c = 0; c < kI32 + kI64; ++c) {
      const uint64_t m = __builtin_amdgcn_ballot_w64(x.iv[c]);
      if (lane == 0) P.ivalid[(int64_t)c * P.W + w] = m;
    }
    for (int k = 0; k < kBools; ++k) {
      const uint64_t m = __builtin_amdgcn_ballot_w64(live && flag_bit(x.flag, k));
      if (lane == 0) P.bools[(int64_t)k * P.W + w] = m;
    }
  }
}

// pass 2: the string bytes at their offsets, the Arrow (int32) offsets
extern "C" __global__ void __launch_bounds__(256) adam_write(AdamParams P) {
  Tag tg[kMaxTags];
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < P.n; i += (int64_t)gridDim.x * blockDim.x) {
    AdamRec x;
    const int64_t r = P.r0 + i;
    adam_record(P, r, x, tg);
    for (int c = 0; c < kStr; ++c) {
      const uint64_t o = P.off[(int64_t)c * (P.n + 1) + i];
      P.soff[(int64_t)c * (P.n + 1) + i] = (int32_t)o;
      if (i == P.n - 1) P.soff[(int64_t)c * (P.n + 1) + P.n] = (int32_t)P.off[(int64_t)c * (P.n + 1) + P.n];
      uint8_t* d = P.sbytes[c] + o;
      if (c == 5) {
        uint32_t code = kAdamOk;
        if (x.code == kAdamOk) (void)attributes_text(P.text, tg, x.nt, d, &code);
      } else if (c == 2) {
        (void)cigar_text(P.cig + P.cig_off[r], (int64_t)(P.cig_off[r + 1] - P.cig_off[r]), d);
      } else if (c == 3 && new_qual(P, r)) {
        const uint64_t slot = P.meta[r].slot + P.out_start[r];
        for (uint32_t k = 0; k < P.out_len[r]; ++k) {
          const uint32_t ch = apply_char(P, slot + k);
          if (ch < 0x80u) {
            *d++ = (uint8_t)ch;
          } else if (ch < 0x800u) {
            *d++ = (uint8_t)(0xC0u | (ch >> 6));
            *d++ = (uint8_t)(0x80u | (ch & 0x3Fu));
          } else {
            *d++ = (uint8_t)(0xE0u | (ch >> 12));
            *d++ = (uint8_t)(0x80u | ((ch >> 6) & 0x3Fu));
            *d++ = (uint8_t)(0x80u | (ch & 0x3Fu));
          }
        }
      } else if (x.sv[c]) {
        for (int64_t k = x.sa[c]; k < x.sb[c]; ++k) *d++ = P.text[k];
      }
    }
  }
}
extern "C" __global__ void adam_empty_offsets(int32_t* soff, int64_t n) {  // n == 0: one zero offset per column
  if (threadIdx.x < kStr) soff[threadIdx.x * (n + 1)] = 0;
}

}  // namespace adamk

// the device buffers of the last bqsr_sam_adam_prepare (kept on the parse)
struct AdamBufs {
  int64_t r0 = 0, n = 0, W = 0;
  int64_t cap_n = -1;
  uint64_t *len = nullptr, *off = nullptr, *part = nullptr, *svalid = nullptr, *ivalid = nullptr, *bools = nullptr;
  int32_t *soff = nullptr, *i32 = nullptr;
  int64_t* i64 = nullptr;
  uint8_t* sbytes[adamk::kStr] = {};
  int64_t tot[adamk::kStr] = {}, cap_bytes[adamk::kStr] = {};
  unsigned long long* err = nullptr;
  bool prepared = false;
  // bqsr_sam_adam_set_quals: the apply's outputs (caller's device buffers)
  // and a sorted copy of its exception list
  const bqsr_batch* qb = nullptr;
  const uint8_t* out_qual = nullptr;
  const uint32_t *out_start = nullptr, *out_len = nullptr;
  uint64_t* exc = nullptr;
  int64_t n_exc = 0;
  void free_rows() {
    for (void* p : {(void*)len, (void*)off, (void*)part, (void*)svalid, (void*)ivalid, (void*)bools, (void*)soff,
                    (void*)i32, (void*)i64})
      if (p) (void)hipFree(p);
    len = off = part = svalid = ivalid = bools = nullptr;
    soff = i32 = nullptr;
    i64 = nullptr;
    cap_n = -1;
  }
  ~AdamBufs() {
    free_rows();
    for (auto& p : sbytes)
      if (p) (void)hipFree(p);
    if (err) (void)hipFree(err);
    if (exc) (void)hipFree(exc);
  }
};

bqsr_sam::~bqsr_sam() {
  delete (AdamBufs*)adam;
  for (void* p : allocs) (void)hipFree(p);
  if (d_text) (void)hipFree(d_text);
}

namespace {
void adam_quals(adamk::AdamParams& P, const AdamBufs& A, const bqsr_sam* s) {
  if (A.out_qual) {
    P.meta = A.qb->rd.meta;
    P.info = (const ReadInfo*)A.qb->d_info;
    P.out_qual = A.out_qual;
    P.out_start = A.out_start;
    P.out_len = A.out_len;
    P.exc = A.exc;
    P.n_exc = A.n_exc;
  }
  P.dup_flags = s->dup_marked ? s->flags : nullptr;
}
}  // namespace

extern "C" {

bqsr_status bqsr_sam_adam_set_quals(bqsr_context* ctx, bqsr_sam* s, const bqsr_batch* b, const uint8_t* out_qual,
                                    const uint32_t* out_start, const uint32_t* out_len, const uint64_t* exceptions,
                                    int64_t n_exc, void* stream) {
  if (!ctx || !s || (b && (!out_qual || !out_start || !out_len)) || n_exc < 0 || (n_exc > 0 && !exceptions))
    return fail(BQSR_ERR_INVALID_ARG, "bqsr_sam_adam_set_quals: bad arguments");
  if (b && b->rd.n_reads != s->n_reads) return fail(BQSR_ERR_INVALID_ARG, "batch and SAM read counts differ");
  if (b && !b->prepped) return fail(BQSR_ERR_INVALID_ARG, "the batch has not been through apply");
  HIP_TRY(hipSetDevice(ctx->device));
  if (!s->adam) s->adam = new AdamBufs;
  AdamBufs& A = *(AdamBufs*)s->adam;
  A.prepared = false;
  if (A.exc) (void)hipFree(A.exc);
  A.exc = nullptr;
  A.n_exc = 0;
  A.qb = b;
  A.out_qual = b ? out_qual : nullptr;
  A.out_start = b ? out_start : nullptr;
  A.out_len = b ? out_len : nullptr;
  if (b && n_exc > 0) {  // the exception list in slot order (binary search)
    hipStream_t st = S(stream);
    std::vector<uint64_t> h((size_t)n_exc);
    HIP_TRY(hipMemcpyAsync(h.data(), exceptions, (size_t)n_exc * 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    std::sort(h.begin(), h.end());
    HIP_TRY(hipMalloc((void**)&A.exc, h.size() * 8));
    HIP_TRY(hipMemcpy(A.exc, h.data(), h.size() * 8, hipMemcpyHostToDevice));
    A.n_exc = n_exc;
  }
  return ok();
}

bqsr_status bqsr_sam_header_text(const bqsr_sam* s, char* dst, int64_t cap, int64_t* len) {
  if (!s || !len || (cap > 0 && !dst)) return fail(BQSR_ERR_INVALID_ARG, "bqsr_sam_header_text: bad arguments");
  *len = (int64_t)s->header_text.size();
  if (dst && cap > 0) memcpy(dst, s->header_text.data(), (size_t)std::min<int64_t>(cap, *len));
  return ok();
}

bqsr_status bqsr_sam_adam_prepare(bqsr_context* ctx, bqsr_sam* s, int64_t r0, int64_t n, void* stream,
                                  bqsr_adam_sizes* out) {
  if (!ctx || !s || !out || r0 < 0 || n < 0 || r0 + n > s->n_reads)
    return fail(BQSR_ERR_INVALID_ARG, "bqsr_sam_adam_prepare: bad arguments");
  HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t st = S(stream);
  if (!s->adam) s->adam = new AdamBufs;
  AdamBufs& A = *(AdamBufs*)s->adam;
  A.prepared = false;
  const int64_t W = n / 64 + 1;
  if (A.cap_n < n) {  // per-record buffers, kept across calls
    A.free_rows();
    const size_t N = (size_t)n + 1, WW = (size_t)W;
    auto al = [&](auto** p, size_t cnt) -> hipError_t {
      return hipMalloc((void**)p, std::max<size_t>(cnt, 1) * sizeof(**p));
    };
    hipError_t e = al(&A.len, adamk::kStr * N);
    if (e == hipSuccess) e = al(&A.off, adamk::kStr * N);
    if (e == hipSuccess) e = al(&A.part, N / samk::kScanChunk + 2);
    if (e == hipSuccess) e = al(&A.svalid, adamk::kStr * WW);
    if (e == hipSuccess) e = al(&A.ivalid, (adamk::kI32 + adamk::kI64) * WW);
    if (e == hipSuccess) e = al(&A.bools, adamk::kBools * WW);
    if (e == hipSuccess) e = al(&A.soff, adamk::kStr * N);
    if (e == hipSuccess) e = al(&A.i32, adamk::kI32 * N);
    if (e == hipSuccess) e = al(&A.i64, adamk::kI64 * N);
    if (e == hipSuccess && !A.err) e = al(&A.err, 1);
    if (e != hipSuccess) {
      A.free_rows();
      return fail(BQSR_ERR_DEVICE, std::string("bqsr_sam_adam_prepare: ") + hipGetErrorString(e));
    }
    A.cap_n = n;
  }
  A.r0 = r0;
  A.n = n;
  A.W = W;
  adamk::AdamParams P{};
  P.text = s->d_text;
  P.line_span = s->line_span;
  P.cig_off = s->cig_off;
  P.cig = s->cig;
  P.r0 = r0;
  P.n = n;
  P.sq = s->sq_tab;
  P.rg = s->rg_tab;
  P.len = A.len;
  P.svalid = A.svalid;
  P.i32 = A.i32;
  P.i64 = A.i64;
  P.ivalid = A.ivalid;
  P.bools = A.bools;
  P.W = W;
  P.err = A.err;
  adam_quals(P, A, s);
  HIP_TRY(hipMemsetAsync(A.err, 0xFF, 8, st));
  const unsigned g = sam_grid(n, 256, ctx->n_cu * 8);
  if (n > 0) hipLaunchKernelGGL(adamk::adam_len, dim3(g), dim3(256), 0, st, P);
  HIP_TRY(hipGetLastError());
  bqsr_status rs;
  for (int c = 0; c < adamk::kStr; ++c)
    if ((rs = sam_scan(A.len + (size_t)c * n, n, A.off + (size_t)c * (n + 1), A.part, st)) != BQSR_OK) return rs;
  unsigned long long ew = ~0ull;
  HIP_TRY(hipMemcpyAsync(&ew, A.err, 8, hipMemcpyDeviceToHost, st));
  uint64_t tot[adamk::kStr] = {};
  for (int c = 0; c < adamk::kStr && n > 0; ++c)
    HIP_TRY(hipMemcpyAsync(&tot[c], A.off + (size_t)c * (n + 1) + n, 8, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  if (ew != ~0ull) {
    const uint32_t code = (uint32_t)(ew & 0xFF);
    const int64_t read = r0 + (int64_t)(ew >> 8);
    const char* what = code == adamk::kAdamTagType   ? "an H or B tag (the reference's attribute conversion throws)"
                       : code == adamk::kAdamIntRange ? "an integer tag outside Int (the reference's attribute conversion fails)"
                       : code == adamk::kAdamTagValue ? "an integer / float tag value that does not parse"
                                                      : "more tags than supported";
    return fail(code == adamk::kAdamTagValue ? BQSR_ERR_SAM_PARSE : BQSR_ERR_UNSUPPORTED,
                "ADAM record of read " + std::to_string(read) + ": " + what, read);
  }
  for (int c = 0; c < adamk::kStr; ++c) {
    if ((int64_t)tot[c] > INT32_MAX)
      return fail(BQSR_ERR_UNSUPPORTED, "bqsr_sam_adam_prepare: a string column above 2 GiB (take fewer records)");
    A.tot[c] = (int64_t)tot[c];
    if (A.cap_bytes[c] < A.tot[c] + 1) {
      if (A.sbytes[c]) (void)hipFree(A.sbytes[c]);
      A.sbytes[c] = nullptr;
      A.cap_bytes[c] = 0;
      HIP_TRY(hipMalloc((void**)&A.sbytes[c], (size_t)A.tot[c] + 64));
      A.cap_bytes[c] = A.tot[c] + 1;
    }
  }
  out->n_reads = n;
  for (int c = 0; c < adamk::kStr; ++c) out->str_bytes[c] = A.tot[c];
  out->bitmap_words = W;
  A.prepared = true;
  return ok();
}

bqsr_status bqsr_sam_adam_columns(bqsr_context* ctx, bqsr_sam* s, const bqsr_adam_host* dst, void* stream) {
  if (!ctx || !s || !dst) return fail(BQSR_ERR_INVALID_ARG, "bqsr_sam_adam_columns: bad arguments");
  AdamBufs* Ap = (AdamBufs*)s->adam;
  if (!Ap || !Ap->prepared) return fail(BQSR_ERR_INVALID_ARG, "bqsr_sam_adam_columns before bqsr_sam_adam_prepare");
  AdamBufs& A = *Ap;
  HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t st = S(stream);
  const int64_t n = A.n;
  adamk::AdamParams P{};
  P.text = s->d_text;
  P.line_span = s->line_span;
  P.cig_off = s->cig_off;
  P.cig = s->cig;
  P.r0 = A.r0;
  P.n = n;
  P.sq = s->sq_tab;
  P.rg = s->rg_tab;
  P.off = A.off;
  P.soff = A.soff;
  for (int c = 0; c < adamk::kStr; ++c) P.sbytes[c] = A.sbytes[c];
  P.W = A.W;
  adam_quals(P, A, s);
  if (n > 0) {
    hipLaunchKernelGGL(adamk::adam_write, dim3(sam_grid(n, 256, ctx->n_cu * 8)), dim3(256), 0, st, P);
  } else {
    hipLaunchKernelGGL(adamk::adam_empty_offsets, dim3(1), dim3(64), 0, st, A.soff, n);
  }
  HIP_TRY(hipGetLastError());
  const size_t N1 = (size_t)n + 1, WB = (size_t)A.W * 8;
  auto cp = [&](void* d, const void* src, size_t bytes) -> hipError_t {
    if (!d || !bytes) return hipSuccess;
    return hipMemcpyAsync(d, src, bytes, hipMemcpyDeviceToHost, st);
  };
  hipError_t e = hipSuccess;
  for (int c = 0; c < adamk::kStr && e == hipSuccess; ++c) {
    e = cp(dst->str_offsets[c], A.soff + c * N1, N1 * 4);
    if (e == hipSuccess) e = cp(dst->str_bytes[c], A.sbytes[c], (size_t)A.tot[c]);
    if (e == hipSuccess) e = cp(dst->str_valid[c], A.svalid + c * (size_t)A.W, WB);
  }
  for (int c = 0; c < adamk::kI32 && e == hipSuccess; ++c) e = cp(dst->i32[c], A.i32 + c * (size_t)n, (size_t)n * 4);
  for (int c = 0; c < adamk::kI64 && e == hipSuccess; ++c) e = cp(dst->i64[c], A.i64 + c * (size_t)n, (size_t)n * 8);
  for (int c = 0; c < adamk::kI32 + adamk::kI64 && e == hipSuccess; ++c)
    e = cp(dst->int_valid[c], A.ivalid + c * (size_t)A.W, WB);
  for (int c = 0; c < adamk::kBools && e == hipSuccess; ++c) e = cp(dst->bools[c], A.bools + c * (size_t)A.W, WB);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) return fail(BQSR_ERR_DEVICE, std::string("bqsr_sam_adam_columns: ") + hipGetErrorString(e));
  return ok();
}

}  // extern "C"
