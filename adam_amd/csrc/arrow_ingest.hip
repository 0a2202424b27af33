// ADAMRecord Parquet on the device (include/adam_sam.h bqsr_arrow_*, SURVEY.md
// §8 f1/f2): Arrow's decoded column buffers (adamLoad with the BQSR projection,
// core/rdd/AdamContext.scala:139-161, Projection.scala:10-34) uploaded as they
// are, turned into the parse layout on the device, packed into a BQSR batch
// (sam_batch.hip), and after apply the recalibrated qual column rebuilt as
// Arrow UTF-8 buffers (adamSave, AdamRDDFunctions.scala:37-56).
// Included by bqsr_capi.cpp after sam_batch.hip.
//
//   load   : per Arrow chunk, its buffers copied to the device; a thread per
//            read turns int32 offsets into global byte ranges and validity /
//            boolean bitmaps into the BQSR_F_* flag word;
//   lens   : a thread per read counts the Java chars of sequence / qual /
//            mismatchingPositions (UTF-8 -> UTF-16 code units: a 4-byte
//            sequence is a surrogate pair) and parses its CIGAR (samtools
//            TextCigarCodec, as records.parse_cigar) for the element count;
//   decode : after the scans, the columns as the host path builds them
//            (parquet.py _string_column): a qual char c -> byte c & 0xFF, a
//            sequence / MD char -> min(c, 0xFF); CIGAR -> BAM elements.
//   quals  : after apply, per read the recalibrated chars as UTF-8 (pass-through
//            reads keep their input string), int32 offsets, validity bits.

namespace arwk {

constexpr int kThreads = 256;
enum { kSeq = 0, kQual = 1, kCigar = 2, kMd = 3, kStr = 4, kName = 4, kAll = 5 };  // kStr: the decoded ones
constexpr int kBools = 6;
// readPaired, readMapped, readNegativeStrand, secondOfPair, primaryAlignment, duplicateRead
__constant__ uint32_t kBoolBit[kBools] = {BQSR_F_PAIRED, BQSR_F_MAPPED, BQSR_F_NEG_STRAND, BQSR_F_SECOND_OF_PAIR,
                                          BQSR_F_PRIMARY, BQSR_F_DUPLICATE};
constexpr uint32_t kStrHas[kAll] = {BQSR_F_HAS_SEQ, BQSR_F_HAS_QUAL, BQSR_F_HAS_CIGAR, BQSR_F_HAS_MD, 0};

// one chunk's buffers on the device (copies of Arrow's)
struct ChunkDev {
  int64_t n, r0;                       // reads; global index of the first
  const int32_t* off[kAll];            // [n + 1] or null (column absent: all null)
  const uint8_t* valid[kAll];          // bitmaps or null (all valid)
  uint64_t dbase[kAll];                // global byte index of the chunk's first data byte
  int32_t obase[kAll];                 // off[0]
  const int32_t* ref;                  // dictionary indices or null
  const uint8_t* ref_valid;
  const int64_t* start;
  const uint8_t* start_valid;
  const int32_t* rg;
  const uint8_t* rg_valid;
  const uint8_t* bools[kBools];        // value bitmaps or null (false)
  const uint8_t* bools_valid[kBools];  // null: all valid
  const int32_t* sq;                   // referenceId (MarkDuplicates) or null
  const uint8_t* sq_valid;
  const int32_t* lib;                  // library rank (MarkDuplicates) or null
};

struct Cols {
  uint64_t* beg[kAll];  // [n + 1] raw UTF-8 byte range of each read's string (beg[r], beg[r + 1])
  uint32_t* flags;
  int32_t* rg;
  int32_t* ref;
  int64_t* start;
  uint8_t* name_valid;
  int32_t* sq;   // referenceId, or the referenceName index without the column (-1: null)
  int32_t* lib;
};

__device__ __forceinline__ bool bit(const uint8_t* bm, int64_t i) { return !bm || ((bm[i >> 3] >> (i & 7)) & 1u); }

extern "C" __global__ void __launch_bounds__(kThreads) arrow_chunk_cols(ChunkDev C, Cols O, int last) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < C.n; r += (int64_t)gridDim.x * blockDim.x) {
    const int64_t g = C.r0 + r;
    uint32_t f = 0;
    for (int k = 0; k < kAll; ++k) {
      if (C.off[k]) {
        O.beg[k][g] = C.dbase[k] + (uint64_t)(int64_t)(C.off[k][r] - C.obase[k]);
        if (last && r == C.n - 1) O.beg[k][g + 1] = C.dbase[k] + (uint64_t)(int64_t)(C.off[k][r + 1] - C.obase[k]);
        if (bit(C.valid[k], r)) f |= kStrHas[k];
      } else {
        O.beg[k][g] = C.dbase[k];
        if (last && r == C.n - 1) O.beg[k][g + 1] = C.dbase[k];
      }
    }
    for (int k = 0; k < kBools; ++k)  // a null boolean reads as false
      if (C.bools[k] && bit(C.bools_valid[k], r) && bit(C.bools[k], r)) f |= kBoolBit[k];
    int32_t ref = -1;
    if (C.ref && bit(C.ref_valid, r)) {
      ref = C.ref[r];
      f |= BQSR_F_HAS_REFNAME;
    }
    int64_t st = 0;
    if (C.start && bit(C.start_valid, r)) {
      st = C.start[r];
      f |= BQSR_F_HAS_START;
    }
    int32_t rg = 0;
    if (C.rg && bit(C.rg_valid, r)) {
      rg = C.rg[r];
      f |= BQSR_F_HAS_RG;
    }
    O.flags[g] = f;
    O.ref[g] = ref;
    O.start[g] = st;
    O.rg[g] = rg;
    O.name_valid[g] = C.off[kName] && bit(C.valid[kName], r);
    O.sq[g] = C.sq ? (bit(C.sq_valid, r) ? C.sq[r] : -1) : ref;
    O.lib[g] = C.lib ? C.lib[r] : 0;
  }
}

// Java chars of a UTF-8 byte range: one per lead byte, two for a 4-byte lead
__device__ __forceinline__ uint64_t java_chars(const uint8_t* p, uint64_t a, uint64_t b) {
  uint64_t n = 0;
  for (uint64_t i = a; i < b; ++i) {
    const uint8_t c = p[i];
    n += ((c & 0xC0u) != 0x80u) + (c >= 0xF0u);
  }
  return n;
}

struct LensParams {
  const uint8_t* raw[kStr];
  const uint64_t* beg[kStr];
  const uint32_t* flags;
  const int32_t* rg;
  int64_t n;
  uint64_t* len[kStr];  // Java chars (seq, qual, md), CIGAR elements
  unsigned long long* bad_cigar;  // first read with a malformed CIGAR
  unsigned int* max_rg;
};

extern "C" __global__ void __launch_bounds__(kThreads) arrow_lens(LensParams P) {
  uint32_t mrg = 0;
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < P.n; r += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t f = P.flags[r];
    for (int k = 0; k < kStr; ++k) {
      const uint64_t a = P.beg[k][r], b = P.beg[k][r + 1];
      uint64_t v = 0;
      if (k == kCigar) {
        if ((f & BQSR_F_HAS_CIGAR) && !samk::parse_cigar_text(P.raw[k], (int64_t)a, (int64_t)b, nullptr, &v)) {
          atomicMin(P.bad_cigar, (unsigned long long)r);
          v = 0;
        }
      } else {
        v = java_chars(P.raw[k], a, b);
      }
      P.len[k][r] = v;
    }
    if (f & BQSR_F_HAS_RG) mrg = max(mrg, (uint32_t)max(P.rg[r], 0) + 1u);
  }
  for (int o = 32; o > 0; o >>= 1) mrg = max(mrg, (uint32_t)__shfl_xor((int)mrg, o));
  if ((threadIdx.x & 63) == 0 && mrg) atomicMax(P.max_rg, mrg);
}

struct DecodeParams {
  const uint8_t* raw[kStr];
  const uint64_t* beg[kStr];
  const uint64_t* off[kStr];  // scanned lengths
  const uint32_t* flags;
  int64_t n;
  uint8_t* seq;
  uint8_t* qual;
  uint8_t* md;
  uint32_t* cig;
};

// UTF-8 -> Java chars -> bytes (qual: c & 0xFF; sequence / MD: min(c, 0xFF))
__device__ void decode_str(const uint8_t* p, uint64_t a, uint64_t b, uint8_t* o, bool low_byte) {
  uint64_t i = a, k = 0;
  while (i < b) {
    const uint32_t c = p[i];
    uint32_t cp;
    int len;
    if (c < 0x80u) { cp = c; len = 1; }
    else if (c < 0xE0u) { cp = c & 0x1Fu; len = 2; }
    else if (c < 0xF0u) { cp = c & 0x0Fu; len = 3; }
    else { cp = c & 0x07u; len = 4; }
    for (int j = 1; j < len && i + j < b; ++j) cp = (cp << 6) | (p[i + j] & 0x3Fu);
    i += (uint64_t)len;
    if (len == 4) {  // a surrogate pair
      const uint32_t v = cp - 0x10000u;
      const uint32_t hi = 0xD800u + (v >> 10), lo = 0xDC00u + (v & 0x3FFu);
      o[k++] = low_byte ? (uint8_t)(hi & 0xFFu) : (uint8_t)0xFF;
      o[k++] = low_byte ? (uint8_t)(lo & 0xFFu) : (uint8_t)0xFF;
    } else {
      o[k++] = low_byte ? (uint8_t)(cp & 0xFFu) : (uint8_t)(cp > 0xFFu ? 0xFFu : cp);
    }
  }
}

extern "C" __global__ void __launch_bounds__(kThreads) arrow_decode(DecodeParams P) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < P.n; r += (int64_t)gridDim.x * blockDim.x) {
    decode_str(P.raw[kSeq], P.beg[kSeq][r], P.beg[kSeq][r + 1], P.seq + P.off[kSeq][r], false);
    decode_str(P.raw[kQual], P.beg[kQual][r], P.beg[kQual][r + 1], P.qual + P.off[kQual][r], true);
    decode_str(P.raw[kMd], P.beg[kMd][r], P.beg[kMd][r + 1], P.md + P.off[kMd][r], false);
    if (P.flags[r] & BQSR_F_HAS_CIGAR) {
      uint64_t nc = 0;
      samk::parse_cigar_text(P.raw[kCigar], (int64_t)P.beg[kCigar][r], (int64_t)P.beg[kCigar][r + 1],
                             P.cig + P.off[kCigar][r], &nc);
    }
  }
}

// ---- the qual column after apply ----
struct QualParams {
  const uint8_t* raw;      // input qual strings (UTF-8)
  const uint64_t* beg;     // [n + 1]
  const uint32_t* flags;
  const ReadMeta* meta;
  const ReadInfo* info;
  const uint8_t* out_qual;
  const uint32_t* out_start;
  const uint32_t* out_len;
  const uint64_t* exc;     // sorted (slot << 16 | char)
  int64_t n_exc;
  int64_t n;
  uint64_t* len;           // [n] UTF-8 bytes (pass 1)
  const uint64_t* off;     // [n + 1] scanned (pass 2)
  uint8_t* out;
  int32_t* off32;          // Arrow offsets [n + 1]
  uint8_t* valid;          // Arrow validity bitmap
};

__device__ __forceinline__ uint32_t qual_char(const QualParams& P, uint64_t slot) {
  uint32_t c = P.out_qual[slot];
  if (P.n_exc > 0) {
    int64_t lo = 0, hi = P.n_exc - 1;
    while (lo <= hi) {
      const int64_t mid = (lo + hi) >> 1;
      const uint64_t v = P.exc[mid], s = v >> 16;
      if (s == slot) return (uint32_t)(v & 0xFFFFull);
      if (s < slot) lo = mid + 1;
      else hi = mid - 1;
    }
  }
  return c;
}

template <bool kWrite>
__device__ void qual_read(const QualParams& P, int64_t r) {
  const bool keep = P.out_qual == nullptr || (P.info[r].fl & kInfoPass);
  const bool present = (P.flags[r] & BQSR_F_HAS_QUAL) || (!keep && P.out_len[r] > 0);
  if (keep) {
    const uint64_t a = P.beg[r], b = P.beg[r + 1];
    if (!kWrite) {
      P.len[r] = b - a;
      return;
    }
    uint8_t* o = P.out + P.off[r];
    for (uint64_t i = a; i < b; ++i) *o++ = P.raw[i];
  } else {
    const uint64_t slot = P.meta[r].slot + P.out_start[r];
    const int64_t n = P.out_len[r];
    if (!kWrite) {
      uint64_t q = 0;
      for (int64_t k = 0; k < n; ++k) q += (uint64_t)samk::utf8_len(qual_char(P, slot + k));
      P.len[r] = q;
      return;
    }
    uint8_t* o = P.out + P.off[r];
    for (int64_t k = 0; k < n; ++k) {
      const uint32_t c = qual_char(P, slot + k);
      if (c < 0x80u) {
        *o++ = (uint8_t)c;
      } else if (c < 0x800u) {
        *o++ = (uint8_t)(0xC0u | (c >> 6));
        *o++ = (uint8_t)(0x80u | (c & 0x3Fu));
      } else {
        *o++ = (uint8_t)(0xE0u | (c >> 12));
        *o++ = (uint8_t)(0x80u | ((c >> 6) & 0x3Fu));
        *o++ = (uint8_t)(0x80u | (c & 0x3Fu));
      }
    }
  }
  P.off32[r] = (int32_t)P.off[r];
  if (r == P.n - 1) P.off32[r + 1] = (int32_t)P.off[r + 1];
  // validity: a wavefront's 64 reads form whole bytes when r0 is 64-aligned
  const uint64_t m = __ballot(present);
  const int lane = threadIdx.x & 63;
  if (lane < 8 && (r - lane) + 8 * lane < P.n) P.valid[((r - lane) >> 3) + lane] = (uint8_t)(m >> (8 * lane));
}

extern "C" __global__ void __launch_bounds__(kThreads) arrow_qual_len(QualParams P) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < P.n; r += (int64_t)gridDim.x * blockDim.x)
    qual_read<false>(P, r);
}
// a wavefront's lanes hold 64 consecutive reads (64-aligned) at every stride
// step, so its validity ballot is whole bytes of the bitmap
extern "C" __global__ void __launch_bounds__(kThreads) arrow_qual_write(QualParams P) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < P.n; r += (int64_t)gridDim.x * blockDim.x)
    qual_read<true>(P, r);
}

}  // namespace arwk

struct bqsr_arrow {
  bqsr_context* ctx = nullptr;
  int64_t n = 0;
  int32_t n_rg = 1;
  uint8_t* raw[arwk::kAll] = {nullptr, nullptr, nullptr, nullptr, nullptr};
  uint64_t* beg[arwk::kAll] = {nullptr, nullptr, nullptr, nullptr, nullptr};
  uint8_t* name_valid = nullptr;  // readName present (MarkDuplicates)
  int32_t *sq = nullptr, *lib = nullptr;
  uint32_t* flags = nullptr;
  int32_t *rg = nullptr, *ref = nullptr;
  int64_t* start = nullptr;
  uint64_t *seq_off = nullptr, *qual_off = nullptr, *md_off = nullptr, *cig_off = nullptr;
  uint8_t *seq = nullptr, *qual = nullptr, *md = nullptr;
  uint32_t* cig = nullptr;
  int64_t seq_bytes = 0, qual_bytes = 0, md_bytes = 0, cig_ops = 0;
  // the qual column after apply (bqsr_arrow_qual_prepare)
  uint8_t* q_out = nullptr;
  int32_t* q_off = nullptr;
  uint8_t* q_valid = nullptr;
  int64_t q_bytes = -1;
  std::vector<void*> allocs;
  ~bqsr_arrow() {
    for (void* p : allocs) (void)hipFree(p);
    for (void* p : {(void*)q_out, (void*)q_off, (void*)q_valid})
      if (p) (void)hipFree(p);
  }
};

namespace {
template <class T>
bqsr_status arrow_h2d(std::vector<void*>& keep, T** dst, const void* src, size_t count, hipStream_t s) {
  *dst = nullptr;
  if (!src) return ok();
  bqsr_status st = dalloc(keep, dst, std::max<size_t>(count, 1));
  if (st != BQSR_OK) return st;
  if (count) HIP_TRY(hipMemcpyAsync(*dst, src, count * sizeof(T), hipMemcpyHostToDevice, s));
  return ok();
}
}  // namespace

bqsr_status bqsr_arrow_load(bqsr_context* ctx, const bqsr_arrow_chunk* chunks, int32_t n_chunks, void* stream,
                            bqsr_arrow** out) {
  using namespace arwk;
  if (!ctx || !out || n_chunks < 0 || (n_chunks && !chunks)) return fail(BQSR_ERR_INVALID_ARG, "bqsr_arrow_load: bad arguments");
  *out = nullptr;
  HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = S(stream);
  std::unique_ptr<bqsr_arrow> A(new bqsr_arrow);
  A->ctx = ctx;
  // totals: reads, raw bytes per string column
  int64_t n = 0;
  uint64_t tot[kAll] = {0, 0, 0, 0, 0};
  for (int32_t c = 0; c < n_chunks; ++c) {
    const bqsr_arrow_chunk& C = chunks[c];
    if (C.n_reads < 0) return fail(BQSR_ERR_INVALID_ARG, "bqsr_arrow_load: negative chunk length");
    const bqsr_arrow_strings* sc[kAll] = {&C.sequence, &C.qual, &C.cigar, &C.md, &C.read_name};
    for (int k = 0; k < kAll; ++k)
      if (sc[k]->offsets) {
        const int32_t a = sc[k]->offsets[0], b = sc[k]->offsets[C.n_reads];
        if (b < a || (b > a && !sc[k]->data)) return fail(BQSR_ERR_INVALID_ARG, "bqsr_arrow_load: bad string offsets");
        tot[k] += (uint64_t)(b - a);
      }
    n += C.n_reads;
  }
  A->n = n;
  std::vector<void*>& K = A->allocs;
  bqsr_status st;
  for (int k = 0; k < kAll; ++k)
    if ((st = dalloc(K, &A->raw[k], (size_t)tot[k] + 16)) || (st = dalloc(K, &A->beg[k], (size_t)n + 1))) return st;
  const size_t n1 = (size_t)std::max<int64_t>(n, 1);
  if ((st = dalloc(K, &A->name_valid, n1)) || (st = dalloc(K, &A->sq, n1)) || (st = dalloc(K, &A->lib, n1))) return st;
  if ((st = dalloc(K, &A->flags, (size_t)std::max<int64_t>(n, 1))) || (st = dalloc(K, &A->rg, (size_t)std::max<int64_t>(n, 1))) ||
      (st = dalloc(K, &A->ref, (size_t)std::max<int64_t>(n, 1))) || (st = dalloc(K, &A->start, (size_t)std::max<int64_t>(n, 1))))
    return st;
  for (int k = 0; k < kAll; ++k) HIP_TRY(hipMemsetAsync(A->beg[k], 0, 8, s));  // n == 0: beg[0] = 0
  // per chunk: its buffers to the device, then its rows of the global columns
  uint64_t dpos[kAll] = {0, 0, 0, 0, 0};
  int64_t r0 = 0;
  std::vector<void*> tmp;
  struct Free {
    std::vector<void*>& v;
    ~Free() {
      for (void* p : v) (void)hipFree(p);
    }
  } fr{tmp};
  for (int32_t c = 0; c < n_chunks; ++c) {
    const bqsr_arrow_chunk& H = chunks[c];
    const int64_t m = H.n_reads;
    if (m == 0) continue;
    const size_t vb = (size_t)(m + 7) / 8;
    ChunkDev D{};
    D.n = m;
    D.r0 = r0;
    const bqsr_arrow_strings* sc[kAll] = {&H.sequence, &H.qual, &H.cigar, &H.md, &H.read_name};
    for (int k = 0; k < kAll; ++k) {
      D.dbase[k] = dpos[k];
      if (!sc[k]->offsets) continue;
      const int32_t a = sc[k]->offsets[0], b = sc[k]->offsets[m];
      if (b > a) HIP_TRY(hipMemcpyAsync(A->raw[k] + dpos[k], sc[k]->data + a, (size_t)(b - a), hipMemcpyHostToDevice, s));
      D.obase[k] = a;
      int32_t* o;
      uint8_t* v;
      if ((st = arrow_h2d(tmp, &o, sc[k]->offsets, (size_t)m + 1, s)) || (st = arrow_h2d(tmp, &v, sc[k]->validity, vb, s)))
        return st;
      D.off[k] = o;
      D.valid[k] = v;
      dpos[k] += (uint64_t)(b - a);
    }
    int32_t *ref, *rg;
    int64_t* start;
    uint8_t *rv, *sv, *gv;
    if ((st = arrow_h2d(tmp, &ref, H.reference, (size_t)m, s)) || (st = arrow_h2d(tmp, &rv, H.reference_validity, vb, s)) ||
        (st = arrow_h2d(tmp, &start, H.start, (size_t)m, s)) || (st = arrow_h2d(tmp, &sv, H.start_validity, vb, s)) ||
        (st = arrow_h2d(tmp, &rg, H.record_group, (size_t)m, s)) || (st = arrow_h2d(tmp, &gv, H.record_group_validity, vb, s)))
      return st;
    D.ref = ref;
    D.ref_valid = H.reference ? rv : nullptr;
    D.start = start;
    D.start_valid = H.start ? sv : nullptr;
    D.rg = rg;
    D.rg_valid = H.record_group ? gv : nullptr;
    for (int k = 0; k < kBools; ++k) {
      uint8_t *bv, *bvv;
      if ((st = arrow_h2d(tmp, &bv, H.bools[k], vb, s)) || (st = arrow_h2d(tmp, &bvv, H.bools_validity[k], vb, s)))
        return st;
      D.bools[k] = bv;
      D.bools_valid[k] = bvv;
    }
    int32_t *sq, *lib;
    uint8_t* qv;
    if ((st = arrow_h2d(tmp, &sq, H.reference_id, (size_t)m, s)) ||
        (st = arrow_h2d(tmp, &qv, H.reference_id_validity, vb, s)) || (st = arrow_h2d(tmp, &lib, H.library, (size_t)m, s)))
      return st;
    D.sq = sq;
    D.sq_valid = H.reference_id ? qv : nullptr;
    D.lib = lib;
    Cols O{{A->beg[0], A->beg[1], A->beg[2], A->beg[3], A->beg[4]}, A->flags, A->rg, A->ref, A->start,
           A->name_valid, A->sq, A->lib};
    hipLaunchKernelGGL(arrow_chunk_cols, dim3(sam_grid(m, kThreads, ctx->n_cu * 16)), dim3(kThreads), 0, s, D, O,
                       (int)(r0 + m == n));
    HIP_TRY(hipGetLastError());
    // the chunk's staging buffers are freed after its kernel ran
    HIP_TRY(hipStreamSynchronize(s));
    for (void* p : tmp) (void)hipFree(p);
    tmp.clear();
    r0 += m;
  }
  // lengths, scans, decode
  uint64_t* len[kStr];
  uint64_t* off[kStr];
  uint64_t* part;
  unsigned long long* bad;
  unsigned int* max_rg;
  for (int k = 0; k < kStr; ++k)
    if ((st = dalloc(tmp, &len[k], (size_t)n + 1)) || (st = dalloc(K, &off[k], (size_t)n + 1))) return st;
  if ((st = dalloc(tmp, &part, (size_t)(n / samk::kScanChunk + 2))) || (st = dalloc(tmp, &bad, 1)) ||
      (st = dalloc(tmp, &max_rg, 1)))
    return st;
  const unsigned long long nb0 = ~0ull;
  HIP_TRY(hipMemcpyAsync(bad, &nb0, 8, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemsetAsync(max_rg, 0, 4, s));
  LensParams LP{};
  for (int k = 0; k < kStr; ++k) {
    LP.raw[k] = A->raw[k];
    LP.beg[k] = A->beg[k];
    LP.len[k] = len[k];
  }
  LP.flags = A->flags;
  LP.rg = A->rg;
  LP.n = n;
  LP.bad_cigar = bad;
  LP.max_rg = max_rg;
  const unsigned g = sam_grid(n, kThreads, ctx->n_cu * 16);
  if (n) hipLaunchKernelGGL(arrow_lens, dim3(g), dim3(kThreads), 0, s, LP);
  for (int k = 0; k < kStr; ++k)
    if ((st = sam_scan(len[k], n, off[k], part, s)) != BQSR_OK) return st;
  uint64_t totals[kStr];
  unsigned long long hbad = 0;
  unsigned int hmrg = 0;
  for (int k = 0; k < kStr; ++k) HIP_TRY(hipMemcpyAsync(&totals[k], off[k] + n, 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(&hbad, bad, 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(&hmrg, max_rg, 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (n == 0)
    for (int k = 0; k < kStr; ++k) totals[k] = 0;
  if (hbad != ~0ull) return fail(BQSR_ERR_SAM_PARSE, "Malformed CIGAR string", (int64_t)hbad);
  A->seq_off = off[kSeq];
  A->qual_off = off[kQual];
  A->cig_off = off[kCigar];
  A->md_off = off[kMd];
  A->seq_bytes = (int64_t)totals[kSeq];
  A->qual_bytes = (int64_t)totals[kQual];
  A->cig_ops = (int64_t)totals[kCigar];
  A->md_bytes = (int64_t)totals[kMd];
  A->n_rg = (int32_t)std::max(1u, hmrg);
  if ((st = dalloc(K, &A->seq, (size_t)A->seq_bytes + 16)) || (st = dalloc(K, &A->qual, (size_t)A->qual_bytes + 16)) ||
      (st = dalloc(K, &A->md, (size_t)A->md_bytes + 16)) || (st = dalloc(K, &A->cig, (size_t)A->cig_ops + 4)))
    return st;
  DecodeParams DP{};
  for (int k = 0; k < kStr; ++k) {
    DP.raw[k] = A->raw[k];
    DP.beg[k] = A->beg[k];
    DP.off[k] = off[k];
  }
  DP.flags = A->flags;
  DP.n = n;
  DP.seq = A->seq;
  DP.qual = A->qual;
  DP.md = A->md;
  DP.cig = A->cig;
  if (n) hipLaunchKernelGGL(arrow_decode, dim3(g), dim3(kThreads), 0, s, DP);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(s));
  *out = A.release();
  return ok();
}

void bqsr_arrow_destroy(bqsr_arrow* a) { delete a; }
int64_t bqsr_arrow_reads(const bqsr_arrow* a) { return a ? a->n : -1; }

bqsr_status bqsr_arrow_batch_create(bqsr_context* ctx, const bqsr_arrow* a, const int32_t* ref_contig, int32_t n_ref,
                                    void* stream, bqsr_batch** out) {
  if (!ctx || !a || !out || n_ref < 0 || (n_ref && !ref_contig))
    return fail(BQSR_ERR_INVALID_ARG, "bqsr_arrow_batch_create: bad arguments");
  if (a->ctx != ctx) return fail(BQSR_ERR_INVALID_ARG, "bqsr_arrow_batch_create: columns of another context");
  *out = nullptr;
  PackCols C{a->flags, a->rg, a->ref, a->start, a->seq_off, a->qual_off, a->cig_off, a->md_off, a->seq, a->qual,
             a->md, a->cig, a->n, a->seq_bytes, a->md_bytes, a->cig_ops, a->n_rg};
  return pack_batch_device(ctx, C, ref_contig, n_ref, stream, out);
}

bqsr_status bqsr_arrow_qual_prepare(bqsr_context* ctx, bqsr_arrow* a, const bqsr_batch* b, const uint8_t* out_qual,
                                    const uint32_t* out_start, const uint32_t* out_len, const uint64_t* exceptions,
                                    int64_t n_exc, void* stream, int64_t* n_bytes) {
  using namespace arwk;
  if (!ctx || !a || (b && (!out_qual || !out_start || !out_len)) || n_exc < 0 || (n_exc > 0 && !exceptions))
    return fail(BQSR_ERR_INVALID_ARG, "bqsr_arrow_qual_prepare: bad arguments");
  if (b && b->rd.n_reads != a->n) return fail(BQSR_ERR_INVALID_ARG, "batch and column read counts differ");
  if (b && !b->prepped) return fail(BQSR_ERR_INVALID_ARG, "the batch has not been through apply");
  HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = S(stream);
  const int64_t n = a->n;
  std::vector<void*> tmp;
  struct Free {
    std::vector<void*>& v;
    ~Free() {
      for (void* p : v) (void)hipFree(p);
    }
  } fr{tmp};
  for (void* p : {(void*)a->q_out, (void*)a->q_off, (void*)a->q_valid})
    if (p) (void)hipFree(p);
  a->q_out = nullptr;
  a->q_off = nullptr;
  a->q_valid = nullptr;
  a->q_bytes = -1;
  bqsr_status st;
  uint64_t *len, *off, *part, *exc_sorted = nullptr;
  if ((st = dalloc(tmp, &len, (size_t)n + 1)) || (st = dalloc(tmp, &off, (size_t)n + 1)) ||
      (st = dalloc(tmp, &part, (size_t)(n / samk::kScanChunk + 2))))
    return st;
  if (b && n_exc > 0) {  // the exception list in slot order (binary search)
    std::vector<uint64_t> h((size_t)n_exc);
    HIP_TRY(hipMemcpyAsync(h.data(), exceptions, (size_t)n_exc * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    std::sort(h.begin(), h.end());
    if ((st = sam_upload(tmp, &exc_sorted, h, s)) != BQSR_OK) return st;
  }
  QualParams P{};
  P.raw = a->raw[kQual];
  P.beg = a->beg[kQual];
  P.flags = a->flags;
  P.meta = b ? b->rd.meta : nullptr;
  P.info = b ? (const ReadInfo*)b->d_info : nullptr;
  P.out_qual = b ? out_qual : nullptr;
  P.out_start = out_start;
  P.out_len = out_len;
  P.exc = exc_sorted;
  P.n_exc = b ? n_exc : 0;
  P.n = n;
  P.len = len;
  P.off = off;
  const unsigned g = sam_grid(n, kThreads, ctx->n_cu * 16);
  if (n) hipLaunchKernelGGL(arrow_qual_len, dim3(g), dim3(kThreads), 0, s, P);
  if ((st = sam_scan(len, n, off, part, s)) != BQSR_OK) return st;
  uint64_t total = 0;
  if (n) HIP_TRY(hipMemcpyAsync(&total, off + n, 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (total > 0x7FFFFFFFull) return fail(BQSR_ERR_UNSUPPORTED, "qual column beyond 2 GiB (int32 Arrow offsets)");
  HIP_TRY(hipMalloc((void**)&a->q_out, (size_t)total + 16));
  HIP_TRY(hipMalloc((void**)&a->q_off, (size_t)(n + 1) * 4));
  HIP_TRY(hipMalloc((void**)&a->q_valid, (size_t)(n + 63) / 8 + 8));
  HIP_TRY(hipMemsetAsync(a->q_off, 0, 4, s));
  HIP_TRY(hipMemsetAsync(a->q_valid, 0, (size_t)(n + 63) / 8 + 8, s));
  P.out = a->q_out;
  P.off32 = a->q_off;
  P.valid = a->q_valid;
  if (n) hipLaunchKernelGGL(arrow_qual_write, dim3(g), dim3(kThreads), 0, s, P);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(s));
  a->q_bytes = (int64_t)total;
  if (n_bytes) *n_bytes = (int64_t)total;
  return ok();
}

bqsr_status bqsr_arrow_qual_column(const bqsr_arrow* a, int32_t* offsets, uint8_t* data, uint8_t* validity) {
  if (!a || a->q_bytes < 0) return fail(BQSR_ERR_INVALID_ARG, "bqsr_arrow_qual_column before bqsr_arrow_qual_prepare");
  HIP_TRY(hipSetDevice(a->ctx->device));
  if (offsets) HIP_TRY(hipMemcpy(offsets, a->q_off, (size_t)(a->n + 1) * 4, hipMemcpyDeviceToHost));
  if (data && a->q_bytes) HIP_TRY(hipMemcpy(data, a->q_out, (size_t)a->q_bytes, hipMemcpyDeviceToHost));
  if (validity) HIP_TRY(hipMemcpy(validity, a->q_valid, (size_t)(a->n + 7) / 8, hipMemcpyDeviceToHost));
  return ok();
}

bqsr_status bqsr_arrow_mark_duplicates(bqsr_context* ctx, bqsr_arrow* a, int64_t* n_duplicates) {
  if (!ctx || !a) return fail(BQSR_ERR_INVALID_ARG, "bqsr_arrow_mark_duplicates: bad arguments");
  if (a->ctx != ctx) return fail(BQSR_ERR_INVALID_ARG, "bqsr_arrow_mark_duplicates: columns of another context");
  HIP_TRY(hipSetDevice(ctx->device));
  bqsr_dup_set* d = nullptr;
  bqsr_status st = bqsr_dup_set_create(ctx, a->n, &d);
  if (st != BQSR_OK) return st;
  std::unique_ptr<bqsr_dup_set> own(d);
  mdupd::DevSam S{};
  S.text = a->raw[arwk::kName];
  S.flags = a->flags;
  S.rg_id = a->rg;
  S.sq_id = a->sq;
  S.start = a->start;
  S.qual_off = a->qual_off;
  S.qual = a->qual;
  S.cig_off = a->cig_off;
  S.cig = a->cig;
  S.n = a->n;
  S.name_beg = a->beg[arwk::kName];
  S.name_valid = a->name_valid;
  S.read_lib = a->lib;
  if ((st = dup_set_add_cols(d, S)) != BQSR_OK) return st;
  int64_t nd = 0;
  if ((st = bqsr_dup_set_finish(d, &nd)) != BQSR_OK) return st;
  if (a->n) {
    hipStream_t s = hipStreamPerThread;
    const unsigned g = sam_grid(a->n, mdupd::kThreads, ctx->n_cu * 16);
    HIP_TRY(hipMemsetAsync(d->cnt, 0, sizeof(unsigned long long), s));
    hipLaunchKernelGGL(mdupd::mdup_set_apply, dim3(g), dim3(mdupd::kThreads), 0, s, (const uint32_t*)d->bits,
                       (int64_t)0, a->n, a->flags, d->cnt);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(s));
  }
  if (n_duplicates) *n_duplicates = nd;
  return ok();
}

namespace arwk {
// bit r of the bitmap = (flags[r] & flag) != 0; a wavefront per 64 reads (8 bytes)
extern "C" __global__ void __launch_bounds__(kThreads) arrow_flag_bits(const uint32_t* flags, int64_t n, uint32_t flag,
                                                                      uint8_t* bits) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t m = __ballot((flags[r] & flag) != 0);
    const int lane = threadIdx.x & 63;
    if (lane < 8 && (r - lane) + 8 * lane < n) bits[((r - lane) >> 3) + lane] = (uint8_t)(m >> (8 * lane));
  }
}
}  // namespace arwk

bqsr_status bqsr_arrow_flag_bitmap(const bqsr_arrow* a, uint32_t flag, uint8_t* bitmap) {
  if (!a || (!bitmap && a->n)) return fail(BQSR_ERR_INVALID_ARG, "bqsr_arrow_flag_bitmap: bad arguments");
  if (a->n == 0) return ok();
  HIP_TRY(hipSetDevice(a->ctx->device));
  hipStream_t s = hipStreamPerThread;
  uint8_t* d = nullptr;
  const size_t nb = (size_t)(a->n + 7) / 8;
  HIP_TRY(hipMalloc((void**)&d, nb + 8));
  hipLaunchKernelGGL(arwk::arrow_flag_bits, dim3(sam_grid(a->n, arwk::kThreads, a->ctx->n_cu * 16)),
                     dim3(arwk::kThreads), 0, s, (const uint32_t*)a->flags, a->n, flag, d);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipMemcpyAsync(bitmap, d, nb, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  (void)hipFree(d);
  if (e != hipSuccess) return fail(BQSR_ERR_DEVICE, hipGetErrorString(e));
  return ok();
}
