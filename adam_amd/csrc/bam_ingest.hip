// BAM -> the device columns of a parsed SAM (include/adam_sam.h bqsr_bam_parse,
// SURVEY.md §8 f1; the reference loads BAM through Hadoop-BAM's
// AnySAMInputFormat, core/rdd/AdamContext.scala:122-137, and converts every
// record with SAMRecordConverter.scala:26-144).
//
// Host: the BGZF blocks (gzip members of <= 64 KiB) are located by their
// BSIZE fields and inflated in parallel by std::threads (zlib, raw deflate)
// into one buffer at the prefix sums of their ISIZE; the BAM header (magic,
// l_text, the SAM header text, the binary reference list) is read, and the
// records' offsets found by a walk over their block_size fields.
// Device: the records' bytes are uploaded once; a thread per record decodes
// it the way the SAM text of the same record parses (bqsr_sam_parse): the
// same flags (FLAG only when non-zero, Q2), referenceName only for a
// dictionary name, start = pos when the read has one, SEQ as text (4-bit
// codes -> "=ACMGRSVTWYHKDBN", "*" when empty), QUAL as text (phred + 33, "*"
// when absent), the BAM CIGAR words as they are, and the last MD / RG tags
// (Z or integer values as their text).  Two passes as the SAM parser: lengths,
// scans, then the columns.
//
// Included by bqsr_capi.cpp after sam_ingest.hip.

#include <zlib.h>

namespace bamk {

struct BamParams {
  const uint8_t* buf;       // the decompressed BAM
  const uint64_t* rec;      // [n + 1] record offsets (block_size field of record r at rec[r])
  int64_t n;
  const int32_t* ref_sq;    // [n_ref] BAM refID -> @SQ header index (-1: not a header name)
  int32_t n_ref;
  samk::NameTable rg;
  uint64_t* len;            // [4][n]: seq, qual, cigar ops, md bytes
  uint64_t* off;            // [4][n + 1] exclusive scans of len
  unsigned long long* err;  // (record << 8) | code, the smallest wins
  // columns (bqsr_sam)
  uint32_t* flags;
  int32_t* rg_id;
  int32_t* ref;
  int32_t* sq_id;
  uint32_t* raw_flag;
  int64_t* start;
  uint64_t *seq_off, *qual_off, *cig_off, *md_off;
  uint8_t *seq, *qual, *md;
  uint32_t* cig;
  uint64_t* line_span;      // the read name's bytes (MarkDuplicates' QNAME)
};

enum : uint32_t { kBamOk = 0, kBamRecord = 1, kBamTag = 2, kBamTagType = 3 };

__device__ __forceinline__ uint32_t rd32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
__device__ __forceinline__ uint16_t rd16(const uint8_t* p) { return (uint16_t)(p[0] | (p[1] << 8)); }

// the text of an integer tag value (htsjdk's attribute value toString)
__device__ __forceinline__ int int_text(int64_t v, uint8_t* out) {
  uint8_t b[24];
  int n = 0;
  const bool neg = v < 0;
  uint64_t u = neg ? (uint64_t)(-(v + 1)) + 1 : (uint64_t)v;
  do {
    b[n++] = (uint8_t)('0' + u % 10);
    u /= 10;
  } while (u);
  int k = 0;
  if (neg) out[k++] = '-';
  while (n) out[k++] = b[--n];
  return k;
}

struct TagVal {
  int64_t a = -1, n = 0;  // Z: bytes [a, a + n) of the record
  int kind = 0;           // 0 none, 1 Z / A (bytes), 2 integer (value)
  int64_t v = 0;
};

// one record: lengths (kWrite false) or the columns of read r
template <bool kWrite>
__device__ void bam_record(const BamParams& P, int64_t r) {
  const uint8_t* b = P.buf + P.rec[r];
  const int64_t bs = (int64_t)rd32(b);
  const int64_t end = 4 + bs;
  if (bs < 32) {
    if (!kWrite) atomicMin(P.err, ((unsigned long long)r << 8) | kBamRecord);
    return;
  }
  const int32_t refid = (int32_t)rd32(b + 4);
  const int32_t pos = (int32_t)rd32(b + 8);
  const int l_name = b[12];
  const int n_cig = rd16(b + 16);
  const uint32_t flag = rd16(b + 18);
  const int64_t l_seq = (int64_t)(int32_t)rd32(b + 20);
  const int64_t o_name = 36, o_cig = o_name + l_name, o_seq = o_cig + 4 * (int64_t)n_cig;
  const int64_t o_qual = o_seq + (l_seq + 1) / 2, o_tag = o_qual + l_seq;
  if (l_seq < 0 || o_tag > end || l_name < 1) {
    if (!kWrite) atomicMin(P.err, ((unsigned long long)r << 8) | kBamRecord);
    return;
  }
  // tags: the last MD and RG win
  TagVal md, rg;
  for (int64_t p = o_tag; p < end;) {
    if (p + 3 > end) {
      if (!kWrite) atomicMin(P.err, ((unsigned long long)r << 8) | kBamTag);
      return;
    }
    const uint8_t t0 = b[p], t1 = b[p + 1], ty = b[p + 2];
    p += 3;
    TagVal v;
    int64_t sz = 0;
    switch (ty) {
      case 'A': v.kind = 1; v.a = p; v.n = 1; sz = 1; break;
      case 'c': v.kind = 2; v.v = (int8_t)b[p]; sz = 1; break;
      case 'C': v.kind = 2; v.v = b[p]; sz = 1; break;
      case 's': v.kind = 2; v.v = (int16_t)rd16(b + p); sz = 2; break;
      case 'S': v.kind = 2; v.v = rd16(b + p); sz = 2; break;
      case 'i': v.kind = 2; v.v = (int32_t)rd32(b + p); sz = 4; break;
      case 'I': v.kind = 2; v.v = rd32(b + p); sz = 4; break;
      case 'f': sz = 4; v.kind = -1; break;  // float: its text is Java's Float.toString (not decoded)
      case 'Z':
      case 'H': {
        int64_t q = p;
        while (q < end && b[q]) ++q;
        if (q >= end) {
          if (!kWrite) atomicMin(P.err, ((unsigned long long)r << 8) | kBamTag);
          return;
        }
        v.kind = ty == 'Z' ? 1 : -1;
        v.a = p;
        v.n = q - p;
        sz = q - p + 1;
        break;
      }
      case 'B': {
        if (p + 5 > end) {
          if (!kWrite) atomicMin(P.err, ((unsigned long long)r << 8) | kBamTag);
          return;
        }
        const uint8_t st = b[p];
        const int64_t cnt = rd32(b + p + 1);
        const int es = (st == 'c' || st == 'C') ? 1 : (st == 's' || st == 'S') ? 2 : 4;
        sz = 5 + cnt * es;
        v.kind = -1;
        break;
      }
      default:
        if (!kWrite) atomicMin(P.err, ((unsigned long long)r << 8) | kBamTag);
        return;
    }
    if (p + sz > end) {
      if (!kWrite) atomicMin(P.err, ((unsigned long long)r << 8) | kBamTag);
      return;
    }
    if (t0 == 'M' && t1 == 'D') md = v;
    if (t0 == 'R' && t1 == 'G') rg = v;
    p += sz;
  }
  if (md.kind < 0 || rg.kind < 0) {  // an MD / RG value whose text is not decoded here
    if (!kWrite) atomicMin(P.err, ((unsigned long long)r << 8) | kBamTagType);
    return;
  }
  uint8_t ibuf[24];
  int64_t md_n = md.kind == 1 ? md.n : md.kind == 2 ? int_text(md.v, ibuf) : 0;
  const int64_t seq_n = l_seq ? l_seq : 1;  // "*"
  const bool no_qual = l_seq == 0 || b[o_qual] == 0xFF;
  const int64_t qual_n = no_qual ? 1 : l_seq;
  if (!kWrite) {
    P.len[r] = (uint64_t)seq_n;
    P.len[P.n + r] = (uint64_t)qual_n;
    P.len[2 * P.n + r] = (uint64_t)n_cig;
    P.len[3 * P.n + r] = (uint64_t)md_n;
    return;
  }
  const int32_t sq = (refid >= 0 && refid < P.n_ref) ? P.ref_sq[refid] : -1;
  int32_t rgv = -1;
  if (rg.kind == 1) {
    rgv = samk::name_lookup(P.rg, b + rg.a, rg.n);
  } else if (rg.kind == 2) {
    const int k = int_text(rg.v, ibuf);
    rgv = samk::name_lookup(P.rg, ibuf, k);
  }
  uint32_t f = BQSR_F_HAS_SEQ | BQSR_F_HAS_QUAL | BQSR_F_HAS_CIGAR;
  if (flag != 0) {  // SAMRecordConverter.scala:72-108: flags only when the word is non-zero (Q2)
    if (flag & 0x1) {
      f |= BQSR_F_PAIRED;
      if (flag & 0x80) f |= BQSR_F_SECOND_OF_PAIR;
    }
    if (flag & 0x400) f |= BQSR_F_DUPLICATE;
    if (flag & 0x10) f |= BQSR_F_NEG_STRAND;
    if (!(flag & 0x100)) f |= BQSR_F_PRIMARY;
    if (!(flag & 0x4)) f |= BQSR_F_MAPPED;
  }
  const bool has_start = sq >= 0 && pos != -1;  // SAM POS = pos + 1: a start when POS != 0
  if (sq >= 0) f |= BQSR_F_HAS_REFNAME;
  if (has_start) f |= BQSR_F_HAS_START;
  if (md.kind > 0) f |= BQSR_F_HAS_MD;
  if (rgv >= 0) f |= BQSR_F_HAS_RG;
  const uint64_t os = P.off[r], oq = P.off[(P.n + 1) + r], oc = P.off[2 * (P.n + 1) + r],
                 om = P.off[3 * (P.n + 1) + r];
  P.flags[r] = f;
  P.rg_id[r] = rgv >= 0 ? rgv : 0;
  P.ref[r] = sq;
  P.sq_id[r] = sq;
  P.raw_flag[r] = flag;
  P.start[r] = has_start ? (int64_t)pos : 0;
  P.seq_off[r] = os;
  P.qual_off[r] = oq;
  P.cig_off[r] = oc;
  P.md_off[r] = om;
  for (int k = 0; k < n_cig; ++k) P.cig[oc + k] = rd32(b + o_cig + 4 * k);
  const char kCodes[] = "=ACMGRSVTWYHKDBN";
  if (l_seq == 0) {
    P.seq[os] = '*';
  } else {
    for (int64_t k = 0; k < l_seq; ++k) P.seq[os + k] = (uint8_t)kCodes[(b[o_seq + (k >> 1)] >> ((k & 1) ? 0 : 4)) & 15];
  }
  if (no_qual) {
    P.qual[oq] = '*';
  } else {
    for (int64_t k = 0; k < l_seq; ++k) P.qual[oq + k] = (uint8_t)(b[o_qual + k] + 33);
  }
  if (md.kind == 1)
    for (int64_t k = 0; k < md_n; ++k) P.md[om + k] = b[md.a + k];
  else if (md.kind == 2)
    for (int64_t k = 0; k < md_n; ++k) P.md[om + k] = ibuf[k];
  P.line_span[2 * r] = P.rec[r] + o_name;
  P.line_span[2 * r + 1] = P.rec[r] + o_name + l_name - 1;  // the name without its NUL
}

extern "C" __global__ void bam_records_len(BamParams P) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < P.n; r += (int64_t)gridDim.x * blockDim.x)
    bam_record<false>(P, r);
}
extern "C" __global__ void bam_records_write(BamParams P) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < P.n; r += (int64_t)gridDim.x * blockDim.x)
    bam_record<true>(P, r);
}
extern "C" __global__ void bam_offsets_close(BamParams P) {
  const int64_t n1 = P.n + 1;
  P.seq_off[P.n] = P.off[P.n];
  P.qual_off[P.n] = P.off[n1 + P.n];
  P.cig_off[P.n] = P.off[2 * n1 + P.n];
  P.md_off[P.n] = P.off[3 * n1 + P.n];
}

}  // namespace bamk

namespace {

uint32_t le32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// BGZF -> the decompressed BAM (pinned host memory), blocks inflated by threads
bqsr_status bgzf_inflate(const uint8_t* data, int64_t n, std::vector<uint8_t>& out) {
  struct Blk {
    int64_t src, csize, dst, isize;
  };
  std::vector<Blk> blks;
  int64_t p = 0, total = 0;
  while (p < n) {
    if (n - p < 18 || data[p] != 31 || data[p + 1] != 139 || data[p + 2] != 8 || !(data[p + 3] & 4))
      return fail(BQSR_ERR_SAM_PARSE, "BAM: not a BGZF block at byte " + std::to_string(p));
    // an untrusted file: every field is bounds-checked before it is read
    const int64_t xlen = data[p + 10] | (data[p + 11] << 8);
    const int64_t xend = p + 12 + xlen;
    if (xend > n) return fail(BQSR_ERR_SAM_PARSE, "BAM: truncated BGZF header at byte " + std::to_string(p));
    int64_t bsize = -1;
    for (int64_t q = p + 12; q + 4 <= xend;) {  // the BC subfield holds BSIZE
      const int64_t sl = data[q + 2] | (data[q + 3] << 8);
      if (q + 4 + sl > xend) return fail(BQSR_ERR_SAM_PARSE, "BAM: BGZF extra subfield overruns its header");
      if (data[q] == 'B' && data[q + 1] == 'C' && sl == 2) bsize = data[q + 4] | (data[q + 5] << 8);
      q += 4 + sl;
    }
    if (bsize < 0 || p + bsize + 1 > n) return fail(BQSR_ERR_SAM_PARSE, "BAM: BGZF block without BSIZE");
    const int64_t blen = bsize + 1;
    const int64_t hdr = 12 + xlen;
    if (blen < hdr + 8) return fail(BQSR_ERR_SAM_PARSE, "BAM: BGZF BSIZE smaller than its header");
    const int64_t isize = le32(data + p + blen - 4);
    if (isize > 65536) return fail(BQSR_ERR_SAM_PARSE, "BAM: BGZF ISIZE above 64 KiB");
    blks.push_back(Blk{p + hdr, blen - hdr - 8, total, isize});
    total += isize;
    p += blen;
  }
  out.resize((size_t)total + 64);
  std::atomic<int64_t> next{0};
  std::atomic<int> bad{0};
  auto work = [&]() {
    for (int64_t i; (i = next.fetch_add(1)) < (int64_t)blks.size();) {
      const Blk& k = blks[(size_t)i];
      if (k.isize == 0) continue;
      z_stream zs{};
      if (inflateInit2(&zs, -15) != Z_OK) {
        bad = 1;
        continue;
      }
      zs.next_in = (Bytef*)(data + k.src);
      zs.avail_in = (uInt)k.csize;
      zs.next_out = (Bytef*)(out.data() + k.dst);
      zs.avail_out = (uInt)k.isize;
      const int rc = inflate(&zs, Z_FINISH);
      const bool ok_len = rc == Z_STREAM_END && zs.total_out == (uLong)k.isize;
      inflateEnd(&zs);
      // the block's CRC32 of its uncompressed bytes (the 4 bytes before ISIZE)
      if (!ok_len || crc32(0L, out.data() + k.dst, (uInt)k.isize) != le32(data + k.src + k.csize)) bad = 1;
    }
  };
  const int nt = (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)std::thread::hardware_concurrency(),
                                                               std::min<int64_t>(16, (int64_t)blks.size())));
  std::vector<std::thread> th;
  for (int t = 0; t < nt; ++t) th.emplace_back(work);
  for (auto& t : th) t.join();
  if (bad) return fail(BQSR_ERR_SAM_PARSE, "BAM: a BGZF block does not inflate or fails its CRC32");
  out.resize((size_t)total);
  return BQSR_OK;
}

}  // namespace

bqsr_status bqsr_bam_parse(bqsr_context* ctx, const uint8_t* data, int64_t n, void* stream, bqsr_sam** out) {
  if (!ctx || !out || n < 0 || (n > 0 && !data)) return fail(BQSR_ERR_INVALID_ARG, "bqsr_bam_parse: bad arguments");
  HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = S(stream);
  std::vector<uint8_t> raw;
  bqsr_status st = bgzf_inflate(data, n, raw);
  if (st != BQSR_OK) return st;
  const int64_t m = (int64_t)raw.size();
  const uint8_t* u = raw.data();
  if (m < 12 || memcmp(u, "BAM\1", 4) != 0) return fail(BQSR_ERR_SAM_PARSE, "BAM: no BAM magic");
  const int64_t l_text = (int32_t)le32(u + 4);
  if (l_text < 0 || 8 + l_text + 4 > m) return fail(BQSR_ERR_SAM_PARSE, "BAM: bad header length");
  // the SAM header text (NULs allowed at its end), as bqsr_sam_parse reads it
  int64_t lt = l_text;
  while (lt > 0 && u[8 + lt - 1] == 0) --lt;
  SamHeader H;
  if ((st = parse_sam_header((const char*)u + 8, lt, &H)) != BQSR_OK) return st;
  int64_t p = 8 + l_text;
  const int64_t n_ref = (int32_t)le32(u + p);
  p += 4;
  std::map<std::string, int32_t> sq_index;
  for (size_t i = 0; i < H.sq_names.size(); ++i) sq_index.emplace(H.sq_names[i], (int32_t)i);
  std::vector<int32_t> ref_sq;
  for (int64_t i = 0; i < n_ref; ++i) {
    if (p + 4 > m) return fail(BQSR_ERR_SAM_PARSE, "BAM: truncated reference list");
    const int64_t l_name = (int32_t)le32(u + p);
    if (l_name < 1 || p + 4 + l_name + 4 > m) return fail(BQSR_ERR_SAM_PARSE, "BAM: bad reference name");
    const std::string name((const char*)u + p + 4, (size_t)(l_name - 1));
    auto it = sq_index.find(name);  // referenceName only for a header @SQ name (records.read_sam)
    ref_sq.push_back(it == sq_index.end() ? -1 : it->second);
    p += 4 + l_name + 4;
  }
  // records: offsets by their block_size fields
  std::vector<uint64_t> rec;
  const int64_t body = p;
  while (p < m) {
    if (p + 4 > m) return fail(BQSR_ERR_SAM_PARSE, "BAM: truncated record");
    const int64_t bs = (int32_t)le32(u + p);
    if (bs < 32 || p + 4 + bs > m) return fail(BQSR_ERR_SAM_PARSE, "BAM: bad record size at byte " + std::to_string(p));
    rec.push_back((uint64_t)(p - body));
    p += 4 + bs;
  }
  const int64_t nr = (int64_t)rec.size();
  rec.push_back((uint64_t)(m - body));

  std::unique_ptr<bqsr_sam> S_(new bqsr_sam);
  bqsr_sam* o = S_.get();
  o->ctx = ctx;
  o->from_bam = true;
  o->n_rg = (int32_t)H.rgh.value.size();
  o->rg_library.assign(H.rg_names.size(), std::string());
  o->rg_has_lb.assign(H.rg_names.size(), 0);
  for (size_t i = 0; i < H.rg_names.size(); ++i) {
    const auto& v = H.rg_lb[H.rg_names[i]];
    o->rg_has_lb[i] = v.first ? 1 : 0;
    o->rg_library[i] = v.second;
  }
  o->header = 0;
  o->n_text = m - body;
  HIP_TRY(hipMalloc(&o->d_text, (size_t)o->n_text + 64));
  std::vector<void*> tmp;
  struct Free {
    std::vector<void*>& v;
    ~Free() {
      for (void* q : v) (void)hipFree(q);
    }
  } free_tmp{tmp};
  if (o->n_text > 0) HIP_TRY(hipMemcpyAsync(o->d_text, u + body, (size_t)o->n_text, hipMemcpyHostToDevice, s));
  bamk::BamParams P{};
  P.buf = o->d_text;
  P.n = nr;
  P.n_ref = (int32_t)ref_sq.size();
  if ((st = sam_upload(tmp, (uint64_t**)&P.rec, rec, s)) != BQSR_OK) return st;
  if ((st = sam_upload(tmp, (int32_t**)&P.ref_sq, ref_sq.empty() ? std::vector<int32_t>{-1} : ref_sq, s)) != BQSR_OK)
    return st;
  if ((st = sam_names_upload(o->allocs, H.rgh, &P.rg, s)) != BQSR_OK) return st;
  if ((st = sam_alloc(tmp, &P.err, 1)) != BQSR_OK) return st;
  HIP_TRY(hipMemsetAsync(P.err, 0xFF, 8, s));
  if ((st = sam_alloc(tmp, &P.len, (size_t)(4 * nr))) != BQSR_OK) return st;
  if ((st = sam_alloc(tmp, &P.off, (size_t)(4 * (nr + 1)))) != BQSR_OK) return st;
  const unsigned g = sam_grid(nr, 256, ctx->n_cu * 16);
  if (nr > 0) hipLaunchKernelGGL(bamk::bam_records_len, dim3(g), dim3(256), 0, s, P);
  HIP_TRY(hipGetLastError());
  unsigned long long e_word = ~0ull;
  HIP_TRY(hipMemcpyAsync(&e_word, P.err, 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (e_word != ~0ull) {
    const uint32_t code = (uint32_t)(e_word & 0xFF);
    char buf[160];
    snprintf(buf, sizeof buf, "BAM record %lld: %s", (long long)(e_word >> 8),
             code == bamk::kBamTagType ? "MD / RG tag of a type whose text is not decoded (f, H, B)"
             : code == bamk::kBamTag   ? "malformed optional field"
                                       : "malformed record");
    return fail(code == bamk::kBamTagType ? BQSR_ERR_UNSUPPORTED : BQSR_ERR_SAM_PARSE, buf);
  }
  uint64_t* part;
  if ((st = sam_alloc(tmp, &part, (size_t)(nr / samk::kScanChunk + 2))) != BQSR_OK) return st;
  for (int c = 0; c < 4; ++c)
    if ((st = sam_scan(P.len + (size_t)c * nr, nr, P.off + (size_t)c * (nr + 1), part, s)) != BQSR_OK) return st;
  uint64_t tot[4] = {0, 0, 0, 0};
  for (int c = 0; c < 4 && nr > 0; ++c)
    HIP_TRY(hipMemcpyAsync(&tot[c], P.off + (size_t)c * (nr + 1) + nr, 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  o->n_reads = nr;
  o->seq_bytes = (int64_t)tot[0];
  o->qual_bytes = (int64_t)tot[1];
  o->cig_ops = (int64_t)tot[2];
  o->md_bytes = (int64_t)tot[3];
  const size_t n1 = (size_t)nr;
  if ((st = sam_alloc(o->allocs, &o->flags, n1)) != BQSR_OK || (st = sam_alloc(o->allocs, &o->rg_id, n1)) != BQSR_OK ||
      (st = sam_alloc(o->allocs, &o->ref, n1)) != BQSR_OK || (st = sam_alloc(o->allocs, &o->start, n1)) != BQSR_OK ||
      (st = sam_alloc(o->allocs, &o->sq_id, n1)) != BQSR_OK || (st = sam_alloc(o->allocs, &o->raw_flag, n1)) != BQSR_OK ||
      (st = sam_alloc(o->allocs, &o->seq_off, n1 + 1)) != BQSR_OK ||
      (st = sam_alloc(o->allocs, &o->seq, (size_t)o->seq_bytes)) != BQSR_OK ||
      (st = sam_alloc(o->allocs, &o->qual_off, n1 + 1)) != BQSR_OK ||
      (st = sam_alloc(o->allocs, &o->qual, (size_t)o->qual_bytes)) != BQSR_OK ||
      (st = sam_alloc(o->allocs, &o->cig_off, n1 + 1)) != BQSR_OK ||
      (st = sam_alloc(o->allocs, &o->cig, (size_t)o->cig_ops)) != BQSR_OK ||
      (st = sam_alloc(o->allocs, &o->md_off, n1 + 1)) != BQSR_OK ||
      (st = sam_alloc(o->allocs, &o->md, (size_t)o->md_bytes)) != BQSR_OK ||
      (st = sam_alloc(o->allocs, &o->line_span, 2 * n1)) != BQSR_OK ||
      (st = sam_alloc(o->allocs, &o->qual_span, 2 * n1)) != BQSR_OK)
    return st;
  P.flags = o->flags;
  P.rg_id = o->rg_id;
  P.ref = o->ref;
  P.sq_id = o->sq_id;
  P.raw_flag = o->raw_flag;
  P.start = o->start;
  P.seq_off = o->seq_off;
  P.seq = o->seq;
  P.qual_off = o->qual_off;
  P.qual = o->qual;
  P.cig_off = o->cig_off;
  P.cig = o->cig;
  P.md_off = o->md_off;
  P.md = o->md;
  P.line_span = o->line_span;
  if (nr > 0) {
    hipLaunchKernelGGL(bamk::bam_records_write, dim3(g), dim3(256), 0, s, P);
    hipLaunchKernelGGL(bamk::bam_offsets_close, dim3(1), dim3(1), 0, s, P);
  } else {
    HIP_TRY(hipMemsetAsync(o->seq_off, 0, 8, s));
    HIP_TRY(hipMemsetAsync(o->qual_off, 0, 8, s));
    HIP_TRY(hipMemsetAsync(o->cig_off, 0, 8, s));
    HIP_TRY(hipMemsetAsync(o->md_off, 0, 8, s));
  }
  HIP_TRY(hipGetLastError());
  // referenceName ids: first appearance order (as bqsr_sam_parse)
  const size_t nsq = H.sq_names.size();
  if (nsq > 0 && nr > 0) {
    unsigned long long* first;
    int32_t* rank_d;
    if ((st = sam_alloc(tmp, &first, nsq)) != BQSR_OK) return st;
    HIP_TRY(hipMemsetAsync(first, 0xFF, nsq * 8, s));
    hipLaunchKernelGGL(samk::sam_ref_first, dim3(g), dim3(256), 0, s, (const int32_t*)o->ref, nr, first);
    std::vector<unsigned long long> fh(nsq);
    HIP_TRY(hipMemcpyAsync(fh.data(), first, nsq * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    std::vector<int32_t> order;
    for (size_t i = 0; i < nsq; ++i)
      if (fh[i] != ~0ull) order.push_back((int32_t)i);
    std::sort(order.begin(), order.end(), [&](int32_t a, int32_t b) { return fh[a] < fh[b]; });
    std::vector<int32_t> rank(nsq, -1);
    for (size_t k = 0; k < order.size(); ++k) {
      rank[order[k]] = (int32_t)k;
      o->ref_names.push_back(H.sq_names[order[k]]);
    }
    if ((st = sam_upload(tmp, &rank_d, rank, s)) != BQSR_OK) return st;
    hipLaunchKernelGGL(samk::sam_ref_remap, dim3(g), dim3(256), 0, s, o->ref, nr, (const int32_t*)rank_d);
    HIP_TRY(hipGetLastError());
  }
  HIP_TRY(hipStreamSynchronize(s));
  *out = S_.release();
  return ok();
}
