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
  const uint8_t* buf;       // the decompressed BAM records
  const uint64_t* rec;      // [n + 1] record offsets (block_size field of record r at rec[r])
  int64_t n;
  const uint8_t* ref_blob;  // the binary reference list's names: ref_blob[ref_off[i], ref_off[i + 1])
  const uint64_t* ref_off;
  int32_t n_ref;
  uint64_t* len;            // [n] SAM line bytes of record r, '\n' included (pass 1)
  const uint64_t* off;      // [n + 1] their exclusive scan (pass 2)
  uint8_t* out;             // the SAM text: the header at [0, hdr), record r's line at hdr + off[r]
  int64_t hdr;
  unsigned long long* err;  // (record << 8) | code, the smallest wins
};

enum : uint32_t { kBamOk = 0, kBamRecord = 1, kBamTag = 2 };

__device__ __forceinline__ uint32_t rd32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
__device__ __forceinline__ uint16_t rd16(const uint8_t* p) { return (uint16_t)(p[0] | (p[1] << 8)); }

// writes (or, out == nullptr, counts) bytes at out[n]
struct Put {
  uint8_t* out;
  int64_t n;
  __device__ __forceinline__ void c(uint8_t v) {
    if (out) out[n] = v;
    ++n;
  }
  __device__ __forceinline__ void bytes(const uint8_t* p, int64_t k) {
    if (out)
      for (int64_t i = 0; i < k; ++i) out[n + i] = p[i];
    n += k;
  }
  __device__ void integer(int64_t v) {  // decimal text (Java's Integer / Long toString)
    uint8_t b[24];
    int m = 0;
    const bool neg = v < 0;
    uint64_t u = neg ? (uint64_t)(-(v + 1)) + 1 : (uint64_t)v;
    do {
      b[m++] = (uint8_t)('0' + u % 10);
      u /= 10;
    } while (u);
    if (neg) c('-');
    while (m) c(b[--m]);
  }
  __device__ void real(float f) { n += samk::java_float_text(f, out ? out + n : nullptr); }
};

// One BAM record as its SAM text line (htsjdk's SAMRecord of the record, as
// the SAM text of the same record would parse; the SAM spec's field order):
// QNAME FLAG RNAME POS MAPQ CIGAR RNEXT PNEXT TLEN SEQ QUAL, then every tag
// TG:TYPE:VALUE in record order -- integer types (c C s S i I) as "i", floats
// by Java's Float.toString, B arrays as "B:t,v,...".  The line then goes
// through the SAM record parser, so BAM and SAM input share one parse, the
// QUAL rewrite and the ADAM columns.
template <bool kWrite>
__device__ void bam_line(const BamParams& P, int64_t r) {
  const uint8_t* b = P.buf + P.rec[r];
  const int64_t bs = (int64_t)rd32(b);
  const int64_t end = 4 + bs;
  const int32_t refid = (int32_t)rd32(b + 4);
  const int32_t pos = (int32_t)rd32(b + 8);
  const int l_name = b[12];
  const int mapq = b[13];
  const int n_cig = rd16(b + 16);
  const uint32_t flag = rd16(b + 18);
  const int64_t l_seq = (int64_t)(int32_t)rd32(b + 20);
  const int32_t next_ref = (int32_t)rd32(b + 24);
  const int32_t next_pos = (int32_t)rd32(b + 28);
  const int32_t tlen = (int32_t)rd32(b + 32);
  const int64_t o_name = 36, o_cig = o_name + l_name, o_seq = o_cig + 4 * (int64_t)n_cig;
  const int64_t o_qual = o_seq + (l_seq + 1) / 2, o_tag = o_qual + l_seq;
  if (!kWrite && (bs < 32 || l_seq < 0 || o_tag > end || l_name < 1)) {
    atomicMin(P.err, ((unsigned long long)r << 8) | kBamRecord);
    P.len[r] = 0;
    return;
  }
  Put o{kWrite ? P.out + P.hdr + P.off[r] : nullptr, 0};
  auto ref_name = [&](int32_t id) {
    if (id >= 0 && id < P.n_ref) o.bytes(P.ref_blob + P.ref_off[id], (int64_t)(P.ref_off[id + 1] - P.ref_off[id]));
    else o.c('*');
  };
  o.bytes(b + o_name, l_name - 1);
  o.c('\t');
  o.integer(flag);
  o.c('\t');
  ref_name(refid);
  o.c('\t');
  o.integer((int64_t)pos + 1);
  o.c('\t');
  o.integer(mapq);
  o.c('\t');
  if (n_cig == 0) {
    o.c('*');
  } else {
    const char kOps[] = "MIDNSHP=X";
    for (int k = 0; k < n_cig; ++k) {
      const uint32_t e = rd32(b + o_cig + 4 * k);
      o.integer(e >> 4);
      o.c((e & 15u) < 9u ? (uint8_t)kOps[e & 15u] : (uint8_t)'?');
    }
  }
  o.c('\t');
  if (next_ref >= 0 && next_ref == refid) o.c('=');
  else ref_name(next_ref);
  o.c('\t');
  o.integer((int64_t)next_pos + 1);
  o.c('\t');
  o.integer(tlen);
  o.c('\t');
  if (l_seq == 0) {
    o.c('*');
  } else {
    const char kCodes[] = "=ACMGRSVTWYHKDBN";
    for (int64_t k = 0; k < l_seq; ++k) o.c((uint8_t)kCodes[(b[o_seq + (k >> 1)] >> ((k & 1) ? 0 : 4)) & 15]);
  }
  o.c('\t');
  if (l_seq == 0 || b[o_qual] == 0xFF) {
    o.c('*');
  } else {
    for (int64_t k = 0; k < l_seq; ++k) o.c((uint8_t)(b[o_qual + k] + 33));
  }
  for (int64_t p = o_tag; p < end;) {
    if (p + 3 > end) {
      if (!kWrite) atomicMin(P.err, ((unsigned long long)r << 8) | kBamTag);
      break;
    }
    const uint8_t ty = b[p + 2];
    const int64_t v = p + 3;
    int64_t sz;
    switch (ty) {
      case 'A': case 'c': case 'C': sz = 1; break;
      case 's': case 'S': sz = 2; break;
      case 'i': case 'I': case 'f': sz = 4; break;
      case 'Z': case 'H': {
        int64_t q = v;
        while (q < end && b[q]) ++q;
        sz = q - v + 1;
        break;
      }
      case 'B': {
        const uint8_t st = v + 5 <= end ? b[v] : 0;
        const int es = (st == 'c' || st == 'C') ? 1 : (st == 's' || st == 'S') ? 2 : (st == 'i' || st == 'I' || st == 'f') ? 4 : 0;
        sz = es && v + 5 <= end ? 5 + (int64_t)rd32(b + v + 1) * es : end;  // (unknown subtype: overruns below)
        break;
      }
      default: sz = end; break;
    }
    if (v + sz > end) {
      if (!kWrite) atomicMin(P.err, ((unsigned long long)r << 8) | kBamTag);
      break;
    }
    o.c('\t');
    o.c(b[p]);
    o.c(b[p + 1]);
    o.c(':');
    switch (ty) {
      case 'A': o.c('A'); o.c(':'); o.c(b[v]); break;
      case 'c': o.c('i'); o.c(':'); o.integer((int8_t)b[v]); break;
      case 'C': o.c('i'); o.c(':'); o.integer(b[v]); break;
      case 's': o.c('i'); o.c(':'); o.integer((int16_t)rd16(b + v)); break;
      case 'S': o.c('i'); o.c(':'); o.integer(rd16(b + v)); break;
      case 'i': o.c('i'); o.c(':'); o.integer((int32_t)rd32(b + v)); break;
      case 'I': o.c('i'); o.c(':'); o.integer(rd32(b + v)); break;
      case 'f': {
        const uint32_t w = rd32(b + v);
        float fv;
        __builtin_memcpy(&fv, &w, 4);
        o.c('f'); o.c(':'); o.real(fv);
        break;
      }
      case 'Z': case 'H': o.c(ty); o.c(':'); o.bytes(b + v, sz - 1); break;
      case 'B': {
        const uint8_t st = b[v];
        const int64_t cnt = rd32(b + v + 1);
        o.c('B'); o.c(':'); o.c(st);
        for (int64_t k = 0; k < cnt; ++k) {
          const uint8_t* e = b + v + 5;
          o.c(',');
          switch (st) {
            case 'c': o.integer((int8_t)e[k]); break;
            case 'C': o.integer(e[k]); break;
            case 's': o.integer((int16_t)rd16(e + 2 * k)); break;
            case 'S': o.integer(rd16(e + 2 * k)); break;
            case 'i': o.integer((int32_t)rd32(e + 4 * k)); break;
            case 'I': o.integer(rd32(e + 4 * k)); break;
            default: {
              const uint32_t w = rd32(e + 4 * k);
              float fv;
              __builtin_memcpy(&fv, &w, 4);
              o.real(fv);
            }
          }
        }
        break;
      }
    }
    p = v + sz;
  }
  o.c('\n');
  if (!kWrite) P.len[r] = (uint64_t)o.n;
}

extern "C" __global__ void bam_lines_len(BamParams P) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < P.n; r += (int64_t)gridDim.x * blockDim.x)
    bam_line<false>(P, r);
}
extern "C" __global__ void bam_lines_write(BamParams P) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < P.n; r += (int64_t)gridDim.x * blockDim.x)
    bam_line<true>(P, r);
}

}  // namespace bamk

namespace {

uint32_t le32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

struct BgzfBlk {
  int64_t src, csize, dst, isize;
};

// Raw DEFLATE + CRC32 of one BGZF block.  libdeflate (the system's
// libdeflate.so.0, loaded at run time: whole-buffer inflate and a folded
// CRC32, ~3x zlib's per thread) when the image has it, zlib otherwise.
struct Deflate {
  typedef void* (*alloc_fn)();
  typedef int (*inflate_fn)(void*, const void*, size_t, void*, size_t, size_t*);
  typedef void (*free_fn)(void*);
  typedef uint32_t (*crc_fn)(uint32_t, const void*, size_t);
  alloc_fn alloc = nullptr;
  inflate_fn inflate = nullptr;
  free_fn free = nullptr;
  crc_fn crc = nullptr;
  static const Deflate& get() {
    static const Deflate d = [] {
      Deflate x;
      const char* off = getenv("ADAM_BQSR_LIBDEFLATE");
      if (off && strcmp(off, "0") == 0) return x;
      void* h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
      if (!h) return x;
      x.alloc = (alloc_fn)dlsym(h, "libdeflate_alloc_decompressor");
      x.inflate = (inflate_fn)dlsym(h, "libdeflate_deflate_decompress");
      x.free = (free_fn)dlsym(h, "libdeflate_free_decompressor");
      x.crc = (crc_fn)dlsym(h, "libdeflate_crc32");
      if (!x.alloc || !x.inflate || !x.free || !x.crc) x = Deflate{};
      return x;
    }();
    return d;
  }
  bool ok() const { return alloc != nullptr; }
};
// one block into o (isize bytes); false: it does not inflate to exactly isize or fails its CRC32
bool inflate_block(const Deflate& D, void* dec, const uint8_t* in, int64_t csize, uint8_t* o, int64_t isize,
                   uint32_t crc_want) {
  if (D.ok()) {
    size_t got = 0;
    if (D.inflate(dec, in, (size_t)csize, o, (size_t)isize, &got) != 0 || got != (size_t)isize) return false;
    return D.crc(0, o, (size_t)isize) == crc_want;
  }
  z_stream zs{};
  if (inflateInit2(&zs, -15) != Z_OK) return false;
  zs.next_in = (Bytef*)in;
  zs.avail_in = (uInt)csize;
  zs.next_out = (Bytef*)o;
  zs.avail_out = (uInt)isize;
  const int rc = inflate(&zs, Z_FINISH);
  const bool ok_len = rc == Z_STREAM_END && zs.total_out == (uLong)isize;
  inflateEnd(&zs);
  return ok_len && crc32(0L, o, (uInt)isize) == crc_want;
}

// ADAM_BQSR_TIMING=1: a BAM parse prints its host / device phases to stderr
bool bam_timing() {
  static const bool v = [] {
    const char* e = getenv("ADAM_BQSR_TIMING");
    return e && strcmp(e, "1") == 0;
  }();
  return v;
}
double now_s() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
struct InflateTimes {
  double wait = 0, inflate = 0, host = 0, drain = 0, read = 0;
};

// The BGZF block list of a file (its headers walked in order; an untrusted
// file: every field is bounds-checked before it is read) and the inflated size.
bqsr_status bgzf_blocks(const uint8_t* data, int64_t n, std::vector<BgzfBlk>& blks, int64_t& total) {
  int64_t p = 0;
  total = 0;
  while (p < n) {
    if (n - p < 18 || data[p] != 31 || data[p + 1] != 139 || data[p + 2] != 8 || !(data[p + 3] & 4))
      return fail(BQSR_ERR_SAM_PARSE, "BAM: not a BGZF block at byte " + std::to_string(p));
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
    blks.push_back(BgzfBlk{p + hdr, blen - hdr - 8, total, isize});
    total += isize;
    p += blen;
  }
  return BQSR_OK;
}

// Inflate straight to the device: runs of whole blocks (at most kStageChunk
// bytes inflated) are inflated by host threads into the context's pinned
// ring and each run is DMA'd to d_out + its offset, while one more thread
// reads the previous run (`host(buf, off, len)`, in stream order: the
// header, the records' block_size chain) and the threads inflate the next.
// No pageable copy of the whole inflated stream: first-touching gigabytes of
// fresh pages was most of a BAM parse.
template <class Host>
bqsr_status bgzf_inflate_device(bqsr_context* ctx, const uint8_t* data, const std::vector<BgzfBlk>& blks,
                                uint8_t* d_out, hipStream_t s, InflateTimes& T, Host&& host) {
  std::lock_guard<std::mutex> lock(ctx->stage_mu);
  bqsr_status st = stage_ring(ctx);
  if (st != BQSR_OK) return st;
  const int nt = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  const Deflate& D = Deflate::get();
  std::thread reader;  // host() over the previous run
  struct Join {
    std::thread& t;
    ~Join() {
      if (t.joinable()) t.join();  // (every return path: a running reader is waited for)
    }
  } join_guard{reader};
  bqsr_status rst = BQSR_OK;
  double t_read = 0;
  const auto join_reader = [&]() {
    if (reader.joinable()) reader.join();
  };
  size_t i = 0;
  int k = 0;
  while (i < blks.size()) {
    size_t j = i;
    int64_t len = 0;
    while (j < blks.size() && len + blks[j].isize <= (int64_t)kStageChunk) len += blks[j++].isize;  // (isize <= 64 KiB)
    const int64_t dst0 = blks[i].dst;
    double t0 = now_s();
    // the slot's previous run: DMA done and read (the reader of the run before
    // this one's predecessor has been joined already, the predecessor's may run on)
    HIP_TRY(hipEventSynchronize(ctx->stage_ev[k]));
    double t1 = now_s();
    T.wait += t1 - t0;
    uint8_t* buf = ctx->stage[k];
    std::atomic<size_t> next{i};
    std::atomic<int> bad{0};
    auto work = [&]() {
      void* dec = D.ok() ? D.alloc() : nullptr;
      if (D.ok() && !dec) {
        bad = 1;
        return;
      }
      for (size_t b; (b = next.fetch_add(1)) < j;) {
        const BgzfBlk& z = blks[b];
        if (z.isize == 0) continue;
        // (the block's CRC32 of its uncompressed bytes: the 4 bytes before ISIZE)
        if (!inflate_block(D, dec, data + z.src, z.csize, buf + (z.dst - dst0), z.isize, le32(data + z.src + z.csize)))
          bad = 1;
      }
      if (dec) D.free(dec);
    };
    {
      std::vector<std::thread> th;
      const int nw = (int)std::min<size_t>((size_t)nt, j - i);
      for (int t = 0; t < nw; ++t) th.emplace_back(work);
      for (auto& t : th) t.join();
    }
    t0 = now_s();
    T.inflate += t0 - t1;
    join_reader();  // the previous run's reader (stream order)
    T.host += now_s() - t0;
    if (bad || rst != BQSR_OK) {
      (void)hipStreamSynchronize(s);
      return rst != BQSR_OK ? rst : fail(BQSR_ERR_SAM_PARSE, "BAM: a BGZF block does not inflate or fails its CRC32");
    }
    if (len > 0) {
      HIP_TRY(hipMemcpyAsync(d_out + dst0, buf, (size_t)len, hipMemcpyHostToDevice, s));
      HIP_TRY(hipEventRecord(ctx->stage_ev[k], s));
    }
    reader = std::thread([&, buf, dst0, len] {
      const double r0 = now_s();
      rst = host(buf, dst0, len);
      t_read += now_s() - r0;
    });
    i = j;
    k ^= 1;
    // the next run reuses slot k: its DMA (event) and its reader -- joined above
    // before this run's reader started -- are both done once the event is
  }
  {
    const double t0 = now_s();
    join_reader();
    T.host += now_s() - t0;
  }
  const double t0 = now_s();
  HIP_TRY(hipStreamSynchronize(s));
  T.drain += now_s() - t0;
  T.read = t_read;
  return rst;
}

// The BAM header (magic, SAM text, binary reference list) from the first m
// bytes of the inflated stream: 1 parsed (body = the first record's offset),
// 0 more bytes needed (`all`: there are none -- an error then).
struct BamHead {
  int64_t l_text = 0, body = 0;
  std::vector<uint8_t> ref_blob;
  std::vector<uint64_t> ref_off{0};
};
int bam_head(const uint8_t* u, int64_t m, bool all, BamHead& H, bqsr_status& st) {
  st = BQSR_OK;
  const auto need = [&](const char* what) {
    if (!all) return 0;
    st = fail(BQSR_ERR_SAM_PARSE, what);
    return -1;
  };
  if (m >= 4 && memcmp(u, "BAM\1", 4) != 0) return (st = fail(BQSR_ERR_SAM_PARSE, "BAM: no BAM magic")), -1;
  if (m < 12) return need("BAM: no BAM magic");
  H.l_text = (int32_t)le32(u + 4);
  if (H.l_text < 0) return (st = fail(BQSR_ERR_SAM_PARSE, "BAM: bad header length")), -1;
  if (8 + H.l_text + 4 > m) return need("BAM: bad header length");
  int64_t p = 8 + H.l_text;
  const int64_t n_ref = (int32_t)le32(u + p);
  p += 4;
  // the binary reference list's names: a record's RNAME / RNEXT text
  // (referenceName then only for a header @SQ name, as for SAM text)
  H.ref_blob.clear();
  H.ref_off.assign(1, 0);
  for (int64_t i = 0; i < n_ref; ++i) {
    if (p + 4 > m) return need("BAM: truncated reference list");
    const int64_t l_name = (int32_t)le32(u + p);
    if (l_name < 1) return (st = fail(BQSR_ERR_SAM_PARSE, "BAM: bad reference name")), -1;
    if (p + 4 + l_name + 4 > m) return need("BAM: bad reference name");
    H.ref_blob.insert(H.ref_blob.end(), u + p + 4, u + p + 4 + (l_name - 1));
    H.ref_off.push_back(H.ref_blob.size());
    p += 4 + l_name + 4;
  }
  H.body = p;
  return 1;
}

// Record offsets by their block_size fields, over the stream's runs in order
// (a field may straddle two runs).
struct RecScan {
  int64_t body = 0, p = 0;  // p: the next record's stream offset
  uint8_t pend[4];
  int pend_n = 0;
  std::vector<uint64_t> rec;
  bool field(uint32_t v) {
    const int64_t bs = (int32_t)v;
    if (bs < 32) return false;
    rec.push_back((uint64_t)(p - body));
    p += 4 + bs;
    return true;
  }
  bqsr_status consume(const uint8_t* buf, int64_t off, int64_t len) {
    const int64_t end = off + len;
    if (pend_n > 0) {
      int64_t q = off;
      while (pend_n < 4 && q < end) pend[pend_n++] = buf[q++ - off];
      if (pend_n < 4) return BQSR_OK;
      pend_n = 0;
      if (!field(le32(pend))) return bad();
    }
    while (p + 4 <= end) {
      if (p < off) return bad();  // (cannot happen: p passed a run's end only as a pending field)
      __builtin_prefetch(buf + (p - off) + 2048);  // the chain's loads depend on each other: fetch ahead
      if (!field(le32(buf + (p - off)))) return bad();
    }
    for (int64_t q = std::max(p, off); q < end; ++q) pend[pend_n++] = buf[q - off];
    return BQSR_OK;
  }
  bqsr_status bad() const { return fail(BQSR_ERR_SAM_PARSE, "BAM: bad record size at byte " + std::to_string(p)); }
};

// The device form (bgzf_inflate.hip): the compressed file uploaded once, a
// thread per BGZF block inflating it into d_raw, the header read back, the
// records' offsets found and checked on the device (*d_rec, n + 1 entries,
// from BH.body).  ok = false when it declines -- a block that does not
// inflate or fails its CRC32, a chain the check rejects, a header it cannot
// read -- and the caller runs the host form, which reports the file's error
// as before.
bqsr_status bam_inflate_device(bqsr_context* ctx, const uint8_t* data, int64_t n, const std::vector<BgzfBlk>& blks,
                               int64_t m, uint8_t* d_raw, hipStream_t s, std::vector<void*>& tmp, BamHead& BH,
                               SamHeader& H, std::string& hdr, uint64_t** d_rec, int64_t& nr, bool& ok) {
  ok = false;
  const int64_t nb = (int64_t)blks.size();
  std::vector<bgzfk::Blk> hb((size_t)nb);
  for (int64_t i = 0; i < nb; ++i) {
    const BgzfBlk& k = blks[(size_t)i];
    hb[(size_t)i] = bgzfk::Blk{k.src, k.csize, k.dst, (int32_t)k.isize, (uint32_t)le32(data + k.src + k.csize)};
  }
  bqsr_status st;
  uint8_t* d_comp;
  bgzfk::Blk* d_blk;
  int32_t* d_status;
  if ((st = sam_alloc(tmp, &d_comp, (size_t)n + 256)) != BQSR_OK || (st = sam_upload(tmp, &d_blk, hb, s)) != BQSR_OK ||
      (st = sam_alloc(tmp, &d_status, (size_t)std::max<int64_t>(1, nb))) != BQSR_OK)
    return st;
  if ((st = upload_staged(ctx, d_comp, data, (size_t)n, s)) != BQSR_OK) return st;
  {  // symbols, then the bytes assembled a block a workgroup in LDS (+ CRC)
    // in runs of whole blocks of at most kTokRun output bytes (1 GiB;
    // ADAM_BQSR_BGZF_RUN overrides it, for the tests), one symbol buffer (4 B
    // a byte of the run's output at most) reused across runs
    int64_t kTokRun = int64_t(1) << 30;
    if (const char* e = getenv("ADAM_BQSR_BGZF_RUN")) kTokRun = std::max<int64_t>(1, atoll(e));
    int64_t cap = 1;
    for (int64_t b0 = 0, b1; b0 < nb; b0 = b1) {
      for (b1 = b0 + 1; b1 < nb && hb[(size_t)b1].dst + hb[(size_t)b1].isize - hb[(size_t)b0].dst <= kTokRun;) ++b1;
      cap = std::max<int64_t>(cap, hb[(size_t)b1 - 1].dst + hb[(size_t)b1 - 1].isize - hb[(size_t)b0].dst);
    }
    uint32_t* d_tok;
    int32_t* d_ntok;
    if ((st = sam_alloc(tmp, &d_tok, (size_t)cap)) != BQSR_OK ||
        (st = sam_alloc(tmp, &d_ntok, (size_t)std::max<int64_t>(1, nb))) != BQSR_OK)
      return st;
    for (int64_t b0 = 0, b1; b0 < nb; b0 = b1) {
      for (b1 = b0 + 1; b1 < nb && hb[(size_t)b1].dst + hb[(size_t)b1].isize - hb[(size_t)b0].dst <= kTokRun;) ++b1;
      const int64_t nr_b = b1 - b0, tok0 = hb[(size_t)b0].dst;
      if (nr_b <= (int64_t)ctx->n_cu * 2 * bgzfk::kInfThreads)  // (all in flight at once)
        hipLaunchKernelGGL(bgzfk::bgzf_tokens_kernel<bgzfk::kInfThreads>,
                           dim3((unsigned)((nr_b + bgzfk::kInfThreads - 1) / bgzfk::kInfThreads)), dim3(bgzfk::kInfThreads),
                           0, s, (const uint8_t*)d_comp, (const bgzfk::Blk*)d_blk + b0, nr_b, d_tok, tok0, d_ntok + b0,
                           d_status + b0);
      else
        hipLaunchKernelGGL(bgzfk::bgzf_tokens_kernel<bgzfk::kInfThreadsDeep>,
                           dim3((unsigned)((nr_b + bgzfk::kInfThreadsDeep - 1) / bgzfk::kInfThreadsDeep)),
                           dim3(bgzfk::kInfThreadsDeep), 0, s, (const uint8_t*)d_comp, (const bgzfk::Blk*)d_blk + b0, nr_b,
                           d_tok, tok0, d_ntok + b0, d_status + b0);
      HIP_TRY(hipGetLastError());
      hipLaunchKernelGGL(bgzfk::bgzf_resolve_kernel, dim3((unsigned)nr_b), dim3(bgzfk::kResThreads), 0, s,
                         (const bgzfk::Blk*)d_blk + b0, (const uint32_t*)d_tok, tok0, (const int32_t*)d_ntok + b0, d_raw,
                         d_status + b0);
      HIP_TRY(hipGetLastError());
    }
  }
  std::vector<int32_t> hs((size_t)std::max<int64_t>(1, nb), 0);
  if (nb > 0) HIP_TRY(hipMemcpyAsync(hs.data(), d_status, (size_t)nb * 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  for (int64_t i = 0; i < nb; ++i)
    if (hs[(size_t)i] != bgzfk::kInfOk) return BQSR_OK;  // (the host form reports the block)
  // the header, read back until it parses
  std::vector<uint8_t> head;
  for (int64_t want = std::min<int64_t>(m, 1 << 16);; want = std::min<int64_t>(m, want * 4)) {
    head.resize((size_t)want);
    HIP_TRY(hipMemcpy(head.data(), d_raw, (size_t)want, hipMemcpyDeviceToHost));
    bqsr_status e;
    const int r = bam_head(head.data(), want, want == m, BH, e);
    if (r < 0) return BQSR_OK;
    if (r == 1) break;
  }
  int64_t lt = BH.l_text;
  while (lt > 0 && head[(size_t)(8 + lt - 1)] == 0) --lt;
  if (parse_sam_header((const char*)head.data() + 8, lt, &H) != BQSR_OK) return BQSR_OK;
  hdr.assign((const char*)head.data() + 8, (size_t)lt);
  // the records: each block's guess and walk, the chain check, the offsets
  bgzfk::ChainParams C{};
  C.u = d_raw;
  C.m = m;
  C.body = BH.body;
  C.blks = d_blk;
  C.n_blk = nb;
  C.n_ref = (int32_t)((int64_t)BH.ref_off.size() - 1);
  uint64_t *part, *base;
  if ((st = sam_alloc(tmp, &C.guess, (size_t)std::max<int64_t>(1, nb))) != BQSR_OK ||
      (st = sam_alloc(tmp, &C.exit, (size_t)std::max<int64_t>(1, nb))) != BQSR_OK ||
      (st = sam_alloc(tmp, &C.count, (size_t)std::max<int64_t>(1, nb))) != BQSR_OK ||
      (st = sam_alloc(tmp, &base, (size_t)nb + 1)) != BQSR_OK ||
      (st = sam_alloc(tmp, &part, (size_t)(nb / samk::kScanChunk + 2))) != BQSR_OK ||
      (st = sam_alloc(tmp, &C.bad, 1)) != BQSR_OK)
    return st;
  HIP_TRY(hipMemsetAsync(C.bad, 0, 4, s));
  const unsigned gb = (unsigned)std::max<int64_t>(1, (nb + 63) / 64);
  if (nb > 0) {
    hipLaunchKernelGGL(bgzfk::bam_chain_guess, dim3(gb), dim3(64), 0, s, C);
    hipLaunchKernelGGL(bgzfk::bam_chain_check, dim3(gb), dim3(64), 0, s, C);
  }
  HIP_TRY(hipGetLastError());
  if ((st = sam_scan(C.count, nb, base, part, s)) != BQSR_OK) return st;
  int32_t bad = 0;
  uint64_t total = 0;
  HIP_TRY(hipMemcpyAsync(&bad, C.bad, 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(&total, base + nb, 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (bad) return BQSR_OK;
  nr = (int64_t)total;
  uint64_t* rec;
  if ((st = sam_alloc(tmp, &rec, (size_t)nr + 1)) != BQSR_OK) return st;
  C.base = base;
  C.rec = rec;
  if (nb > 0) hipLaunchKernelGGL(bgzfk::bam_chain_write, dim3(gb), dim3(64), 0, s, C);
  HIP_TRY(hipGetLastError());
  const uint64_t end = (uint64_t)(m - BH.body);
  HIP_TRY(hipMemcpyAsync(rec + nr, &end, 8, hipMemcpyHostToDevice, s));
  HIP_TRY(hipStreamSynchronize(s));
  *d_rec = rec;
  ok = true;
  return BQSR_OK;
}

}  // namespace

bqsr_status bqsr_bam_parse(bqsr_context* ctx, const uint8_t* data, int64_t n, void* stream, bqsr_sam** out) {
  if (!ctx || !out || n < 0 || (n > 0 && !data)) return fail(BQSR_ERR_INVALID_ARG, "bqsr_bam_parse: bad arguments");
  HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = S(stream);
  const double t_start = now_s();
  std::vector<BgzfBlk> blks;
  int64_t m = 0;
  bqsr_status st = bgzf_blocks(data, n, blks, m);
  const double t_blocks = now_s();
  if (st != BQSR_OK) return st;
  if (m < 12) return fail(BQSR_ERR_SAM_PARSE, "BAM: no BAM magic");
  std::vector<void*> tmp;
  struct Free {
    std::vector<void*>& v;
    ~Free() {
      for (void* q : v) (void)hipFree(q);
    }
  } free_tmp{tmp};
  uint8_t* d_raw;  // the whole inflated stream; the records start at H.body
  if ((st = sam_alloc(tmp, &d_raw, (size_t)m + 64)) != BQSR_OK) return st;
  HIP_TRY(hipMemsetAsync(d_raw + m, 0, 64, s));
  // on the host, as the runs pass: the header bytes until it parses, then the record offsets
  BamHead BH;
  SamHeader H;
  std::string hdr;
  std::vector<uint8_t> head;
  bool have_head = false;
  RecScan scan;
  InflateTimes IT;
  const double t_alloc = now_s();
  uint64_t* d_rec = nullptr;  // the records' offsets on the device (the device form), else uploaded from scan.rec
  int64_t nr_dev = 0;
  bool dev = false;
  if (ctx->tune_bgzf && (st = bam_inflate_device(ctx, data, n, blks, m, d_raw, s, tmp, BH, H, hdr, &d_rec, nr_dev, dev)) != BQSR_OK)
    return st;
  if (!dev) {
  st = bgzf_inflate_device(ctx, data, blks, d_raw, s, IT, [&](const uint8_t* buf, int64_t off, int64_t len) -> bqsr_status {
    if (have_head) return scan.consume(buf, off, len);
    head.insert(head.end(), buf, buf + len);
    bqsr_status e;
    const int r = bam_head(head.data(), (int64_t)head.size(), off + len == m, BH, e);
    if (r < 0) return e;
    if (r == 0) return BQSR_OK;
    have_head = true;
    // the SAM header text (NULs allowed at its end), as bqsr_sam_parse reads it
    int64_t lt = BH.l_text;
    while (lt > 0 && head[(size_t)(8 + lt - 1)] == 0) --lt;
    if ((e = parse_sam_header((const char*)head.data() + 8, lt, &H)) != BQSR_OK) return e;
    hdr.assign((const char*)head.data() + 8, (size_t)lt);
    scan.body = scan.p = BH.body;
    e = scan.consume(head.data(), 0, (int64_t)head.size());
    std::vector<uint8_t>().swap(head);
    return e;
  });
  if (st != BQSR_OK) return st;
  if (!have_head) return fail(BQSR_ERR_SAM_PARSE, "BAM: truncated header");
  if (scan.pend_n > 0 || scan.p < m) return fail(BQSR_ERR_SAM_PARSE, "BAM: truncated record");
  if (scan.p > m) {  // the last record overruns the stream
    scan.p = BH.body + (int64_t)scan.rec.back();
    return scan.bad();
  }
  }  // (host form)
  const double t_inflated = now_s();
  const int64_t body = BH.body;
  std::vector<uint64_t>& rec = scan.rec;
  std::vector<uint8_t>& ref_blob = BH.ref_blob;
  std::vector<uint64_t>& ref_off = BH.ref_off;
  const int64_t n_ref = (int64_t)ref_off.size() - 1;
  const int64_t nr = dev ? nr_dev : (int64_t)rec.size();
  if (!dev) rec.push_back((uint64_t)(m - body));
  // the header text, newline-terminated, then the records' SAM lines
  if (!hdr.empty() && hdr.back() != '\n') hdr.push_back('\n');
  H.body = (int64_t)hdr.size();
  bamk::BamParams P{};
  P.buf = d_raw + body;
  P.n = nr;
  P.n_ref = (int32_t)n_ref;
  P.hdr = H.body;
  if (dev)
    P.rec = d_rec;
  else if ((st = sam_upload(tmp, (uint64_t**)&P.rec, rec, s)) != BQSR_OK)
    return st;
  if ((st = sam_upload(tmp, (uint8_t**)&P.ref_blob, ref_blob.empty() ? std::vector<uint8_t>{0} : ref_blob, s)) != BQSR_OK)
    return st;
  if ((st = sam_upload(tmp, (uint64_t**)&P.ref_off, ref_off, s)) != BQSR_OK) return st;
  if ((st = sam_alloc(tmp, &P.err, 1)) != BQSR_OK) return st;
  HIP_TRY(hipMemsetAsync(P.err, 0xFF, 8, s));
  uint64_t *len, *off, *part;
  if ((st = sam_alloc(tmp, &len, (size_t)nr)) != BQSR_OK || (st = sam_alloc(tmp, &off, (size_t)nr + 1)) != BQSR_OK ||
      (st = sam_alloc(tmp, &part, (size_t)(nr / samk::kScanChunk + 2))) != BQSR_OK)
    return st;
  P.len = len;
  P.off = off;
  const unsigned g = sam_grid(nr, 256, ctx->n_cu * 16);
  if (nr > 0) hipLaunchKernelGGL(bamk::bam_lines_len, dim3(g), dim3(256), 0, s, P);
  HIP_TRY(hipGetLastError());
  if ((st = sam_scan(len, nr, off, part, s)) != BQSR_OK) return st;
  unsigned long long e_word = ~0ull;
  uint64_t body_bytes = 0;
  HIP_TRY(hipMemcpyAsync(&e_word, P.err, 8, hipMemcpyDeviceToHost, s));
  if (nr > 0) HIP_TRY(hipMemcpyAsync(&body_bytes, off + nr, 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (e_word != ~0ull) {
    const uint32_t code = (uint32_t)(e_word & 0xFF);
    char buf[160];
    snprintf(buf, sizeof buf, "BAM record %lld: %s", (long long)(e_word >> 8),
             code == bamk::kBamTag ? "malformed optional field" : "malformed record");
    return fail(BQSR_ERR_SAM_PARSE, buf);
  }
  const int64_t n_text = H.body + (int64_t)body_bytes;
  uint8_t* d_text = nullptr;
  HIP_TRY(hipMalloc(&d_text, (size_t)n_text + 64));
  hipError_t e = hipMemsetAsync(d_text + n_text, 0, 64, s);
  if (e == hipSuccess && H.body > 0) e = hipMemcpyAsync(d_text, hdr.data(), hdr.size(), hipMemcpyHostToDevice, s);
  P.out = d_text;
  if (e == hipSuccess && nr > 0) {
    hipLaunchKernelGGL(bamk::bam_lines_write, dim3(g), dim3(256), 0, s, P);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipStreamSynchronize(s);  // (the header copy reads `hdr`)
  if (e != hipSuccess) {
    (void)hipFree(d_text);
    return fail(BQSR_ERR_DEVICE, std::string("bqsr_bam_parse: ") + hipGetErrorString(e));
  }
  const double t_lines = now_s();
  st = sam_parse_device(ctx, H, hdr.data(), d_text, n_text, s, true, out);  // (owns d_text from here)
  if (bam_timing())
    fprintf(stderr,
            "[bam_parse] %lld reads, %.2f GB inflated (%s): blocks %.3f, alloc %.3f, runs %.3f (slot waits %.3f, "
            "inflate %.3f, reader wait %.3f (reading %.3f), drain %.3f), lines %.3f, SAM parse %.3f s\n",
            (long long)nr, m / 1e9, dev ? "device" : Deflate::get().ok() ? "libdeflate" : "zlib", t_blocks - t_start, t_alloc - t_blocks, t_inflated - t_alloc, IT.wait, IT.inflate,
            IT.host, IT.read, IT.drain, t_lines - t_inflated, now_s() - t_lines);
  return st;
}
