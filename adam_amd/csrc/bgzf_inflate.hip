// bgzf_inflate.hip -- BAM's BGZF blocks inflated on the device, and the BAM
// records found in the inflated stream there (the reference
// reads BAM through Hadoop-BAM / htsjdk, core/rdd/AdamContext.scala:122-137,
// whose BlockGunzipper inflates one BGZF block at a time).
//
// A BGZF file is a chain of gzip members of at most 64 KiB inflated each; no
// DEFLATE back-reference crosses a member, so every block inflates on its own:
// a thread per block (bgzf_inflate_kernel), its Huffman tables in the
// thread's slice of LDS, the output written straight to the block's place in
// the inflated stream (the host's prefix sum of the blocks' ISIZE), and the
// CRC32 of the member folded as the bytes are produced (the block is rejected
// as the host path rejects it: a code that does not decode, an overrun of
// ISIZE, a short output, a CRC mismatch).
//
// The records' offsets (a chain of block_size fields from the first record
// after the header) are found without walking the chain in order: each block
// guesses the first record that starts inside it (the first offset whose
// fixed fields and the next record's are plausible), walks its records to the
// first start past its end, and the guesses are accepted only if every
// block's walk lands exactly on the next guessing block's guess (the blocks
// between without one) and the last lands on the end of the stream.  The
// first block's start is the header's end, so an accepted chain IS the
// chain: any implausible, damaged or unusual file fails the check and the
// caller takes the host path, which reports errors as before.
//
// Measured (profiles/r06t_bgzf_device_inflate.txt): correct on every DEFLATE
// block form, but a thread per block -- 64 blocks a wavefront in lock step,
// one wavefront a CU (its tables take 99 KB of LDS), each symbol a chain of
// dependent LDS and global round trips -- inflates 0.43 GB in 189 ms where 16
// libdeflate threads take 57 ms; the record chain costs 0.5 ms.  So the host
// form stays the default (BQSR_TUNE_BGZF 0) and this one is selectable.
//
// Included by bqsr_capi.cpp before bam_ingest.hip.

namespace bgzfk {

struct Blk {          // one BGZF member
  int64_t src;        // its raw DEFLATE data in the compressed file
  int64_t csize;      // bytes of it
  int64_t dst;        // its output's offset in the inflated stream
  int32_t isize;      // bytes it inflates to (<= 65536)
  uint32_t crc;       // CRC32 of those bytes (the member's trailer)
};

constexpr int kInfThreads = 64;  // a wavefront per workgroup, a thread per block
enum : int32_t { kInfOk = 0, kInfBadCode = 1, kInfOverrun = 2, kInfShort = 3, kInfCrc = 4, kInfBadBlock = 5 };

// canonical Huffman code of a DEFLATE block (RFC 1951 §3.2.2): symbols by
// code, counted per length (decoded bit by bit, the code's bits MSB first)
struct Huff {
  uint16_t count[16];
  uint16_t sym[288];
};
// a thread's LDS: the literal / length and distance codes, the code lengths
// being read, and the construction's offsets
struct InfLds {
  Huff lit, dist;
  uint8_t len[320];
  uint16_t offs[16];
};

__constant__ uint16_t kLenBase[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31,
                                      35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ uint8_t kLenExtra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ uint16_t kDistBase[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129,
                                       193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
__constant__ uint8_t kDistExtra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
__constant__ uint8_t kClOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// LSB-first bit reader over one member's compressed bytes [p, end)
struct Bits {
  const uint8_t* p;
  const uint8_t* end;
  uint64_t buf;
  int cnt;
  bool over;  // read past the data (a damaged block)
  __device__ __forceinline__ void refill() {
    while (cnt <= 56) {
      uint64_t b = 0;
      if (p < end) {
        b = *p++;
      } else {
        over = cnt < 0 || over;  // (zero bits fed past the end; a decode that uses them fails below)
        p++;
      }
      buf |= b << cnt;
      cnt += 8;
    }
  }
  __device__ __forceinline__ uint32_t need(int n) {  // n <= 32 bits
    if (cnt < n) refill();
    const uint32_t v = (uint32_t)(buf & ((n == 32) ? 0xFFFFFFFFull : ((1ull << n) - 1ull)));
    buf >>= n;
    cnt -= n;
    return v;
  }
  __device__ __forceinline__ bool past() const { return p - (cnt >> 3) > end; }  // bits consumed beyond the data
};

// puff-style construction: counts, completeness; 0 complete, > 0 incomplete, < 0 over-subscribed
__device__ int huff_build(Huff& h, uint16_t* offs, const uint8_t* length, int n) {
  for (int l = 0; l < 16; ++l) h.count[l] = 0;
  for (int s = 0; s < n; ++s) h.count[length[s]]++;
  if (h.count[0] == n) return 0;
  int left = 1;
  for (int l = 1; l < 16; ++l) {
    left <<= 1;
    left -= h.count[l];
    if (left < 0) return left;
  }
  offs[1] = 0;
  for (int l = 1; l < 15; ++l) offs[l + 1] = (uint16_t)(offs[l] + h.count[l]);
  for (int s = 0; s < n; ++s)
    if (length[s]) h.sym[offs[length[s]]++] = (uint16_t)s;
  return left;
}

// one symbol: the code's bits one at a time (MSB of the code first), from a 16-bit peek
__device__ __forceinline__ int huff_decode(Bits& b, const Huff& h) {
  if (b.cnt < 16) b.refill();
  const uint32_t bits = (uint32_t)b.buf;
  int code = 0, first = 0, index = 0;
#pragma unroll 1
  for (int len = 1; len < 16; ++len) {
    code |= (int)((bits >> (len - 1)) & 1u);
    const int count = h.count[len];
    if (code - count < first) {
      b.buf >>= len;
      b.cnt -= len;
      return h.sym[index + (code - first)];
    }
    index += count;
    first += count;
    first <<= 1;
    code <<= 1;
  }
  return -1;
}

__device__ __forceinline__ uint32_t crc_byte(const uint32_t* tab, uint32_t crc, uint32_t v) {
  return tab[(crc ^ v) & 0xFFu] ^ (crc >> 8);
}

// A thread per block.  out: the inflated stream; status[b]: kInf*.
extern "C" __global__ void __launch_bounds__(kInfThreads) bgzf_inflate_kernel(const uint8_t* comp, const Blk* blks,
                                                                              int64_t n_blk, uint8_t* out,
                                                                              int32_t* status) {
  __shared__ uint32_t crc_tab[256];
  __shared__ InfLds lds[kInfThreads];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) {
    uint32_t c = (uint32_t)i;
    for (int k = 0; k < 8; ++k) c = (c & 1u) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
    crc_tab[i] = c;
  }
  __syncthreads();
  const int64_t bi = (int64_t)blockIdx.x * kInfThreads + threadIdx.x;
  if (bi >= n_blk) return;
  const Blk B = blks[bi];
  InfLds& L = lds[threadIdx.x];
  Bits b{comp + B.src, comp + B.src + B.csize, 0ull, 0, false};
  uint8_t* o = out + B.dst;
  const int32_t isize = B.isize;
  int32_t pos = 0;
  uint32_t crc = 0xFFFFFFFFu;
  int32_t st = kInfOk;
  bool last = false;
  while (!last && st == kInfOk) {
    last = b.need(1);
    const uint32_t type = b.need(2);
    if (type == 0) {  // stored: to a byte boundary, LEN, ~LEN, the bytes
      b.need(b.cnt & 7);
      const uint32_t len = b.need(16), nlen = b.need(16);
      if ((len ^ 0xFFFFu) != nlen) { st = kInfBadBlock; break; }
      if (pos + (int32_t)len > isize) { st = kInfOverrun; break; }
      for (uint32_t i = 0; i < len; ++i) {
        const uint32_t v = b.need(8);
        o[pos++] = (uint8_t)v;
        crc = crc_byte(crc_tab, crc, v);
      }
      if (b.past()) { st = kInfBadBlock; break; }
      continue;
    }
    if (type == 3) { st = kInfBadBlock; break; }
    if (type == 1) {  // fixed codes (RFC 1951 §3.2.6)
      for (int s = 0; s < 288; ++s) L.len[s] = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8;
      huff_build(L.lit, L.offs, L.len, 288);
      for (int s = 0; s < 30; ++s) L.len[s] = 5;
      huff_build(L.dist, L.offs, L.len, 30);
    } else {  // dynamic codes (§3.2.7)
      const int nlen = (int)b.need(5) + 257, ndist = (int)b.need(5) + 1, ncode = (int)b.need(4) + 4;
      if (nlen > 286 || ndist > 30) { st = kInfBadBlock; break; }
      for (int i = 0; i < 19; ++i) L.len[kClOrder[i]] = i < ncode ? (uint8_t)b.need(3) : 0;
      if (huff_build(L.lit, L.offs, L.len, 19) != 0) { st = kInfBadBlock; break; }  // must be complete
      int idx = 0;
      while (idx < nlen + ndist) {
        int sym = huff_decode(b, L.lit);
        if (sym < 0) { st = kInfBadCode; break; }
        if (sym < 16) {
          L.len[idx++] = (uint8_t)sym;
        } else {
          int rep;
          uint8_t v = 0;
          if (sym == 16) {
            if (idx == 0) { st = kInfBadBlock; break; }
            v = L.len[idx - 1];
            rep = 3 + (int)b.need(2);
          } else if (sym == 17) {
            rep = 3 + (int)b.need(3);
          } else {
            rep = 11 + (int)b.need(7);
          }
          if (idx + rep > nlen + ndist) { st = kInfBadBlock; break; }
          while (rep--) L.len[idx++] = v;
        }
      }
      if (st != kInfOk) break;
      if (L.len[256] == 0) { st = kInfBadBlock; break; }  // no end-of-block code
      const int el = huff_build(L.lit, L.offs, L.len, nlen);
      if (el < 0 || (el > 0 && nlen - L.lit.count[0] != 1)) { st = kInfBadBlock; break; }
      // (the distance lengths start at len[nlen]: copied down for the build)
      for (int i = 0; i < ndist; ++i) L.len[i] = L.len[nlen + i];
      const int ed = huff_build(L.dist, L.offs, L.len, ndist);
      if (ed < 0 || (ed > 0 && ndist - L.dist.count[0] != 1)) { st = kInfBadBlock; break; }
    }
    // the block's codes
    while (true) {
      const int sym = huff_decode(b, L.lit);
      if (sym < 0) { st = kInfBadCode; break; }
      if (sym < 256) {
        if (pos >= isize) { st = kInfOverrun; break; }
        o[pos++] = (uint8_t)sym;
        crc = crc_byte(crc_tab, crc, (uint32_t)sym);
        continue;
      }
      if (sym == 256) break;
      const int ls = sym - 257;
      if (ls >= 29) { st = kInfBadCode; break; }
      const int len = kLenBase[ls] + (int)b.need(kLenExtra[ls]);
      const int ds = huff_decode(b, L.dist);
      if (ds < 0 || ds >= 30) { st = kInfBadCode; break; }
      const int dist = kDistBase[ds] + (int)b.need(kDistExtra[ds]);
      if (dist > pos) { st = kInfBadCode; break; }
      if (pos + len > isize) { st = kInfOverrun; break; }
      const uint8_t* src = o + pos - dist;
      for (int i = 0; i < len; ++i) {  // (overlapping copies repeat the last dist bytes, in order)
        const uint8_t v = src[i];
        o[pos + i] = v;
        crc = crc_byte(crc_tab, crc, v);
      }
      pos += len;
    }
    if (st == kInfOk && b.past()) st = kInfBadBlock;
  }
  if (st == kInfOk && pos != isize) st = kInfShort;
  if (st == kInfOk && (crc ^ 0xFFFFFFFFu) != B.crc) st = kInfCrc;
  status[bi] = st;
}

// ---- the records' offsets ----
__device__ __forceinline__ int32_t ld32(const uint8_t* p) {
  return (int32_t)((uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24));
}
// a plausible BAM record at stream offset p (u: the stream, m bytes): the
// fixed fields in range, its variable parts inside block_size, its read name
// NUL-terminated
__device__ bool rec_plausible(const uint8_t* u, int64_t p, int64_t m, int32_t n_ref) {
  if (p < 0 || p + 36 > m) return false;
  const int64_t bs = ld32(u + p);
  if (bs < 32 || p + 4 + bs > m) return false;
  const int32_t ref = ld32(u + p + 4), pos = ld32(u + p + 8), nref = ld32(u + p + 24), npos = ld32(u + p + 28);
  const int32_t l_name = u[p + 12];
  const int32_t n_cig = (int32_t)((uint32_t)u[p + 16] | ((uint32_t)u[p + 17] << 8));
  const int32_t l_seq = ld32(u + p + 20);
  if (ref < -1 || ref >= n_ref || nref < -1 || nref >= n_ref || pos < -1 || npos < -1 || l_name < 1 || l_seq < 0)
    return false;
  const int64_t fixed = 32 + (int64_t)l_name + 4 * (int64_t)n_cig + ((int64_t)l_seq + 1) / 2 + l_seq;
  if (fixed > bs) return false;
  return u[p + 36 + l_name - 1] == 0;
}
struct ChainParams {
  const uint8_t* u;   // the inflated stream
  int64_t m;          // its length
  int64_t body;       // the first record's offset (the header's end)
  const Blk* blks;
  int64_t n_blk;
  int32_t n_ref;
  int64_t* guess;     // [n_blk] the first record start inside the block, -1 none
  int64_t* exit;      // [n_blk] the first record start at or past the block's end (its walk from guess)
  uint64_t* count;    // [n_blk] records starting inside the block
  const uint64_t* base;  // [n_blk + 1] their exclusive scan (pass 3)
  uint64_t* rec;      // [n + 1] record offsets from body (pass 3)
  int32_t* bad;       // set when the chain check fails
};
__device__ __forceinline__ void blk_range(const ChainParams& C, int64_t b, int64_t& lo, int64_t& hi) {
  lo = max(C.blks[b].dst, C.body);
  hi = min(C.blks[b].dst + (int64_t)C.blks[b].isize, C.m);
}
// pass 1: each block's guess and its walk to its exit
extern "C" __global__ void bam_chain_guess(ChainParams C) {
  const int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (b >= C.n_blk) return;
  int64_t lo, hi;
  blk_range(C, b, lo, hi);
  int64_t g = -1;
  if (lo < hi) {
    if (C.body >= C.blks[b].dst && C.body < hi) {
      g = C.body;  // the header ends in this block: the chain's first record
    } else {
      for (int64_t p = lo; p < hi; ++p) {
        if (!rec_plausible(C.u, p, C.m, C.n_ref)) continue;
        const int64_t q = p + 4 + ld32(C.u + p);
        if (q == C.m || rec_plausible(C.u, q, C.m, C.n_ref)) {
          g = p;
          break;
        }
      }
    }
  }
  uint64_t n = 0;
  int64_t p = g;
  if (g >= 0) {
    while (p < hi) {
      if (p + 4 > C.m) { atomicOr(C.bad, 1); break; }
      const int64_t bs = ld32(C.u + p);
      if (bs < 32) { atomicOr(C.bad, 1); break; }
      p += 4 + bs;
      ++n;
    }
  }
  C.guess[b] = g;
  C.exit[b] = p;
  C.count[b] = n;
}
// pass 2: every block with a guess lands on the next guessing block's guess,
// the blocks between it and that one have none, the last lands on m
extern "C" __global__ void bam_chain_check(ChainParams C) {
  const int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (b >= C.n_blk) return;
  int64_t lo, hi;
  blk_range(C, b, lo, hi);
  const bool has_body = lo < hi && C.body >= C.blks[b].dst && C.body < hi;
  if (C.guess[b] < 0) {
    if (has_body) atomicOr(C.bad, 1);
    return;
  }
  const int64_t e = C.exit[b];
  if (e == C.m) {  // the chain's end: no block after this one may hold a start
    for (int64_t k = b + 1; k < C.n_blk; ++k)
      if (C.guess[k] >= 0) { atomicOr(C.bad, 1); break; }
    return;
  }
  if (e > C.m) { atomicOr(C.bad, 1); return; }
  for (int64_t k = b + 1; k < C.n_blk; ++k) {
    int64_t l2, h2;
    blk_range(C, k, l2, h2);
    if (e >= h2) {  // passed over block k: it holds no start
      if (C.guess[k] >= 0) { atomicOr(C.bad, 1); return; }
      continue;
    }
    if (C.guess[k] != e) atomicOr(C.bad, 1);
    return;
  }
  atomicOr(C.bad, 1);  // (an exit short of m past the last block: cannot happen for e < m)
}
// pass 3: the offsets, at the blocks' scanned counts
extern "C" __global__ void bam_chain_write(ChainParams C) {
  const int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (b >= C.n_blk) return;
  int64_t lo, hi;
  blk_range(C, b, lo, hi);
  int64_t p = C.guess[b];
  if (p < 0) return;
  uint64_t i = C.base[b];
  while (p < hi) {
    C.rec[i++] = (uint64_t)(p - C.body);
    p += 4 + ld32(C.u + p);
  }
}

}  // namespace bgzfk
