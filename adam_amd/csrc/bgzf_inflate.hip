// bgzf_inflate.hip -- BAM's BGZF blocks inflated on the device, and the BAM
// records found in the inflated stream there (the reference
// reads BAM through Hadoop-BAM / htsjdk, core/rdd/AdamContext.scala:122-137,
// whose BlockGunzipper inflates one BGZF block at a time).
//
// A BGZF file is a chain of gzip members of at most 64 KiB inflated each; no
// DEFLATE back-reference crosses a member, so every block inflates on its own,
// in two passes: a thread per block (bgzf_tokens_kernel, kInfThreads blocks a
// workgroup) decodes it to 32-bit symbols in HBM, its decode tables and a
// ring its compressed bytes are staged through in the thread's slice of LDS;
// then a workgroup per block (bgzf_resolve_kernel) assembles its bytes in LDS
// from the symbols, checks its CRC32 there (256 chunks combined in GF(2)) and
// stores them at the block's place in the inflated stream (the host's prefix
// sum of the blocks' ISIZE).  A block is rejected as the host path rejects
// it: a code that does not decode, an overrun of ISIZE, a short output, a
// CRC mismatch.
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
// Measured (profiles/r06t_bgzf_device_inflate.txt): a thread per block is
// serial per member, so pass 1's time is one member's decode latency; what
// set it, in turn: 64 lanes a wavefront diverging (16 now), the canonical
// bit-by-bit decode (two-level tables now), a global load per bit refill
// waiting behind the lane's stores (the LDS ring now), and -- in the one-pass
// form that wrote bytes and copied matches from HBM (tools/variants/
// bgzf_one_pass.diff) -- the matches' L2 round trips (symbols now, the copies
// in LDS).  0.43 GB: 189 ms -> 22.4 + 5.0 ms, where 16 libdeflate threads
// take 57 ms.
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

// blocks a workgroup (lanes of one wavefront), a thread per block: 16 while
// every block of a run is in flight at once (32 a CU, two workgroups' LDS);
// 12 for longer runs (36 a CU, three workgroups: fewer rounds, at 1 ms more a
// round, profiles/r06t_*)
constexpr int kInfThreads = 16;
constexpr int kInfThreadsDeep = 12;
constexpr int kLitRoot = 9;      // the decode tables' root index bits
constexpr int kLitCap = 512;     // and their second-level entries (zlib's bound for 286 codes, root 9: 852 in all)
constexpr int kDistRoot = 8;
constexpr int kDistCap = 256;    // (a code needing more fails the block over to the host form)
enum : int32_t { kInfOk = 0, kInfBadCode = 1, kInfOverrun = 2, kInfShort = 3, kInfCrc = 4, kInfBadBlock = 5 };

// canonical Huffman code of a DEFLATE block (RFC 1951 §3.2.2): symbols by
// code, counted per length (decoded bit by bit, the code's bits MSB first)
template <int kSyms>
struct Huff {
  uint16_t count[16];
  uint16_t sym[kSyms];
};
// a thread's LDS: the literal / length and distance codes (canonical, and as
// two-level decode tables, table_build), the code lengths being read, the
// construction's offsets, and the ring its compressed bytes are staged
// through; an odd number of dwords, so the lanes' copies of one field fall in
// different banks
struct InfLds {
  Huff<288> lit;
  Huff<32> dist;
  uint16_t tlit[(1 << kLitRoot) + kLitCap];
  uint16_t tdist[(1 << kDistRoot) + kDistCap];
  uint8_t len[320];
  uint16_t offs[16];
  uint32_t ring[64];
  uint32_t pad;
};
static_assert((sizeof(InfLds) / 4) % 2 == 1, "InfLds: an odd number of dwords");

// the length / distance codes' bases and extra bits (RFC 1951 §3.2.5), by
// arithmetic: each group of four codes doubles the step
__device__ __forceinline__ int len_extra(int ls) { return (ls < 8 || ls == 28) ? 0 : (ls - 4) >> 2; }
__device__ __forceinline__ int len_base(int ls, int e) {
  return ls < 8 ? ls + 3 : ls == 28 ? 258 : ((4 + (ls & 3)) << e) + 3;
}
__device__ __forceinline__ int dist_extra(int ds) { return ds < 4 ? 0 : (ds >> 1) - 1; }
__device__ __forceinline__ int dist_base(int ds, int e) { return ds < 4 ? ds + 1 : ((2 + (ds & 1)) << e) + 1; }
__constant__ uint8_t kClOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// LSB-first bit reader over one member's compressed bytes.  The bytes come
// through a 256-byte ring in the thread's LDS, staged 128 bytes at a time
// from the 16-byte-aligned address at or below the member's start, each half
// loaded into registers (eight 16-byte loads) a half ahead of its staging:
// a global load per symbol would wait, in the lane's one counter of
// outstanding memory operations, behind every symbol stored before it.  (The
// staging is inline: as a call it cost 10 ms of 36, profiles/r06t_*.)  A half
// that starts before the member's end may read up to 127 bytes past it (the
// compressed buffer carries 256 bytes of padding); halves past the end are
// zeros.  A decode that uses bits past the end fails its checks.
struct Bits {
  const uint4* g;    // the member's bytes, aligned down to 16
  uint32_t* ring;    // 64 words: word w of the stream at [w & 63]
  uint64_t buf;
  int cnt;           // bits in buf
  int q;             // the next word into buf
  int staged;        // words staged so far
  int64_t endbits;   // the member's last bit + 1, counted from g
  uint32_t nextw;    // word q, read ahead of its use
  uint4 pre[8];      // the half after the staged ones, loaded a half ahead
  __device__ __forceinline__ void prefetch() {
    // (through a global-space pointer: a flat load would also count in the
    // LDS counter, so every LDS wait of the decode would wait for it)
    typedef unsigned int u4v __attribute__((ext_vector_type(4)));
    const __attribute__((address_space(1))) u4v* s = (const __attribute__((address_space(1))) u4v*)(g + (staged >> 2));
    const bool in = 32ll * staged < endbits;  // (a decode running on past the end reads zeros)
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      u4v v = {0u, 0u, 0u, 0u};
      if (in) v = s[k];
      pre[k] = make_uint4(v.x, v.y, v.z, v.w);
    }
  }
  // the prefetched half into the ring (over words all taken), the next one's loads issued
  __device__ __forceinline__ void stage() {
    uint32_t* r = ring + (staged & 63);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      r[4 * k] = pre[k].x;
      r[4 * k + 1] = pre[k].y;
      r[4 * k + 2] = pre[k].z;
      r[4 * k + 3] = pre[k].w;
    }
    staged += 32;
    prefetch();
  }
  // to > 32 bits; the next word's LDS read is issued here and waited for at
  // the next refill, off the decode's chain
  __device__ __forceinline__ void refill() {
    while (cnt <= 32) {
      buf |= (uint64_t)nextw << cnt;
      cnt += 32;
      q++;
      if (q >= staged) stage();
      nextw = ring[q & 63];
    }
  }
  __device__ __forceinline__ uint32_t need_short(int n) {  // n <= 16 bits
    if (cnt < n) refill();
    const uint32_t v = (uint32_t)buf & ((1u << n) - 1u);
    buf >>= n;
    cnt -= n;
    return v;
  }
  __device__ __forceinline__ uint32_t need(int n) {  // n <= 32 bits
    if (cnt < n) refill();
    const uint32_t v = (uint32_t)(buf & ((n == 32) ? 0xFFFFFFFFull : ((1ull << n) - 1ull)));
    buf >>= n;
    cnt -= n;
    return v;
  }
  __device__ __forceinline__ bool past() const { return 32ll * q - cnt > endbits; }  // bits consumed beyond the data
};

// puff-style construction: counts, completeness; 0 complete, > 0 incomplete, < 0 over-subscribed
template <int kSyms>
__device__ __attribute__((noinline)) int huff_build(Huff<kSyms>& h, uint16_t* offs, const uint8_t* length, int n) {
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

// The decode table of a built (not over-subscribed) code, indexed by the
// next kRoot bits of the stream (the code's first bit lowest): an entry is
// symbol | code length << 9 for a code of at most kRoot bits (0: no code), or
// 0x8000 | sub bits << 12 | offset for the root prefix of longer codes, whose
// second-level table (2^sub entries, indexed by the bits after the root) sits
// at t[2^kRoot + offset].  The canonical codes are walked in code order
// (h.sym): the longer codes sharing a root prefix are consecutive there, the
// last the longest.  false: the second level needs more than kCap entries.
template <int kRoot, int kCap, int kSyms>
__device__ __attribute__((noinline)) bool table_build(uint16_t* t, const Huff<kSyms>& h) {
  constexpr int kN = 1 << kRoot;
  for (int i = 0; i < kN; ++i) t[i] = 0;
  int idx = 0, off = 0, gprev = -1, gbits = 0;
  uint32_t code = 0;
  for (int l = 1; l < 16; ++l, code <<= 1) {
    for (int j = 0, c = h.count[l]; j < c; ++j, ++code, ++idx) {
      const uint32_t rev = __builtin_bitreverse32(code) >> (32 - l);
      if (l <= kRoot) {
        const uint16_t e = (uint16_t)(h.sym[idx] | (l << 9));
        for (uint32_t i = rev; i < (uint32_t)kN; i += 1u << l) t[i] = e;
        continue;
      }
      const int g = (int)(rev & (kN - 1));
      if (g != gprev) {
        if (gprev >= 0) off += 1 << gbits;
        gprev = g;
      }
      gbits = l - kRoot;
      t[g] = (uint16_t)(0x8000 | (gbits << 12) | off);
    }
  }
  if (gprev >= 0) off += 1 << gbits;
  if (off > kCap) return false;
  for (int i = 0; i < off; ++i) t[kN + i] = 0;
  idx = 0;
  code = 0;
  for (int l = 1; l < 16; ++l, code <<= 1) {
    for (int j = 0, c = h.count[l]; j < c; ++j, ++code, ++idx) {
      if (l <= kRoot) continue;
      const uint32_t rev = __builtin_bitreverse32(code) >> (32 - l);
      const uint32_t e = t[rev & (kN - 1)];
      uint16_t* sub = t + kN + (e & 0xFFFu);
      const uint32_t n = 1u << ((e >> 12) & 7u);
      const uint16_t leaf = (uint16_t)(h.sym[idx] | (l << 9));
      for (uint32_t i = rev >> kRoot; i < n; i += 1u << (l - kRoot)) sub[i] = leaf;
    }
  }
  return true;
}

// one symbol: the code's bits one at a time (MSB of the code first), from a 16-bit peek
template <int kSyms>
__device__ __forceinline__ int huff_decode(Bits& b, const Huff<kSyms>& h) {
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
// one symbol by a decode table: a root read, a second-level read for a
// longer code; -1 for bits that start no code
template <int kRoot>
__device__ __forceinline__ int table_decode(Bits& b, const uint16_t* t) {
  if (b.cnt < 16) b.refill();
  uint32_t e = t[b.buf & ((1u << kRoot) - 1u)];
  if (e & 0x8000u)
    e = t[(1u << kRoot) + (e & 0xFFFu) + ((uint32_t)(b.buf >> kRoot) & ((1u << ((e >> 12) & 7u)) - 1u))];
  const int l = (int)((e >> 9) & 15u);
  if (l == 0) return -1;
  b.buf >>= l;
  b.cnt -= l;
  return (int)(e & 511u);
}

// ---- the members' CRC32 ----
// Each chunk's CRC32 by slicing-by-8 (tables in LDS), then the chunks' CRCs
// combined in GF(2)[x] mod the CRC polynomial, as zlib's crc32_combine does:
// crc(A B) = crc(A) * x^(8 |B|) + crc(B), so crc = sum over chunks t of
// crc_t * x^(8 * (bytes after chunk t)).
constexpr uint32_t kCrcPoly = 0xEDB88320u;

// a * b mod P, bit-reflected (bit 31 is x^0)
__device__ __forceinline__ uint32_t crc_mult(uint32_t a, uint32_t b) {
  uint32_t p = 0;
  for (uint32_t m = 1u << 31; m; m >>= 1) {
    if (a & m) p ^= b;
    b = (b & 1u) ? (b >> 1) ^ kCrcPoly : b >> 1;
  }
  return p;
}
// x^(8 n) mod P: squarings of x^8 (x2n[k] = x^(8 * 2^k))
__device__ __forceinline__ uint32_t crc_x8n(const uint32_t* x2n, uint32_t n) {
  uint32_t p = 1u << 31;
  for (int k = 0; n; n >>= 1, ++k)
    if (n & 1u) p = crc_mult(x2n[k], p);
  return p;
}

// Pass 1 of the inflate: a thread per block, its symbols to tok (+ dst -
// tok0), one a word (a literal byte, or 0x80000000 | (distance - 1) << 9 |
// length), and their count to ntok.  status[b]: kInf* (the CRC is checked by
// pass 2).
template <int kThreads>
__global__ void __launch_bounds__(kThreads) bgzf_tokens_kernel(const uint8_t* comp, const Blk* blks, int64_t n_blk,
                                                               uint32_t* tok, int64_t tok0, int32_t* ntok,
                                                               int32_t* status) {
  __shared__ InfLds lds[kThreads];
  const int64_t bi = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (bi >= n_blk) return;
  const Blk B = blks[bi];
  InfLds& L = lds[threadIdx.x];
  const uintptr_t a0 = (uintptr_t)(comp + B.src), skip = a0 & 15u;
  Bits b{(const uint4*)(a0 - skip), L.ring, 0ull, 0, (int)(skip >> 2), 0, 8 * ((int64_t)skip + B.csize), 0u, {}};
  b.prefetch();
  b.stage();
  b.nextw = L.ring[b.q & 63];
  b.refill();
  b.need((int)(skip & 3u) * 8);
  uint32_t* tk = tok + (B.dst - tok0);
  int32_t k = 0;  // (tokens written)
  const int32_t isize = B.isize;
  int32_t pos = 0;
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
        tk[k++] = v;
        pos++;
      }
      if (b.past()) { st = kInfBadBlock; break; }
      continue;
    }
    if (type == 3) { st = kInfBadBlock; break; }
    if (type == 1) {  // fixed codes (RFC 1951 §3.2.6)
      for (int s = 0; s < 288; ++s) L.len[s] = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8;
      huff_build(L.lit, L.offs, L.len, 288);
      table_build<kLitRoot, kLitCap>(L.tlit, L.lit);
      for (int s = 0; s < 30; ++s) L.len[s] = 5;
      huff_build(L.dist, L.offs, L.len, 30);
      table_build<kDistRoot, kDistCap>(L.tdist, L.dist);
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
      if (!table_build<kLitRoot, kLitCap>(L.tlit, L.lit)) { st = kInfBadBlock; break; }
      // (the distance lengths start at len[nlen]: copied down for the build)
      for (int i = 0; i < ndist; ++i) L.len[i] = L.len[nlen + i];
      const int ed = huff_build(L.dist, L.offs, L.len, ndist);
      if (ed < 0 || (ed > 0 && ndist - L.dist.count[0] != 1)) { st = kInfBadBlock; break; }
      if (!table_build<kDistRoot, kDistCap>(L.tdist, L.dist)) { st = kInfBadBlock; break; }
    }
    // the block's codes
    while (true) {
      const int sym = table_decode<kLitRoot>(b, L.tlit);
      if (sym < 0) { st = kInfBadCode; break; }
      if (sym < 256) {
        if (pos >= isize) { st = kInfOverrun; break; }
        tk[k++] = (uint32_t)sym;
        pos++;
        // a second literal in the same step when its code is a root leaf
        // already in the buffer
        const uint32_t e = L.tlit[b.buf & ((1u << kLitRoot) - 1u)];
        const int l2 = (int)((e >> 9) & 15u);
        if (!(e & 0x8000u) && l2 != 0 && l2 <= b.cnt && (e & 511u) < 256u && pos < isize) {
          b.buf >>= l2;
          b.cnt -= l2;
          tk[k++] = e & 511u;
          pos++;
        }
        continue;
      }
      if (sym == 256) break;
      const int ls = sym - 257;
      if (ls >= 29) { st = kInfBadCode; break; }
      const int le = len_extra(ls);
      const int len = len_base(ls, le) + (int)b.need_short(le);
      const int ds = table_decode<kDistRoot>(b, L.tdist);
      if (ds < 0 || ds >= 30) { st = kInfBadCode; break; }
      const int de = dist_extra(ds);
      const int dist = dist_base(ds, de) + (int)b.need_short(de);
      if (dist > pos) { st = kInfBadCode; break; }
      if (pos + len > isize) { st = kInfOverrun; break; }
      tk[k++] = 0x80000000u | ((uint32_t)(dist - 1) << 9) | (uint32_t)len;
      pos += len;
      {  // (and a literal after it, the same way)
        const uint32_t e = L.tlit[b.buf & ((1u << kLitRoot) - 1u)];
        const int l2 = (int)((e >> 9) & 15u);
        if (!(e & 0x8000u) && l2 != 0 && l2 <= b.cnt && (e & 511u) < 256u && pos < isize) {
          b.buf >>= l2;
          b.cnt -= l2;
          tk[k++] = e & 511u;
          pos++;
        }
      }
    }
    if (st == kInfOk && b.past()) st = kInfBadBlock;
  }
  if (st == kInfOk && pos != isize) st = kInfShort;
  status[bi] = st;
  ntok[bi] = k;
}

// Pass 2 of the inflate: a workgroup per block, its output assembled in
// LDS (a block inflates to at most 64 KiB) from its tokens 512 at a time --
// each thread a token, its output offset by a workgroup scan, the literals
// written at once, then rounds in which every match whose source bytes lie
// below the first unresolved token's output copies (the first one always
// can) -- then its CRC32 checked from LDS (132-byte chunks, combined as
// above) and the bytes stored to out (+ dst).
constexpr int kResThreads = 512;
constexpr int kResChunk = 132;  // kResThreads * kResChunk >= 65536; a 33-dword stride puts the lanes' reads in distinct banks
extern "C" __global__ void __launch_bounds__(kResThreads) bgzf_resolve_kernel(const Blk* blks, const uint32_t* tok,
                                                                              int64_t tok0, const int32_t* ntok,
                                                                              uint8_t* out, int32_t* status) {
  __shared__ uint32_t win32[65536 / 4 + 1];
  __shared__ uint32_t tab[8 * 256];
  __shared__ uint32_t x2n[20];
  __shared__ int32_t red[kResThreads / 64];
  uint8_t* win = (uint8_t*)win32;
  const int64_t bi = blockIdx.x;
  if (status[bi] != kInfOk) return;  // (uniform over the workgroup)
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  if (t < 256) {
    uint32_t c = (uint32_t)t;
    for (int k = 0; k < 8; ++k) c = (c & 1u) ? kCrcPoly ^ (c >> 1) : c >> 1;
    tab[t] = c;
  }
  if (t == 0) {
    x2n[0] = 1u << 23;  // x^8
    for (int k = 1; k < 20; ++k) x2n[k] = crc_mult(x2n[k - 1], x2n[k - 1]);
  }
  const Blk B = blks[bi];
  const int n = ntok[bi];
  const uint32_t* T = tok + (B.dst - tok0);
  int cur = 0;
  uint32_t nx = t < n ? T[t] : 0u;
  for (int g0 = 0; g0 < n; g0 += kResThreads) {
    const int j = g0 + t;
    const uint32_t w = nx;
    nx = j + kResThreads < n ? T[j + kResThreads] : 0u;  // (the next group's, in flight)
    const bool is_m = j < n && (w >> 31);
    const int ln = j < n ? (is_m ? (int)(w & 511u) : 1) : 0;
    // the workgroup's exclusive scan of ln
    int inc = ln;
    for (int o = 1; o < 64; o <<= 1) {
      const int v = __shfl_up(inc, o);
      if (lane >= o) inc += v;
    }
    __syncthreads();  // (red: the last group's readers are done)
    if (lane == 63) red[wv] = inc;
    __syncthreads();
    int before = 0, total = 0;
    for (int q = 0; q < kResThreads / 64; ++q) {
      before += q < wv ? red[q] : 0;
      total += red[q];
    }
    const int p = cur + before + inc - ln;
    if (j < n && !is_m) win[p] = (uint8_t)w;
    const int dist = (int)((w >> 9) & 0x7FFFu) + 1;
    bool pend = is_m;
    while (true) {
      // the first unresolved token's output offset: every byte below it is final
      int f = pend ? p : 0x7FFFFFFF;
      for (int o = 32; o > 0; o >>= 1) f = min(f, __shfl_xor(f, o));
      __syncthreads();  // (the round's writes; red's readers)
      if (lane == 0) red[wv] = f;
      __syncthreads();
      int F = red[0];
      for (int q = 1; q < kResThreads / 64; ++q) F = min(F, red[q]);
      if (F == 0x7FFFFFFF) break;
      if (pend && p - dist + min(ln, dist) <= F) {
        int i = 0;
        if (dist >= 8) {  // 8 bytes a step, their reads in flight together (sources before the step)
          for (; i + 8 <= ln; i += 8) {
            uint8_t v[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) v[q] = win[p - dist + i + q];
#pragma unroll
            for (int q = 0; q < 8; ++q) win[p + i + q] = v[q];
          }
        }
        for (; i < ln; ++i) win[p + i] = win[p - dist + i];  // (forward: a period repeats)
        pend = false;
      }
    }
    cur += total;
  }
  __syncthreads();
  // CRC32 of the 256-byte chunks, combined
  for (int k = 1; k < 8; ++k) {
    if (t < 256) tab[k * 256 + t] = (tab[(k - 1) * 256 + t] >> 8) ^ tab[tab[(k - 1) * 256 + t] & 0xFFu];
    __syncthreads();
  }
  const int isize = B.isize, lo = t * kResChunk, hi = min(isize, lo + kResChunk);
  uint32_t r = 0;
  if (lo < hi) {
    uint32_t crc = 0xFFFFFFFFu;
    int i = lo;
    for (; i + 8 <= hi; i += 8) {
      const uint32_t a = win32[i >> 2] ^ crc, b = win32[(i >> 2) + 1];
      crc = tab[7 * 256 + (a & 0xFFu)] ^ tab[6 * 256 + ((a >> 8) & 0xFFu)] ^ tab[5 * 256 + ((a >> 16) & 0xFFu)] ^
            tab[4 * 256 + (a >> 24)] ^ tab[3 * 256 + (b & 0xFFu)] ^ tab[2 * 256 + ((b >> 8) & 0xFFu)] ^
            tab[1 * 256 + ((b >> 16) & 0xFFu)] ^ tab[b >> 24];
    }
    for (; i < hi; ++i) crc = tab[(crc ^ win[i]) & 0xFFu] ^ (crc >> 8);
    r = crc_mult(crc ^ 0xFFFFFFFFu, crc_x8n(x2n, (uint32_t)(isize - hi)));
  }
  for (int o = 32; o > 0; o >>= 1) r ^= __shfl_xor(r, o);
  if (lane == 0) red[wv] = (int32_t)r;
  // the bytes out: dwords once the destination is aligned
  uint8_t* o = out + B.dst;
  const int head = (int)((4u - ((uintptr_t)o & 3u)) & 3u) < isize ? (int)((4u - ((uintptr_t)o & 3u)) & 3u) : isize;
  if (t < head) o[t] = win[t];
  const int nw = (isize - head) >> 2;
  uint32_t* o32 = (uint32_t*)(o + head);
  for (int i = t; i < nw; i += kResThreads) {
    const int q = head + 4 * i;  // (LDS bytes q .. q+3, not dword-aligned unless head is 0)
    const int s = (q & 3) * 8;
    const uint32_t v = s ? (win32[q >> 2] >> s) | (win32[(q >> 2) + 1] << (32 - s)) : win32[q >> 2];
    o32[i] = v;
  }
  for (int i = head + 4 * nw + t; i < isize; i += kResThreads) o[i] = win[i];
  __syncthreads();
  if (t == 0) {
    uint32_t c = 0;
    for (int q = 0; q < kResThreads / 64; ++q) c ^= (uint32_t)red[q];
    if (c != B.crc) status[bi] = kInfCrc;
  }
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
