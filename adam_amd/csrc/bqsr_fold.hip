// bqsr_fold.hip -- the partition's expectedMismatch, replayed exactly.
//
// The reference folds expectedMismatch += pow10cache[q] sequentially over the
// partition's folded bases (every trimmed base of every usable read, masked
// ones included: RecalTable.scala:61), and the low bits of
// that double decide Q59 vs Q60 in apply: the fold is replayed
// bit for bit, not approximated.
//
// While the running sum S stays inside one binade [2^e, 2^(e+1)),
//   fl(S + t) = S + u * round(t / u),   u = 2^(e - 52),
// unless t / u is exactly a half-integer (a tie: the result then depends on
// the parity of S / u).  So a run of additions inside a binade is an exact
// integer sum of per-qual increments, and only the additions that leave the
// binade (about log2 of the sum's growth: ~22 for 1e9 bases), the ties, and
// the first ones while S < 1/16 (the binade changes every few additions) are
// performed one at a time in double arithmetic, as the JVM performs them.
//
// Where can an event be?  The exact S_k stays within a relative
// k * 2^-53 of the real sum R_k (each rounding error is at most half an ulp of
// a partial sum <= S_k), so the real sum, widened by
// delta = (N + 64) * 2^-52, bounds S everywhere.  The work is split so that
// everything but a short chain of dependent steps runs across the GPU:
//
//   bqsr_fold_plan    1 workgroup: per fold block (one observe workgroup's
//                     reads) the real sum and count from the block's qual
//                     histogram, their prefix, and either "no event in this
//                     block" (then the block's exact increment at its binade)
//                     or "candidate";
//   bqsr_fold_tiles   candidate blocks' tiles (<= 64 reads) across the GPU,
//                     one wavefront each: real sum, count, and the exact
//                     increment at the four binades the block may be in;
//   bqsr_fold_segs    one workgroup per candidate block: the tiles' real
//                     prefix, then runs of tiles that surely stay in one
//                     binade (their summed increment) and the tiles that may
//                     hold an event, whose quals are copied, in fold order,
//                     into a compact stream;
//   bqsr_fold_chain   one workgroup: prefetches blocks, segments and streams
//                     into LDS, then one wavefront walks the job in order:
//                     whole blocks and runs by one integer addition each,
//                     event streams by a wavefront-parallel search for the
//                     next binade crossing or tie and one IEEE addition there.
//
// Every shortcut is verified where it is taken (S in the expected binade, no
// crossing): should a bound ever fail, the chain folds those tiles element by
// element from the read columns instead.  The result is exact either way.

namespace bqsr {

constexpr double kFoldSeqLimit = 0.0625;  // below, binades change every few additions: events only
constexpr double kTwo53 = 9007199254740992.0;
constexpr int kChainLdsSegs = 384;         // segments prefetched into the chain's LDS
constexpr int kSegThreads = 1024, kSegWaves = kSegThreads / 64;  // bqsr_fold_segs workgroup (1024: cfg2 49 -> 41 us, r05x)
constexpr int kChainLdsStream = 80 * 1024;  // stream bytes prefetched into the chain's LDS
constexpr size_t chain_lds(int n_blocks) {
  return kChainLdsStream + 64 + (size_t)kChainLdsStream / 64 * 2 * sizeof(double) + (size_t)kChainLdsSegs * sizeof(FoldSeg) +
         (size_t)n_blocks * sizeof(FoldBlock);
}

// the binade of a positive normal double (its unbiased exponent); 0 -> -1023
__device__ __forceinline__ int expo(double x) {
  return (int)(((uint64_t)__double_as_longlong(x) >> 52) & 0x7FF) - 1023;
}
// 2^k as a double from its exponent bits (k in the normal range)
__device__ __forceinline__ double pow2i(int k) { return __longlong_as_double((long long)(1023 + k) << 52); }

// round(t / u) at binade e and whether it is a tie; t / u = t * 2^(52 - e) is exact
__device__ __forceinline__ double fold_inc(double t, int e, bool* tie) {
  const double x = t * pow2i(52 - e);
  const double r = rint(x);  // round half to even, as the IEEE addition does
  *tie = (x - floor(x)) == 0.5;
  return r;
}

// the binades a candidate block's tiles may stay in: from where its widened
// real span reaches kFoldSeqLimit (or its start) to its end; eb0 and count
__device__ __forceinline__ int block_eb0(const FoldBlock& B, double delta) {
  return expo(fmax(B.r0 * (1.0 - delta), kFoldSeqLimit));
}
__device__ __forceinline__ int block_nbin(const FoldBlock& B, double delta) {
  return min(expo(fmax(B.r1 * (1.0 + delta), kFoldSeqLimit)) - block_eb0(B, delta) + 1, kSegBinades);
}

// ---------------------------------------------------------------- plan ----
// One workgroup of 1024 threads (n_blocks <= kMaxFoldBlocks): per block the
// real sum and count (4 threads x 32 histogram bins), their prefix in block
// order, the classification, the increment of each event-free block at its
// binade, and the candidate list in block order.
extern "C" __global__ void __launch_bounds__(1024) bqsr_fold_plan(FoldParams P) {
  __shared__ double t[kQBins];
  __shared__ double sre[kMaxFoldBlocks];
  __shared__ int64_t scn[kMaxFoldBlocks];
  __shared__ double pre[kMaxFoldBlocks];
  __shared__ int32_t cnd[kMaxFoldBlocks];
  __shared__ double wsum[16];
  __shared__ int64_t wcnt[16];
  __shared__ int32_t wc[16];
  __shared__ uint32_t qm[4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int q = tid; q < kQBins; q += 1024) t[q] = P.pow10[q];
  if (tid < 4) qm[tid] = 0;
  __syncthreads();
  const int nb = P.n_blocks;
  // (1) per block: real sum and count
  for (int b0 = 0; b0 < nb; b0 += 256) {
    const int b = b0 + (tid >> 2), part = tid & 3;
    double re = 0.0;
    int64_t n = 0;
    if (b < nb) {
      const uint4* row = (const uint4*)(P.hq_block + (int64_t)b * kQBins + part * 32);
      uint4 v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = row[i];
      uint32_t used = 0;  // bins part * 32 + k holding a base
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const uint32_t h[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          re += (double)h[j] * t[part * 32 + i * 4 + j];
          n += h[j];
          used |= (h[j] != 0u ? 1u : 0u) << (i * 4 + j);
        }
      }
      if (used) atomicOr(&qm[part], used);
    }
    re += __shfl_xor(re, 1);
    re += __shfl_xor(re, 2);
    n += __shfl_xor(n, 1);
    n += __shfl_xor(n, 2);
    if (b < nb && part == 0) {
      sre[b] = re;
      scn[b] = n;
    }
  }
  __syncthreads();
  if (tid < 4 && P.qmask) P.qmask[tid] = qm[tid];
  // (2) exclusive prefix of the real sums in block order (thread = block)
  {
    const double v0 = tid < nb ? sre[tid] : 0.0;
    const int64_t c0 = tid < nb ? scn[tid] : 0;
    double v = v0;
    int64_t c = c0;
    for (int off = 1; off < 64; off <<= 1) {
      const double x = __shfl_up(v, off);
      const int64_t y = __shfl_up(c, off);
      if (lane >= off) {
        v += x;
        c += y;
      }
    }
    if (lane == 63) {
      wsum[wave] = v;
      wcnt[wave] = c;
    }
    __syncthreads();
    double base = 0.0;
    for (int w = 0; w < wave; ++w) base += wsum[w];
    if (tid < nb) pre[tid] = base + (v - v0);
  }
  double total_n = 0.0;
  for (int w = 0; w < 16; ++w) total_n += (double)wcnt[w];
  const double delta = (total_n + 64.0) * 0x1p-52 + 1e-12;
  __syncthreads();
  // (3) classify, 4 threads per block: a block holds no event if its widened
  // real span lies in one binade at or above kFoldSeqLimit and no present
  // qual ties there; then its exact increment at that binade
  for (int b0 = 0; b0 < nb; b0 += 256) {
    const int b = b0 + (tid >> 2), part = tid & 3;
    const bool live = b < nb && scn[min(b, nb - 1)] > 0;
    const double R0 = b < nb ? pre[b] : 0.0, R1 = b < nb ? pre[b] + sre[b] : 0.0;
    const double lo = R0 * (1.0 - delta), hi = R1 * (1.0 + delta);
    bool cand = live && (lo < kFoldSeqLimit * (1.0 + delta) || expo(lo) != expo(hi));
    const int e = (live && !cand) ? expo(lo) : 0;
    double inc = 0.0;
    bool tie = false;
    if (live && !cand) {
      const uint32_t* row = P.hq_block + (int64_t)b * kQBins + part * 32;
      for (int i = 0; i < 32; ++i) {
        const uint32_t h = row[i];
        bool tq;
        const double d = fold_inc(t[part * 32 + i], e, &tq);
        if (h) {
          inc += (double)h * d;
          tie |= tq;
        }
      }
    }
    inc += __shfl_xor(inc, 1);
    inc += __shfl_xor(inc, 2);
    tie |= __shfl_xor((int)tie, 1) != 0;
    tie |= __shfl_xor((int)tie, 2) != 0;
    if (live && !cand && (tie || !(inc < 0x1p52))) cand = true;  // below 2^52 every partial sum was exact
    if (b < nb && part == 0) {
      cnd[b] = cand;
      if (!live) P.blk[b] = FoldBlock{R0, R1, 0.0, kFoldNoBase, -1};
      else if (!cand) P.blk[b] = FoldBlock{R0, R1, inc, e, -1};
      else P.blk[b] = FoldBlock{R0, R1, 0.0, 0, 0};  // cidx set below
    }
  }
  __syncthreads();
  // (4) candidate list in block order (thread = block)
  const int cand = tid < nb ? cnd[tid] : 0;
  const uint64_t m = __builtin_amdgcn_ballot_w64(cand != 0);
  if (lane == 0) wc[wave] = __popcll(m);
  __syncthreads();
  int cb = 0, ctot = 0;
  for (int w = 0; w < 16; ++w) {
    if (w < wave) cb += wc[w];
    ctot += wc[w];
  }
  if (cand) {
    const int ci = cb + __popcll(m & ((1ull << lane) - 1ull));
    P.cand_list[ci] = tid;
    P.blk[tid].cidx = ci;
  }
  if (tid == 0) {
    *P.n_cand = ctot;
    *P.delta = delta;
    *P.stream_used = 0ull;
    *P.seg_used = 0u;
  }
  // (5) runs of event-free blocks of one binade become one addition: the
  // run's first block holds the summed increment and cidx = -(run length)
  // (a run adds less than 2^53 units: its integer sum is exact)
  __shared__ unsigned long long rsum[kMaxFoldBlocks];
  __shared__ int32_t rkey[kMaxFoldBlocks], rlen[kMaxFoldBlocks];
  __syncthreads();
  const bool blive = tid < nb;
  FoldBlock mine{};
  if (blive) mine = P.blk[tid];
  const int key = !blive ? INT32_MIN : (mine.cidx >= 0 ? INT32_MIN + 1 : (mine.e == kFoldNoBase ? INT32_MIN + 2 : mine.e));
  rkey[tid] = key;
  rsum[tid] = 0ull;
  rlen[tid] = 0;
  __syncthreads();
  const bool evfree = blive && mine.cidx < 0 && mine.e != kFoldNoBase;
  const bool rstart = evfree && (tid == 0 || rkey[tid - 1] != key);
  // the run's first block: the last start at or before this block (a max-scan of start indices)
  int f = rstart ? tid : -1;
  for (int off = 1; off < 64; off <<= 1) {
    const int x = __shfl_up(f, off);
    if (lane >= off) f = max(f, x);
  }
  if (lane == 63) wc[wave] = f;
  __syncthreads();
  for (int w = 0; w < wave; ++w) f = max(f, wc[w]);
  if (evfree) {
    atomicAdd(&rsum[f], (unsigned long long)mine.inc);
    atomicAdd(&rlen[f], 1);
  }
  __syncthreads();
  if (rstart) P.blk[tid] = FoldBlock{mine.r0, mine.r1, (double)rsum[tid], mine.e, -rlen[tid]};
}

// ----------------------------------------------------------- tile sums ----
// Candidate blocks' tiles, one wavefront each: the folded bases (usable
// valid reads, trimmed ranges) become an LDS slot bitmap, then every folded
// slot counts its qual into the wavefront's histogram (8 copies by lane & 7
// against same-bin conflicts, rows 129 words apart); out: the tile's
// histogram, real sum and count.
constexpr int kFtWaves = 4, kFtCopies = 8, kFtStride = kQBins + 1;
extern "C" __global__ void __launch_bounds__(kFtWaves * 64) bqsr_fold_tiles(FoldParams P, int64_t max_tpb) {
  __shared__ double t[kQBins];
  __shared__ uint32_t hist[kFtWaves][kFtCopies * kFtStride];
  __shared__ uint32_t bm[kFtWaves][kTileSlots / 32];
  for (int q = threadIdx.x; q < kQBins; q += blockDim.x) t[q] = P.pow10[q];
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const ReadsDev& rd = P.rd;
  const int64_t nt = rd.n_tiles;
  const int64_t total = (int64_t)(*P.n_cand) * max_tpb;
  uint32_t* hw = &hist[wv][(lane & (kFtCopies - 1)) * kFtStride];
  for (int64_t v = (int64_t)blockIdx.x * kFtWaves + wv; v < total; v += (int64_t)gridDim.x * kFtWaves) {
    const int64_t b = P.cand_list[v / max_tpb];
    const int64_t tl = nt * b / P.n_blocks + v % max_tpb;
    if (tl >= nt * (b + 1) / P.n_blocks) continue;
    const int64_t r0 = tl * (int64_t)rd.reads_per_tile;
    const int nr = (int)min((int64_t)rd.reads_per_tile, rd.n_reads - r0);
    ReadMeta m{0, 0, 0, 0, 0};
    ReadInfo inf{0, 0, 0, 0};
    if (lane < nr) {
      m = rd.meta[r0 + lane];
      inf = resolve_info(rd, info_load(P.info + r0 + lane), m.slot, m.lq);
    }
    const uint64_t ts0 = __shfl(m.slot, 0);
    const int nslots = (int)(__shfl(m.slot + max(m.lq, m.ls), nr - 1) - ts0);
    for (int i = lane; i < kTileSlots / 32; i += 64) bm[wv][i] = 0;
    for (int i = lane; i < kFtCopies * kFtStride; i += 64) hist[wv][i] = 0;
    wave_sync();
    if (lane < nr && (inf.fl & kInfoObs) && inf.en > inf.st) {
      int lo = (int)(m.slot - ts0) + inf.st;
      const int hi = (int)(m.slot - ts0) + inf.en;
      while (lo < hi) {
        const int n = min(32 - (lo & 31), hi - lo);
        atomicOr(&bm[wv][lo >> 5], (n == 32 ? 0xFFFFFFFFu : ((1u << n) - 1u)) << (lo & 31));
        lo += n;
      }
    }
    wave_sync();
    // the tile's quals, 16 slots per lane and step, every step's load issued
    // before the first is used (one 4-B load per step and lane was 16
    // dependent round trips a tile: the kernel took 47 us on cfg2)
    const uint8_t* qt = rd.qual + ts0;
    constexpr int kSteps = kTileSlots / (64 * 16);
    uint4 qv[kSteps];
#pragma unroll
    for (int i = 0; i < kSteps; ++i) {
      const int s0 = 16 * (lane + 64 * i);
      qv[i] = s0 < nslots ? *(const uint4*)(qt + s0) : make_uint4(0, 0, 0, 0);  // (the qual column has 32 B of padding)
    }
#pragma unroll
    for (int i = 0; i < kSteps; ++i) {
      const int s0 = 16 * (lane + 64 * i);
      if (s0 >= nslots) continue;
      const uint32_t bits = (bm[wv][s0 >> 5] >> (s0 & 31)) & 0xFFFFu;
      const uint32_t w[4] = {qv[i].x, qv[i].y, qv[i].z, qv[i].w};
#pragma unroll
      for (int k = 0; k < 16; ++k)
        if (((bits >> k) & 1u) && s0 + k < nslots) atomicAdd(&hw[(w[k >> 2] >> (8 * (k & 3))) & 0x7Fu], 1u);
    }
    wave_sync();
    double re = 0.0;
    uint32_t cnt = 0, h2[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int q = lane + 64 * i;
      uint32_t h = 0;
#pragma unroll
      for (int c = 0; c < kFtCopies; ++c) h += hist[wv][c * kFtStride + q];
      h2[i] = h;
      re += (double)h * t[q];
      cnt += h;
    }
    for (int off = 32; off > 0; off >>= 1) {
      re += __shfl_xor(re, off);
      cnt += __shfl_xor(cnt, off);
    }
    if (lane == 0) {
      P.rtile[tl] = re;
      P.ntile[tl] = (int32_t)cnt;
    }
    // exact increments at every binade the block may be in (from the histogram)
    const FoldBlock B = P.blk[b];
    const int eb0 = block_eb0(B, *P.delta), nbin = block_nbin(B, *P.delta);
    for (int k = 0; k < nbin; ++k) {
      double d = 0.0;
      bool tie = false;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        bool tq;
        const double iq = fold_inc(t[lane + 64 * i], eb0 + k, &tq);
        d += (double)h2[i] * iq;  // integers: exact while below 2^53
        tie |= h2[i] != 0 && tq;
      }
      for (int off = 32; off > 0; off >>= 1) d += __shfl_xor(d, off);
      const bool anytie = __builtin_amdgcn_ballot_w64(tie) != 0;
      if (lane == 0) P.dtile[tl * kSegBinades + k] = anytie ? kFoldTie : (d < 0x1p52 ? d : kFoldUnknown);
    }
    wave_sync();
  }
}

// ------------------------------------------------------------ segments ----
// One workgroup per candidate block (blockIdx.x < n_cand).  Tiles in chunks
// of 1024 (one per thread), carried across chunks: the real prefix, the
// current segment, its summed increment and the stream offsets.

// copy the folded quals of tile tl, in fold order, to dst (one wavefront)
__device__ void fold_copy_tile(const FoldParams& P, int64_t tl, uint8_t* dst, int lane) {
  const ReadsDev& rd = P.rd;
  const int64_t r0 = tl * (int64_t)rd.reads_per_tile;
  const int nr = (int)min((int64_t)rd.reads_per_tile, rd.n_reads - r0);
  int len = 0;
  uint64_t src = 0;
  if (lane < nr) {
    const ReadMeta m = rd.meta[r0 + lane];
    const ReadInfo inf = resolve_info(rd, info_load(P.info + r0 + lane), m.slot, m.lq);
    if ((inf.fl & kInfoObs) && inf.en > inf.st) {
      len = inf.en - inf.st;
      src = m.slot + inf.st;
    }
  }
  int pre = len;  // inclusive prefix over the tile's reads
  for (int off = 1; off < 64; off <<= 1) {
    const int x = __shfl_up(pre, off);
    if (lane >= off) pre += x;
  }
  // 16-B pieces (unaligned global loads and stores are fine on gfx950), the
  // read's last < 16 bytes one by one: lanes never write each other's bytes
  uint8_t* __restrict__ d = dst + (pre - len);
  const uint8_t* __restrict__ sp = rd.qual + src;
  const int full = len & ~15;
#pragma unroll 4
  for (int i = 0; i < full; i += 16) *(uint4*)(d + i) = *(const uint4*)(sp + i);
  for (int i = full; i < len; ++i) d[i] = sp[i];
}

extern "C" __global__ void __launch_bounds__(kSegThreads) bqsr_fold_segs(FoldParams P) {
  const int c = blockIdx.x;
  if (c >= *P.n_cand) return;
  __shared__ double t[kQBins];
  __shared__ double wsum[kSegWaves];
  __shared__ int32_t wcount[kSegWaves], wev[kSegWaves];
  __shared__ int32_t keys[kSegThreads];
  __shared__ unsigned long long s_inc[kFoldMaxSegs];
  __shared__ int32_t s_n[kFoldMaxSegs], s_t0[kFoldMaxSegs], s_t1[kFoldMaxSegs], s_key[kFoldMaxSegs];
  __shared__ int32_t s_e0[kFoldMaxSegs], s_epos0[kFoldMaxSegs];
  __shared__ int64_t s_off[kFoldMaxSegs];
  __shared__ int32_t carry_sid, chunk_sid0;
  __shared__ double carry_r;
  __shared__ int32_t ev_tile[kSegThreads];
  __shared__ int64_t ev_dst[kSegThreads];
  __shared__ int32_t seg0;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int q = tid; q < kQBins; q += kSegThreads) t[q] = P.pow10[q];
  const int b = P.cand_list[c];
  const FoldBlock B = P.blk[b];
  const double delta = *P.delta;
  const int eb0 = block_eb0(B, delta), nbin = block_nbin(B, delta);
  const int64_t nt = P.rd.n_tiles;
  const int64_t c0 = nt * b / P.n_blocks, c1 = nt * (b + 1) / P.n_blocks;
  constexpr int kEvent = INT32_MIN + 1;    // the key of tiles that may hold an event
  constexpr int kLast = kFoldMaxSegs - 1;  // segment index absorbing any overflow (folded from the columns)
  if (tid < kFoldMaxSegs) {
    s_inc[tid] = 0;
    s_n[tid] = 0;
    s_t0[tid] = INT32_MAX;
    s_t1[tid] = -1;
    s_key[tid] = kEvent;
    s_off[tid] = -1;
  }
  if (tid == 0) {
    carry_sid = -1;
    carry_r = B.r0;
  }
  __syncthreads();
  for (int64_t k0 = c0; k0 < c1; k0 += kSegThreads) {
    const int64_t tl = k0 + tid;
    const bool live = tl < c1;
    const double re = live ? P.rtile[tl] : 0.0;
    const int32_t cnt = live ? P.ntile[tl] : 0;
    // real prefix at the tile's start and end
    double v = re;
    for (int off = 1; off < 64; off <<= 1) {
      const double x = __shfl_up(v, off);
      if (lane >= off) v += x;
    }
    if (lane == 63) wsum[wave] = v;
    __syncthreads();
    double base = carry_r;
    for (int w = 0; w < wave; ++w) base += wsum[w];
    const double Rt = base + (v - re), Re = base + v;
    // a tile that surely stays in binade e >= kFoldSeqLimit, with a
    // tie-free increment there, has key e; any other has key kEvent
    int key = kEvent;
    int64_t inc = 0;
    if (live) {
      const double lo = Rt * (1.0 - delta), hi = Re * (1.0 + delta);
      const int e = expo(lo), k = e - eb0;
      if (lo >= kFoldSeqLimit * (1.0 + delta) && e == expo(hi) && k >= 0 && k < nbin) {
        const double d = P.dtile[tl * kSegBinades + k];
        if (d >= 0.0) {
          key = e;
          inc = (int64_t)d;
        }
      }
    }
    keys[tid] = live ? key : INT32_MIN;
    __syncthreads();
    // a segment starts where the key changes, and at every chunk's first tile
    // (event tiles of a run form one segment; segments never span chunks)
    const int prev = tid > 0 ? keys[tid - 1] : INT32_MIN;
    const bool start = live && key != prev;
    const bool ev = live && key == kEvent;
    const uint64_t sm = __builtin_amdgcn_ballot_w64(start);
    int ecnt = ev ? cnt : 0;  // event elements of the chunk: inclusive prefix
    for (int off = 1; off < 64; off <<= 1) {
      const int x = __shfl_up(ecnt, off);
      if (lane >= off) ecnt += x;
    }
    if (lane == 0) wcount[wave] = __popcll(sm);
    if (lane == 63) wev[wave] = ecnt;
    __syncthreads();
    int sid = carry_sid, ebase = 0;
    for (int w = 0; w < wave; ++w) {
      sid += wcount[w];
      ebase += wev[w];
    }
    sid += __popcll(sm & ((2ull << lane) - 1ull));      // inclusive: this tile's segment
    const int epos = ebase + ecnt - (ev ? cnt : 0);    // this tile's first element among the chunk's events
    if (tid == 0) chunk_sid0 = carry_sid + 1;           // the first segment starting in this chunk
    if (live) {
      const int s = min(sid, kLast);
      atomicMin(&s_t0[s], (int32_t)tl);
      atomicMax(&s_t1[s], (int32_t)tl);
      if (sid >= kLast) {
        s_key[kLast] = INT32_MAX;  // overflow: folded from the read columns
      } else {
        if (start) {
          s_key[s] = key;
          s_epos0[s] = epos;
          s_e0[s] = expo(fmax(Rt * (1.0 - delta), kFoldSeqLimit));
        }
        if (ev) atomicAdd(&s_n[s], cnt);
        else atomicAdd(&s_inc[s], (unsigned long long)inc);
      }
    }
    const int last = (int)(min(c1, k0 + kSegThreads) - k0) - 1;  // the chunk's last tile
    __syncthreads();
    // the chunk's event segments (complete now): 64-B aligned stream space
    if (tid == last) carry_sid = sid;
    __syncthreads();
    const int s_lo = chunk_sid0, s_hi = min(carry_sid, kLast - 1);
    if (tid <= s_hi - s_lo) {
      const int s = s_lo + tid;
      if (s_key[s] == kEvent) {
        const unsigned long long need = ((unsigned long long)s_n[s] + 63ull) & ~63ull;
        const unsigned long long o = atomicAdd(P.stream_used, need);
        s_off[s] = (o + need <= (unsigned long long)P.stream_cap) ? (int64_t)o : -1;
      }
    }
    __syncthreads();
    // copy the chunk's event tiles, one wavefront per tile
    const bool cp = ev && sid < kLast && s_off[min(sid, kLast)] >= 0;
    const uint64_t cm = __builtin_amdgcn_ballot_w64(cp);
    if (lane == 0) wcount[wave] = __popcll(cm);
    __syncthreads();
    int cb = 0, ctot = 0;
    for (int w = 0; w < kSegWaves; ++w) {
      if (w < wave) cb += wcount[w];
      ctot += wcount[w];
    }
    if (cp) {
      const int i = cb + __popcll(cm & ((1ull << lane) - 1ull));
      ev_tile[i] = (int32_t)tl;
      ev_dst[i] = s_off[sid] + (epos - s_epos0[sid]);
    }
    __syncthreads();
    for (int k = wave; k < ctot; k += kSegWaves) fold_copy_tile(P, ev_tile[k], P.streams + ev_dst[k], lane);
    __syncthreads();  // (the copies are visible to the workgroup)
    // per 64 quals of the chunk's event streams: exact increments at the
    // segment's binades e0, e0 + 1, one thread per 64 quals
    int64_t tot = 0;
    for (int s = s_lo; s <= s_hi; ++s)
      if (s_key[s] == kEvent && s_off[s] >= 0) tot += (s_n[s] + 63) / 64;
    for (int64_t f = tid; f < tot; f += kSegThreads) {
      int s = s_lo;
      int64_t j = f;
      for (; s <= s_hi; ++s) {
        if (!(s_key[s] == kEvent && s_off[s] >= 0)) continue;
        const int64_t nch = (s_n[s] + 63) / 64;
        if (j < nch) break;
        j -= nch;
      }
      const int64_t o = s_off[s] + 64 * j;  // 64-B aligned
      const int m = (int)min((int64_t)64, (int64_t)s_n[s] - 64 * j);
      const int e0 = s_e0[s];
      uint4 w4[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) w4[i] = *(const uint4*)(P.streams + o + 16 * i);  // (the stream has 64 B of slack)
      double d0 = 0.0, d1 = 0.0;
      bool t0 = false, t1 = false;
#pragma unroll
      for (int i = 0; i < 64; ++i) {
        const uint4 v4 = w4[i >> 4];
        const uint32_t word = ((i >> 2) & 3) == 0 ? v4.x : ((i >> 2) & 3) == 1 ? v4.y : ((i >> 2) & 3) == 2 ? v4.z : v4.w;
        const int q = (int)((word >> (8 * (i & 3))) & 0x7Fu);
        bool a0, a1;
        const double i0 = fold_inc(t[q], e0, &a0), i1 = fold_inc(t[q], e0 + 1, &a1);
        if (i < m) {
          d0 += i0;
          d1 += i1;
          t0 |= a0;
          t1 |= a1;
        }
      }
      P.csum[(o / 64) * 2] = t0 ? kFoldTie : (d0 < 0x1p52 ? d0 : kFoldUnknown);
      P.csum[(o / 64) * 2 + 1] = t1 ? kFoldTie : (d1 < 0x1p52 ? d1 : kFoldUnknown);
    }
    if (tid == last) carry_r = Re;
    __syncthreads();
  }
  const int ns = min(carry_sid + 1, kFoldMaxSegs);
  if (tid == 0) {
    seg0 = (int32_t)atomicAdd(P.seg_used, (uint32_t)ns);  // this block's place in the compact list
    P.seg_base[c] = seg0;
    P.nseg[c] = ns;
  }
  __syncthreads();
  if (tid < ns) {
    FoldSeg g;
    g.t0 = s_t0[tid];
    g.t1 = s_t1[tid];
    g.e = 0;
    g.off = 0;
    const int key = s_key[tid];
    if (key == INT32_MAX) {
      g.kind = kSegGlobal;
      g.inc = 0;
    } else if (key == kEvent) {
      g.inc = s_n[tid];  // element count
      g.off = s_off[tid];
      g.e = s_e0[tid];
      g.kind = g.off >= 0 ? kSegEvent : kSegGlobal;  // no stream room: folded from the read columns
    } else {
      g.kind = kSegRun;
      g.e = key;
      g.inc = (int64_t)s_inc[tid];
    }
    P.seg[seg0 + tid] = g;
  }
}

// --------------------------------------------------------------- chain ----

// Fold elements [0, n) of q (LDS) into S exactly, one wavefront, no serial
// loop over elements:
//  * S < kFoldSeqLimit: one addition at a time, 64 operands per load round;
//  * at a 64-element boundary, in binade e0 or e0 + 1 of the precomputed
//    per-64 increments cs (kSegEvent streams): lane l takes the sum of the
//    l-th next 64 elements, a wavefront scan finds the first group that leaves
//    the binade or holds a tie;
//  * otherwise lane l sums the increments of elements pos + 64 l .. + 63;
//  * inside the group found (or the rest of a partial group) lane j takes
//    element j, a second scan finds the element, which is added in IEEE
//    double arithmetic.
// inc: LDS table of binade cur_e (a tie is a negative increment).
// Wavefront scans and broadcasts without LDS (DPP / readlane): the chain is
// one wavefront on one CU, its cost is the latency of these steps.
template <int kCtrl, int kRowMask = 0xF>
__device__ __forceinline__ double dpp_f64(double x) {
  const uint64_t b = (uint64_t)__double_as_longlong(x);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)b, kCtrl, kRowMask, 0xF, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(b >> 32), kCtrl, kRowMask, 0xF, false);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));  // 0.0 where no source lane
}
// inclusive prefix sum over the 64 lanes (row_shr 1, 2, 4, 8, then row_bcast 15 / 31)
__device__ __forceinline__ double wave_incl_scan(double x) {
  x += dpp_f64<0x111>(x);
  x += dpp_f64<0x112>(x);
  x += dpp_f64<0x114>(x);
  x += dpp_f64<0x118>(x);
  x += dpp_f64<0x142, 0xA>(x);
  x += dpp_f64<0x143, 0xC>(x);
  return x;
}
// the value of the previous lane (0.0 in lane 0): wave_shr 1
__device__ __forceinline__ double wave_shr1(double x) { return dpp_f64<0x138>(x); }
__device__ __forceinline__ double readlane_f64(double x, int l) {
  const uint64_t b = (uint64_t)__double_as_longlong(x);
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)b, l), hi = __builtin_amdgcn_readlane((uint32_t)(b >> 32), l);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

#define FPF(i, v) (void)0
#define LDS __attribute__((address_space(3)))
// one copy (noinline: the chain is a single wavefront whose time goes to
// latency, and a kernel this size also misses in the instruction cache);
// every buffer is LDS, cur_e included
__device__ __noinline__ double wave_fold(double S, const LDS uint8_t* q, int n, const LDS double* cs, int e0,
                                         const LDS double* t, LDS double* inc, LDS int* cur_ep, int lane) {
  int cur_e = *cur_ep;
  int pos = 0;
  while (pos < n) {
    if (S < kFoldSeqLimit) {
      // small S: binades change every few additions and ties are common --
      // add one by one (every lane the same chain), 64 operands per load round
      const int k = pos + lane;
      const double x = k < n ? t[q[k] & 0x7F] : 0.0;
      const int m = min(64, n - pos);
      int j = 0;
      for (; j < m && S < kFoldSeqLimit; ++j) S = S + readlane_f64(x, j);
      pos += j;
      FPF(0, j);
      FPF(1, clock64() - c0);
      continue;
    }
    const int e = expo(S);
    if (e != cur_e) {
      FPF(6, 1);
      for (int k = lane; k < kQBins; k += 64) {
        bool tq;
        const double d = fold_inc(t[k], e, &tq);
        inc[k] = tq ? -1.0 : d;  // a tie is flagged by a negative increment
      }
      cur_e = e;
      wave_sync();
    }
    const double N0 = S * pow2i(52 - e);  // S / u, an integer < 2^53
    const double head = kTwo53 - N0;     // increments left before the binade ends
    // (a sum only needs to be exact below head <= 2^52: rounding above it cannot bring it back below)
    int g0 = pos;    // start of the group the element step examines
    int gn = 64;     // its length
    double excl = 0.0;
    bool element_step = false;
    if ((pos & 63) != 0) {  // the rest of a partial group first
      gn = 64 - (pos & 63);
      element_step = true;
    } else {
      double sum = 0.0;
      bool bad = false;
      const int a = pos + 64 * lane;
      if (cs && (e == e0 || e == e0 + 1)) {
        if (a < n) {
          const double d = cs[(a >> 6) * 2 + (e - e0)];
          bad = d < 0.0;  // a tie, or not exact (then it surely leaves the binade)
          sum = bad ? 0.0 : d;
        }
        FPF(7, 1);
      } else if (a < n) {
        double s4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int i0 = 0; i0 < 64; i0 += 16) {
          int qq[16];
#pragma unroll
          for (int j = 0; j < 16; ++j) qq[j] = q[a + i0 + j];  // (buffers have 64 B of slack)
#pragma unroll
          for (int j = 0; j < 16; ++j) {
            const double d = inc[qq[j] & 0x7F];
            const bool ok = a + i0 + j < n;
            bad |= ok && d < 0.0;
            s4[j & 3] += ok ? fmax(d, 0.0) : 0.0;
          }
        }
        sum = (s4[0] + s4[1]) + (s4[2] + s4[3]);
      }
      const double incl = wave_incl_scan(sum);
      const uint64_t hit = __builtin_amdgcn_ballot_w64(a < n && (incl >= head || bad));
      if (!hit) {  // the whole window stays in the binade
        S = (N0 + readlane_f64(incl, 63)) * pow2i(e - 52);
        pos = min(n, pos + 64 * 64);
        FPF(2, 1);
        FPF(3, clock64() - c0);
        continue;
      }
      const int L = (int)__builtin_ctzll(hit);
      excl = L > 0 ? readlane_f64(incl, L - 1) : 0.0;  // < head: exact
      g0 = pos + 64 * L;
      element_step = true;
    }
    if (element_step) {
      // elements g0 .. g0 + gn - 1, one per lane
      const int k = g0 + lane;
      const bool valid = lane < gn && k < n;
      const int qk = (int)q[k] & 0x7F;
      const double d = inc[qk];
      const bool tk = valid && d < 0.0;
      const double v = valid ? fmax(d, 0.0) : 0.0;
      const double sc = wave_incl_scan(v);
      const double scx = wave_shr1(sc);  // exclusive prefix
      const uint64_t evm = __builtin_amdgcn_ballot_w64(valid && (tk || excl + sc >= head));
      if (!evm) {  // (only a partial group can have none): it stays in the binade
        S = (N0 + excl + readlane_f64(sc, 63)) * pow2i(e - 52);
        pos = min(n, g0 + gn);
        FPF(5, clock64() - c0);
        continue;
      }
      const int j = (int)__builtin_ctzll(evm);
      const double before = N0 + excl + readlane_f64(scx, j);                // exact: below head <= 2^52
      S = before * pow2i(e - 52) + t[__builtin_amdgcn_readlane((uint32_t)qk, j)];  // the exact IEEE addition
      pos = g0 + j + 1;
      FPF(4, 1);
      FPF(5, clock64() - c0);
    }
  }
  *cur_ep = cur_e;
  return S;
}

// one tile's folded quals into LDS scratch (the fallback path), then fold
__device__ __noinline__ double fold_tile_global(const FoldParams& P, double S, int64_t tl, LDS uint8_t* scratch,
                                                const LDS double* t, LDS double* inc, LDS int* cur_e, int lane) {
  const ReadsDev& rd = P.rd;
  const int64_t r0 = tl * (int64_t)rd.reads_per_tile;
  const int nr = (int)min((int64_t)rd.reads_per_tile, rd.n_reads - r0);
  int len = 0;
  if (lane < nr) {
    const ReadMeta m = rd.meta[r0 + lane];
    const ReadInfo inf = resolve_info(rd, info_load(P.info + r0 + lane), m.slot, m.lq);
    if ((inf.fl & kInfoObs) && inf.en > inf.st) len = inf.en - inf.st;
  }
  int tot = len;
  for (int off = 32; off > 0; off >>= 1) tot += __shfl_xor(tot, off);
  fold_copy_tile(P, tl, (uint8_t*)scratch, lane);
  wave_sync();
  S = wave_fold(S, scratch, tot, nullptr, 0, t, inc, cur_e, lane);
  wave_sync();  // the scratch is free again
  return S;
}

extern "C" __global__ void __launch_bounds__(1024) bqsr_fold_chain(FoldParams P) {
  extern __shared__ __align__(16) unsigned char chain_smem[];
  __shared__ double t[kQBins];
  __shared__ double inc[kQBins];
  __shared__ __align__(16) uint8_t scratch[kTileSlots + 64];
  __shared__ int32_t nseg_l[kMaxFoldBlocks], sbase_l[kMaxFoldBlocks];
  const int tid = threadIdx.x, lane = tid & 63;
  const int nb = P.n_blocks, nc = *P.n_cand;
  // dynamic LDS (chain_lds): streams | per-64 increments | segments | blocks
  uint8_t* streams = chain_smem;                                             // [kChainLdsStream + 64]
  double* csum = (double*)(chain_smem + kChainLdsStream + 64);               // [kChainLdsStream / 64][2]
  FoldSeg* segs = (FoldSeg*)(csum + kChainLdsStream / 64 * 2);               // [kChainLdsSegs]
  FoldBlock* blk = (FoldBlock*)(segs + kChainLdsSegs);                       // [n_blocks]
  const int64_t used = (int64_t)*P.stream_used;
  const int64_t sl = min(used, (int64_t)kChainLdsStream);
  const int nsl = min((int)*P.seg_used, kChainLdsSegs);
  // prefetch: every thread issues its loads before any is used -- through
  // global-typed pointers (the parameter block's pointers are generic: flat
  // loads, each waited for with every LDS access before it)
  typedef const __attribute__((address_space(1))) uint64_t* G64;
  typedef const __attribute__((address_space(1))) double* GF64;
  typedef const __attribute__((address_space(1))) int32_t* G32;
  for (int q = tid; q < kQBins; q += 1024) t[q] = ((GF64)P.pow10)[q];
  for (int i = tid; i < nc; i += 1024) {
    nseg_l[i] = ((G32)P.nseg)[i];
    sbase_l[i] = ((G32)P.seg_base)[i];
  }
  {
    const G64 src = (G64)P.blk;
    uint64_t* dst = (uint64_t*)blk;
    const int nw = nb * (int)(sizeof(FoldBlock) / 8);
    for (int i = tid; i < nw; i += 1024) dst[i] = src[i];
    const G64 ss = (G64)P.seg;
    uint64_t* sd = (uint64_t*)segs;
    const int sw = nsl * (int)(sizeof(FoldSeg) / 8);
    for (int i = tid; i < sw; i += 1024) sd[i] = ss[i];
    const G64 s8 = (G64)P.streams;
    uint64_t* d8 = (uint64_t*)streams;
    const int64_t n16 = (sl + 15) / 16;
#pragma unroll 4
    for (int64_t i = tid; i < n16; i += 1024) {
      const uint64_t a = s8[2 * i], b = s8[2 * i + 1];
      d8[2 * i] = a;
      d8[2 * i + 1] = b;
    }
    const int64_t nc2 = sl / 64 * 2;
    const GF64 cs = (GF64)P.csum;
#pragma unroll 2
    for (int64_t i = tid; i < nc2; i += 1024) csum[i] = cs[i];
  }
  __syncthreads();
  if (tid >= 64) return;  // one wavefront walks the job
  double S = 0.0;
  __shared__ int cur_e_s;
  if (lane == 0) cur_e_s = INT32_MIN;
  wave_sync();
  LDS int* cur_e = (LDS int*)&cur_e_s;
  const LDS uint8_t* lstreams = (const LDS uint8_t*)streams;
  const LDS double* lcsum = (const LDS double*)csum;
  const LDS double* lt = (const LDS double*)t;
  LDS double* linc = (LDS double*)inc;
  LDS uint8_t* lscratch = (LDS uint8_t*)scratch;
  const int64_t nt = P.rd.n_tiles;
#define PF(x)
  for (int b = 0; b < nb; ++b) {
    const FoldBlock B = blk[b];
    if (B.cidx < 0) {  // a run of -cidx event-free blocks in binade e: one integer addition
      if (B.e == kFoldNoBase) continue;
      const int nrun = -B.cidx;
      if (S >= kFoldSeqLimit && expo(S) == B.e) {
        const double N0 = S * pow2i(52 - B.e);
        if (N0 + B.inc < kTwo53) {
          S = (N0 + B.inc) * pow2i(B.e - 52);
          b += nrun - 1;
          PF(++pf_blk; pf_nc += clock64() - bt0);
          continue;
        }
      }
      PF(++pf_blk_fb);
      // the bound failed (not expected): fold the run's tiles element by element
      for (int64_t tl = nt * b / nb; tl < nt * (b + nrun) / nb; ++tl)
        S = fold_tile_global(P, S, tl, lscratch, lt, linc, cur_e, lane);
      b += nrun - 1;
      continue;
    }
    const int c = B.cidx;
    const int ns = nseg_l[c];
    for (int s = 0; s < ns; ++s) {
      const int64_t si = (int64_t)sbase_l[c] + s;
      FoldSeg G;
      if (si < nsl) G = segs[si];  // (two branches: a select of the pointers would make it a flat load)
      else G = P.seg[si];
      if (G.kind == kSegRun) {
        if (S >= kFoldSeqLimit && expo(S) == G.e) {
          const double N0 = S * pow2i(52 - G.e);
          if (N0 + (double)G.inc < kTwo53) {
            S = (N0 + (double)G.inc) * pow2i(G.e - 52);
            PF(++pf_run);
            continue;
          }
        }
        PF(++pf_run_fb);
      } else if (G.kind == kSegEvent) {
        if (G.off + G.inc <= sl) {  // (the LDS copy has 64 B of slack past sl)
          S = wave_fold(S, lstreams + G.off, (int)G.inc, lcsum + G.off / 64 * 2, G.e, lt, linc, cur_e, lane);
          PF(pf_glob_tiles += clock64() - w0);
        } else {  // beyond the prefetched bytes: through the scratch buffer, 4 KB at a time
          for (int64_t o = 0; o < G.inc; o += kTileSlots) {
            const int m = (int)min((int64_t)kTileSlots, G.inc - o);
            for (int i = lane; i < m; i += 64) scratch[i] = P.streams[G.off + o + i];
            wave_sync();
            S = wave_fold(S, lscratch, m, nullptr, 0, lt, linc, cur_e, lane);
            wave_sync();
          }
        }
        PF(++pf_ev; pf_ev_el += G.inc);
        continue;
      }
      PF(++pf_glob);
      // kSegGlobal, or a run whose bound failed: element by element
      for (int64_t tl = G.t0; tl <= G.t1; ++tl) S = fold_tile_global(P, S, tl, lscratch, lt, linc, cur_e, lane);
    }
    PF(pf_cb += clock64() - bt0);
  }
  if (lane == 0) P.em_out[0] = S;
}

}  // namespace bqsr
