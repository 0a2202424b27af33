// bqsr_observe_lean.hip -- observe in read order, a lane per read, with the
// per-base VALU cut to the table updates (RecalTable.+=, RecalTable.scala:42-62;
// ErrorCount.+=, :195-201; covariates ReadCovariates.scala:30-60,
// StandardCovariate.scala:39-70).
//
// Same counts as bqsr_observe_kernel<false> (read order, one read group), laid
// out so that a clean 16-offset chunk costs about 4 VALU per offset beside its
// two ds_add_u32 (bqsr_observe_kernel: ~27 per offset, VALU-issue-bound at
// 0.95 ms cfg2):
//  * contexts from two v_perm byte-table lookups per 4 offsets.  Slot(a, b) =
//    T1[a] + T2[b] with T1 = 4 (idx + 1), T2 = idx + 1 (other: 0), and an N
//    in either position lands on 21..42: 22 "junk" context cells per window
//    row that bqsr_window_reduce folds into slot 4 (context 0, BaseContext's
//    N rule).  The reverse strand (quirk Q9) swaps in the complemented tables
//    and mirrors the 16 slots: no reverse complement of the window.
//  * processing order: a lane whose cycle cell decreases with the offset
//    (DiscreteCycle, StandardCovariate.scala:39-48) walks its chunk's quals,
//    slots and bits mirrored, so the cycle address of position p is one
//    per-chunk base + 4p, an immediate offset of the ds_add.
//  * partial chunks (a read's first and last) take the clean form too, their
//    positions outside [st, en) exec-masked.
//  * the three loads a chunk needs issue for a read's 8 chunks at once (its
//    cache lines fetched once), bases as 12-B dword-aligned pieces.
// Masked offsets (clips, insertions, known sites: counted on the key only)
// and mismatches are fixed up in one loop over their bits, as in
// observe_clean.  Chunks with quals outside the window, check-only reads
// (kInfoObsCheck) and the batch's first bases keep the exact per-offset path.

namespace bqsr {

constexpr int kCtxJunk = 22;                     // context cells 21..42 of a lean window row
constexpr int kCtxCells = kCtxSlots + kCtxJunk;  // 43
constexpr int kLeanSub = 8;                      // chunks per step

// 4 x T[code] for codes 0..7 (A C G T N other, 6 and 7 unused), as v_perm
// byte tables {lo: codes 0..3, hi: codes 4..7}
constexpr uint32_t kT1lo = 0x40302010u, kT1hi = 0x00000054u;   // 4 (idx(a) + 1) x 4; N 84 = 4 x 21
constexpr uint32_t kT2lo = 0x100C0804u, kT2hi = 0x00000054u;   // (idx(b) + 1) x 4
constexpr uint32_t kT1clo = 0x10203040u, kT2clo = 0x04080C10u;  // complemented (A<->T, C<->G)
constexpr uint32_t kPermId = 0x03020100u, kPermRev = 0x04050607u;

// bytes k of 16 with klo <= k < khi set to 0xFF (k as byte k & 3 of word k >> 2)
__device__ __forceinline__ uint32_t byte_range(int w, int klo, int khi) {
  const int a = min(max(klo - 4 * w, 0), 4), b = min(max(khi - 4 * w, 0), 4);
  const uint32_t lo = a >= 4 ? 0u : (0xFFFFFFFFu << (8 * a));
  const uint32_t hi = b >= 4 ? 0xFFFFFFFFu : ((1u << (8 * b)) - 1u);
  return lo & hi;
}

typedef __attribute__((address_space(3))) uint32_t* LdsU32;

// A clean chunk in processing order: both increments of every position, then
// masked positions moved back out and mismatches added (as observe_clean).
// a_cyc = LDS byte address of (row 0 - q_lo, cycle cell of position 0), a_ctx
// of (row 0 - q_lo, context cell 0); q[] holds window rows at the positions
// of vp.  kPart: a partial chunk, positions outside vp skipped (exec-masked:
// a shared dump row for them took 64-way same-address adds, cfg2 observe
// 0.95 -> 1.16 ms)
// Mismatches go to the mm window (one copy, rows of w4 bytes): a_mcyc / a_mctx
// as a_cyc / a_ctx.
template <bool kPart>
__device__ __forceinline__ void lean_clean(const uint32_t q[4], const uint32_t xo[4], uint32_t a_cyc, uint32_t a_ctx,
                                           uint32_t o4, uint32_t bm, uint32_t bx, uint32_t a_mcyc, uint32_t a_mctx,
                                           uint32_t w4, uint32_t lmasked, int q_lo, uint32_t vp) {
#pragma unroll
  for (int p = 0; p < kChunk; ++p) {
    if (kPart && !((vp >> p) & 1u)) continue;
    const uint32_t qv = __builtin_amdgcn_ubfe(q[p >> 2], 8 * (p & 3), 8);
    const uint32_t xs4 = __builtin_amdgcn_ubfe(xo[p >> 2], 8 * (p & 3), 8);
    const uint32_t rq = __mul24(qv, o4);
    __hip_atomic_fetch_add((LdsU32)(uintptr_t)(rq + a_cyc) + p, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __hip_atomic_fetch_add((LdsU32)(uintptr_t)(rq + xs4 + a_ctx), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  uint32_t mk = bm | bx;
  if (__builtin_amdgcn_ballot_w64(mk != 0)) {
    const uint64_t x01 = ((uint64_t)xo[1] << 32) | xo[0], x23 = ((uint64_t)xo[3] << 32) | xo[2];
    const uint64_t q01 = ((uint64_t)q[1] << 32) | q[0], q23 = ((uint64_t)q[3] << 32) | q[2];
    while (mk) {
      const int p = __builtin_ctz(mk);
      mk &= mk - 1;
      const uint32_t qv = (uint32_t)((p < 8 ? q01 : q23) >> (8 * (p & 7))) & 0xFFu;
      const uint32_t xs4 = (uint32_t)((p < 8 ? x01 : x23) >> (8 * (p & 7))) & 0xFFu;
      const bool masked = (bm >> p) & 1u;
      // masked: undo both increments (-1 in the obs window); mismatch: +1 in the mm window
      const uint32_t rq = __mul24(qv, masked ? o4 : w4), val = masked ? ~0u : 1u;
      lds_add(rq + (masked ? a_cyc : a_mcyc) + 4u * (uint32_t)p, val);
      lds_add(rq + (masked ? a_ctx : a_mctx) + xs4, val);
      if (masked) lds_add(lmasked + 4u * (qv - (uint32_t)q_lo), 1u);
    }
  }
}

// LDS: [obs rows qw][mm rows qw][masked qw][block hist 128][list count]
// obs rows of P.orow words: nc copies of the C cycle cells, then nc copies of
// the 43 context cells (21 contexts, 22 junk), padded to 2 mod 4; lane l adds
// to copy l % nc (same-address adds of a wavefront's lanes -- same qual, same
// cycle -- split nc ways).  mm rows (rare adds): one copy, wcells = C + 43
// padded, the slab layout.
// Prep ran before: ReadInfo and the slot bitmap.  (A form with the common
// read's prep done in the observing lane -- the "fused prep" -- measured 2.15
// against 2.06 ms a cfg2 job and was removed in round 6; git history holds it.)
template <bool kIdent>
__global__ void __launch_bounds__(kBlockThreads) bqsr_observe_lean(ObserveParams P) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int qw = P.w.qw, cells = P.g.cells, C = P.g.C, L = P.g.L;
  const int wcells = P.wcells, orow = P.orow, nc = P.nc;
  uint32_t* w_obs = (uint32_t*)smem;
  uint32_t* w_mm = w_obs + qw * orow;
  uint32_t* w_masked = w_mm + qw * wcells;
  uint32_t* blk_hist = w_masked + qw;
  const uint32_t lds_obs = (uint32_t)(uintptr_t)(LdsWords)w_obs, lds_masked = (uint32_t)(uintptr_t)(LdsWords)w_masked;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int G = P.n_blocks;
  const int q_lo = P.w.q_lo;
  const uint32_t w4 = 4u * (uint32_t)wcells, o4 = 4u * (uint32_t)orow;
  const uint32_t copy = (uint32_t)(lane % nc);
  const uint32_t qoff = (uint32_t)q_lo * o4;
  const uint32_t lds_mm = (uint32_t)(uintptr_t)(LdsWords)w_mm;
  const uint32_t lo4 = (uint32_t)q_lo * 0x01010101u, hi4 = (uint32_t)(q_lo + qw) * 0x01010101u;
  constexpr int kSup = kLeanSub * kChunk;
  constexpr int NW = (kSup + 31) / 32 + 1;
  // read order: one piece, every cycle cell in the window; bucketed batches
  // (OrderDev): a piece per key (read group, mate class) the workgroup's sorted
  // range meets, its window holding the key's half of the cycle cells
  constexpr bool ident = kIdent;  // P.ord.perm == nullptr
  const int nk = kIdent ? 1 : order_keys(P.ord);
  const int64_t wa = pass_begin(P.rd, P.ord, blockIdx.x, G), wb = pass_begin(P.rd, P.ord, blockIdx.x + 1, G);
  for (int i = tid; i < kQBins; i += blockDim.x) blk_hist[i] = 0;

  for (int key = kIdent ? 0 : (wa < wb ? key_at(P.ord, wa) : nk); key < nk; ++key) {
  const int64_t p0 = kIdent ? wa : max(wa, key_begin(P.ord, P.rd.n_reads, key));
  const int64_t p1 = kIdent ? wb : min(wb, key_begin(P.ord, P.rd.n_reads, key + 1));
  if (!kIdent && p0 >= wb) break;
  if (!kIdent && p0 >= p1) continue;
  const int rg_w = kIdent ? P.w.rg_lo : key_rg(P.ord, key, P.w.rg_lo);  // the read group of the window rows
  const WinGeom gm = kIdent ? WinGeom{0, C} : win_geom(P.ord, P.g, key);
  const int c_lo = gm.c_lo, cw = gm.cw;  // window cycle cell c = table cell c_lo + c
  const uint32_t a_ctx = lds_obs + 4u * ((uint32_t)(nc * cw) + copy * kCtxCells) - qoff;
  const uint32_t a_mctx = lds_mm + 4u * (uint32_t)cw - (uint32_t)q_lo * w4;
  for (int i = tid; i < qw * (orow + wcells) + qw; i += blockDim.x) w_obs[i] = 0;
  __syncthreads();

  for (int64_t g0 = p0 + 64 * wave; g0 < p1; g0 += 64 * kWaves) {
    const bool live = g0 + lane < p1;
    LaneRead x;
    {
      const int64_t r = !live ? 0 : (kIdent ? g0 + lane : order_read(P.ord, g0 + lane));
      x = lane_read(P.rd, P.info, r, live, L);
      if (x.trimmed) info_store(P.info + x.r, x.inf);  // fold and apply read the trimmed range
    }
    const bool act = x.fl & (kInfoObs | kInfoObsCheck);
    const bool full = x.fl & kInfoObs;
    const int n = act ? x.en - x.st : 0;
    const bool clean_rd = full && x.rg == rg_w;
    const bool neg = x.fl & kInfoNeg, sec = x.fl & kInfoSecond;
    const bool rev = x.dir < 0;
    const uint32_t u1lo = neg ? kT2clo : kT1lo, u2lo = neg ? kT1clo : kT2lo;
    const uint32_t sel_q = rev ? kPermRev : kPermId, sel_x = sec ? kPermRev : kPermId;
    const int jb = P.rd.slots_aligned ? -(x.st & 15) : 0;
    const uint8_t* qp = P.rd.qual + x.slot;
    for (int j0 = jb; __builtin_amdgcn_ballot_w64(j0 < n); j0 += kSup) {
      if (j0 >= n) continue;
      uint4 qs[kLeanSub];
      uint3 cr[kLeanSub];
      uint64_t bw[NW];
      const uint64_t s0 = x.slot + (uint64_t)(x.st + j0);
#pragma unroll
      for (int i = 0; i < kLeanSub; ++i) {
        const bool lv = j0 + kChunk * i < n;
        const int o0 = x.st + j0 + kChunk * i;
        qs[i] = lv ? *(const uint4*)(qp + o0) : make_uint4(0, 0, 0, 0);
        const int64_t n0 = chunk_n0(x, o0);
        cr[i] = (lv && full && n0 >= 0) ? *(const uint3*)(P.rd.bases + ((n0 >> 3) << 2)) : make_uint3(0, 0, 0);
      }
#pragma unroll
      for (int w = 0; w < NW; ++w)
        bw[w] = !(full && !(x.fl & kInfoNoBits) && (w == 0 || 32 * w - 32 < n - j0)) ? 0ull : P.sbits[(s0 >> 5) + w];
#pragma clang loop unroll(full)
      for (int i = 0; i < kLeanSub; ++i) {
        const int j = j0 + kChunk * i;
        if (j >= n) continue;
        const int o0 = x.st + j;
        // valid offsets k of the chunk: klo <= k < khi
        const int klo = j < 0 ? -j : 0, khi = min(kChunk, n - j);
        const uint32_t vmask = (0xFFFFu >> (kChunk - khi)) & (0xFFFFu << klo);
        uint32_t bm = 0, bx = 0;
        uint32_t h[4] = {0x10101010u, 0x10101010u, 0x10101010u, 0x10101010u};  // slot 4
        if (full) {
          if (P.rd.slots_aligned)
            sub_bits16<NW>(bw, (uint32_t)(s0 >> 4) & 1u, i, bm, bx);
          else
            sub_bits<NW>(bw, (uint32_t)(s0 & 31), i, bm, bx);
          const int64_t n0 = chunk_n0(x, o0);
          uint64_t clo;
          uint32_t chi;
          if (__builtin_expect(n0 >= 0, 1)) {
            const uint32_t sh = 4u * (uint32_t)(n0 & 7);
            clo = ((uint64_t)__builtin_amdgcn_alignbit(cr[i].z, cr[i].y, sh) << 32) |
                  __builtin_amdgcn_alignbit(cr[i].y, cr[i].x, sh);
            chi = (cr[i].z >> sh) & 0xFu;
          } else {
            load_window_head(P.rd.bases, n0, P.rd.n_slots, clo, chi);
          }
          lean_ctx(clo, chi, u1lo, kT1hi, u2lo, kT2hi, h);
        }
        bm &= vmask;
        bx &= vmask;
        // processing order p: offset k = rev ? 15 - p : p
        uint32_t qd[4] = {qs[i].x, qs[i].y, qs[i].z, qs[i].w};
        mirror16(qd, sel_q);
        mirror16(h, sel_x);
        if (j <= 0) {  // the read's first visited offset (k = -j): context 0 (slot 4)
          const int pf = rev ? 15 + j : -j;
#pragma unroll
          for (int w = 0; w < 4; ++w) {
            const uint32_t m = (pf >> 2) == w ? 0xFFu << (8 * (pf & 3)) : 0u;
            h[w] = (h[w] & ~m) | (0x10101010u & m);
          }
        }
        const uint32_t bmp = mirror_bits16(bm, rev), bxp = mirror_bits16(bx, rev);
        const uint32_t vp = mirror_bits16(vmask, rev);
        const int plo = rev ? kChunk - khi : klo, phi = rev ? kChunk - klo : khi;
        // the window cycle cell of position 0 (read order: the window holds every cycle cell)
        const int cc0 = x.cell0 + __mul24(x.dir, o0);
        const int cb = (rev ? cc0 - (kChunk - 1) : cc0) - c_lo;  // window cycle cell of position 0
        // clean: the read's group, every valid qual a window row
        const bool part = __builtin_amdgcn_ballot_w64(vp != 0xFFFFu) != 0;
        bool clean = clean_rd;
        if (!P.rows_all) {  // (every qual of the batch a window row: nothing to test)
          uint32_t bad = 0;
#pragma unroll
          for (int w = 0; w < 4; ++w) {
            uint32_t v = qd[w];
            if (part) {  // positions outside [plo, phi) tested as q_lo
              const uint32_t vb = byte_range(w, plo, phi);
              v = (v & vb) | (lo4 & ~vb);
            }
            const uint32_t t = v | 0x80808080u;
            bad |= v | ~(t - lo4) | (t - hi4);
          }
          clean = clean && (bad & 0x80808080u) == 0u;
        }
        const uint32_t a_cyc = lds_obs + 4u * (copy * (uint32_t)cw + (uint32_t)cb) - qoff;
        const uint32_t a_mcyc = lds_mm + 4u * (uint32_t)cb - (uint32_t)q_lo * w4;
        uint32_t fastm = 0;
        if (clean) {
          if (part)
            lean_clean<true>(qd, h, a_cyc, a_ctx, o4, bmp, bxp, a_mcyc, a_mctx, w4, lds_masked, q_lo, vp);
          else
            lean_clean<false>(qd, h, a_cyc, a_ctx, o4, bmp, bxp, a_mcyc, a_mctx, w4, lds_masked, q_lo, vp);
          fastm = vp;
        } else {
          // per position: window rows of the read's group; the rest below
#pragma unroll
          for (int p = 0; p < kChunk; ++p) {
            const int q = (int)__builtin_amdgcn_ubfe(qd[p >> 2], 8 * (p & 3), 8);
            const int row = q - q_lo;
            const bool f = clean_rd && (unsigned)row < (unsigned)qw && ((vp >> p) & 1u);
            const bool m = (bmp >> p) & 1u;
            if (f) {
              const int ob = __mul24(row, orow);
              atomicAdd(m ? &w_masked[row] : &w_obs[ob + (int)copy * cw + cb + p], 1u);
              if (!m)
                atomicAdd(&w_obs[ob + nc * cw + (int)copy * kCtxCells +
                                 (int)(__builtin_amdgcn_ubfe(h[p >> 2], 8 * (p & 3), 8) >> 2)],
                          1u);
            }
            fastm |= (uint32_t)f << p;
          }
          uint32_t mmk = fastm & ~bmp & bxp;
          if (__builtin_amdgcn_ballot_w64(mmk != 0)) {
            const uint64_t x01 = ((uint64_t)h[1] << 32) | h[0], x23 = ((uint64_t)h[3] << 32) | h[2];
            const uint64_t q01 = ((uint64_t)qd[1] << 32) | qd[0], q23 = ((uint64_t)qd[3] << 32) | qd[2];
            while (mmk) {
              const int p = __builtin_ctz(mmk);
              mmk &= mmk - 1;
              const int q = (int)(((p < 8 ? q01 : q23) >> (8 * (p & 7))) & 0xFFu);
              const int xs = (int)((((p < 8 ? x01 : x23) >> (8 * (p & 7))) & 0xFFu) >> 2);
              const int base = __mul24(q - q_lo, wcells);
              atomicAdd(&w_mm[base + cb + p], 1u);
              atomicAdd(&w_mm[base + cw + xs], 1u);
            }
          }
        }
        uint32_t slow = vp & ~fastm;
        if (__builtin_amdgcn_ballot_w64(slow != 0)) {
          const uint64_t x01 = ((uint64_t)h[1] << 32) | h[0], x23 = ((uint64_t)h[3] << 32) | h[2];
          const uint64_t q01 = ((uint64_t)qd[1] << 32) | qd[0], q23 = ((uint64_t)qd[3] << 32) | qd[2];
          while (slow) {
            const int p = __builtin_ctz(slow);
            slow &= slow - 1;
            const int k = rev ? kChunk - 1 - p : p;
            const int o = o0 + k;
            const int q = (int)(int8_t)(((p < 8 ? q01 : q23) >> (8 * (p & 7))) & 0xFFu);
            if (q < 0) {  // RecalTable.+= : phredToErrorProbabilityCache(qual)
              report(P.err, err_key((uint64_t)x.r, (uint32_t)o, kRankTable, BQSR_ERR_QUAL_RANGE));
            } else if (full) {  // outside the LDS window: straight to the int64 table
              const bool masked = (bmp >> p) & 1u, mism = (bxp >> p) & 1u;
              const int ccell = cc0 + __mul24(x.dir, k);
              const int xs = (int)((((p < 8 ? x01 : x23) >> (8 * (p & 7))) & 0xFFu) >> 2);
              const int xcell = C + (xs < kCtxSlots ? xs : 4);  // junk slots: an N, context 0
              if (ident) atomicAdd(&blk_hist[q], 1u);
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
    }
  }
  __syncthreads();
  // ---- the window -> the piece's slab [obs qw rows][mm qw rows][touched qw]; row totals into the block histogram
  uint32_t* pb = P.part + (int64_t)(blockIdx.x + (ident ? 0 : key)) * P.part_stride;
  const int nw = qw * wcells;
  for (int i = tid; i < nw; i += blockDim.x) {
    const int r = i / wcells, c = i - r * wcells;
    const uint32_t* ro = w_obs + r * orow;
    uint32_t v = 0;
    if (c < cw)
      for (int k = 0; k < nc; ++k) v += ro[k * cw + c];
    else if (c < cw + kCtxCells)
      for (int k = 0; k < nc; ++k) v += ro[nc * cw + k * kCtxCells + (c - cw)];
    pb[i] = v;
    pb[nw + i] = w_mm[i];
  }
  for (int slot = wave; slot < qw; slot += kWaves) {
    uint32_t v = 0;
    for (int c = lane; c < nc * cw; c += 64) v += w_obs[slot * orow + c];  // every unmasked base hits one cycle cell
    v = wave_sum(v);
    if (lane == 0) {
      const uint32_t tot = v + w_masked[slot];
      pb[2 * nw + slot] = tot;
      if (ident && tot && q_lo + slot < kQBins) atomicAdd(&blk_hist[q_lo + slot], tot);
    }
  }
  __syncthreads();
  }  // pieces
  if (ident)
    for (int k = tid; k < kQBins; k += blockDim.x) P.hq_block[(int64_t)blockIdx.x * kQBins + k] = blk_hist[k];
}

template __global__ void bqsr_observe_lean<true>(ObserveParams);

}  // namespace bqsr
