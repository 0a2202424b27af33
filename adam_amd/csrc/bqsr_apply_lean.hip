// bqsr_apply_lean.hip -- apply in read order, a lane per read
// (RecalUtil.recalibrate, RecalUtil.scala:31-42, over every eligible read:
// RecalibrateBaseQualities.scala:66-76).
//
// The counterpart of bqsr_observe_lean: a lane walks its read's 16-offset
// chunks, a read's 8 chunks' loads issued at once; contexts from the v_perm
// byte tables (an N in the pair gives a slot >= 21, sent to the checked path);
// a lane whose cycle cell decreases walks its chunk mirrored, so the char
// table address of position p is one per-chunk base + 21 p, an immediate
// offset of the ds_read_u8.  The char table (bqsr_apply_chars: (row, cycle
// cell, context) -> errorProbabilityToPhred(s1 + d2) + 33, 0 where the
// checked path decides) is the whole LDS: no context table, no walk markers
// (more rows than bqsr_apply_kernel's).  Quals outside the table's clean rows,
// N contexts, check-only reads and other read groups take apply_slow, the
// exact checked path, as in bqsr_apply_kernel.

namespace bqsr {

// bit k of the result: byte k of the 16 (4 words) has its high bit set
__device__ __forceinline__ uint32_t byte_flags16(const uint32_t f[4]) {
  uint32_t m = 0;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const uint32_t b = (f[w] & 0x80808080u) >> 7;
    m |= ((b | (b >> 7) | (b >> 14) | (b >> 21)) & 0xFu) << (4 * w);
  }
  return m;
}

// LDS: [clean rows 16 B][char table qw x C x 21]
__global__ void __launch_bounds__(kBlockThreads) bqsr_apply_lean(ApplyParams P) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int qw = P.w.qw, C = P.g.C, L = P.g.L, q_lo = P.w.q_lo;
  uint32_t* clean_rows = (uint32_t*)smem;
  uint8_t* lut = smem + 16;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int G = gridDim.x;
  const int64_t wa = wg_begin(P.rd, blockIdx.x, G), wb = wg_begin(P.rd, blockIdx.x + 1, G);
  {  // the char table (bqsr_apply_chars, piece 0) into LDS, 16 B a thread
    const uint4* src = (const uint4*)P.chars;
    uint4* dst = (uint4*)lut;
    const int n16 = (int)(P.piece_stride >> 4);
    for (int i = tid; i < n16; i += blockDim.x) dst[i] = src[i];
  }
  if (tid == 0) {  // the longest run of rows without a 0 entry: quals there need no per-entry check
    const uint4 rb = *(const uint4*)P.rowbad;
    const uint32_t rw[4] = {rb.x, rb.y, rb.z, rb.w};
    int best_lo = 0, best_n = 0, run = 0;
    for (int r = 0; r < qw; ++r) {
      run = ((rw[r >> 5] >> (r & 31)) & 1u) ? 0 : run + 1;
      if (run > best_n) {
        best_n = run;
        best_lo = r - run + 1;
      }
    }
    clean_rows[0] = (uint32_t)(q_lo + best_lo);
    clean_rows[1] = (uint32_t)(q_lo + best_lo + best_n);
  }
  __syncthreads();
  const uint32_t lo4 = clean_rows[0] * 0x01010101u, hi4 = clean_rows[1] * 0x01010101u;
  const uint32_t C21 = (uint32_t)C * kCtxSlots;
  const uint32_t a0 = (uint32_t)(uintptr_t)(LdsBytes)lut - (uint32_t)q_lo * C21;
  constexpr int kSup = kLeanSub * kChunk;

  for (int64_t g0 = wa + 64 * wave; g0 < wb; g0 += 64 * kWaves) {
    const bool live = g0 + lane < wb;
    const LaneRead x = lane_read(P.rd, P.info, live ? g0 + lane : 0, live, L);
    const bool pass = x.fl & kInfoPass, app = x.fl & kInfoApp;
    if (live) {
      P.out_start[x.ro] = pass ? 0u : (uint32_t)x.st;
      P.out_len[x.ro] = pass ? (uint32_t)x.en : app ? (uint32_t)(x.en - x.st) : 0u;
    }
    const bool act = live && (x.fl & (kInfoApp | kInfoAppCheck | kInfoPass));
    const int n = act ? x.en - x.st : 0;
    const bool cok = app && x.rg == P.w.rg_lo;
    const bool neg = x.fl & kInfoNeg, sec = x.fl & kInfoSecond;
    const bool rev = x.dir < 0;
    const uint32_t u1lo = neg ? kA2clo : kA1lo, u2lo = neg ? kA1clo : kA2lo;
    const uint32_t sel_q = rev ? kPermRev : kPermId, sel_x = sec ? kPermRev : kPermId;
    const int jb = P.rd.slots_aligned ? -(x.st & 15) : 0;
    const uint8_t* qp = P.rd.qual + x.slot;
    uint8_t* op = P.out_qual + x.oslot;
    for (int j0 = jb; __builtin_amdgcn_ballot_w64(j0 < n); j0 += kSup) {
      if (j0 >= n) continue;
      uint4 qs[kLeanSub];
      uint3 cr[kLeanSub];
#pragma unroll
      for (int i = 0; i < kLeanSub; ++i) {
        const bool lv = j0 + kChunk * i < n;
        const int o0 = x.st + j0 + kChunk * i;
        qs[i] = lv ? *(const uint4*)(qp + o0) : make_uint4(0, 0, 0, 0);
        const int64_t n0 = chunk_n0(x, o0);
        cr[i] = (lv && !pass && n0 >= 0) ? *(const uint3*)(P.rd.bases + ((n0 >> 3) << 2)) : make_uint3(0, 0, 0);
      }
#pragma clang loop unroll(full)
      for (int i = 0; i < kLeanSub; ++i) {
        const int j = j0 + kChunk * i;
        if (j >= n) continue;
        const int o0 = x.st + j;
        uint32_t out[4];
        if (pass) {  // the original chars: (qual + 33) byte-wise
          const uint32_t qd[4] = {qs[i].x, qs[i].y, qs[i].z, qs[i].w};
#pragma unroll
          for (int w = 0; w < 4; ++w) out[w] = ((qd[w] & 0x7F7F7F7Fu) + 0x21212121u) ^ (qd[w] & 0x80808080u);
        } else {
          const int klo = j < 0 ? -j : 0, khi = min(kChunk, n - j);
          const uint32_t vmask = (0xFFFFu >> (kChunk - khi)) & (0xFFFFu << klo);
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
          uint32_t h[4];
          lean_ctx(clo, chi, u1lo, kA1hi, u2lo, kA2hi, h);
          // processing order p: offset k = rev ? 15 - p : p
          uint32_t qd[4] = {qs[i].x, qs[i].y, qs[i].z, qs[i].w};
          mirror16(qd, sel_q);
          mirror16(h, sel_x);
          if (j <= 0) {  // the read's first visited offset (k = -j): context 0 (slot 4)
            const int pf = rev ? 15 + j : -j;
#pragma unroll
            for (int w = 0; w < 4; ++w) {
              const uint32_t m = (pf >> 2) == w ? 0xFFu << (8 * (pf & 3)) : 0u;
              h[w] = (h[w] & ~m) | (0x04040404u & m);
            }
          }
          const uint32_t vp = mirror_bits16(vmask, rev);
          // positions the table cannot answer: quals outside the clean rows, N contexts (slots >= 21)
          uint32_t fb[4], fj[4];
#pragma unroll
          for (int w = 0; w < 4; ++w) {
            const uint32_t t = qd[w] | 0x80808080u;
            fb[w] = qd[w] | ~(t - lo4) | (t - hi4);
            fj[w] = h[w] + 0x6B6B6B6Bu;  // slot + 107 >= 128 <=> slot >= 21 (slots <= 42: no carry)
          }
          const uint32_t slow_p = vp & (cok ? (byte_flags16(fb) | byte_flags16(fj)) : 0xFFFFu);
          const uint32_t fm = vp & ~slow_p;
          const int cc0 = x.cell0 + __mul24(x.dir, o0);
          const uint32_t a_c = a0 + (uint32_t)(rev ? cc0 - (kChunk - 1) : cc0) * kCtxSlots;
          uint32_t ea[kChunk];
#pragma unroll
          for (int p = 0; p < kChunk; ++p)
            ea[p] = __builtin_amdgcn_ubfe(h[p >> 2], 8 * (p & 3), 8) +
                    __mul24(__builtin_amdgcn_ubfe(qd[p >> 2], 8 * (p & 3), 8), C21) + a_c;
          // 16 byte reads into 16-bit halves, two halves per register, merged by byte permutes
          if (__builtin_amdgcn_ballot_w64(fm != 0xFFFFu) == 0) {
#pragma unroll
            for (int w = 0; w < 4; ++w) {
              u16x2 a, b;  // a: bytes 0 and 2 of the word, b: bytes 1 and 3
              a.x = *((LdsBytes)(uintptr_t)ea[4 * w] + kCtxSlots * (4 * w));
              b.x = *((LdsBytes)(uintptr_t)ea[4 * w + 1] + kCtxSlots * (4 * w + 1));
              a.y = *((LdsBytes)(uintptr_t)ea[4 * w + 2] + kCtxSlots * (4 * w + 2));
              b.y = *((LdsBytes)(uintptr_t)ea[4 * w + 3] + kCtxSlots * (4 * w + 3));
              out[w] = __builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, b), __builtin_bit_cast(uint32_t, a), 0x06020400u);
            }
          } else {  // positions outside fm are not read (their addresses may lie past the table)
#pragma unroll
            for (int w = 0; w < 4; ++w) {
              u16x2 a = {0, 0}, b = {0, 0};
              if ((fm >> (4 * w)) & 1u) a.x = *((LdsBytes)(uintptr_t)ea[4 * w] + kCtxSlots * (4 * w));
              if ((fm >> (4 * w + 1)) & 1u) b.x = *((LdsBytes)(uintptr_t)ea[4 * w + 1] + kCtxSlots * (4 * w + 1));
              if ((fm >> (4 * w + 2)) & 1u) a.y = *((LdsBytes)(uintptr_t)ea[4 * w + 2] + kCtxSlots * (4 * w + 2));
              if ((fm >> (4 * w + 3)) & 1u) b.y = *((LdsBytes)(uintptr_t)ea[4 * w + 3] + kCtxSlots * (4 * w + 3));
              out[w] = __builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, b), __builtin_bit_cast(uint32_t, a), 0x06020400u);
            }
          }
          mirror16(out, sel_q);  // back to offset order
          if (__builtin_amdgcn_ballot_w64(slow_p != 0)) {
            if (slow_p) {
              // the checked path in offset order, with N slots as context 0 (slot 4)
              uint32_t xk[4];
#pragma unroll
              for (int w = 0; w < 4; ++w) {
                const uint32_t jm = fj[w] & 0x80808080u;
                const uint32_t M = (jm << 1) - (jm >> 7);  // 0xFF per flagged byte
                xk[w] = (h[w] & ~M) | (0x04040404u & M);
              }
              mirror16(xk, sel_q);  // processing order -> offset order
              const uint4 r = apply_slow(&P, x, o0, mirror_bits16(slow_p, rev), ((uint64_t)xk[1] << 32) | xk[0],
                                         ((uint64_t)xk[3] << 32) | xk[2], make_uint4(out[0], out[1], out[2], out[3]));
              out[0] = r.x;
              out[1] = r.y;
              out[2] = r.z;
              out[3] = r.w;
            }
          }
        }
        if (app || pass) {
          if (j + kChunk <= n || P.rd.slots_aligned) {  // aligned: the chunk's other bytes are this read's scratch
            *(uint4*)(op + o0) = make_uint4(out[0], out[1], out[2], out[3]);
          } else {
#pragma unroll
            for (int k = 0; k < kChunk; ++k)
              if (k < n - j) op[o0 + k] = (uint8_t)(out[k >> 2] >> (8 * (k & 3)));
          }
        }
      }
    }
  }
}

}  // namespace bqsr
