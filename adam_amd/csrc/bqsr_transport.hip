// Transport kernels around the BQSR path (not the per-base passes): the
// staged link format's expansion on the device (bqsr_batch_upload_async),
// kernel copies over PCIe (bqsr_copy_async, bqsr_copy_dyn_async) and the
// compaction of a partition's outputs before they leave the device
// (bqsr_compact_outputs_async).  Included by bqsr_capi.cpp after
// bqsr_kernels.hip.

namespace bqsr {

// ------------------------------------------------ staged base codes -----
// 2 bits a slot -> the 4-bit column (bqsr_batch_upload_async): a thread per
// 16 slots, the 2-bit groups spread to nibbles; n = bytes of the 4-bit column
extern "C" __global__ void bqsr_bases_expand(const uint32_t* b2, int64_t n, uint8_t* bases) {
  const int64_t nw = (n + 7) / 8;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < nw; t += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t x = b2[t];
    uint64_t y = 0;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      uint32_t v = (x >> (16 * h)) & 0xFFFFu;
      v = (v | (v << 8)) & 0x00FF00FFu;
      v = (v | (v << 4)) & 0x0F0F0F0Fu;
      v = (v | (v << 2)) & 0x33333333u;
      y |= (uint64_t)v << (32 * h);
    }
    if (8 * t + 8 <= n) {
      *(uint64_t*)(bases + 8 * t) = y;
    } else {
      for (int64_t k = 0; 8 * t + k < n; ++k) bases[8 * t + k] = (uint8_t)(y >> (8 * k));
    }
  }
}
// the N / other codes over their slots' zero nibbles
extern "C" __global__ void bqsr_bases_exceptions(const uint64_t* exc, int64_t n, uint8_t* bases) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t e = exc[i], slot = e >> 8;
    const uint32_t code = (uint32_t)(e & 0xFu);
    atomicOr((unsigned int*)(bases + ((slot >> 1) & ~(uint64_t)3)), code << (4 * (uint32_t)(slot & 7)));
  }
}

// staged quals (bqsr_batch_upload_async): a thread per 16-slot chunk, code c
// -> base + c - 7, 0 for the zero code and (overwritten next) exceptions;
// nq = bytes of the qual column
extern "C" __global__ void bqsr_quals_expand(const uint64_t* codes, const uint8_t* base, int64_t n16, int64_t nq,
                                             uint8_t* qual) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < n16; t += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t w = codes[t];
    const uint32_t b = (uint32_t)base[t] - 7u;
    uint32_t out[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      uint32_t v = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t c = (uint32_t)(w >> (16 * i + 4 * k)) & 15u;
        v |= (c >= 14u ? 0u : ((b + c) & 0xFFu)) << (8 * k);
      }
      out[i] = v;
    }
    if (16 * t + 16 <= nq) {
      *(uint4*)(qual + 16 * t) = make_uint4(out[0], out[1], out[2], out[3]);
    } else {
      for (int64_t k = 0; 16 * t + k < nq; ++k) qual[16 * t + k] = (uint8_t)(out[k >> 2] >> (8 * (k & 3)));
    }
  }
}
extern "C" __global__ void bqsr_quals_exceptions(const uint64_t* exc, int64_t n, uint8_t* qual) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t e = exc[i];
    qual[e >> 8] = (uint8_t)(e & 0xFFu);
  }
}

// ---------------------------------------------------- kernel copies -----
// dst / src may be pinned host memory (device stores / loads over PCIe): a
// D2H by a kernel runs beside the DMA engines' H2D at once, where two DMA
// copies share the link (tools/link_probe.hip: DMA H2D 58 + kernel D2H
// concurrently 85 GB/s in total, two DMA copies 57).  16-B pieces, then the
// tail bytes (all of an unaligned buffer), both grid-stride.
extern "C" __global__ void bqsr_copy16(const uint4* __restrict__ src, uint4* __restrict__ dst, int64_t n16,
                                       const uint8_t* __restrict__ tsrc, uint8_t* __restrict__ tdst, int64_t ntail) {
  const int64_t t0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x, step = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = t0; i < n16; i += step) dst[i] = src[i];
  for (int64_t i = t0; i < ntail; i += step) tdst[i] = tsrc[i];
}

// ------------------------------------------- compact outputs (streamed) -----
// A partition's recalibrated chars leave the device compacted: read r's
// out_len[r] chars of its slot range [slot + out_start, + out_len) at
// off[r] (u32 exclusive scan of out_len), so the link carries the chars
// (Q13: the trimmed ranges) rather than the padded slot array.
extern "C" __global__ void bqsr_compact_lens(const uint32_t* out_len, int64_t n, uint64_t* len64) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x)
    len64[r] = out_len[r];
}
// a wavefront per 64 reads: offsets by lane, then the reads' bytes 64 lanes wide
extern "C" __global__ void __launch_bounds__(256) bqsr_compact_chars(const ReadMeta* meta, const uint8_t* out_qual,
                                                                     const uint32_t* out_start, const uint64_t* off64,
                                                                     int64_t n, uint8_t* chars, uint32_t* off32,
                                                                     uint16_t* len16) {
  const int lane = threadIdx.x & 63;
  for (int64_t r0 = blockIdx.x * (int64_t)blockDim.x + (threadIdx.x & ~63); r0 < n;
       r0 += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = r0 + lane;
    uint64_t src = 0, dst = 0, len = 0;
    if (r < n) {
      dst = off64[r];
      len = off64[r + 1] - dst;
      src = meta[r].slot + out_start[r];
      off32[r] = (uint32_t)dst;
      if (len16) len16[r] = (uint16_t)len;  // (a read's chars <= kMaxReadLen)
      if (r == n - 1) off32[n] = (uint32_t)off64[n];
    }
    for (int j = 0; j < 64; ++j) {
      const uint64_t l = __shfl(len, j), a = __shfl(src, j), d = __shfl(dst, j);
      for (uint64_t k = lane; k < l; k += 64) chars[d + k] = out_qual[a + k];
    }
  }
}
// the exception list's slots -> positions in the compacted chars (the read
// holding the slot: binary search over the batch's read slots)
extern "C" __global__ void bqsr_compact_exceptions(const ReadMeta* meta, int64_t n, const uint32_t* out_start,
                                                   const uint64_t* off64, unsigned long long* exc,
                                                   const unsigned long long* n_exc, int64_t max_exc) {
  const int64_t ne = min((int64_t)*n_exc, max_exc);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < ne; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t e = exc[i], slot = e >> 16;
    int64_t lo = 0, hi = n - 1;  // the last read whose slot <= slot
    while (lo < hi) {
      const int64_t mid = (lo + hi + 1) >> 1;
      if (meta[mid].slot <= slot) lo = mid; else hi = mid - 1;
    }
    const uint64_t pos = off64[lo] + (slot - meta[lo].slot - out_start[lo]);
    exc[i] = (pos << 16) | (e & 0xFFFFull);
  }
}
// a kernel copy of a byte count the device holds: bytes = min(*count * scale, max)
extern "C" __global__ void bqsr_copy_dyn(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                         const void* count, int32_t count_bytes, int64_t scale, int64_t max_bytes) {
  const int64_t c = count_bytes == 4 ? (int64_t)*(const uint32_t*)count : (int64_t)*(const uint64_t*)count;
  const int64_t bytes = min(c * scale, max_bytes);
  const int64_t t0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x, step = (int64_t)gridDim.x * blockDim.x;
  if (((uintptr_t)src | (uintptr_t)dst) % 16 == 0) {
    const int64_t n16 = bytes / 16;
    for (int64_t i = t0; i < n16; i += step) ((uint4*)dst)[i] = ((const uint4*)src)[i];
    for (int64_t i = 16 * n16 + t0; i < bytes; i += step) dst[i] = src[i];
  } else {
    for (int64_t i = t0; i < bytes; i += step) dst[i] = src[i];
  }
}

}  // namespace bqsr
