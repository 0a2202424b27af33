// bqsr_sam_batch_create (include/adam_sam.h): a parse's records packed into
// the BQSR device layout on the device -- what bqsr_batch_create builds on the
// host from downloaded columns (pack(), bqsr_capi.cpp), without the columns
// leaving HBM.  Included by bqsr_capi.cpp after sam_ingest.hip.
//
//   1. a thread per read: field lengths (checked against the layout's u16
//      fields), its slot span, read-group / length maxima;
//   2. rocPRIM exclusive scan of the spans -> each read's first slot;
//   3. a wavefront per read: ReadMeta / ReadAlign, phred bytes (char - 33) and
//      4-bit base codes at the read's slots (slots are 16-aligned, so a read's
//      code bytes are its own), kSeqOther by ballot;
//   4. the qual histogram of the packed column (the launch window), per-thread
//      LDS counters without conflicts (sam_batch_qhist).
// CIGAR and MD columns are copied whole; a read's offsets are the parse's.

namespace sbk {

constexpr int kThreads = 256;

struct Lens {
  uint64_t max_slot;    // atomicMax
  uint32_t n_rg;        // max rg id + 1
  uint32_t max_len;     // max sequence length
  unsigned long long bad_read;  // first read whose fields overflow the layout (~0: none)
  unsigned long long n_qual;    // Σ Lq: qual bytes in the slots (the rest of the column is zero padding)
};

__device__ __forceinline__ uint32_t field_len(const uint64_t* off, int64_t r) { return (uint32_t)(off[r + 1] - off[r]); }

extern "C" __global__ void __launch_bounds__(kThreads) sam_batch_spans(const uint32_t* flags, const int32_t* rg,
                                                                      const uint64_t* seq_off, const uint64_t* qual_off,
                                                                      const uint64_t* cig_off, const uint64_t* md_off,
                                                                      int64_t n, uint64_t* span, Lens* L) {
  uint64_t ms = 0, nq = 0;
  uint32_t nrg = 1, ml = 1;
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t f = flags[r];
    const uint64_t lq = (f & BQSR_F_HAS_QUAL) ? field_len(qual_off, r) : 0;
    const uint64_t ls = (f & BQSR_F_HAS_SEQ) ? field_len(seq_off, r) : 0;
    const uint64_t nmd = (f & BQSR_F_HAS_MD) ? field_len(md_off, r) : 0;
    const uint64_t ncig = (f & BQSR_F_HAS_CIGAR) ? field_len(cig_off, r) : 0;
    const bool has_rg = f & BQSR_F_HAS_RG;
    if (lq > 65535 || ls > 65535 || nmd > 65535 || ncig > 65535 || (has_rg && (rg[r] < 0 || rg[r] > 65535)))
      atomicMin(&L->bad_read, (unsigned long long)r);
    const uint64_t sl = slot_span(lq, ls);
    span[r] = sl;
    nq += lq;
    ms = sl > ms ? sl : ms;
    if (has_rg && rg[r] >= 0) nrg = max(nrg, (uint32_t)rg[r] + 1u);
    ml = max(ml, field_len(seq_off, r));  // dims_of: the longest sequence
  }
  // one atomic per wave
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t x = __shfl_xor(ms, o);
    ms = x > ms ? x : ms;
    nq += __shfl_xor(nq, o);
    nrg = max(nrg, (uint32_t)__shfl_xor((int)nrg, o));
    ml = max(ml, (uint32_t)__shfl_xor((int)ml, o));
  }
  if ((threadIdx.x & 63) == 0) {
    atomicMax((unsigned long long*)&L->max_slot, (unsigned long long)ms);
    atomicAdd(&L->n_qual, (unsigned long long)nq);
    atomicMax(&L->n_rg, nrg);
    atomicMax(&L->max_len, ml);
  }
}

__device__ __forceinline__ uint32_t base_code(uint8_t c) {
  switch (c) {
    case 'A': return kCodeA;
    case 'C': return kCodeC;
    case 'G': return kCodeG;
    case 'T': return kCodeT;
    case 'N': return kCodeN;
    default: return kCodeOther;
  }
}

extern "C" __global__ void __launch_bounds__(kThreads) sam_batch_pack(
    const uint32_t* flags, const int32_t* rg, const int32_t* ref, const int64_t* start, const uint64_t* seq_off,
    const uint8_t* seq, const uint64_t* qual_off, const uint8_t* qual_in, const uint64_t* cig_off, const uint64_t* md_off,
    const int32_t* ref_contig, int32_t n_ref, const uint64_t* slot, int64_t n, ReadMeta* meta, ReadAlign* align,
    uint8_t* qual, uint8_t* bases, unsigned long long* rghist, int32_t n_rg_hist) {
  // read-group counts in LDS (one global atomic per group and workgroup at the
  // end: a global atomic per read on one address serialised at the memory side)
  constexpr int kRgLds = 1024;
  __shared__ uint32_t rgh[kRgLds];
  for (int i = threadIdx.x; i < kRgLds; i += blockDim.x) rgh[i] = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t w0 = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t r = w0; r < n; r += nw) {
    const uint32_t f = flags[r];
    const uint32_t lq = (f & BQSR_F_HAS_QUAL) ? field_len(qual_off, r) : 0;
    const uint32_t ls = (f & BQSR_F_HAS_SEQ) ? field_len(seq_off, r) : 0;
    const uint64_t s0 = slot[r];
    const uint8_t* q = qual_in + qual_off[r];
    for (uint32_t i = lane; i < lq; i += 64) {
      qual[s0 + i] = (uint8_t)(q[i] - 33);  // (char - 33).toByte
    }
    const uint8_t* sq = seq + seq_off[r];
    bool other = false;
    for (uint32_t j = lane; 2 * j < ls; j += 64) {
      const uint32_t c0 = base_code(sq[2 * j]);
      const uint32_t c1 = 2 * j + 1 < ls ? base_code(sq[2 * j + 1]) : 0u;
      other |= c0 == kCodeOther || (2 * j + 1 < ls && c1 == kCodeOther);
      bases[(s0 >> 1) + j] = (uint8_t)(c0 | (c1 << 4));
    }
    const bool any_other = __ballot(other) != 0;
    if (lane == 0) {
      const bool has_rg = f & BQSR_F_HAS_RG;
      ReadMeta m;
      m.slot = s0;
      m.lq = (uint16_t)lq;
      m.ls = (uint16_t)ls;
      m.flags = (uint16_t)((f & 0x7FFF) | (any_other ? kSeqOther : 0));
      m.rg = has_rg ? (uint16_t)rg[r] : 0;
      meta[r] = m;
      ReadAlign a;
      a.start = start[r];
      a.cigar_off = (uint32_t)cig_off[r];
      a.md_off = (uint32_t)md_off[r];
      const int32_t ri = ref[r];
      a.contig = (ri >= 0 && ri < n_ref) ? ref_contig[ri] : BQSR_CONTIG_UNKNOWN;
      a.n_cigar = (uint16_t)((f & BQSR_F_HAS_CIGAR) ? field_len(cig_off, r) : 0);
      a.md_len = (uint16_t)((f & BQSR_F_HAS_MD) ? field_len(md_off, r) : 0);
      align[r] = a;
      if (has_rg && rg[r] >= 0 && rg[r] < n_rg_hist) {
        if (rg[r] < kRgLds) atomicAdd(&rgh[rg[r]], 1u);
        else atomicAdd(&rghist[rg[r]], 1ull);
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kRgLds && i < n_rg_hist; i += blockDim.x)
    if (rgh[i]) atomicAdd(&rghist[i], (unsigned long long)rgh[i]);
}

// The packed qual column's histogram (the batch's launch window): 16-B loads,
// per-thread counters for quals 0..127 in LDS laid out bin-major (thread t's
// bin b at word b * kHistThreads + t: the lanes of a wavefront never share a
// bank or a word, so the adds neither conflict nor need atomics), quals >=
// 128 in a register; zero padding between reads is counted in bin 0 and
// taken out on the host (n_slots - Σ Lq).
constexpr int kHistThreads = 128;
extern "C" __global__ void __launch_bounds__(kHistThreads) sam_batch_qhist(const uint4* q16, int64_t n16,
                                                                          unsigned long long* qhist) {
  __shared__ uint32_t h[kQBins * kHistThreads];
  const int t = threadIdx.x;
  for (int b = 0; b < kQBins; ++b) h[b * kHistThreads + t] = 0;
  uint32_t high = 0;
  for (int64_t i = blockIdx.x * (int64_t)kHistThreads + t; i < n16; i += (int64_t)gridDim.x * kHistThreads) {
    const uint4 v = q16[i];
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const uint32_t b = (w[k >> 2] >> (8 * (k & 3))) & 0xFFu;
      if (b < (uint32_t)kQBins) h[b * kHistThreads + t] += 1u;
      else ++high;
    }
  }
  __syncthreads();
  for (int b = t; b < kQBins; b += kHistThreads) {  // a thread per bin sums the block's counters
    uint64_t c = 0;
    for (int j = 0; j < kHistThreads; ++j) c += h[b * kHistThreads + ((j + b) & (kHistThreads - 1))];
    if (c) atomicAdd(&qhist[b], (unsigned long long)c);
  }
  for (int o = 32; o > 0; o >>= 1) high += __shfl_xor(high, o);
  if ((t & 63) == 0 && high) atomicAdd(&qhist[kQBins], (unsigned long long)high);
}

}  // namespace sbk

namespace {
// device record columns in the parse layout (bqsr_sam, bqsr_arrow)
struct PackCols {
  const uint32_t* flags;
  const int32_t* rg_id;
  const int32_t* ref;  // index into the ref_contig map (-1: none)
  const int64_t* start;
  const uint64_t *seq_off, *qual_off, *cig_off, *md_off;
  const uint8_t *seq, *qual, *md;
  const uint32_t* cig;
  int64_t n_reads, seq_bytes, md_bytes, cig_ops;
  int32_t n_rg;  // read-group ids below this are counted for the launch window
};

bqsr_status pack_batch_device(bqsr_context* ctx, const PackCols& C, const int32_t* ref_contig, int32_t n_ref,
                              void* stream, bqsr_batch** out) {
  using namespace sbk;
  const PackCols* s = &C;
  HIP_TRY(hipSetDevice(ctx->device));
  if ((uint64_t)s->md_bytes > 0xFFFFFFFFull || (uint64_t)s->cig_ops > 0xFFFFFFFFull)
    return fail(BQSR_ERR_UNSUPPORTED, "partition MD / CIGAR columns exceed 4 GiB");
  hipStream_t st = S(stream);
  const int64_t n = s->n_reads;
  std::unique_ptr<bqsr_batch> b(new bqsr_batch);
  b->ctx = ctx;
  b->owned = true;
  b->rd.n_reads = n;
  std::vector<void*> tmp;
  struct Free {
    std::vector<void*>& v;
    ~Free() {
      for (void* p : v) (void)hipFree(p);
    }
  } fr{tmp};
  uint64_t *span = nullptr, *slot = nullptr;
  Lens* dl = nullptr;
  int32_t* d_map = nullptr;
  unsigned long long *qh = nullptr, *rgh = nullptr;
  const int32_t n_rgh = std::max(1, s->n_rg);
  bqsr_status e;
  if ((e = dalloc(tmp, &span, (size_t)n + 1)) || (e = dalloc(tmp, &slot, (size_t)n + 1)) || (e = dalloc(tmp, &dl, 1)) ||
      (e = dalloc(tmp, &d_map, (size_t)std::max(1, n_ref))) || (e = dalloc(tmp, &qh, 256)) ||
      (e = dalloc(tmp, &rgh, (size_t)n_rgh)))
    return e;
  Lens h0{0, 1, 1, ~0ull, 0};
  HIP_TRY(hipMemcpyAsync(dl, &h0, sizeof h0, hipMemcpyHostToDevice, st));
  if (n_ref) HIP_TRY(hipMemcpyAsync(d_map, ref_contig, (size_t)n_ref * 4, hipMemcpyHostToDevice, st));
  HIP_TRY(hipMemsetAsync(qh, 0, 256 * 8, st));
  HIP_TRY(hipMemsetAsync(rgh, 0, (size_t)n_rgh * 8, st));
  HIP_TRY(hipMemsetAsync(span + n, 0, 8, st));
  const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + kThreads - 1) / kThreads, (int64_t)ctx->n_cu * 16));
  if (n) {
    hipLaunchKernelGGL(sam_batch_spans, dim3(g), dim3(kThreads), 0, st, (const uint32_t*)s->flags,
                       (const int32_t*)s->rg_id, (const uint64_t*)s->seq_off, (const uint64_t*)s->qual_off,
                       (const uint64_t*)s->cig_off, (const uint64_t*)s->md_off, n, span, dl);
    HIP_TRY(hipGetLastError());
  }
  size_t tb = 0;
  HIP_TRY(rocprim::exclusive_scan(nullptr, tb, span, slot, (uint64_t)0, (size_t)n + 1, rocprim::plus<uint64_t>(), st));
  void* temp = nullptr;
  if ((e = dalloc(tmp, (uint8_t**)&temp, std::max<size_t>(tb, 1)))) return e;
  HIP_TRY(rocprim::exclusive_scan(temp, tb, span, slot, (uint64_t)0, (size_t)n + 1, rocprim::plus<uint64_t>(), st));
  Lens hl;
  uint64_t n_slots = 0;
  HIP_TRY(hipMemcpyAsync(&hl, dl, sizeof hl, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipMemcpyAsync(&n_slots, slot + n, 8, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  if (hl.bad_read != ~0ull)
    return fail(BQSR_ERR_UNSUPPORTED, "read field longer than 65535 or recordGroupId outside [0, 65535]",
                (int64_t)hl.bad_read);
  if ((int64_t)hl.max_slot > kMaxReadLen)
    return fail(BQSR_ERR_UNSUPPORTED, "reads longer than " + std::to_string(kMaxReadLen) + " bases are not supported");
  ReadMeta* meta;
  ReadAlign* align;
  uint8_t *qual, *bases, *md;
  uint32_t* cigar;
  if ((e = dalloc(b->allocs, &meta, (size_t)std::max<int64_t>(1, n))) ||
      (e = dalloc(b->allocs, &align, (size_t)std::max<int64_t>(1, n))) ||
      (e = dalloc(b->allocs, &qual, (size_t)n_slots + kColumnPad)) ||
      (e = dalloc(b->allocs, &bases, (size_t)n_slots / 2 + 1 + kColumnPad)) ||
      (e = dalloc(b->allocs, &md, (size_t)s->md_bytes + kColumnPad)) ||
      (e = dalloc(b->allocs, &cigar, (size_t)s->cig_ops + kColumnPad / 4)))
    return e;
  // zero slots past each read's bases / quals (and the pads), as pack() leaves them
  HIP_TRY(hipMemsetAsync(qual, 0, (size_t)n_slots + kColumnPad, st));
  HIP_TRY(hipMemsetAsync(bases, 0, (size_t)n_slots / 2 + 1 + kColumnPad, st));
  HIP_TRY(hipMemsetAsync(md + s->md_bytes, 0, kColumnPad, st));
  HIP_TRY(hipMemsetAsync(cigar + s->cig_ops, 0, kColumnPad, st));
  if (s->md_bytes) HIP_TRY(hipMemcpyAsync(md, s->md, (size_t)s->md_bytes, hipMemcpyDeviceToDevice, st));
  if (s->cig_ops) HIP_TRY(hipMemcpyAsync(cigar, s->cig, (size_t)s->cig_ops * 4, hipMemcpyDeviceToDevice, st));
  if (n) {
    const unsigned gw = (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 3) / 4, (int64_t)ctx->n_cu * 8));
    hipLaunchKernelGGL(sam_batch_pack, dim3(gw), dim3(kThreads), 0, st, (const uint32_t*)s->flags,
                       (const int32_t*)s->rg_id, (const int32_t*)s->ref, (const int64_t*)s->start,
                       (const uint64_t*)s->seq_off, (const uint8_t*)s->seq, (const uint64_t*)s->qual_off,
                       (const uint8_t*)s->qual, (const uint64_t*)s->cig_off, (const uint64_t*)s->md_off,
                       (const int32_t*)d_map, n_ref, (const uint64_t*)slot, n, meta, align, qual, bases, rgh, n_rgh);
    HIP_TRY(hipGetLastError());
    const int64_t n16 = (int64_t)n_slots / 16;  // (16-aligned slots: the column's whole slot range)
    const unsigned gh = (unsigned)std::max<int64_t>(1, std::min<int64_t>((n16 + kHistThreads - 1) / kHistThreads,
                                                                          (int64_t)ctx->n_cu * 2));
    hipLaunchKernelGGL(sam_batch_qhist, dim3(gh), dim3(kHistThreads), 0, st, (const uint4*)qual, n16, qh);
    HIP_TRY(hipGetLastError());
  }
  std::vector<unsigned long long> hq(256), hrg((size_t)n_rgh);
  HIP_TRY(hipMemcpyAsync(hq.data(), qh, 256 * 8, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipMemcpyAsync(hrg.data(), rgh, (size_t)n_rgh * 8, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  b->rd.n_slots = (int64_t)n_slots;
  b->n_slots = (int64_t)n_slots;
  b->n_bases = s->seq_bytes;
  b->dims = bqsr_dims{(int32_t)hl.n_rg, (int32_t)hl.max_len};
  int32_t rg_lo = 0;  // as bqsr_batch_create: most frequent read group, densest qual range
  for (int32_t i = 0; i < n_rgh; ++i)
    if (hrg[(size_t)i] > hrg[(size_t)rg_lo]) rg_lo = i;
  b->rg_lo = rg_lo;
  int64_t qhist[kQBins];
  for (int q = 0; q < kQBins; ++q) qhist[q] = (int64_t)hq[(size_t)q];
  qhist[0] -= (int64_t)n_slots - (int64_t)hl.n_qual;  // the slots' zero padding
  b->q_lo = best_q_lo(qhist, 40);
  b->have_qhist = true;
  for (int q = 0; q < kQBins; ++q) b->qhist[q] = qhist[q];
  b->qhigh = (int64_t)hq[kQBins];
  b->rd.meta = meta;
  b->rd.align = align;
  b->rd.qual = qual;
  b->rd.bases = bases;
  b->rd.md = md;
  b->rd.cigar = cigar;
  b->rd.slots_aligned = align_slots();
  if ((e = finish_batch(b.get(), (int64_t)hl.max_slot)) != BQSR_OK || (e = layout_build(b.get(), st)) != BQSR_OK)
    return e;
  HIP_TRY(hipStreamSynchronize(st));
  *out = b.release();
  return ok();
}
}  // namespace

bqsr_status bqsr_sam_batch_create(bqsr_context* ctx, const bqsr_sam* s, const int32_t* ref_contig, int32_t n_ref,
                                  void* stream, bqsr_batch** out) {
  if (!ctx || !s || !out || n_ref < 0 || (n_ref && !ref_contig))
    return fail(BQSR_ERR_INVALID_ARG, "bqsr_sam_batch_create: bad arguments");
  if (s->ctx != ctx) return fail(BQSR_ERR_INVALID_ARG, "bqsr_sam_batch_create: parse of another context");
  *out = nullptr;
  PackCols C{s->flags, s->rg_id, s->ref, s->start, s->seq_off, s->qual_off, s->cig_off, s->md_off, s->seq, s->qual,
             s->md, s->cig, s->n_reads, s->seq_bytes, s->md_bytes, s->cig_ops, s->n_rg};
  return pack_batch_device(ctx, C, ref_contig, n_ref, stream, out);
}
