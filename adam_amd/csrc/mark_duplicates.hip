// MarkDuplicates on the device (include/adam_sam.h bqsr_sam_mark_duplicates,
// SURVEY.md §8 f3) over a parsed SAM's device columns.
//
// adam-core/.../rdd/MarkDuplicates.scala:24-111 as sorts and segmented passes:
//   1. SingleReadBucket (models/SingleReadBucket.scala:27-37): a 64-bit key
//      per read -- FNV-1a of (recordGroupId, readName) -- radix-sorted with
//      the read index (stable: a bucket's reads stay in input order); a run of
//      equal keys is a bucket once every read's QNAME bytes are compared with
//      the run head's (a hash collision sends the job to the host path).
//   2. per bucket: primary mapped / secondary mapped / unmapped reads, the
//      5' positions of its first two primary reads (ReferencePositionPair,
//      RichADAMRecord.fivePrimePosition: unclipped start, or unclipped end for
//      reverse reads), the library of allReads(0), the score of its primary
//      reads (MarkDuplicates.score: Σ phred >= 15, :37-39);
//   3. buckets ordered by first appearance, then (stable) by right position,
//      then by (left position, library): groupBy(leftPositionAndLibrary) and
//      groupBy(rightPosition) become runs (:60-66);
//   4. a thread per group walks it: no left position -> markReads(false);
//      pairs present -> fragments markReads(true), each right-position run
//      scoreAndMarkReads; else scoreAndMarkReads over the fragments (:67-108);
//      scoreAndMarkReads' sortBy is stable, so the first bucket of the best
//      score wins -- first appearance, the host path's rule (Spark's order
//      inside a group is its shuffle's: parity unpinned for ties);
//   5. a thread per read sets or clears FLAG 0x400.
// Included by bqsr_capi.cpp after mark_duplicates.cpp (the host path, kept
// for bqsr_mark_duplicates on host columns and as the collision fallback).

#include <rocprim/rocprim.hpp>

namespace mdupd {

constexpr int kThreads = 256;
// bucket outcome (per read: dup = f(outcome, read class))
enum : uint8_t { kNone = 0, kFragDup = 1, kWin = 2, kLose = 3 };
constexpr uint64_t kNoPos = 0;  // packed None (below every Some)

struct DevSam {
  const uint8_t* text;
  const uint64_t* line_span;
  const uint32_t* flags;
  const int32_t* rg_id;
  const int32_t* sq_id;
  const int64_t* start;
  const uint64_t* qual_off;
  const uint8_t* qual;
  const uint64_t* cig_off;
  const uint32_t* cig;
  const int32_t* rg_lib;  // library rank of read group i (0: no LB)
  int32_t n_rg;
  int64_t n;
  // columns without SAM text (bqsr_arrow): names at [name_beg[r], name_beg[r + 1]) of text,
  // name_valid[r] = 0 for a null readName, the library rank per read
  const uint64_t* name_beg;
  const uint8_t* name_valid;
  const int32_t* read_lib;
};

__device__ __forceinline__ int name_len(const DevSam& S, int64_t r, const uint8_t** p) {
  if (S.name_beg) {
    *p = S.text + S.name_beg[r];
    return (int)(S.name_beg[r + 1] - S.name_beg[r]);
  }
  const uint64_t a = S.line_span[2 * r], b = S.line_span[2 * r + 1];
  const uint8_t* t = S.text + a;
  int k = 0;
  while (a + (uint64_t)k < b && t[k] != '\t') ++k;
  *p = t;
  return k;
}

// ReferencePositionWithOrientation packed so that the packed order is
// (None < Some, referenceId, position, forward < reverse): 1 | ref+1 (15
// bits) | pos + 2^34 (35 bits) | neg; sets *bad when a field does not fit
__device__ __forceinline__ uint64_t pack_pos(int32_t ref, int64_t pos, bool neg, int* bad) {
  const int64_t rr = (int64_t)ref + 1, pp = pos + (1ll << 34);
  if (rr < 0 || rr >= (1 << 15) || pp < 0 || pp >= (1ll << 35)) atomicOr(bad, 2);
  return (1ull << 51) | ((uint64_t)(rr & 0x7FFF) << 36) | ((uint64_t)(pp & ((1ll << 35) - 1)) << 1) | (neg ? 1u : 0u);
}

// RichADAMRecord.fivePrimePosition (the host path's five_prime)
__device__ __forceinline__ int64_t five_prime(const DevSam& S, int64_t r) {
  const uint32_t* c = S.cig + S.cig_off[r];
  const int64_t n = (int64_t)(S.cig_off[r + 1] - S.cig_off[r]);
  const int64_t start = S.start[r];
  auto clipped = [](uint32_t e) {
    const uint32_t op = e & 0xF;
    return op == BQSR_CIGAR_S || op == BQSR_CIGAR_H;
  };
  if (!(S.flags[r] & BQSR_F_NEG_STRAND)) {
    int64_t p = start;
    for (int64_t i = 0; i < n && clipped(c[i]); ++i) p -= (int64_t)(c[i] >> 4);
    return p;
  }
  int64_t end = start;
  for (int64_t i = 0; i < n; ++i) {
    const uint32_t op = c[i] & 0xF;
    if (op == BQSR_CIGAR_M || op == BQSR_CIGAR_D || op == BQSR_CIGAR_N || op == BQSR_CIGAR_EQ || op == BQSR_CIGAR_X)
      end += (int64_t)(c[i] >> 4);
  }
  for (int64_t i = n - 1; i >= 0 && clipped(c[i]); --i) end += (int64_t)(c[i] >> 4);
  return end;
}

// 0 unmapped, 1 primary mapped, 2 secondary mapped (SingleReadBucket)
__device__ __forceinline__ int read_class(uint32_t f) {
  return !(f & BQSR_F_MAPPED) ? 0 : (f & BQSR_F_PRIMARY) ? 1 : 2;
}

extern "C" __global__ void __launch_bounds__(kThreads) mdup_keys(DevSam S, uint64_t* key, uint32_t* idx) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < S.n; r += (int64_t)gridDim.x * blockDim.x) {
    const uint8_t* p;
    const int k = name_len(S, r, &p);
    uint64_t h = 0xcbf29ce484222325ull;  // FNV-1a over (has rg, rg id, QNAME)
    const uint32_t f = S.flags[r];
    const uint32_t g = (f & BQSR_F_HAS_RG) ? (uint32_t)S.rg_id[r] + 1u : 0u;
    for (int i = 0; i < 4; ++i) h = (h ^ ((g >> (8 * i)) & 0xFFu)) * 0x100000001b3ull;
    for (int i = 0; i < k; ++i) h = (h ^ p[i]) * 0x100000001b3ull;
    key[r] = h;
    idx[r] = (uint32_t)r;
  }
}

// bucket heads of the sorted keys, and every read's name against its run head
extern "C" __global__ void __launch_bounds__(kThreads) mdup_heads(const uint64_t* ks, int64_t n, uint32_t* head) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    head[i] = (i == 0 || ks[i] != ks[i - 1]) ? 1u : 0u;
}

// bid = inclusive scan of head - 1; head_pos[b] = first sorted position of bucket b
extern "C" __global__ void __launch_bounds__(kThreads) mdup_head_pos(const uint32_t* head, const uint32_t* incl,
                                                                    int64_t n, uint32_t* head_pos) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    if (head[i]) head_pos[incl[i] - 1] = (uint32_t)i;
}

extern "C" __global__ void __launch_bounds__(kThreads) mdup_verify(DevSam S, const uint32_t* idx, const uint32_t* incl,
                                                                  const uint32_t* head_pos, int* bad) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < S.n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t h = head_pos[incl[i] - 1];
    if (h == (uint32_t)i) continue;
    const int64_t r = idx[i], r0 = idx[h];
    const uint32_t f = S.flags[r], f0 = S.flags[r0];
    const bool g = f & BQSR_F_HAS_RG, g0 = f0 & BQSR_F_HAS_RG;
    bool same = g == g0 && (!g || S.rg_id[r] == S.rg_id[r0]);
    const uint8_t *p, *p0;
    const int k = name_len(S, r, &p), k0 = name_len(S, r0, &p0);
    same = same && k == k0;
    for (int j = 0; same && j < k; ++j) same = p[j] == p0[j];
    if (!same) atomicOr(bad, 1);  // a 64-bit hash collision: the host path decides
  }
}

// per bucket: first appearance, its left/right positions, library, score
struct BucketInfo {
  uint64_t kll;    // left << 12 | library rank
  uint64_t kr;     // right
  uint32_t first;  // first read (input order)
  int32_t score;   // Σ score of the primary reads (int: the reference's Int sum)
};

extern "C" __global__ void __launch_bounds__(kThreads) mdup_buckets(DevSam S, const uint32_t* idx,
                                                                   const uint32_t* head_pos, int64_t nb,
                                                                   uint64_t* kll, uint64_t* kr, uint32_t* first,
                                                                   int32_t* score, int* bad) {
  for (int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; b < nb; b += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i0 = head_pos[b], i1 = b + 1 < nb ? (int64_t)head_pos[b + 1] : S.n;
    int64_t p0 = -1, p1 = -1, s0 = -1, u0 = -1;
    int32_t sc = 0;
    for (int64_t i = i0; i < i1; ++i) {
      const int64_t r = idx[i];
      const int c = read_class(S.flags[r]);
      if (c == 1) {
        if (p0 < 0) p0 = r; else if (p1 < 0) p1 = r;
        int32_t s = 0;  // MarkDuplicates.score: (char - 33).toByte, phred >= 15 summed
        for (uint64_t k = S.qual_off[r]; k < S.qual_off[r + 1]; ++k) {
          const int v = (int)(int8_t)(uint8_t)(S.qual[k] - 33);
          if (v >= 15) s += v;
        }
        sc += s;
      } else if (c == 2) {
        if (s0 < 0) s0 = r;
      } else if (u0 < 0) {
        u0 = r;
      }
    }
    uint64_t left = kNoPos, right = kNoPos;
    if (p0 >= 0) {
      const uint64_t a = pack_pos(S.sq_id[p0], five_prime(S, p0), S.flags[p0] & BQSR_F_NEG_STRAND, bad);
      if (p1 >= 0) {  // the first two primary reads, ordered (ReferencePositionPair)
        const uint64_t c = pack_pos(S.sq_id[p1], five_prime(S, p1), S.flags[p1] & BQSR_F_NEG_STRAND, bad);
        left = a < c ? a : c;
        right = a < c ? c : a;
      } else {
        left = a;
      }
    }
    const int64_t r0 = p0 >= 0 ? p0 : s0 >= 0 ? s0 : u0;  // allReads(0)
    const uint32_t f0 = S.flags[r0];
    int32_t lib = 0;
    if ((f0 & BQSR_F_HAS_RG) && S.rg_id[r0] >= 0 && S.rg_id[r0] < S.n_rg) lib = S.rg_lib[S.rg_id[r0]];
    if (lib >= 4096) atomicOr(bad, 4);
    kll[b] = (left << 12) | (uint64_t)(lib & 0xFFF);
    kr[b] = right;
    first[b] = (uint32_t)idx[i0];  // the run is in input order: its head is the bucket's first read
    score[b] = sc;
  }
}

// gather a 64-bit key through a permutation (the next stable sort pass's keys)
extern "C" __global__ void __launch_bounds__(kThreads) mdup_gather(const uint64_t* src, const uint32_t* perm,
                                                                  int64_t n, uint64_t* dst) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = src[perm[i]];
}
extern "C" __global__ void __launch_bounds__(kThreads) mdup_first_keys(const uint32_t* first, int64_t n,
                                                                      uint64_t* key, uint32_t* id) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    key[i] = first[i];
    id[i] = (uint32_t)i;
  }
}

__device__ __forceinline__ bool has_left(uint64_t kll) { return (kll >> 12) != kNoPos; }

// a thread per group head (sorted bucket order): the group's outcome per bucket
extern "C" __global__ void __launch_bounds__(kThreads) mdup_groups(const uint32_t* order, const uint64_t* kll,
                                                                  const uint64_t* kr, const int32_t* score, int64_t nb,
                                                                  uint8_t* outcome) {
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < nb; p += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t g = kll[order[p]];
    if (!has_left(g)) {  // buckets without a primary mapped read: markReads(false), each on its own
      outcome[order[p]] = kNone;  // (their group -- every such bucket of a library -- can be huge)
      continue;
    }
    if (p > 0 && kll[order[p - 1]] == g) continue;  // not a group head
    int64_t q = p;
    bool pairs = false;
    while (q < nb && kll[order[q]] == g) {
      pairs |= kr[order[q]] != kNoPos;
      ++q;
    }
    // scoring runs: each right position when the group has pairs (its
    // fragments are duplicates), else the whole group
    int64_t i = p;
    while (i < q) {
      const uint64_t rk = kr[order[i]];
      if (pairs && rk == kNoPos) {
        outcome[order[i]] = kFragDup;
        ++i;
        continue;
      }
      int64_t j = i;
      int64_t best = i;
      while (j < q && (!pairs || kr[order[j]] == rk)) {
        if (score[order[j]] > score[order[best]]) best = j;  // sortBy(-score), stable: the first best wins
        ++j;
      }
      for (int64_t k = i; k < j; ++k) outcome[order[k]] = k == best ? kWin : kLose;
      i = j;
    }
  }
}

// a thread per read: FLAG 0x400 from its bucket's outcome and its class
extern "C" __global__ void __launch_bounds__(kThreads) mdup_mark(const uint32_t* idx, const uint32_t* incl, int64_t n,
                                                                const uint8_t* outcome, uint32_t* flags,
                                                                unsigned long long* n_dup) {
  uint32_t cnt = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = idx[i];
    const uint8_t o = outcome[incl[i] - 1];
    const uint32_t f = flags[r];
    const int c = read_class(f);
    const bool dup = c == 1 ? (o == kFragDup || o == kLose) : c == 2 ? (o != kNone) : false;
    flags[r] = dup ? (f | BQSR_F_DUPLICATE) : (f & ~(uint32_t)BQSR_F_DUPLICATE);
    cnt += dup;
  }
  if (cnt) atomicAdd(n_dup, (unsigned long long)cnt);
}

}  // namespace mdupd

namespace {
// ADAM_BQSR_MARKDUP=host forces the host path (tests compare the two)
bool markdup_host_forced() {
  static const bool v = [] {
    const char* e = getenv("ADAM_BQSR_MARKDUP");
    return e && strcmp(e, "host") == 0;
  }();
  return v;
}
bqsr_status mark_duplicates_device(bqsr_sam* s, int64_t* n_duplicates, std::vector<void*>& tmp, bool* fallback);
}  // namespace

// device path; a hash collision or a field beyond the packed keys falls back
// to the host path (same rules, same order)
bqsr_status bqsr_sam_mark_duplicates(bqsr_sam* s, int64_t* n_duplicates) {
  if (!s) return fail(BQSR_ERR_INVALID_ARG, "null");
  HIP_TRY(hipSetDevice(s->ctx->device));
  if (s->n_reads == 0) {
    s->dup_marked = true;
    if (n_duplicates) *n_duplicates = 0;
    return ok();
  }
  if (markdup_host_forced() || s->n_reads >= (1ll << 31) - 1) return mark_duplicates_host(s, n_duplicates);
  std::vector<void*> tmp;
  bool fallback = false;
  const bqsr_status st = mark_duplicates_device(s, n_duplicates, tmp, &fallback);
  for (void* p : tmp) (void)hipFree(p);
  if (st == BQSR_OK && fallback) return mark_duplicates_host(s, n_duplicates);
  return st;
}

namespace {
bqsr_status mark_duplicates_device(bqsr_sam* s, int64_t* n_duplicates, std::vector<void*>& tmp, bool* fallback) {
  using namespace mdupd;
  const int64_t n = s->n_reads;
  // library ranks: LB strings of the read groups, sorted (1 + rank; 0 = no LB)
  std::vector<std::string> libs;
  for (size_t g = 0; g < s->rg_library.size(); ++g)
    if (g < s->rg_has_lb.size() && s->rg_has_lb[g]) libs.push_back(s->rg_library[g]);
  std::sort(libs.begin(), libs.end());
  libs.erase(std::unique(libs.begin(), libs.end()), libs.end());
  std::vector<int32_t> rg_lib((size_t)std::max(1, s->n_rg), 0);
  for (int32_t g = 0; g < s->n_rg; ++g)
    if ((size_t)g < s->rg_has_lb.size() && s->rg_has_lb[(size_t)g])
      rg_lib[(size_t)g] = 1 + (int32_t)(std::lower_bound(libs.begin(), libs.end(), s->rg_library[(size_t)g]) - libs.begin());
  auto alloc = [&](auto** p, size_t count) -> bqsr_status {
    const bqsr_status st = dalloc(tmp, p, std::max<size_t>(count, 1));
    return st;
  };
  hipStream_t st = hipStreamPerThread;
  uint64_t *key = nullptr, *key2 = nullptr, *kll = nullptr, *kr = nullptr, *ka = nullptr, *kb = nullptr;
  uint32_t *idx = nullptr, *idx2 = nullptr, *head = nullptr, *incl = nullptr, *hpos = nullptr, *first = nullptr;
  uint32_t *ord = nullptr, *ord2 = nullptr;
  int32_t *score = nullptr, *d_rglib = nullptr;
  uint8_t* outcome = nullptr;
  int* bad = nullptr;
  unsigned long long* ndup = nullptr;
  bqsr_status e = BQSR_OK;
  const size_t N = (size_t)n;
  if ((e = alloc(&key, N)) || (e = alloc(&key2, N)) || (e = alloc(&idx, N)) || (e = alloc(&idx2, N)) ||
      (e = alloc(&head, N)) || (e = alloc(&incl, N)) || (e = alloc(&hpos, N)) || (e = alloc(&kll, N)) ||
      (e = alloc(&kr, N)) || (e = alloc(&ka, N)) || (e = alloc(&kb, N)) || (e = alloc(&first, N)) ||
      (e = alloc(&ord, N)) || (e = alloc(&ord2, N)) || (e = alloc(&score, N)) || (e = alloc(&outcome, N)) ||
      (e = alloc(&d_rglib, rg_lib.size())) || (e = alloc(&bad, 1)) || (e = alloc(&ndup, 1)))
    return e;
  size_t tb = 0, tb2 = 0;
  HIP_TRY(rocprim::radix_sort_pairs(nullptr, tb, key, key2, idx, idx2, (size_t)n, 0, 64, st));
  HIP_TRY(rocprim::inclusive_scan(nullptr, tb2, head, incl, (size_t)n, rocprim::plus<uint32_t>(), st));
  void* temp = nullptr;
  if ((e = dalloc(tmp, (uint8_t**)&temp, std::max(tb, tb2)))) return e;
  tb = std::max(tb, tb2);
  DevSam S{s->d_text, s->line_span, s->flags, s->rg_id, s->sq_id, s->start, s->qual_off, s->qual, s->cig_off,
           s->cig, d_rglib, s->n_rg, n};
  const unsigned g = (unsigned)std::min<int64_t>((n + kThreads - 1) / kThreads, (int64_t)s->ctx->n_cu * 16);
  hipError_t he = hipMemcpyAsync(d_rglib, rg_lib.data(), rg_lib.size() * 4, hipMemcpyHostToDevice, st);
  if (he == hipSuccess) he = hipMemsetAsync(bad, 0, sizeof(int), st);
  if (he == hipSuccess) he = hipMemsetAsync(ndup, 0, sizeof(unsigned long long), st);
  if (he != hipSuccess) return fail(BQSR_ERR_DEVICE, hipGetErrorString(he));
  // 1. buckets: (rg, QNAME) keys sorted with the read index
  hipLaunchKernelGGL(mdup_keys, dim3(g), dim3(kThreads), 0, st, S, key, idx);
  size_t t1 = tb;
  HIP_TRY(rocprim::radix_sort_pairs(temp, t1, key, key2, idx, idx2, (size_t)n, 0, 64, st));
  hipLaunchKernelGGL(mdup_heads, dim3(g), dim3(kThreads), 0, st, (const uint64_t*)key2, n, head);
  size_t t2 = tb;
  HIP_TRY(rocprim::inclusive_scan(temp, t2, head, incl, (size_t)n, rocprim::plus<uint32_t>(), st));
  hipLaunchKernelGGL(mdup_head_pos, dim3(g), dim3(kThreads), 0, st, (const uint32_t*)head, (const uint32_t*)incl, n,
                     hpos);
  hipLaunchKernelGGL(mdup_verify, dim3(g), dim3(kThreads), 0, st, S, (const uint32_t*)idx2, (const uint32_t*)incl,
                     (const uint32_t*)hpos, bad);
  uint32_t nb32 = 0;
  HIP_TRY(hipMemcpyAsync(&nb32, incl + (n - 1), 4, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  const int64_t nb = nb32;
  const unsigned gb = (unsigned)std::min<int64_t>((nb + kThreads - 1) / kThreads, (int64_t)s->ctx->n_cu * 16);
  // 2. per bucket
  hipLaunchKernelGGL(mdup_buckets, dim3(gb), dim3(kThreads), 0, st, S, (const uint32_t*)idx2, (const uint32_t*)hpos,
                     nb, kll, kr, first, score, bad);
  // 3. bucket order: first appearance, then right position, then (left, library) -- stable passes
  hipLaunchKernelGGL(mdup_first_keys, dim3(gb), dim3(kThreads), 0, st, (const uint32_t*)first, nb, ka, ord2);
  size_t t3 = tb;
  HIP_TRY(rocprim::radix_sort_pairs(temp, t3, ka, kb, ord2, ord, (size_t)nb, 0, 32, st));
  hipLaunchKernelGGL(mdup_gather, dim3(gb), dim3(kThreads), 0, st, (const uint64_t*)kr, (const uint32_t*)ord, nb, ka);
  t3 = tb;
  HIP_TRY(rocprim::radix_sort_pairs(temp, t3, ka, kb, ord, ord2, (size_t)nb, 0, 52, st));
  hipLaunchKernelGGL(mdup_gather, dim3(gb), dim3(kThreads), 0, st, (const uint64_t*)kll, (const uint32_t*)ord2, nb, ka);
  t3 = tb;
  HIP_TRY(rocprim::radix_sort_pairs(temp, t3, ka, kb, ord2, ord, (size_t)nb, 0, 64, st));
  // 4. groups; 5. flags
  hipLaunchKernelGGL(mdup_groups, dim3(gb), dim3(kThreads), 0, st, (const uint32_t*)ord, (const uint64_t*)kll,
                     (const uint64_t*)kr, (const int32_t*)score, nb, outcome);
  int hbad = 0;
  HIP_TRY(hipMemcpyAsync(&hbad, bad, sizeof(int), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  if (hbad) {  // a hash collision, or a position / library beyond the packed keys
    *fallback = true;
    return ok();
  }
  hipLaunchKernelGGL(mdup_mark, dim3(g), dim3(kThreads), 0, st, (const uint32_t*)idx2, (const uint32_t*)incl, n,
                     (const uint8_t*)outcome, s->flags, ndup);
  unsigned long long hn = 0;
  HIP_TRY(hipMemcpyAsync(&hn, ndup, sizeof hn, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  HIP_TRY(hipGetLastError());
  s->dup_marked = true;
  if (n_duplicates) *n_duplicates = (int64_t)hn;
  return ok();
}
}  // namespace

// ------------------------------------------------ across partitions ----
// bqsr_dup_set (include/adam_sam.h): MarkDuplicates' groupBy over every
// partition of one input.  Each partition's parse leaves a compact record
// per read -- a 128-bit bucket key (two independent 64-bit hashes of (rg,
// QNAME)), class, packed 5' position and score of primary reads, library
// rank -- appended in input order, so a read's global index is its slot.
// finish() runs the single-parse passes over the records (the bucket keys
// sorted stably with the slot: a bucket's reads stay in input order) and
// leaves one duplicate bit per read; apply() sets the bits of a re-parse.
// Names of reads in different partitions are never compared: two names share
// a bucket only when both 64-bit hashes agree (no host fallback here).

namespace mdupd {

__device__ __forceinline__ void name_hashes(const DevSam& S, int64_t r, uint64_t* a, uint64_t* b) {
  const uint8_t* p;
  const int k = name_len(S, r, &p);
  uint64_t h = 0xcbf29ce484222325ull, g2 = 0x243F6A8885A308D3ull;
  const uint32_t f = S.flags[r];
  const uint32_t g = (f & BQSR_F_HAS_RG) ? (uint32_t)S.rg_id[r] + 1u : 0u;
  auto step2 = [](uint64_t x, uint32_t c) {
    x = (x ^ (c + 0x9E3779B97F4A7C15ull)) * 0xBF58476D1CE4E5B9ull;
    return x ^ (x >> 29);
  };
  for (int i = 0; i < 4; ++i) {
    const uint32_t c = (g >> (8 * i)) & 0xFFu;
    h = (h ^ c) * 0x100000001b3ull;
    g2 = step2(g2, c);
  }
  for (int i = 0; i < k; ++i) {
    h = (h ^ p[i]) * 0x100000001b3ull;
    g2 = step2(g2, p[i]);
  }
  const bool named = !S.name_valid || S.name_valid[r];
  g2 = step2(g2, named ? 0x100u + (uint32_t)k : 0x3FFu);  // a null readName is its own key
  if (!named) h ^= 0x9E3779B97F4A7C15ull;
  *a = h;
  *b = g2;
}

// a thread per read of one partition: its record at slot base + r
extern "C" __global__ void __launch_bounds__(kThreads) mdup_set_records(DevSam S, int64_t base, uint64_t* k1,
                                                                       uint64_t* k2, uint64_t* pos, int32_t* score,
                                                                       uint16_t* lib, uint8_t* cls, int* bad) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < S.n; r += (int64_t)gridDim.x * blockDim.x) {
    const int64_t o = base + r;
    name_hashes(S, r, &k1[o], &k2[o]);
    const uint32_t f = S.flags[r];
    const int c = read_class(f);
    uint64_t p = kNoPos;
    int32_t sc = 0;
    if (c == 1) {
      p = pack_pos(S.sq_id[r], five_prime(S, r), f & BQSR_F_NEG_STRAND, bad);
      for (uint64_t k = S.qual_off[r]; k < S.qual_off[r + 1]; ++k) {
        const int v = (int)(int8_t)(uint8_t)(S.qual[k] - 33);
        if (v >= 15) sc += v;
      }
    }
    int32_t lb = 0;
    if (S.read_lib) lb = S.read_lib[r];
    else if ((f & BQSR_F_HAS_RG) && S.rg_id[r] >= 0 && S.rg_id[r] < S.n_rg) lb = S.rg_lib[S.rg_id[r]];
    if (lb < 0 || lb >= 4096) atomicOr(bad, 4);
    pos[o] = p;
    score[o] = sc;
    lib[o] = (uint16_t)(lb & 0xFFF);
    cls[o] = (uint8_t)c;
  }
}

extern "C" __global__ void __launch_bounds__(kThreads) mdup_iota(int64_t n, uint32_t* idx) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    idx[i] = (uint32_t)i;
}

// heads of the (k1, k2)-sorted slots
extern "C" __global__ void __launch_bounds__(kThreads) mdup_set_heads(const uint64_t* k1s, const uint64_t* k2,
                                                                     const uint32_t* idx, int64_t n, uint32_t* head) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    head[i] = (i == 0 || k1s[i] != k1s[i - 1] || k2[idx[i]] != k2[idx[i - 1]]) ? 1u : 0u;
}

// mdup_buckets over the records
extern "C" __global__ void __launch_bounds__(kThreads) mdup_set_buckets(
    const uint64_t* pos, const int32_t* rscore, const uint16_t* lib, const uint8_t* cls, const uint32_t* idx,
    const uint32_t* head_pos, int64_t nb, int64_t n, uint64_t* kll, uint64_t* kr, uint32_t* first, int32_t* score) {
  for (int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; b < nb; b += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i0 = head_pos[b], i1 = b + 1 < nb ? (int64_t)head_pos[b + 1] : n;
    int64_t p0 = -1, p1 = -1, s0 = -1, u0 = -1;
    int32_t sc = 0;
    for (int64_t i = i0; i < i1; ++i) {
      const int64_t r = idx[i];
      const int c = cls[r];
      if (c == 1) {
        if (p0 < 0) p0 = r; else if (p1 < 0) p1 = r;
        sc += rscore[r];
      } else if (c == 2) {
        if (s0 < 0) s0 = r;
      } else if (u0 < 0) {
        u0 = r;
      }
    }
    uint64_t left = kNoPos, right = kNoPos;
    if (p0 >= 0) {
      const uint64_t a = pos[p0];
      if (p1 >= 0) {
        const uint64_t c = pos[p1];
        left = a < c ? a : c;
        right = a < c ? c : a;
      } else {
        left = a;
      }
    }
    const int64_t r0 = p0 >= 0 ? p0 : s0 >= 0 ? s0 : u0;
    kll[b] = (left << 12) | (uint64_t)lib[r0];
    kr[b] = right;
    first[b] = idx[i0];
    score[b] = sc;
  }
}

// the duplicate bit of every slot
extern "C" __global__ void __launch_bounds__(kThreads) mdup_set_mark(const uint32_t* idx, const uint32_t* incl,
                                                                    int64_t n, const uint8_t* outcome,
                                                                    const uint8_t* cls, uint32_t* bits,
                                                                    unsigned long long* n_dup) {
  uint32_t cnt = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t r = idx[i];
    const uint8_t o = outcome[incl[i] - 1];
    const int c = cls[r];
    const bool dup = c == 1 ? (o == kFragDup || o == kLose) : c == 2 ? (o != kNone) : false;
    if (dup) {
      atomicOr(&bits[r >> 5], 1u << (r & 31));
      ++cnt;
    }
  }
  if (cnt) atomicAdd(n_dup, (unsigned long long)cnt);
}

// a re-parse of slots [base, base + n): FLAG 0x400 from the bits
extern "C" __global__ void __launch_bounds__(kThreads) mdup_set_apply(const uint32_t* bits, int64_t base, int64_t n,
                                                                     uint32_t* flags, unsigned long long* n_dup) {
  uint32_t cnt = 0;
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t o = (uint64_t)(base + r);
    const bool dup = (bits[o >> 5] >> (o & 31)) & 1u;
    const uint32_t f = flags[r];
    flags[r] = dup ? (f | BQSR_F_DUPLICATE) : (f & ~(uint32_t)BQSR_F_DUPLICATE);
    cnt += dup;
  }
  if (cnt) atomicAdd(n_dup, (unsigned long long)cnt);
}

}  // namespace mdupd

struct bqsr_dup_set {
  bqsr_context* ctx = nullptr;
  int64_t n = 0, cap = 0;
  uint64_t *k1 = nullptr, *k2 = nullptr, *pos = nullptr;
  int32_t* score = nullptr;
  uint16_t* lib = nullptr;
  uint8_t* cls = nullptr;
  int* bad = nullptr;
  unsigned long long* cnt = nullptr;
  uint32_t* bits = nullptr;
  std::vector<int64_t> part_base, part_n;
  std::vector<std::string> libs;  // sorted LB strings of the header (the first partition's)
  bool have_libs = false, finished = false;
  int64_t n_dup = 0;
  void free_records() {
    for (void* p : {(void*)k1, (void*)k2, (void*)pos, (void*)score, (void*)lib, (void*)cls})
      if (p) (void)hipFree(p);
    k1 = k2 = pos = nullptr;
    score = nullptr;
    lib = nullptr;
    cls = nullptr;
    cap = 0;
  }
  ~bqsr_dup_set() {
    free_records();
    for (void* p : {(void*)bad, (void*)cnt, (void*)bits})
      if (p) (void)hipFree(p);
  }
};

namespace {
std::vector<std::string> sam_libraries(const bqsr_sam* s) {
  std::vector<std::string> libs;
  for (size_t g = 0; g < s->rg_library.size(); ++g)
    if (g < s->rg_has_lb.size() && s->rg_has_lb[g]) libs.push_back(s->rg_library[g]);
  std::sort(libs.begin(), libs.end());
  libs.erase(std::unique(libs.begin(), libs.end()), libs.end());
  return libs;
}

template <class T>
bqsr_status grow(T** p, int64_t n_old, int64_t cap, hipStream_t st) {
  T* q = nullptr;
  HIP_TRY(hipMalloc((void**)&q, (size_t)cap * sizeof(T)));
  if (*p && n_old) {
    const hipError_t e = hipMemcpyAsync(q, *p, (size_t)n_old * sizeof(T), hipMemcpyDeviceToDevice, st);
    if (e == hipSuccess) (void)hipStreamSynchronize(st);
    if (e != hipSuccess) {
      (void)hipFree(q);
      return fail(BQSR_ERR_DEVICE, hipGetErrorString(e));
    }
  }
  if (*p) (void)hipFree(*p);
  *p = q;
  return ok();
}
}  // namespace

bqsr_status bqsr_dup_set_create(bqsr_context* ctx, int64_t reads_hint, bqsr_dup_set** out) {
  if (!ctx || !out) return fail(BQSR_ERR_INVALID_ARG, "null");
  *out = nullptr;
  HIP_TRY(hipSetDevice(ctx->device));
  auto* d = new bqsr_dup_set();
  d->ctx = ctx;
  d->cap = std::max<int64_t>(0, reads_hint);
  hipStream_t st = hipStreamPerThread;
  bqsr_status e = BQSR_OK;
  if (d->cap) {
    const int64_t c = d->cap;
    d->cap = 0;
    if ((e = grow(&d->k1, 0, c, st)) || (e = grow(&d->k2, 0, c, st)) || (e = grow(&d->pos, 0, c, st)) ||
        (e = grow(&d->score, 0, c, st)) || (e = grow(&d->lib, 0, c, st)) || (e = grow(&d->cls, 0, c, st))) {
      delete d;
      return e;
    }
    d->cap = c;
  }
  if (hipMalloc((void**)&d->bad, sizeof(int)) != hipSuccess ||
      hipMalloc((void**)&d->cnt, sizeof(unsigned long long)) != hipSuccess) {
    delete d;
    return fail(BQSR_ERR_DEVICE, "dup set: out of device memory");
  }
  HIP_TRY(hipMemset(d->bad, 0, sizeof(int)));
  *out = d;
  return ok();
}

void bqsr_dup_set_destroy(bqsr_dup_set* d) { delete d; }

namespace {
bqsr_status dup_set_add_cols(bqsr_dup_set* d, const mdupd::DevSam& S);
}

bqsr_status bqsr_dup_set_add(bqsr_dup_set* d, const bqsr_sam* s) {
  using namespace mdupd;
  if (!d || !s) return fail(BQSR_ERR_INVALID_ARG, "null");
  if (d->finished) return fail(BQSR_ERR_INVALID_ARG, "bqsr_dup_set_add after bqsr_dup_set_finish");
  if (s->ctx != d->ctx) return fail(BQSR_ERR_INVALID_ARG, "parse of another context");
  HIP_TRY(hipSetDevice(d->ctx->device));
  const std::vector<std::string> libs = sam_libraries(s);
  if (!d->have_libs) {
    d->libs = libs;
    d->have_libs = true;
  } else if (libs != d->libs) {
    return fail(BQSR_ERR_INVALID_ARG, "partitions of one input must share the header's libraries");
  }
  std::vector<int32_t> rg_lib((size_t)std::max(1, s->n_rg), 0);
  for (int32_t g = 0; g < s->n_rg; ++g)
    if ((size_t)g < s->rg_has_lb.size() && s->rg_has_lb[(size_t)g])
      rg_lib[(size_t)g] = 1 + (int32_t)(std::lower_bound(libs.begin(), libs.end(), s->rg_library[(size_t)g]) - libs.begin());
  int32_t* d_rglib = nullptr;
  HIP_TRY(hipMalloc((void**)&d_rglib, rg_lib.size() * 4));
  hipError_t he = hipMemcpy(d_rglib, rg_lib.data(), rg_lib.size() * 4, hipMemcpyHostToDevice);
  bqsr_status e = he == hipSuccess ? BQSR_OK : fail(BQSR_ERR_DEVICE, hipGetErrorString(he));
  if (e == BQSR_OK) {
    mdupd::DevSam S{s->d_text, s->line_span, s->flags, s->rg_id, s->sq_id, s->start, s->qual_off, s->qual,
                    s->cig_off, s->cig, d_rglib, s->n_rg, s->n_reads};
    e = dup_set_add_cols(d, S);
  }
  (void)hipFree(d_rglib);
  return e;
}

namespace {
// one partition's records appended to the set (slots [d->n, d->n + S.n))
bqsr_status dup_set_add_cols(bqsr_dup_set* d, const mdupd::DevSam& S) {
  using namespace mdupd;
  const int64_t n = S.n;
  if (d->n + n >= (1ll << 32) - 1) return fail(BQSR_ERR_UNSUPPORTED, "more than 2^32 - 1 reads in a dup set");
  hipStream_t st = hipStreamPerThread;
  if (d->n + n > d->cap) {
    const int64_t c = std::max<int64_t>(d->n + n, d->cap + d->cap / 2 + 1024);
    bqsr_status e;
    if ((e = grow(&d->k1, d->n, c, st)) || (e = grow(&d->k2, d->n, c, st)) || (e = grow(&d->pos, d->n, c, st)) ||
        (e = grow(&d->score, d->n, c, st)) || (e = grow(&d->lib, d->n, c, st)) || (e = grow(&d->cls, d->n, c, st)))
      return e;
    d->cap = c;
  }
  d->part_base.push_back(d->n);
  d->part_n.push_back(n);
  if (n == 0) return ok();
  const unsigned g = (unsigned)std::min<int64_t>((n + kThreads - 1) / kThreads, (int64_t)d->ctx->n_cu * 16);
  hipLaunchKernelGGL(mdup_set_records, dim3(g), dim3(kThreads), 0, st, S, d->n, d->k1, d->k2, d->pos, d->score,
                     d->lib, d->cls, d->bad);
  hipError_t he = hipGetLastError();
  if (he == hipSuccess) he = hipStreamSynchronize(st);
  if (he != hipSuccess) return fail(BQSR_ERR_DEVICE, hipGetErrorString(he));
  d->n += n;
  return ok();
}
}  // namespace

bqsr_status bqsr_dup_set_finish(bqsr_dup_set* d, int64_t* n_duplicates) {
  using namespace mdupd;
  if (!d) return fail(BQSR_ERR_INVALID_ARG, "null");
  if (d->finished) {
    if (n_duplicates) *n_duplicates = d->n_dup;
    return ok();
  }
  HIP_TRY(hipSetDevice(d->ctx->device));
  hipStream_t st = hipStreamPerThread;
  const int64_t n = d->n;
  const size_t words = (size_t)(n + 31) / 32 + 1;
  HIP_TRY(hipMalloc((void**)&d->bits, words * 4));
  HIP_TRY(hipMemsetAsync(d->bits, 0, words * 4, st));
  HIP_TRY(hipMemsetAsync(d->cnt, 0, sizeof(unsigned long long), st));
  if (n == 0) {
    HIP_TRY(hipStreamSynchronize(st));
    d->finished = true;
    d->free_records();
    if (n_duplicates) *n_duplicates = 0;
    return ok();
  }
  int hbad = 0;
  HIP_TRY(hipMemcpyAsync(&hbad, d->bad, sizeof(int), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  if (hbad) return fail(BQSR_ERR_UNSUPPORTED, "MarkDuplicates: a position or library beyond the packed keys");
  std::vector<void*> tmp;
  struct Free {
    std::vector<void*>& v;
    ~Free() {
      for (void* p : v) (void)hipFree(p);
    }
  } fr{tmp};
  auto alloc = [&](auto** p, size_t count) -> bqsr_status { return dalloc(tmp, p, std::max<size_t>(count, 1)); };
  const size_t N = (size_t)n;
  uint64_t *ka = nullptr, *kb = nullptr, *kll = nullptr, *kr = nullptr;
  uint32_t *idx = nullptr, *idx2 = nullptr, *head = nullptr, *incl = nullptr, *hpos = nullptr, *first = nullptr;
  uint32_t *ord = nullptr, *ord2 = nullptr;
  int32_t* score = nullptr;
  uint8_t* outcome = nullptr;
  bqsr_status e = BQSR_OK;
  if ((e = alloc(&ka, N)) || (e = alloc(&kb, N)) || (e = alloc(&idx, N)) || (e = alloc(&idx2, N)) ||
      (e = alloc(&head, N)) || (e = alloc(&incl, N)) || (e = alloc(&hpos, N)))
    return e;
  size_t tb = 0, tb2 = 0;
  HIP_TRY(rocprim::radix_sort_pairs(nullptr, tb, ka, kb, idx, idx2, N, 0, 64, st));
  HIP_TRY(rocprim::inclusive_scan(nullptr, tb2, head, incl, N, rocprim::plus<uint32_t>(), st));
  tb = std::max(tb, tb2);
  void* temp = nullptr;
  if ((e = dalloc(tmp, (uint8_t**)&temp, tb))) return e;
  const unsigned g = (unsigned)std::min<int64_t>((n + kThreads - 1) / kThreads, (int64_t)d->ctx->n_cu * 16);
  // 1. slots sorted by (k1, k2), stable: k2 pass, then k1 pass
  hipLaunchKernelGGL(mdup_iota, dim3(g), dim3(kThreads), 0, st, n, idx);
  size_t t = tb;
  HIP_TRY(rocprim::radix_sort_pairs(temp, t, d->k2, kb, idx, idx2, N, 0, 64, st));
  hipLaunchKernelGGL(mdup_gather, dim3(g), dim3(kThreads), 0, st, (const uint64_t*)d->k1, (const uint32_t*)idx2, n, ka);
  t = tb;
  HIP_TRY(rocprim::radix_sort_pairs(temp, t, ka, kb, idx2, idx, N, 0, 64, st));
  hipLaunchKernelGGL(mdup_set_heads, dim3(g), dim3(kThreads), 0, st, (const uint64_t*)kb, (const uint64_t*)d->k2,
                     (const uint32_t*)idx, n, head);
  t = tb;
  HIP_TRY(rocprim::inclusive_scan(temp, t, head, incl, N, rocprim::plus<uint32_t>(), st));
  hipLaunchKernelGGL(mdup_head_pos, dim3(g), dim3(kThreads), 0, st, (const uint32_t*)head, (const uint32_t*)incl, n,
                     hpos);
  uint32_t nb32 = 0;
  HIP_TRY(hipMemcpyAsync(&nb32, incl + (n - 1), 4, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  const int64_t nb = nb32;
  if ((e = alloc(&kll, (size_t)nb)) || (e = alloc(&kr, (size_t)nb)) || (e = alloc(&first, (size_t)nb)) ||
      (e = alloc(&ord, (size_t)nb)) || (e = alloc(&ord2, (size_t)nb)) || (e = alloc(&score, (size_t)nb)) ||
      (e = alloc(&outcome, (size_t)nb)))
    return e;
  const unsigned gb = (unsigned)std::min<int64_t>((nb + kThreads - 1) / kThreads, (int64_t)d->ctx->n_cu * 16);
  // 2. per bucket; 3. bucket order; 4. groups (the single-parse passes)
  hipLaunchKernelGGL(mdup_set_buckets, dim3(gb), dim3(kThreads), 0, st, (const uint64_t*)d->pos,
                     (const int32_t*)d->score, (const uint16_t*)d->lib, (const uint8_t*)d->cls, (const uint32_t*)idx,
                     (const uint32_t*)hpos, nb, n, kll, kr, first, score);
  hipLaunchKernelGGL(mdup_first_keys, dim3(gb), dim3(kThreads), 0, st, (const uint32_t*)first, nb, ka, ord2);
  t = tb;
  HIP_TRY(rocprim::radix_sort_pairs(temp, t, ka, kb, ord2, ord, (size_t)nb, 0, 32, st));
  hipLaunchKernelGGL(mdup_gather, dim3(gb), dim3(kThreads), 0, st, (const uint64_t*)kr, (const uint32_t*)ord, nb, ka);
  t = tb;
  HIP_TRY(rocprim::radix_sort_pairs(temp, t, ka, kb, ord, ord2, (size_t)nb, 0, 52, st));
  hipLaunchKernelGGL(mdup_gather, dim3(gb), dim3(kThreads), 0, st, (const uint64_t*)kll, (const uint32_t*)ord2, nb, ka);
  t = tb;
  HIP_TRY(rocprim::radix_sort_pairs(temp, t, ka, kb, ord2, ord, (size_t)nb, 0, 64, st));
  hipLaunchKernelGGL(mdup_groups, dim3(gb), dim3(kThreads), 0, st, (const uint32_t*)ord, (const uint64_t*)kll,
                     (const uint64_t*)kr, (const int32_t*)score, nb, outcome);
  // 5. the bits
  hipLaunchKernelGGL(mdup_set_mark, dim3(g), dim3(kThreads), 0, st, (const uint32_t*)idx, (const uint32_t*)incl, n,
                     (const uint8_t*)outcome, (const uint8_t*)d->cls, d->bits, d->cnt);
  unsigned long long hn = 0;
  HIP_TRY(hipMemcpyAsync(&hn, d->cnt, sizeof hn, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  HIP_TRY(hipGetLastError());
  d->n_dup = (int64_t)hn;
  d->finished = true;
  d->free_records();
  if (n_duplicates) *n_duplicates = d->n_dup;
  return ok();
}

bqsr_status bqsr_dup_set_apply(bqsr_dup_set* d, int64_t part, bqsr_sam* s, int64_t* n_duplicates) {
  using namespace mdupd;
  if (!d || !s) return fail(BQSR_ERR_INVALID_ARG, "null");
  if (!d->finished) return fail(BQSR_ERR_INVALID_ARG, "bqsr_dup_set_apply before bqsr_dup_set_finish");
  if (part < 0 || (size_t)part >= d->part_n.size()) return fail(BQSR_ERR_INVALID_ARG, "no such partition");
  if (d->part_n[(size_t)part] != s->n_reads)
    return fail(BQSR_ERR_INVALID_ARG, "the parse's read count differs from the partition added");
  HIP_TRY(hipSetDevice(d->ctx->device));
  hipStream_t st = hipStreamPerThread;
  const int64_t n = s->n_reads;
  unsigned long long hn = 0;
  if (n) {
    HIP_TRY(hipMemsetAsync(d->cnt, 0, sizeof(unsigned long long), st));
    const unsigned g = (unsigned)std::min<int64_t>((n + kThreads - 1) / kThreads, (int64_t)d->ctx->n_cu * 16);
    hipLaunchKernelGGL(mdup_set_apply, dim3(g), dim3(kThreads), 0, st, (const uint32_t*)d->bits,
                       d->part_base[(size_t)part], n, s->flags, d->cnt);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(&hn, d->cnt, sizeof hn, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
  }
  s->dup_marked = true;
  if (n_duplicates) *n_duplicates = (int64_t)hn;
  return ok();
}
