// bqsr_capi.cpp -- host side of the C ABI declared in include/adam_bqsr.h.
//
// Owns HIP resources, packs ADAMRecord columns into the device layout
// (bqsr_internal.h), launches the kernels of bqsr_kernels.hip and maps device
// error words back to the reference's exception classes.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <dlfcn.h>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include <rocprim/rocprim.hpp>

#include "bqsr_internal.h"

using namespace bqsr;

// the kernels are compiled in this translation unit (one HIP module)
#include "bqsr_kernels.hip"
#include "bqsr_observe_lean.hip"
#include "bqsr_fold.hip"
#include "bqsr_transport.hip"

// ------------------------------------------------------------- errors -----

namespace {
thread_local std::string g_err;
thread_local int64_t g_err_read = -1;

bqsr_status fail(bqsr_status s, const std::string& msg, int64_t read = -1) {
  g_err = msg;
  g_err_read = read;
  return s;
}
bqsr_status ok() {
  g_err.clear();
  g_err_read = -1;
  return BQSR_OK;
}

#define HIP_TRY(expr)                                                                          \
  do {                                                                                         \
    hipError_t e_ = (expr);                                                                    \
    if (e_ != hipSuccess)                                                                      \
      return fail(BQSR_ERR_DEVICE, std::string(#expr " failed: ") + hipGetErrorString(e_));    \
  } while (0)

hipStream_t S(void* s) { return s ? (hipStream_t)s : hipStreamPerThread; }

const char* kStatusNames[] = {"OK",          "NULL_RG",      "MD_PARSE",       "CIGAR_SHORT", "BAD_REVCOMP_BASE",
                              "EMPTY_TABLE", "MISSING_KEY",  "QUAL_RANGE",     "NULL_FIELD",  "SEQ_SHORT",
                              "CIGAR_INVALID", "INVALID_ARG", "DEVICE",        "UNSUPPORTED", "SAM_PARSE"};

// map a device error key to (status, read) and record the message
bqsr_status from_err_key(unsigned long long k, int64_t read_base) {
  if (k == kNoError) return ok();
  const int code = (int)(k & 0xF);
  const int64_t read = (int64_t)(k >> 28) + read_base;
  const uint32_t o = (uint32_t)((k >> 8) & 0xFFFFF);
  char buf[160];
  snprintf(buf, sizeof buf, "%s at read %lld, read offset %u", kStatusNames[code], (long long)read, o);
  return fail((bqsr_status)code, buf, read);
}

// ------------------------------------------------- static numeric tables ---

// PhredUtils.phredToErrorProbabilityCache (PhredUtils.scala:22-24)
struct Pow10 {
  double v[256];
  Pow10() {
    for (int p = 0; p < 256; ++p) v[p] = std::pow(10.0, (double)(-p) / 10.0);
  }
};
const Pow10& pow10tab() {
  static Pow10 t;
  return t;
}

// log10 correctly rounded to double (one rounding of the long double result)
double cr_log10(double x) { return (double)log10l((long double)x); }
int32_t java_d2i(double d) {
  if (std::isnan(d)) return 0;
  if (d >= 2147483647.0) return INT32_MAX;
  if (d <= -2147483648.0) return INT32_MIN;
  return (int32_t)d;
}
int32_t phred_of(double p) { return java_d2i(-10.0 * cr_log10(p)); }  // PhredUtils.scala:34-38

// errorProbabilityToPhred is a non-increasing step function of p; its breaks:
// thr[n - qmin] = the largest positive double p with phred_of(p) >= n.
struct PhredThresholds {
  std::vector<double> thr;
  PhredThresholds() {
    thr.resize(kThrN);
    const uint64_t lo_bits = 1, hi_bits = 0x7FEFFFFFFFFFFFFFull;
    auto val = [](uint64_t b) {
      double d;
      memcpy(&d, &b, 8);
      return d;
    };
    for (int i = 0; i < kThrN; ++i) {
      const int n = kThrQmin + i;
      if (phred_of(val(hi_bits)) >= n) {
        thr[i] = val(hi_bits);
        continue;
      }
      if (phred_of(val(lo_bits)) < n) {
        thr[i] = 0.0;
        continue;
      }
      uint64_t a = lo_bits, b = hi_bits;  // phred(a) >= n > phred(b)
      while (b - a > 1) {
        const uint64_t m = a + (b - a) / 2;
        if (phred_of(val(m)) >= n) a = m; else b = m;
      }
      thr[i] = val(a);
    }
  }
};
const PhredThresholds& thresholds() {
  static PhredThresholds t;
  return t;
}

// Buckets of p by binade and top kQbBits mantissa bits (bqsr_internal.h):
// each holds at most one threshold, so Q = p <= thr_b ? q_b : q_b - 1.
struct PhredBuckets {
  std::vector<double> thr;
  std::vector<int16_t> q;
  PhredBuckets() {
    thr.resize(kQbN);
    q.resize(kQbN);
    const auto& T = thresholds().thr;
    for (int i = 0; i < kQbN; ++i) {
      const int e = kQbElo + (i >> kQbBits), m = i & ((1 << kQbBits) - 1);
      const double lo = std::ldexp(1.0 + (double)m / (1 << kQbBits), e);
      const double hi = std::ldexp(1.0 + (double)(m + 1) / (1 << kQbBits), e);
      const double last = std::nextafter(hi, 0.0);
      const int qhi = phred_of(lo), qlo = phred_of(last);
      if (qhi - qlo > 1 || qhi - kThrQmin < 0 || qhi - kThrQmin >= kThrN || qhi > 32767 || qhi < -32767) {
        q[(size_t)i] = -32768;  // not representable: full table
        thr[(size_t)i] = 0.0;
      } else {
        q[(size_t)i] = (int16_t)qhi;
        thr[(size_t)i] = T[(size_t)(qhi - kThrQmin)];
      }
    }
  }
};
const PhredBuckets& buckets() {
  static PhredBuckets b;
  return b;
}

int64_t table_words(const bqsr_dims& d) {
  const int64_t K = 60LL * (d.n_rg - 1) + 128, cells = 2LL * d.max_len + 1 + kCtxSlots;
  return K + 2 * K * cells;
}
TableGeom geom(const bqsr_dims& d) {
  TableGeom g;
  g.K = 60 * (d.n_rg - 1) + 128;
  g.L = d.max_len;
  g.C = 2 * d.max_len + 1;
  g.cells = g.C + kCtxSlots;
  return g;
}

constexpr size_t kLdsMax = 163840;
// LDS of the per-base passes: the context table (both), observe's u32 window
// [qw][wcells] x {obs, mm} + masked counts + block histogram, apply's char
// table [qw][cw][21]
// (the context table only for the chunk walk, bqsr_observe_chunks)
size_t observe_lds(int qw, int wcells, bool table) {
  return (table ? (size_t)kCtxTabBytes : 0) + (size_t)qw * wcells * 8 + (size_t)qw * 4 + kQBins * 4 +
         (size_t)kMkWords * 4;
}
// a piece's char table, rounded up to 16 B (the 16-B copy into LDS)
int64_t piece_bytes(int qw, int cw) { return ((int64_t)qw * cw * kCtxSlots + 15) & ~(int64_t)15; }
size_t apply_lds(int qw, int cw) { return 16 + (size_t)kMkWords * 4 + kCtxTabBytes + (size_t)piece_bytes(qw, cw); }
// bqsr_observe_lean: obs rows qw of orow words (nc copies of the cycle and the context cells), mm rows
// qw of wcells, masked qw, block histogram
int lean_orow(int nc, int cw) {
  int o = nc * (cw + kCtxCells);
  while ((o & 3) != 2) ++o;
  return o;
}
size_t lean_lds(int qw, int orow, int wcells) { return ((size_t)qw * (orow + wcells) + qw + kQBins + 1) * 4; }
// copies of the lean window's counters: the most (<= 4) whose rows still hold the batch's qual span
constexpr int kLeanCopiesMax = 4;
int observe_rows(int wcells, bool table) {
  int qw = kQBins;
  while (qw > 1 && observe_lds(qw, wcells, table) > kLdsMax) --qw;
  return qw;
}
// the host-packed layout is 16-aligned (ReadsDev::slots_aligned); device batches may be either
constexpr bool align_slots() { return true; }
// Fronts of a bucketed batch (OrderDev::n_base), for the chunk-walk passes:
// the sorted order becomes (front, read group, mate class), a front being a
// contiguous share of the read indices, and each key a workgroup of its own.
// Keyed ranges cut anywhere left every workgroup at its own point of the
// read-index space, so each cache line of the qual / base / bitmap columns,
// records and ReadInfo was fetched once per key whose reads it holds (PMC
// 2.1x algorithmic on cfg4, the MALL catching some); the workgroups of one
// front now start together and sweep the same range.  About eight pieces per
// CU (cfg4, 192 base keys: apply 5.7 -> 4.2 / 3.9 / 3.9 / 4.1 ms at 4 / 8 / 12
// / 32 fronts, observe 4.4 -> 4.0 ms), pieces of at least 8192 reads; none
// when that leaves fewer pieces than CUs or there are more base keys than 4
// per CU.  BQSR_TUNE_FRONTS forces f fronts, 0 turns them off (A/B, tests).
int fronts(int n_base, int n_cu, int64_t n_reads, int forced) {
  if (forced == 0) return 0;
  int f = forced;
  if (f < 0) {
    if (n_base > 4 * n_cu) return 0;
    f = (int)std::min<int64_t>((8 * n_cu + n_base - 1) / n_base, n_reads / (8192 * (int64_t)n_base));
    if ((int64_t)std::max(f, 1) * n_base < n_cu) return 0;
    f = std::max(f, 1);
  }
  while (f > 1 && (int64_t)f * n_base > 4096) --f;  // keys kept in the sort's LDS
  return f;
}
int apply_rows(int cw) {
  int qw = kQBins;
  while (qw > 1 && apply_lds(qw, cw) > kLdsMax) --qw;
  return qw;
}

}  // namespace

// ------------------------------------------------------------ handles -----

struct bqsr_context {
  int device = 0;
  int n_cu = 256;
  double* d_pow10 = nullptr;  // 256 doubles
  double* d_thr = nullptr;    // kThrN doubles
  double* d_qbt = nullptr;    // kQbN bucket thresholds
  int16_t* d_qbq = nullptr;   // kQbN bucket phred values
  // upload_staged: a pinned ring for large pageable uploads (allocated on first use)
  std::mutex stage_mu;
  uint8_t* stage[2] = {nullptr, nullptr};
  hipEvent_t stage_ev[2] = {nullptr, nullptr};
  // bqsr_context_tune
  int tune_order = -1;
  int tune_fronts = -1;
  int tune_keymajor = 0;
  int tune_bgzf = 1;  // BAM ingest: BGZF inflated on the device (BQSR_TUNE_BGZF), 0 by host threads
};

namespace {
// H2D of a large pageable host buffer (SAM text, inflated BAM records):
// chunks copied by host threads into a pinned ring of two buffers while the
// DMA engine moves the previous chunk -- the runtime's own pageable path
// stages through one thread's memcpy (~20 GB/s).  Synchronous on return.
constexpr size_t kStageChunk = 64ull << 20;
// the ring's two pinned buffers and events, allocated on first use (caller holds stage_mu)
bqsr_status stage_ring(bqsr_context* ctx) {
  for (int i = 0; i < 2; ++i) {
    if (!ctx->stage[i]) HIP_TRY(hipHostMalloc((void**)&ctx->stage[i], kStageChunk, hipHostMallocDefault));
    if (!ctx->stage_ev[i]) HIP_TRY(hipEventCreateWithFlags(&ctx->stage_ev[i], hipEventDisableTiming));
  }
  return BQSR_OK;
}
bqsr_status upload_staged(bqsr_context* ctx, void* dst, const void* src, size_t n, hipStream_t s) {
  hipPointerAttribute_t attr{};
  const bool pinned = hipPointerGetAttributes(&attr, src) == hipSuccess && attr.type == hipMemoryTypeHost;
  (void)hipGetLastError();  // (pageable memory: the query fails)
  if (pinned || n < 2 * kStageChunk) {
    HIP_TRY(hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, s));
    HIP_TRY(hipStreamSynchronize(s));
    return BQSR_OK;
  }
  std::lock_guard<std::mutex> lock(ctx->stage_mu);
  bqsr_status st = stage_ring(ctx);
  if (st != BQSR_OK) return st;
  const int nth = (int)std::max(1u, std::min(8u, std::thread::hardware_concurrency()));
  const uint8_t* p = (const uint8_t*)src;
  uint8_t* d = (uint8_t*)dst;
  int k = 0;
  for (size_t off = 0; off < n; off += kStageChunk, k ^= 1) {
    const size_t len = std::min(kStageChunk, n - off);
    HIP_TRY(hipEventSynchronize(ctx->stage_ev[k]));  // the ring buffer's previous DMA is done
    std::vector<std::thread> th;
    for (int t = 0; t < nth; ++t)
      th.emplace_back([&, t] {
        const size_t a = len * (size_t)t / (size_t)nth, b = len * (size_t)(t + 1) / (size_t)nth;
        memcpy(ctx->stage[k] + a, p + off + a, b - a);
      });
    for (auto& x : th) x.join();
    HIP_TRY(hipMemcpyAsync(d + off, ctx->stage[k], len, hipMemcpyHostToDevice, s));
    HIP_TRY(hipEventRecord(ctx->stage_ev[k], s));
  }
  HIP_TRY(hipStreamSynchronize(s));
  return BQSR_OK;
}
}  // namespace

struct bqsr_sites {
  bqsr_context* ctx = nullptr;
  std::vector<std::string> names;
  int64_t* pos = nullptr;
  uint64_t* off = nullptr;
  uint32_t* bucket = nullptr;
  uint64_t* bucket_off = nullptr;
  int64_t* bucket_base = nullptr;
  uint64_t* bm = nullptr;
  uint64_t* bm_off = nullptr;
  int64_t* bm_base = nullptr;
  int32_t n = 0;
  int32_t shift = 8;
  SitesDev dev() const { return SitesDev{pos, off, bucket, bucket_off, bucket_base, bm, bm_off, bm_base, n, shift}; }
};

struct bqsr_batch {
  bqsr_context* ctx = nullptr;
  bool owned = false;
  ReadsDev rd{};
  bqsr_dims dims{1, 1};
  int64_t n_slots = 0;
  int64_t n_bases = 0;
  int32_t q_lo = 0, rg_lo = 0;  // LDS window choice
  bool have_qhist = false;      // q_lo follows qhist at each launch's window width
  int64_t qhist[kQBins] = {0};
  int64_t qhigh = 0;            // quals >= 128 (negative Java bytes) in the batch
  std::vector<void*> allocs;
  std::vector<size_t> staged_cnt;  // column element counts (bqsr_batch_create_staged)
  const bqsr_staged* staged_src = nullptr;  // the one staged partition this batch uploads
  uint8_t* d_bases2 = nullptr;     // staged: the uploaded 2-bit base codes
  uint64_t* d_bexc = nullptr;      //         and their exceptions
  uint64_t* d_qcodes = nullptr;    // staged: the uploaded qual chunks (codes, base bytes)
  uint8_t* d_qbase = nullptr;
  uint64_t* d_qexc = nullptr;      //         and their exceptions
  // per-read prep results (valid once `prepped`)
  ReadInfo* d_info = nullptr;
  uint64_t* d_sbits = nullptr;  // slot bitmap (PrepParams::sbits)
  uint32_t* d_work = nullptr;   // prep worklist (PrepParams::work), count at d_work[n_reads]
  uint64_t* d_bnd = nullptr;    // prep pass 1 wavefront-boundary shares (PrepParams::bnd)
  int64_t sbits_words = 0;      // even: the apply kernel clears it 16 B at a time
  bool err_fresh = false;     // bqsr_job_reset_async reset the error words since the last prep
  bool prepped = false;
  const bqsr_sites* prep_sites = nullptr;
  // per-call scratch
  uint32_t* d_hq = nullptr;        // [n_blocks][128] fold blocks' qual histograms
  uint32_t* d_qmask = nullptr;     // [4] their bins holding a base (bqsr_fold_plan)
  bool hq_valid = false;           // d_qmask written by a fold of this batch (its quals and trims are fixed)
  FoldParams fold{};               // the fold's device buffers (FoldParams)
  uint32_t* d_part = nullptr;      // per-block window counts
  size_t part_words = 0;
  uint8_t* d_chars = nullptr;      // apply: the pieces' char tables (ApplyParams::chars)
  const bqsr_lut* chars_lut = nullptr;  // the LUT they were built from (BQSR_STAGE_LUT)
  uint64_t* d_off64 = nullptr;     // bqsr_compact_outputs_async scratch (lengths, scan)
  int64_t off64_n = -1;
  size_t chars_bytes = 0;
  unsigned long long* d_err = nullptr;  // [kErrWords]: observe, apply-prep, apply-kernel errors, exception count
  double* d_em = nullptr;
  int32_t n_blocks = 0;
  // read-group buckets (OrderDev): several read groups -> the per-base passes
  // walk the reads grouped by read group
  bool bucketed = false;
  int32_t n_keys = 1;   // n_base * fronts
  int32_t n_base = 1;   // 2 * read group + mate class
  int32_t fronts = 0;   // > 0: front-ordered pieces, a chunk-walk workgroup per key (OrderDev::n_base)
  uint32_t* d_perm = nullptr;
  int64_t* d_key_off = nullptr;
  uint32_t* d_key_cnt = nullptr;
  uint32_t* d_cursor = nullptr;
  // key-major copy of the quals / base codes (layout_build): the bucketed
  // passes' reads of a piece contiguous; the perm it follows is computed once
  // (allocated once with the batch's other buffers, key_major_alloc; valid once km_ready)
  uint8_t *k_qual = nullptr, *k_bases = nullptr;
  uint64_t* d_kslot = nullptr;
  uint64_t* d_kspan = nullptr;  // layout_build scratch: slot spans in perm order, and the scan's temp
  void* d_ktemp = nullptr;
  size_t ktemp_bytes = 0;
  bool km_ready = false;
  double km_alloc_ms = -1.0, km_build_ms = -1.0;  // wall times of the copy's allocation / kernels (bqsr_batch_layout_times)
  bool perm_static = false;  // d_perm / d_key_off built once (layout_build): prep skips the key sort
  OrderDev order() const {
    return bucketed ? OrderDev{d_perm, d_key_off, n_keys, fronts > 0 ? n_base : 0, km_ready ? d_kslot : nullptr}
                    : OrderDev{nullptr, nullptr, 1};
  }
  // the reads as the per-base passes see them (qual / base columns: the key-major copy when there is one)
  ReadsDev pass_rd() const {
    ReadsDev r = rd;
    if (bucketed && km_ready) {
      r.qual = k_qual;
      r.bases = k_bases;
    }
    return r;
  }
  // workgroups of the chunk-walk passes: a piece each with fronts, else the fold's blocks
  int32_t pass_blocks() const { return bucketed && fronts > 0 ? n_keys : n_blocks; }
  uint64_t* h_status = nullptr;  // pinned: bqsr_job_result's one transfer (kJobStatusWords)
  // bucketed batches: the fold on a stream of its own, beside the observe
  // kernel and bqsr_window_reduce -- it needs prep's trims, not the table
  // (ev_obs: recorded after prep, pending until a FOLD stage takes it)
  hipStream_t side = nullptr;
  hipEvent_t ev_obs = nullptr, ev_fold = nullptr;
  bool obs_pending = false;
  ~bqsr_batch() {
    if (side) (void)hipStreamDestroy(side);
    for (hipEvent_t e : {ev_obs, ev_fold})
      if (e) (void)hipEventDestroy(e);
    if (d_part) (void)hipFree(d_part);
    if (d_off64) (void)hipFree(d_off64);
    if (d_chars) (void)hipFree(d_chars);
    if (h_status) (void)hipHostFree(h_status);
    for (void* p : allocs) (void)hipFree(p);
  }
};

struct bqsr_table {
  bqsr_context* ctx = nullptr;
  bqsr_dims dims{1, 1};
  int64_t* words = nullptr;
  bool owned = false;
  ~bqsr_table() {
    if (owned && words) (void)hipFree(words);
  }
  TableGeom g() const { return geom(dims); }
  int64_t* touched() const { return words; }
  int64_t* obs() const { return words + g().K; }
  int64_t* mm() const { return words + g().K + (int64_t)g().K * g().cells; }
};

struct bqsr_lut {
  bqsr_context* ctx = nullptr;
  bqsr_dims dims{1, 1};
  int32_t n_groups = 0;
  std::vector<void*> allocs;
  int64_t *qk_obs = nullptr, *qk_mm = nullptr, *grp_obs = nullptr, *grp_mm = nullptr;
  uint8_t *grp_ok = nullptr, *key_ok = nullptr, *rq_ok = nullptr;
  double *a2 = nullptr, *s1 = nullptr, *d2 = nullptr;
  FinalOut* d_out = nullptr;
  FinalOut out{};
  bool out_pending = false;  // bqsr_finalize_device: `out` not copied back yet (bqsr_job_result / lut_out)
  // host mirror for stats / shifts queries (filled lazily)
  bool host_ready = false;
  std::vector<int64_t> h_words, h_qk_obs, h_qk_mm, h_grp_obs, h_grp_mm;
  std::vector<uint8_t> h_grp_ok;
  const bqsr_table* src = nullptr;
  ~bqsr_lut() {
    for (void* p : allocs) (void)hipFree(p);
  }
};

namespace {
template <class T>
bqsr_status dalloc(std::vector<void*>& v, T** p, size_t n) {
  void* q = nullptr;
  HIP_TRY(hipMalloc(&q, std::max<size_t>(n, 1) * sizeof(T)));
  v.push_back(q);
  *p = (T*)q;
  return BQSR_OK;
}
}  // namespace

// ------------------------------------------------------------- library ----

extern "C" {

int bqsr_abi_version(void) { return BQSR_ABI_VERSION; }
const char* bqsr_last_error(void) { return g_err.c_str(); }
int64_t bqsr_last_error_read(void) { return g_err_read; }
const char* bqsr_status_name(bqsr_status s) {
  if ((int)s < 0 || (int)s > 14) return "UNKNOWN";
  return kStatusNames[(int)s];
}

bqsr_status bqsr_context_tune(bqsr_context* ctx, int knob, int64_t value) {
  if (!ctx) return fail(BQSR_ERR_INVALID_ARG, "bqsr_context_tune: null context");
  switch (knob) {
    case BQSR_TUNE_ORDER:
      if (value < -1 || value > 1) break;
      ctx->tune_order = (int)value;
      return BQSR_OK;
    case BQSR_TUNE_FRONTS:
      if (value < -1 || value > 4096) break;
      ctx->tune_fronts = (int)value;
      return BQSR_OK;
    case BQSR_TUNE_KEYMAJOR:
      if (value < 0 || value > 1) break;
      ctx->tune_keymajor = (int)value;
      return BQSR_OK;
    case BQSR_TUNE_FUSED_PREP:  // (the fused form was removed in round 6: only "off" is accepted)
      if (value != 0) break;
      return BQSR_OK;
    case BQSR_TUNE_BGZF:
      if (value < 0 || value > 1) break;
      ctx->tune_bgzf = (int)value;
      return BQSR_OK;
    default:
      return fail(BQSR_ERR_INVALID_ARG, "bqsr_context_tune: unknown knob");
  }
  return fail(BQSR_ERR_INVALID_ARG, "bqsr_context_tune: value out of range");
}

bqsr_status bqsr_context_create(int device, bqsr_context** out) {
  if (!out) return fail(BQSR_ERR_INVALID_ARG, "null out");
  HIP_TRY(hipSetDevice(device));
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, device));
  bqsr_context* c = new bqsr_context;
  c->device = device;
  c->n_cu = prop.multiProcessorCount;
  hipError_t e = hipMalloc(&c->d_pow10, 256 * sizeof(double));
  if (e == hipSuccess) e = hipMalloc(&c->d_thr, kThrN * sizeof(double));
  if (e == hipSuccess) e = hipMemcpy(c->d_pow10, pow10tab().v, 256 * sizeof(double), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(c->d_thr, thresholds().thr.data(), kThrN * sizeof(double), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMalloc(&c->d_qbt, kQbN * sizeof(double));
  if (e == hipSuccess) e = hipMalloc(&c->d_qbq, kQbN * sizeof(int16_t));
  if (e == hipSuccess) e = hipMemcpy(c->d_qbt, buckets().thr.data(), kQbN * sizeof(double), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(c->d_qbq, buckets().q.data(), kQbN * sizeof(int16_t), hipMemcpyHostToDevice);
  for (const void* f : {(const void*)bqsr_apply_kernel, (const void*)bqsr_observe_chunks,
                        (const void*)bqsr_observe_lean<true>})
    if (e == hipSuccess) e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsMax);
  if (e == hipSuccess)
    e = hipFuncSetAttribute((const void*)bqsr_fold_hist, hipFuncAttributeMaxDynamicSharedMemorySize, (int)fold_hist_lds());
  if (e == hipSuccess)
    e = hipFuncSetAttribute((const void*)bqsr_fold_chain, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)chain_lds(kMaxFoldBlocks));
  if (e != hipSuccess) {
    bqsr_context_destroy(c);
    return fail(BQSR_ERR_DEVICE, std::string("context: ") + hipGetErrorString(e));
  }
  *out = c;
  return ok();
}

void bqsr_context_destroy(bqsr_context* c) {
  if (!c) return;
  if (c->d_pow10) (void)hipFree(c->d_pow10);
  if (c->d_thr) (void)hipFree(c->d_thr);
  if (c->d_qbt) (void)hipFree(c->d_qbt);
  if (c->d_qbq) (void)hipFree(c->d_qbq);
  for (int i = 0; i < 2; ++i) {
    if (c->stage[i]) (void)hipHostFree(c->stage[i]);
    if (c->stage_ev[i]) (void)hipEventDestroy(c->stage_ev[i]);
  }
  delete c;
}

// ---------------------------------------------------------------- sites ----

bqsr_status bqsr_sites_create(bqsr_context* ctx, const char* const* contigs, const int64_t* const* pos,
                              const uint64_t* n, int32_t n_contigs, bqsr_sites** out) {
  if (!ctx || !out || n_contigs < 0 || (n_contigs > 0 && (!contigs || !pos || !n)))
    return fail(BQSR_ERR_INVALID_ARG, "bqsr_sites_create: bad arguments");
  HIP_TRY(hipSetDevice(ctx->device));
  bqsr_sites* s = new bqsr_sites;
  s->ctx = ctx;
  s->n = n_contigs;
  std::vector<int64_t> all;
  std::vector<uint64_t> off(1, 0);
  std::vector<uint32_t> bucket;
  std::vector<uint64_t> boff(1, 0);
  std::vector<int64_t> bbase;
  std::vector<uint64_t> bm, bmoff(1, 0);
  std::vector<int64_t> bmbase;
  for (int32_t c = 0; c < n_contigs; ++c) {
    s->names.emplace_back(contigs[c] ? contigs[c] : "");
    std::vector<int64_t> v(pos[c], pos[c] + n[c]);  // SnpTable: Set[Long] per contig
    std::sort(v.begin(), v.end());
    v.erase(std::unique(v.begin(), v.end()), v.end());
    const int64_t base = v.empty() ? 0 : v.front();
    const int64_t nb = v.empty() ? 0 : ((v.back() - base) >> s->shift) + 1;
    size_t j = 0;
    for (int64_t b = 0; b < nb; ++b) {
      const int64_t lo = base + (b << s->shift);
      while (j < v.size() && v[j] < lo) ++j;
      bucket.push_back((uint32_t)j);
    }
    bbase.push_back(base);
    boff.push_back(bucket.size());
    // the position bitmap (a 16-24 B read per read in the prep kernel's
    // common path), unless it would hold over 64 words per site
    const int64_t b0 = v.empty() ? 0 : (int64_t)((uint64_t)base & ~(uint64_t)63);  // floor to 64
    const int64_t nw = v.empty() ? 0 : ((v.back() - b0) >> 6) + 1;
    const bool dense = nw > 0 && nw <= 64 * (int64_t)v.size() + 64 && nw <= (int64_t(1) << 28);
    if (dense) {
      const size_t w0 = bm.size();
      bm.resize(w0 + (size_t)nw, 0ull);
      for (const int64_t p : v) bm[w0 + (size_t)((p - b0) >> 6)] |= 1ull << ((p - b0) & 63);
    }
    bmbase.push_back(dense ? b0 : 0);
    bmoff.push_back(bm.size());
    all.insert(all.end(), v.begin(), v.end());
    off.push_back(all.size());
  }
  std::vector<void*> keep;
  auto up = [&](auto** dst, const auto& src) -> hipError_t {
    using T = typename std::remove_reference<decltype(src[0])>::type;
    hipError_t e = hipMalloc((void**)dst, std::max<size_t>(src.size(), 1) * sizeof(T));
    if (e != hipSuccess) return e;
    if (!src.empty()) e = hipMemcpy(*dst, src.data(), src.size() * sizeof(T), hipMemcpyHostToDevice);
    return e;
  };
  hipError_t e = up(&s->pos, all);
  if (e == hipSuccess) e = up(&s->off, off);
  if (e == hipSuccess) e = up(&s->bucket, bucket);
  if (e == hipSuccess) e = up(&s->bucket_off, boff);
  if (e == hipSuccess) e = up(&s->bucket_base, bbase);
  if (e == hipSuccess) e = up(&s->bm, bm);
  if (e == hipSuccess) e = up(&s->bm_off, bmoff);
  if (e == hipSuccess) e = up(&s->bm_base, bmbase);
  if (e != hipSuccess) {
    bqsr_sites_destroy(s);
    return fail(BQSR_ERR_DEVICE, std::string("sites upload: ") + hipGetErrorString(e));
  }
  *out = s;
  return ok();
}

void bqsr_sites_destroy(bqsr_sites* s) {
  if (!s) return;
  for (void* p : {(void*)s->pos, (void*)s->off, (void*)s->bucket, (void*)s->bucket_off, (void*)s->bucket_base,
                  (void*)s->bm, (void*)s->bm_off, (void*)s->bm_base})
    if (p) (void)hipFree(p);
  delete s;
}

// ---------------------------------------------------------------- batch ----

namespace {

inline uint8_t code_of(uint8_t c) {
  switch (c) {
    case 'A': return kCodeA;
    case 'C': return kCodeC;
    case 'G': return kCodeG;
    case 'T': return kCodeT;
    case 'N': return kCodeN;
    default: return kCodeOther;
  }
}

Window window_rows(const bqsr_batch* b, int max_rows);

bqsr_status finish_batch(bqsr_batch* b, int64_t max_slot_len) {
  if (max_slot_len > kMaxReadLen)
    return fail(BQSR_ERR_UNSUPPORTED, "reads longer than " + std::to_string(kMaxReadLen) + " bases are not supported");
  const int64_t n = b->rd.n_reads;
  b->rd.reads_per_tile = (int32_t)std::max<int64_t>(1, std::min<int64_t>(kMaxTileReads, kTileSlots / std::max<int64_t>(1, max_slot_len)));
  b->rd.n_tiles = (n + b->rd.reads_per_tile - 1) / b->rd.reads_per_tile;
  b->n_blocks = std::min(b->ctx->n_cu, kMaxFoldBlocks);
  bqsr_status st;
  if ((st = dalloc(b->allocs, &b->d_hq, (size_t)b->n_blocks * kQBins)) != BQSR_OK) return st;
  if ((st = dalloc(b->allocs, &b->d_qmask, 4)) != BQSR_OK) return st;
  {  // the fold's buffers (bqsr_fold.hip)
    FoldParams& F = b->fold;
    const size_t nt = (size_t)std::max<int64_t>(1, b->rd.n_tiles), nbk = (size_t)b->n_blocks;
    F.stream_cap = std::max<int64_t>(1 << 20, std::min<int64_t>(16 << 20, b->rd.n_slots));
    if ((st = dalloc(b->allocs, &F.blk, nbk)) != BQSR_OK || (st = dalloc(b->allocs, &F.cand_list, nbk)) != BQSR_OK ||
        (st = dalloc(b->allocs, &F.n_cand, 1)) != BQSR_OK || (st = dalloc(b->allocs, &F.delta, 1)) != BQSR_OK ||
        (st = dalloc(b->allocs, &F.rtile, nt)) != BQSR_OK || (st = dalloc(b->allocs, &F.ntile, nt)) != BQSR_OK ||
        (st = dalloc(b->allocs, &F.dtile, nt * kSegBinades)) != BQSR_OK ||
        (st = dalloc(b->allocs, &F.seg, nbk * kFoldMaxSegs)) != BQSR_OK ||
        (st = dalloc(b->allocs, &F.seg_base, nbk)) != BQSR_OK || (st = dalloc(b->allocs, &F.nseg, nbk)) != BQSR_OK ||
        (st = dalloc(b->allocs, &F.seg_used, 1)) != BQSR_OK ||
        (st = dalloc(b->allocs, &F.streams, (size_t)F.stream_cap + 64)) != BQSR_OK ||
        (st = dalloc(b->allocs, &F.csum, (size_t)F.stream_cap / 64 * 2 + 2)) != BQSR_OK ||
        (st = dalloc(b->allocs, &F.stream_used, 1)) != BQSR_OK)
      return st;
  }
  if ((st = dalloc(b->allocs, &b->d_err, kErrWords)) != BQSR_OK) return st;
  if ((st = dalloc(b->allocs, &b->d_info, (size_t)std::max<int64_t>(1, n))) != BQSR_OK) return st;
  b->sbits_words = (b->rd.n_slots / 32 + 5) & ~(int64_t)1;  // the per-base passes read 3 words from any slot's word
  if ((st = dalloc(b->allocs, &b->d_sbits, (size_t)b->sbits_words)) != BQSR_OK) return st;
  if ((st = dalloc(b->allocs, &b->d_em, 2)) != BQSR_OK) return st;
  if ((st = dalloc(b->allocs, &b->d_bnd, (size_t)2 * (size_t)(n / 64 + kPrepChunk / 64 + 1))) != BQSR_OK) return st;
  if ((st = dalloc(b->allocs, &b->d_work,
                   (size_t)(n + kPrepChunk) + (size_t)std::max<int64_t>(n / kPrepChunk + 1, kMaxFoldBlocks))) != BQSR_OK)
    return st;
  // read-group buckets (OrderDev): on for several read groups, or when the
  // apply window over all cycle cells would leave more than 0.1% of the bases
  // outside its qual rows (BQSR_TUNE_ORDER forces either)
  if (b->ctx->tune_order >= 0) {
    b->bucketed = b->ctx->tune_order == 1;
  } else {
    b->bucketed = b->dims.n_rg > 1;
    if (!b->bucketed && b->have_qhist) {
      const int cw = geom(b->dims).C;
      const Window w = window_rows(b, apply_rows(cw));
      int64_t in = 0, all = 0;
      for (int q = 0; q < kQBins; ++q) {
        all += b->qhist[q];
        if (q >= w.q_lo && q < w.q_lo + w.qw) in += b->qhist[q];
      }
      b->bucketed = (double)(all - in) > 1e-3 * (double)all;
    }
  }
  if (b->bucketed) {
    b->n_base = 2 * std::max<int32_t>(1, b->dims.n_rg);  // 2 * read group + mate class
    b->fronts = fronts(b->n_base, b->ctx->n_cu, n, b->ctx->tune_fronts);
    b->n_keys = b->n_base * std::max(1, b->fronts);
    if ((st = dalloc(b->allocs, &b->d_perm, (size_t)std::max<int64_t>(1, n))) != BQSR_OK) return st;
    if ((st = dalloc(b->allocs, &b->d_key_off, (size_t)b->n_keys + 1)) != BQSR_OK) return st;
    if ((st = dalloc(b->allocs, &b->d_key_cnt, (size_t)b->n_keys)) != BQSR_OK) return st;
    if ((st = dalloc(b->allocs, &b->d_cursor, (size_t)b->n_keys)) != BQSR_OK) return st;
  }
  return BQSR_OK;
}

// Per-batch layout of a bucketed batch whose data is on the device (created
// from records or a parse; a staged batch uploads later and keeps the per-job
// sort), built once at creation:
//  * the piece order: the reads sorted by their piece key (the counting sort
//    prep otherwise runs per job), kept (perm_static);
//  * with BQSR_TUNE_KEYMAJOR 1, the key-major copy of the quals and base
//    codes (OrderDev::kslot): the reads' slot spans (written by the sort's
//    scatter) scanned in piece order and each read's 16-aligned slot range
//    copied to its key-major slots.  A piece's reads are then contiguous in
//    the copy: the bucketed chunk walks read it sequentially where the
//    read-order layout scattered them over every key's reads (cfg4: 96 read
//    groups).  1.5 B a slot more HBM.
bool layout_wanted(const bqsr_batch* b) { return b->bucketed && b->rd.slots_aligned && b->rd.n_reads > 0; }
bool key_major_wanted(const bqsr_batch* b) { return layout_wanted(b) && b->ctx->tune_keymajor; }
// the copy's buffers and the scan's scratch, once per batch (freed with it)
bqsr_status key_major_alloc(bqsr_batch* b) {
  if (b->k_qual) return BQSR_OK;
  const int64_t n = b->rd.n_reads;
  bqsr_status st;
  size_t tb = 0;
  HIP_TRY(rocprim::exclusive_scan(nullptr, tb, (const uint64_t*)nullptr, (uint64_t*)nullptr, (uint64_t)0, (size_t)n + 1,
                                  rocprim::plus<uint64_t>(), (hipStream_t)0));
  b->ktemp_bytes = std::max<size_t>(tb, 1);
  if ((st = dalloc(b->allocs, &b->d_kslot, (size_t)(n + 1))) != BQSR_OK ||
      (st = dalloc(b->allocs, &b->d_kspan, (size_t)(n + 1))) != BQSR_OK ||
      (st = dalloc(b->allocs, (uint8_t**)&b->d_ktemp, b->ktemp_bytes)) != BQSR_OK ||
      (st = dalloc(b->allocs, &b->k_qual, (size_t)b->rd.n_slots + kColumnPad)) != BQSR_OK ||
      (st = dalloc(b->allocs, &b->k_bases, (size_t)b->rd.n_slots / 2 + 1 + kColumnPad)) != BQSR_OK)
    return st;
  return BQSR_OK;
}
// the piece-key counting sort (span: each sorted position's slot span as well, or null)
void launch_key_sort(bqsr_batch* b, uint64_t* span, hipStream_t s) {
  const int64_t n = b->rd.n_reads;
  const int n_cu = b->ctx->n_cu;
  (void)hipMemsetAsync(b->d_key_cnt, 0, (size_t)b->n_keys * 4, s);
  const unsigned cb = (unsigned)std::min<int64_t>((n + 255) / 256, (int64_t)n_cu * 4);
  hipLaunchKernelGGL(bqsr_key_count, dim3(cb), dim3(256), 0, s, (const ReadMeta*)b->rd.meta, n, b->n_keys, b->n_base,
                     std::max(1, b->fronts), b->d_key_cnt);
  hipLaunchKernelGGL(bqsr_key_scan, dim3(1), dim3(1024), 0, s, (const uint32_t*)b->d_key_cnt, b->n_keys, b->d_key_off,
                     b->d_cursor);
  const unsigned sb = (unsigned)std::min<int64_t>((n + 4095) / 4096, (int64_t)n_cu * 8);
  hipLaunchKernelGGL(bqsr_key_scatter, dim3(sb), dim3(256), 0, s, (const ReadMeta*)b->rd.meta, n, b->n_keys, b->n_base,
                     std::max(1, b->fronts), b->d_cursor, b->d_perm, span);
}
bqsr_status layout_build(bqsr_batch* b, hipStream_t s) {
  if (!layout_wanted(b)) return BQSR_OK;
  const int64_t n = b->rd.n_reads;
  bqsr_context* ctx = b->ctx;
  const bool km = key_major_wanted(b);
  b->km_ready = false;
  const auto t0 = std::chrono::steady_clock::now();
  bqsr_status st = km ? key_major_alloc(b) : BQSR_OK;
  if (st != BQSR_OK) return st;
  const auto t1 = std::chrono::steady_clock::now();
  if (km) HIP_TRY(hipMemsetAsync(b->d_kspan + n, 0, 8, s));
  launch_key_sort(b, km ? b->d_kspan : nullptr, s);
  HIP_TRY(hipGetLastError());
  if (km) {  // key-major slots: the spans in perm order, scanned; then the copy
    size_t tb = b->ktemp_bytes;
    HIP_TRY(rocprim::exclusive_scan(b->d_ktemp, tb, b->d_kspan, b->d_kslot, (uint64_t)0, (size_t)n + 1,
                                    rocprim::plus<uint64_t>(), s));
    HIP_TRY(hipMemsetAsync(b->k_qual + b->rd.n_slots, 0, kColumnPad, s));
    HIP_TRY(hipMemsetAsync(b->k_bases + b->rd.n_slots / 2, 0, 1 + kColumnPad, s));
    const unsigned gw = (unsigned)std::min<int64_t>((n + 16 * kKmPer - 1) / (16 * kKmPer), (int64_t)ctx->n_cu * 64 / kKmPer);
    hipLaunchKernelGGL(bqsr_km_gather, dim3(gw), dim3(256), 0, s, b->rd, (const uint32_t*)b->d_perm,
                       (const uint64_t*)b->d_kslot, b->k_qual, b->k_bases);
    HIP_TRY(hipGetLastError());
  }
  HIP_TRY(hipStreamSynchronize(s));
  const auto t2 = std::chrono::steady_clock::now();
  b->km_alloc_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
  b->km_build_ms = std::chrono::duration<double, std::milli>(t2 - t1).count();
  b->km_ready = km;
  b->perm_static = true;
  return BQSR_OK;
}

// host pack of one record partition (bqsr_records -> device layout)
struct Packed {
  std::vector<ReadMeta> meta;
  std::vector<ReadAlign> align;
  std::vector<uint8_t> qual, bases, md;
  std::vector<uint32_t> cigar;
  int64_t n_slots = 0, n_bases = 0, max_slot = 0;
  int32_t n_rg = 1, max_len = 1;
  int64_t qhist[256] = {0};
  std::vector<int64_t> rghist;
};

bqsr_status pack(const bqsr_records* R, Packed& P) {
  const int64_t n = R->n_reads;
  P.meta.resize((size_t)n);
  P.align.resize((size_t)n);
  uint64_t slot = 0, md_tot = 0, cig_tot = 0;
  for (int64_t r = 0; r < n; ++r) {
    const uint32_t f = R->flags[r];
    const uint64_t lq = (f & BQSR_F_HAS_QUAL) ? R->qual_offset[r + 1] - R->qual_offset[r] : 0;
    const uint64_t ls = (f & BQSR_F_HAS_SEQ) ? R->seq_offset[r + 1] - R->seq_offset[r] : 0;
    const uint64_t nmd = (f & BQSR_F_HAS_MD) ? R->md_offset[r + 1] - R->md_offset[r] : 0;
    const uint64_t ncig = (f & BQSR_F_HAS_CIGAR) ? R->cigar_offset[r + 1] - R->cigar_offset[r] : 0;
    if (lq > 65535 || ls > 65535 || nmd > 65535 || ncig > 65535)
      return fail(BQSR_ERR_UNSUPPORTED, "read field longer than 65535", r);
    if ((f & BQSR_F_HAS_RG) && (R->rg_id[r] < 0 || R->rg_id[r] > 65535))
      return fail(BQSR_ERR_UNSUPPORTED, "recordGroupId outside [0, 65535]", r);
    ReadMeta& m = P.meta[(size_t)r];
    m.slot = slot;
    m.lq = (uint16_t)lq;
    m.ls = (uint16_t)ls;
    m.flags = (uint16_t)(f & 0x7FFF);
    m.rg = (f & BQSR_F_HAS_RG) ? (uint16_t)R->rg_id[r] : 0;
    ReadAlign& a = P.align[(size_t)r];
    a.start = R->start[r];
    a.cigar_off = (uint32_t)cig_tot;
    a.md_off = (uint32_t)md_tot;
    a.contig = R->contig_id[r];
    a.n_cigar = (uint16_t)ncig;
    a.md_len = (uint16_t)nmd;
    const uint64_t sl = align_slots() ? slot_span(lq, ls) : std::max(lq, ls);  // ReadsDev::slots_aligned
    slot += sl;
    P.max_slot = std::max<int64_t>(P.max_slot, (int64_t)sl);
    md_tot += nmd;
    cig_tot += ncig;
    P.n_bases += (int64_t)(R->seq_offset[r + 1] - R->seq_offset[r]);
    if (f & BQSR_F_HAS_RG) P.n_rg = std::max<int32_t>(P.n_rg, R->rg_id[r] + 1);
    P.max_len = std::max<int32_t>(P.max_len, (int32_t)ls);
  }
  if (md_tot > 0xFFFFFFFFull || cig_tot > 0xFFFFFFFFull)
    return fail(BQSR_ERR_UNSUPPORTED, "partition MD / CIGAR columns exceed 4 GiB");
  P.n_slots = (int64_t)slot;
  // kColumnPad readable bytes past each column's end: the per-base passes load 16 B at a time
  P.qual.assign((size_t)slot + kColumnPad, 0);
  P.bases.assign((size_t)slot / 2 + 1 + kColumnPad, 0);
  P.md.resize(md_tot + kColumnPad);        // the prep kernel loads 32 B of MD at a time
  P.cigar.resize(cig_tot + kColumnPad / 4);  // and 16 B of CIGAR
  P.rghist.assign((size_t)P.n_rg, 0);
  // per-base columns, parallel over read ranges
  const int nth = (int)std::max<int64_t>(1, std::min<int64_t>(16, n / 65536));
  std::vector<std::thread> th;
  std::vector<std::array<int64_t, 256>> qh((size_t)nth);
  for (auto& h : qh) h.fill(0);
  auto work = [&](int t) {
    const int64_t r0 = n * t / nth, r1 = n * (t + 1) / nth;
    for (int64_t r = r0; r < r1; ++r) {
      const ReadMeta& m = P.meta[(size_t)r];
      const ReadAlign& a = P.align[(size_t)r];
      const uint8_t* q = R->qual + R->qual_offset[r];
      for (uint32_t i = 0; i < m.lq; ++i) {
        const uint8_t v = (uint8_t)(q[i] - 33);  // (char - 33).toByte
        P.qual[m.slot + i] = v;
        qh[(size_t)t][v]++;
      }
      const uint8_t* s = R->seq + R->seq_offset[r];
      bool other = false;
      for (uint32_t i = 0; i < m.ls; ++i) {
        const uint8_t c = code_of(s[i]);
        other |= c == kCodeOther;
        const uint64_t k = m.slot + i;
        // two reads can share a byte only at odd boundaries: threads own whole reads,
        // so write nibbles with a CAS-free scheme: even nibble by value, odd by or
        if (k & 1) __atomic_fetch_or(&P.bases[k >> 1], (uint8_t)(c << 4), __ATOMIC_RELAXED);
        else __atomic_fetch_or(&P.bases[k >> 1], c, __ATOMIC_RELAXED);
      }
      if (other) P.meta[(size_t)r].flags |= kSeqOther;
      if (m.flags & BQSR_F_HAS_MD) memcpy(&P.md[a.md_off], R->md + R->md_offset[r], a.md_len);
      if (m.flags & BQSR_F_HAS_CIGAR) memcpy(&P.cigar[a.cigar_off], R->cigar + R->cigar_offset[r], a.n_cigar * 4u);
    }
  };
  for (int t = 0; t < nth; ++t) th.emplace_back(work, t);
  for (auto& x : th) x.join();
  for (auto& h : qh)
    for (int i = 0; i < 256; ++i) P.qhist[i] += h[(size_t)i];
  for (int64_t r = 0; r < n; ++r)
    if (P.meta[(size_t)r].flags & BQSR_F_HAS_RG) P.rghist[P.meta[(size_t)r].rg]++;
  return BQSR_OK;
}

// LDS window start: the 64-wide qual range holding the most bases
int32_t best_q_lo(const int64_t* qhist, int qw) {
  int best = 0;
  int64_t bestv = -1;
  for (int lo = 0; lo + 1 <= kQBins; ++lo) {
    int64_t v = 0;
    for (int q = lo; q < std::min(kQBins, lo + qw); ++q) v += qhist[q];
    if (v > bestv) {
      bestv = v;
      best = lo;
    }
    if (lo + qw >= kQBins) break;
  }
  return best;
}

}  // namespace

bqsr_status bqsr_batch_create(bqsr_context* ctx, const bqsr_records* R, void* stream, bqsr_batch** out) {
  if (!ctx || !R || !out || R->n_reads < 0) return fail(BQSR_ERR_INVALID_ARG, "bqsr_batch_create: bad arguments");
  HIP_TRY(hipSetDevice(ctx->device));
  Packed P;
  bqsr_status st = pack(R, P);
  if (st != BQSR_OK) return st;
  bqsr_batch* b = new bqsr_batch;
  b->ctx = ctx;
  b->owned = true;
  b->rd.n_reads = R->n_reads;
  b->rd.n_slots = P.n_slots;
  b->n_slots = P.n_slots;
  b->n_bases = P.n_bases;
  b->dims = bqsr_dims{P.n_rg, P.max_len};
  // window: most frequent read group, densest qual range (the window width is
  // decided per launch from the table geometry; 40 is a typical width)
  int32_t rg_lo = 0;
  for (int32_t i = 0; i < (int32_t)P.rghist.size(); ++i)
    if (P.rghist[(size_t)i] > P.rghist[(size_t)rg_lo]) rg_lo = i;
  b->rg_lo = rg_lo;
  b->q_lo = best_q_lo(P.qhist, 40);
  b->have_qhist = true;
  for (int q = 0; q < kQBins; ++q) b->qhist[q] = P.qhist[q];
  for (int q = kQBins; q < 256; ++q) b->qhigh += P.qhist[q];
  ReadMeta* meta;
  ReadAlign* align;
  uint8_t *qual, *bases, *md;
  uint32_t* cigar;
  hipStream_t s = S(stream);
  auto up = [&](auto** dst, const auto& v) -> bqsr_status {
    using T = typename std::remove_reference<decltype(v[0])>::type;
    bqsr_status x = dalloc(b->allocs, dst, v.size());
    if (x != BQSR_OK) return x;
    if (!v.empty()) HIP_TRY(hipMemcpyAsync(*dst, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, s));
    return BQSR_OK;
  };
  if ((st = up(&meta, P.meta)) != BQSR_OK || (st = up(&align, P.align)) != BQSR_OK || (st = up(&qual, P.qual)) != BQSR_OK ||
      (st = up(&bases, P.bases)) != BQSR_OK || (st = up(&md, P.md)) != BQSR_OK || (st = up(&cigar, P.cigar)) != BQSR_OK) {
    delete b;
    return st;
  }
  b->rd.meta = meta;
  b->rd.align = align;
  b->rd.qual = qual;
  b->rd.bases = bases;
  b->rd.md = md;
  b->rd.cigar = cigar;
  b->rd.slots_aligned = align_slots();
  if ((st = finish_batch(b, P.max_slot)) != BQSR_OK || (st = layout_build(b, s)) != BQSR_OK) {
    delete b;
    return st;
  }
  hipError_t e = hipStreamSynchronize(s);
  if (e != hipSuccess) {
    delete b;
    return fail(BQSR_ERR_DEVICE, hipGetErrorString(e));
  }
  *out = b;
  return ok();
}

// ---- host-staged partitions: pinned device-layout columns, async upload ----
// The streaming form of bqsr_batch_create (cfg5: partitions streamed from
// the host).  bqsr_stage_records packs a partition once into one pinned
// block; bqsr_batch_create_staged allocates matching device columns;
// bqsr_batch_upload_async enqueues the six H2D copies on a copy stream, so
// the next partition's transfer overlaps the current one's kernels.
// A partition staged for streaming: pinned host columns in the device layout,
// except the base codes, which travel as 2 bits per slot (A C G T) plus an
// exception list (slot << 8 | code) for N / other bytes and are expanded to
// the 4-bit column on the device after the upload (a third of the bytes the
// link would carry for them), and the quals, which travel as 16-slot chunks:
// a base byte and sixteen 4-bit codes (qual - base + 7 for -7 .. +6, 15 for a
// 0 byte -- the slots' padding --, 14 for an exception), plus an exception
// list (slot << 8 | byte) -- 9 bytes a chunk instead of 16 when a chunk's
// quals span at most 14 values, which neighbouring quals of a read mostly do
// (quals_expand on the device).
constexpr int kStagedCols = 11;  // meta | align | qual (device only) | bases (device only) | md | cigar | bases2 |
                                 // base exceptions | qual codes | qual bases | qual exceptions
constexpr uint32_t kQCodeZero = 15u, kQCodeExc = 14u;
// One 16-slot chunk of quals (n <= 16 bytes) -> base byte and codes; exceptions appended.
static void encode_qual_chunk(const uint8_t* q, int n, uint64_t slot0, uint8_t& base, uint64_t& codes,
                              std::vector<uint64_t>& exc) {
  int mn = 256, mx = -1;
  for (int k = 0; k < n; ++k)
    if (q[k]) {
      mn = std::min(mn, (int)q[k]);
      mx = std::max(mx, (int)q[k]);
    }
  int b = mn + 7;  // covers mn .. mn + 13
  if (mx >= 0 && mx - mn > 13) {  // wider: of three windows, the one covering the most quals
    const int cand[3] = {mn, mx - 13, (mn + mx) / 2 - 7};
    int best = -1;
    for (int c : cand) {
      int cnt = 0;
      for (int k = 0; k < n; ++k) cnt += q[k] && q[k] >= c && q[k] <= c + 13;
      if (cnt > best) {
        best = cnt;
        b = c + 7;
      }
    }
  }
  b = std::min(std::max(b, 0), 255);
  uint64_t w = 0;
  for (int k = 0; k < 16; ++k) {
    uint32_t c = kQCodeZero;
    if (k < n && q[k]) {
      const int d = (int)q[k] - b;
      if (d >= -7 && d <= 6) {
        c = (uint32_t)(d + 7);
      } else {
        c = kQCodeExc;
        exc.push_back(((slot0 + (uint64_t)k) << 8) | q[k]);
      }
    }
    w |= (uint64_t)c << (4 * k);
  }
  base = (uint8_t)b;
  codes = w;
}
struct bqsr_staged {
  unsigned char* host = nullptr;  // pinned: the columns, bases excepted
  size_t bytes = 0;
  size_t off[kStagedCols] = {0}, cnt[kStagedCols] = {0};  // byte offset, element count per column
  int64_t n_reads = 0, n_slots = 0, n_bases = 0, max_slot = 0;
  bqsr_dims dims{1, 1};
  int32_t rg_lo = 0, q_lo = 0;
  int64_t qhist[kQBins] = {0};
  int64_t qhigh = 0;
  ~bqsr_staged() {
    if (host) (void)hipHostFree(host);
  }
};

bqsr_status bqsr_stage_records(bqsr_context* ctx, const bqsr_records* R, bqsr_staged** out) {
  if (!ctx || !R || !out || R->n_reads < 0) return fail(BQSR_ERR_INVALID_ARG, "bqsr_stage_records: bad arguments");
  HIP_TRY(hipSetDevice(ctx->device));
  Packed P;
  bqsr_status st = pack(R, P);
  if (st != BQSR_OK) return st;
  if (P.max_slot > kMaxReadLen)
    return fail(BQSR_ERR_UNSUPPORTED, "reads longer than " + std::to_string(kMaxReadLen) + " bases are not supported");
  std::unique_ptr<bqsr_staged> s(new bqsr_staged);
  // base codes: 2 bits a slot (4 slots a byte; N / other as A plus an exception)
  const size_t nb = P.bases.size();
  std::vector<uint8_t> b2((nb + 1) / 2 + 8, 0);
  std::vector<uint64_t> exc;
  for (size_t j = 0; j < nb; ++j) {
    const uint8_t v = P.bases[j];
    for (int h = 0; h < 2; ++h) {
      const uint32_t c = (v >> (4 * h)) & 0xFu;
      const uint64_t slot = 2 * (uint64_t)j + (uint64_t)h;
      if (c >= 4) exc.push_back((slot << 8) | c);
      else b2[slot >> 2] |= (uint8_t)(c << (2 * (slot & 3)));
    }
  }
  // quals: 16-slot chunks (threads over chunk ranges, exception lists joined in slot order)
  const size_t nq = P.qual.size(), n16 = (nq + 15) / 16;
  std::vector<uint64_t> qcodes(std::max<size_t>(n16, 1), 0);
  std::vector<uint8_t> qbase(std::max<size_t>(n16, 1), 0);
  const int nt = (int)std::max<size_t>(1, std::min<size_t>(16, n16 / 65536));
  std::vector<std::vector<uint64_t>> qexc_t((size_t)nt);
  {
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t)
      th.emplace_back([&, t] {
        const size_t c0 = n16 * (size_t)t / (size_t)nt, c1 = n16 * (size_t)(t + 1) / (size_t)nt;
        for (size_t c = c0; c < c1; ++c)
          encode_qual_chunk(P.qual.data() + 16 * c, (int)std::min<size_t>(16, nq - 16 * c), 16 * (uint64_t)c,
                            qbase[c], qcodes[c], qexc_t[(size_t)t]);
      });
    for (auto& x : th) x.join();
  }
  std::vector<uint64_t> qexc;
  for (auto& v : qexc_t) qexc.insert(qexc.end(), v.begin(), v.end());
  const size_t esz[kStagedCols] = {sizeof(ReadMeta), sizeof(ReadAlign), 1, 1, 1, sizeof(uint32_t), 1, 8, 8, 1, 8};
  const size_t cnt[kStagedCols] = {P.meta.size(), P.align.size(), nq,          nb,          P.md.size(), P.cigar.size(),
                                   b2.size(),     exc.size(),     n16,         n16,         qexc.size()};
  const void* src[kStagedCols] = {P.meta.data(), P.align.data(), nullptr,       nullptr,      P.md.data(), P.cigar.data(),
                                  b2.data(),     exc.data(),     qcodes.data(), qbase.data(), qexc.data()};
  size_t tot = 0;
  for (int i = 0; i < kStagedCols; ++i) {
    s->off[i] = tot;
    s->cnt[i] = cnt[i];
    if (src[i]) tot = (tot + cnt[i] * esz[i] + 255) & ~(size_t)255;
  }
  HIP_TRY(hipHostMalloc((void**)&s->host, std::max<size_t>(tot, 1), hipHostMallocDefault));
  s->bytes = tot;
  for (int i = 0; i < kStagedCols; ++i)
    if (cnt[i] && src[i]) memcpy(s->host + s->off[i], src[i], cnt[i] * esz[i]);
  s->n_reads = R->n_reads;
  s->n_slots = P.n_slots;
  s->n_bases = P.n_bases;
  s->max_slot = P.max_slot;
  s->dims = bqsr_dims{P.n_rg, P.max_len};
  for (int32_t i = 0; i < (int32_t)P.rghist.size(); ++i)
    if (P.rghist[(size_t)i] > P.rghist[(size_t)s->rg_lo]) s->rg_lo = i;  // as bqsr_batch_create
  s->q_lo = best_q_lo(P.qhist, 40);
  for (int q = 0; q < kQBins; ++q) s->qhist[q] = P.qhist[q];
  for (int q = kQBins; q < 256; ++q) s->qhigh += P.qhist[q];
  *out = s.release();
  return ok();
}

void bqsr_staged_destroy(bqsr_staged* s) { delete s; }
int64_t bqsr_staged_bytes(const bqsr_staged* s) { return s ? (int64_t)s->bytes : 0; }
int64_t bqsr_staged_reads(const bqsr_staged* s) { return s ? s->n_reads : 0; }
int64_t bqsr_staged_bases(const bqsr_staged* s) { return s ? s->n_bases : 0; }

bqsr_status bqsr_batch_create_staged(bqsr_context* ctx, const bqsr_staged* S_, bqsr_batch** out) {
  if (!ctx || !S_ || !out) return fail(BQSR_ERR_INVALID_ARG, "bqsr_batch_create_staged: bad arguments");
  HIP_TRY(hipSetDevice(ctx->device));
  std::unique_ptr<bqsr_batch> b(new bqsr_batch);
  b->ctx = ctx;
  b->owned = true;
  b->rd.n_reads = S_->n_reads;
  b->rd.n_slots = S_->n_slots;
  b->n_slots = S_->n_slots;
  b->n_bases = S_->n_bases;
  b->dims = S_->dims;
  b->rg_lo = S_->rg_lo;
  b->q_lo = S_->q_lo;
  b->have_qhist = true;
  for (int q = 0; q < kQBins; ++q) b->qhist[q] = S_->qhist[q];
  b->qhigh = S_->qhigh;
  ReadMeta* meta;
  ReadAlign* align;
  uint8_t *qual, *bases, *md;
  uint32_t* cigar;
  bqsr_status st;
  if ((st = dalloc(b->allocs, &meta, S_->cnt[0])) != BQSR_OK || (st = dalloc(b->allocs, &align, S_->cnt[1])) != BQSR_OK ||
      (st = dalloc(b->allocs, &qual, S_->cnt[2])) != BQSR_OK || (st = dalloc(b->allocs, &bases, S_->cnt[3])) != BQSR_OK ||
      (st = dalloc(b->allocs, &md, S_->cnt[4])) != BQSR_OK || (st = dalloc(b->allocs, &cigar, S_->cnt[5])) != BQSR_OK)
    return st;
  b->rd.meta = meta;
  b->rd.align = align;
  b->rd.qual = qual;
  b->rd.bases = bases;
  b->rd.md = md;
  b->rd.cigar = cigar;
  b->rd.slots_aligned = align_slots();
  if ((st = dalloc(b->allocs, &b->d_bases2, S_->cnt[6] + 16)) != BQSR_OK ||
      (st = dalloc(b->allocs, &b->d_bexc, std::max<size_t>(S_->cnt[7], 1))) != BQSR_OK ||
      (st = dalloc(b->allocs, &b->d_qcodes, std::max<size_t>(S_->cnt[8], 1))) != BQSR_OK ||
      (st = dalloc(b->allocs, &b->d_qbase, std::max<size_t>(S_->cnt[9], 1))) != BQSR_OK ||
      (st = dalloc(b->allocs, &b->d_qexc, std::max<size_t>(S_->cnt[10], 1))) != BQSR_OK)
    return st;
  if ((st = finish_batch(b.get(), S_->max_slot)) != BQSR_OK) return st;
  b->staged_cnt.assign(S_->cnt, S_->cnt + kStagedCols);
  b->staged_src = S_;
  *out = b.release();
  return ok();
}

bqsr_status bqsr_batch_upload_async(bqsr_batch* b, const bqsr_staged* S_, void* stream) {
  if (!b || !S_) return fail(BQSR_ERR_INVALID_ARG, "bqsr_batch_upload_async: bad arguments");
  // the batch's launch parameters (quality window, qual histogram, read-group
  // order) were derived from the staged partition it was created from: any
  // other partition, even one of the same shape, is refused
  if (b->staged_src != S_ || b->staged_cnt.size() != kStagedCols ||
      !std::equal(b->staged_cnt.begin(), b->staged_cnt.end(), S_->cnt) || b->rd.n_reads != S_->n_reads)
    return fail(BQSR_ERR_INVALID_ARG, "bqsr_batch_upload_async: batch was not created from this staged partition");
  HIP_TRY(hipSetDevice(b->ctx->device));
  void* dst[kStagedCols] = {(void*)b->rd.meta,  (void*)b->rd.align,  nullptr,           nullptr,
                            (void*)b->rd.md,    (void*)b->rd.cigar,  (void*)b->d_bases2, (void*)b->d_bexc,
                            (void*)b->d_qcodes, (void*)b->d_qbase,   (void*)b->d_qexc};
  const size_t esz[kStagedCols] = {sizeof(ReadMeta), sizeof(ReadAlign), 1, 1, 1, sizeof(uint32_t), 1, 8, 8, 1, 8};
  hipStream_t s = S(stream);
  for (int i = 0; i < kStagedCols; ++i)
    if (S_->cnt[i] && dst[i])
      HIP_TRY(hipMemcpyAsync(dst[i], S_->host + S_->off[i], S_->cnt[i] * esz[i], hipMemcpyHostToDevice, s));
  // the 4-bit base codes back from 2 bits a slot, then the exceptions (on the upload's stream)
  const int64_t nw = (int64_t)(S_->cnt[3] + 7) / 8;  // u64 words of the 4-bit column
  const unsigned g = (unsigned)std::min<int64_t>(std::max<int64_t>(1, (nw + 255) / 256), (int64_t)b->ctx->n_cu * 16);
  hipLaunchKernelGGL(bqsr_bases_expand, dim3(g), dim3(256), 0, s, (const uint32_t*)b->d_bases2, (int64_t)S_->cnt[3],
                     (uint8_t*)b->rd.bases);
  if (S_->cnt[7]) {
    const unsigned ge = (unsigned)std::min<int64_t>(((int64_t)S_->cnt[7] + 255) / 256, (int64_t)b->ctx->n_cu * 16);
    hipLaunchKernelGGL(bqsr_bases_exceptions, dim3(ge), dim3(256), 0, s, (const uint64_t*)b->d_bexc,
                       (int64_t)S_->cnt[7], (uint8_t*)b->rd.bases);
  }
  // the quals from their 16-slot chunks, then their exceptions
  const int64_t n16 = (int64_t)S_->cnt[8];
  if (n16) {
    const unsigned gq = (unsigned)std::min<int64_t>((n16 + 255) / 256, (int64_t)b->ctx->n_cu * 16);
    hipLaunchKernelGGL(bqsr_quals_expand, dim3(gq), dim3(256), 0, s, (const uint64_t*)b->d_qcodes,
                       (const uint8_t*)b->d_qbase, n16, (int64_t)S_->cnt[2], (uint8_t*)b->rd.qual);
  }
  if (S_->cnt[10]) {
    const unsigned ge = (unsigned)std::min<int64_t>(((int64_t)S_->cnt[10] + 255) / 256, (int64_t)b->ctx->n_cu * 16);
    hipLaunchKernelGGL(bqsr_quals_exceptions, dim3(ge), dim3(256), 0, s, (const uint64_t*)b->d_qexc,
                       (int64_t)S_->cnt[10], (uint8_t*)b->rd.qual);
  }
  HIP_TRY(hipGetLastError());
  b->prepped = false;  // new contents: the next observe / apply re-runs prep
  return ok();
}

bqsr_status bqsr_batch_wrap_device(bqsr_context* ctx, const bqsr_device_reads* dev, bqsr_batch** out) {
  if (!ctx || !dev || !out || dev->n_reads < 0 || dev->dims.n_rg < 1 || dev->dims.max_len < 1)
    return fail(BQSR_ERR_INVALID_ARG, "bqsr_batch_wrap_device: bad arguments");
  if (dev->dims.max_len > kMaxReadLen)
    return fail(BQSR_ERR_UNSUPPORTED, "reads longer than " + std::to_string(kMaxReadLen) + " bases are not supported");
  HIP_TRY(hipSetDevice(ctx->device));
  bqsr_batch* b = new bqsr_batch;
  b->ctx = ctx;
  b->rd.n_reads = dev->n_reads;
  b->rd.meta = (const ReadMeta*)dev->meta;
  b->rd.align = (const ReadAlign*)dev->align;
  b->rd.qual = dev->qual;
  b->rd.bases = dev->bases;
  b->rd.cigar = dev->cigar;
  b->rd.md = dev->md;
  b->n_slots = dev->n_slots;
  b->rd.n_slots = dev->n_slots;
  b->n_bases = -1;
  b->dims = dev->dims;
  b->q_lo = 0;
  b->rg_lo = 0;
  b->rd.slots_aligned = dev->slots_aligned != 0;
  bqsr_status st = finish_batch(b, b->rd.slots_aligned ? (int64_t)slot_span(0, (uint64_t)dev->dims.max_len)
                                                       : (int64_t)dev->dims.max_len);
  if (st != BQSR_OK) {
    delete b;
    return st;
  }
  *out = b;
  return ok();
}

void bqsr_batch_destroy(bqsr_batch* b) { delete b; }
int64_t bqsr_batch_reads(const bqsr_batch* b) { return b ? b->rd.n_reads : -1; }
int64_t bqsr_batch_bases(const bqsr_batch* b) { return b ? b->n_bases : -1; }
int64_t bqsr_batch_slots(const bqsr_batch* b) { return b ? b->n_slots : -1; }
bqsr_dims bqsr_batch_dims(const bqsr_batch* b) { return b ? b->dims : bqsr_dims{0, 0}; }

// the per-batch layout work a bucketed batch pays once at creation (the
// piece-key counting sort and the key-major copy, layout_build), done
// again: its wall time is what bench.py reports as layout_ms
bqsr_status bqsr_batch_relayout(bqsr_batch* b, void* stream, double* ms) {
  if (!b) return fail(BQSR_ERR_INVALID_ARG, "bqsr_batch_relayout: null batch");
  hipStream_t s = (hipStream_t)stream;
  HIP_TRY(hipStreamSynchronize(s));
  const auto t0 = std::chrono::steady_clock::now();
  const bool has = b->perm_static;
  if (has) {  // the sort (and the copy) again into the batch's buffers (allocated with it)
    b->perm_static = false;
    bqsr_status st = layout_build(b, s);
    if (st != BQSR_OK) return st;
  }
  HIP_TRY(hipStreamSynchronize(s));
  if (ms) *ms = has ? std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() : -1.0;
  return ok();
}

// the key-major copy's cost when the batch was created: allocation and kernels (wall, each synchronised)
bqsr_status bqsr_batch_layout_times(const bqsr_batch* b, double* alloc_ms, double* build_ms) {
  if (!b) return fail(BQSR_ERR_INVALID_ARG, "bqsr_batch_layout_times: null batch");
  if (alloc_ms) *alloc_ms = b->km_alloc_ms;
  if (build_ms) *build_ms = b->km_build_ms;
  return ok();
}

// window override (exported for device batches whose quals the host never saw)
bqsr_status bqsr_batch_set_window(bqsr_batch* b, int32_t q_lo, int32_t rg_lo) {
  if (!b || q_lo < 0 || q_lo >= kQBins || rg_lo < 0) return fail(BQSR_ERR_INVALID_ARG, "bad window");
  b->q_lo = q_lo;
  b->rg_lo = rg_lo;
  b->have_qhist = false;
  return ok();
}
int32_t bqsr_batch_reads_per_tile(const bqsr_batch* b) { return b ? b->rd.reads_per_tile : -1; }

// ---------------------------------------------------------------- table ----

int64_t bqsr_table_words(bqsr_dims d) { return (d.n_rg < 1 || d.max_len < 1) ? -1 : table_words(d); }

bqsr_status bqsr_table_create(bqsr_context* ctx, bqsr_dims d, void* device_words, bqsr_table** out) {
  if (!ctx || !out || d.n_rg < 1 || d.max_len < 1 || d.max_len > 65535)
    return fail(BQSR_ERR_INVALID_ARG, "bqsr_table_create: bad arguments");
  HIP_TRY(hipSetDevice(ctx->device));
  bqsr_table* t = new bqsr_table;
  t->ctx = ctx;
  t->dims = d;
  const size_t bytes = (size_t)table_words(d) * 8;
  if (device_words) {
    t->words = (int64_t*)device_words;
  } else {
    hipError_t e = hipMalloc((void**)&t->words, bytes);
    if (e != hipSuccess) {
      delete t;
      return fail(BQSR_ERR_DEVICE, hipGetErrorString(e));
    }
    t->owned = true;
  }
  hipError_t e = hipMemset(t->words, 0, bytes);
  if (e != hipSuccess) {
    delete t;
    return fail(BQSR_ERR_DEVICE, hipGetErrorString(e));
  }
  *out = t;
  return ok();
}
void bqsr_table_destroy(bqsr_table* t) { delete t; }
bqsr_dims bqsr_table_dims(const bqsr_table* t) { return t ? t->dims : bqsr_dims{0, 0}; }
void* bqsr_table_device_ptr(bqsr_table* t) { return t ? t->words : nullptr; }

bqsr_status bqsr_table_download(const bqsr_table* t, int64_t* host) {
  if (!t || !host) return fail(BQSR_ERR_INVALID_ARG, "null");
  HIP_TRY(hipSetDevice(t->ctx->device));
  HIP_TRY(hipMemcpy(host, t->words, (size_t)table_words(t->dims) * 8, hipMemcpyDeviceToHost));
  return ok();
}
bqsr_status bqsr_table_upload(bqsr_table* t, const int64_t* host) {
  if (!t || !host) return fail(BQSR_ERR_INVALID_ARG, "null");
  HIP_TRY(hipSetDevice(t->ctx->device));
  HIP_TRY(hipMemcpy(t->words, host, (size_t)table_words(t->dims) * 8, hipMemcpyHostToDevice));
  return ok();
}

bqsr_status bqsr_table_merge(bqsr_table* acc, const bqsr_table* part, double* acc_em, double part_em) {
  if (!acc || !part || !acc_em) return fail(BQSR_ERR_INVALID_ARG, "null");
  if (acc->dims.n_rg != part->dims.n_rg || acc->dims.max_len != part->dims.max_len)
    return fail(BQSR_ERR_INVALID_ARG, "table dims differ");
  HIP_TRY(hipSetDevice(acc->ctx->device));
  const int64_t n = table_words(acc->dims);
  hipLaunchKernelGGL(bqsr_table_add, dim3((unsigned)std::min<int64_t>(4096, (n + 255) / 256)), dim3(256), 0,
                     hipStreamPerThread, acc->words, part->words, n);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(hipStreamPerThread));
  *acc_em = *acc_em + part_em;  // RecalTable.++: this.expectedMismatch + other.expectedMismatch
  return ok();
}

// -------------------------------------------------------------- observe ----

namespace {
// window rows (q_lo, qw) for at most max_rows rows: the batch's whole qual
// span when it fits, else the densest max_rows-wide range; without a
// histogram the caller's choice (bqsr_batch_set_window)
Window window_rows(const bqsr_batch* b, int max_rows) {
  Window w{max_rows, std::min(b->q_lo, kQBins - 1), b->rg_lo};
  if (!b->have_qhist) {
    w.qw = std::min(w.qw, kQBins - w.q_lo);
    return w;
  }
  int lo = 0, hi = kQBins - 1;
  while (lo < kQBins - 1 && b->qhist[lo] == 0) ++lo;
  while (hi > lo && b->qhist[hi] == 0) --hi;
  if (hi - lo + 1 <= max_rows) {
    w.q_lo = lo;
    w.qw = hi - lo + 1;
  } else {
    w.q_lo = best_q_lo(b->qhist, max_rows);
  }
  w.qw = std::min(w.qw, kQBins - w.q_lo);  // rows stay below qual 128 (Java byte >= 0)
  return w;
}
// cycle cells of the windows: all of them in read order, one mate class's
// half when bucketed (OrderDev, WinGeom)
int window_cw(const bqsr_batch* b, const TableGeom& g) { return b->bucketed ? g.L : g.C; }
// rows the batch's quals span (all 128 without a histogram)
int qual_span(const bqsr_batch* b) {
  if (!b->have_qhist) return kQBins;
  int lo = 0, hi = kQBins - 1;
  while (lo < kQBins - 1 && b->qhist[lo] == 0) ++lo;
  while (hi > lo && b->qhist[hi] == 0) --hi;
  return hi - lo + 1;
}
int lane_shift(const bqsr_batch* b) {
  const int c = (b->dims.max_len + kSuper - 1) / kSuper;
  int s = 0;
  while ((1 << s) < c && s < 6) ++s;
  return s;
}
bqsr_status check_dims(const bqsr_batch* b, const bqsr_table* t) {
  if (b->dims.n_rg > t->dims.n_rg || b->dims.max_len > t->dims.max_len)
    return fail(BQSR_ERR_INVALID_ARG, "table dims smaller than the batch's (n_rg / max_len)");
  return BQSR_OK;
}
}  // namespace

// Stages of observe, launched on `stream` without synchronising (results land
// in the batch's error words / expectedMismatch slot):
//   BQSR_STAGE_RESET   clear the observe error word
//   BQSR_STAGE_PREP    the per-read prep kernel (also validates for apply)
//   BQSR_STAGE_KERNEL  the observe kernel (counts into `t`)
//   BQSR_STAGE_FOLD    the expectedMismatch fold kernel
// Exposed separately so a caller can bracket one kernel with HIP events.
namespace {
bqsr_status launch_prep(bqsr_context* ctx, bqsr_batch* b, const bqsr_sites* sites, hipStream_t s) {
  if (!b->err_fresh) HIP_TRY(hipMemsetAsync(b->d_err + kErrAppPrep, 0xFF, 8, s));  // (else the job reset did)
  b->err_fresh = false;
  // a new prep: the fold's qual mask belongs to the previous job until this
  // job's fold rewrites it (wrapped device columns may have changed since)
  b->hq_valid = false;
  if (b->rd.n_reads > 0) {
    PrepParams P{};
    P.rd = b->rd;
    if (sites) P.sites = sites->dev();
    // with known sites and reads of <= 128 bases, pass 1 stores every bitmap
    // word (no zeroing pass, no read-modify-write atomics: cfg3 prep 3.0 ->
    // 2.2 ms); without sites the few mismatch bits as atomics onto a zeroed
    // bitmap cost less (cfg2: 0.25 + 0.03 ms against 0.30)
    P.store_words = b->dims.max_len <= 128 && P.sites.n_contigs > 0;
    P.bnd = b->d_bnd;
    // (the atomic form's workgroups clear their own slots' words first: no fill)
    P.info = b->d_info;
    P.sbits = b->d_sbits;
    P.err = b->d_err;
    P.work = b->d_work;
    P.n_work = b->d_work + b->rd.n_reads + kPrepChunk;
    // pass 1: the common reads in lock step; the rest, one thread each (in
    // pass 1's workgroups, or pass 2 after word stores)
    const int64_t blocks = (b->rd.n_reads + kPrepChunk - 1) / kPrepChunk;
    if (P.store_words) {
      hipLaunchKernelGGL(bqsr_prep_kernel<true>, dim3((unsigned)blocks), dim3(kPrepThreads), 0, s, P);
      hipLaunchKernelGGL(bqsr_prep_complex, dim3((unsigned)blocks), dim3(kComplexThreads), 0, s, P);
    } else {  // the listed reads finished by the same workgroups
      hipLaunchKernelGGL(bqsr_prep_kernel<false>, dim3((unsigned)blocks), dim3(kPrepThreads), 0, s, P);
    }
    HIP_TRY(hipGetLastError());
    if (b->bucketed && !b->perm_static) {  // counting sort of the reads by read group
      launch_key_sort(b, nullptr, s);
      HIP_TRY(hipGetLastError());
    }
  }
  b->prepped = true;
  b->prep_sites = sites;
  return BQSR_OK;
}
}  // namespace

bqsr_status bqsr_observe_stage(bqsr_context* ctx, bqsr_batch* b, const bqsr_sites* sites, bqsr_table* t,
                               int32_t stages, void* stream) {
  if (!ctx || !b || !t) return fail(BQSR_ERR_INVALID_ARG, "null");
  bqsr_status st = check_dims(b, t);
  if (st != BQSR_OK) return st;
  HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = S(stream);
  if (stages & BQSR_STAGE_RESET) HIP_TRY(hipMemsetAsync(b->d_err + kErrObs, 0xFF, 8, s));
  if (stages & BQSR_STAGE_PREP) {
    if ((st = launch_prep(ctx, b, sites, s)) != BQSR_OK) return st;
  }
  if (b->rd.n_reads == 0) {
    if (stages & BQSR_STAGE_FOLD) HIP_TRY(hipMemsetAsync(b->d_em, 0, 8, s));
    return ok();
  }
  if ((stages & BQSR_STAGE_KERNEL) && (!b->prepped || b->prep_sites != sites))
    return fail(BQSR_ERR_INVALID_ARG, "observe kernel before the prep stage (or with other known sites)");
  if (stages & BQSR_STAGE_KERNEL) {
    ObserveParams P{};
    P.rd = b->pass_rd();
    P.ord = b->order();
    P.info = b->d_info;
    P.sbits = b->d_sbits;
    P.g = geom(t->dims);
    // window row length padded to 2 mod 4 words: the lanes of a wavefront add
    // to one cycle cell of many rows at once, which a row length sharing a
    // factor 4 or more with the 32 banks folds onto few banks (cfg3, 224
    // words: 7.6 ms observe; 225: 5.8; cfg2 222 against 223 / 224: 0.94 /
    // 1.00 / 1.25 ms).  Pad words stay 0.
    // Read order: the lean lane per read (bqsr_observe_lean.hip); bucketed
    // batches: the lane-per-chunk walk (cfg4 observe 4.51 ms against the lean
    // form's 6.42, profiles/r03w_cfg4_lean_bucketed_ab.txt).  Measured and
    // removed (round 3, in git history): the round-2 lane per read, lanes per
    // super-chunk and the lane-per-offset rows kernel (SALU-bound, 6.0 ms cfg2).
    const bool lean = !b->bucketed;
    P.wcells = window_cw(b, P.g) + (lean ? kCtxCells : kCtxSlots);
    while ((P.wcells & 3) != 2) ++P.wcells;  // (chunk walk, cfg4: 0 mod 4 5.72 ms, 1 mod 4 4.32, 2 mod 4 4.34)
    if (lean) {
      const int cw = window_cw(b, P.g), span = qual_span(b);
      int best_rows = 0;
      for (int nc = kLeanCopiesMax; nc >= 1 && best_rows < span; --nc) {
        const int orow = lean_orow(nc, cw);
        int qw = kQBins;
        while (qw > 1 && lean_lds(qw, orow, P.wcells) > kLdsMax) --qw;
        if (qw > best_rows) {
          best_rows = qw;
          P.nc = nc;
          P.orow = orow;
        }
      }
      P.w = window_rows(b, best_rows);
      // every qual of the batch a window row: the kernel skips the per-chunk row test
      P.rows_all = b->have_qhist && b->qhigh == 0;
      for (int q = 0; q < kQBins && P.rows_all; ++q)
        if (b->qhist[q] && (q < P.w.q_lo || q >= P.w.q_lo + P.w.qw)) P.rows_all = 0;
    } else {
      P.w = window_rows(b, observe_rows(P.wcells, true));
    }
    P.touched = t->touched();
    P.obs = t->obs();
    P.mm = t->mm();
    P.part_stride = 2 * P.w.qw * P.wcells + P.w.qw;
    // bucketed: bqsr_fold_hist makes the fold's histograms from prep's trims,
    // so the fold runs beside the observe kernel (cfg4: 1.4 ms of fold_hist
    // and 0.8 ms of fold hidden, the observe kernel 1.6 ms slower beside
    // them).  In read order the histograms are the observe kernel's, and a
    // fork after it would only hide bqsr_window_reduce (17 us on cfg2) at
    // the price of two event records (~15 us each on this runtime)
    if (!lean) {
      if (!b->side) {
        HIP_TRY(hipStreamCreateWithFlags(&b->side, hipStreamNonBlocking));
        HIP_TRY(hipEventCreateWithFlags(&b->ev_obs, hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&b->ev_fold, hipEventDisableTiming));
      }
      HIP_TRY(hipEventRecord(b->ev_obs, s));
      b->obs_pending = true;
    }
    // slabs w + key
    const size_t need = (size_t)P.part_stride * (b->pass_blocks() + b->n_keys - 1);
    if (b->part_words < need) {  // grows with the table geometry; kept across calls
      if (b->d_part) {
        HIP_TRY(hipStreamSynchronize(s));
        (void)hipFree(b->d_part);
        b->d_part = nullptr;
        b->part_words = 0;
      }
      HIP_TRY(hipMalloc((void**)&b->d_part, need * sizeof(uint32_t)));
      b->part_words = need;
    }
    P.part = b->d_part;
    P.hq_block = b->d_hq;
    P.err = b->d_err + kErrObs;
    P.n_blocks = lean ? b->n_blocks : b->pass_blocks();  // (fronts: a chunk-walk workgroup per piece)
    const size_t lds = lean ? lean_lds(P.w.qw, P.orow, P.wcells) : observe_lds(P.w.qw, P.wcells, true);
    if (lean) {
      hipLaunchKernelGGL((bqsr_observe_lean<true>), dim3(P.n_blocks), dim3(kBlockThreads), lds, s, P);
    } else {
      hipLaunchKernelGGL(bqsr_observe_chunks, dim3(P.n_blocks), dim3(kBlockThreads), lds, s, P);
    }
    HIP_TRY(hipGetLastError());
    const int rb = (int)std::min<int64_t>(4096, ((int64_t)P.part_stride * (b->bucketed ? b->n_base : 1) + 255) / 256);
    const unsigned ry = b->bucketed ? 1u : (unsigned)((b->n_blocks + kRedSlabs - 1) / kRedSlabs);
    hipLaunchKernelGGL(bqsr_window_reduce, dim3(rb, ry), dim3(256), 0, s, (const uint32_t*)b->d_part, b->rd, P.ord,
                       P.n_blocks, P.part_stride, P.wcells, P.w, P.g, P.touched, P.obs, P.mm, lean ? kCtxJunk : 0);
    HIP_TRY(hipGetLastError());
  }
  if (stages & BQSR_STAGE_FOLD) {
    // bucketed: on the side stream after prep, concurrent with the observe
    // kernel and bqsr_window_reduce (the fold reads the quals in read order
    // and resolves deferred trims itself, resolve_info, as observe does; the
    // observe kernel writes the same trims back) -- the caller's stream
    // waits at the end
    const hipStream_t caller = s;
    const bool fork = b->obs_pending;
    if (fork) {
      HIP_TRY(hipStreamWaitEvent(b->side, b->ev_obs, 0));
      s = b->side;
      b->obs_pending = false;
    }
    if (b->bucketed) {  // the observe kernel did not walk the fold's blocks in read order: their histograms
      HIP_TRY(hipMemsetAsync(b->d_hq, 0, (size_t)b->n_blocks * kQBins * 4, s));
      hipLaunchKernelGGL(bqsr_fold_hist, dim3(b->n_blocks * kFhSplit), dim3(kFhWaves * 64), fold_hist_lds(), s, b->rd, (const ReadInfo*)b->d_info,
                         b->n_blocks, lane_shift(b), b->d_hq);
      HIP_TRY(hipGetLastError());
    }
    FoldParams F = b->fold;
    F.rd = b->rd;
    F.info = b->d_info;
    F.hq_block = b->d_hq;
    F.pow10 = ctx->d_pow10;
    F.n_blocks = b->n_blocks;
    F.em_out = b->d_em;
    F.qmask = b->d_qmask;
    hipLaunchKernelGGL(bqsr_fold_plan, dim3(1), dim3(1024), 0, s, F);
    const int64_t max_tpb = (b->rd.n_tiles + b->n_blocks - 1) / b->n_blocks + 1;
    hipLaunchKernelGGL(bqsr_fold_tiles, dim3(ctx->n_cu * 4), dim3(kFtWaves * 64), 0, s, F, max_tpb);
    hipLaunchKernelGGL(bqsr_fold_segs, dim3(b->n_blocks), dim3(kSegThreads), 0, s, F);
    hipLaunchKernelGGL(bqsr_fold_chain, dim3(1), dim3(1024), chain_lds(b->n_blocks), s, F);
    HIP_TRY(hipGetLastError());
    b->hq_valid = true;
    if (fork) {
      HIP_TRY(hipEventRecord(b->ev_fold, s));
      HIP_TRY(hipStreamWaitEvent(caller, b->ev_fold, 0));
    }
  }
  return ok();
}

// launch observe + fold; does not synchronise
bqsr_status bqsr_observe_async(bqsr_context* ctx, bqsr_batch* b, const bqsr_sites* sites, bqsr_table* t, void* stream) {
  return bqsr_observe_stage(ctx, b, sites, t, BQSR_STAGE_RESET | BQSR_STAGE_PREP | BQSR_STAGE_KERNEL | BQSR_STAGE_FOLD,
                            stream);
}

// zero a table on a stream (a fresh `new RecalTable` for the next job)
bqsr_status bqsr_table_zero_async(bqsr_table* t, void* stream) {
  if (!t) return fail(BQSR_ERR_INVALID_ARG, "null");
  HIP_TRY(hipSetDevice(t->ctx->device));
  HIP_TRY(hipMemsetAsync(t->words, 0, (size_t)table_words(t->dims) * 8, S(stream)));
  return ok();
}

// device pointer of the batch's expectedMismatch result (one double)
void* bqsr_batch_em_device_ptr(bqsr_batch* b) { return b ? (void*)b->d_em : nullptr; }

bqsr_status bqsr_observe_result(bqsr_batch* b, double* em, void* stream) {
  HIP_TRY(hipSetDevice(b->ctx->device));
  hipStream_t s = S(stream);
  unsigned long long err = 0;
  double e = 0;
  HIP_TRY(hipMemcpyAsync(&err, b->d_err + kErrObs, 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(&e, b->d_em, 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (em) *em = e;
  return from_err_key(err, 0);
}

bqsr_status bqsr_observe(bqsr_context* ctx, bqsr_batch* b, const bqsr_sites* sites, bqsr_table* t,
                         double* expected_mismatch, void* stream) {
  bqsr_status st = bqsr_observe_async(ctx, b, sites, t, stream);
  if (st != BQSR_OK) return st;
  return bqsr_observe_result(b, expected_mismatch, stream);
}

bqsr_status bqsr_observe_records(bqsr_context* ctx, const bqsr_records* recs, const bqsr_sites* sites, bqsr_dims dims,
                                 bqsr_table** out_partial, double* out_em) {
  if (!out_partial || !out_em) return fail(BQSR_ERR_INVALID_ARG, "null out");
  bqsr_batch* b = nullptr;
  bqsr_status st = bqsr_batch_create(ctx, recs, nullptr, &b);
  if (st != BQSR_OK) return st;
  bqsr_table* t = nullptr;
  st = bqsr_table_create(ctx, dims, nullptr, &t);
  if (st == BQSR_OK) st = bqsr_observe(ctx, b, sites, t, out_em, nullptr);
  bqsr_batch_destroy(b);
  if (st != BQSR_OK) {
    bqsr_table_destroy(t);
    return st;
  }
  *out_partial = t;
  return ok();
}

// ------------------------------------------------------------- finalize ----

namespace {
bqsr_status finalize_impl(bqsr_context* ctx, const bqsr_table* t, double em, const double* em_dev, bqsr_lut** out,
                          void* stream) {
  if (!ctx || !t || !out) return fail(BQSR_ERR_INVALID_ARG, "null");
  HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = S(stream);
  const TableGeom g = geom(t->dims);
  const int n_rg = t->dims.n_rg;
  // *out is NULL or a LUT from an earlier finalize: one of the same dims and
  // context is reused (no allocation); any other is destroyed and replaced
  bqsr_lut* L = *out;
  const bool reuse = L && L->ctx == ctx && L->dims.n_rg == t->dims.n_rg && L->dims.max_len == t->dims.max_len;
  if (L && !reuse) {
    (void)hipStreamSynchronize(s);  // its buffers may still be read by queued work
    delete L;
    *out = nullptr;
  }
  if (!reuse) L = new bqsr_lut;
  L->ctx = ctx;
  L->dims = t->dims;
  L->src = t;
  L->host_ready = false;
  L->n_groups = (g.K - 1) / kMaxQ + 2;
  bqsr_status st;
  if (!reuse && ((st = dalloc(L->allocs, &L->qk_obs, g.K)) != BQSR_OK || (st = dalloc(L->allocs, &L->qk_mm, g.K)) != BQSR_OK ||
      (st = dalloc(L->allocs, &L->grp_obs, L->n_groups)) != BQSR_OK ||
      (st = dalloc(L->allocs, &L->grp_mm, L->n_groups)) != BQSR_OK ||
      (st = dalloc(L->allocs, &L->grp_ok, L->n_groups)) != BQSR_OK || (st = dalloc(L->allocs, &L->key_ok, g.K)) != BQSR_OK ||
      (st = dalloc(L->allocs, &L->rq_ok, (size_t)n_rg * kQBins)) != BQSR_OK ||
      (st = dalloc(L->allocs, &L->a2, (size_t)n_rg * kQBins)) != BQSR_OK ||
      (st = dalloc(L->allocs, &L->s1, (size_t)n_rg * kQBins * g.C)) != BQSR_OK ||
      (st = dalloc(L->allocs, &L->d2, (size_t)n_rg * kQBins * kCtxSlots)) != BQSR_OK ||
      (st = dalloc(L->allocs, &L->d_out, 1)) != BQSR_OK)) {
    delete L;
    return st;
  }
  hipLaunchKernelGGL(bqsr_final_keys, dim3((g.K + 3) / 4), dim3(256), 0, s, t->touched(), t->obs(), t->mm(), g, L->qk_obs,
                     L->qk_mm);
  hipLaunchKernelGGL(bqsr_final_groups, dim3(1), dim3(256), 0, s, t->touched(), L->qk_obs, L->qk_mm, g, n_rg, em,
                     em_dev, ctx->d_pow10, L->n_groups, L->grp_obs, L->grp_mm, L->grp_ok, L->key_ok, L->a2, L->rq_ok, L->d_out);
  const int64_t ncell = (int64_t)n_rg * kQBins * (g.C + kCtxSlots);
  hipLaunchKernelGGL(bqsr_final_tables, dim3((unsigned)std::min<int64_t>(8192, (ncell + 255) / 256)), dim3(256), 0, s,
                     t->obs(), t->mm(), g, n_rg, L->a2, L->rq_ok, pow10tab().v[kMaxQ], L->s1, L->d2);
  hipError_t e = hipGetLastError();
  // the device path (em in HBM) leaves `out` on the device: bqsr_job_result
  // fetches it with the job's other status words in one transfer
  L->out_pending = em_dev != nullptr;
  if (e == hipSuccess && !em_dev) e = hipMemcpyAsync(&L->out, L->d_out, sizeof(FinalOut), hipMemcpyDeviceToHost, s);
  if (e != hipSuccess) {
    if (!reuse) delete L;
    return fail(BQSR_ERR_DEVICE, hipGetErrorString(e));
  }
  *out = L;
  return ok();
}
}  // namespace

bqsr_status bqsr_finalize_async(bqsr_context* ctx, const bqsr_table* t, double em, bqsr_lut** out, void* stream) {
  return finalize_impl(ctx, t, em, nullptr, out, stream);
}

bqsr_status bqsr_finalize_device(bqsr_context* ctx, const bqsr_table* t, const double* em_device, bqsr_lut** out,
                                 void* stream) {
  if (!em_device) return fail(BQSR_ERR_INVALID_ARG, "null em_device");
  return finalize_impl(ctx, t, 0.0, em_device, out, stream);
}

bqsr_status bqsr_em_fold_async(bqsr_context* ctx, const double* ems, int64_t n, double* out, void* stream) {
  if (!ctx || !out || n < 0 || (n > 0 && !ems)) return fail(BQSR_ERR_INVALID_ARG, "bqsr_em_fold_async: bad arguments");
  HIP_TRY(hipSetDevice(ctx->device));
  hipLaunchKernelGGL(bqsr_em_fold, dim3(1), dim3(64), 0, S(stream), ems, n, out);
  HIP_TRY(hipGetLastError());
  return ok();
}

bqsr_status bqsr_batch_em_copy_async(bqsr_batch* b, double* dst, void* stream) {
  if (!b || !dst) return fail(BQSR_ERR_INVALID_ARG, "null");
  HIP_TRY(hipSetDevice(b->ctx->device));
  HIP_TRY(hipMemcpyAsync(dst, b->d_em, sizeof(double), hipMemcpyDeviceToDevice, S(stream)));
  return ok();
}

bqsr_status bqsr_finalize_result(bqsr_lut* L, void* stream) {
  HIP_TRY(hipSetDevice(L->ctx->device));
  HIP_TRY(hipStreamSynchronize(S(stream)));
  if (L->out_pending) {
    HIP_TRY(hipMemcpy(&L->out, L->d_out, sizeof(FinalOut), hipMemcpyDeviceToHost));
    L->out_pending = false;
  }
  if (!L->out.any_key)  // readGroupCounts.values.reduce on an empty map (RecalTable.scala:123)
    return fail(BQSR_ERR_EMPTY_TABLE, "empty.reduceLeft: no usable base was observed");
  return ok();
}

bqsr_status bqsr_finalize(bqsr_context* ctx, const bqsr_table* t, double em, bqsr_lut** out) {
  if (!out) return fail(BQSR_ERR_INVALID_ARG, "null out");
  bqsr_lut* L = nullptr;
  bqsr_status st = bqsr_finalize_async(ctx, t, em, &L, nullptr);
  if (st != BQSR_OK) return st;
  st = bqsr_finalize_result(L, nullptr);
  if (st != BQSR_OK) {
    delete L;
    return st;
  }
  *out = L;
  return ok();
}

void bqsr_lut_destroy(bqsr_lut* l) { delete l; }

namespace {
bqsr_status lut_host(bqsr_lut* L) {
  if (L->host_ready) return BQSR_OK;
  HIP_TRY(hipSetDevice(L->ctx->device));
  if (L->out_pending) {
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(&L->out, L->d_out, sizeof(FinalOut), hipMemcpyDeviceToHost));
    L->out_pending = false;
  }
  const TableGeom g = geom(L->dims);
  L->h_words.resize((size_t)table_words(L->dims));
  L->h_qk_obs.resize((size_t)g.K);
  L->h_qk_mm.resize((size_t)g.K);
  L->h_grp_obs.resize((size_t)L->n_groups);
  L->h_grp_mm.resize((size_t)L->n_groups);
  L->h_grp_ok.resize((size_t)L->n_groups);
  HIP_TRY(hipMemcpy(L->h_words.data(), L->src->words, L->h_words.size() * 8, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(L->h_qk_obs.data(), L->qk_obs, (size_t)g.K * 8, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(L->h_qk_mm.data(), L->qk_mm, (size_t)g.K * 8, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(L->h_grp_obs.data(), L->grp_obs, (size_t)L->n_groups * 8, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(L->h_grp_mm.data(), L->grp_mm, (size_t)L->n_groups * 8, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(L->h_grp_ok.data(), L->grp_ok, (size_t)L->n_groups, hipMemcpyDeviceToHost));
  L->host_ready = true;
  return BQSR_OK;
}
bool eprob(int64_t obs, int64_t mm, double* v) {
  if (obs == 0) return false;
  const double x = (double)mm / (double)obs;
  *v = std::max(pow10tab().v[kMaxQ], x);
  return true;
}
}  // namespace

bqsr_status bqsr_lut_stats(const bqsr_lut* lc, bqsr_final_stats* out) {
  bqsr_lut* L = const_cast<bqsr_lut*>(lc);
  if (!L || !out) return fail(BQSR_ERR_INVALID_ARG, "null");
  if (L->out_pending) {
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(&L->out, L->d_out, sizeof(FinalOut), hipMemcpyDeviceToHost));
    L->out_pending = false;
  }
  out->average_reported_error = L->out.avg;
  out->global_error = L->out.global_error;
  out->global_obs = L->out.g_obs;
  out->global_mm = L->out.g_mm;
  out->n_groups = L->n_groups;
  return ok();
}

// per-group counts (index r + 1); returns 0 when the group does not exist
int bqsr_lut_group(const bqsr_lut* lc, int32_t r, int64_t* obs, int64_t* mm) {
  bqsr_lut* L = const_cast<bqsr_lut*>(lc);
  if (!L || lut_host(L) != BQSR_OK) return -1;
  if (r + 1 < 0 || r + 1 >= L->n_groups || !L->h_grp_ok[(size_t)(r + 1)]) return 0;
  *obs = L->h_grp_obs[(size_t)(r + 1)];
  *mm = L->h_grp_mm[(size_t)(r + 1)];
  return 1;
}

bqsr_status bqsr_lut_shifts(const bqsr_lut* lc, int32_t key, int32_t qual, int32_t cyc, int32_t ctx, double sh[4],
                            int32_t* new_q) {
  bqsr_lut* L = const_cast<bqsr_lut*>(lc);
  if (!L || !sh || !new_q) return fail(BQSR_ERR_INVALID_ARG, "null");
  bqsr_status st = lut_host(L);
  if (st != BQSR_OK) return st;
  const TableGeom g = geom(L->dims);
  if (cyc < -g.L || cyc > g.L || ctx < -4 || ctx > 16) return fail(BQSR_ERR_INVALID_ARG, "covariate out of range");
  const int64_t r = ((int64_t)key - 1) / kMaxQ;
  if (r + 1 < 0 || r + 1 >= L->n_groups || !L->h_grp_ok[(size_t)(r + 1)])
    return fail(BQSR_ERR_MISSING_KEY, "read group missing");
  const double avg = L->out.avg;
  double v;
  const double rgd = (eprob(L->h_grp_obs[(size_t)(r + 1)], L->h_grp_mm[(size_t)(r + 1)], &v) ? v : avg) - avg;
  if (key < 0 || key >= g.K || L->h_words[(size_t)key] == 0) return fail(BQSR_ERR_MISSING_KEY, "key missing");
  if (qual < 0 || qual > 255) return fail(BQSR_ERR_QUAL_RANGE, "qual out of range");
  const double e = pow10tab().v[qual];
  const double a1 = e + rgd;
  const double qd = (eprob(L->h_qk_obs[(size_t)key], L->h_qk_mm[(size_t)key], &v) ? v : a1) - a1;
  const double a2 = a1 + qd;
  const int64_t* obs = L->h_words.data() + g.K;
  const int64_t* mm = obs + (int64_t)g.K * g.cells;
  const int64_t c1 = (int64_t)key * g.cells + cyc + g.L, c2 = (int64_t)key * g.cells + g.C + ctx + 4;
  const double cd = (eprob(obs[c1], mm[c1], &v) ? v : a2) - a2;
  const double xd = (eprob(obs[c2], mm[c2], &v) ? v : a2) - a2;
  sh[0] = rgd;
  sh[1] = qd;
  sh[2] = cd;
  sh[3] = xd;
  double p = e;
  for (int i = 0; i < 4; ++i) p = p + sh[i];
  *new_q = phred_of(p);
  return ok();
}

// the threshold form of errorProbabilityToPhred, as the apply kernel uses it
int32_t bqsr_phred_threshold_table(double* out, int32_t cap, int32_t* qmin) {
  const auto& t = thresholds().thr;
  if (qmin) *qmin = kThrQmin;
  if (out) memcpy(out, t.data(), sizeof(double) * (size_t)std::min<int32_t>(cap, (int32_t)t.size()));
  return (int32_t)t.size();
}

// ---------------------------------------------------------------- apply ----

// stages: BQSR_STAGE_RESET (apply-kernel error word, exception count),
// BQSR_STAGE_KERNEL (apply kernel).  The prep kernel runs first when observe
// has not run it on this batch.
// bucketed batches: the per-read outputs by bqsr_apply_outs in read order
// instead of the walk's scattered stores (cfg4: apply 3.95 -> 3.67 ms + 0.13
// ms for the pass, profiles/r04aa_cfg4_apply_outs_ab.txt)

bqsr_status bqsr_apply_stage(bqsr_context* ctx, bqsr_batch* b, const bqsr_lut* L, uint8_t* out_qual,
                             uint32_t* out_start, uint32_t* out_len, uint64_t* exceptions, int64_t max_exceptions,
                             int32_t stages, void* stream) {
  if (!ctx || !b || !L || !out_qual || !out_start || !out_len) return fail(BQSR_ERR_INVALID_ARG, "null");
  if (b->dims.n_rg > L->dims.n_rg || b->dims.max_len > L->dims.max_len)
    return fail(BQSR_ERR_INVALID_ARG, "table dims smaller than the batch's");
  HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = S(stream);
  if (stages & BQSR_STAGE_RESET) {
    HIP_TRY(hipMemsetAsync(b->d_err + kErrAppKern, 0xFF, 8, s));
    HIP_TRY(hipMemsetAsync(b->d_err + kNExc, 0, 8, s));
  }
  if (!b->prepped || (stages & BQSR_STAGE_PREP)) {
    bqsr_status st = launch_prep(ctx, b, nullptr, s);
    if (st != BQSR_OK) return st;
  }
  if (b->rd.n_reads == 0 || !(stages & (BQSR_STAGE_KERNEL | BQSR_STAGE_LUT))) return ok();
  ApplyParams P{};
  P.rd = b->pass_rd();
  P.ord = b->order();
  P.info = b->d_info;
  P.g = geom(L->dims);
  const int cw = window_cw(b, P.g);
  // (measured and removed, round 3: a lean lane per read, 2.34 ms against the walk's 0.84 cfg2 --
  // its scattered 16-B result stores -- and a lane-per-offset rows kernel, SALU-bound at 5.9 ms)
  P.w = window_rows(b, apply_rows(cw));
  P.n_rg = L->dims.n_rg;
  P.s1 = L->s1;
  P.d2 = L->d2;
  P.rq_ok = L->rq_ok;
  P.key_ok = L->key_ok;
  P.grp_ok = L->grp_ok;
  P.n_groups = L->n_groups;
  P.thr = ctx->d_thr;
  P.thr_qmin = kThrQmin;
  P.thr_n = kThrN;
  P.qb_thr = ctx->d_qbt;
  P.qb_q = ctx->d_qbq;
  P.out_qual = out_qual;
  P.out_start = out_start;
  P.out_len = out_len;
  P.exc = (unsigned long long*)exceptions;
  P.max_exc = exceptions ? max_exceptions : 0;
  P.n_exc = b->d_err + kNExc;
  P.err = b->d_err + kErrAppKern;
  P.piece_stride = piece_bytes(P.w.qw, cw);
  // a char table per base key (fronts share their read group's)
  const size_t need = (size_t)P.piece_stride * (size_t)b->n_base + (size_t)b->n_base * 16;  // + rowbad
  if (b->chars_bytes < need) {  // grows with the window; kept across calls
    if (b->d_chars) {
      HIP_TRY(hipStreamSynchronize(s));
      (void)hipFree(b->d_chars);
      b->d_chars = nullptr;
      b->chars_bytes = 0;
    }
    HIP_TRY(hipMalloc((void**)&b->d_chars, need));
    b->chars_bytes = need;
    b->chars_lut = nullptr;
  }
  P.chars = b->d_chars;
  P.rowbad = (uint32_t*)(b->d_chars + (size_t)P.piece_stride * (size_t)b->n_base);
  P.qmask = b->hq_valid ? b->d_qmask : nullptr;
  const bool lut_stage = (stages & BQSR_STAGE_LUT) || ((stages & BQSR_STAGE_KERNEL) && !(stages & BQSR_STAGE_NO_LUT));
  if (lut_stage) {
    HIP_TRY(hipMemsetAsync(P.rowbad, 0, (size_t)b->n_base * 16, s));
    const unsigned cb = (unsigned)std::min<int64_t>(((int64_t)need + 255) / 256, (int64_t)ctx->n_cu * 16);
    hipLaunchKernelGGL(bqsr_apply_chars, dim3(cb), dim3(256), 0, s, P, b->d_chars);
    b->chars_lut = L;
  }
  if (stages & BQSR_STAGE_KERNEL) {
    if (b->chars_lut != L) return fail(BQSR_ERR_INVALID_ARG, "apply kernel before the LUT stage of this LUT");
    P.outs_apart = b->bucketed;
    hipLaunchKernelGGL(bqsr_apply_kernel, dim3(b->pass_blocks()), dim3(kBlockThreads), apply_lds(P.w.qw, cw), s, P);
    if (P.outs_apart) {
      ApplyParams Q = P;
      Q.rd = b->rd;  // (read order: the batch's own qual column, where a read not yet trimmed is)
      hipLaunchKernelGGL(bqsr_apply_outs, dim3((unsigned)std::min<int64_t>((b->rd.n_reads + 255) / 256, (int64_t)ctx->n_cu * 8)),
                         dim3(256), 0, s, Q);
    }
  }
  HIP_TRY(hipGetLastError());
  return ok();
}

bqsr_status bqsr_apply_async(bqsr_context* ctx, bqsr_batch* b, const bqsr_lut* L, uint8_t* out_qual,
                             uint32_t* out_start, uint32_t* out_len, uint64_t* exceptions, int64_t max_exceptions,
                             void* stream) {
  return bqsr_apply_stage(ctx, b, L, out_qual, out_start, out_len, exceptions, max_exceptions,
                          BQSR_STAGE_RESET | BQSR_STAGE_KERNEL, stream);
}

bqsr_status bqsr_apply_result(bqsr_batch* b, int64_t* n_exceptions, void* stream) {
  HIP_TRY(hipSetDevice(b->ctx->device));
  hipStream_t s = S(stream);
  unsigned long long w[kErrWords];
  HIP_TRY(hipMemcpyAsync(w, b->d_err, sizeof w, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (n_exceptions) *n_exceptions = (int64_t)w[kNExc];
  return from_err_key(std::min(w[kErrAppPrep], w[kErrAppKern]), 0);
}

bqsr_status bqsr_apply(bqsr_context* ctx, bqsr_batch* b, const bqsr_lut* l, uint8_t* out_qual, uint32_t* out_start,
                       uint32_t* out_len, uint64_t* exceptions, int64_t max_exceptions, int64_t* n_exceptions,
                       void* stream) {
  bqsr_status st = bqsr_apply_async(ctx, b, l, out_qual, out_start, out_len, exceptions, max_exceptions, stream);
  if (st != BQSR_OK) return st;
  return bqsr_apply_result(b, n_exceptions, stream);
}

bqsr_status bqsr_apply_records(bqsr_context* ctx, const bqsr_records* R, const bqsr_lut* l, uint16_t* out_qual,
                               uint32_t* out_len) {
  if (!ctx || !R || !l || !out_qual || !out_len) return fail(BQSR_ERR_INVALID_ARG, "null");
  bqsr_batch* b = nullptr;
  bqsr_status st = bqsr_batch_create(ctx, R, nullptr, &b);
  if (st != BQSR_OK) return st;
  const int64_t n = R->n_reads;
  uint8_t* d_out = nullptr;
  uint32_t *d_start = nullptr, *d_len = nullptr;
  uint64_t* d_exc = nullptr;
  const int64_t max_exc = 1 << 16;
  std::vector<void*> tmp;
  if ((st = dalloc(tmp, &d_out, (size_t)b->n_slots + 16)) != BQSR_OK || (st = dalloc(tmp, &d_start, (size_t)n)) != BQSR_OK ||
      (st = dalloc(tmp, &d_len, (size_t)n)) != BQSR_OK || (st = dalloc(tmp, &d_exc, (size_t)max_exc)) != BQSR_OK) {
    for (void* p : tmp) (void)hipFree(p);
    bqsr_batch_destroy(b);
    return st;
  }
  int64_t n_exc = 0;
  st = bqsr_apply(ctx, b, l, d_out, d_start, d_len, d_exc, max_exc, &n_exc, nullptr);
  if (st == BQSR_OK && n_exc > max_exc) st = fail(BQSR_ERR_UNSUPPORTED, "too many non-byte quality chars");
  if (st == BQSR_OK) {
    std::vector<uint8_t> h_out((size_t)b->n_slots + 16);
    std::vector<uint32_t> h_start((size_t)std::max<int64_t>(n, 1)), h_len((size_t)std::max<int64_t>(n, 1));
    std::vector<uint64_t> h_exc((size_t)std::max<int64_t>(n_exc, 1));
    hipError_t e = hipMemcpy(h_out.data(), d_out, h_out.size(), hipMemcpyDeviceToHost);
    if (e == hipSuccess && n) e = hipMemcpy(h_start.data(), d_start, (size_t)n * 4, hipMemcpyDeviceToHost);
    if (e == hipSuccess && n) e = hipMemcpy(h_len.data(), d_len, (size_t)n * 4, hipMemcpyDeviceToHost);
    if (e == hipSuccess && n_exc) e = hipMemcpy(h_exc.data(), d_exc, (size_t)n_exc * 8, hipMemcpyDeviceToHost);
    if (e != hipSuccess) {
      st = fail(BQSR_ERR_DEVICE, hipGetErrorString(e));
    } else {
      // slots of read r start at the packed offsets; rebuild them on the host
      std::vector<uint64_t> slot((size_t)n + 1, 0);
      for (int64_t r = 0; r < n; ++r) {
        const uint32_t f = R->flags[r];
        const uint64_t lq = (f & BQSR_F_HAS_QUAL) ? R->qual_offset[r + 1] - R->qual_offset[r] : 0;
        const uint64_t ls = (f & BQSR_F_HAS_SEQ) ? R->seq_offset[r + 1] - R->seq_offset[r] : 0;
        slot[(size_t)r + 1] = slot[(size_t)r] + (b->rd.slots_aligned ? slot_span(lq, ls) : std::max(lq, ls));
      }
      std::vector<uint16_t> wide;  // exceptions keyed by slot
      std::vector<std::pair<uint64_t, uint16_t>> ex;
      for (int64_t i = 0; i < n_exc; ++i) ex.push_back({h_exc[(size_t)i] >> 16, (uint16_t)(h_exc[(size_t)i] & 0xFFFF)});
      std::sort(ex.begin(), ex.end());
      for (int64_t r = 0; r < n; ++r) {
        uint16_t* dst = out_qual + R->qual_offset[r];
        const uint64_t s0 = slot[(size_t)r] + h_start[(size_t)r];
        for (uint32_t k = 0; k < h_len[(size_t)r]; ++k) {
          uint16_t v = h_out[s0 + k];
          if (!ex.empty()) {
            auto it = std::lower_bound(ex.begin(), ex.end(), std::make_pair(s0 + k, (uint16_t)0));
            if (it != ex.end() && it->first == s0 + k) v = it->second;
          }
          dst[k] = v;
        }
        out_len[r] = h_len[(size_t)r];
      }
    }
  }
  for (void* p : tmp) (void)hipFree(p);
  bqsr_batch_destroy(b);
  return st;
}


// ---- one job's launches with the fewest host round trips (adam_amd/job.py) ----
// bqsr_job_reset_async: the count table zeroed and the batch's error words /
// exception count reset in one kernel (bqsr_table_zero_async + the RESET
// stages).  bqsr_job_result: the batch's error words, expectedMismatch and
// the LUT's finalize status in one kernel writing pinned host memory, one
// stream sync, then the job's errors in the order the reference raises them
// (observe, EMPTY_TABLE at finalize, apply).
bqsr_status bqsr_job_reset_async(bqsr_batch* b, bqsr_table* t, void* stream) {
  if (!b || !t) return fail(BQSR_ERR_INVALID_ARG, "null");
  HIP_TRY(hipSetDevice(b->ctx->device));
  const int64_t n = table_words(t->dims);
  const unsigned g = (unsigned)std::min<int64_t>(std::max<int64_t>(1, (n + 255) / 256), (int64_t)b->ctx->n_cu * 8);
  hipLaunchKernelGGL(bqsr_job_reset_kernel, dim3(g), dim3(256), 0, S(stream), t->words, n, b->d_err);
  HIP_TRY(hipGetLastError());
  b->err_fresh = true;
  return ok();
}

bqsr_status bqsr_job_errors_export_async(bqsr_batch* b, int64_t read_base, int64_t* dst_device, void* stream) {
  if (!b || !dst_device || read_base < 0) return fail(BQSR_ERR_INVALID_ARG, "null / negative read base");
  HIP_TRY(hipSetDevice(b->ctx->device));
  hipLaunchKernelGGL(bqsr_job_err_export, dim3(1), dim3(64), 0, S(stream), (const unsigned long long*)b->d_err,
                     read_base, dst_device);
  HIP_TRY(hipGetLastError());
  return ok();
}

bqsr_status bqsr_job_errors_import_async(bqsr_batch* b, const int64_t* src_device, void* stream) {
  if (!b || !src_device) return fail(BQSR_ERR_INVALID_ARG, "null");
  HIP_TRY(hipSetDevice(b->ctx->device));
  hipLaunchKernelGGL(bqsr_job_err_import, dim3(1), dim3(64), 0, S(stream), (unsigned long long*)b->d_err, src_device);
  HIP_TRY(hipGetLastError());
  return ok();
}

// Snapshots for pipelined jobs (adam_amd/stream.py): the batch's status words
// of a job copied on `stream` into pinned slot `slot`, read after the caller
// has waited for the stream past that point; the next job may already reset
// the live words.
bqsr_status bqsr_job_status_async(bqsr_batch* b, bqsr_lut* L, int32_t slot, void* stream) {
  if (!b || !L || slot < 0 || slot >= kStatusSlots) return fail(BQSR_ERR_INVALID_ARG, "null / bad slot");
  HIP_TRY(hipSetDevice(b->ctx->device));
  if (!b->h_status)
    HIP_TRY(hipHostMalloc((void**)&b->h_status, kJobStatusWords * 8 * (1 + kStatusSlots), hipHostMallocDefault));
  hipLaunchKernelGGL(bqsr_job_status_kernel, dim3(1), dim3(64), 0, S(stream), (const unsigned long long*)b->d_err,
                     (const double*)b->d_em, (const FinalOut*)L->d_out, b->h_status + kJobStatusWords * (1 + slot));
  HIP_TRY(hipGetLastError());
  return ok();
}

bqsr_status bqsr_job_status_get(const bqsr_batch* b, int32_t slot, int32_t part, double* em, int64_t* n_exceptions) {
  if (!b || !b->h_status || slot < 0 || slot >= kStatusSlots || part < 0 || part > 2)
    return fail(BQSR_ERR_INVALID_ARG, "no snapshot / bad slot or part");
  const uint64_t* h = b->h_status + kJobStatusWords * (1 + slot);
  if (em) std::memcpy(em, h + kErrWords, 8);
  if (n_exceptions) *n_exceptions = (int64_t)h[kNExc];
  if (part == 0) return from_err_key(h[kErrObs], 0);
  if (part == 1) {
    FinalOut fo;
    std::memcpy(&fo, h + kErrWords + 1, sizeof(FinalOut));
    return fo.any_key ? ok() : fail(BQSR_ERR_EMPTY_TABLE, "empty.reduceLeft: no usable base was observed");
  }
  return from_err_key(std::min(h[kErrAppPrep], h[kErrAppKern]), 0);
}

// workgroups of a kernel copy: enough stores in flight for the link, few
// enough CUs that the compute streams' kernels keep running beside it
// (32: cfg5 374.8 / 402.9 / 407.0 ms per job at 32 / 128 / 512 workgroups on
// one box, profiles/r03n_cfg3_sites_bitmap_ab.txt; 16-64 within the spread,
// profiles/r04u_cfg5_copy_blocks_ab.txt)
static int64_t copy_blocks(const bqsr_context* ctx) { return std::min<int64_t>(32, (int64_t)ctx->n_cu * 8); }
bqsr_status bqsr_copy_async(bqsr_context* ctx, void* dst, const void* src, int64_t bytes, void* stream) {
  if (!ctx || bytes < 0 || (bytes && (!dst || !src))) return fail(BQSR_ERR_INVALID_ARG, "bqsr_copy_async: bad arguments");
  if (!bytes) return ok();
  HIP_TRY(hipSetDevice(ctx->device));
  const bool vec = (((uintptr_t)dst | (uintptr_t)src) & 15) == 0;
  const int64_t n16 = vec ? bytes / 16 : 0;
  const int64_t head = 16 * n16, tail = bytes - head;
  const int64_t need = std::max<int64_t>((n16 + 255) / 256, (tail + 255) / 256);
  const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>(need, copy_blocks(ctx)));
  hipLaunchKernelGGL(bqsr_copy16, dim3(g), dim3(256), 0, S(stream), (const uint4*)src, (uint4*)dst, n16,
                     (const uint8_t*)src + head, (uint8_t*)dst + head, tail);
  HIP_TRY(hipGetLastError());
  return ok();
}

bqsr_status bqsr_job_result(bqsr_batch* b, bqsr_lut* L, double* em, int64_t* n_exceptions, void* stream) {
  if (!b || !L) return fail(BQSR_ERR_INVALID_ARG, "null");
  HIP_TRY(hipSetDevice(b->ctx->device));
  hipStream_t s = S(stream);
  if (!b->h_status)
    HIP_TRY(hipHostMalloc((void**)&b->h_status, kJobStatusWords * 8 * (1 + kStatusSlots), hipHostMallocDefault));
  hipLaunchKernelGGL(bqsr_job_status_kernel, dim3(1), dim3(64), 0, s, (const unsigned long long*)b->d_err,
                     (const double*)b->d_em, (const FinalOut*)L->d_out, b->h_status);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(s));
  const uint64_t* h = b->h_status;
  std::memcpy(&L->out, h + kErrWords + 1, sizeof(FinalOut));
  L->out_pending = false;
  if (em) std::memcpy(em, h + kErrWords, 8);
  if (n_exceptions) *n_exceptions = (int64_t)h[kNExc];
  bqsr_status st = from_err_key(h[kErrObs], 0);
  if (st != BQSR_OK) return st;
  if (!L->out.any_key) return fail(BQSR_ERR_EMPTY_TABLE, "empty.reduceLeft: no usable base was observed");
  return from_err_key(std::min(h[kErrAppPrep], h[kErrAppKern]), 0);
}

}  // extern "C"

// ---- SAM ingest / output (include/adam_sam.h) ----
#include "sam_ingest.hip"
#include "bgzf_inflate.hip"
#include "bam_ingest.hip"
#include "mark_duplicates.cpp"
#include "adam_out.hip"
#include "sam_batch.hip"
#include "arrow_ingest.hip"
#include "parquet_gzip.cpp"

// ---- streamed outputs: compaction (uses the SAM code's scans) ----
extern "C" {

bqsr_status bqsr_compact_outputs_async(bqsr_context* ctx, bqsr_batch* b, const uint8_t* out_qual,
                                       const uint32_t* out_start, const uint32_t* out_len, uint64_t* exceptions,
                                       int64_t max_exceptions, uint8_t* chars, uint32_t* offsets, uint16_t* lengths,
                                       void* stream) {
  if (!ctx || !b || !out_qual || !out_start || !out_len || !chars || !offsets || max_exceptions < 0 ||
      (max_exceptions > 0 && !exceptions))
    return fail(BQSR_ERR_INVALID_ARG, "bqsr_compact_outputs_async: bad arguments");
  if (b->n_slots > (int64_t)UINT32_MAX) return fail(BQSR_ERR_UNSUPPORTED, "compacted chars above 4 GiB");
  HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = S(stream);
  const int64_t n = b->rd.n_reads;
  if (!b->d_off64 || b->off64_n < n) {  // scratch: u64 lengths and their scan (kept on the batch)
    if (b->d_off64) {
      HIP_TRY(hipStreamSynchronize(s));
      (void)hipFree(b->d_off64);
      b->d_off64 = nullptr;
    }
    const size_t words = 2 * ((size_t)n + 1) + (size_t)n / samk::kScanChunk + 2;
    HIP_TRY(hipMalloc((void**)&b->d_off64, words * 8));
    b->off64_n = n;
  }
  uint64_t* len64 = b->d_off64;
  uint64_t* off64 = len64 + n + 1;
  uint64_t* part = off64 + n + 1;
  const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, (int64_t)ctx->n_cu * 8));
  if (n > 0) hipLaunchKernelGGL(bqsr_compact_lens, dim3(g), dim3(256), 0, s, out_len, n, len64);
  bqsr_status st = sam_scan(len64, n, off64, part, s);
  if (st != BQSR_OK) return st;
  if (n > 0) {
    hipLaunchKernelGGL(bqsr_compact_chars, dim3(g), dim3(256), 0, s, (const ReadMeta*)b->rd.meta, out_qual, out_start,
                       (const uint64_t*)off64, n, chars, offsets, lengths);
    if (max_exceptions > 0)
      hipLaunchKernelGGL(bqsr_compact_exceptions, dim3(4), dim3(256), 0, s, (const ReadMeta*)b->rd.meta, n, out_start,
                         (const uint64_t*)off64, (unsigned long long*)exceptions,
                         (const unsigned long long*)(b->d_err + kNExc), max_exceptions);
  } else {
    HIP_TRY(hipMemsetAsync(offsets, 0, 4, s));
  }
  HIP_TRY(hipGetLastError());
  return ok();
}

const void* bqsr_batch_exception_count_ptr(const bqsr_batch* b) { return b ? (const void*)(b->d_err + kNExc) : nullptr; }

bqsr_status bqsr_copy_dyn_async(bqsr_context* ctx, void* dst, const void* src, const void* count, int32_t count_bytes,
                                int64_t scale, int64_t max_bytes, void* stream) {
  if (!ctx || !dst || !src || !count || (count_bytes != 4 && count_bytes != 8) || scale < 0 || max_bytes < 0)
    return fail(BQSR_ERR_INVALID_ARG, "bqsr_copy_dyn_async: bad arguments");
  HIP_TRY(hipSetDevice(ctx->device));
  const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>((max_bytes / 16 + 255) / 256, copy_blocks(ctx)));
  hipLaunchKernelGGL(bqsr_copy_dyn, dim3(g), dim3(256), 0, S(stream), (const uint8_t*)src, (uint8_t*)dst, count,
                     count_bytes, scale, max_bytes);
  HIP_TRY(hipGetLastError());
  return ok();
}

}  // extern "C"
