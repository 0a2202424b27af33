// SAM text <-> device columns around the BQSR path.
//
// Ingest (bqsr_sam_parse): the header on the host (its @RG IDs sorted into
// the RecordGroupDictionary, RecordGroupDictionary.scala:36-43; its @SQ
// names), the records on the device:
//   sam_nl_count / sam_nl_scan / sam_nl_write   newline positions (a count per
//       16-KB chunk, a scan, the positions written in order)
//   sam_lines(pass 1)   one thread per line: field split, FLAG / POS / CIGAR /
//       tags parsed with SAMRecordConverter's semantics
//       (SAMRecordConverter.scala:26-144, as adam_amd/records.py:read_sam
//       restates them), per-line column lengths out
//   scan_* (exclusive u64 scans)   lengths -> column offsets, kept lines -> read ids
//   sam_lines(pass 2)   the same parse, writing the columns
//   sam_ref_first / sam_ref_remap   referenceName ids in first-appearance order
//       (RecordBatch.from_records)
// Output (bqsr_sam_rewrite_quals): one thread per record computes its new
// line length (QUAL field -> the recalibrated chars as UTF-8), a scan places
// the lines, a second pass copies the bytes.
//
// Included by bqsr_capi.cpp (one code object with the BQSR kernels).

#include <map>
#include <memory>

#include "../../include/adam_sam.h"

namespace samk {

constexpr int kNlThreads = 256;
constexpr int kNlBytes = 64;                           // per thread
constexpr int64_t kNlChunk = kNlThreads * kNlBytes;    // bytes per workgroup
constexpr int kScanThreads = 256;
constexpr int kScanPer = 8;                            // u64 per thread
constexpr int64_t kScanChunk = kScanThreads * kScanPer;

// error word: (line << 8) | code, the smallest wins (the first bad line)
enum : uint32_t {
  kSamOk = 0,
  kSamFields = 1,     // fewer than 11 tab-separated fields (tuple unpacking, records.py:322)
  kSamTag = 2,        // an optional field without two ':' (t.split(":", 2), records.py:326)
  kSamFlag = 3,       // FLAG not an integer (int(flag))
  kSamPos = 4,        // POS not an integer (int(pos))
  kSamCigar = 5,      // malformed CIGAR (TextCigarCodec.decode)
  kSamHeader = 6,     // a header line after the first record
  kSamCr = 7,         // a '\r' inside a line
};

__host__ __device__ inline uint64_t fnv1a(const uint8_t* p, int64_t n) {
  uint64_t h = 1469598103934665603ull;
  for (int64_t i = 0; i < n; ++i) h = (h ^ p[i]) * 1099511628211ull;
  return h;
}

// open-addressing name -> value table, built on the host
struct NameTable {
  const uint8_t* blob;
  const uint64_t* off;  // [n + 1]
  const int32_t* slot;  // [mask + 1] name index or -1
  const int32_t* value; // [n]
  uint32_t mask;
  int32_t n;
};

__device__ int32_t name_lookup(const NameTable& t, const uint8_t* p, int64_t n) {
  if (t.n == 0) return -1;
  uint32_t i = (uint32_t)fnv1a(p, n) & t.mask;
  for (;;) {
    const int32_t k = t.slot[i];
    if (k < 0) return -1;
    const int64_t a = (int64_t)t.off[k], len = (int64_t)t.off[k + 1] - a;
    if (len == n) {
      int64_t j = 0;
      while (j < n && t.blob[a + j] == p[j]) ++j;
      if (j == n) return t.value[k];
    }
    i = (i + 1) & t.mask;
  }
}

struct SamParams {
  const uint8_t* text;
  int64_t body, n;       // records occupy text[body, n)
  const uint64_t* nl;    // newline positions in [body, n), ascending
  int64_t n_nl, n_lines;
  NameTable sq, rg;
  uint64_t* len;         // [5][n_lines]: keep, seq, qual, cigar ops, md bytes
  uint64_t* off;         // [5][n_lines + 1]: their exclusive scans
  // per read (pass 2)
  uint32_t* flags;
  int32_t* rg_id;
  int32_t* ref;          // @SQ index until sam_ref_remap
  int32_t* sq_id;        // the @SQ header index (referenceId), -1 = none
  uint32_t* raw_flag;    // the FLAG word
  int64_t* start;
  uint64_t* seq_off;
  uint8_t* seq;
  uint64_t* qual_off;
  uint8_t* qual;
  uint64_t* cig_off;
  uint32_t* cig;
  uint64_t* md_off;
  uint8_t* md;
  uint64_t* line_span;   // [2n]: line start, line end (no newline)
  uint64_t* qual_span;   // [2n]: the QUAL field
  unsigned long long* err;
};

// ---- newline positions ----
__device__ __forceinline__ uint32_t nl_mask_word(uint32_t w) {  // 0x80 in every byte equal to '\n'
  const uint32_t x = w ^ 0x0A0A0A0Au;
  return ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);
}
__device__ __forceinline__ int thread_nl(const uint8_t* t, int64_t lo, int64_t hi, uint32_t m[kNlBytes / 4]) {
  // m: per-word masks of the thread's 64 bytes [lo, lo + 64) clipped to hi
  int c = 0;
  if (lo + kNlBytes <= hi && (((uintptr_t)(t + lo)) & 15) == 0) {
#pragma unroll
    for (int v = 0; v < kNlBytes / 16; ++v) {
      const uint4 q = *(const uint4*)(t + lo + 16 * v);
      m[4 * v] = nl_mask_word(q.x);
      m[4 * v + 1] = nl_mask_word(q.y);
      m[4 * v + 2] = nl_mask_word(q.z);
      m[4 * v + 3] = nl_mask_word(q.w);
    }
  } else {
#pragma unroll
    for (int w = 0; w < kNlBytes / 4; ++w) {
      uint32_t mm = 0;
      for (int b = 0; b < 4; ++b) {
        const int64_t p = lo + 4 * w + b;
        if (p < hi && t[p] == '\n') mm |= 0x80u << (8 * b);
      }
      m[w] = mm;
    }
  }
#pragma unroll
  for (int w = 0; w < kNlBytes / 4; ++w) c += __popc(m[w]);
  return c;
}

__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* total) {
  __shared__ uint32_t s[kNlThreads];
  const int tid = threadIdx.x;
  s[tid] = v;
  __syncthreads();
  for (int d = 1; d < kNlThreads; d <<= 1) {
    const uint32_t a = tid >= d ? s[tid - d] : 0u;
    __syncthreads();
    s[tid] += a;
    __syncthreads();
  }
  const uint32_t incl = s[tid];
  *total = s[kNlThreads - 1];
  __syncthreads();
  return incl - v;
}

extern "C" __global__ void __launch_bounds__(kNlThreads) sam_nl_count(const uint8_t* t, int64_t lo, int64_t hi,
                                                                      uint64_t* cnt) {
  const int64_t b0 = lo + (int64_t)blockIdx.x * kNlChunk + (int64_t)threadIdx.x * kNlBytes;
  uint32_t m[kNlBytes / 4];
  const uint32_t c = b0 < hi ? (uint32_t)thread_nl(t, b0, hi, m) : 0u;
  uint32_t total;
  (void)block_excl_scan(c, &total);
  if (threadIdx.x == 0) cnt[blockIdx.x] = total;
}

extern "C" __global__ void __launch_bounds__(kNlThreads) sam_nl_write(const uint8_t* t, int64_t lo, int64_t hi,
                                                                      const uint64_t* base, uint64_t* nl) {
  const int64_t b0 = lo + (int64_t)blockIdx.x * kNlChunk + (int64_t)threadIdx.x * kNlBytes;
  uint32_t m[kNlBytes / 4];
  const uint32_t c = b0 < hi ? (uint32_t)thread_nl(t, b0, hi, m) : 0u;
  uint32_t total;
  uint64_t k = base[blockIdx.x] + block_excl_scan(c, &total);
  if (b0 >= hi) return;
#pragma unroll
  for (int w = 0; w < kNlBytes / 4; ++w) {
    uint32_t mm = m[w];
    while (mm) {
      const int bit = __builtin_ctz(mm);
      mm &= mm - 1;
      nl[k++] = (uint64_t)(b0 + 4 * w + (bit >> 3));
    }
  }
}

// ---- exclusive u64 scans: out[0..n] (out[n] = total) ----
extern "C" __global__ void __launch_bounds__(kScanThreads) scan_partials(const uint64_t* in, int64_t n,
                                                                         uint64_t* part) {
  __shared__ uint64_t s[kScanThreads];
  const int64_t i0 = (int64_t)blockIdx.x * kScanChunk + (int64_t)threadIdx.x * kScanPer;
  uint64_t v = 0;
#pragma unroll
  for (int k = 0; k < kScanPer; ++k)
    if (i0 + k < n) v += in[i0 + k];
  s[threadIdx.x] = v;
  __syncthreads();
  for (int d = kScanThreads / 2; d > 0; d >>= 1) {
    if ((int)threadIdx.x < d) s[threadIdx.x] += s[threadIdx.x + d];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = s[0];
}

// one workgroup: part[0..nb) -> exclusive scan in place, part[nb] = total
extern "C" __global__ void __launch_bounds__(1024) scan_top(uint64_t* part, int64_t nb) {
  __shared__ uint64_t s[1024];
  const int tid = threadIdx.x;
  const int64_t per = (nb + 1023) / 1024;
  const int64_t k0 = min(nb, tid * per), k1 = min(nb, k0 + per);
  uint64_t v = 0;
  for (int64_t k = k0; k < k1; ++k) v += part[k];
  s[tid] = v;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {
    const uint64_t a = tid >= d ? s[tid - d] : 0ull;
    __syncthreads();
    s[tid] += a;
    __syncthreads();
  }
  uint64_t acc = s[tid] - v;
  for (int64_t k = k0; k < k1; ++k) {
    const uint64_t x = part[k];
    part[k] = acc;
    acc += x;
  }
  if (tid == 1023) part[nb] = s[1023];
}

extern "C" __global__ void __launch_bounds__(kScanThreads) scan_apply(const uint64_t* in, int64_t n,
                                                                      const uint64_t* part, uint64_t* out) {
  __shared__ uint64_t s[kScanThreads];
  const int tid = threadIdx.x;
  const int64_t i0 = (int64_t)blockIdx.x * kScanChunk + (int64_t)tid * kScanPer;
  uint64_t x[kScanPer];
  uint64_t v = 0;
#pragma unroll
  for (int k = 0; k < kScanPer; ++k) {
    x[k] = i0 + k < n ? in[i0 + k] : 0ull;
    v += x[k];
  }
  s[tid] = v;
  __syncthreads();
  for (int d = 1; d < kScanThreads; d <<= 1) {
    const uint64_t a = tid >= d ? s[tid - d] : 0ull;
    __syncthreads();
    s[tid] += a;
    __syncthreads();
  }
  uint64_t acc = part[blockIdx.x] + s[tid] - v;
#pragma unroll
  for (int k = 0; k < kScanPer; ++k) {
    if (i0 + k < n) out[i0 + k] = acc;
    acc += x[k];
  }
  if (blockIdx.x == gridDim.x - 1 && tid == 0) out[n] = part[gridDim.x];
}

// ---- Java float text (tag values of type 'f') ----
// java.lang.Float.toString: the fewest significant digits (at most 9) that
// read back as the same float; plain notation for 1e-3 <= |f| < 1e7
// ("100.0", "0.00125"), else "d.dddE[-]n" ("1.0E7", "1.5E-4"); "NaN",
// "Infinity", "0.0" / "-0.0".  Powers of ten and the read-back are double
// arithmetic: exact for the float's digits except at decimal ties (parity
// unpinned).  out == nullptr: the length only.
__device__ double pow10_d(int k) {
  const double kP[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                         1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
  double v = 1.0;
  int a = k < 0 ? -k : k;
  while (a > 22) {
    v *= 1e22;
    a -= 22;
  }
  v *= kP[a];
  return k < 0 ? 1.0 / v : v;
}
__device__ int put_text(uint8_t* out, int n, const char* t) {
  int k = 0;
  for (; t[k]; ++k)
    if (out) out[n + k] = (uint8_t)t[k];
  return n + k;
}
__device__ int java_float_text(float f, uint8_t* out) {
  int n = 0;
  if (f != f) return put_text(out, 0, "NaN");
  if (__builtin_signbit(f)) n = put_text(out, n, "-");
  const double x = fabs((double)f);
  if (isinf(x)) return put_text(out, n, "Infinity");
  if (x == 0.0) return put_text(out, n, "0.0");
  int k = (int)floor(log10(x));
  while (k > -60 && pow10_d(k) > x) --k;
  while (k < 60 && pow10_d(k + 1) <= x) ++k;
  uint32_t dig = 0;
  int e = k, p = 1;
  for (; p <= 9; ++p) {
    const int sh = p - 1 - k;
    const double y = sh >= 0 ? x * pow10_d(sh) : x / pow10_d(-sh);
    const double d = rint(y);
    const double v = sh >= 0 ? d / pow10_d(sh) : d * pow10_d(-sh);
    if ((float)v == fabsf(f) || p == 9) {
      dig = (uint32_t)d;
      e = k;
      if (d >= pow10_d(p)) {  // rounded up to 10^p: one more decade
        dig /= 10u;
        e = k + 1;
      }
      break;
    }
  }
  uint8_t D[10];
  int nd = 0;
  {
    uint8_t t[10];
    int m = 0;
    do {
      t[m++] = (uint8_t)('0' + dig % 10u);
      dig /= 10u;
    } while (dig);
    for (int i = 0; i < m; ++i) D[i] = t[m - 1 - i];
    nd = m;
    while (nd > 1 && D[nd - 1] == '0') --nd;  // digits without trailing zeros
  }
  auto put = [&](uint8_t c) {
    if (out) out[n] = c;
    ++n;
  };
  if (e >= -3 && e < 7) {
    if (e >= 0) {
      for (int i = 0; i <= e; ++i) put(i < nd ? D[i] : (uint8_t)'0');
      put('.');
      if (nd > e + 1)
        for (int i = e + 1; i < nd; ++i) put(D[i]);
      else
        put('0');
    } else {
      put('0');
      put('.');
      for (int i = 0; i < -e - 1; ++i) put('0');
      for (int i = 0; i < nd; ++i) put(D[i]);
    }
  } else {
    put(D[0]);
    put('.');
    if (nd > 1)
      for (int i = 1; i < nd; ++i) put(D[i]);
    else
      put('0');
    put('E');
    int a = e;
    if (a < 0) {
      put('-');
      a = -a;
    }
    uint8_t t[4];
    int m = 0;
    do {
      t[m++] = (uint8_t)('0' + a % 10);
      a /= 10;
    } while (a);
    while (m) put(t[--m]);
  }
  return n;
}
// java.lang.Float.parseFloat of t[a, b) (decimal forms, NaN / Infinity);
// false when it would throw NumberFormatException
__device__ bool java_parse_float(const uint8_t* t, int64_t a, int64_t b, float* v) {
  while (a < b && t[a] <= ' ') ++a;  // String.trim
  while (b > a && t[b - 1] <= ' ') --b;
  bool neg = false;
  if (a < b && (t[a] == '+' || t[a] == '-')) {
    neg = t[a] == '-';
    ++a;
  }
  auto is = [&](const char* w) {
    int64_t i = 0;
    for (; w[i]; ++i)
      if (a + i >= b || t[a + i] != (uint8_t)w[i]) return false;
    return a + i == b;
  };
  if (is("NaN")) {
    *v = __builtin_nanf("");
    return true;
  }
  if (is("Infinity")) {
    *v = neg ? -__builtin_inff() : __builtin_inff();
    return true;
  }
  uint64_t m = 0;
  int nd = 0, dexp = 0;
  bool any = false, dot = false;
  int64_t i = a;
  for (; i < b; ++i) {
    const uint8_t c = t[i];
    if (c >= '0' && c <= '9') {
      any = true;
      if (nd < 19) {
        if (m || c != '0') {
          m = m * 10 + (c - '0');
          ++nd;
        }
        if (dot) --dexp;
      } else if (!dot) {
        ++dexp;
      }
    } else if (c == '.' && !dot) {
      dot = true;
    } else {
      break;
    }
  }
  if (!any) return false;
  if (i < b && (t[i] == 'e' || t[i] == 'E')) {
    ++i;
    bool en = false;
    if (i < b && (t[i] == '+' || t[i] == '-')) en = t[i++] == '-';
    if (i >= b) return false;
    int x = 0;
    for (; i < b && t[i] >= '0' && t[i] <= '9'; ++i) x = x < 100000 ? x * 10 + (t[i] - '0') : x;
    dexp += en ? -x : x;
  }
  if (i < b && (t[i] == 'f' || t[i] == 'F' || t[i] == 'd' || t[i] == 'D')) ++i;  // Java's type suffixes
  if (i != b) return false;
  double d = (double)m;
  if (dexp < -340) d = 0.0;
  else if (dexp > 0) d *= pow10_d(dexp > 320 ? 320 : dexp);
  else if (dexp < 0) d /= pow10_d(-dexp > 320 ? 320 : -dexp);
  *v = neg ? -(float)d : (float)d;
  return true;
}

// ---- the record parser ----
__device__ __forceinline__ void sam_error(const SamParams& P, int64_t line, uint32_t code) {
  atomicMin(P.err, (unsigned long long)(((uint64_t)line << 8) | code));
}

// Python int() of a field (digits with an optional sign, spaces around)
__device__ bool parse_int(const uint8_t* t, int64_t a, int64_t b, int64_t* v) {
  while (a < b && t[a] == ' ') ++a;
  while (b > a && t[b - 1] == ' ') --b;
  bool neg = false;
  if (a < b && (t[a] == '+' || t[a] == '-')) {
    neg = t[a] == '-';
    ++a;
  }
  if (a >= b || b - a > 18) return false;
  int64_t x = 0;
  for (int64_t i = a; i < b; ++i) {
    const uint8_t c = t[i];
    if (c < '0' || c > '9') return false;
    x = x * 10 + (c - '0');
  }
  *v = neg ? -x : x;
  return true;
}

// samtools TextCigarCodec.decode as records.py:parse_cigar: "*" / "" -> no
// elements; else (digits op)+ with op in MIDNSHP=X and length < 2^28
__device__ bool parse_cigar_text(const uint8_t* t, int64_t a, int64_t b, uint32_t* out, uint64_t* n_ops) {
  uint64_t k = 0;
  if (b - a == 1 && t[a] == '*') {
    *n_ops = 0;
    return true;
  }
  int64_t num = -1;
  for (int64_t i = a; i < b; ++i) {
    const uint8_t c = t[i];
    if (c >= '0' && c <= '9') {
      num = (num < 0 ? 0 : num) * 10 + (c - '0');
      if (num > (int64_t(1) << 40)) num = int64_t(1) << 40;  // stays >= 2^28: rejected at its op
      continue;
    }
    int op = -1;
    switch (c) {
      case 'M': op = 0; break;
      case 'I': op = 1; break;
      case 'D': op = 2; break;
      case 'N': op = 3; break;
      case 'S': op = 4; break;
      case 'H': op = 5; break;
      case 'P': op = 6; break;
      case '=': op = 7; break;
      case 'X': op = 8; break;
      default: break;
    }
    if (op < 0 || num < 0 || num >= (int64_t(1) << 28)) return false;
    if (out) out[k] = ((uint32_t)num << 4) | (uint32_t)op;
    ++k;
    num = -1;
  }
  if (num >= 0) return false;
  *n_ops = k;
  return true;
}

__device__ __forceinline__ void line_bounds(const SamParams& P, int64_t i, int64_t* s, int64_t* e) {
  *s = i == 0 ? P.body : (int64_t)P.nl[i - 1] + 1;
  *e = i < P.n_nl ? (int64_t)P.nl[i] : P.n;
}

// the byte columns a line's read fills (pass 2 copies them wavefront-wide)
struct LineCopy {
  int64_t seq_src, seq_n, qual_src, qual_n, md_src, md_n;
  uint64_t seq_dst, qual_dst, md_dst;
};

// pass 1 (write == false): lengths per line; pass 2: the columns of read `r`
template <bool kWrite>
__device__ void parse_line(const SamParams& P, int64_t i, LineCopy* cp) {
  const uint8_t* t = P.text;
  int64_t s, e;
  line_bounds(P, i, &s, &e);
  if (e > s && t[e - 1] == '\r') --e;  // universal newlines: "\r\n" ends a line
  if (e == s) {  // empty line: skipped
    if (!kWrite)
      for (int c = 0; c < 5; ++c) P.len[(int64_t)c * P.n_lines + i] = 0;
    return;
  }
  if (!kWrite) {
    if (t[s] == '@') {
      sam_error(P, i, kSamHeader);
      return;
    }
  }
  // the 11 mandatory fields
  int64_t fa[11], fb[11];
  int64_t p = s;
  bool more = false;
  for (int f = 0; f < 11; ++f) {
    fa[f] = p;
    while (p < e && t[p] != '\t') {
      if (!kWrite && t[p] == '\r') {
        sam_error(P, i, kSamCr);
        return;
      }
      ++p;
    }
    fb[f] = p;
    if (p < e) {
      ++p;
      if (f == 10) more = true;
    } else if (f < 10) {
      if (!kWrite) sam_error(P, i, kSamFields);
      return;
    }
  }
  // optional fields: the last MD and RG win (dict)
  int64_t md_a = -1, md_b = -1, rg_a = -1, rg_b = -1;
  while (more) {
    const int64_t ta = p;
    int64_t c1 = -1, c2 = -1;
    while (p < e && t[p] != '\t') {
      if (t[p] == ':') {
        if (c1 < 0) c1 = p;
        else if (c2 < 0) c2 = p;
      } else if (!kWrite && t[p] == '\r') {
        sam_error(P, i, kSamCr);
        return;
      }
      ++p;
    }
    const int64_t tb = p;
    more = p < e;
    if (more) ++p;
    if (c2 < 0) {
      if (!kWrite) sam_error(P, i, kSamTag);
      return;
    }
    if (c1 - ta == 2 && t[ta] == 'M' && t[ta + 1] == 'D') {
      md_a = c2 + 1;
      md_b = tb;
    } else if (c1 - ta == 2 && t[ta] == 'R' && t[ta + 1] == 'G') {
      rg_a = c2 + 1;
      rg_b = tb;
    }
  }
  int64_t flag = 0;
  if (!parse_int(t, fa[1], fb[1], &flag)) {
    if (!kWrite) sam_error(P, i, kSamFlag);
    return;
  }
  // RNAME: referenceName only when it is a header @SQ name; POS only then
  int32_t sq = -1;
  int64_t start = 0;
  bool has_start = false;
  if (!(fb[2] - fa[2] == 1 && t[fa[2]] == '*')) sq = name_lookup(P.sq, t + fa[2], fb[2] - fa[2]);
  if (sq >= 0) {
    int64_t pos;
    if (!parse_int(t, fa[3], fb[3], &pos)) {
      if (!kWrite) sam_error(P, i, kSamPos);
      return;
    }
    if (pos != 0) {
      start = pos - 1;
      has_start = true;
    }
  }
  uint64_t n_ops = 0;
  if (!kWrite) {
    if (!parse_cigar_text(t, fa[5], fb[5], nullptr, &n_ops)) {
      sam_error(P, i, kSamCigar);
      return;
    }
  }
  const int32_t rg = rg_a >= 0 ? name_lookup(P.rg, t + rg_a, rg_b - rg_a) : -1;
  // SAMRecordConverter.scala:72-108: flags only when the word is non-zero (Q2)
  uint32_t f = BQSR_F_HAS_SEQ | BQSR_F_HAS_QUAL | BQSR_F_HAS_CIGAR;
  if (flag != 0) {
    if (flag & 0x1) {
      f |= BQSR_F_PAIRED;
      if (flag & 0x80) f |= BQSR_F_SECOND_OF_PAIR;
    }
    if (flag & 0x400) f |= BQSR_F_DUPLICATE;
    if (flag & 0x10) f |= BQSR_F_NEG_STRAND;
    if (!(flag & 0x100)) f |= BQSR_F_PRIMARY;
    if (!(flag & 0x4)) f |= BQSR_F_MAPPED;
  }
  if (sq >= 0) f |= BQSR_F_HAS_REFNAME;
  if (has_start) f |= BQSR_F_HAS_START;
  if (md_a >= 0) f |= BQSR_F_HAS_MD;
  if (rg >= 0) f |= BQSR_F_HAS_RG;
  const int64_t seq_n = fb[9] - fa[9], qual_n = fb[10] - fa[10], md_n = md_a >= 0 ? md_b - md_a : 0;
  if (!kWrite) {
    const int64_t L = P.n_lines;
    P.len[i] = 1;
    P.len[L + i] = (uint64_t)seq_n;
    P.len[2 * L + i] = (uint64_t)qual_n;
    P.len[3 * L + i] = n_ops;
    P.len[4 * L + i] = (uint64_t)md_n;
    return;
  }
  const int64_t L1 = P.n_lines + 1;
  const int64_t r = (int64_t)P.off[i];
  const uint64_t os = P.off[L1 + i], oq = P.off[2 * L1 + i], oc = P.off[3 * L1 + i], om = P.off[4 * L1 + i];
  P.flags[r] = f;
  P.rg_id[r] = rg >= 0 ? rg : 0;
  P.ref[r] = sq;
  P.sq_id[r] = sq;
  P.raw_flag[r] = (uint32_t)flag;
  P.start[r] = start;
  P.seq_off[r] = os;
  P.qual_off[r] = oq;
  P.cig_off[r] = oc;
  P.md_off[r] = om;
  (void)parse_cigar_text(t, fa[5], fb[5], P.cig + oc, &n_ops);
  cp->seq_src = fa[9];
  cp->seq_dst = os;
  cp->seq_n = seq_n;
  cp->qual_src = fa[10];
  cp->qual_dst = oq;
  cp->qual_n = qual_n;
  cp->md_src = md_a;
  cp->md_dst = om;
  cp->md_n = md_n;
  P.line_span[2 * r] = (uint64_t)s;
  P.line_span[2 * r + 1] = (uint64_t)e;
  P.qual_span[2 * r] = (uint64_t)fa[10];
  P.qual_span[2 * r + 1] = (uint64_t)fb[10];
}

extern "C" __global__ void sam_lines_len(SamParams P) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < P.n_lines; i += (int64_t)gridDim.x * blockDim.x)
    parse_line<false>(P, i, nullptr);
}

__device__ __forceinline__ int64_t rl64(int64_t v, int j) {
  return (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), j) << 32) |
                   (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, j));
}
// a wavefront copies one line's bytes at a time, 64 lanes wide
__device__ __forceinline__ void wave_copy(const uint8_t* src, uint8_t* dst, int64_t n, int lane) {
  for (int64_t k = lane; k < n; k += 64) dst[k] = src[k];
}

// pass 2: a lane per line parses and writes the scalar columns and CIGAR,
// then the wavefront copies SEQ / QUAL / MD of its 64 lines together
extern "C" __global__ void __launch_bounds__(256) sam_lines_write(SamParams P) {
  const int lane = threadIdx.x & 63;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i0 = blockIdx.x * (int64_t)blockDim.x + (threadIdx.x & ~63); i0 < P.n_lines; i0 += stride) {
    const int64_t i = i0 + lane;
    LineCopy c{0, 0, 0, 0, 0, 0, 0, 0, 0};
    if (i < P.n_lines && P.len[i]) parse_line<true>(P, i, &c);
    for (int j = 0; j < 64; ++j) {
      const int64_t sn = rl64(c.seq_n, j), qn = rl64(c.qual_n, j), mn = rl64(c.md_n, j);
      if (sn) wave_copy(P.text + rl64(c.seq_src, j), P.seq + rl64((int64_t)c.seq_dst, j), sn, lane);
      if (qn) wave_copy(P.text + rl64(c.qual_src, j), P.qual + rl64((int64_t)c.qual_dst, j), qn, lane);
      if (mn) wave_copy(P.text + rl64(c.md_src, j), P.md + rl64((int64_t)c.md_dst, j), mn, lane);
    }
  }
}
// the closing offsets (column totals) of the read columns
extern "C" __global__ void sam_offsets_close(SamParams P, int64_t n_reads) {
  const int64_t L1 = P.n_lines + 1;
  P.seq_off[n_reads] = P.off[L1 + P.n_lines];
  P.qual_off[n_reads] = P.off[2 * L1 + P.n_lines];
  P.cig_off[n_reads] = P.off[3 * L1 + P.n_lines];
  P.md_off[n_reads] = P.off[4 * L1 + P.n_lines];
}

// referenceName ids in first-appearance order: the first read of each @SQ name
// (only a lane whose name differs from the previous lane's competes: the
// reads of one reference come in runs, and same-address atomics serialise)
extern "C" __global__ void sam_ref_first(const int32_t* ref, int64_t n, unsigned long long* first) {
  const int lane = threadIdx.x & 63;
  for (int64_t r0 = blockIdx.x * (int64_t)blockDim.x + (threadIdx.x & ~63); r0 < n; r0 += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = r0 + lane;
    const int32_t v = r < n ? ref[r] : -1;
    const int32_t prev = __shfl_up(v, 1);
    if (v >= 0 && (lane == 0 || v != prev)) atomicMin(&first[v], (unsigned long long)r);
  }
}
extern "C" __global__ void sam_ref_remap(int32_t* ref, int64_t n, const int32_t* rank) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x)
    if (ref[r] >= 0) ref[r] = rank[ref[r]];
}

// ---- output: QUAL fields rewritten ----
struct RewriteParams {
  const uint8_t* text;
  const uint64_t* line_span;
  const uint64_t* qual_span;
  const ReadMeta* meta;    // the batch's reads: slot of read r
  const uint8_t* out_qual;
  const uint32_t* out_start;
  const uint32_t* out_len;
  const uint64_t* exc;     // sorted (slot << 16 | char)
  int64_t n_exc;
  int64_t n_reads;
  int64_t header;          // text[0, header) is copied first
  uint64_t* new_len;       // [n_reads] line bytes incl. '\n' (pass 1), scanned to offsets
  uint8_t* out;            // the new text
  const uint64_t* new_off; // [n_reads + 1]
  const uint8_t* pass;     // [n_reads] 1: QUAL passed through (bytes kept)
  uint64_t* span_out;      // [4 n]: the new text's line and QUAL spans (write pass)
  const uint32_t* raw_flag; // FLAG words, and
  const uint32_t* flags;    // the duplicateRead bits MarkDuplicates set: FLAG 0x400 rewritten when non-null
};

// FLAG with 0x400 following duplicateRead, as decimal text; returns its length
__device__ __forceinline__ int flag_text(uint32_t v, uint8_t d[10]) {
  int n = 0;
  uint8_t t[10];
  do {
    t[n++] = (uint8_t)('0' + v % 10u);
    v /= 10u;
  } while (v);
  for (int k = 0; k < n; ++k) d[k] = t[n - 1 - k];
  return n;
}

// the exception list entry of `slot` (sorted by slot): its char above 0xFF
__device__ __forceinline__ bool exc_char(const RewriteParams& P, uint64_t slot, uint32_t* c) {
  int64_t lo = 0, hi = P.n_exc - 1;
  while (lo <= hi) {
    const int64_t mid = (lo + hi) >> 1;
    const uint64_t v = P.exc[mid], s = v >> 16;
    if (s == slot) {
      *c = (uint32_t)(v & 0xFFFFull);
      return true;
    }
    if (s < slot) lo = mid + 1;
    else hi = mid - 1;
  }
  return false;
}
// the recalibrated char at slot: the u8 column, or the exception list for chars above 0xFF
__device__ __forceinline__ uint32_t new_char(const RewriteParams& P, uint64_t slot) {
  uint32_t c = (uint32_t)P.out_qual[slot];
  uint32_t x = 0;
  if (P.n_exc > 0 && exc_char(P, slot, &x)) c = x;
  return c;
}
__device__ __forceinline__ int utf8_len(uint32_t c) { return c < 0x80u ? 1 : (c < 0x800u ? 2 : 3); }

template <bool kWrite>
__device__ void rewrite_read(const RewriteParams& P, int64_t r) {
  const int64_t s = (int64_t)P.line_span[2 * r], e = (int64_t)P.line_span[2 * r + 1];
  const int64_t qa = (int64_t)P.qual_span[2 * r], qb = (int64_t)P.qual_span[2 * r + 1];
  const bool keep = P.out_qual == nullptr || P.pass[r] != 0;
  const uint64_t slot = keep ? 0 : P.meta[r].slot + P.out_start[r];
  const int64_t n = keep ? 0 : P.out_len[r];
  // the FLAG field [fa, fb) and its new text
  int64_t fa = s, fb = s;
  uint8_t ft[10];
  int fn = 0;
  if (P.flags) {
    while (P.text[fa] != '\t') ++fa;
    fb = ++fa;
    while (P.text[fb] != '\t') ++fb;
    const uint32_t f = P.raw_flag[r];
    fn = flag_text((P.flags[r] & BQSR_F_DUPLICATE) ? (f | 0x400u) : (f & ~0x400u), ft);
  }
  if (!kWrite) {
    int64_t q = 0;
    if (keep) q = qb - qa;
    else
      for (int64_t k = 0; k < n; ++k) q += utf8_len(new_char(P, slot + k));
    P.new_len[r] = (uint64_t)((qa - s) - (fb - fa) + fn + q + (e - qb) + 1);
    return;
  }
  uint8_t* const o0 = P.out + P.header + P.new_off[r];
  uint8_t* o = o0;
  for (int64_t k = s; k < fa; ++k) *o++ = P.text[k];
  for (int k = 0; k < fn; ++k) *o++ = ft[k];
  for (int64_t k = fb; k < qa; ++k) *o++ = P.text[k];
  const int64_t nqa = P.header + (int64_t)P.new_off[r] + (o - o0);
  if (keep) {
    for (int64_t k = qa; k < qb; ++k) *o++ = P.text[k];
  } else {
    for (int64_t k = 0; k < n; ++k) {
      const uint32_t c = new_char(P, slot + k);
      if (c < 0x80u) {
        *o++ = (uint8_t)c;
      } else if (c < 0x800u) {
        *o++ = (uint8_t)(0xC0u | (c >> 6));
        *o++ = (uint8_t)(0x80u | (c & 0x3Fu));
      } else {
        *o++ = (uint8_t)(0xE0u | (c >> 12));
        *o++ = (uint8_t)(0x80u | ((c >> 6) & 0x3Fu));
        *o++ = (uint8_t)(0x80u | (c & 0x3Fu));
      }
    }
  }
  const int64_t nqb = P.header + (int64_t)P.new_off[r] + (o - o0);
  for (int64_t k = qb; k < e; ++k) *o++ = P.text[k];
  *o = '\n';
  P.span_out[4 * r] = (uint64_t)(P.header + (int64_t)P.new_off[r]);
  P.span_out[4 * r + 1] = (uint64_t)(P.header + (int64_t)P.new_off[r] + (o - o0));
  P.span_out[4 * r + 2] = (uint64_t)nqa;
  P.span_out[4 * r + 3] = (uint64_t)nqb;
}
extern "C" __global__ void sam_rewrite_len(RewriteParams P) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < P.n_reads; r += (int64_t)gridDim.x * blockDim.x)
    rewrite_read<false>(P, r);
}
extern "C" __global__ void sam_rewrite_write(RewriteParams P) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < P.n_reads; r += (int64_t)gridDim.x * blockDim.x)
    rewrite_read<true>(P, r);
}
extern "C" __global__ void sam_copy_bytes(const uint8_t* src, uint8_t* dst, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}
// pass-through reads: apply marked them kInfoPass
extern "C" __global__ void sam_pass_flags(const ReadInfo* info, int64_t n, uint8_t* pass) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x)
    pass[r] = (info[r].fl & kInfoPass) ? 1 : 0;
}

// the rewrite's spans back into the parse's [2n] line / QUAL span columns
extern "C" __global__ void sam_spans_update(const uint64_t* span_out, int64_t n, uint64_t* line_span,
                                            uint64_t* qual_span) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    line_span[2 * r] = span_out[4 * r];
    line_span[2 * r + 1] = span_out[4 * r + 1];
    qual_span[2 * r] = span_out[4 * r + 2];
    qual_span[2 * r + 1] = span_out[4 * r + 3];
  }
}

}  // namespace samk

// ------------------------------------------------------------ host side ----

struct bqsr_sam {
  bqsr_context* ctx = nullptr;
  uint8_t* d_text = nullptr;
  int64_t n_text = 0;
  int64_t header = 0;  // text[0, header): the header lines
  std::vector<std::string> ref_names;
  int32_t n_rg = 0;
  int64_t n_reads = 0, seq_bytes = 0, qual_bytes = 0, cig_ops = 0, md_bytes = 0;
  uint32_t* flags = nullptr;
  int32_t* rg_id = nullptr;
  int32_t* ref = nullptr;
  int32_t* sq_id = nullptr;     // referenceId: the @SQ header index
  uint32_t* raw_flag = nullptr; // the SAM FLAG word
  std::vector<std::string> rg_library;  // LB of read group id i ("" + rg_has_lb[i] = 0: none)
  std::vector<uint8_t> rg_has_lb;
  int64_t* start = nullptr;
  uint64_t* seq_off = nullptr;
  uint8_t* seq = nullptr;
  uint64_t* qual_off = nullptr;
  uint8_t* qual = nullptr;
  uint64_t* cig_off = nullptr;
  uint32_t* cig = nullptr;
  uint64_t* md_off = nullptr;
  uint8_t* md = nullptr;
  uint64_t* line_span = nullptr;
  uint64_t* qual_span = nullptr;
  bool dup_marked = false;  // bqsr_sam_mark_duplicates ran: FLAG 0x400 rewritten on output
  bool from_bam = false;    // bqsr_bam_parse: d_text holds the records converted to SAM text on the device
  samk::NameTable sq_tab{}, rg_tab{};  // @SQ / @RG name tables on the device (ADAM columns)
  std::string header_text;  // the header lines (host copy)
  void* adam = nullptr;     // ADAM column buffers (adam_out.hip), freed with the handle
  std::vector<void*> allocs;
  ~bqsr_sam();
};

namespace {

// a name table on the device (freed with the returned allocations)
struct HostNames {
  std::vector<uint8_t> blob;
  std::vector<uint64_t> off{0};
  std::vector<int32_t> value;
  std::vector<int32_t> slot;
  uint32_t mask = 0;
  void add(const std::string& n, int32_t v) {
    blob.insert(blob.end(), n.begin(), n.end());
    off.push_back(blob.size());
    value.push_back(v);
  }
  void build() {
    uint32_t cap = 16;
    while (cap < 2 * value.size() + 2) cap <<= 1;
    mask = cap - 1;
    slot.assign(cap, -1);
    for (size_t k = 0; k < value.size(); ++k) {
      uint32_t i = (uint32_t)samk::fnv1a(blob.data() + off[k], (int64_t)(off[k + 1] - off[k])) & mask;
      while (slot[i] >= 0) i = (i + 1) & mask;
      slot[i] = (int32_t)k;
    }
  }
};

template <class T>
bqsr_status sam_alloc(std::vector<void*>& keep, T** p, size_t n) {
  HIP_TRY(hipMalloc((void**)p, std::max<size_t>(n, 1) * sizeof(T)));
  keep.push_back((void*)*p);
  return BQSR_OK;
}
template <class T>
bqsr_status sam_upload(std::vector<void*>& keep, T** p, const std::vector<T>& v, hipStream_t s) {
  bqsr_status st = sam_alloc(keep, p, v.size());
  if (st != BQSR_OK) return st;
  if (!v.empty()) HIP_TRY(hipMemcpyAsync(*p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, s));
  return BQSR_OK;
}
bqsr_status sam_names_upload(std::vector<void*>& keep, const HostNames& h, samk::NameTable* t, hipStream_t s) {
  uint8_t* blob;
  uint64_t* off;
  int32_t *slot, *value;
  bqsr_status st;
  if ((st = sam_upload(keep, &blob, h.blob, s)) != BQSR_OK) return st;
  if ((st = sam_upload(keep, &off, h.off, s)) != BQSR_OK) return st;
  if ((st = sam_upload(keep, &slot, h.slot, s)) != BQSR_OK) return st;
  if ((st = sam_upload(keep, &value, h.value, s)) != BQSR_OK) return st;
  *t = samk::NameTable{blob, off, slot, value, h.mask, (int32_t)h.value.size()};
  return BQSR_OK;
}
// exclusive scan of n u64 into out[0..n]
bqsr_status sam_scan(const uint64_t* in, int64_t n, uint64_t* out, uint64_t* part, hipStream_t s) {
  const int64_t nb = std::max<int64_t>(1, (n + samk::kScanChunk - 1) / samk::kScanChunk);
  hipLaunchKernelGGL(samk::scan_partials, dim3((unsigned)nb), dim3(samk::kScanThreads), 0, s, in, n, part);
  hipLaunchKernelGGL(samk::scan_top, dim3(1), dim3(1024), 0, s, part, nb);
  hipLaunchKernelGGL(samk::scan_apply, dim3((unsigned)nb), dim3(samk::kScanThreads), 0, s, in, n, (const uint64_t*)part,
                     out);
  HIP_TRY(hipGetLastError());
  return BQSR_OK;
}
unsigned sam_grid(int64_t n, int threads, int cap) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + threads - 1) / threads, cap));
}
const char* kSamErrors[] = {"ok", "fewer than 11 fields", "optional field without two ':'", "FLAG is not an integer",
                            "POS is not an integer", "malformed CIGAR", "header line after the first record",
                            "'\\r' inside a line"};

// the SAM header text (SAM input, or a BAM's l_text): @RG IDs sorted into
// the RecordGroupDictionary (RecordGroupDictionary.scala:36-43) with their LB,
// @SQ names -> header index; body = where the records start
struct SamHeader {
  int64_t body = 0;
  std::vector<std::string> rg_names, sq_names;
  std::map<std::string, std::pair<bool, std::string>> rg_lb;
  HostNames rgh, sqh;
};
bqsr_status parse_sam_header(const char* text, int64_t n, SamHeader* H) {
  std::vector<std::string>& rg_names = H->rg_names;
  std::vector<std::string>& sq_names = H->sq_names;
  std::map<std::string, std::pair<bool, std::string>>& rg_lb = H->rg_lb;  // the last @RG line of an ID
  int64_t p = 0;
  while (p < n) {
    const char* nlp = (const char*)memchr(text + p, '\n', (size_t)(n - p));
    const int64_t e0 = nlp ? (int64_t)(nlp - text) : n;
    int64_t e = e0;
    if (e > p && text[e - 1] == '\r') --e;
    if (e == p) {  // empty line
      p = e0 + 1;
      continue;
    }
    if (text[p] != '@') break;
    std::string line(text + p, (size_t)(e - p));
    std::vector<std::string> f;
    size_t a = 0;
    for (;;) {
      const size_t t = line.find('\t', a);
      f.push_back(line.substr(a, t == std::string::npos ? std::string::npos : t - a));
      if (t == std::string::npos) break;
      a = t + 1;
    }
    std::string id, sn, lb;
    bool has_id = false, has_sn = false, has_lb = false;
    for (size_t k = 1; k < f.size(); ++k) {  // dict(t.split(":", 1) for t in f[1:] if ":" in t)
      const size_t c = f[k].find(':');
      if (c == std::string::npos) continue;
      const std::string key = f[k].substr(0, c);
      if (key == "ID") {
        id = f[k].substr(c + 1);
        has_id = true;
      } else if (key == "SN") {
        sn = f[k].substr(c + 1);
        has_sn = true;
      } else if (key == "LB") {
        lb = f[k].substr(c + 1);
        has_lb = true;
      }
    }
    if (f[0] == "@RG") {
      if (!has_id) return fail(BQSR_ERR_SAM_PARSE, "@RG header line without ID");
      rg_names.push_back(id);
      rg_lb[id] = std::make_pair(has_lb, lb);
    } else if (f[0] == "@SQ") {
      if (!has_sn) return fail(BQSR_ERR_SAM_PARSE, "@SQ header line without SN");
      sq_names.push_back(sn);
    }
    p = e0 + 1;
  }
  H->body = std::min(p, n);
  std::sort(rg_names.begin(), rg_names.end());  // readGroupNames.sorted.zipWithIndex (the last duplicate wins)
  HostNames& rgh = H->rgh;
  HostNames& sqh = H->sqh;
  for (size_t i = 0; i < rg_names.size(); ++i) {
    if (i + 1 < rg_names.size() && rg_names[i + 1] == rg_names[i]) continue;
    rgh.add(rg_names[i], (int32_t)i);
  }
  {  // @SQ names -> header index (the first line of a name)
    std::map<std::string, int32_t> seen;
    for (size_t i = 0; i < sq_names.size(); ++i)
      if (seen.emplace(sq_names[i], (int32_t)i).second) sqh.add(sq_names[i], (int32_t)i);
  }
  rgh.build();
  sqh.build();

  return BQSR_OK;
}

}  // namespace

namespace {
// The record parse of a SAM text already on the device (d_text: n bytes +
// 64 readable, owned by the result; the header lines parsed into H, the
// records from H.body): bqsr_sam_parse's text, or bqsr_bam_parse's records
// converted to SAM lines on the device.
bqsr_status sam_parse_device(bqsr_context* ctx, SamHeader& H, const char* header, uint8_t* d_text, int64_t n,
                             hipStream_t s, bool from_bam, bqsr_sam** out) {
  std::unique_ptr<bqsr_sam> S_(new bqsr_sam);
  bqsr_sam* o = S_.get();
  o->d_text = d_text;
  o->from_bam = from_bam;
  const int64_t body = H.body;
  o->header_text.assign(header, (size_t)body);
  std::vector<std::string>& rg_names = H.rg_names;
  std::vector<std::string>& sq_names = H.sq_names;
  std::map<std::string, std::pair<bool, std::string>>& rg_lb = H.rg_lb;
  HostNames& rgh = H.rgh;
  HostNames& sqh = H.sqh;

  o->ctx = ctx;
  o->n_rg = (int32_t)rgh.value.size();
  o->rg_library.assign(rg_names.size(), std::string());
  o->rg_has_lb.assign(rg_names.size(), 0);
  for (size_t i = 0; i < rg_names.size(); ++i) {
    const auto& v = rg_lb[rg_names[i]];
    o->rg_has_lb[i] = v.first ? 1 : 0;
    o->rg_library[i] = v.second;
  }
  o->header = body;
  o->n_text = n;
  std::vector<void*> tmp;  // per-line temporaries
  struct Free {
    std::vector<void*>& v;
    ~Free() {
      for (void* q : v) (void)hipFree(q);
    }
  } free_tmp{tmp};
  samk::SamParams P{};
  P.text = o->d_text;
  P.body = body;
  P.n = n;
  bqsr_status st;
  if ((st = sam_names_upload(o->allocs, sqh, &P.sq, s)) != BQSR_OK) return st;
  if ((st = sam_names_upload(o->allocs, rgh, &P.rg, s)) != BQSR_OK) return st;
  o->sq_tab = P.sq;
  o->rg_tab = P.rg;
  // ---- newline positions ----
  const int64_t nb = std::max<int64_t>(1, (n - body + samk::kNlChunk - 1) / samk::kNlChunk);
  uint64_t* cnt;
  if ((st = sam_alloc(tmp, &cnt, (size_t)nb + 1)) != BQSR_OK) return st;
  hipLaunchKernelGGL(samk::sam_nl_count, dim3((unsigned)nb), dim3(samk::kNlThreads), 0, s, (const uint8_t*)o->d_text,
                     body, n, cnt);
  hipLaunchKernelGGL(samk::scan_top, dim3(1), dim3(1024), 0, s, cnt, nb);
  HIP_TRY(hipGetLastError());
  uint64_t n_nl = 0;
  HIP_TRY(hipMemcpyAsync(&n_nl, cnt + nb, 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  uint64_t* nl;
  if ((st = sam_alloc(tmp, &nl, (size_t)n_nl)) != BQSR_OK) return st;
  hipLaunchKernelGGL(samk::sam_nl_write, dim3((unsigned)nb), dim3(samk::kNlThreads), 0, s, (const uint8_t*)o->d_text,
                     body, n, (const uint64_t*)cnt, nl);
  P.nl = nl;
  P.n_nl = (int64_t)n_nl;
  const int64_t L = n > body ? (int64_t)n_nl + 1 : 0;  // the last "line" may be empty
  P.n_lines = L;
  // ---- pass 1: lengths ----
  unsigned long long* err;
  if ((st = sam_alloc(tmp, &err, 1)) != BQSR_OK) return st;
  HIP_TRY(hipMemsetAsync(err, 0xFF, 8, s));
  P.err = err;
  if ((st = sam_alloc(tmp, &P.len, (size_t)(5 * L))) != BQSR_OK) return st;
  if ((st = sam_alloc(tmp, &P.off, (size_t)(5 * (L + 1)))) != BQSR_OK) return st;
  const unsigned lg = sam_grid(L, 256, ctx->n_cu * 16);  // sam_lines_write: whole wavefronts per stride step
  if (L > 0) hipLaunchKernelGGL(samk::sam_lines_len, dim3(lg), dim3(256), 0, s, P);
  HIP_TRY(hipGetLastError());
  unsigned long long e_word = ~0ull;
  HIP_TRY(hipMemcpyAsync(&e_word, err, 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (e_word != ~0ull) {
    const uint32_t code = (uint32_t)(e_word & 0xFF);
    const int64_t line = (int64_t)(e_word >> 8);
    char buf[160];
    snprintf(buf, sizeof buf, "SAM record line %lld (after the header): %s", (long long)line,
             code < 8 ? kSamErrors[code] : "?");
    return fail(code == samk::kSamHeader || code == samk::kSamCr ? BQSR_ERR_UNSUPPORTED : BQSR_ERR_SAM_PARSE, buf);
  }
  // ---- scans: read ids and column offsets ----
  uint64_t* part;
  if ((st = sam_alloc(tmp, &part, (size_t)(L / samk::kScanChunk + 2))) != BQSR_OK) return st;
  for (int c = 0; c < 5; ++c)
    if ((st = sam_scan(P.len + (size_t)c * L, L, P.off + (size_t)c * (L + 1), part, s)) != BQSR_OK) return st;
  uint64_t tot[5] = {0, 0, 0, 0, 0};
  for (int c = 0; c < 5; ++c)
    HIP_TRY(hipMemcpyAsync(&tot[c], P.off + (size_t)c * (L + 1) + L, 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (L == 0) std::fill(tot, tot + 5, 0ull);
  o->n_reads = (int64_t)tot[0];
  o->seq_bytes = (int64_t)tot[1];
  o->qual_bytes = (int64_t)tot[2];
  o->cig_ops = (int64_t)tot[3];
  o->md_bytes = (int64_t)tot[4];
  const size_t nr = (size_t)o->n_reads;
  if ((st = sam_alloc(o->allocs, &o->flags, nr)) != BQSR_OK) return st;
  if ((st = sam_alloc(o->allocs, &o->rg_id, nr)) != BQSR_OK) return st;
  if ((st = sam_alloc(o->allocs, &o->ref, nr)) != BQSR_OK) return st;
  if ((st = sam_alloc(o->allocs, &o->start, nr)) != BQSR_OK) return st;
  if ((st = sam_alloc(o->allocs, &o->sq_id, nr)) != BQSR_OK) return st;
  if ((st = sam_alloc(o->allocs, &o->raw_flag, nr)) != BQSR_OK) return st;
  if ((st = sam_alloc(o->allocs, &o->seq_off, nr + 1)) != BQSR_OK) return st;
  if ((st = sam_alloc(o->allocs, &o->seq, (size_t)o->seq_bytes)) != BQSR_OK) return st;
  if ((st = sam_alloc(o->allocs, &o->qual_off, nr + 1)) != BQSR_OK) return st;
  if ((st = sam_alloc(o->allocs, &o->qual, (size_t)o->qual_bytes)) != BQSR_OK) return st;
  if ((st = sam_alloc(o->allocs, &o->cig_off, nr + 1)) != BQSR_OK) return st;
  if ((st = sam_alloc(o->allocs, &o->cig, (size_t)o->cig_ops)) != BQSR_OK) return st;
  if ((st = sam_alloc(o->allocs, &o->md_off, nr + 1)) != BQSR_OK) return st;
  if ((st = sam_alloc(o->allocs, &o->md, (size_t)o->md_bytes)) != BQSR_OK) return st;
  if ((st = sam_alloc(o->allocs, &o->line_span, 2 * nr)) != BQSR_OK) return st;
  if ((st = sam_alloc(o->allocs, &o->qual_span, 2 * nr)) != BQSR_OK) return st;
  P.flags = o->flags;
  P.rg_id = o->rg_id;
  P.ref = o->ref;
  P.sq_id = o->sq_id;
  P.raw_flag = o->raw_flag;
  P.start = o->start;
  P.seq_off = o->seq_off;
  P.seq = o->seq;
  P.qual_off = o->qual_off;
  P.qual = o->qual;
  P.cig_off = o->cig_off;
  P.cig = o->cig;
  P.md_off = o->md_off;
  P.md = o->md;
  P.line_span = o->line_span;
  P.qual_span = o->qual_span;
  // ---- pass 2: the columns ----
  if (L > 0) {
    hipLaunchKernelGGL(samk::sam_lines_write, dim3(lg), dim3(256), 0, s, P);
    hipLaunchKernelGGL(samk::sam_offsets_close, dim3(1), dim3(1), 0, s, P, o->n_reads);
  } else {
    HIP_TRY(hipMemsetAsync(o->seq_off, 0, 8, s));
    HIP_TRY(hipMemsetAsync(o->qual_off, 0, 8, s));
    HIP_TRY(hipMemsetAsync(o->cig_off, 0, 8, s));
    HIP_TRY(hipMemsetAsync(o->md_off, 0, 8, s));
  }
  HIP_TRY(hipGetLastError());
  // ---- referenceName ids: first appearance order ----
  const size_t nsq = sq_names.size();
  if (nsq > 0 && nr > 0) {
    unsigned long long* first;
    int32_t* rank_d;
    if ((st = sam_alloc(tmp, &first, nsq)) != BQSR_OK) return st;
    HIP_TRY(hipMemsetAsync(first, 0xFF, nsq * 8, s));
    const unsigned rgd = sam_grid((int64_t)nr, 256, ctx->n_cu * 16);
    hipLaunchKernelGGL(samk::sam_ref_first, dim3(rgd), dim3(256), 0, s, (const int32_t*)o->ref, (int64_t)nr, first);
    std::vector<unsigned long long> fh(nsq);
    HIP_TRY(hipMemcpyAsync(fh.data(), first, nsq * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    std::vector<int32_t> order;
    for (size_t i = 0; i < nsq; ++i)
      if (fh[i] != ~0ull) order.push_back((int32_t)i);
    std::sort(order.begin(), order.end(), [&](int32_t a, int32_t b) { return fh[a] < fh[b]; });
    std::vector<int32_t> rank(nsq, -1);
    for (size_t k = 0; k < order.size(); ++k) {
      rank[order[k]] = (int32_t)k;
      o->ref_names.push_back(sq_names[order[k]]);
    }
    if ((st = sam_upload(tmp, &rank_d, rank, s)) != BQSR_OK) return st;
    hipLaunchKernelGGL(samk::sam_ref_remap, dim3(rgd), dim3(256), 0, s, o->ref, (int64_t)nr, (const int32_t*)rank_d);
    HIP_TRY(hipGetLastError());
  }
  HIP_TRY(hipStreamSynchronize(s));
  *out = S_.release();
  return ok();
}
}  // namespace

bqsr_status bqsr_sam_parse(bqsr_context* ctx, const char* text, int64_t n, void* stream, bqsr_sam** out) {
  if (!ctx || !out || n < 0 || (n > 0 && !text)) return fail(BQSR_ERR_INVALID_ARG, "bqsr_sam_parse: bad arguments");
  HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = S(stream);
  // ---- header (host): @RG IDs sorted (RecordGroupDictionary), @SQ names ----
  SamHeader H;
  bqsr_status hst = parse_sam_header(text, n, &H);
  if (hst != BQSR_OK) return hst;
  uint8_t* d_text = nullptr;
  HIP_TRY(hipMalloc(&d_text, (size_t)n + 64));
  hipError_t e = hipMemsetAsync(d_text + n, 0, 64, s);
  if (e == hipSuccess && n > 0) {
    const bqsr_status ust = upload_staged(ctx, d_text, text, (size_t)n, s);
    if (ust != BQSR_OK) {
      (void)hipFree(d_text);
      return ust;
    }
  }
  if (e != hipSuccess) {
    (void)hipFree(d_text);
    return fail(BQSR_ERR_DEVICE, std::string("bqsr_sam_parse: ") + hipGetErrorString(e));
  }
  return sam_parse_device(ctx, H, text, d_text, n, s, false, out);  // (owns d_text from here)
}

void bqsr_sam_destroy(bqsr_sam* s) { delete s; }

bqsr_status bqsr_sam_get_counts(const bqsr_sam* s, bqsr_sam_counts* out) {
  if (!s || !out) return fail(BQSR_ERR_INVALID_ARG, "null");
  *out = bqsr_sam_counts{s->n_reads, s->seq_bytes, s->qual_bytes, s->cig_ops, s->md_bytes, s->n_text,
                         (int32_t)s->ref_names.size(), s->n_rg};
  return ok();
}

const char* bqsr_sam_ref_name(const bqsr_sam* s, int32_t i) {
  if (!s || i < 0 || i >= (int32_t)s->ref_names.size()) return nullptr;
  return s->ref_names[(size_t)i].c_str();
}

bqsr_status bqsr_sam_device_columns(const bqsr_sam* s, bqsr_sam_columns* o) {
  if (!s || !o) return fail(BQSR_ERR_INVALID_ARG, "null");
  *o = bqsr_sam_columns{s->flags, s->rg_id, s->ref, s->start, s->seq_off, s->seq, s->qual_off, s->qual,
                        s->cig_off, s->cig, s->md_off, s->md};
  return ok();
}

bqsr_status bqsr_sam_download(const bqsr_sam* s, const bqsr_sam_columns* d) {
  if (!s || !d) return fail(BQSR_ERR_INVALID_ARG, "null");
  HIP_TRY(hipSetDevice(s->ctx->device));
  const size_t n = (size_t)s->n_reads;
  auto cp = [&](void* dst, const void* src, size_t bytes) -> hipError_t {
    if (!bytes) return hipSuccess;
    if (!dst) return hipErrorInvalidValue;
    return hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost);
  };
  hipError_t e = cp(d->flags, s->flags, n * 4);
  if (e == hipSuccess) e = cp(d->rg_id, s->rg_id, n * 4);
  if (e == hipSuccess) e = cp(d->ref_index, s->ref, n * 4);
  if (e == hipSuccess) e = cp(d->start, s->start, n * 8);
  if (e == hipSuccess) e = cp(d->seq_offset, s->seq_off, (n + 1) * 8);
  if (e == hipSuccess) e = cp(d->seq, s->seq, (size_t)s->seq_bytes);
  if (e == hipSuccess) e = cp(d->qual_offset, s->qual_off, (n + 1) * 8);
  if (e == hipSuccess) e = cp(d->qual, s->qual, (size_t)s->qual_bytes);
  if (e == hipSuccess) e = cp(d->cigar_offset, s->cig_off, (n + 1) * 8);
  if (e == hipSuccess) e = cp(d->cigar, s->cig, (size_t)s->cig_ops * 4);
  if (e == hipSuccess) e = cp(d->md_offset, s->md_off, (n + 1) * 8);
  if (e == hipSuccess) e = cp(d->md, s->md, (size_t)s->md_bytes);
  if (e != hipSuccess) return fail(BQSR_ERR_DEVICE, std::string("bqsr_sam_download: ") + hipGetErrorString(e));
  return ok();
}

bqsr_status bqsr_sam_rewrite_quals(bqsr_context* ctx, bqsr_sam* sm, const bqsr_batch* b, const uint8_t* out_qual,
                                   const uint32_t* out_start, const uint32_t* out_len, const uint64_t* exceptions,
                                   int64_t n_exc, void* stream) {
  if (!ctx || !sm || (b && (!out_qual || !out_start || !out_len)) || n_exc < 0 || (n_exc > 0 && !exceptions))
    return fail(BQSR_ERR_INVALID_ARG, "bqsr_sam_rewrite_quals: bad arguments");
  if (b && b->rd.n_reads != sm->n_reads) return fail(BQSR_ERR_INVALID_ARG, "batch and SAM read counts differ");
  if (b && !b->prepped) return fail(BQSR_ERR_INVALID_ARG, "the batch has not been through apply");
  if (!b) {  // QUAL fields kept (only FLAG rewritten, after MarkDuplicates)
    out_qual = nullptr;
    n_exc = 0;
  }
  HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = S(stream);
  const int64_t n = sm->n_reads;
  std::vector<void*> tmp;
  struct Free {
    std::vector<void*>& v;
    ~Free() {
      for (void* q : v) (void)hipFree(q);
    }
  } free_tmp{tmp};
  bqsr_status st;
  samk::RewriteParams R{};
  uint8_t* pass;
  uint64_t *new_len, *new_off, *part, *span_out;
  if ((st = sam_alloc(tmp, &pass, (size_t)n)) != BQSR_OK) return st;
  if ((st = sam_alloc(tmp, &new_len, (size_t)n)) != BQSR_OK) return st;
  if ((st = sam_alloc(tmp, &new_off, (size_t)n + 1)) != BQSR_OK) return st;
  if ((st = sam_alloc(tmp, &part, (size_t)(n / samk::kScanChunk + 2))) != BQSR_OK) return st;
  if ((st = sam_alloc(tmp, &span_out, (size_t)(4 * n))) != BQSR_OK) return st;
  uint64_t* exc_sorted = nullptr;
  if (n_exc > 0) {  // the exception list in slot order (binary search)
    std::vector<uint64_t> h((size_t)n_exc);
    HIP_TRY(hipMemcpyAsync(h.data(), exceptions, (size_t)n_exc * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    std::sort(h.begin(), h.end());
    if ((st = sam_upload(tmp, &exc_sorted, h, s)) != BQSR_OK) return st;
  }
  const unsigned g = sam_grid(n, 256, ctx->n_cu * 16);
  if (n > 0 && b)
    hipLaunchKernelGGL(samk::sam_pass_flags, dim3(g), dim3(256), 0, s, (const ReadInfo*)b->d_info, n, pass);
  R.text = sm->d_text;
  R.line_span = sm->line_span;
  R.qual_span = sm->qual_span;
  R.meta = b ? b->rd.meta : nullptr;
  R.raw_flag = sm->raw_flag;
  R.flags = sm->dup_marked ? sm->flags : nullptr;
  R.out_qual = out_qual;
  R.out_start = out_start;
  R.out_len = out_len;
  R.exc = exc_sorted;
  R.n_exc = n_exc;
  R.n_reads = n;
  R.header = sm->header;
  R.new_len = new_len;
  R.new_off = new_off;
  R.pass = pass;
  R.span_out = span_out;
  if (n > 0) hipLaunchKernelGGL(samk::sam_rewrite_len, dim3(g), dim3(256), 0, s, R);
  if ((st = sam_scan(new_len, n, new_off, part, s)) != BQSR_OK) return st;
  uint64_t body = 0;
  if (n > 0) HIP_TRY(hipMemcpyAsync(&body, new_off + n, 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  const int64_t total = sm->header + (int64_t)body;
  uint8_t* nt = nullptr;
  HIP_TRY(hipMalloc(&nt, (size_t)total + 64));
  HIP_TRY(hipMemsetAsync(nt + total, 0, 64, s));
  if (sm->header > 0) HIP_TRY(hipMemcpyAsync(nt, sm->d_text, (size_t)sm->header, hipMemcpyDeviceToDevice, s));
  R.out = nt;
  if (n > 0) {
    hipLaunchKernelGGL(samk::sam_rewrite_write, dim3(g), dim3(256), 0, s, R);
    hipLaunchKernelGGL(samk::sam_spans_update, dim3(g), dim3(256), 0, s, (const uint64_t*)span_out, n,
                       sm->line_span, sm->qual_span);
  }
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) {
    (void)hipFree(nt);
    return fail(BQSR_ERR_DEVICE, std::string("bqsr_sam_rewrite_quals: ") + hipGetErrorString(e));
  }
  (void)hipFree(sm->d_text);
  sm->d_text = nt;
  sm->n_text = total;
  return ok();
}

bqsr_status bqsr_sam_text_download(const bqsr_sam* s, char* dst) {
  if (!s || (!dst && s->n_text > 0)) return fail(BQSR_ERR_INVALID_ARG, "null");
  HIP_TRY(hipSetDevice(s->ctx->device));
  if (s->n_text > 0) HIP_TRY(hipMemcpy(dst, s->d_text, (size_t)s->n_text, hipMemcpyDeviceToHost));
  return ok();
}
