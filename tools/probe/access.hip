// Access-pattern probe (tools/probe, not part of the library): how fast can a
// wavefront read a 1 GB byte column of 100-byte records
//   A  coalesced: lane l reads bytes [16 l + 1024 i, +16) of a wave's span
//   B  lane per record: lane l walks its own record in 16-B loads, 4 loads in
//      flight (the observe/apply super-chunk pattern), records in order
//   C  as B, records visited through a random permutation (bucketed order)
//   D  8 lanes per record: lane l reads bytes 16 (l & 7) .. of record l >> 3
//   E  D through the permutation
//   F  lane per record, copy (16-B loads and stores, the apply pattern)
//   G  8 lanes per record, copy
//   H  G through the permutation
// Build: hipcc --offload-arch=gfx950 -O3 access.hip -o access
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));          \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

constexpr int kRec = 100;

__global__ void __launch_bounds__(1024) coalesced(const uint4* p, int64_t n16, uint32_t* out) {
  uint32_t acc = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n16; i += (int64_t)gridDim.x * blockDim.x) {
    const uint4 v = p[i];
    acc ^= v.x + v.y + v.z + v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

template <bool kPerm>
__global__ void __launch_bounds__(1024) per_record(const uint8_t* p, const uint32_t* perm, int64_t n_rec,
                                                   uint32_t* out) {
  uint32_t acc = 0;
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n_rec; r += (int64_t)gridDim.x * blockDim.x) {
    const int64_t rr = kPerm ? (int64_t)perm[r] : r;
    const uint8_t* q = p + rr * kRec;
    for (int j0 = 0; j0 < kRec; j0 += 64) {
      uint4 v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = (j0 + 16 * i < kRec) ? *(const uint4*)(q + j0 + 16 * i) : make_uint4(0, 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 4; ++i) acc ^= v[i].x + v[i].y + v[i].z + v[i].w;
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ void __launch_bounds__(1024) eight_lanes(const uint8_t* p, int64_t n_rec, uint32_t* out) {
  uint32_t acc = 0;
  const int sub = threadIdx.x & 7;
  for (int64_t r = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 3; r < n_rec;
       r += ((int64_t)gridDim.x * blockDim.x) >> 3) {
    const uint8_t* q = p + r * kRec;
    const uint4 v = (16 * sub < kRec) ? *(const uint4*)(q + 16 * sub) : make_uint4(0, 0, 0, 0);
    acc ^= v.x + v.y + v.z + v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

template <bool kPerm>
__global__ void __launch_bounds__(1024) eight_lanes_p(const uint8_t* p, const uint32_t* perm, int64_t n_rec,
                                                      uint32_t* out) {
  uint32_t acc = 0;
  const int sub = threadIdx.x & 7;
  for (int64_t r = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 3; r < n_rec;
       r += ((int64_t)gridDim.x * blockDim.x) >> 3) {
    const int64_t rr = kPerm ? (int64_t)perm[r] : r;
    const uint8_t* q = p + rr * kRec;
    const uint4 v = (16 * sub < kRec) ? *(const uint4*)(q + 16 * sub) : make_uint4(0, 0, 0, 0);
    acc ^= v.x + v.y + v.z + v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ void __launch_bounds__(1024) copy_lane(const uint8_t* p, uint8_t* o, int64_t n_rec) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n_rec; r += (int64_t)gridDim.x * blockDim.x) {
    const uint8_t* q = p + r * kRec;
    uint8_t* d = o + r * kRec;
    for (int j0 = 0; j0 < kRec; j0 += 64) {
      uint4 v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = (j0 + 16 * i < kRec) ? *(const uint4*)(q + j0 + 16 * i) : make_uint4(0, 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int j = j0 + 16 * i;
        if (j + 16 <= kRec) {
          uint4 w = v[i];
          w.x += 1;
          *(uint4*)(d + j) = w;
        } else if (j < kRec) {
          for (int k = 0; k < kRec - j; ++k) d[j + k] = (uint8_t)(v[i].x >> (8 * (k & 3)));
        }
      }
    }
  }
}

template <bool kPerm>
__global__ void __launch_bounds__(1024) copy_eight(const uint8_t* p, uint8_t* o, const uint32_t* perm, int64_t n_rec) {
  const int sub = threadIdx.x & 7;
  for (int64_t r = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 3; r < n_rec;
       r += ((int64_t)gridDim.x * blockDim.x) >> 3) {
    const int64_t rr = kPerm ? (int64_t)perm[r] : r;
    const uint8_t* q = p + rr * kRec;
    uint8_t* d = o + rr * kRec;
    const int j = 16 * sub;
    if (j + 16 <= kRec) {
      uint4 w = *(const uint4*)(q + j);
      w.x += 1;
      *(uint4*)(d + j) = w;
    } else if (j < kRec) {
      const uint4 w = *(const uint4*)(q + j);
      for (int k = 0; k < kRec - j; ++k) d[j + k] = (uint8_t)(w.x >> (8 * (k & 3)));
    }
  }
}

// I: plain coalesced copy (16 B per lane, a wavefront's 1 KB contiguous)
__global__ void __launch_bounds__(1024) copy_coalesced(const uint4* p, uint4* o, int64_t n16) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n16; i += (int64_t)gridDim.x * blockDim.x) {
    uint4 w = p[i];
    w.x += 1;
    o[i] = w;
  }
}

// J: the apply kernel's store pattern: 112-B (16-aligned) records, 2 lanes per
// record, each lane four 16-B chunks of its 64-B piece
constexpr int kRec2 = 112;
__global__ void __launch_bounds__(1024) copy_two(const uint8_t* p, uint8_t* o, int64_t n_rec) {
  const int sub = threadIdx.x & 1;
  for (int64_t r = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 1; r < n_rec;
       r += ((int64_t)gridDim.x * blockDim.x) >> 1) {
    const uint8_t* q = p + r * kRec2 + 64 * sub;
    uint8_t* d = o + r * kRec2 + 64 * sub;
    uint4 v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = (64 * sub + 16 * i < kRec2) ? *(const uint4*)(q + 16 * i) : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (64 * sub + 16 * i < kRec2) {
        v[i].x += 1;
        *(uint4*)(d + 16 * i) = v[i];
      }
  }
}

// K: as J, but the wavefront's 32 records (3584 contiguous bytes) leave
// through LDS as coalesced 16-B-per-lane stores
__global__ void __launch_bounds__(1024) copy_two_lds(const uint8_t* p, uint8_t* o, int64_t n_rec) {
  __shared__ __align__(16) uint8_t st[16][32 * kRec2];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, sub = lane & 1, rl = lane >> 1;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t w0 = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6; w0 * 32 < n_rec; w0 += nw) {
    const int64_t r = w0 * 32 + rl;
    const int nrec = (int)(n_rec - w0 * 32 < 32 ? n_rec - w0 * 32 : 32);
    if (rl < nrec) {
      const uint8_t* q = p + r * kRec2 + 64 * sub;
      uint4 v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = (64 * sub + 16 * i < kRec2) ? *(const uint4*)(q + 16 * i) : make_uint4(0, 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (64 * sub + 16 * i < kRec2) {
          v[i].x += 1;
          *(uint4*)&st[wave][rl * kRec2 + 64 * sub + 16 * i] = v[i];
        }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    uint8_t* d = o + w0 * 32 * kRec2;
    const int nb = nrec * kRec2;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int off = 16 * (lane + 64 * k);
      if (off < nb) *(uint4*)(d + off) = *(const uint4*)&st[wave][off];
    }
    __builtin_amdgcn_wave_barrier();
  }
}

int main() {
  const int64_t n_rec = 10'000'000;
  const int64_t bytes = n_rec * kRec;
  uint8_t *d, *o;
  uint32_t *out, *perm;
  CK(hipMalloc(&d, bytes + 64));
  CK(hipMalloc(&o, bytes + 64));
  CK(hipMalloc(&out, 4));
  CK(hipMalloc(&perm, n_rec * 4));
  CK(hipMemset(d, 1, bytes + 64));
  std::vector<uint32_t> h(n_rec);
  std::iota(h.begin(), h.end(), 0u);
  std::shuffle(h.begin(), h.end(), std::mt19937(1));
  CK(hipMemcpy(perm, h.data(), n_rec * 4, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto time = [&](const char* name, auto launch) {
    for (int i = 0; i < 3; ++i) launch();
    CK(hipEventRecord(a));
    const int reps = 20;
    for (int i = 0; i < reps; ++i) launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= reps;
    printf("%-28s %8.3f ms  %7.1f GB/s\n", name, ms, bytes / (ms * 1e-3) / 1e9);
  };
  const int grid = 256 * 2;
  time("A coalesced 16B/lane", [&] { hipLaunchKernelGGL(coalesced, dim3(grid), dim3(1024), 0, 0, (const uint4*)d, bytes / 16, out); });
  time("B lane/record, in order", [&] { hipLaunchKernelGGL(per_record<false>, dim3(grid), dim3(1024), 0, 0, d, perm, n_rec, out); });
  time("C lane/record, permuted", [&] { hipLaunchKernelGGL(per_record<true>, dim3(grid), dim3(1024), 0, 0, d, perm, n_rec, out); });
  time("D 8 lanes/record", [&] { hipLaunchKernelGGL(eight_lanes, dim3(grid), dim3(1024), 0, 0, d, n_rec, out); });
  time("E 8 lanes/record, permuted", [&] { hipLaunchKernelGGL(eight_lanes_p<true>, dim3(grid), dim3(1024), 0, 0, d, perm, n_rec, out); });
  time("F copy lane/record (x2 B)", [&] { hipLaunchKernelGGL(copy_lane, dim3(grid), dim3(1024), 0, 0, d, o, n_rec); });
  time("G copy 8 lanes/rec (x2 B)", [&] { hipLaunchKernelGGL(copy_eight<false>, dim3(grid), dim3(1024), 0, 0, d, o, perm, n_rec); });
  time("H copy 8 lanes/rec perm (x2)", [&] { hipLaunchKernelGGL(copy_eight<true>, dim3(grid), dim3(1024), 0, 0, d, o, perm, n_rec); });
  const int64_t n_rec2 = bytes / kRec2;
  time("I copy coalesced (x2 B)", [&] { hipLaunchKernelGGL(copy_coalesced, dim3(grid), dim3(1024), 0, 0, (const uint4*)d, (uint4*)o, bytes / 16); });
  time("J copy 2 lanes/112B rec (x2)", [&] { hipLaunchKernelGGL(copy_two, dim3(grid), dim3(1024), 0, 0, d, o, n_rec2); });
  time("K as J, LDS-staged stores (x2)", [&] { hipLaunchKernelGGL(copy_two_lds, dim3(grid), dim3(1024), 0, 0, d, o, n_rec2); });
  CK(hipGetLastError());
  return 0;
}
