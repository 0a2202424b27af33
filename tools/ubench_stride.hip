// Microbenchmark: what the lane-per-read load pattern of bqsr_observe_lean costs
// against the same bytes read contiguously across a wavefront.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_stride.hip -o tools/ubench_stride
// Reads of R bytes (112: a 100-bp read in 16-aligned slots) laid end to end;
// one 1024-thread workgroup per CU with 160 KB of LDS (the observe kernel's
// occupancy: 16 waves per CU); each wave takes 64 reads per step.
//   lane : lane l loads chunk i of read l (16 B at read_l + 16 i), i < R / 16
//   coal : lane l loads 16 B at wave_base + 16 (l + 64 i) (same bytes, contiguous)
//   lane3: lane l loads 12 B pieces (dwordx3) of a read's half-size code column
// Prints useful GB/s per form.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int kMode, int kCh>
__global__ void __launch_bounds__(1024) walk(const uint8_t* __restrict__ buf, int64_t n_reads, int rbytes, uint32_t* out) {
  extern __shared__ uint32_t lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t acc = 0;
  for (int64_t g0 = ((int64_t)blockIdx.x * 16 + wave) * 64; g0 < n_reads; g0 += (int64_t)gridDim.x * 16 * 64) {
    uint4 v[kCh];
    if (kMode == 0) {
      const uint8_t* p = buf + (g0 + lane) * rbytes;
#pragma unroll
      for (int i = 0; i < kCh; ++i) v[i] = *(const uint4*)(p + 16 * i);
    } else if (kMode == 1) {
      const uint8_t* p = buf + g0 * rbytes;
#pragma unroll
      for (int i = 0; i < kCh; ++i) v[i] = *(const uint4*)(p + 16 * (lane + 64 * i));
    } else {
      const uint8_t* p = buf + (g0 + lane) * (rbytes / 2);
#pragma unroll
      for (int i = 0; i < kCh; ++i) {
        const uint3 c = *(const uint3*)(p + 8 * i);
        v[i] = make_uint4(c.x, c.y, c.z, 0);
      }
    }
#pragma unroll
    for (int i = 0; i < kCh; ++i) acc ^= v[i].x + v[i].y * 3u + v[i].z * 5u + v[i].w * 7u;
  }
  if (acc == 0x12345678u) lds[threadIdx.x] = acc;  // (never: keeps the LDS request)
  out[blockIdx.x * 1024 + threadIdx.x] = acc;
}

int main() {
  const int rbytes = 112, kCh = 7;
  const int64_t n_reads = 10000000;
  const size_t bytes = (size_t)n_reads * rbytes + 4096;
  uint8_t* buf;
  uint32_t* out;
  CK(hipMalloc(&buf, bytes));
  CK(hipMemset(buf, 1, bytes));
  int dev = 0, n_cu = 0;
  CK(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
  CK(hipMalloc(&out, (size_t)n_cu * 1024 * 4));
  const size_t lds = 160 * 1024;
  CK(hipFuncSetAttribute((const void*)walk<0, kCh>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  CK(hipFuncSetAttribute((const void*)walk<1, kCh>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  CK(hipFuncSetAttribute((const void*)walk<2, kCh>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const char* names[3] = {"lane (16 B per lane, 112 B stride)", "coal (16 B per lane, contiguous)", "lane3 (12 B per lane, 56 B stride)"};
  for (int mode = 0; mode < 3; ++mode) {
    for (int rep = 0; rep < 4; ++rep) {
      CK(hipEventRecord(a, 0));
      for (int it = 0; it < 10; ++it) {
        if (mode == 0) hipLaunchKernelGGL((walk<0, kCh>), dim3(n_cu), dim3(1024), lds, 0, buf, n_reads, rbytes, out);
        if (mode == 1) hipLaunchKernelGGL((walk<1, kCh>), dim3(n_cu), dim3(1024), lds, 0, buf, n_reads, rbytes, out);
        if (mode == 2) hipLaunchKernelGGL((walk<2, kCh>), dim3(n_cu), dim3(1024), lds, 0, buf, n_reads, rbytes, out);
      }
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      const double useful = (double)n_reads * (mode == 2 ? kCh * 12 : kCh * 16);
      if (rep > 0) printf("%-40s %8.1f us/launch  %7.1f GB/s useful\n", names[mode], ms * 100.0, useful / (ms / 10 * 1e-3) / 1e9);
    }
  }
  return 0;
}
