// PCIe link probe (cfg5 planning): H2D / D2H rates between pinned host memory
// and HBM, alone and at once, by DMA copies (hipMemcpyAsync on two streams) and
// by kernels that read or write host memory directly (mapped pinned memory).
// Build: hipcc --offload-arch=gfx950 -O2 tools/link_probe.hip -o tools/link_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                    \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

// 16-B vector copy, grid-stride (either side may be mapped host memory)
__global__ void copy16(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const size_t bytes = (size_t)(argc > 1 ? atof(argv[1]) : 2.0) * (1ull << 30);
  const size_t n16 = bytes / 16;
  void *h_up, *h_dn, *d_up, *d_dn;
  CK(hipHostMalloc(&h_up, bytes, hipHostMallocMapped));
  CK(hipHostMalloc(&h_dn, bytes, hipHostMallocMapped));
  CK(hipMalloc(&d_up, bytes));
  CK(hipMalloc(&d_dn, bytes));
  CK(hipMemset(d_dn, 2, bytes));
  for (size_t i = 0; i < bytes; i += 4096) ((char*)h_up)[i] = 1;
  void *m_up, *m_dn;  // device views of the pinned buffers
  CK(hipHostGetDevicePointer(&m_up, h_up, 0));
  CK(hipHostGetDevicePointer(&m_dn, h_dn, 0));
  hipStream_t a, b;
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  const unsigned grid = (unsigned)ncu * 4;
  auto run = [&](const char* name, int up, int dn) {  // up/dn: 0 none, 1 DMA, 2 kernel
    double best = 1e30;
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipDeviceSynchronize());
      const double t0 = now();
      if (up == 1) CK(hipMemcpyAsync(d_up, h_up, bytes, hipMemcpyHostToDevice, a));
      if (up == 2) hipLaunchKernelGGL(copy16, dim3(grid), dim3(256), 0, a, (const uint4*)m_up, (uint4*)d_up, n16);
      if (dn == 1) CK(hipMemcpyAsync(h_dn, d_dn, bytes, hipMemcpyDeviceToHost, b));
      if (dn == 2) hipLaunchKernelGGL(copy16, dim3(grid), dim3(256), 0, b, (const uint4*)d_dn, (uint4*)m_dn, n16);
      CK(hipDeviceSynchronize());
      const double t = now() - t0;
      if (t < best) best = t;
    }
    const double moved = (double)bytes * ((up ? 1 : 0) + (dn ? 1 : 0));
    printf("{\"case\": \"%s\", \"seconds\": %.4f, \"GBps_total\": %.1f}\n", name, best, moved / best / 1e9);
    fflush(stdout);
  };
  run("h2d_dma", 1, 0);
  run("d2h_dma", 0, 1);
  run("both_dma", 1, 1);
  run("h2d_kernel", 2, 0);
  run("d2h_kernel", 0, 2);
  run("h2d_dma+d2h_kernel", 1, 2);
  run("h2d_kernel+d2h_dma", 2, 1);
  run("both_kernel", 2, 2);
  return 0;
}
