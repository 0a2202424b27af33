// Probe: do 16-B global loads/stores at byte-unaligned addresses return the
// bytes a byte-wise copy does on this device?  (tools/probe; not product code)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
__global__ void ld(const uint8_t* src, uint8_t* dst, int n) {
  int i = threadIdx.x;
  if (i < n) {
    uint4 v = *(const uint4*)(src + 1 + 3 * i);
    *(uint4*)(dst + 16 * i) = v;
    uint4 w = *(const uint4*)(src + 16 * i);
    *(uint4*)(dst + 4096 + 7 + 17 * i) = w;   // unaligned store
    uint2 x = *(const uint2*)(src + 5 + 9 * i);
    *(uint2*)(dst + 8192 + 8 * i) = x;
  }
}
int main() {
  uint8_t h[16384], o[16384];
  for (int i = 0; i < 16384; ++i) h[i] = (uint8_t)(i * 131 + 7);
  uint8_t *s, *d;
  hipMalloc(&s, 16384); hipMalloc(&d, 16384);
  hipMemcpy(s, h, 16384, hipMemcpyHostToDevice);
  hipMemset(d, 0, 16384);
  hipLaunchKernelGGL(ld, 1, 64, 0, 0, s, d, 64);
  if (hipDeviceSynchronize() != hipSuccess) { printf("FAULT\n"); return 2; }
  hipMemcpy(o, d, 16384, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 64; ++i) for (int j = 0; j < 16; ++j) {
    bad += o[16 * i + j] != h[1 + 3 * i + j];
  }
  for (int i = 0; i < 64; ++i) for (int j = 0; j < 16; ++j) bad += o[4096 + 7 + 17 * i + j] != h[16 * i + j];
  for (int i = 0; i < 64; ++i) for (int j = 0; j < 8; ++j) bad += o[8192 + 8 * i + j] != h[5 + 9 * i + j];
  printf("unaligned probe: %s (%d bad bytes)\n", bad ? "MISMATCH" : "OK", bad);
  return bad ? 1 : 0;
}
