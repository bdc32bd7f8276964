// Probe of ds_read_b64_tr_b16's lane map on integer data: LDS holds a [64][16] matrix of 16-bit
// values 16*row + col; lane l of group g (q = (l&15)>>2, c4 = l&3) points at row 4g + q, columns
// 4*c4 .. +3. Prints what every lane received.   hipcc --offload-arch=gfx950 -O2 tools/tr_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
typedef short s16x4 __attribute__((ext_vector_type(4)));
__global__ void probe(short* out) {
  __shared__ __attribute__((aligned(16))) short m[64 * 16];
  for (int i = threadIdx.x; i < 64 * 16; i += 64) m[i] = (short)i;
  __syncthreads();
  const int l = threadIdx.x, g = l >> 4, q = (l & 15) >> 2, c4 = l & 3;
  const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(m + (4 * g + q) * 16 + 4 * c4));
  for (int e = 0; e < 4; ++e) out[l * 4 + e] = v[e];
}
int main() {
  short* d;
  short h[256];
  if (hipMalloc(&d, 512) != hipSuccess) return 1;
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
  if (hipMemcpy(h, d, 512, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  int bad = 0;
  for (int l = 0; l < 64; ++l) {
    const int g = l >> 4, i = l & 15;
    printf("lane %2d:", l);
    for (int e = 0; e < 4; ++e) {
      printf(" %4d", h[l * 4 + e]);
      bad += h[l * 4 + e] != (4 * g + e) * 16 + i;
    }
    printf("\n");
  }
  printf("mismatches vs (row 4g+e, col lane&15): %d\n", bad);
  return 0;
}
