// Probe: verify the gfx950 lane layout of v_mfma_i32_16x16x64_i8 with exact integer data.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
typedef int v4i __attribute__((ext_vector_type(4)));

__global__ void k(const int8_t* A, const int8_t* B, int* D) {
  int l = threadIdx.x;
  int8_t a[16], b[16];
  for (int j = 0; j < 16; ++j) {
    a[j] = A[(l & 15) * 64 + 16 * (l >> 4) + j];   // A[m][k]
    b[j] = B[(16 * (l >> 4) + j) * 16 + (l & 15)];  // B[k][n]
  }
  v4i av, bv;
  __builtin_memcpy(&av, a, 16);
  __builtin_memcpy(&bv, b, 16);
  v4i c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bv, c, 0, 0, 0);
  for (int i = 0; i < 4; ++i) D[(4 * (l >> 4) + i) * 16 + (l & 15)] = c[i];
}

int main() {
  int8_t hA[16 * 64], hB[64 * 16];
  for (int i = 0; i < 16 * 64; ++i) hA[i] = (int8_t)((i * 37 + 11) % 255 - 127);
  for (int i = 0; i < 64 * 16; ++i) hB[i] = (int8_t)((i * 53 + 7) % 255 - 127);
  int8_t *dA, *dB; int* dD;
  hipMalloc(&dA, sizeof hA); hipMalloc(&dB, sizeof hB); hipMalloc(&dD, 256 * 4);
  hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
  hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
  k<<<1, 64>>>(dA, dB, dD);
  int hD[256];
  hipMemcpy(hD, dD, sizeof hD, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int m = 0; m < 16; ++m)
    for (int n = 0; n < 16; ++n) {
      int ref = 0;
      for (int kk = 0; kk < 64; ++kk) ref += hA[m * 64 + kk] * hB[kk * 16 + n];
      if (ref != hD[m * 16 + n]) ++bad;
    }
  printf("mfma_i32_16x16x64_i8 layout mismatches: %d / 256\n", bad);
  hipDeviceProp_t p; hipGetDeviceProperties(&p, 0);
  printf("device %s CUs %d l2 %d\n", p.gcnArchName, p.multiProcessorCount, p.l2CacheSize);
  return bad != 0;
}
