#include <hip/hip_runtime.h>
#include <cstdio>
typedef int v2i __attribute__((ext_vector_type(2)));
__global__ void k(unsigned char* out, int mode) {
  __shared__ unsigned char buf[2048];
  const int l = threadIdx.x;
  for (int i = l; i < 2048; i += 64) buf[i] = (unsigned char)(i & 0xFF);
  __syncthreads();
  // mode 0: lane L supplies address 8*L (lanes >= 32 wrap into 0..255 + 256) -> values = addr & 255
  int addr = 8 * l;
  v2i r = __builtin_amdgcn_ds_read_tr8_b64_v2i32((__attribute__((address_space(3))) v2i*)(buf + addr));
  *(v2i*)(out + 8 * l) = r;
}
int main() {
  unsigned char* d; hipMalloc(&d, 512);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, 0);
  unsigned char h[512]; hipMemcpy(h, d, 512, hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; ++l) { printf("lane %2d:", l); for (int j = 0; j < 8; ++j) printf(" %3d", h[8*l+j]); printf("\n"); }
  return 0;
}
