// Diagnostic: print the lane mapping of v_permlane32_swap / v_permlane16_swap / DPP row ops.
#include <hip/hip_runtime.h>
#include <cstdio>
template <int CTRL> __device__ float dpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
__global__ void k(float* out) {
  int l = threadIdx.x;
  float x = l, y = 100 + l;
  auto r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, x), __builtin_bit_cast(unsigned, y), false, false);
  out[0 * 64 + l] = __builtin_bit_cast(float, r[0]);
  out[1 * 64 + l] = __builtin_bit_cast(float, r[1]);
  auto s = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, x), __builtin_bit_cast(unsigned, y), false, false);
  out[2 * 64 + l] = __builtin_bit_cast(float, s[0]);
  out[3 * 64 + l] = __builtin_bit_cast(float, s[1]);
  out[4 * 64 + l] = dpp<0x140>(x);
  out[5 * 64 + l] = dpp<0x141>(x);
  out[6 * 64 + l] = dpp<0x4E>(x);
  out[7 * 64 + l] = dpp<0xB1>(x);
}
int main() {
  float* d; hipMalloc(&d, 8 * 64 * 4);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  float h[8 * 64]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  const char* names[8] = {"swap32 r0", "swap32 r1", "swap16 r0", "swap16 r1", "row_mirror", "row_half_mirror", "quad 2301", "quad 1032"};
  for (int t = 0; t < 8; ++t) { printf("%s:", names[t]); for (int l = 0; l < 64; ++l) printf(" %g", h[t * 64 + l]); printf("\n"); }
  return 0;
}
