// Loss terms of the reference training step, evaluated on the rendered views
// (scripts/training/train_script.py:30-36 get_iou_loss, :128-130 img_loss).
//
// One streaming pass: every workgroup reduces a fixed pixel range of one view into four
// sums {I = sum a m, U = sum (a + m - a m), M = sum m, S = sum_k |t_k - rgb_k|} (per-lane
// fp32, then a fixed-order wave/LDS tree), and a one-workgroup finaliser adds the
// workgroup partials in index order and forms the two losses.  Fixed order throughout, so
// the loss is bitwise reproducible.  HBM-bound: 32 B per pixel (rgb 12, alpha 4, target 12,
// mask 4).  The cotangents of these losses are generated inside the raster backward
// (raster.hip, gsr3d_raster_bwd_loss) from the sums written here.
#include "gsr_common.h"

namespace gsr {

constexpr int kLossThreads = 256;
constexpr int kLossBlocksPerView = 96;   // 6 views -> 576 workgroups over 256 CUs

__global__ __launch_bounds__(kLossThreads) void k_loss_partials(
    const float* __restrict__ rgb, const float* __restrict__ alpha, const float* __restrict__ timg,
    const float* __restrict__ tmask, int64_t HW, float4* __restrict__ part) {
  const int c = blockIdx.y;
  const int64_t per = (HW + gridDim.x - 1) / gridDim.x;
  const int64_t p0 = (int64_t)blockIdx.x * per;
  const int64_t p1 = p0 + per < HW ? p0 + per : HW;
  const float* a_v = alpha + c * HW;
  const float* m_v = tmask + c * HW;
  const float* r_v = rgb + c * HW * 3;
  const float* t_v = timg + c * HW * 3;
  float I = 0.f, U = 0.f, M = 0.f, S = 0.f;
  for (int64_t p = p0 + threadIdx.x; p < p1; p += kLossThreads) {
    const float a = a_v[p], m = m_v[p];
    const float am = a * m;
    I += am;
    U += a + m - am;
    M += m;
    S += fabsf(t_v[p] - r_v[p * 3 + 0]) + fabsf(t_v[HW + p] - r_v[p * 3 + 1]) +
         fabsf(t_v[2 * HW + p] - r_v[p * 3 + 2]);
  }
  I = wave_sum(I);
  U = wave_sum(U);
  M = wave_sum(M);
  S = wave_sum(S);
  __shared__ float4 s_w[kLossThreads / 64];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) s_w[w] = make_float4(I, U, M, S);
  __syncthreads();
  if (threadIdx.x == 0) {
    float4 r = s_w[0];
#pragma unroll
    for (int k = 1; k < kLossThreads / 64; ++k) {
      r.x += s_w[k].x;
      r.y += s_w[k].y;
      r.z += s_w[k].z;
      r.w += s_w[k].w;
    }
    part[(int64_t)c * gridDim.x + blockIdx.x] = r;
  }
}

// One workgroup: lane t < 4C sums component (t&3) of view t>>2 over its partials in order.
__global__ __launch_bounds__(kLossThreads) void k_loss_finalize(const float4* __restrict__ part, int C, int B,
                                                                float img_lambda, float* __restrict__ sums,
                                                                float* __restrict__ iou_loss,
                                                                float* __restrict__ img_loss) {
  for (int t = threadIdx.x; t < 4 * C; t += kLossThreads) {
    const int c = t >> 2, k = t & 3;
    const float* pc = (const float*)(part + (int64_t)c * B) + k;
    float v = 0.f;
    for (int b = 0; b < B; ++b) v += pc[4 * b];
    sums[t] = v;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float iou = 0.f, M = 0.f, S = 0.f;
    for (int c = 0; c < C; ++c) {
      iou += (sums[4 * c + 0] + 1e-6f) / (sums[4 * c + 1] + 1e-6f);
      M += sums[4 * c + 2];
      S += sums[4 * c + 3];
    }
    sums[4 * C + 0] = 0.f;
    sums[4 * C + 1] = 0.f;
    sums[4 * C + 2] = M;
    sums[4 * C + 3] = S;
    *iou_loss = 1.f - iou / (float)C;
    *img_loss = img_lambda * S / M;
  }
}

}  // namespace gsr

using namespace gsr;

extern "C" {

size_t gsr_loss_workspace(int C, int width, int height) {
  (void)width;
  (void)height;
  return (size_t)(C > 0 ? C : 0) * kLossBlocksPerView * sizeof(float4);
}

int gsr_loss_iou_l1_fwd(const float* rgb, const float* alpha, const float* target_img, const float* target_mask,
                        int C, int width, int height, float img_lambda, void* ws, size_t ws_bytes, float* sums,
                        float* iou_loss, float* img_loss, void* stream) {
  GSR_REQUIRE(C >= 1 && width > 0 && height > 0, "gsr_loss_iou_l1_fwd: bad C=%d or image %dx%d", C, width,
              height);
  GSR_REQUIRE(rgb && alpha && target_img && target_mask && sums && iou_loss && img_loss, "gsr_loss_iou_l1_fwd: null pointer");
  GSR_REQUIRE(ws != nullptr && ws_bytes >= gsr_loss_workspace(C, width, height),
              "gsr_loss_iou_l1_fwd: workspace too small");
  const int64_t HW = (int64_t)width * height;
  hipLaunchKernelGGL(k_loss_partials, dim3(kLossBlocksPerView, C), dim3(kLossThreads), 0, (hipStream_t)stream, rgb,
                     alpha, target_img, target_mask, HW, (float4*)ws);
  GSR_LAUNCH_CHECK("k_loss_partials");
  hipLaunchKernelGGL(k_loss_finalize, dim3(1), dim3(kLossThreads), 0, (hipStream_t)stream, (const float4*)ws, C,
                     kLossBlocksPerView, img_lambda, sums, iou_loss, img_loss);
  GSR_LAUNCH_CHECK("k_loss_finalize");
  return GSR_OK;
}

}  // extern "C"
