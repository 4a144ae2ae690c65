// SSIM term of the reference training loss (scripts/training/train_script.py:129,
// ssim_lambda * (1 - ssim(target_img, rgb)) with torchmetrics' StructuralSimilarityIndexMeasure
// (data_range=1.0)), forward and backward, for C views at once (the batch mean).
//
// torchmetrics pads by reflection, convolves x, y, x^2, y^2, xy with the 11x11 Gaussian
// (sigma 1.5; the outer product of the normalised 1-D taps) and crops the 5-pixel border of
// the SSIM map again, so every kept window lies inside the image: the value is the mean,
// over 3 channels and the (H-10) x (W-10) window centres, of
//   S = (2 mx my + C1)(2 sxy + C2) / ((mx^2 + my^2 + C1)(sx + sy + C2)),
//   sx = E[x^2] - mx^2, sy = E[y^2] - my^2, sxy = E[xy] - mx my,  C1 = 0.01^2, C2 = 0.03^2,
// and the padding never enters.  Here the blur is separable (horizontal, then vertical) over
// an LDS tile with its halo -- fp32 rounding differs from the 2-D convolution, not the value.
//
// Backward, for the rendered image y: per window q, a = dS/dmy, b = dS/dE[y^2], c = dS/dE[xy]
//   a = 2 mx (A2 - A1) / (B1 B2) - 2 my S (1/B1 - 1/B2),  b = -S / B2,  c = 2 A1 / (B1 B2),
// and dL/dy_p = g / count * sum_q G(q - p) (a_q + 2 y_p b_q + x_p c_q): the same blur applied
// to the a, b, c maps (zero outside the kept windows).  The forward stores a, b, c per window
// (12 B) when a backward will follow; the backward blurs them onto 16x16 pixel tiles.
//
// Reductions are fixed-order (per-workgroup partials, then one workgroup sums them in index
// order), so the value is bitwise reproducible.
#include "gsr_common.h"

namespace gsr {

constexpr int kSsimK = 11;               // taps
constexpr int kSsimR = 5;                // radius
constexpr int kSsimT = 16;               // output tile side
constexpr int kSsimThreads = 256;
constexpr float kSsimC1 = 0.01f * 0.01f;   // (k1 * data_range)^2
constexpr float kSsimC2 = 0.03f * 0.03f;

struct SsimTaps {
  float g[kSsimK];
};

// image accessor: element (c, ch, i, j) at base + c*sc + ch*sch + i*sr + j*sp
struct Img {
  const float* p;
  int64_t sc, sch, sr, sp;
  __device__ __forceinline__ float at(int c, int ch, int i, int j) const {
    return p[c * sc + ch * sch + (int64_t)i * sr + (int64_t)j * sp];
  }
};

struct WinStats {
  float mx, my, exx, eyy, exy;
};

__device__ __forceinline__ float ssim_of(const WinStats& w) {
  const float mxy = w.mx * w.my, mxx = w.mx * w.mx, myy = w.my * w.my;
  const float A1 = 2.f * mxy + kSsimC1, A2 = 2.f * (w.exy - mxy) + kSsimC2;
  const float B1 = mxx + myy + kSsimC1, B2 = (w.exx - mxx) + (w.eyy - myy) + kSsimC2;
  return (A1 * A2) / (B1 * B2);
}

// Window statistics of the R x R windows whose top-left centre is (i0, j0) (window centres
// i0 .. i0+R-1), from the (R+10) x (R+10) input patch at (i0-5, j0-5): horizontal pass into
// s_h[5][(R+10)][R], then the vertical pass per window (thread loop).  Patch pixels outside
// the image read as 0 (only windows inside the image are used).
template <int R>
__device__ __forceinline__ void load_patch(const Img& X, const Img& Y, int c, int ch, int H, int W, int i0, int j0,
                                           float (*s_x)[R + 2 * kSsimR], float (*s_y)[R + 2 * kSsimR]) {
  constexpr int P = R + 2 * kSsimR;
  for (int t = threadIdx.x; t < P * P; t += kSsimThreads) {
    const int r = t / P, q = t - r * P;
    const int i = i0 - kSsimR + r, j = j0 - kSsimR + q;
    const bool in = i >= 0 && i < H && j >= 0 && j < W;
    s_x[r][q] = in ? X.at(c, ch, i, j) : 0.f;
    s_y[r][q] = in ? Y.at(c, ch, i, j) : 0.f;
  }
}

template <int R>
__device__ __forceinline__ void hblur5(const SsimTaps& tp, float (*s_x)[R + 2 * kSsimR], float (*s_y)[R + 2 * kSsimR],
                                       float (*s_h)[R + 2 * kSsimR][R]) {
  constexpr int P = R + 2 * kSsimR;
  for (int t = threadIdx.x; t < P * R; t += kSsimThreads) {
    const int r = t / R, q = t - r * R;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f, a4 = 0.f;
#pragma unroll
    for (int k = 0; k < kSsimK; ++k) {
      const float x = s_x[r][q + k], y = s_y[r][q + k], g = tp.g[k];
      a0 += g * x;
      a1 += g * y;
      a2 += g * (x * x);
      a3 += g * (y * y);
      a4 += g * (x * y);
    }
    s_h[0][r][q] = a0;
    s_h[1][r][q] = a1;
    s_h[2][r][q] = a2;
    s_h[3][r][q] = a3;
    s_h[4][r][q] = a4;
  }
}

template <int R>
__device__ __forceinline__ WinStats vblur5(const SsimTaps& tp, float (*s_h)[R + 2 * kSsimR][R], int wi, int wj) {
  WinStats w{0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < kSsimK; ++k) {
    const float g = tp.g[k];
    w.mx += g * s_h[0][wi + k][wj];
    w.my += g * s_h[1][wi + k][wj];
    w.exx += g * s_h[2][wi + k][wj];
    w.eyy += g * s_h[3][wi + k][wj];
    w.exy += g * s_h[4][wi + k][wj];
  }
  return w;
}

__device__ __forceinline__ float block_sum(float v, float* s_red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) s_red[wv] = v;
  __syncthreads();
  float t = 0.f;
  if (threadIdx.x == 0)
    for (int k = 0; k < kSsimThreads / 64; ++k) t += s_red[k];
  return t;
}

// dS/dmy, dS/dE[y^2], dS/dE[xy] of one window (the backward's per-window factors)
__device__ __forceinline__ float3 ssim_dy(const WinStats& w, float& S) {
  const float mxy = w.mx * w.my, mxx = w.mx * w.mx, myy = w.my * w.my;
  const float A1 = 2.f * mxy + kSsimC1, A2 = 2.f * (w.exy - mxy) + kSsimC2;
  const float B1 = mxx + myy + kSsimC1, B2 = (w.exx - mxx) + (w.eyy - myy) + kSsimC2;
  const float den = 1.f / (B1 * B2);
  S = (A1 * A2) / (B1 * B2);
  return make_float3(2.f * w.mx * (A2 - A1) * den - 2.f * w.my * S * (1.f / B1 - 1.f / B2), -S / B2,
                     2.f * A1 * den);
}

// forward: one workgroup per (16x16 tile of window centres, channel, view); partial[block],
// and (abc != null) the window's backward factors at abc[((view*3 + ch)*3 + k) * Hw*Ww + window]
__global__ __launch_bounds__(kSsimThreads) void k_ssim_fwd(const Img X, const Img Y, int H, int W,
                                                          const SsimTaps tp, float* __restrict__ partial,
                                                          float* __restrict__ abc) {
  constexpr int R = kSsimT, P = R + 2 * kSsimR;
  __shared__ float s_x[P][P], s_y[P][P];
  __shared__ float s_h[5][P][R];
  __shared__ float s_red[kSsimThreads / 64];
  const int c = blockIdx.z / 3, ch = blockIdx.z - 3 * c;
  const int i0 = kSsimR + blockIdx.y * R, j0 = kSsimR + blockIdx.x * R;   // first window centre
  load_patch<R>(X, Y, c, ch, H, W, i0, j0, s_x, s_y);
  __syncthreads();
  hblur5<R>(tp, s_x, s_y, s_h);
  __syncthreads();
  const int wi = threadIdx.x / R, wj = threadIdx.x % R;
  const bool kept = i0 + wi < H - kSsimR && j0 + wj < W - kSsimR;
  float s = 0.f;
  if (kept) {
    const WinStats w = vblur5<R>(tp, s_h, wi, wj);
    if (abc) {
      const float3 d = ssim_dy(w, s);
      const int64_t Hw = H - 2 * kSsimR, Ww = W - 2 * kSsimR;
      float* o = abc + (int64_t)blockIdx.z * 3 * Hw * Ww + (int64_t)(i0 - kSsimR + wi) * Ww + (j0 - kSsimR + wj);
      o[0] = d.x;
      o[Hw * Ww] = d.y;
      o[2 * Hw * Ww] = d.z;
    } else {
      s = ssim_of(w);
    }
  }
  const float t = block_sum(s, s_red);
  if (threadIdx.x == 0)
    partial[((int64_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x] = t;
}

// one workgroup: mean over everything, in index order -> *ssim (the batch mean)
__global__ __launch_bounds__(kSsimThreads) void k_ssim_finalize(const float* __restrict__ partial, int64_t nb,
                                                               double inv_count, float* __restrict__ ssim) {
  __shared__ float s_red[kSsimThreads / 64];
  float v = 0.f;
  for (int64_t k = threadIdx.x; k < nb; k += kSsimThreads) v += partial[k];
  const float t = block_sum(v, s_red);
  if (threadIdx.x == 0) *ssim = (float)((double)t * inv_count);
}

// backward: one workgroup per (16x16 tile of pixels, channel, view): the per-window factors
// a, b, c the forward stored (zero outside the kept windows) blurred back onto the pixels
// (the taps are symmetric, so the transpose blur is the blur), grad = g/count (A + 2 y B + x C),
// written through the Y layout's strides into gy
__global__ __launch_bounds__(kSsimThreads) void k_ssim_bwd(const Img X, const Img Y, int H, int W, const SsimTaps tp,
                                                          const float* __restrict__ abc, const float* __restrict__ g_out,
                                                          float inv_count, float* __restrict__ gy) {
  constexpr int T = kSsimT;                 // output pixels per side
  constexpr int R = T + 2 * kSsimR;         // windows per side (26)
  __shared__ float s_abc[3][R][R];
  __shared__ float s_h2[3][R][T];
  const int c = blockIdx.z / 3, ch = blockIdx.z - 3 * c;
  const int pi0 = blockIdx.y * T, pj0 = blockIdx.x * T;   // first output pixel
  const int Hw = H - 2 * kSsimR, Ww = W - 2 * kSsimR;
  const float* m = abc + (int64_t)blockIdx.z * 3 * Hw * Ww;
  // window (wi, wj) of the tile is centred at pixel (pi0 - 5 + wi, pj0 - 5 + wj), i.e. window
  // index (pi0 - 10 + wi, pj0 - 10 + wj) of the map
  for (int t = threadIdx.x; t < R * R; t += kSsimThreads) {
    const int wi = t / R, wj = t - wi * R;
    const int mi = pi0 - 2 * kSsimR + wi, mj = pj0 - 2 * kSsimR + wj;
    const bool in = mi >= 0 && mi < Hw && mj >= 0 && mj < Ww;
    const int64_t o = (int64_t)mi * Ww + mj;
    s_abc[0][wi][wj] = in ? m[o] : 0.f;
    s_abc[1][wi][wj] = in ? m[(int64_t)Hw * Ww + o] : 0.f;
    s_abc[2][wi][wj] = in ? m[2 * (int64_t)Hw * Ww + o] : 0.f;
  }
  __syncthreads();
  for (int t = threadIdx.x; t < R * T; t += kSsimThreads) {
    const int r = t / T, q = t - r * T;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f;
#pragma unroll
    for (int k = 0; k < kSsimK; ++k) {
      const float g = tp.g[k];
      a0 += g * s_abc[0][r][q + k];
      a1 += g * s_abc[1][r][q + k];
      a2 += g * s_abc[2][r][q + k];
    }
    s_h2[0][r][q] = a0;
    s_h2[1][r][q] = a1;
    s_h2[2][r][q] = a2;
  }
  __syncthreads();
  const int pi = threadIdx.x / T, pj = threadIdx.x % T;
  const int i = pi0 + pi, j = pj0 + pj;
  if (i < H && j < W) {
    float A = 0.f, B = 0.f, Cc = 0.f;
#pragma unroll
    for (int k = 0; k < kSsimK; ++k) {
      const float g = tp.g[k];
      A += g * s_h2[0][pi + k][pj];
      B += g * s_h2[1][pi + k][pj];
      Cc += g * s_h2[2][pi + k][pj];
    }
    const float x = X.at(c, ch, i, j), y = Y.at(c, ch, i, j);
    const float gs = g_out[0] * inv_count;
    gy[c * Y.sc + ch * Y.sch + (int64_t)i * Y.sr + (int64_t)j * Y.sp] = gs * (A + 2.f * y * B + x * Cc);
  }
}

static SsimTaps taps(const float* g) {
  SsimTaps t;
  for (int k = 0; k < kSsimK; ++k) t.g[k] = g[k];
  return t;
}

}  // namespace gsr

using namespace gsr;

extern "C" {

size_t gsr_ssim_workspace(int C, int width, int height) {
  if (C < 1 || width <= 2 * kSsimR || height <= 2 * kSsimR) return 16;
  const int64_t nb = (int64_t)C * 3 * ceil_div(width - 2 * kSsimR, kSsimT) * ceil_div(height - 2 * kSsimR, kSsimT);
  return (size_t)nb * sizeof(float) + 16;
}

size_t gsr_ssim_factors_size(int C, int width, int height) {
  if (C < 1 || width <= 2 * kSsimR || height <= 2 * kSsimR) return 0;
  return (size_t)C * 9 * (size_t)(width - 2 * kSsimR) * (size_t)(height - 2 * kSsimR);
}

int gsr_ssim_fwd(const float* x, const int64_t* x_strides, const float* y, const int64_t* y_strides, int C, int width,
                 int height, const float* taps11, void* ws, size_t ws_bytes, float* ssim, float* factors,
                 void* stream) {
  GSR_REQUIRE(C >= 1 && width > 2 * kSsimR && height > 2 * kSsimR,
              "gsr_ssim_fwd: need C >= 1 and an image larger than %dx%d, got C=%d %dx%d", 2 * kSsimR + 1,
              2 * kSsimR + 1, C, width, height);
  GSR_REQUIRE(x && y && x_strides && y_strides && taps11 && ssim && ws, "gsr_ssim_fwd: null pointer");
  GSR_REQUIRE(ws_bytes >= gsr_ssim_workspace(C, width, height), "gsr_ssim_fwd: workspace too small");
  const Img X{x, x_strides[0], x_strides[1], x_strides[2], x_strides[3]};
  const Img Y{y, y_strides[0], y_strides[1], y_strides[2], y_strides[3]};
  const dim3 grid(ceil_div(width - 2 * kSsimR, kSsimT), ceil_div(height - 2 * kSsimR, kSsimT), 3 * C);
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(k_ssim_fwd, grid, dim3(kSsimThreads), 0, s, X, Y, height, width, taps(taps11), (float*)ws,
                     factors);
  GSR_LAUNCH_CHECK("k_ssim_fwd");
  const int64_t nb = (int64_t)grid.x * grid.y * grid.z;
  const double count = 3.0 * C * (double)(width - 2 * kSsimR) * (double)(height - 2 * kSsimR);
  hipLaunchKernelGGL(k_ssim_finalize, dim3(1), dim3(kSsimThreads), 0, s, (const float*)ws, nb, 1.0 / count, ssim);
  GSR_LAUNCH_CHECK("k_ssim_finalize");
  return GSR_OK;
}

int gsr_ssim_bwd(const float* x, const int64_t* x_strides, const float* y, const int64_t* y_strides, int C, int width,
                 int height, const float* taps11, const float* factors, const float* g_out, float* grad_y,
                 void* stream) {
  GSR_REQUIRE(C >= 1 && width > 2 * kSsimR && height > 2 * kSsimR, "gsr_ssim_bwd: bad C=%d or image %dx%d", C, width,
              height);
  GSR_REQUIRE(x && y && x_strides && y_strides && taps11 && factors && g_out && grad_y, "gsr_ssim_bwd: null pointer");
  const Img X{x, x_strides[0], x_strides[1], x_strides[2], x_strides[3]};
  const Img Y{y, y_strides[0], y_strides[1], y_strides[2], y_strides[3]};
  const dim3 grid(ceil_div(width, kSsimT), ceil_div(height, kSsimT), 3 * C);
  const double count = 3.0 * C * (double)(width - 2 * kSsimR) * (double)(height - 2 * kSsimR);
  hipLaunchKernelGGL(k_ssim_bwd, grid, dim3(kSsimThreads), 0, (hipStream_t)stream, X, Y, height, width, taps(taps11),
                     factors, g_out, (float)(1.0 / count), grad_y);
  GSR_LAUNCH_CHECK("k_ssim_bwd");
  return GSR_OK;
}

}  // extern "C"
