// Shape carving: the project-and-gather volume builder of
// ShapeCarver.forward (src/shape_carver.py:330-366; adaptive cameras move the mask volume's
// principal points, Ks_mask, and keep the carver's K for colours, as the reference does), with the scatter-min
// visibility of ray_cast_visibility_torch (:132-204, torch_scatter.scatter_min at :197) as
// a 64-bit atomicMin on (distance bits, voxel index) keys.
//
// Three passes over the n1*n2*n3 voxel grid, no host synchronisation:
//   k_carve_mask     grid point (rotated + centred, get_grid_points :369-374), projected into
//                    every camera (project_points_torch :57-103), nearest mask pixel
//                    (sample_nearest_pixels_torch :106-129), mean over cameras -> the two
//                    threshold flags (mask_volume >= 1, >= (C-1)/C);
//   k_carve_zbuf     for each threshold's voxels and each camera: distance to the camera
//                    centre and the flattened pixel (project_points_torch_single_cam), then
//                    atomicMin(key = dist_bits << 32 | voxel) — the front-most voxel per
//                    pixel, ties to the lower voxel index (torch_scatter's CPU order);
//   k_carve_volume   visibility (own key == pixel minimum), nearest rgb samples, weights
//                    1 / nonvisible 0.25 normalised over cameras (compute_voxel_colors_torch
//                    :238-301), and the 4-channel volume summed over both thresholds / 2.
//
// Reproduced as the reference has it: compute_voxel_colors_torch reads (H, W) from a
// [C,3,H,W] tensor as `_, H, W, _`, so visibility runs on a 3 x H_img pixel raster
// (rows clamp to [0,2], columns to [0,H_img-1]); the batched projection divides by
// z + 1e-8, the single-camera one by max(z, 1e-8); pixel rounding is half-to-even.
#include "gsr_common.h"

namespace gsr {

constexpr int kCarveThreads = 256;
constexpr int kCarveMaxCams = 32;

struct CarveCams {
  float E[kCarveMaxCams][12];   // rows 0..2 of each extrinsic [4,4]
  float K[kCarveMaxCams][9];    // colour / visibility intrinsics (the carver's own K)
  float Km[kCarveMaxCams][9];   // mask-volume intrinsics (adaptive: principal points moved)
  float pos[kCarveMaxCams][3];  // camera centres -R^T t
};

__device__ __forceinline__ void grid_point(const float* __restrict__ grid, int64_t i, float c, float s,
                                           const float* __restrict__ center, float p[3]) {
  const float g0 = grid[i * 3 + 0], g1 = grid[i * 3 + 1], g2 = grid[i * 3 + 2];
  // einsum("abci,ji->abcj", grid, rot_mat): p_j = sum_i g_i R_ji, rows (c,-s,0) (s,c,0) (0,0,1)
  p[0] = fmaf(g2, 0.f, fmaf(g1, -s, g0 * c)) + center[0];
  p[1] = fmaf(g2, 0.f, fmaf(g1, c, g0 * s)) + center[1];
  p[2] = fmaf(g2, 1.f, fmaf(g1, 0.f, g0 * 0.f)) + center[2];
}

// K (E [p;1])[:3] -> (u, v, w) homogeneous pixel; MASK selects the mask-volume intrinsics
template <bool MASK = false>
__device__ __forceinline__ void project_h(const CarveCams& cm, int c, const float p[3], float& u, float& v,
                                          float& w) {
  float q[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const float* e = cm.E[c] + 4 * k;
    q[k] = fmaf(e[3], 1.f, fmaf(e[2], p[2], fmaf(e[1], p[1], e[0] * p[0])));
  }
  const float* K = MASK ? cm.Km[c] : cm.K[c];
  u = fmaf(K[2], q[2], fmaf(K[1], q[1], K[0] * q[0]));
  v = fmaf(K[5], q[2], fmaf(K[4], q[1], K[3] * q[0]));
  w = fmaf(K[8], q[2], fmaf(K[7], q[1], K[6] * q[0]));
}

// .round().long().clamp(0, n-1)
__device__ __forceinline__ int round_clamp(float x, int n) {
  const float r = rintf(x);
  if (!(r >= 0.f)) return 0;               // negative or NaN
  if (r >= (float)(n - 1)) return n - 1;
  return (int)r;
}

__global__ __launch_bounds__(kCarveThreads) void k_carve_mask(
    const float* __restrict__ grid, int64_t N, float c, float s, const float* __restrict__ center,
    const CarveCams cm, int C, const float* __restrict__ mask, int H, int W, uint8_t* __restrict__ flags) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  float p[3];
  grid_point(grid, i, c, s, center, p);
  float sum = 0.f;
  for (int cam = 0; cam < C; ++cam) {
    float u, v, w;
    project_h<true>(cm, cam, p, u, v, w);
    const float d = w + 1e-8f;
    const int x = round_clamp(u / d, W), y = round_clamp(v / d, H);
    sum += mask[((int64_t)cam * H + y) * W + x];
  }
  const float mv = sum / (float)C;
  const float t2 = (float)((double)(C - 1) / (double)C);
  flags[i] = (uint8_t)((mv >= 1.f ? 1 : 0) | (mv >= t2 ? 2 : 0));
}

// visibility raster of compute_voxel_colors_torch: rows 0..2, columns 0..H_img-1
__device__ __forceinline__ int vis_pixel(float u, float v, float w, int H_img) {
  const float d = fmaxf(w, 1e-8f);
  const int px = round_clamp(u / d, H_img), py = round_clamp(v / d, 3);
  return py * H_img + px;
}

__device__ __forceinline__ float cam_distance(const CarveCams& cm, int c, const float p[3]) {
  const float dx = p[0] - cm.pos[c][0], dy = p[1] - cm.pos[c][1], dz = p[2] - cm.pos[c][2];
  return sqrtf(dx * dx + dy * dy + dz * dz);
}

__global__ __launch_bounds__(kCarveThreads) void k_carve_zbuf(
    const float* __restrict__ grid, int64_t N, float c, float s, const float* __restrict__ center,
    const CarveCams cm, int C, int H_img, const uint8_t* __restrict__ flags,
    unsigned long long* __restrict__ zbuf) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  const int f = flags[i];
  if (f == 0) return;
  float p[3];
  grid_point(grid, i, c, s, center, p);
  const int P = 3 * H_img;
  for (int cam = 0; cam < C; ++cam) {
    float u, v, w;
    project_h(cm, cam, p, u, v, w);
    const int pix = vis_pixel(u, v, w, H_img);
    const unsigned long long key =
        ((unsigned long long)__float_as_uint(cam_distance(cm, cam, p)) << 32) | (unsigned long long)(uint32_t)i;
    if (f & 1) atomicMin(&zbuf[((int64_t)0 * C + cam) * P + pix], key);
    if (f & 2) atomicMin(&zbuf[((int64_t)1 * C + cam) * P + pix], key);
  }
}

__global__ __launch_bounds__(kCarveThreads) void k_carve_volume(
    const float* __restrict__ grid, int64_t N, float c, float s, const float* __restrict__ center,
    const CarveCams cm, int C, const float* __restrict__ rgb, int H, int W, float fill, float nonvisible_w,
    const uint8_t* __restrict__ flags, const unsigned long long* __restrict__ zbuf, float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  const int f = flags[i];
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  float col[2][3];
  if (f) {
    float p[3];
    grid_point(grid, i, c, s, center, p);
    const int P = 3 * H;   // the visibility raster width is H_img (see header)
    // pass 1: weight sums; pass 2: normalised weights times samples (cameras in order)
    float wsum[2] = {0.f, 0.f};
    for (int cam = 0; cam < C; ++cam) {
      float u, v, w;
      project_h(cm, cam, p, u, v, w);
      const int pix = vis_pixel(u, v, w, H);
      const unsigned long long key =
          ((unsigned long long)__float_as_uint(cam_distance(cm, cam, p)) << 32) | (unsigned long long)(uint32_t)i;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const bool vis = (f >> t & 1) && zbuf[((int64_t)t * C + cam) * P + pix] == key;
        wsum[t] += vis ? 1.f : nonvisible_w;
      }
    }
    const float den[2] = {fmaxf(wsum[0], 1e-8f), fmaxf(wsum[1], 1e-8f)};
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int k = 0; k < 3; ++k) col[t][k] = 0.f;
    for (int cam = 0; cam < C; ++cam) {
      float u, v, w;
      project_h(cm, cam, p, u, v, w);
      const int pix = vis_pixel(u, v, w, H);
      const unsigned long long key =
          ((unsigned long long)__float_as_uint(cam_distance(cm, cam, p)) << 32) | (unsigned long long)(uint32_t)i;
      const float d = fmaxf(w, 1e-8f);
      const int x = round_clamp(u / d, W), y = round_clamp(v / d, H);
      float smp[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) smp[k] = rgb[(((int64_t)cam * 3 + k) * H + y) * W + x];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const bool vis = (f >> t & 1) && zbuf[((int64_t)t * C + cam) * P + pix] == key;
        const float wn = (vis ? 1.f : nonvisible_w) / den[t];
#pragma unroll
        for (int k = 0; k < 3; ++k) col[t][k] += wn * smp[k];
      }
    }
  }
  // out = (0 + volume_1 / 2) + volume_2 / 2, volume_t = (binary_t, colours_t or fill)
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const bool b = f >> t & 1;
    acc[0] = acc[0] + (b ? 1.f : 0.f) / 2.f;
#pragma unroll
    for (int k = 0; k < 3; ++k) acc[1 + k] = acc[1 + k] + (b ? col[t][k] : fill) / 2.f;
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) out[(int64_t)k * N + i] = acc[k];
}

// ---------------------------------------------------------------- adaptive cameras: mask medoids
// adjust_principal_points_to_seed (src/shape_carving.py:173-245) step 1 on the device: per view,
// the mask pixel nearest the mask centroid (numpy: ys, xs = nonzero(mask); cy, cx = means;
// argmin of (ys-cy)^2 + (xs-cx)^2, first in row-major order).  The coordinate sums are exact
// int64 (so the float64 means equal numpy's), the distances are float64 with numpy's
// rounding (no fused multiply-add), the minimum is an atomicMin on the distance's bits
// (non-negative doubles order like uint64) and the tie goes to the lowest flat index.
__global__ __launch_bounds__(kCarveThreads) void k_medoid_sums(const float* __restrict__ mask, int H, int W,
                                                              unsigned long long* __restrict__ sums) {
  const int c = blockIdx.y;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool in = i < (int64_t)H * W && mask[(int64_t)c * H * W + i] != 0.f;
  unsigned long long n = in ? 1ull : 0ull, sx = in ? (unsigned long long)(i % W) : 0ull,
                     sy = in ? (unsigned long long)(i / W) : 0ull;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    n += __shfl_xor(n, o, 64);
    sx += __shfl_xor(sx, o, 64);
    sy += __shfl_xor(sy, o, 64);
  }
  if ((threadIdx.x & 63) == 0 && n) {
    atomicAdd(&sums[3 * c + 0], n);
    atomicAdd(&sums[3 * c + 1], sx);
    atomicAdd(&sums[3 * c + 2], sy);
  }
}

__device__ __forceinline__ double medoid_d2(int64_t i, int W, const unsigned long long* s) {
  const double n = (double)s[0];
  const double cx = (double)s[1] / n, cy = (double)s[2] / n;
  const double dy = __dsub_rn((double)(i / W), cy), dx = __dsub_rn((double)(i % W), cx);
  return __dadd_rn(__dmul_rn(dy, dy), __dmul_rn(dx, dx));
}

__global__ __launch_bounds__(kCarveThreads) void k_medoid_min(const float* __restrict__ mask, int H, int W,
                                                             const unsigned long long* __restrict__ sums,
                                                             unsigned long long* __restrict__ best) {
  const int c = blockIdx.y;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)H * W || mask[(int64_t)c * H * W + i] == 0.f) return;
  atomicMin(&best[c], (unsigned long long)__double_as_longlong(medoid_d2(i, W, sums + 3 * c)));
}

__global__ __launch_bounds__(kCarveThreads) void k_medoid_arg(const float* __restrict__ mask, int H, int W,
                                                             const unsigned long long* __restrict__ sums,
                                                             const unsigned long long* __restrict__ best,
                                                             int32_t* __restrict__ arg) {
  const int c = blockIdx.y;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)H * W || mask[(int64_t)c * H * W + i] == 0.f) return;
  if ((unsigned long long)__double_as_longlong(medoid_d2(i, W, sums + 3 * c)) == best[c]) atomicMin(&arg[c], (int32_t)i);
}

__global__ void k_medoid_init(int C, unsigned long long* sums, unsigned long long* best, int32_t* arg) {
  const int t = threadIdx.x;
  for (int k = t; k < 3 * C; k += blockDim.x) sums[k] = 0ull;
  for (int k = t; k < C; k += blockDim.x) {
    best[k] = ~0ull;
    arg[k] = 0x7fffffff;
  }
}

}  // namespace gsr

using namespace gsr;

extern "C" {

size_t gsr_carve_workspace(int64_t n_voxels, int C, int height) {
  return (size_t)n_voxels + 16 + (size_t)2 * C * 3 * height * sizeof(unsigned long long);
}

int gsr_carve_volume(const float* grid, int64_t n_voxels, const float* center, double angle, const float* Ks,
                     const float* Ks_mask, const float* Es, int C, const float* mask, const float* rgb, int height,
                     int width, float fill, float nonvisible_weight, void* ws, size_t ws_bytes, float* out,
                     void* stream) {
  GSR_REQUIRE(n_voxels >= 0 && C >= 1 && C <= kCarveMaxCams && height > 0 && width > 0,
              "gsr_carve_volume: bad sizes (voxels=%lld, C=%d (max %d), image %dx%d)", (long long)n_voxels, C,
              kCarveMaxCams, width, height);
  GSR_REQUIRE(n_voxels < (1ll << 32), "gsr_carve_volume: too many voxels");
  if (n_voxels == 0) return GSR_OK;
  GSR_REQUIRE(grid && center && Ks && Es && mask && rgb && out, "gsr_carve_volume: null pointer");
  GSR_REQUIRE(ws != nullptr && ws_bytes >= gsr_carve_workspace(n_voxels, C, height),
              "gsr_carve_volume: workspace too small");
  // cameras are host arrays (the model's fixed K / E), passed by value to every kernel
  CarveCams cm;
  for (int c = 0; c < C; ++c) {
    for (int k = 0; k < 12; ++k) cm.E[c][k] = Es[c * 16 + k];
    for (int k = 0; k < 9; ++k) cm.K[c][k] = Ks[c * 9 + k];
    for (int k = 0; k < 9; ++k) cm.Km[c][k] = (Ks_mask ? Ks_mask : Ks)[c * 9 + k];
    // -R^T t, einsum('cij,cj->ci', R^T, t)
    for (int i = 0; i < 3; ++i) {
      float a = 0.f;
      for (int j = 0; j < 3; ++j) a += Es[c * 16 + j * 4 + i] * Es[c * 16 + j * 4 + 3];
      cm.pos[c][i] = -a;
    }
  }
  const float cf = (float)cos(angle), sf = (float)sin(angle);
  hipStream_t s = (hipStream_t)stream;
  unsigned long long* zbuf = (unsigned long long*)(((uintptr_t)ws + 7) & ~(uintptr_t)7);
  uint8_t* flags = (uint8_t*)(zbuf + (size_t)2 * C * 3 * height);
  const size_t zbytes = (size_t)2 * C * 3 * height * sizeof(unsigned long long);
  if (hipMemsetAsync(zbuf, 0xFF, zbytes, s) != hipSuccess) {
    set_error("gsr_carve_volume: hipMemsetAsync failed");
    return GSR_ELAUNCH;
  }
  const unsigned nb = (unsigned)ceil_div64(n_voxels, kCarveThreads);
  hipLaunchKernelGGL(k_carve_mask, dim3(nb), dim3(kCarveThreads), 0, s, grid, n_voxels, cf, sf, center, cm, C, mask,
                     height, width, flags);
  GSR_LAUNCH_CHECK("k_carve_mask");
  hipLaunchKernelGGL(k_carve_zbuf, dim3(nb), dim3(kCarveThreads), 0, s, grid, n_voxels, cf, sf, center, cm, C,
                     height, (const uint8_t*)flags, zbuf);
  GSR_LAUNCH_CHECK("k_carve_zbuf");
  hipLaunchKernelGGL(k_carve_volume, dim3(nb), dim3(kCarveThreads), 0, s, grid, n_voxels, cf, sf, center, cm, C, rgb,
                     height, width, fill, nonvisible_weight, (const uint8_t*)flags, (const unsigned long long*)zbuf,
                     out);
  GSR_LAUNCH_CHECK("k_carve_volume");
  return GSR_OK;
}

size_t gsr_carve_medoids_workspace(int C) { return (size_t)C * 4 * sizeof(unsigned long long) + 16; }

int gsr_carve_medoids(const float* masks, int C, int height, int width, void* ws, size_t ws_bytes, int32_t* medoid,
                      void* stream) {
  GSR_REQUIRE(C >= 1 && height > 0 && width > 0 && (int64_t)height * width < (1ll << 31),
              "gsr_carve_medoids: bad sizes (C=%d, image %dx%d)", C, width, height);
  GSR_REQUIRE(masks && medoid && ws, "gsr_carve_medoids: null pointer");
  GSR_REQUIRE(ws_bytes >= gsr_carve_medoids_workspace(C), "gsr_carve_medoids: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  unsigned long long* sums = (unsigned long long*)(((uintptr_t)ws + 7) & ~(uintptr_t)7);
  unsigned long long* best = sums + 3 * C;
  hipLaunchKernelGGL(k_medoid_init, dim3(1), dim3(256), 0, s, C, sums, best, medoid);
  GSR_LAUNCH_CHECK("k_medoid_init");
  const dim3 grid((unsigned)ceil_div64((int64_t)height * width, kCarveThreads), (unsigned)C);
  hipLaunchKernelGGL(k_medoid_sums, grid, dim3(kCarveThreads), 0, s, masks, height, width, sums);
  GSR_LAUNCH_CHECK("k_medoid_sums");
  hipLaunchKernelGGL(k_medoid_min, grid, dim3(kCarveThreads), 0, s, masks, height, width,
                     (const unsigned long long*)sums, best);
  GSR_LAUNCH_CHECK("k_medoid_min");
  hipLaunchKernelGGL(k_medoid_arg, grid, dim3(kCarveThreads), 0, s, masks, height, width,
                     (const unsigned long long*)sums, (const unsigned long long*)best, medoid);
  GSR_LAUNCH_CHECK("k_medoid_arg");
  return GSR_OK;
}

}  // extern "C"
