// Projection backward: per Gaussian, reduce its per-entry partials (fixed order → bitwise
// deterministic), chain through the screen-space parameters, the projection and the
// adapter activations, and sum over cameras.  One thread per Gaussian n.
//
// 3D chain (oracle/oracle3d.py restates the forward; its autograd is the parity check):
//   record (a,b,c) = (A/2, B, C/2) of conic = inv(cov2d + eps2d I)
//   V_cov = -Cinv V_sym Cinv,  V_sym = [[vA, vB/2],[vB/2, vC]]
//   cov2d = J Sc J^T:  V_Sc = J^T V_cov J,  V_J = 2 V_cov J Sc
//   J(x,y,z) with FOV-clamped tx/ty (gradient through x/y only where unclamped)
//   mean2d = (fx x/z + cx, fy y/z + cy);  mean_c = Rv m + t;  Sc = Rv S Rv^T
//   S = M M^T, M = R(q) diag(s):  V_M = 2 V_S M
//   R(q) with q re-normalised (gsplat) after the adapter's q/(|q|+1e-8)
//   scales = exp, colours clamp(0,1) (pass-through on [0,1] inclusive), opacity sigmoid.
// 2D chain: (a,b,c)(theta, ia, ib), ia = 1/(2 sx^2 + 1e-8), sx = exp(ls).
#include <algorithm>
#include <cstdint>

// GSR_PBWD_CONTRACT 0: the projection backward's chain compiled without fp contraction -- every
// multiply and add rounded on its own, as the oracle's torch ops evaluate it (a
// one-ulp contraction change moved the 200-step fit's dPSNR from 0.024 to 0.061 dB).  Measured
// in round 6 it costs the kernel 11 % at config 3 (55.5 -> 61.5 us) and 25 % at config 5 (0.41
// -> 0.51 ms), so the default keeps contraction (1) and tests/test_fit_gpu.py pins the fit's
// dPSNR over three starts instead (profiles/r06_fit_contract.txt).
#ifndef GSR_PBWD_CONTRACT
#define GSR_PBWD_CONTRACT 1
#endif
#if !GSR_PBWD_CONTRACT
#pragma clang fp contract(off)
#endif
#include "project_math.h"

namespace gsr {

constexpr int kBwdThreads = 256;

// Sum the partial rows of one (c,n): entry j (row-major tile of its rect) has row
// isect_offset[c*N+n] + j (emission order); it was written by the raster backward iff the
// entry precedes its tile's cut (key < tile_cut[tile]), otherwise it contributes nothing.
__device__ __forceinline__ void gather_partials(const uint2 r, int tw, int64_t ct_base, uint64_t key, int off,
                                                const uint64_t* __restrict__ tile_cut,
                                                const float* __restrict__ partial, float (&acc)[kPartial]) {
  const int x0 = r.x & 0xffff, x1 = r.x >> 16, y0 = r.y & 0xffff, y1 = r.y >> 16;
  const int cnt = (x1 - x0) * (y1 - y0);
  const float* rows = partial + (int64_t)off * kPartialStride;
  // four tiles per round: their cut keys first, then the rows that exist (two dependent
  // memory round trips per four tiles instead of two per tile)
  int tx = x0, ty = y0;   // tile of entry j0 (row-major over the rect)
  for (int j0 = 0; j0 < cnt; j0 += 4) {
    bool has[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      has[u] = j0 + u < cnt && key < tile_cut[ct_base + ty * tw + tx];
      if (++tx == x1) {
        tx = x0;
        ++ty;
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (has[u]) {
        const float* row = rows + kPartialStride * (j0 + u);
#pragma unroll
        for (int q = 0; q < kPartial; ++q) acc[q] += row[q];
      }
    }
  }
}

// (camera, Gaussian)-parallel: a workgroup owns G Gaussians and CPB = min(C, 256) camera
// slots (thread = slot * G + g; slot s handles cameras s, s+CPB, ...).  Each thread gathers
// its (c,n) partial rows and chains them to the camera's contribution {v_mean, V_M (the
// gradient of M = R diag(s)), v_colour, v_opacity}; the slots are then summed in LDS in
// fixed order (deterministic) and one thread per Gaussian applies the camera-independent
// chain (rotation / scale / quaternion normalisation / adapter activations).
constexpr int kContrib = 16;   // v_m[3], V_M[9], v_col[3], v_op
constexpr int kCamLds = 16;    // cameras staged in LDS per workgroup (calls of more read them from global)

// 5 workgroups of 256 threads per CU (96 VGPRs, 16 B/lane spilled): the kernel waits on its
// gathers (tile cut keys, then the partial rows) most of the time, so occupancy pays --
// config 5 486 -> 449 us, config 3 56.5 -> 54.7 us; 6 per CU (80 VGPRs, 88 B spilled) is
// slower (636 / 77 us)
#ifndef GSR_PBWD_MINB
#define GSR_PBWD_MINB 5
#endif
// ROWS: the Gaussians are those listed in a row block (gsr3d_touched_rows; row 1 + i holds n)
// and the gradients go to their rows instead of v_params (the sparse exchange of a band share).
template <bool ROWS>
__global__ __launch_bounds__(kBwdThreads, GSR_PBWD_MINB) void k_project3d_bwd(
    const float* __restrict__ params, int64_t N, int64_t stride, const float* __restrict__ viewmats,
    const float* __restrict__ Ks, int C, int W, int H, float eps2d, int input_mode, int tw, int th,
    const uint2* __restrict__ rect,
    const int32_t* __restrict__ isect_offset, const int32_t* __restrict__ isect_count,
    const float* __restrict__ depth, const uint64_t* __restrict__ tile_cut, const float* __restrict__ partial,
    int CPB, int G, int64_t n_begin, int64_t n_end, const gsr_bin_stats* __restrict__ stats,
    float* __restrict__ v_params, float* __restrict__ block, int64_t cap) {
  __shared__ float s_con[kBwdThreads][kContrib + 1];
  __shared__ int s_any[kBwdThreads];
  // the cameras, staged once per workgroup (four b128 LDS reads per camera instead of ~6 global
  // loads per (camera, Gaussian) thread: this kernel is bound by its memory instructions)
  __shared__ float4 s_cam[kCamLds][4];
  const bool cam_lds = C <= kCamLds;
  if (cam_lds && (int)threadIdx.x < 4 * C) {
    const int cc = threadIdx.x >> 2, part = threadIdx.x & 3;
    const float* V = viewmats + cc * 16;
    const float* Kc = Ks + cc * 9;
    float4 v;
    if (part == 0) v = make_float4(V[0], V[1], V[2], V[4]);
    else if (part == 1) v = make_float4(V[5], V[6], V[8], V[9]);
    else if (part == 2) v = make_float4(V[10], V[3], V[7], V[11]);
    else v = make_float4(Kc[0], Kc[4], Kc[2], Kc[5]);
    s_cam[cc][part] = v;
  }
  __syncthreads();
  const int g_loc = threadIdx.x % G;
  const int slot = threadIdx.x / G;
  const int64_t i_row = (int64_t)blockIdx.x * G + g_loc;   // ROWS: the row of this Gaussian
  int64_t n;
  bool listed = true;
  if constexpr (ROWS) {
    const int64_t count = min((int64_t)reinterpret_cast<const int32_t*>(block)[0], cap);
    listed = i_row < count;
    n = listed ? reinterpret_cast<const int32_t*>(block)[(1 + i_row) * GSR_ROW_FLOATS] : 0;
    // (after a forward overflow the header is past the cap and the rows hold no indices: kept
    // in range; those rows are written NaN below, and gsr_rows_scatter_add NaN-fills anyway)
    n = min(max(n, (int64_t)0), max(N - 1, (int64_t)0));
  } else {
    n = n_begin + i_row;
    listed = n < n_end;
  }
  // the forward's bounds did not hold: NaN rows, and no partial row is read (their offsets may
  // lie past the buffers).  The flag loads with the first gathers and is tested inside the
  // camera loop, so it adds no round trip of its own.
  const bool ovf = stats != nullptr && stats->overflow != 0;
  const bool active = slot < CPB && listed;
  const int T = tw * th;
  float v_m[3] = {0.f, 0.f, 0.f};
  float v_M[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) v_M[k] = 0.f;
  float v_col[3] = {0.f, 0.f, 0.f};
  float v_op = 0.f;
  int any = 0;
  if (active) {
    const Act3D a = activate3d(params + n * stride, input_mode);
    Geo3D g;
    for (int c = slot; c < C; c += CPB) {
      const int64_t cn = (int64_t)c * N + n;
      // the (c,n) scalars load together (no dependent round trip before the rect / key).  Pinned
      // by the empty asm: the compiler sank the rect / offset / depth loads below the cnt test,
      // three more dependent round trips per camera (config 3 55 -> 53.5 us, config 5 453 -> 438
      // us).  (Issuing all four cut keys and rows of a round unconditionally -- an entry without
      // a row reading another one -- was slower: 55 -> 81 us.  This kernel is bound by its memory
      // instructions, not only by their latency, so masked-off loads are worth their branches.)
      // (the entry count is the rect's area, as the forward wrote it: isect_count is not read,
      // 4 B less per (c,n) -- 48 MB of the config-5 launch's traffic)
      const uint2 rc = rect[cn];
      const int off = isect_offset[cn];
      const uint64_t key = sort_key(depth, cn, GSR_ORDER_DEPTH);
      asm volatile("" ::"v"(rc.x), "v"(rc.y), "v"(off), "v"((uint32_t)(key >> 32)));
      const int cnt = (int)(((rc.x >> 16) - (rc.x & 0xffffu)) * ((rc.y >> 16) - (rc.y & 0xffffu)));
      if (cnt <= 0 || ovf) continue;
      float acc[kPartial];
#pragma unroll
      for (int v = 0; v < kPartial; ++v) acc[v] = 0.f;
      gather_partials(rc, tw, (int64_t)c * T, key, off, tile_cut, partial, acc);
      Cam cam;
      if (cam_lds) {
        const float4 a = s_cam[c][0], b = s_cam[c][1], d = s_cam[c][2], k = s_cam[c][3];
        cam.R[0] = a.x; cam.R[1] = a.y; cam.R[2] = a.z; cam.R[3] = a.w;
        cam.R[4] = b.x; cam.R[5] = b.y; cam.R[6] = b.z; cam.R[7] = b.w;
        cam.R[8] = d.x; cam.t[0] = d.y; cam.t[1] = d.z; cam.t[2] = d.w;
        cam.fx = k.x; cam.fy = k.y; cam.cx = k.z; cam.cy = k.w;
      } else {
        cam = load_cam(viewmats + c * 16, Ks + c * 9);
      }
      // recompute the forward geometry (not culled: it has intersections)
      geo3d(a, cam, W, H, 0.f, 3.4e38f, eps2d, g);
      any = 1;
      v_op += acc[5];
      v_col[0] += acc[6];
      v_col[1] += acc[7];
      v_col[2] += acc[8];
      // conic (A,B,C) from record (a,b,c) = (A/2, B, C/2)
      const float vA = 0.5f * acc[2], vB = acc[3], vC = 0.5f * acc[4];
      // V_cov = -Cinv V_sym Cinv ; Cinv = [[A,B],[B,C]]
      const float A = g.A, B = g.B, Cc = g.C;
      const float hb = 0.5f * vB;
      // X = V_sym Cinv
      const float X00 = vA * A + hb * B, X01 = vA * B + hb * Cc;
      const float X10 = hb * A + vC * B, X11 = hb * B + vC * Cc;
      const float G00 = -(A * X00 + B * X10);
      const float G01 = -(A * X01 + B * X11);
      const float G11 = -(B * X01 + Cc * X11);
      // V_Sc = J^T G J  (J = [[J00,0,J02],[0,J11,J12]])
      const float J00 = g.J00, J02 = g.J02, J11 = g.J11, J12 = g.J12;
      float VSc[9];
      {
        // G J : 2x3
        const float GJ00 = G00 * J00, GJ01 = G01 * J11, GJ02 = G00 * J02 + G01 * J12;
        const float GJ10 = G01 * J00, GJ11 = G11 * J11, GJ12 = G01 * J02 + G11 * J12;
        // J^T (GJ): 3x3, J^T rows: (J00,0), (0,J11), (J02,J12)
        VSc[0] = J00 * GJ00;
        VSc[1] = J00 * GJ01;
        VSc[2] = J00 * GJ02;
        VSc[3] = J11 * GJ10;
        VSc[4] = J11 * GJ11;
        VSc[5] = J11 * GJ12;
        VSc[6] = J02 * GJ00 + J12 * GJ10;
        VSc[7] = J02 * GJ01 + J12 * GJ11;
        VSc[8] = J02 * GJ02 + J12 * GJ12;
      }
      // V_J = 2 G J Sc  (2x3), only the entries J00, J02, J11, J12 matter
      const float* S = g.Sc;  // s00 s01 s02 s11 s12 s22
      const float Sf[9] = {S[0], S[1], S[2], S[1], S[3], S[4], S[2], S[4], S[5]};
      float JS[6];
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        JS[k] = J00 * Sf[0 * 3 + k] + J02 * Sf[2 * 3 + k];
        JS[3 + k] = J11 * Sf[1 * 3 + k] + J12 * Sf[2 * 3 + k];
      }
      const float vJ00 = 2.f * (G00 * JS[0] + G01 * JS[3]);
      const float vJ02 = 2.f * (G00 * JS[2] + G01 * JS[5]);
      const float vJ11 = 2.f * (G01 * JS[1] + G11 * JS[4]);
      const float vJ12 = 2.f * (G01 * JS[2] + G11 * JS[5]);
      // mean_c gradients
      const float x = g.mc[0], y = g.mc[1];
      const float rz = g.rz, rz2 = rz * rz, rz3 = rz2 * rz;
      const float fx = cam.fx, fy = cam.fy;
      const float vu = acc[0], vv = acc[1];
      float vmc0 = fx * rz * vu;
      float vmc1 = fy * rz * vv;
      float vmc2 = -(fx * x * vu + fy * y * vv) * rz2;
      vmc2 += -fx * rz2 * vJ00 - fy * rz2 * vJ11;
      if (g.clx) {
        vmc0 += -fx * rz2 * vJ02;
        vmc2 += 2.f * fx * g.tx * rz3 * vJ02;
      } else {
        vmc2 += fx * g.tx * rz3 * vJ02;
      }
      if (g.cly) {
        vmc1 += -fy * rz2 * vJ12;
        vmc2 += 2.f * fy * g.ty * rz3 * vJ12;
      } else {
        vmc2 += fy * g.ty * rz3 * vJ12;
      }
      const float* Rv = cam.R;
      // v_m += Rv^T v_mc
#pragma unroll
      for (int k = 0; k < 3; ++k) v_m[k] += Rv[0 * 3 + k] * vmc0 + Rv[1 * 3 + k] * vmc1 + Rv[2 * 3 + k] * vmc2;
      // V_S = Rv^T V_Sc Rv
      float T1[9];
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int k = 0; k < 3; ++k)
          T1[r * 3 + k] = Rv[0 * 3 + r] * VSc[0 * 3 + k] + Rv[1 * 3 + r] * VSc[1 * 3 + k] + Rv[2 * 3 + r] * VSc[2 * 3 + k];
      float VS[9];
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int k = 0; k < 3; ++k)
          VS[r * 3 + k] = T1[r * 3 + 0] * Rv[0 * 3 + k] + T1[r * 3 + 1] * Rv[1 * 3 + k] + T1[r * 3 + 2] * Rv[2 * 3 + k];
      // V_M = (V_S + V_S^T) M   (M = R diag(s); converted to v_R, v_s after the camera sum)
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          float vm = 0.f;
#pragma unroll
          for (int l = 0; l < 3; ++l) vm += (VS[r * 3 + l] + VS[l * 3 + r]) * g.M[l * 3 + k];
          v_M[r * 3 + k] += vm;
        }
    }
  }
  {
    float* d = s_con[threadIdx.x];
    d[0] = v_m[0]; d[1] = v_m[1]; d[2] = v_m[2];
#pragma unroll
    for (int k = 0; k < 9; ++k) d[3 + k] = v_M[k];
    d[12] = v_col[0]; d[13] = v_col[1]; d[14] = v_col[2];
    d[15] = v_op;
    s_any[threadIdx.x] = any;
  }
  __syncthreads();
  if (slot != 0 || !listed) return;
  any = 0;
  for (int sl = 1; sl < CPB; ++sl) {
    const float* d = s_con[sl * G + g_loc];
    v_m[0] += d[0]; v_m[1] += d[1]; v_m[2] += d[2];
#pragma unroll
    for (int k = 0; k < 9; ++k) v_M[k] += d[3 + k];
    v_col[0] += d[12]; v_col[1] += d[13]; v_col[2] += d[14];
    v_op += d[15];
    any |= s_any[sl * G + g_loc];
  }
  any |= s_any[threadIdx.x];
  float* out = ROWS ? block + (1 + i_row) * GSR_ROW_FLOATS + 2 : v_params + n * 14;
  if (ovf) {
#pragma unroll
    for (int k = 0; k < 14; ++k) out[k] = __builtin_nanf("");
    return;
  }
  if (!any) {
#pragma unroll
    for (int k = 0; k < 14; ++k) out[k] = 0.f;
    return;
  }
  const Act3D a = activate3d(params + n * stride, input_mode);
  // M = R diag(s):  v_R = V_M diag(s),  v_s = sum_r V_M[r][k] R[r][k]
  float Rq[9], qn[4], qinv;
  quat_rotmat(a.q, Rq, qn, &qinv);
  float v_R[9], v_s[3] = {0.f, 0.f, 0.f};
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      v_R[r * 3 + k] = v_M[r * 3 + k] * a.s[k];
      v_s[k] += v_M[r * 3 + k] * Rq[r * 3 + k];
    }
  // R(qn) → v_qn (normalised quaternion)
  const float w = qn[0], x = qn[1], y = qn[2], z = qn[3];
  const float* V = v_R;
  float vq[4];
  vq[0] = 2.f * (z * (V[3] - V[1]) + y * (V[2] - V[6]) + x * (V[7] - V[5]));
  vq[1] = 2.f * (y * V[1] + z * V[2] + y * V[3] - 2.f * x * V[4] - w * V[5] + z * V[6] + w * V[7] - 2.f * x * V[8]);
  vq[2] = 2.f * (-2.f * y * V[0] + x * V[1] + w * V[2] + x * V[3] + z * V[5] - w * V[6] + z * V[7] - 2.f * y * V[8]);
  vq[3] = 2.f * (-2.f * z * V[0] - w * V[1] + x * V[2] + w * V[3] - 2.f * z * V[4] + y * V[5] + x * V[6] + y * V[7]);
  // gsplat normalisation vjp: v_qa = (vq - (vq.qn) qn) / |qa|
  const float dqn = vq[0] * w + vq[1] * x + vq[2] * y + vq[3] * z;
  float vqa[4] = {(vq[0] - dqn * w) * qinv, (vq[1] - dqn * x) * qinv, (vq[2] - dqn * y) * qinv,
                  (vq[3] - dqn * z) * qinv};
#pragma unroll
  for (int k = 0; k < 3; ++k) out[k] = v_m[k];
  if (input_mode == GSR_INPUT_GSPLAT) {   // gradients w.r.t. the activated gsplat inputs
#pragma unroll
    for (int k = 0; k < 3; ++k) out[3 + k] = v_s[k];
#pragma unroll
    for (int k = 0; k < 4; ++k) out[6 + k] = vqa[k];
#pragma unroll
    for (int k = 0; k < 3; ++k) out[10 + k] = v_col[k];
    out[13] = v_op;
    return;
  }
  // adapter: qa = q / (r + 1e-8), r = |q|:  v_q = v_qa/(r+eps) - q (q.v_qa) / (r (r+eps)^2)
  const float den = a.rq + 1e-8f;
  const float qdot = a.qraw[0] * vqa[0] + a.qraw[1] * vqa[1] + a.qraw[2] * vqa[2] + a.qraw[3] * vqa[3];
  const float coef = qdot / (a.rq * den * den);
#pragma unroll
  for (int k = 0; k < 3; ++k) out[3 + k] = v_s[k] * a.s[k];
#pragma unroll
  for (int k = 0; k < 4; ++k) out[6 + k] = vqa[k] / den - a.qraw[k] * coef;
#pragma unroll
  for (int k = 0; k < 3; ++k) out[10 + k] = (a.craw[k] >= 0.f && a.craw[k] <= 1.f) ? v_col[k] : 0.f;
  out[13] = v_op * a.op * (1.f - a.op);
}

// The Gaussians a band share's backward gives a gradient: those with at least one list entry
// before its tile's cut (tile_end), i.e. a partial row the raster backward wrote.  (A nonzero
// rect is not enough: in config 5's dense centre nearly every Gaussian reaches a band's tiles,
// but the walks stop early and ~11 % of them get a gradient.)  One workgroup per busy tile
// flags its consumed entries' Gaussians; the flags are then compacted into the row block.
__global__ __launch_bounds__(kBwdThreads) void k_mark_touched(const int32_t* __restrict__ sorted_ids,
                                                              const int32_t* __restrict__ tile_offset,
                                                              const int32_t* __restrict__ tile_end,
                                                              const int32_t* __restrict__ order,
                                                              const gsr_bin_stats* __restrict__ stats, int64_t N,
                                                              uint8_t* __restrict__ flag) {
  if ((int)blockIdx.x >= stats->n_busy || stats->overflow) return;
  const int ct = order[blockIdx.x];
  const int b = tile_offset[ct], e = tile_end[ct];
  for (int k = b + (int)threadIdx.x; k < e; k += kBwdThreads) flag[sorted_ids[k] % N] = 1;
}

// One returning atomic per wave claims the wave's rows (positions follow arrival order; the
// exchange's sum is per row, so the order does not change a bit of the result).  A forward
// whose bounds did not hold (stats->overflow; k_mark_touched flagged nothing) sets the header
// past the cap instead, so the exchange reports GSR_OVF_EXCHANGE and NaN-fills the gradient
// rather than summing a share that silently lacks this rank's rows.
__global__ __launch_bounds__(kBwdThreads) void k_touched_rows(const uint8_t* __restrict__ flag, int64_t N, int64_t cap,
                                                              float* __restrict__ block,
                                                              const gsr_bin_stats* __restrict__ stats) {
  if (stats->overflow) {
    if (blockIdx.x == 0 && threadIdx.x == 0)
      reinterpret_cast<int32_t*>(block)[0] = (int32_t)min<int64_t>(cap + 1, INT32_MAX);
    return;
  }
  const int64_t n = (int64_t)blockIdx.x * kBwdThreads + threadIdx.x;
  const bool any = n < N && flag[n] != 0;
  const unsigned long long m = __ballot(any);
  const int lane = threadIdx.x & 63;
  int base = 0;
  if (lane == 0 && m) base = atomicAdd(reinterpret_cast<int32_t*>(block), __popcll(m));
  base = __builtin_amdgcn_readfirstlane(base);
  if (any) {
    const int64_t i = base + __popcll(m & ((1ull << lane) - 1ull));
    if (i < cap) {
      int32_t* row = reinterpret_cast<int32_t*>(block + (1 + i) * GSR_ROW_FLOATS);
      row[0] = (int32_t)n;
      row[1] = 0;
    }
  }
}

__global__ void k_zero_u32(uint32_t* __restrict__ p, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) p[i] = 0u;
}

__global__ void k_rows_header(float* __restrict__ block, int64_t cap) {
  int32_t* h = reinterpret_cast<int32_t*>(block);
  if (threadIdx.x < GSR_ROW_FLOATS) h[threadIdx.x] = threadIdx.x == 1 ? (int32_t)min<int64_t>(cap, INT32_MAX) : 0;
}

// v_params += rank r's rows (a rank lists an n once: plain read-add-writes, no atomics; the
// ranks follow in launch order, so every rank sums in the same order).  Any header over its
// cap: the exchange lost rows, so the result is NaN and the sticky status says why.
__global__ __launch_bounds__(kBwdThreads) void k_rows_scatter_add(const float* __restrict__ blocks, int world,
                                                                  int64_t cap, int r, float* __restrict__ v_params,
                                                                  int64_t N, int32_t* __restrict__ status) {
  bool bad = false;
  for (int q = 0; q < world; ++q) bad |= reinterpret_cast<const int32_t*>(blocks + (int64_t)q * (cap + 1) * GSR_ROW_FLOATS)[0] > cap;
  const int64_t i = (int64_t)blockIdx.x * kBwdThreads + threadIdx.x;
  if (bad) {
    if (r == 0) {
      for (int64_t k = i; k < N * 14; k += (int64_t)gridDim.x * kBwdThreads) v_params[k] = __builtin_nanf("");
      if (i == 0 && status != nullptr) atomicOr(status, GSR_OVF_EXCHANGE);
    }
    return;
  }
  const float* blk = blocks + (int64_t)r * (cap + 1) * GSR_ROW_FLOATS;
  const int64_t count = reinterpret_cast<const int32_t*>(blk)[0];
  if (i >= count) return;
  const float4* row = reinterpret_cast<const float4*>(blk + (1 + i) * GSR_ROW_FLOATS);
  const float4 a = row[0], b = row[1], c = row[2], d = row[3];
  const int64_t n = __float_as_int(a.x);
  if (n < 0 || n >= N) return;
  float* o = v_params + n * 14;
  const float g[14] = {a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y, c.z, c.w, d.x, d.y, d.z, d.w};
#pragma unroll
  for (int k = 0; k < 14; ++k) o[k] += g[k];
}

// The 2D chain of one (set f, Gaussian n) from its camera-summed partials.
__device__ __forceinline__ void chain2d(const float* __restrict__ prm, const float (&acc)[kPartial],
                                        float* __restrict__ out) {
  const Geo2D g = geo2d(prm);
  const float va = acc[2], vb = acc[3], vc = acc[4];
  const float C = g.cs, S = g.sn;
  const float C2 = C * C, S2 = S * S, CS = C * S;
  const float v_ia = va * C2 + vb * 2.f * CS + vc * S2;
  const float v_ib = va * S2 - vb * 2.f * CS + vc * C2;
  const float dd = g.ia - g.ib;
  const float v_th = dd * (-2.f * CS * va + 2.f * (C2 - S2) * vb + 2.f * CS * vc);
  const float v_lsx = v_ia * (-4.f * g.sx * g.ia * g.ia) * g.sx;
  const float v_lsy = v_ib * (-4.f * g.sy * g.ib * g.ib) * g.sy;
  out[0] = acc[0];
  out[1] = acc[1];
  out[2] = v_lsx;
  out[3] = v_lsy;
  out[4] = v_th;
#pragma unroll
  for (int k = 0; k < 3; ++k) out[5 + k] = (g.craw[k] >= 0.f && g.craw[k] <= 1.f) ? acc[6 + k] : 0.f;
  out[8] = acc[5] * g.op * (1.f - g.op);
}

// 2D: a workgroup owns 256 consecutive Gaussians n of one parameter set f (the set's cameras
// [set_begin[f], set_begin[f+1])).  Inside one projection workgroup (kProjPerBlock, a multiple
// of 256) the (c,n) items of consecutive n own consecutive emission ranges (alloc_offsets),
// so per camera the workgroup's partial rows are one run [lo, hi).  The run is read through
// LDS in coalesced float4 rounds and every thread sums its own rows from there, cameras in
// order and each camera's rows in rect order (deterministic).  The camera-summed partials are
// chained once: the 2D chain is linear in them and the same for every view.  Thread-per-
// Gaussian gathers of the 48-B rows at scattered addresses took 2.10 ms at config 4, the
// staged reads 1.54 ms.  Correct for any layout: [lo, hi) is the hull of the workgroup's
// rows, whatever else lies inside it.
constexpr int kStageRows = 512;   // rows per LDS round (18 KB)
__global__ __launch_bounds__(kBwdThreads) void k_project2d_bwd_staged(
    const float* __restrict__ params, int64_t N, int64_t stride, int64_t set_stride,
    const int32_t* __restrict__ set_begin, int F, int n_cam, int tw, int th, const uint2* __restrict__ rect,
    const int32_t* __restrict__ isect_offset, const int32_t* __restrict__ isect_count,
    const uint64_t* __restrict__ tile_cut, const float* __restrict__ partial, const gsr_bin_stats* __restrict__ stats,
    float* __restrict__ v_params, int first_only) {
  __shared__ float s_rows[kPartialStride * kStageRows];
  __shared__ int s_lo, s_hi;
  const int f = blockIdx.y;
  const int64_t n = (int64_t)blockIdx.x * kBwdThreads + threadIdx.x;
  const bool own = n < N;
  // the forward's bounds did not hold: NaN rows, no partial row read (loaded with the first
  // gathers, tested in the camera loop: no round trip of its own)
  const bool ovf = stats != nullptr && stats->overflow != 0;
  const int c0 = set_begin ? set_begin[f] : 0;
  // (rows2d_per_set: the set's summed rows are its first camera's)
  const int c1 = first_only ? min(set_begin[f + 1], c0 + 1) : set_begin ? set_begin[f + 1] : n_cam;
  static_assert(kPartialStride * kStageRows % kBwdThreads == 0, "whole rounds of floats per thread");
  float acc[kPartial];
#pragma unroll
  for (int v = 0; v < kPartial; ++v) acc[v] = 0.f;
  bool any = false;
  for (int c = c0; c < c1; ++c) {
    const int64_t cn = (int64_t)c * N + n;
    const int cnt = own && !ovf ? isect_count[cn] : 0;
    uint2 r = make_uint2(0u, 0u);
    int off = 0;
    if (cnt > 0) {
      r = rect[cn];
      off = isect_offset[cn];
      any = true;
    }
    if (threadIdx.x == 0) {
      s_lo = 0x7fffffff;
      s_hi = -0x7fffffff - 1;
    }
    __syncthreads();
    if (cnt > 0) {
      atomicMin(&s_lo, off);
      atomicMax(&s_hi, off + cnt);
    }
    __syncthreads();
    const int lo = s_lo, hi = s_hi;
    const uint64_t key = ((uint64_t)(uint32_t)cn << 32) | (uint64_t)(uint32_t)cn;   // sort_key, index order
    const int x0 = r.x & 0xffff, x1 = r.x >> 16, y0 = r.y & 0xffff;
    const int w = max(x1 - x0, 1);
    const int64_t ct_base = (int64_t)c * tw * th;
    for (int r0 = lo; r0 < hi; r0 += kStageRows) {
      const int nr = min(kStageRows, hi - r0);
      __syncthreads();   // the previous round's rows are consumed
      {
        constexpr int kPer = kPartialStride * kStageRows / kBwdThreads;   // floats per thread (coalesced)
        float v[kPer];
        const float* src = partial + (int64_t)kPartialStride * r0;
#pragma unroll
        for (int u = 0; u < kPer; ++u) {
          const int i = u * kBwdThreads + threadIdx.x;
          v[u] = i < kPartialStride * nr ? src[i] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < kPer; ++u) s_rows[u * kBwdThreads + threadIdx.x] = v[u];
      }
      __syncthreads();
      if (cnt > 0) {
        // this thread's rows j with off + j in [r0, r0 + nr), in order
        const int ja = max(0, r0 - off), jb = min(cnt, r0 + nr - off);
        int ty = y0 + ja / w, tx = x0 + ja % w;
        for (int j = ja; j < jb; ++j) {
          if (key < tile_cut[ct_base + ty * tw + tx]) {
            const float* sr = s_rows + kPartialStride * (off + j - r0);
#pragma unroll
            for (int q = 0; q < kPartial; ++q) acc[q] += sr[q];
          }
          if (++tx == x1) {
            tx = x0;
            ++ty;
          }
        }
      }
    }
    __syncthreads();   // s_lo / s_hi are reset for the next camera
  }
  if (!own) return;
  const int64_t fn = (int64_t)f * N + n;
  float* out = v_params + fn * 9;
  if (ovf) {
#pragma unroll
    for (int k = 0; k < 9; ++k) out[k] = __builtin_nanf("");
    return;
  }
  if (!any) {
#pragma unroll
    for (int k = 0; k < 9; ++k) out[k] = 0.f;
    return;
  }
  chain2d(params + (int64_t)f * set_stride + n * stride, acc, out);
}

}  // namespace gsr

using namespace gsr;

extern "C" {

int gsr3d_project_bwd(const float* params, int64_t N, int64_t row_stride, const float* viewmats, const float* Ks,
                      int C, int width, int height, float eps2d, int input_mode, const float* depth,
                      const uint32_t* rect,
                      const int32_t* isect_offset, const int32_t* isect_count, const uint64_t* tile_cut,
                      const float* partial, int64_t n_begin, int64_t n_end, const gsr_bin_stats* stats,
                      float* v_params, void* stream) {
  GSR_REQUIRE(N >= 0 && C >= 1 && width > 0 && height > 0, "gsr3d_project_bwd: bad arguments");
  GSR_REQUIRE(row_stride >= 14, "gsr3d_project_bwd: row_stride < 14");
  GSR_REQUIRE(input_mode == GSR_INPUT_ADAPTER || input_mode == GSR_INPUT_GSPLAT,
              "gsr3d_project_bwd: bad input_mode %d", input_mode);
  if (n_end < 0) n_end = N;
  GSR_REQUIRE(n_begin >= 0 && n_begin <= n_end && n_end <= N, "gsr3d_project_bwd: bad Gaussian range [%lld,%lld) of %lld",
              (long long)n_begin, (long long)n_end, (long long)N);
  if (n_end == n_begin) return GSR_OK;
  const int tw = ceil_div(width, kTile), th = ceil_div(height, kTile);
  const int CPB = C < kBwdThreads ? C : kBwdThreads;   // camera slots per Gaussian
  const int G = kBwdThreads / CPB;                       // Gaussians per workgroup
  hipLaunchKernelGGL(k_project3d_bwd<false>, dim3(ceil_div(n_end - n_begin, G)), dim3(kBwdThreads), 0,
                     (hipStream_t)stream, params, N, row_stride, viewmats, Ks, C, width, height, eps2d, input_mode, tw,
                     th, (const uint2*)rect, isect_offset, isect_count, depth, tile_cut, partial, CPB, G, n_begin,
                     n_end, stats, v_params, nullptr, (int64_t)0);
  GSR_LAUNCH_CHECK("k_project3d_bwd");
  return GSR_OK;
}

int gsr3d_touched_rows(const int32_t* sorted_ids, const int32_t* tile_offset, const int32_t* tile_end,
                       const int32_t* tile_order, const gsr_bin_stats* stats, int32_t n_busy, int64_t N, int64_t cap,
                       uint8_t* flags, float* block, void* stream) {
  GSR_REQUIRE(N >= 0 && n_busy >= 0 && cap >= 0 && block != nullptr, "gsr3d_touched_rows: bad arguments");
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(k_rows_header, dim3(1), dim3(64), 0, s, block, cap);
  GSR_LAUNCH_CHECK("k_rows_header");
  if (N == 0 || n_busy == 0) return GSR_OK;
  GSR_REQUIRE(sorted_ids && tile_offset && tile_end && tile_order && stats && flags, "gsr3d_touched_rows: null buffer");
  const int64_t words = ceil_div(N, (int64_t)4);
  hipLaunchKernelGGL(k_zero_u32, dim3((unsigned)std::min<int64_t>(ceil_div(words, (int64_t)kBwdThreads), 1024)),
                     dim3(kBwdThreads), 0, s, (uint32_t*)flags, words);
  GSR_LAUNCH_CHECK("k_zero_u32");
  hipLaunchKernelGGL(k_mark_touched, dim3(n_busy), dim3(kBwdThreads), 0, s, sorted_ids, tile_offset, tile_end,
                     tile_order, stats, N, flags);
  GSR_LAUNCH_CHECK("k_mark_touched");
  hipLaunchKernelGGL(k_touched_rows, dim3(ceil_div(N, kBwdThreads)), dim3(kBwdThreads), 0, s, flags, N, cap, block,
                     stats);
  GSR_LAUNCH_CHECK("k_touched_rows");
  return GSR_OK;
}

int gsr3d_project_bwd_rows(const float* params, int64_t N, int64_t row_stride, const float* viewmats, const float* Ks,
                           int C, int width, int height, float eps2d, int input_mode, const float* depth,
                           const uint32_t* rect, const int32_t* isect_offset, const int32_t* isect_count,
                           const uint64_t* tile_cut, const float* partial, const gsr_bin_stats* stats, int64_t cap,
                           float* block, void* stream) {
  GSR_REQUIRE(N >= 0 && C >= 1 && width > 0 && height > 0 && cap >= 0 && block != nullptr,
              "gsr3d_project_bwd_rows: bad arguments");
  GSR_REQUIRE(row_stride >= 14, "gsr3d_project_bwd_rows: row_stride < 14");
  GSR_REQUIRE(input_mode == GSR_INPUT_ADAPTER || input_mode == GSR_INPUT_GSPLAT,
              "gsr3d_project_bwd_rows: bad input_mode %d", input_mode);
  if (N == 0 || cap == 0) return GSR_OK;
  const int tw = ceil_div(width, kTile), th = ceil_div(height, kTile);
  const int CPB = C < kBwdThreads ? C : kBwdThreads;
  const int G = kBwdThreads / CPB;
  // the grid covers cap rows; workgroups past the header's count exit at once
  hipLaunchKernelGGL(k_project3d_bwd<true>, dim3(ceil_div(cap, G)), dim3(kBwdThreads), 0, (hipStream_t)stream, params,
                     N, row_stride, viewmats, Ks, C, width, height, eps2d, input_mode, tw, th, (const uint2*)rect,
                     isect_offset, isect_count, depth, tile_cut, partial, CPB, G, (int64_t)0, N, stats,
                     (float*)nullptr, block, cap);
  GSR_LAUNCH_CHECK("k_project3d_bwd<rows>");
  return GSR_OK;
}

int gsr_rows_scatter_add(const float* blocks, int world, int64_t cap, float* v_params, int64_t N, int32_t* status,
                         void* stream) {
  GSR_REQUIRE(blocks != nullptr && v_params != nullptr && world >= 1 && cap >= 0 && N >= 0,
              "gsr_rows_scatter_add: bad arguments");
  if (N == 0) return GSR_OK;
  // the grid covers cap rows and (for the NaN fill) is grid-strided over v_params
  const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(ceil_div(std::max<int64_t>(cap, 1), kBwdThreads), 1 << 20));
  for (int r = 0; r < world; ++r) {
    hipLaunchKernelGGL(k_rows_scatter_add, dim3(grid), dim3(kBwdThreads), 0, (hipStream_t)stream, blocks, world, cap, r,
                       v_params, N, status);
    GSR_LAUNCH_CHECK("k_rows_scatter_add");
  }
  return GSR_OK;
}

int gsr2d_project_bwd(const float* params, int64_t N, int64_t row_stride, int64_t set_stride,
                      const int32_t* set_begin, int F, int C, int width, int height,
                      const uint32_t* rect, const int32_t* isect_offset, const int32_t* isect_count,
                      const uint64_t* tile_cut, const float* partial, const gsr_bin_stats* stats, float* v_params,
                      void* stream) {
  GSR_REQUIRE(N >= 0 && width > 0 && height > 0, "gsr2d_project_bwd: bad arguments");
  GSR_REQUIRE(C >= 1 && F >= 1 && (set_begin != nullptr || F == 1), "gsr2d_project_bwd: bad C=%d / F=%d", C, F);
  GSR_REQUIRE(row_stride >= 9, "gsr2d_project_bwd: row_stride < 9");
  GSR_REQUIRE(F == 1 || set_stride >= N * row_stride, "gsr2d_project_bwd: set_stride < N*row_stride");
  if (N == 0) return GSR_OK;
  const int tw = ceil_div(width, kTile), th = ceil_div(height, kTile);
  GSR_REQUIRE(F <= 65535, "gsr2d_project_bwd: F=%d > 65535 parameter sets", F);
  hipLaunchKernelGGL(k_project2d_bwd_staged, dim3(ceil_div(N, kBwdThreads), F), dim3(kBwdThreads), 0,
                     (hipStream_t)stream, params, N, row_stride, set_stride, set_begin, F, C, tw, th,
                     (const uint2*)rect, isect_offset, isect_count, tile_cut, partial, stats, v_params,
                     rows2d_per_set(set_begin, F, C) ? 1 : 0);
  GSR_LAUNCH_CHECK("k_project2d_bwd_staged");
  return GSR_OK;
}

}  // extern "C"
