// Gaussian parameter head + pose transform, per Gaussian, fused.
//
// Restates PoseSplatter.get_gaussian_params_from_volume_unified after its MLP
// (src/model.py:209-254) and apply_pose_transform_3d (src/model.py:258-298) with its
// quaternion helpers (src/model.py:378-421), forward and backward, in one thread per
// Gaussian.  The reference turns each quaternion into a matrix, rotates it, and recovers
// the quaternion with a batched float64 torch.linalg.eigh of a 4x4 (Bar-Itzhack) matrix;
// here that eigenproblem is solved in registers by cyclic Jacobi in float64, and its
// backward uses the same (skew-projected) eigenvector derivative torch applies.  The
// reference's matrix helper is reproduced as written (its [1][1] entry is 1 + q00 - q00 and
// its [1][0] entry repeats [0][1]); the result is therefore the reference's, not a textbook
// quaternion product.
//
// Also the mask-threshold search of src/model.py:185-197 (the host-synchronising while
// loops) as one device workgroup, and the ordered compaction of the selected voxels.
#include "gsr_common.h"

namespace gsr {

struct HeadConsts {
  float mt;          // final mask threshold (as float: torch subtracts the scalar in fp32)
  float pt;          // prob_threshold
  float inv1mpt;     // float(1 / (1 - pt))
  float clip_lo, clip_hi;
  float two_vs;      // float(2 * voxel_size)
  float c, s;        // float(cos angle), float(sin angle)
  int pose;          // 1: apply the pose transform
};

// ----------------------------------------------------------------- float64 4x4 Jacobi
// Symmetric A (row-major 4x4) -> eigenvalues lam[4] and eigenvectors V (columns).
__device__ __forceinline__ void jacobi4(double A[4][4], double lam[4], double V[4][4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) V[i][j] = i == j ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 24; ++sweep) {
    double off = 0.0, diag = 0.0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      diag += A[i][i] * A[i][i];
#pragma unroll
      for (int j = i + 1; j < 4; ++j) off += A[i][j] * A[i][j];
    }
    if (off <= 1e-36 * diag || off == 0.0) break;
#pragma unroll
    for (int p = 0; p < 3; ++p) {
#pragma unroll
      for (int q = p + 1; q < 4; ++q) {
        const double apq = A[p][q];
        if (apq == 0.0) continue;
        const double theta = (A[q][q] - A[p][p]) / (2.0 * apq);
        const double t = (theta >= 0.0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
        const double cs = 1.0 / sqrt(t * t + 1.0);
        const double sn = t * cs;
#pragma unroll
        for (int k = 0; k < 4; ++k) {   // A <- J^T A J (columns p,q then rows p,q)
          const double akp = A[k][p], akq = A[k][q];
          A[k][p] = cs * akp - sn * akq;
          A[k][q] = sn * akp + cs * akq;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const double apk = A[p][k], aqk = A[q][k];
          A[p][k] = cs * apk - sn * aqk;
          A[q][k] = sn * apk + cs * aqk;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const double vkp = V[k][p], vkq = V[k][q];
          V[k][p] = cs * vkp - sn * vkq;
          V[k][q] = sn * vkp + cs * vkq;
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) lam[i] = A[i][i];
}

// quaternion_matrix_torch_batch (src/model.py:378-403), 3x3 block, float64.  Returns false
// for the near-zero quaternion (identity, no gradient).
struct QuatMat {
  double qs[4];   // q * sqrt(2/n)
  double f, n;
  bool ok;
};

__device__ __forceinline__ QuatMat quat_matrix_ref(const float qin[4], double M[3][3]) {
  QuatMat r;
  double q[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) q[k] = (double)qin[k];
  r.n = q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3];
  r.ok = !(r.n < 4.0 * 2.220446049250313e-16);
  r.f = r.ok ? sqrt(2.0 / r.n) : 1.0;
#pragma unroll
  for (int k = 0; k < 4; ++k) r.qs[k] = q[k] * r.f;
  if (!r.ok) {
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) M[i][j] = i == j ? 1.0 : 0.0;
    return r;
  }
  const double* u = r.qs;
  const double O00 = u[0] * u[0], O11 = u[1] * u[1], O22 = u[2] * u[2], O33 = u[3] * u[3];
  const double O12 = u[1] * u[2], O30 = u[3] * u[0], O13 = u[1] * u[3], O20 = u[2] * u[0];
  const double O23 = u[2] * u[3], O10 = u[1] * u[0];
  M[0][0] = (1.0 - O22) - O33;
  M[0][1] = O12 - O30;
  M[0][2] = O13 + O20;
  M[1][0] = O12 - O30;
  M[1][1] = (1.0 + O00) - O00;
  M[1][2] = O23 - O10;
  M[2][0] = O13 - O20;
  M[2][1] = O23 + O10;
  M[2][2] = (1.0 - O11) - O22;
  return r;
}

// Everything the quaternion backward needs, recomputed from the input quaternion.
struct PoseQuat {
  QuatMat qm;
  float Mf[3][3];   // float32 matrix (quaternion_matrix_torch_batch returns float32)
  float Rm[3][3];   // rot_mat_2 @ Mf, float32
  double lam[4], V[4][4];
  int top;
  bool flip;
  float qout[4];
};

__device__ __forceinline__ void pose_quat_fwd(const float qin[4], float c, float s, PoseQuat& P) {
  double M[3][3];
  P.qm = quat_matrix_ref(qin, M);
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) P.Mf[i][j] = (float)M[i][j];
  // einsum("ij,bjk->bik", rot_mat_2, r) in float32; rot_mat_2 rows: (c,-s,0,0) (s,c,0,0) (0,0,1,0)
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    P.Rm[0][k] = __fadd_rn(__fmul_rn(c, P.Mf[0][k]), __fmul_rn(-s, P.Mf[1][k]));
    P.Rm[1][k] = __fadd_rn(__fmul_rn(s, P.Mf[0][k]), __fmul_rn(c, P.Mf[1][k]));
    P.Rm[2][k] = P.Mf[2][k];
  }
  // quaternion_from_matrix_torch_batch (src/model.py:406-421)
  double m[3][3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) m[i][j] = (double)P.Rm[i][j];
  double K[4][4] = {
      {m[0][0] - m[1][1] - m[2][2], m[0][1] + m[1][0], m[0][2] + m[2][0], m[2][1] - m[1][2]},
      {m[0][1] + m[1][0], m[1][1] - m[0][0] - m[2][2], m[1][2] + m[2][1], m[0][2] - m[2][0]},
      {m[0][2] + m[2][0], m[1][2] + m[2][1], m[2][2] - m[0][0] - m[1][1], m[1][0] - m[0][1]},
      {m[2][1] - m[1][2], m[0][2] - m[2][0], m[1][0] - m[0][1], m[0][0] + m[1][1] + m[2][2]}};
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) K[i][j] = K[i][j] / 3.0;
  jacobi4(K, P.lam, P.V);
  // largest eigenvalue (eigh's last column) moved to slot 3 with static indexing only
  double best = P.lam[0];
  int top = 0;
#pragma unroll
  for (int i = 1; i < 4; ++i) {
    const bool gt = P.lam[i] > best;
    best = gt ? P.lam[i] : best;
    top = gt ? i : top;
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    if (top == i) {
      const double l = P.lam[i];
      P.lam[i] = P.lam[3];
      P.lam[3] = l;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const double v = P.V[k][i];
        P.V[k][i] = P.V[k][3];
        P.V[k][3] = v;
      }
    }
  }
  P.top = 3;
  // V[:, :, -1] reordered [3,0,1,2]: (w,x,y,z); w < 0 flips the sign
  double q[4] = {P.V[3][3], P.V[0][3], P.V[1][3], P.V[2][3]};
  P.flip = q[0] < 0.0;
#pragma unroll
  for (int k = 0; k < 4; ++k) P.qout[k] = (float)(P.flip ? -q[k] : q[k]);
}

// d(qout) -> d(qin), the reverse of pose_quat_fwd (torch's autograd chain, float64 where
// the reference computes in float64, float32 where it casts).
__device__ __forceinline__ void pose_quat_bwd(const float qin[4], float c, float s, const PoseQuat& P,
                                              const float gq[4], float gqin[4]) {
  // un-flip, un-reorder: g_v in eigenvector coordinates (x,y,z,w)
  const double sg = P.flip ? -1.0 : 1.0;
  const double gv[4] = {sg * (double)gq[1], sg * (double)gq[2], sg * (double)gq[3], sg * (double)gq[0]};
  // eigh backward, skew-projected: gK = sum_i a_i / (2 (l_top - l_i)) (v_i v_top^T + v_top v_i^T)
  double gK[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) gK[i][j] = 0.0;
  constexpr int t = 3;   // pose_quat_fwd keeps the top eigenpair in slot 3
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    double a = 0.0;
#pragma unroll
    for (int k = 0; k < 4; ++k) a += P.V[k][i] * gv[k];
    const double w = 0.5 * a / (P.lam[t] - P.lam[i]);
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int cc = 0; cc < 4; ++cc) gK[r][cc] += w * (P.V[r][i] * P.V[cc][t] + P.V[r][t] * P.V[cc][i]);
  }
  double G[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) G[i][j] = gK[i][j] / 3.0;
  double gm[3][3];
  gm[0][0] = G[0][0] - G[1][1] - G[2][2] + G[3][3];
  gm[1][1] = -G[0][0] + G[1][1] - G[2][2] + G[3][3];
  gm[2][2] = -G[0][0] - G[1][1] + G[2][2] + G[3][3];
  gm[0][1] = G[0][1] + G[1][0] - G[2][3] - G[3][2];
  gm[1][0] = G[0][1] + G[1][0] + G[2][3] + G[3][2];
  gm[0][2] = G[0][2] + G[2][0] + G[1][3] + G[3][1];
  gm[2][0] = G[0][2] + G[2][0] - G[1][3] - G[3][1];
  gm[1][2] = G[1][2] + G[2][1] - G[0][3] - G[3][0];
  gm[2][1] = G[1][2] + G[2][1] + G[0][3] + G[3][0];
  // .double() of the float32 einsum output: gradient back to float32; einsum backward R2^T g
  float gR[3][3], gMf[3][3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) gR[i][j] = (float)gm[i][j];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    gMf[0][k] = __fadd_rn(__fmul_rn(c, gR[0][k]), __fmul_rn(s, gR[1][k]));
    gMf[1][k] = __fadd_rn(__fmul_rn(-s, gR[0][k]), __fmul_rn(c, gR[1][k]));
    gMf[2][k] = gR[2][k];
  }
  if (!P.qm.ok) {
#pragma unroll
    for (int k = 0; k < 4; ++k) gqin[k] = 0.f;
    return;
  }
  // res.to(float32) backward (to float64), then the outer-product entries
  double g[3][3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) g[i][j] = (double)gMf[i][j];
  double gO[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) gO[i][j] = 0.0;
  gO[2][2] -= g[0][0];
  gO[3][3] -= g[0][0];
  gO[1][2] += g[0][1];
  gO[3][0] -= g[0][1];
  gO[1][3] += g[0][2];
  gO[2][0] += g[0][2];
  gO[1][2] += g[1][0];
  gO[3][0] -= g[1][0];
  gO[2][3] += g[1][2];
  gO[1][0] -= g[1][2];
  gO[1][3] += g[2][0];
  gO[2][0] -= g[2][0];
  gO[2][3] += g[2][1];
  gO[1][0] += g[2][1];
  gO[1][1] -= g[2][2];
  gO[2][2] -= g[2][2];
  // O = u u^T, u = q f: g_u_i = sum_j (gO_ij + gO_ji) u_j
  const double* u = P.qm.qs;
  double gu[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    double a = 0.0;
#pragma unroll
    for (int j = 0; j < 4; ++j) a += (gO[i][j] + gO[j][i]) * u[j];
    gu[i] = a;
  }
  // u = q sqrt(2/n), n = |q|^2:  g_q = f g_u - (f/n) (g_u . q) q
  double q[4], gq_dot = 0.0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    q[k] = (double)qin[k];
    gq_dot += gu[k] * q[k];
  }
  const double f = P.qm.f, n = P.qm.n;
#pragma unroll
  for (int k = 0; k < 4; ++k) gqin[k] = (float)(f * gu[k] - (f / n) * gq_dot * q[k]);
}

__device__ __forceinline__ float sigmoidf_ref(float x) { return 1.f / (1.f + expf(-x)); }

// ---------------------------------------------------------------- head 3D forward / backward
// net row (src/model.py:213-215 split): quats 0:4, scales 4:7, opacity 7 (unused), colors 8:11,
// delta_means 11:14.  Output row (renderer layout): means 0:3, log_scales 3:6, quats 6:10,
// colors 10:13, logit_opacity 13.
__global__ __launch_bounds__(256) void k_head3d_fwd(const float* __restrict__ net, int64_t net_stride,
                                                   const float* __restrict__ v0, const float* __restrict__ grid,
                                                   const float* __restrict__ scale, int64_t N, HeadConsts k,
                                                   const float* __restrict__ p3d, float* __restrict__ out) {
  const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  const float* r = net + n * net_stride;
  float* o = out + n * 14;
  // colours: sigmoid then clamp(color_clip)
#pragma unroll
  for (int k2 = 0; k2 < 3; ++k2) o[10 + k2] = fminf(fmaxf(sigmoidf_ref(r[8 + k2]), k.clip_lo), k.clip_hi);
  const float sc = scale[0];
#pragma unroll
  for (int k2 = 0; k2 < 3; ++k2) o[3 + k2] = r[4 + k2] + sc;
  // logit(clamp((1/(1-pt)) (sigmoid(v0 - mt) - pt), 1e-6, 1 - 1e-6))
  const float p = sigmoidf_ref(v0[n] - k.mt);
  const float x = fminf(fmaxf(k.inv1mpt * (p - k.pt), 1e-6f), 1.f - 1e-6f);
  o[13] = logf(x / (1.f - x));
  float m[3];
#pragma unroll
  for (int k2 = 0; k2 < 3; ++k2) m[k2] = grid[n * 3 + k2] + k.two_vs * tanhf(r[11 + k2]);
  float q[4] = {r[0], r[1], r[2], r[3]};
  if (k.pose) {
    // means @ rot_mat.T + p_3d; rot_mat rows (c,-s,0) (s,c,0) (0,0,1)
    const float mx = __fadd_rn(__fmul_rn(k.c, m[0]), __fmul_rn(-k.s, m[1]));
    const float my = __fadd_rn(__fmul_rn(k.s, m[0]), __fmul_rn(k.c, m[1]));
    m[0] = mx + p3d[0];
    m[1] = my + p3d[1];
    m[2] = m[2] + p3d[2];
    PoseQuat P;
    pose_quat_fwd(q, k.c, k.s, P);
#pragma unroll
    for (int k2 = 0; k2 < 4; ++k2) q[k2] = P.qout[k2];
  }
#pragma unroll
  for (int k2 = 0; k2 < 3; ++k2) o[k2] = m[k2];
#pragma unroll
  for (int k2 = 0; k2 < 4; ++k2) o[6 + k2] = q[k2];
}

__global__ __launch_bounds__(256) void k_head3d_bwd(const float* __restrict__ net, int64_t net_stride,
                                                   const float* __restrict__ v0, const float* __restrict__ grid,
                                                   int64_t N, HeadConsts k, const float* __restrict__ g_out,
                                                   float* __restrict__ g_net, float* __restrict__ g_v0) {
  const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  const float* r = net + n * net_stride;
  const float* g = g_out + n * 14;
  float* gn = g_net + n * 14;
  // colours: clamp passes where lo <= y <= hi (inclusive), sigmoid' = y (1 - y)
#pragma unroll
  for (int k2 = 0; k2 < 3; ++k2) {
    const float y = sigmoidf_ref(r[8 + k2]);
    const bool pass = y >= k.clip_lo && y <= k.clip_hi;
    gn[8 + k2] = pass ? g[10 + k2] * (y * (1.f - y)) : 0.f;
  }
#pragma unroll
  for (int k2 = 0; k2 < 3; ++k2) gn[4 + k2] = g[3 + k2];
  gn[7] = 0.f;   // the network's opacity column is discarded by the reference
  {
    const float p = sigmoidf_ref(v0[n] - k.mt);
    const float a = k.inv1mpt * (p - k.pt);
    const bool pass = a >= 1e-6f && a <= 1.f - 1e-6f;
    const float x = fminf(fmaxf(a, 1e-6f), 1.f - 1e-6f);
    const float gx = pass ? g[13] / (x * (1.f - x)) : 0.f;
    g_v0[n] = gx * k.inv1mpt * (p * (1.f - p));
  }
  // means: pose rotation transposed, then tanh'
  float gm[3] = {g[0], g[1], g[2]};
  float q[4] = {r[0], r[1], r[2], r[3]};
  float gq[4] = {g[6], g[7], g[8], g[9]};
  if (k.pose) {
    const float gx = __fadd_rn(__fmul_rn(k.c, gm[0]), __fmul_rn(k.s, gm[1]));
    const float gy = __fadd_rn(__fmul_rn(-k.s, gm[0]), __fmul_rn(k.c, gm[1]));
    gm[0] = gx;
    gm[1] = gy;
    PoseQuat P;
    pose_quat_fwd(q, k.c, k.s, P);
    float gqi[4];
    pose_quat_bwd(q, k.c, k.s, P, gq, gqi);
#pragma unroll
    for (int k2 = 0; k2 < 4; ++k2) gq[k2] = gqi[k2];
  }
#pragma unroll
  for (int k2 = 0; k2 < 3; ++k2) {
    const float t = tanhf(r[11 + k2]);
    gn[11 + k2] = gm[k2] * k.two_vs * (1.f - t * t);
  }
#pragma unroll
  for (int k2 = 0; k2 < 4; ++k2) gn[k2] = gq[k2];
}

// Pose transform alone (apply_pose_transform_3d on renderer-layout rows).
__global__ __launch_bounds__(256) void k_pose3d_fwd(const float* __restrict__ params, int64_t stride, int64_t N,
                                                   HeadConsts k, const float* __restrict__ p3d,
                                                   float* __restrict__ out) {
  const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  const float* r = params + n * stride;
  float* o = out + n * 14;
  o[0] = __fadd_rn(__fmul_rn(k.c, r[0]), __fmul_rn(-k.s, r[1])) + p3d[0];
  o[1] = __fadd_rn(__fmul_rn(k.s, r[0]), __fmul_rn(k.c, r[1])) + p3d[1];
  o[2] = r[2] + p3d[2];
  float q[4] = {r[6], r[7], r[8], r[9]};
  PoseQuat P;
  pose_quat_fwd(q, k.c, k.s, P);
#pragma unroll
  for (int k2 = 0; k2 < 3; ++k2) o[3 + k2] = r[3 + k2];
#pragma unroll
  for (int k2 = 0; k2 < 4; ++k2) o[6 + k2] = P.qout[k2];
#pragma unroll
  for (int k2 = 0; k2 < 4; ++k2) o[10 + k2] = r[10 + k2];
}

__global__ __launch_bounds__(256) void k_pose3d_bwd(const float* __restrict__ params, int64_t stride, int64_t N,
                                                   HeadConsts k, const float* __restrict__ g_out,
                                                   float* __restrict__ g_params) {
  const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  const float* r = params + n * stride;
  const float* g = g_out + n * 14;
  float* o = g_params + n * 14;
  o[0] = __fadd_rn(__fmul_rn(k.c, g[0]), __fmul_rn(k.s, g[1]));
  o[1] = __fadd_rn(__fmul_rn(-k.s, g[0]), __fmul_rn(k.c, g[1]));
  o[2] = g[2];
  float q[4] = {r[6], r[7], r[8], r[9]};
  float gq[4] = {g[6], g[7], g[8], g[9]}, gqi[4];
  PoseQuat P;
  pose_quat_fwd(q, k.c, k.s, P);
  pose_quat_bwd(q, k.c, k.s, P, gq, gqi);
#pragma unroll
  for (int k2 = 0; k2 < 3; ++k2) o[3 + k2] = g[3 + k2];
#pragma unroll
  for (int k2 = 0; k2 < 4; ++k2) o[6 + k2] = gqi[k2];
#pragma unroll
  for (int k2 = 0; k2 < 4; ++k2) o[10 + k2] = g[10 + k2];
}

// ---------------------------------------------------------------- threshold search + compaction
constexpr int kSelThreads = 1024;
constexpr int kSelPerBlock = 8192;
constexpr int kSelSteps = 512;   // threshold steps resolved by one histogram pass, each direction

// Selection test of the reference, sigmoid(v - mt) > pt with v - mt and the sigmoid in fp32,
// as one compare: sigmoidf is monotone, so it passes iff fl(v - mt) > x0, where x0 is the
// largest float whose sigmoidf is <= pt (found once by bisection on the float order).
__device__ __forceinline__ bool passes(float v, float mt, float x0) { return (v - mt) > x0; }

struct SelWs {      // workspace layout
  double up[kSelSteps], dn[kSelSteps];   // mt after k raises / k lowers (sequential float64 sums)
  int32_t hist_up[kSelSteps + 1], hist_dn[kSelSteps + 1];
  float x0;
  int32_t pad;
};

__device__ __forceinline__ int32_t float_order(float f) {
  const int32_t i = __float_as_int(f);
  return i >= 0 ? i : (int32_t)(0x80000000u - (uint32_t)i) - 1;   // monotone int key (no NaN)
}
__device__ __forceinline__ float order_float(int32_t k) {
  return __int_as_float(k >= 0 ? k : (int32_t)(0x80000000u - (uint32_t)(k + 1)));
}

// One workgroup: x0, the two threshold tables, zeroed histograms.
__global__ __launch_bounds__(64) void k_select_tables(double mt0, double delta, float pt, SelWs* __restrict__ w) {
  if (threadIdx.x == 0) {
    double u = mt0, d = mt0;
    for (int k = 0; k < kSelSteps; ++k) {
      w->up[k] = u;
      w->dn[k] = d;
      u += delta;
      d -= delta;
    }
    // largest x with sigmoidf(x) <= pt: bisection over the float order in [-1e4, 1e4]
    int32_t lo = float_order(-1e4f), hi = float_order(1e4f);   // invariant: f(lo) <= pt < f(hi)
    if (sigmoidf_ref(order_float(lo)) > pt) {
      w->x0 = -INFINITY;
    } else if (!(sigmoidf_ref(order_float(hi)) > pt)) {
      w->x0 = INFINITY;
    } else {
      while ((int64_t)hi - (int64_t)lo > 1) {
        const int32_t mid = (int32_t)(((int64_t)lo + (int64_t)hi) >> 1);
        if (sigmoidf_ref(order_float(mid)) > pt) hi = mid; else lo = mid;
      }
      w->x0 = order_float(lo);
    }
  }
  for (int i = threadIdx.x; i <= kSelSteps; i += 64) {
    w->hist_up[i] = 0;
    w->hist_dn[i] = 0;
  }
}

// Every voxel: c_up = number of raises it survives (passes at up[k] for k < c_up) and
// c_dn = the first lowering at which it passes (kSelSteps: none in the table); two
// histograms give the pass count at every table threshold in one pass over the volume.
__global__ __launch_bounds__(kSelThreads) void k_select_hist(const float* __restrict__ v0, int64_t M,
                                                             SelWs* __restrict__ w) {
  __shared__ float s_up[kSelSteps], s_dn[kSelSteps];
  __shared__ int32_t s_hu[kSelSteps + 1], s_hd[kSelSteps + 1];
  for (int i = threadIdx.x; i < kSelSteps; i += kSelThreads) {
    s_up[i] = (float)w->up[i];
    s_dn[i] = (float)w->dn[i];
  }
  for (int i = threadIdx.x; i <= kSelSteps; i += kSelThreads) {
    s_hu[i] = 0;
    s_hd[i] = 0;
  }
  __syncthreads();
  const float x0 = w->x0;
  for (int k = 0; k < kSelPerBlock / kSelThreads; ++k) {
    const int64_t i = (int64_t)blockIdx.x * kSelPerBlock + k * kSelThreads + threadIdx.x;
    if (i >= M) break;
    const float v = v0[i];
    int lo = 0, hi = kSelSteps;   // c_up: first k with !passes(v, up[k]) (up increasing)
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (passes(v, s_up[mid], x0)) lo = mid + 1; else hi = mid;
    }
    atomicAdd(&s_hu[lo], 1);
    lo = 0;
    hi = kSelSteps;               // c_dn: first j with passes(v, dn[j]) (dn decreasing)
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (passes(v, s_dn[mid], x0)) hi = mid; else lo = mid + 1;
    }
    atomicAdd(&s_hd[lo], 1);
  }
  __syncthreads();
  for (int i = threadIdx.x; i <= kSelSteps; i += kSelThreads) {
    if (s_hu[i]) atomicAdd(&w->hist_up[i], s_hu[i]);
    if (s_hd[i]) atomicAdd(&w->hist_dn[i], s_hd[i]);
  }
}

// src/model.py:185-197: raise mt by delta while more than max_n pass, then lower it while
// fewer than min_n pass (mt a float64 like the Python float; each test in fp32).  The
// steps inside the tables are read from the histograms; a search that leaves them (or the
// rare second loop after raises) continues with direct counting passes.
__global__ __launch_bounds__(kSelThreads) void k_select_search(const float* __restrict__ v0, int64_t M,
                                                               double delta, int min_n, int max_n, int max_iter,
                                                               const SelWs* __restrict__ w,
                                                               double* __restrict__ mt_out,
                                                               int32_t* __restrict__ info) {
  __shared__ int s_cnt[kSelThreads / 64];
  __shared__ int s_res[2];
  const float x0 = w->x0;
  auto count = [&](double m) {
    const float mf = (float)m;
    int c = 0;
    for (int64_t i = threadIdx.x; i < M; i += kSelThreads) c += passes(v0[i], mf, x0);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) s_cnt[threadIdx.x >> 6] = c;
    __syncthreads();
    int t = 0;
#pragma unroll
    for (int q = 0; q < kSelThreads / 64; ++q) t += s_cnt[q];
    return t;
  };
  if (threadIdx.x == 0) {
    // cnt_up(k) = #{c_up > k}; the raise loop stops at the first k with cnt_up(k) <= max_n
    int tail = (int)M, k = 0;   // tail = #{c_up > k}
    tail -= w->hist_up[0];
    while (k < kSelSteps - 1 && tail > max_n) {
      ++k;
      tail -= w->hist_up[k];
    }
    s_res[0] = k;
    s_res[1] = tail;
  }
  __syncthreads();
  int it = s_res[0];
  int cnt = s_res[1];
  double mt = w->up[it];
  while (cnt > max_n && it < max_iter) {   // beyond the table
    mt += delta;
    cnt = count(mt);
    ++it;
  }
  if (it == 0 && cnt < min_n) {
    // lowering from mt0: cnt_dn(j) = #{c_dn <= j}
    __syncthreads();
    if (threadIdx.x == 0) {
      int j = 0, acc = w->hist_dn[0];
      while (j < kSelSteps - 1 && acc < min_n) {
        ++j;
        acc += w->hist_dn[j];
      }
      s_res[0] = j;
      s_res[1] = acc;
    }
    __syncthreads();
    it = s_res[0];
    cnt = s_res[1];
    mt = w->dn[it];
  }
  while (cnt < min_n && it < max_iter) {
    mt -= delta;
    cnt = count(mt);
    ++it;
  }
  if (threadIdx.x == 0) {
    *mt_out = mt;
    info[0] = cnt;
    info[1] = it;
    info[2] = it >= max_iter;
  }
}

__global__ __launch_bounds__(kSelThreads) void k_select_count(const float* __restrict__ v0, int64_t M,
                                                              const double* __restrict__ mt_in,
                                                              const SelWs* __restrict__ w,
                                                              int32_t* __restrict__ block_cnt) {
  __shared__ int s_cnt[kSelThreads / 64];
  const float mf = (float)*mt_in;
  const float x0 = w->x0;
  const int64_t base = (int64_t)blockIdx.x * kSelPerBlock;
  int c = 0;
#pragma unroll
  for (int k = 0; k < kSelPerBlock / kSelThreads; ++k) {
    const int64_t i = base + k * kSelThreads + threadIdx.x;
    c += i < M && passes(v0[i], mf, x0);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0) s_cnt[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = 0;
#pragma unroll
    for (int q = 0; q < kSelThreads / 64; ++q) t += s_cnt[q];
    block_cnt[blockIdx.x] = t;
  }
}

// Ordered write: block offset = sum of earlier block counts; inside the block, element order
// (sub-rounds of 1024, wave ballots, wave prefix in LDS).
__global__ __launch_bounds__(kSelThreads) void k_select_write(const float* __restrict__ v0, int64_t M,
                                                              const double* __restrict__ mt_in,
                                                              const SelWs* __restrict__ ws,
                                                              const int32_t* __restrict__ block_cnt,
                                                              int64_t* __restrict__ idx) {
  __shared__ int s_w[kSelThreads / 64];
  __shared__ int s_base;
  if (threadIdx.x < 64) {
    int b = 0;
    for (int k = threadIdx.x; k < (int)blockIdx.x; k += 64) b += block_cnt[k];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) b += __shfl_xor(b, o, 64);
    if (threadIdx.x == 0) s_base = b;
  }
  __syncthreads();
  const float mf = (float)*mt_in;
  const float x0 = ws->x0;
  int base = s_base;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int k = 0; k < kSelPerBlock / kSelThreads; ++k) {
    const int64_t i = (int64_t)blockIdx.x * kSelPerBlock + k * kSelThreads + threadIdx.x;
    const bool sel = i < M && passes(v0[i], mf, x0);
    const unsigned long long bal = __ballot(sel);
    const int before = __popcll(bal & ((1ull << lane) - 1ull));
    if (lane == 0) s_w[w] = __popcll(bal);
    __syncthreads();
    int wbase = 0, tot = 0;
#pragma unroll
    for (int q = 0; q < kSelThreads / 64; ++q) {
      wbase += q < w ? s_w[q] : 0;
      tot += s_w[q];
    }
    if (sel) idx[base + wbase + before] = i;
    base += tot;
    __syncthreads();
  }
}

inline HeadConsts make_consts(float mt, float pt, float clip_lo, float clip_hi, float voxel_size, double angle,
                              int pose) {
  HeadConsts k;
  k.mt = mt;
  k.pt = pt;
  k.inv1mpt = (float)(1.0 / (1.0 - (double)pt));
  k.clip_lo = clip_lo;
  k.clip_hi = clip_hi;
  k.two_vs = (float)(2.0 * (double)voxel_size);
  k.c = (float)cos(angle);
  k.s = (float)sin(angle);
  k.pose = pose;
  return k;
}

}  // namespace gsr

using namespace gsr;

extern "C" {

size_t gsr_head_select_workspace(int64_t M) {
  return sizeof(SelWs) + (size_t)ceil_div64(M > 0 ? M : 0, kSelPerBlock) * sizeof(int32_t) + 64;
}

int gsr_head_select(const float* v0, int64_t M, double mask_threshold, float prob_threshold, double delta,
                    int32_t min_n, int32_t max_n, int32_t max_iter, void* ws, size_t ws_bytes, int32_t* info,
                    double* mt_out, int64_t* idx, void* stream) {
  GSR_REQUIRE(M == 0 || (M > 0 && v0 != nullptr), "gsr_head_select: bad volume (M=%lld)", (long long)M);
  GSR_REQUIRE(min_n >= 0 && max_n >= min_n && max_iter > 0, "gsr_head_select: bad min_n/max_n/max_iter");
  GSR_REQUIRE(ws != nullptr && ws_bytes >= gsr_head_select_workspace(M), "gsr_head_select: workspace too small");
  GSR_REQUIRE(((uintptr_t)ws & 7) == 0, "gsr_head_select: workspace must be 8-byte aligned");
  GSR_REQUIRE(info != nullptr && mt_out != nullptr && idx != nullptr, "gsr_head_select: null output");
  hipStream_t s = (hipStream_t)stream;
  SelWs* w = (SelWs*)ws;
  int32_t* block_cnt = (int32_t*)((char*)ws + sizeof(SelWs));
  const int64_t nb = ceil_div64(M, kSelPerBlock);
  hipLaunchKernelGGL(k_select_tables, dim3(1), dim3(64), 0, s, mask_threshold, delta, prob_threshold, w);
  GSR_LAUNCH_CHECK("k_select_tables");
  if (nb > 0) {
    hipLaunchKernelGGL(k_select_hist, dim3((unsigned)nb), dim3(kSelThreads), 0, s, v0, M, w);
    GSR_LAUNCH_CHECK("k_select_hist");
  }
  hipLaunchKernelGGL(k_select_search, dim3(1), dim3(kSelThreads), 0, s, v0, M, delta, min_n, max_n, max_iter,
                     (const SelWs*)w, mt_out, info);
  GSR_LAUNCH_CHECK("k_select_search");
  if (nb > 0) {
    hipLaunchKernelGGL(k_select_count, dim3((unsigned)nb), dim3(kSelThreads), 0, s, v0, M, mt_out,
                       (const SelWs*)w, block_cnt);
    GSR_LAUNCH_CHECK("k_select_count");
    hipLaunchKernelGGL(k_select_write, dim3((unsigned)nb), dim3(kSelThreads), 0, s, v0, M, mt_out,
                       (const SelWs*)w, block_cnt, idx);
    GSR_LAUNCH_CHECK("k_select_write");
  }
  return GSR_OK;
}

int gsr_head3d_fwd(const float* net, int64_t N, int64_t net_stride, const float* v0, const float* grid,
                   const float* scale, float mt, float prob_threshold, float clip_lo, float clip_hi,
                   float voxel_size, int pose, double angle, const float* p3d, float* out, void* stream) {
  GSR_REQUIRE(N >= 0 && net_stride >= 14, "gsr_head3d_fwd: bad N or stride");
  if (N == 0) return GSR_OK;
  GSR_REQUIRE(net && v0 && grid && scale && out && (p3d || !pose), "gsr_head3d_fwd: null pointer");
  const HeadConsts k = make_consts(mt, prob_threshold, clip_lo, clip_hi, voxel_size, angle, pose);
  hipLaunchKernelGGL(k_head3d_fwd, dim3((unsigned)ceil_div64(N, 256)), dim3(256), 0, (hipStream_t)stream, net,
                     net_stride, v0, grid, scale, N, k, p3d, out);
  GSR_LAUNCH_CHECK("k_head3d_fwd");
  return GSR_OK;
}

int gsr_head3d_bwd(const float* net, int64_t N, int64_t net_stride, const float* v0, const float* grid,
                   float mt, float prob_threshold, float clip_lo, float clip_hi, float voxel_size, int pose,
                   double angle, const float* g_out, float* g_net, float* g_v0, void* stream) {
  GSR_REQUIRE(N >= 0 && net_stride >= 14, "gsr_head3d_bwd: bad N or stride");
  if (N == 0) return GSR_OK;
  GSR_REQUIRE(net && v0 && grid && g_out && g_net && g_v0, "gsr_head3d_bwd: null pointer");
  const HeadConsts k = make_consts(mt, prob_threshold, clip_lo, clip_hi, voxel_size, angle, pose);
  hipLaunchKernelGGL(k_head3d_bwd, dim3((unsigned)ceil_div64(N, 256)), dim3(256), 0, (hipStream_t)stream, net,
                     net_stride, v0, grid, N, k, g_out, g_net, g_v0);
  GSR_LAUNCH_CHECK("k_head3d_bwd");
  return GSR_OK;
}

int gsr_pose3d_fwd(const float* params, int64_t N, int64_t row_stride, double angle, const float* p3d,
                   float* out, void* stream) {
  GSR_REQUIRE(N >= 0 && row_stride >= 14, "gsr_pose3d_fwd: bad N or stride");
  if (N == 0) return GSR_OK;
  GSR_REQUIRE(params && p3d && out, "gsr_pose3d_fwd: null pointer");
  const HeadConsts k = make_consts(0.f, 0.f, 0.f, 1.f, 0.f, angle, 1);
  hipLaunchKernelGGL(k_pose3d_fwd, dim3((unsigned)ceil_div64(N, 256)), dim3(256), 0, (hipStream_t)stream, params,
                     row_stride, N, k, p3d, out);
  GSR_LAUNCH_CHECK("k_pose3d_fwd");
  return GSR_OK;
}

int gsr_pose3d_bwd(const float* params, int64_t N, int64_t row_stride, double angle, const float* g_out,
                   float* g_params, void* stream) {
  GSR_REQUIRE(N >= 0 && row_stride >= 14, "gsr_pose3d_bwd: bad N or stride");
  if (N == 0) return GSR_OK;
  GSR_REQUIRE(params && g_out && g_params, "gsr_pose3d_bwd: null pointer");
  const HeadConsts k = make_consts(0.f, 0.f, 0.f, 1.f, 0.f, angle, 1);
  hipLaunchKernelGGL(k_pose3d_bwd, dim3((unsigned)ceil_div64(N, 256)), dim3(256), 0, (hipStream_t)stream, params,
                     row_stride, N, k, g_out, g_params);
  GSR_LAUNCH_CHECK("k_pose3d_bwd");
  return GSR_OK;
}

}  // extern "C"
