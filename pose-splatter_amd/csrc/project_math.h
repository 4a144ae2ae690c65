// Per-Gaussian projection math shared by the forward and backward kernels.
//
// 3D: adapter activations (src/gaussian_renderer.py:190-193) fused with gsplat-classic
//     projection semantics (oracle/oracle3d.py:project3d).
// 2D: activations (src/gaussian_renderer.py:321-323) and the rotated-Gaussian exponent of
//     _render_vectorized (src/gaussian_renderer.py:395-410) rewritten as a conic.
#pragma once

#include "gsr_common.h"

namespace gsr {

struct Cam {
  float R[9];  // world->camera rotation, row-major
  float t[3];
  float fx, fy, cx, cy;
};

__device__ __forceinline__ Cam load_cam(const float* __restrict__ V, const float* __restrict__ K) {
  Cam c;
#pragma unroll
  for (int r = 0; r < 3; ++r) {
#pragma unroll
    for (int k = 0; k < 3; ++k) c.R[r * 3 + k] = V[r * 4 + k];
    c.t[r] = V[r * 4 + 3];
  }
  c.fx = K[0];
  c.cx = K[2];
  c.fy = K[4];
  c.cy = K[5];
  return c;
}

struct Act3D {
  float m[3];   // mean (world)
  float s[3];   // scale = exp(log_scale)
  float q[4];   // adapter-normalised quaternion q/(|q|+1e-8)  (w,x,y,z)
  float rq;     // |q| of the raw quaternion
  float qraw[4];
  float col[3];
  float craw[3];
  float op;     // sigmoid(logit)
};

// mode GSR_INPUT_ADAPTER: raw pose-splatter params (exp / q/(|q|+1e-8) / clamp / sigmoid,
// src/gaussian_renderer.py:183-194).  GSR_INPUT_GSPLAT: gsplat rasterization() inputs, already
// activated (scales, opacities and colours as given; the quaternion only gets gsplat's own
// renormalisation in quat_rotmat).  Same row layout in both modes.
__device__ __forceinline__ Act3D activate3d(const float* __restrict__ p, int mode) {
  Act3D a;
  const bool raw = mode == GSR_INPUT_ADAPTER;
#pragma unroll
  for (int k = 0; k < 3; ++k) a.m[k] = p[k];
#pragma unroll
  for (int k = 0; k < 3; ++k) a.s[k] = raw ? expf(p[3 + k]) : p[3 + k];
  float qq = 0.f;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    a.qraw[k] = p[6 + k];
    qq += a.qraw[k] * a.qraw[k];
  }
  a.rq = sqrtf(qq);
  const float den = raw ? a.rq + 1e-8f : 1.f;
#pragma unroll
  for (int k = 0; k < 4; ++k) a.q[k] = a.qraw[k] / den;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    a.craw[k] = p[10 + k];
    a.col[k] = raw ? fminf(fmaxf(a.craw[k], 0.f), 1.f) : a.craw[k];
  }
  a.op = raw ? 1.f / (1.f + expf(-p[13])) : p[13];
  return a;
}

// Rotation from a (re-normalised) (w,x,y,z) quaternion, row-major.
__device__ __forceinline__ void quat_rotmat(const float qin[4], float R[9], float qn[4], float* inv_norm) {
  const float inv = rsqrtf(qin[0] * qin[0] + qin[1] * qin[1] + qin[2] * qin[2] + qin[3] * qin[3]);
  const float w = qin[0] * inv, x = qin[1] * inv, y = qin[2] * inv, z = qin[3] * inv;
  qn[0] = w; qn[1] = x; qn[2] = y; qn[3] = z;
  *inv_norm = inv;
  R[0] = 1.f - 2.f * (y * y + z * z);
  R[1] = 2.f * (x * y - w * z);
  R[2] = 2.f * (x * z + w * y);
  R[3] = 2.f * (x * y + w * z);
  R[4] = 1.f - 2.f * (x * x + z * z);
  R[5] = 2.f * (y * z - w * x);
  R[6] = 2.f * (x * z - w * y);
  R[7] = 2.f * (y * z + w * x);
  R[8] = 1.f - 2.f * (x * x + y * y);
}

struct Geo3D {
  float Rq[9];     // rotation of the Gaussian
  float qn[4];     // re-normalised quaternion
  float qinv;      // 1/|q_adapter|
  float M[9];      // R diag(s)
  float S[6];      // world covariance (00,01,02,11,12,22)
  float Sc[6];     // camera covariance
  float mc[3];     // camera-space mean
  float rz;        // 1/z
  float tx, ty;    // FOV-clamped
  bool clx, cly;   // true if tx / ty NOT clamped
  float J00, J02, J11, J12;
  float c00, c01, c11;   // cov2d after blur
  float det;
  float A, B, C;         // conic
  float u, v;            // mean2d
};

// Returns false if culled by near/far or det <= 0 (radius/offscreen tests are separate).
__device__ __forceinline__ bool geo3d(const Act3D& a, const Cam& cam, int W, int H, float near_plane,
                                      float far_plane, float eps2d, Geo3D& g) {
  quat_rotmat(a.q, g.Rq, g.qn, &g.qinv);
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int k = 0; k < 3; ++k) g.M[i * 3 + k] = g.Rq[i * 3 + k] * a.s[k];
  const float* M = g.M;
  g.S[0] = M[0] * M[0] + M[1] * M[1] + M[2] * M[2];
  g.S[1] = M[0] * M[3] + M[1] * M[4] + M[2] * M[5];
  g.S[2] = M[0] * M[6] + M[1] * M[7] + M[2] * M[8];
  g.S[3] = M[3] * M[3] + M[4] * M[4] + M[5] * M[5];
  g.S[4] = M[3] * M[6] + M[4] * M[7] + M[5] * M[8];
  g.S[5] = M[6] * M[6] + M[7] * M[7] + M[8] * M[8];
  const float* R = cam.R;
#pragma unroll
  for (int r = 0; r < 3; ++r)
    g.mc[r] = R[r * 3 + 0] * a.m[0] + R[r * 3 + 1] * a.m[1] + R[r * 3 + 2] * a.m[2] + cam.t[r];
  const float x = g.mc[0], y = g.mc[1], z = g.mc[2];
  if (!(z >= near_plane && z <= far_plane)) return false;
  // Sc = R S R^T
  float Sf[9] = {g.S[0], g.S[1], g.S[2], g.S[1], g.S[3], g.S[4], g.S[2], g.S[4], g.S[5]};
  float RS[9];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int k = 0; k < 3; ++k)
      RS[i * 3 + k] = R[i * 3 + 0] * Sf[0 * 3 + k] + R[i * 3 + 1] * Sf[1 * 3 + k] + R[i * 3 + 2] * Sf[2 * 3 + k];
  g.Sc[0] = RS[0] * R[0] + RS[1] * R[1] + RS[2] * R[2];
  g.Sc[1] = RS[0] * R[3] + RS[1] * R[4] + RS[2] * R[5];
  g.Sc[2] = RS[0] * R[6] + RS[1] * R[7] + RS[2] * R[8];
  g.Sc[3] = RS[3] * R[3] + RS[4] * R[4] + RS[5] * R[5];
  g.Sc[4] = RS[3] * R[6] + RS[4] * R[7] + RS[5] * R[8];
  g.Sc[5] = RS[6] * R[6] + RS[7] * R[7] + RS[8] * R[8];
  const float fx = cam.fx, fy = cam.fy, cx = cam.cx, cy = cam.cy;
  const float tan_fovx = 0.5f * (float)W / fx;
  const float tan_fovy = 0.5f * (float)H / fy;
  const float lim_x_pos = ((float)W - cx) / fx + 0.3f * tan_fovx;
  const float lim_x_neg = cx / fx + 0.3f * tan_fovx;
  const float lim_y_pos = ((float)H - cy) / fy + 0.3f * tan_fovy;
  const float lim_y_neg = cy / fy + 0.3f * tan_fovy;
  const float rz = 1.f / z;
  const float rz2 = rz * rz;
  const float xr = x * rz, yr = y * rz;
  g.clx = (xr <= lim_x_pos) && (xr >= -lim_x_neg);
  g.cly = (yr <= lim_y_pos) && (yr >= -lim_y_neg);
  g.tx = z * fminf(lim_x_pos, fmaxf(-lim_x_neg, xr));
  g.ty = z * fminf(lim_y_pos, fmaxf(-lim_y_neg, yr));
  g.rz = rz;
  g.J00 = fx * rz;
  g.J02 = -fx * g.tx * rz2;
  g.J11 = fy * rz;
  g.J12 = -fy * g.ty * rz2;
  const float* Sc = g.Sc;  // s00 s01 s02 s11 s12 s22
  // rows of J*Sc
  const float a0 = g.J00 * Sc[0] + g.J02 * Sc[2];
  const float a1 = g.J00 * Sc[1] + g.J02 * Sc[4];
  const float a2 = g.J00 * Sc[2] + g.J02 * Sc[5];
  const float b1 = g.J11 * Sc[3] + g.J12 * Sc[4];
  const float b2 = g.J11 * Sc[4] + g.J12 * Sc[5];
  g.c00 = a0 * g.J00 + a2 * g.J02 + eps2d;
  g.c01 = a1 * g.J11 + a2 * g.J12;
  g.c11 = b1 * g.J11 + b2 * g.J12 + eps2d;
  g.u = fx * x * rz + cx;
  g.v = fy * y * rz + cy;
  g.det = g.c00 * g.c11 - g.c01 * g.c01;
  if (!(g.det > 0.f)) return false;
  const float inv_det = 1.f / g.det;
  g.A = g.c11 * inv_det;
  g.B = -g.c01 * inv_det;
  g.C = g.c00 * inv_det;
  return true;
}

// 2D: exponent q = a dx^2 + b dx dy + c dy^2 with
//   a = C^2 ia + S^2 ib,  b = 2 C S (ia - ib),  c = S^2 ia + C^2 ib,
//   ia = 1/(2 sx^2 + 1e-8), ib = 1/(2 sy^2 + 1e-8)      (src/gaussian_renderer.py:401-410)
struct Geo2D {
  float u, v, sx, sy, th, cs, sn, ia, ib, a, b, c, op, col[3], craw[3];
};

__device__ __forceinline__ Geo2D geo2d(const float* __restrict__ p) {
  Geo2D g;
  g.u = p[0];
  g.v = p[1];
  g.sx = expf(p[2]);
  g.sy = expf(p[3]);
  g.th = p[4];
  g.cs = cosf(g.th);
  g.sn = sinf(g.th);
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    g.craw[k] = p[5 + k];
    g.col[k] = fminf(fmaxf(g.craw[k], 0.f), 1.f);
  }
  g.op = 1.f / (1.f + expf(-p[8]));
  g.ia = 1.f / (2.f * g.sx * g.sx + 1e-8f);
  g.ib = 1.f / (2.f * g.sy * g.sy + 1e-8f);
  const float c2 = g.cs * g.cs, s2 = g.sn * g.sn, csn = g.cs * g.sn;
  g.a = c2 * g.ia + s2 * g.ib;
  g.b = 2.f * csn * (g.ia - g.ib);
  g.c = s2 * g.ia + c2 * g.ib;
  return g;
}

}  // namespace gsr
