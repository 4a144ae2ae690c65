// Shared device/host helpers for libgsr (gfx950 / CDNA4, wave64).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gsr.h"

namespace gsr {

constexpr int kTile = GSR_TILE;          // 16x16 pixel tiles (gsplat's binning granule)
constexpr int kTilePix = kTile * kTile;  // 256 pixels = 4 waves of 64
constexpr int kWave = 64;
constexpr float kAlphaThreshold = 1.f / 255.f;   // gsplat ALPHA_THRESHOLD
constexpr float kAlphaMax = 0.999f;              // gsplat alpha clamp
constexpr float kTMin = 1e-4f;                   // gsplat transmittance stop
constexpr float kExtendMax = 3.33f;              // gsplat >=1.5 max sigma extent
constexpr int kPartial = 9;                      // per-entry gradient partial width
constexpr int kPartialStride = GSR_PARTIAL_STRIDE;   // floats per partial row (the 9 partials, 36 B)

// Splat record: 3 x float4 (48 B) per (camera, Gaussian).  See include/gsr.h.
struct __align__(16) Splat {
  float4 p0;  // x, y, opacity, depth
  float4 p1;  // a, b, c, 0     (sigma = a dx^2 + b dx dy + c dy^2)
  float4 p2;  // r, g, b, 0
};

// Sort key of (c,n)'s entries: (sort word << 32) | c*N+n.  3D sort word = the depth's float
// bits (depth > 0: integer order = float order; depth [C*N] from gsr3d_project_fwd); 2D = the
// index itself (depth unused, may be null).  Keys are unique inside a tile, so "sorted
// position < tile_end" <=> "key < key of the entry at tile_end".
__device__ __forceinline__ uint64_t sort_key(const float* depth, int64_t cn, int order) {
  const uint32_t w = order == GSR_ORDER_DEPTH ? __float_as_uint(depth[cn]) : (uint32_t)cn;
  return ((uint64_t)w << 32) | (uint64_t)(uint32_t)cn;
}

// ---------------------------------------------------------------- host-side error state
void set_error(const char* fmt, ...);

#define GSR_REQUIRE(cond, ...)            \
  do {                                    \
    if (!(cond)) {                        \
      ::gsr::set_error(__VA_ARGS__);      \
      return GSR_EINVAL;                  \
    }                                     \
  } while (0)

#define GSR_LAUNCH_CHECK(name)                                                   \
  do {                                                                           \
    hipError_t e_ = hipGetLastError();                                           \
    if (e_ != hipSuccess) {                                                      \
      ::gsr::set_error("%s: launch failed: %s", name, hipGetErrorString(e_));   \
      return GSR_ELAUNCH;                                                        \
    }                                                                            \
  } while (0)

inline int ceil_div(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }
inline int64_t ceil_div64(int64_t a, int64_t b) { return (a + b - 1) / b; }

// ---------------------------------------------------------------- device helpers
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __builtin_bit_cast(
      float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}

// Inclusive prefix sum over the 64 lanes of a wave in six DPP adds (Hillis-Steele inside each
// 16-lane row with row_shr 1/2/4/8 -- lanes shifted in from outside the row read 0 -- then
// row_bcast:15 adds row r's last lane into row r+1 for rows 1 and 3, and row_bcast:31 adds
// lane 31 into rows 2 and 3).  Register-to-register: a __shfl_up ladder is six dependent
// ds_bpermute round trips through the LDS crossbar.  Every lane must be active.
__device__ __forceinline__ int wave_incl_scan_dpp(int v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, true);   // row_shr:1
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, true);   // row_shr:2
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, true);   // row_shr:4
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, true);   // row_shr:8
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
  v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
  return v;
}

// Wave-wide reductions with a wave-uniform result: xor-1 / xor-2 quad swaps and the two row
// mirrors reduce each 16-lane row in registers (DPP), then the four row results are combined
// from v_readlane (scalar).  Every lane must be active.
template <int CTRL>
__device__ __forceinline__ int dpp_row_i(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, true);
}
#define GSR_WAVE_REDUCE(NAME, OP)                                                              \
  __device__ __forceinline__ int NAME(int v) {                                                 \
    v = OP(v, dpp_row_i<0xB1>(v));  /* quad_perm [1,0,3,2] */                                  \
    v = OP(v, dpp_row_i<0x4E>(v));  /* quad_perm [2,3,0,1] */                                  \
    v = OP(v, dpp_row_i<0x141>(v)); /* row_half_mirror */                                      \
    v = OP(v, dpp_row_i<0x140>(v)); /* row_mirror */                                           \
    return OP(OP(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 16)),            \
              OP(__builtin_amdgcn_readlane(v, 32), __builtin_amdgcn_readlane(v, 48)));          \
  }
__device__ __forceinline__ int gsr_add_i(int a, int b) { return a + b; }
__device__ __forceinline__ int gsr_max_i(int a, int b) { return a > b ? a : b; }
__device__ __forceinline__ int gsr_or_i(int a, int b) { return a | b; }
GSR_WAVE_REDUCE(wave_sum_i, gsr_add_i)
GSR_WAVE_REDUCE(wave_max_i, gsr_max_i)
GSR_WAVE_REDUCE(wave_or_i, gsr_or_i)
#undef GSR_WAVE_REDUCE

__device__ __forceinline__ float readlane_f(float v, int lane) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), lane));
}

// Full-wave (64-lane) sum; every lane must be active.  Returns the total in all lanes.
// quad xor-1, quad xor-2, half-row mirror, row mirror → 16-lane row sums; then 4 readlanes.
__device__ __forceinline__ float wave_sum(float v) {
  v += dpp_mov<0xB1>(v);    // quad_perm [1,0,3,2]
  v += dpp_mov<0x4E>(v);    // quad_perm [2,3,0,1]
  v += dpp_mov<0x141>(v);   // row_half_mirror
  v += dpp_mov<0x140>(v);   // row_mirror
  return (readlane_f(v, 0) + readlane_f(v, 16)) + (readlane_f(v, 32) + readlane_f(v, 48));
}

// ---------------------------------------------------------------- transposed reduction
// reduce64(v): every lane holds 64 values; afterwards lane l holds sum over all 64 lanes of
// v[l].  A butterfly that halves the number of live registers at every level:
//   xor-32 and xor-16 levels: one v_permlane32_swap / v_permlane16_swap (gfx950) + one add
//   per register pair; the four intra-row levels pair lanes with row_mirror, row_half_mirror
//   and two quad_perms (DPP), the lane's bit choosing which register it keeps.
// ~150 VALU ops for 64 sums, versus ~11 per sum for independent full-wave reductions.
// NOTE: ROCm 7.2's clang returns the FIRST result register for both halves of
// __builtin_amdgcn_permlane{32,16}_swap (the second result is mis-lowered), so the swaps are
// issued as inline asm.  Hardware semantics (verified on MI355X, tools/diag_lanes.hip):
//   v_permlane32_swap a, b:  a' = [a_lo32, b_lo32],  b' = [a_hi32, b_hi32]
//   v_permlane16_swap a, b:  a' = [a_r0, b_r0, a_r2, b_r2],  b' = [a_r1, b_r1, a_r3, b_r3]
// The swaps of one level are issued 8 pairs per asm block behind ONE s_nop 1, which covers
// the VALU-write -> permlane-read hazard the compiler cannot see in asm (the swaps inside a
// block read only registers no other swap of the block writes).
#define GSR_SWAP8(OP)                                                                          \
  asm(OP " %0, %8\n\t" OP " %1, %9\n\t" OP " %2, %10\n\t" OP " %3, %11\n\t" OP " %4, %12\n\t" \
      OP " %5, %13\n\t" OP " %6, %14\n\t" OP " %7, %15"                                        \
      : "+v"(lo[0]), "+v"(lo[1]), "+v"(lo[2]), "+v"(lo[3]), "+v"(lo[4]), "+v"(lo[5]), "+v"(lo[6]),   \
        "+v"(lo[7]), "+v"(hi[0]), "+v"(hi[1]), "+v"(hi[2]), "+v"(hi[3]), "+v"(hi[4]), "+v"(hi[5]),   \
        "+v"(hi[6]), "+v"(hi[7]))
__device__ __forceinline__ void swap32x8(float* lo, float* hi) {
  asm("s_nop 1");
  GSR_SWAP8("v_permlane32_swap_b32");
}
__device__ __forceinline__ void swap16x8(float* lo, float* hi) {
  asm("s_nop 1");
  GSR_SWAP8("v_permlane16_swap_b32");
}
#undef GSR_SWAP8

// Intra-row level: a lane in the upper half (of the row / half-row / quad pair) keeps the
// `hi` register, one in the lower half keeps `lo`; each adds its partner's copy of the same
// register (DPP), so out = upper ? hi + dpp(hi) : lo + dpp(lo).
template <int CTRL>
__device__ __forceinline__ float pair_level(float lo, float hi, bool upper) {
  const float l = lo + dpp_mov<CTRL>(lo);
  const float h = hi + dpp_mov<CTRL>(hi);
  return upper ? h : l;
}

__device__ __forceinline__ float reduce64(float (&v)[64]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int g = 0; g < 4; ++g) swap32x8(&v[8 * g], &v[32 + 8 * g]);
  float a[32];
#pragma unroll
  for (int i = 0; i < 32; ++i) a[i] = v[i] + v[i + 32];
#pragma unroll
  for (int g = 0; g < 2; ++g) swap16x8(&a[8 * g], &a[16 + 8 * g]);
  float b[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) b[i] = a[i] + a[i + 16];
  float c[8];
  const bool b3 = (lane & 8) != 0, b2 = (lane & 4) != 0, b1 = (lane & 2) != 0, b0 = (lane & 1) != 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) c[i] = pair_level<0x140>(b[i], b[i + 8], b3);   // row_mirror
  float d[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) d[i] = pair_level<0x141>(c[i], c[i + 4], b2);   // row_half_mirror
  float e[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) e[i] = pair_level<0x4E>(d[i], d[i + 2], b1);    // quad_perm [2,3,0,1]
  return pair_level<0xB1>(e[0], e[1], b0);                                     // quad_perm [1,0,3,2]
}

// reduce_box16(v, out): the 16 lanes with equal lane bits 0-1 (a "box" of the raster
// backward) sum each of the 64 registers; afterwards out[i] of lane l is the box sum of
// register 4*(l>>2) + i.  The same halving butterfly as reduce64 over lane bits 5 and 4
// (permlane32 / permlane16 swaps), then bit 3 (row_ror:8 is xor 8 inside a row) and bit 2
// (the lower lane of a pair reads lane+4 with row_shl:4, the upper lane-4 with row_shr:4),
// and stops there: bits 0-1 separate the boxes.  132 VALU ops for 4 x 16-lane sums of 64 values.
__device__ __forceinline__ void reduce_box16(float (&v)[64], float (&out)[4]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int g = 0; g < 4; ++g) swap32x8(&v[8 * g], &v[32 + 8 * g]);
  float a[32];
#pragma unroll
  for (int i = 0; i < 32; ++i) a[i] = v[i] + v[i + 32];
#pragma unroll
  for (int g = 0; g < 2; ++g) swap16x8(&a[8 * g], &a[16 + 8 * g]);
  float b[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) b[i] = a[i] + a[i + 16];
  const bool b3 = (lane & 8) != 0, b2 = (lane & 4) != 0;
  float c[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) c[i] = pair_level<0x128>(b[i], b[i + 8], b3);   // row_ror:8
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float l = c[i] + dpp_mov<0x104>(c[i]);           // row_shl:4: lane + 4
    const float h = c[i + 4] + dpp_mov<0x114>(c[i + 4]);   // row_shr:4: lane - 4
    out[i] = b2 ? h : l;
  }
}

// reduce_box8(v, out): the 8 lanes with equal lane bits 0-2 (a "box" of the 2D pair backward,
// k_raster2d_bwd_pair) sum each of the 64 registers; afterwards out[i] of lane l is the box sum
// of register 8*(l>>3) + i.  The halving butterfly of reduce_box16 over lane bits 5 and 4
// (permlane swaps) and 3 (row_ror:8), stopping there: 96 VALU ops for 8 x 8-lane sums of 64.
__device__ __forceinline__ void reduce_box8(float (&v)[64], float (&out)[8]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int g = 0; g < 4; ++g) swap32x8(&v[8 * g], &v[32 + 8 * g]);
  float a[32];
#pragma unroll
  for (int i = 0; i < 32; ++i) a[i] = v[i] + v[i + 32];
#pragma unroll
  for (int g = 0; g < 2; ++g) swap16x8(&a[8 * g], &a[16 + 8 * g]);
  float b[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) b[i] = a[i] + a[i + 16];
  const bool b3 = (lane & 8) != 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) out[i] = pair_level<0x128>(b[i], b[i + 8], b3);   // row_ror:8
}

// ---------------------------------------------------------------- b128-group-aligned box reductions
// A ds_read_b128 serves a wave in four 16-lane groups (MI355X_MICROARCH.md §LDS), one LDS cycle
// per group when its lanes read at most one address per bank set; group of lane l =
// (bit 5, bit 2 ^ bit 3 ^ bit 4).  With the backward's box = lane & 3 (reduce_box16) or lane & 7
// (reduce_box8) every group held four or eight boxes, each reading ITS survivor's record in the
// walk: four / eight addresses per group, a bank conflict whenever two records sat 16 apart
// (32 % / 45 % of the backward kernels' LDS cycles, r04_pmc_sq_cfg{3,4,5}_p2).  These reductions
// sum over lane sets that lie INSIDE one b128 group, so a walk read is one (16-lane boxes) or two
// (8-lane boxes) addresses per group.
//
// The one level that crosses 16-lane rows pairs lanes l and l ^ 0x18: a v_permlane16_swap (rows
// r <-> r^1) whose partner register is read through DPP row_ror:8 (xor 8 inside a row), fused into
// the add.  Every lane computes a' + ror8(b'): a low-row lane (bit 4 clear) gets reg i of {l, l^0x18},
// a high-row lane reg i+32 of {l^16, l^8} -- the box of l^16 (a relabelling: the output box of
// lane l is that of l & ~16).  The remaining levels stay inside rows (row_mirror = xor 15, quad
// xor 2 / xor 1), all in the group's direction space {x : bit5 = 0, bit2^bit3^bit4 = 0}.
// (the leading s_nop inside the block: a separate asm("s_nop 1") statement is dropped by the
// compiler -- none appears in the ISA of swap16x8 / swap32x8)
__device__ __forceinline__ void swap16x8_dpp(float* lo, float* hi) {
  asm("s_nop 1\n\t"
      "v_permlane16_swap_b32 %0, %8\n\t"
      "v_permlane16_swap_b32 %1, %9\n\t"
      "v_permlane16_swap_b32 %2, %10\n\t"
      "v_permlane16_swap_b32 %3, %11\n\t"
      "v_permlane16_swap_b32 %4, %12\n\t"
      "v_permlane16_swap_b32 %5, %13\n\t"
      "v_permlane16_swap_b32 %6, %14\n\t"
      "v_permlane16_swap_b32 %7, %15\n\t"
      "s_nop 1"   // the VALU-write -> DPP-read hazard of the adds that read these through row_ror:8
      : "+v"(lo[0]), "+v"(lo[1]), "+v"(lo[2]), "+v"(lo[3]), "+v"(lo[4]), "+v"(lo[5]), "+v"(lo[6]), "+v"(lo[7]),
        "+v"(hi[0]), "+v"(hi[1]), "+v"(hi[2]), "+v"(hi[3]), "+v"(hi[4]), "+v"(hi[5]), "+v"(hi[6]), "+v"(hi[7]));
}
// b128 lane group of lane l (0..3)
__device__ __forceinline__ int b128_group(int l) { return ((l >> 5) << 1) | (((l >> 2) ^ (l >> 3) ^ (l >> 4)) & 1); }

// reduce_grp16(v, out): the 16 lanes of each b128 group sum each of the 64 registers; afterwards
// out[i] of lane l is the sum of register 4 * grp16_slot(l) + i over the group
// grp16_out_box(l).  Levels: xor 0x18 (swap16 + ror8), row_mirror, quad xor 2, quad xor 1
// (132 VALU ops, as reduce_box16).
__device__ __forceinline__ int grp16_slot(int l) {
  return (((l >> 4) & 1) << 3) | (((l >> 3) & 1) << 2) | (((l >> 1) & 1) << 1) | (l & 1);
}
__device__ __forceinline__ int grp16_out_box(int l) { return ((l >> 5) << 1) | (((l >> 2) ^ (l >> 3)) & 1); }
// position of lane l inside its walk box b128_group(l) (bits 0, 1, 3, 4; bit 2 follows)
__device__ __forceinline__ int grp16_pos(int l) { return (l & 3) | (((l >> 3) & 3) << 2); }
__device__ __forceinline__ void reduce_grp16(float (&v)[64], float (&out)[4]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int g = 0; g < 4; ++g) swap16x8_dpp(&v[8 * g], &v[32 + 8 * g]);
  float a[32];
#pragma unroll
  for (int i = 0; i < 32; ++i) a[i] = dpp_mov<0x128>(v[i + 32]) + v[i];   // row_ror:8 of the swapped partner
  const bool b3 = (lane & 8) != 0, b1 = (lane & 2) != 0, b0 = (lane & 1) != 0;
  float b[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) b[i] = pair_level<0x140>(a[i], a[i + 16], b3);   // row_mirror
  float c[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) c[i] = pair_level<0x4E>(b[i], b[i + 8], b1);      // quad_perm [2,3,0,1]
#pragma unroll
  for (int i = 0; i < 4; ++i) out[i] = pair_level<0xB1>(c[i], c[i + 4], b0);    // quad_perm [1,0,3,2]
}

// reduce_grp8(v, out): 8-lane boxes, two per b128 group: box of lane l (its walk box) =
// 4 bit5 + 2 (bit2^bit3^bit4) + (bit1^bit3^bit4), position (bits 0, 3, 4) grp8_pos.  Afterwards
// out[i] of lane l is the sum of register 8 * grp8_slot(l) + i over box grp8_out_box(l).
// Levels: xor 0x18 (swap16 + ror8), row_mirror, quad xor 1 (136 VALU ops; reduce_box8 120).
__device__ __forceinline__ int grp8_box(int l) {
  return ((l >> 5) << 2) | ((((l >> 2) ^ (l >> 3) ^ (l >> 4)) & 1) << 1) | (((l >> 1) ^ (l >> 3) ^ (l >> 4)) & 1);
}
__device__ __forceinline__ int grp8_pos(int l) { return (l & 1) | (((l >> 3) & 3) << 1); }
__device__ __forceinline__ int grp8_slot(int l) { return (((l >> 4) & 1) << 2) | (((l >> 3) & 1) << 1) | (l & 1); }
__device__ __forceinline__ int grp8_out_box(int l) {
  return ((l >> 5) << 2) | ((((l >> 2) ^ (l >> 3)) & 1) << 1) | (((l >> 1) ^ (l >> 3)) & 1);
}
__device__ __forceinline__ void reduce_grp8(float (&v)[64], float (&out)[8]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int g = 0; g < 4; ++g) swap16x8_dpp(&v[8 * g], &v[32 + 8 * g]);
  float a[32];
#pragma unroll
  for (int i = 0; i < 32; ++i) a[i] = dpp_mov<0x128>(v[i + 32]) + v[i];
  const bool b3 = (lane & 8) != 0, b0 = (lane & 1) != 0;
  float b[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) b[i] = pair_level<0x140>(a[i], a[i + 16], b3);   // row_mirror
#pragma unroll
  for (int i = 0; i < 8; ++i) out[i] = pair_level<0xB1>(b[i], b[i + 8], b0);    // quad_perm [1,0,3,2]
}
// Staging of the reduced sums (box-major rows of 64 floats, XOR-swizzled so that the b128 stores
// of 8 consecutive lanes and the b32 reads of flat index f = 0..63 of one box are conflict-free):
//   grp16: sum i of lane l at  box * 64 + ((4 grp16_slot(l) + i) ^ grp16_swz(box))
//   grp8:  sum i of lane l at  box * 64 + ((8 grp8_slot(l) + i) ^ grp8_swz(box))
__device__ __forceinline__ int grp16_swz(int box) { return (box & 1) << 4; }
__device__ __forceinline__ int grp8_swz(int box) { return ((box & 2) << 3) | ((box & 1) << 2); }
// grp8 in two halves (sums 0-3, then 4-7): row of 32 per box, compressed index
// 4 grp8_slot(l) + (i & 3), swizzle 8 (box & 3)
__device__ __forceinline__ int grp8h_swz(int box) { return (box & 3) << 3; }

__device__ __forceinline__ unsigned long long wave_ballot(bool p) { return __ballot(p); }

// gsr_set_fwd_heavy (raster.hip): the 3D forward's heavy-tile threshold, log2 of the list length
// (0: off); the tile scan (binning.hip) counts those tiles into gsr_bin_stats.n_heavy -- at most
// kFwdHeavyMax of them: the threshold is raised to the smallest power of two (>= 2^k) that leaves
// at most that many, so the heavy set depends only on the list lengths (the busy order inside a
// log2 bucket is the tile scan's arrival order: a cap taken from the order's head would make the
// layout, and with it the fp32 rounding, vary from run to run)
extern int g_fwd_heavy_log2;
#ifndef GSR_FWD_HEAVY_MAX
#define GSR_FWD_HEAVY_MAX 64
#endif
constexpr int kFwdHeavyMax = GSR_FWD_HEAVY_MAX;

// Block-wide exclusive scan of one int per thread (NT threads, multiple of 64).
// s_tmp must hold NT/64 + 1 ints.  Returns the exclusive prefix; *total = block sum.
template <int NT>
__device__ __forceinline__ int block_exclusive_scan(int v, int* s_tmp, int* total) {
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int x = wave_incl_scan_dpp(v);
  if (lane == 63) s_tmp[w] = x;
  __syncthreads();
  if (threadIdx.x < 64) {   // wave 0 scans the wave totals (lane k: wave k)
    const int t = lane < NT / 64 ? s_tmp[lane] : 0;
    const int it = wave_incl_scan_dpp(t);
    if (lane < NT / 64) s_tmp[lane] = it - t;
    if (lane == NT / 64 - 1) s_tmp[NT / 64] = it;
  }
  __syncthreads();
  int res = x - v + s_tmp[w];
  *total = s_tmp[NT / 64];
  __syncthreads();
  return res;
}

__device__ __forceinline__ uint32_t pack_rect_lo(int a, int b) {
  return (uint32_t)a | ((uint32_t)b << 16);
}

// binning.hip: the lazy path's second sort (every tile flagged by the forward, sorted whole)
int bin_sort_rest(const int32_t* tile_offset, int64_t CT, int32_t max_seg, int32_t n_max, void* workspace,
                  size_t workspace_bytes, int32_t* lazy, int32_t* tile_end, int32_t* sorted_ids, int32_t* k_of_s,
                  gsr_bin_stats* stats, hipStream_t s);

// ---------------------------------------------------------------- per-wave culling
// A wave owns an 8x8 sub-tile of its 16x16 tile.  An entry can only change a pixel of the
// sub-tile if its level set {opacity*exp(-sigma) >= cut} (3D: cut = 1/255, gsplat's skip
// threshold; 2D: eps_cut) meets the sub-tile's pixel-centre box B, i.e. iff
// min over B of sigma <= L = ln(opacity/cut).  That minimum is computed exactly: sigma is a
// convex quadratic with its minimum at the mean, so when the mean lies outside B the
// minimiser lies on an edge of B facing the mean, and along an edge the best point is the
// clamped 1-D optimum.  With dx fixed to the mean's nearest x in B, the best dy is
// clamp(-b dx / 2c); likewise for y; the smaller of the two values is the box minimum (the
// non-facing "edge" evaluates a segment inside B, never below the true minimum).  A small
// relative margin absorbs rounding, so culling changes the work, never the result.  The
// per-Gaussian constants (L and the two edge slopes) come precomputed in the record's .w
// slots (gsr3d_project_fwd), so the test has no transcendental.
// sigma = a dx^2 + b dx dy + c dy^2 of a record's conic (a, b, c) = p1.xyz, one definition
// for every kernel (the backward's alpha must be the forward's, bit for bit)
__device__ __forceinline__ float conic_sigma(const float4 p1, float dx, float dy) {
  return p1.x * dx * dx + p1.z * dy * dy + p1.y * dx * dy;
}

// exp(-sigma) of a record's conic.  Records store the conic and L scaled by log2(e)
// (k_project2d_fwd since ABI 11, k_project3d_fwd since ABI 12): sigma' = sigma log2(e), so
// exp(-sigma) = 2^(-sigma') is ONE v_exp_f32 (__expf is a multiply by -log2(e) and the same
// v_exp_f32); sigma' >= 0 iff sigma >= 0.  The gradients that sum v_sig * dx^2 ... stay
// derivatives by the unscaled conic (v_sig is dL/dsigma either way); only the mean's chain
// through the conic needs the unscaled a, b, c (kLn2 * stored).
constexpr float kLog2e = 1.44269504088896341f;
constexpr float kLn2 = 0.693147180559945309f;
#ifndef GSR_CONIC3D_LOG2E
#define GSR_CONIC3D_LOG2E 1   // 0: 3D records unscaled (the ABI-11 form; a build knob for A/B runs)
#endif
template <bool IS2D>
__device__ __forceinline__ float gauss_exp(float sigma) {
  if constexpr (IS2D || GSR_CONIC3D_LOG2E)
    return __builtin_amdgcn_exp2f(-sigma);
  else
    return __expf(-sigma);
}
// factor from a stored conic to the true one (the rows phases' mean chain)
template <bool IS2D>
__device__ __forceinline__ constexpr float conic_unscale() {
  return (IS2D || GSR_CONIC3D_LOG2E) ? kLn2 : 1.f;
}

#ifndef GSR_CULL_BRANCHFREE
#define GSR_CULL_BRANCHFREE 1
#endif
template <bool IS2D>
__device__ __forceinline__ bool cull_keep(const float4 p0, const float4 p1, const float4 p2, float bx0, float bx1,
                                          float by0, float by1) {
  (void)IS2D;   // 3D: L = ln(opacity * 255); 2D: L = ln(opacity / eps_cut)
  const float L = p0.w;   // < 0: the Gaussian never reaches the cut anywhere
  const float a = p1.x, b = p1.y, c = p1.z;
#if GSR_CULL_BRANCHFREE
  // the same decision without early exits (every term is evaluated; the selects pick as the
  // branches did): exec-mask branches cost scalar instructions on every culled entry
  const bool pd = a > 0.f && c > 0.f && 4.f * a * c > b * b;   // not positive definite: keep
  const float dxe = p0.x - fminf(fmaxf(p0.x, bx0), bx1);
  const float dye = p0.y - fminf(fmaxf(p0.y, by0), by1);
  const float dy1 = fminf(fmaxf(p1.w * dxe, p0.y - by1), p0.y - by0);
  const float dx2 = fminf(fmaxf(p2.w * dye, p0.x - bx1), p0.x - bx0);
  const float s1 = a * dxe * dxe + b * dxe * dy1 + c * dy1 * dy1;
  const float s2 = a * dx2 * dx2 + b * dx2 * dye + c * dye * dye;
  return (L >= 0.f) & (!pd | (fminf(s1, s2) <= L * 1.001f + 1e-3f));
#else
  if (!(L >= 0.f)) return false;
  if (!(a > 0.f && c > 0.f && 4.f * a * c > b * b)) return true;   // not positive definite: keep
  const float dxe = p0.x - fminf(fmaxf(p0.x, bx0), bx1);
  const float dye = p0.y - fminf(fmaxf(p0.y, by0), by1);
  const float dy1 = fminf(fmaxf(p1.w * dxe, p0.y - by1), p0.y - by0);   // p1.w = -b / 2c
  const float dx2 = fminf(fmaxf(p2.w * dye, p0.x - bx1), p0.x - bx0);   // p2.w = -b / 2a
  const float s1 = a * dxe * dxe + b * dxe * dy1 + c * dy1 * dy1;
  const float s2 = a * dx2 * dx2 + b * dx2 * dye + c * dye * dye;
  return fminf(s1, s2) <= L * 1.001f + 1e-3f;
#endif
}

// Quadrant mask of a (record, tile) list entry: bit q (q = 2 * (quadrant row) + quadrant
// column of the 16x16 tile) is set iff cull_keep keeps the record for that 8x8 quadrant's
// pixel-centre box -- the same test on the same fp32 box bounds as the raster forward's
// quadrant workgroups, so a workgroup may skip (not even gather) an entry whose bit is clear.
// Stored by the emission in the top bits of the entry's emission index (k_of_s).
// gsr_bin_stats.masks: bit 0 -- the 3D emission stored quadrant masks (k_of_s bits 28..31); bit 1 --
// the 2D pair forward wrote the colour planes that the split per-set backward starts from
constexpr int kStatsMasks3D = 1;
constexpr int kStatsPlanes2D = 2;
constexpr int kStatsBoxMasks = 4;   // bit 2: the 3D quad forward wrote per-box survivor masks (box_masks)
constexpr int kMaskShift = 28;                         // k_of_s bits 28..31
constexpr int32_t kEmitIndexMask = (1 << kMaskShift) - 1;
template <bool IS2D>
__device__ __forceinline__ int quad_mask(const float4 p0, const float4 p1, const float4 p2, int tx, int ty) {
  const float off = IS2D ? 0.f : 0.5f;
  int m = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float x0 = (float)(tx * kTile + (q & 1) * 8) + off, y0 = (float)(ty * kTile + (q >> 1) * 8) + off;
    if (cull_keep<IS2D>(p0, p1, p2, x0, x0 + 7.f, y0, y0 + 7.f)) m |= 1 << q;
  }
  return m;
}

// Parameter set of camera c: cameras are grouped by set, set f owning cameras
// [set_begin[f], set_begin[f+1]) (null: one set).  Uniform per workgroup (scalar loads).
__device__ __forceinline__ int set_of_camera(const int32_t* __restrict__ set_begin, int F, int c) {
  if (set_begin == nullptr) return 0;
  int f = 0;
  while (f + 1 < F && set_begin[f + 1] <= c) ++f;
  return f;
}
__device__ __forceinline__ int set_first_camera(const int32_t* __restrict__ set_begin, int F, int c) {
  return set_begin == nullptr ? 0 : set_begin[set_of_camera(set_begin, F, c)];
}

// 2D: with several cameras per parameter set (views ignored: identical renders), the raster
// backward walks each (set, tile) once for all the set's cameras (k_raster2d_bwd_frame) and
// writes their summed partial rows at the set's first camera's emission indices only;
// gsr2d_project_bwd then reads only those.  Both sides decide by this one rule.
#ifndef GSR_BWD2D_FRAME
#define GSR_BWD2D_FRAME 1
#endif
inline bool rows2d_per_set(const int32_t* set_begin, int F, int C) {
  return GSR_BWD2D_FRAME && set_begin != nullptr && C > F;
}
// ... and, under the same rule with the automatic 2D forward layout (raster.hip), the binning
// emits only each set's first camera's lists (its cameras' lists would be identical copies): the
// projection gives the other cameras no tiles, and their forwards render the first camera's
// list (k_raster2d_fwd_pair).  Host-side: it reads the forward-layout setting.
bool lists2d_per_set(const int32_t* set_begin, int F, int C);
// ... and when the call has few (set, tile) pairs for the chip (a frame owner's one frame), the
// per-set backward splits each tile's consumed list into frame_parts2d(...) unit-aligned parts
// walked by separate workgroups; the forward then also stores, per pixel, its colour sum before
// every unit and in total (three planes after the T anchors, colour_plane2d floats apart), so a
// part starts from the suffix state at its end.  1: no split.  Host-side (raster.hip).
int frame_parts2d(const int32_t* set_begin, int F, int C, int T);

// 2D: the record of entry id = c*N + n lives in the copy of camera c's set's first camera
// (k_project2d_fwd writes one copy per set): rec[id + rec_offset2d(c)].
__device__ __forceinline__ int64_t rec_offset2d(const int32_t* __restrict__ set_begin, int F, int c, int64_t N) {
  return (int64_t)(set_first_camera(set_begin, F, c) - c) * N;
}

// 2D visit order, XCD-aware.  A grid of 8*S workgroups (S = ceil(CT/8)) is dealt to the 8 XCDs
// round-robin by id, so workgroup b runs on XCD b % 8; it takes position (b % 8) * S + b / 8 of
// the sweep (set, tile row, tile column, camera of the set).  Each XCD thus walks its eighth of
// the sweep in order: the cameras of a set (identical lists over one shared record copy) render
// a tile back to back, and tile rows follow each other, so each record comes from HBM into the
// XCD's L2 about once per set instead of once per (camera, tile).  -1 past the end.
__device__ __forceinline__ int sweep_tile2d(int b, int64_t CT, int T, const int32_t* __restrict__ set_begin, int F) {
  const int64_t S = (CT + 7) / 8;
  const int64_t p = (int64_t)(b & 7) * S + (b >> 3);
  if (p >= CT) return -1;
  int c0 = 0, c1 = (int)(CT / T);
  if (set_begin != nullptr) {
    int f = 0;
    while (f + 1 < F && (int64_t)set_begin[f + 1] * T <= p) ++f;
    c0 = set_begin[f];
    c1 = set_begin[f + 1];
  }
  const int V = c1 - c0;
  const int q = (int)(p - (int64_t)c0 * T);
  const int t = q / V, v = q - t * V;
  return (c0 + v) * T + t;
}
__host__ __device__ __forceinline__ int sweep_grid2d(int64_t CT) { return (int)(8 * ((CT + 7) / 8)); }
// floats between the 2D T anchors and each colour plane (frame_parts2d): one plane per colour
// channel, as many rows as the call's units (the chunk-state buffer holds 4 floats per row slot)
__device__ __forceinline__ int64_t colour_plane2d(const gsr_bin_stats* __restrict__ stats) {
  return (int64_t)stats->n_chunks * 256;
}

}  // namespace gsr
