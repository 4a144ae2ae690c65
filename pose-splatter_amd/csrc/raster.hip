// (c) Per-tile compositing, forward and backward.
//
// One 256-thread workgroup per 16x16 tile (4 waves of 64 pixels).  The tile's sorted list
// is staged through LDS in batches of 256 splat records (each record gathered once per
// tile, broadcast-read by all 4 waves); each wave leaves the inner loop as soon as all of
// its 64 pixels are done (exec-mask early-out), the workgroup as soon as all 4 are.
//
// Backward gradient scatter: instead of per-Gaussian float atomics (memory-side on MI355X,
// ~0.08 TB/s for scattered lanes), every sorted entry's gradient is summed over the tile's
// pixels on chip (DPP wave sums + a 4-wave LDS combine) and stored ONCE, coalesced, as a
// 9-float partial; *_project_bwd reduces each Gaussian's partials in a fixed order, so the
// gradients are bitwise deterministic.
#include "gsr_common.h"

#include <type_traits>

namespace gsr {


constexpr int kRasterThreads = 256;
constexpr int kChunk3 = GSR_CHUNK;   // backward work unit: list entries per chunk
constexpr int kFillBlocks = 1024;    // workgroups that fill the empty tiles
#ifndef GSR_FWD_PAD_3D
#define GSR_FWD_PAD_3D 0   // 3D quad rounds (26.4 KB LDS: 6 per CU): padded to 5 per CU +2 us, to 4 per CU +12 us (round 6, profiles/r06_ab_fwd_pad.txt)
#endif
constexpr int kFwdLdsPad = GSR_FWD_PAD_3D;
#ifndef GSR_FWD_PAD_2D
#define GSR_FWD_PAD_2D 0   // 2D: every tile busy, no L2 locality to protect (6 per CU by VGPRs: measured 10% faster)
#endif
constexpr int kFwdLdsPad2D = GSR_FWD_PAD_2D;
static int g_fwd_lanes = 0;   // gsr_set_fwd_lanes: 0 automatic, 1 / 4 / 16 forced
#ifndef GSR_FWD_HEAVY_LOG2
#define GSR_FWD_HEAVY_LOG2 0   // default heavy-tile threshold (0 = off; 12: lists of >= 4096 entries)
#endif
int g_fwd_heavy_log2 = GSR_FWD_HEAVY_LOG2;   // gsr_set_fwd_heavy (gsr_common.h)
// gsr_set_bwd2d_parts (frame_parts2d): 0, the default, is off -- a caller that sized chunk_state by
// the 2D contract of revision 12 (one float per slot) keeps it; the Python binding, which
// allocates four floats per slot, turns it on
int g_bwd2d_part_wgs = 0;
static int g_bwd_layout = 0;  // gsr_set_bwd_layout: 0 automatic, 1 chunk kernel, 2 pixel pairs (3D)
// box forward (k_raster_fwd_box) build knobs, for A/B measurements: lanes grouped by box along
// the ds_read_b128 lane groups, and the 2D walk's records packed into 2 x b128 + b32
#ifndef GSR_BOX_LANES
#define GSR_BOX_LANES 1
#endif
#ifndef GSR_BOX_PACK
#define GSR_BOX_PACK 1
#endif
constexpr int kBoxStride = 132;   // survivor-list row of one 4x4 box (128 + a read-ahead word)


__device__ __forceinline__ void tile_coords(int ct, int tw, int th, int& c, int& ty, int& tx) {
  const int T = tw * th;
  c = ct / T;
  const int t = ct - c * T;
  ty = t / tw;
  tx = t - ty * tw;
}

// (per-wave culling: conic_sigma / cull_keep / quad_mask live in gsr_common.h -- the binning
// computes each entry's quadrant mask with the same test)

// The survivors list[0, nsurv) of an 8x8 quadrant (origin (qx, qy), pixel centres) against its
// four 4x4 boxes, ONE survivor per lane: its record is read from LDS once and tested against all
// four boxes (box b at (qx + 4 (b & 1), qy + 4 (b >> 1))); box b's survivors are appended in
// list order to boxl[b * stride + ..].  n[b]: the four counts (wave-uniform).  (A lane per
// (survivor, box) pair read every record four times and walked 16 survivors per round trip.)
// Packed record parts (PACKED): q0 = (x, y, opacity, r), q1 = (a, b, c, g), q2 = (b_colour, L,
// -b/2c, -b/2a) -- the walk's nine values in two b128 reads and one b32 instead of three b128;
// unpack_rec restores the Splat parts for the culls.  2D records are STORED packed
// (k_project2d_fwd, ABI 8), so the 2D kernels stage them as they come.
__device__ __forceinline__ void pack_rec(float4& p0, float4& p1, float4& p2) {
  const float4 q0 = make_float4(p0.x, p0.y, p0.z, p2.x);
  const float4 q1 = make_float4(p1.x, p1.y, p1.z, p2.y);
  const float4 q2 = make_float4(p2.z, p0.w, p1.w, p2.w);
  p0 = q0;
  p1 = q1;
  p2 = q2;
}
template <bool PACKED>
__device__ __forceinline__ void unpack_rec(float4& p0, float4& p1, float4& p2) {
  if constexpr (PACKED) {
    const float4 s0 = make_float4(p0.x, p0.y, p0.z, p2.y);
    const float4 s1 = make_float4(p1.x, p1.y, p1.z, p2.z);
    const float4 s2 = make_float4(p0.w, p1.w, p2.x, p2.w);
    p0 = s0;
    p1 = s1;
    p2 = s2;
  }
}

// Survivor-list slot of list position p when the backward reads its groups of 7 as one 8-byte
// word: a pad byte after every 7 (p + p / 7; the multiply-shift is exact for p < 400).
__device__ __forceinline__ int grouped_slot(int p) { return p + ((p * 293) >> 11); }

template <bool IS2D, bool PACKED = false, bool GROUPED = false>
__device__ __forceinline__ void box4_cull(const unsigned char* __restrict__ list, int nsurv, const float4* r0,
                                          const float4* r1, const float4* r2, float qx, float qy,
                                          unsigned char* boxl, int stride, int (&n)[4]) {
  const int lane = threadIdx.x & 63;
  const unsigned long long below = (1ull << lane) - 1ull;
  n[0] = n[1] = n[2] = n[3] = 0;
  for (int s0 = 0; s0 < nsurv; s0 += 64) {
    const int s = s0 + lane;
    const bool in = s < nsurv;
    const int k = list[in ? s : 0];
    float4 a = r0[k], b = r1[k], c = r2[k];
    unpack_rec<PACKED>(a, b, c);
#pragma unroll
    for (int bx = 0; bx < 4; ++bx) {
      const float x0 = qx + (float)((bx & 1) * 4), y0 = qy + (float)((bx >> 1) * 4);
      const bool keep = in && cull_keep<IS2D>(a, b, c, x0, x0 + 3.f, y0, y0 + 3.f);
      const unsigned long long m = __ballot(keep);
      if (keep) {
        const int p = n[bx] + __popcll(m & below);
        boxl[bx * stride + (GROUPED ? grouped_slot(p) : p)] = (unsigned char)k;
      }
      n[bx] += __popcll(m);
    }
  }
}

// 2D parameter sets of the cameras (gsr2d_*: one record copy per set, rec_offset2d; the XCD-aware
// sweep, sweep_tile2d).  3D: {0, nullptr, 1}, unused.
struct Sets2D {
  int64_t N;
  const int32_t* begin;
  int F;
};

// ---------------------------------------------------------------- empty tiles
// Tiles with an empty list only need the background.  The forward launches them as extra
// workgroups (after the busy tiles' ones) that stride over order[n_busy..CT): cheap stores that
// run beside the busy tiles instead of one short-lived workgroup per empty tile.
__device__ void nan_tile(int c, int ty, int tx, int W, int H, float* __restrict__ out_rgb, float* __restrict__ out_alpha);
__device__ __forceinline__ bool lists2d_missing(const int32_t* __restrict__ tile_offset, const Sets2D& sets, int c,
                                                int ct, int T);
template <bool IS2D>
__device__ void fill_empty(const int32_t* __restrict__ order, const int32_t* __restrict__ tile_offset, int n_busy,
                           int busy_blocks, int64_t CT, int W, int H, int tw, int th, const float* __restrict__ bg,
                           float* __restrict__ out_rgb, float* __restrict__ out_alpha, float* __restrict__ out_T,
                           int32_t* __restrict__ out_last, int32_t* __restrict__ tile_end,
                           uint64_t* __restrict__ tile_cut, const Sets2D sets, int32_t* status) {
  const int G = gridDim.x - busy_blocks;
  for (int64_t t = n_busy + (blockIdx.x - busy_blocks); t < CT; t += G) {
    const int ct = order[t];
    int c, ty, tx;
    tile_coords(ct, tw, th, c, ty, tx);
    if (IS2D && lists2d_missing(tile_offset, sets, c, ct, tw * th)) {
      if (threadIdx.x == 0 && status != nullptr) atomicOr(status, GSR_OVF_LAYOUT);
      nan_tile(c, ty, tx, W, H, out_rgb, out_alpha);
      continue;
    }
    for (int p = threadIdx.x; p < kTilePix; p += blockDim.x) {   // (256- and 512-thread forwards)
      const int i = ty * kTile + (p >> 4), j = tx * kTile + (p & 15);
      if (i >= H || j >= W) continue;
      const int64_t pix = ((int64_t)c * H + i) * W + j;
      const float* bgc = bg + c * 3;
      out_rgb[pix * 3 + 0] = bgc[0];
      out_rgb[pix * 3 + 1] = bgc[1];
      out_rgb[pix * 3 + 2] = bgc[2];
      out_alpha[pix] = 0.f;
      if (IS2D)
        reinterpret_cast<float2*>(out_T)[pix] = make_float2(1.f, 1.f);
      else
        out_T[pix] = 1.f;
      out_last[pix] = -1;
    }
    if (threadIdx.x == 0) {
      tile_end[ct] = tile_offset[ct];
      tile_cut[ct] = ~0ull;
    }
  }
}

// A bounded call whose bounds did not hold (stats->overflow): every pixel of the call gets NaN
// rgb / alpha (tile-strided over the whole grid), so the failure cannot pass as a render.
__device__ void nan_fill(int64_t CT, int W, int H, int tw, int th, float* __restrict__ out_rgb,
                         float* __restrict__ out_alpha) {
  const float nan = __builtin_nanf("");
  for (int64_t t = blockIdx.x; t < CT; t += gridDim.x) {
    int c, ty, tx;
    tile_coords((int)t, tw, th, c, ty, tx);
    for (int p = threadIdx.x; p < kTile * kTile; p += blockDim.x) {   // (128- and 256-thread kernels)
      const int i = ty * kTile + (p >> 4), j = tx * kTile + (p & 15);
      if (i < H && j < W) {
        const int64_t pix = ((int64_t)c * H + i) * W + j;
        out_rgb[pix * 3 + 0] = nan;
        out_rgb[pix * 3 + 1] = nan;
        out_rgb[pix * 3 + 2] = nan;
        out_alpha[pix] = nan;
      }
    }
  }
}

// One tile's pixels NaN (a 2D layout mismatch, lists2d_missing below)
__device__ void nan_tile(int c, int ty, int tx, int W, int H, float* __restrict__ out_rgb, float* __restrict__ out_alpha) {
  const float nan = __builtin_nanf("");
  for (int p = threadIdx.x; p < kTile * kTile; p += blockDim.x) {
    const int i = ty * kTile + (p >> 4), j = tx * kTile + (p & 15);
    if (i < H && j < W) {
      const int64_t pix = ((int64_t)c * H + i) * W + j;
      out_rgb[pix * 3 + 0] = nan;
      out_rgb[pix * 3 + 1] = nan;
      out_rgb[pix * 3 + 2] = nan;
      out_alpha[pix] = nan;
    }
  }
}

// gsr2d_project_fwd and the 2D raster forward decide lists2d_per_set on the host each
// (the rule reads gsr_set_fwd_lanes).  A forward that renders a camera from its OWN list after a
// projection that binned only its set's first camera would draw it as background: its list is
// then empty where the first camera's is not -- impossible otherwise, a set's cameras render
// identical lists -- so such a tile is NaN and GSR_OVF_LAYOUT goes to the sticky status.
__device__ __forceinline__ bool lists2d_missing(const int32_t* __restrict__ tile_offset, const Sets2D& sets, int c,
                                                int ct, int T) {
  if (sets.begin == nullptr) return false;
  const int cf = set_first_camera(sets.begin, sets.F, c);
  if (cf == c) return false;
  const int ctl = cf * T + (ct - c * T);
  return tile_offset[ctl + 1] > tile_offset[ctl];
}

// ---------------------------------------------------------------- 3D forward
// Work unit: a 4x4-pixel sub-tile per wave, FOUR lanes per pixel, 4 workgroups of 4 waves per
// tile (one per 8x8 quadrant).  3D: the quadrant's waves share 256-entry rounds -- each entry
// is gathered and culled against the 8x8 quadrant once, into a double-buffered LDS queue, and
// each wave then culls that queue against its 4x4 box (one barrier per round).  2D (every
// tile long and busy): each wave walks the list alone in 64-entry batches.  Either way the
// survivors of a wave's box are composited four at a time: lane
// (pixel p, slot q) evaluates survivor 4t+q for pixel p, and the quad (the 4 lanes of a
// pixel, a DPP quad) combines the four in list order:
//   x_q = 1 - a_q (1 for skipped entries),  T_q = T * prod_{i<q} x_i   (quad prefix product)
//   the first q with T * prod_{i<=q} x_i <= 1e-4 stops the pixel (that entry and the later
//   ones are not composited), the others add c_q a_q T_q,  T <- T * prod_{i<stop} x_i.
// That is gsplat's sequential recursion with the product regrouped in fours (fp32 rounding
// only).  The serial chain per wave is a quarter of the list walk, and the finer cull box
// cuts the evaluated (pixel, entry) pairs.
constexpr int kQuadPrefix1 = 0x90;   // quad_perm [0,0,1,2]: lane q reads lane max(q-1,0)
constexpr int kQuadPrefix2 = 0x40;   // quad_perm [0,0,0,1]: lane q reads lane max(q-2,0)
constexpr int kQuadXor1 = 0xB1;      // quad_perm [1,0,3,2]
constexpr int kQuadXor2 = 0x4E;      // quad_perm [2,3,0,1]

template <int CTRL>
__device__ __forceinline__ int dpp_i(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, true);
}
__device__ __forceinline__ float quad_sum(float v) {
  v += dpp_mov<kQuadXor1>(v);
  return v + dpp_mov<kQuadXor2>(v);
}
__device__ __forceinline__ int quad_min_i(int v) {
  v = min(v, dpp_i<kQuadXor1>(v));
  return min(v, dpp_i<kQuadXor2>(v));
}
// quad minimum of non-negative floats (transmittances): their bit patterns order like int32, so
// the DPP-fused integer min applies (a float min needs NaN-canonicalising moves around it)
__device__ __forceinline__ float quad_min_nonneg(float v) {
  return __int_as_float(quad_min_i(__float_as_int(v)));
}
__device__ __forceinline__ int quad_max_i(int v) {
  v = max(v, dpp_i<kQuadXor1>(v));
  return max(v, dpp_i<kQuadXor2>(v));
}
// A workgroup barrier that also tells whether any thread passed `live` (the forward round loops'
// exit test).  __syncthreads_count took three barriers around an LDS atomic; here each wave posts
// its ballot to its own word of `flags` and ONE barrier follows.  The caller double-buffers
// `flags` by round parity: a fast wave writes round r+2's words only after the barrier of round
// r+1, which every wave reaches after reading round r's.
template <int NW>
__device__ __forceinline__ bool sync_any(bool live, int* flags) {
  const bool w = __ballot(live) != 0ull;
  if ((threadIdx.x & 63) == 0) flags[threadIdx.x >> 6] = w ? 1 : 0;
  __syncthreads();
  int a = 0;
#pragma unroll
  for (int i = 0; i < NW; ++i) a |= flags[i];
  return a != 0;
}

// Operations over the LPP lanes that serve one pixel in the forward: a DPP quad (LPP 4) or a
// DPP row (LPP 16); q = the lane's slot in its group.  prefix: inclusive (Q) and exclusive (P)
// products over the slots in order; suffix_excl: sum over the slots after q; next: slot q+1's
// value.  The DPP moves run in every lane (a DPP read of a lane that is switched off returns
// 0); only the selects depend on the slot.
template <int LPP>
struct PixGroup;
template <>
struct PixGroup<4> {
  static __device__ __forceinline__ int min_i(int v) { return quad_min_i(v); }
  static __device__ __forceinline__ int max_i(int v) { return quad_max_i(v); }
  static __device__ __forceinline__ float sum(float v) { return quad_sum(v); }
  static __device__ __forceinline__ void prefix(float x, int q, float& Q, float& P) {
    const float d1 = dpp_mov<kQuadPrefix1>(x);
    const float q1 = x * (q >= 1 ? d1 : 1.f);
    const float d2 = dpp_mov<kQuadPrefix2>(q1);
    Q = q1 * (q >= 2 ? d2 : 1.f);
    const float d3 = dpp_mov<kQuadPrefix1>(Q);
    P = q >= 1 ? d3 : 1.f;
  }
  static __device__ __forceinline__ float suffix_excl(float v, int q) {
    const float d1 = dpp_mov<0xF9>(v);   // quad_perm [1,2,3,3]
    const float y1 = v + (q < 3 ? d1 : 0.f);
    const float d2 = dpp_mov<0xFE>(y1);  // quad_perm [2,3,3,3]
    const float y2 = y1 + (q < 2 ? d2 : 0.f);
    const float e = dpp_mov<0xF9>(y2);
    return q < 3 ? e : 0.f;
  }
  static __device__ __forceinline__ float next(float v) { return dpp_mov<0xF9>(v); }
};
template <>
struct PixGroup<16> {
  static __device__ __forceinline__ int min_i(int v) {
    v = quad_min_i(v);
    v = min(v, dpp_i<0x141>(v));   // row_half_mirror
    return min(v, dpp_i<0x140>(v));   // row_mirror
  }
  static __device__ __forceinline__ int max_i(int v) {
    v = quad_max_i(v);
    v = max(v, dpp_i<0x141>(v));
    return max(v, dpp_i<0x140>(v));
  }
  static __device__ __forceinline__ float sum(float v) {
    v = quad_sum(v);
    v += dpp_mov<0x141>(v);
    return v + dpp_mov<0x140>(v);
  }
  static __device__ __forceinline__ void prefix(float x, int q, float& Q, float& P) {
    float y = x, d;
    d = dpp_mov<0x111>(y); y *= (q >= 1 ? d : 1.f);   // row_shr:1 (lane - 1)
    d = dpp_mov<0x112>(y); y *= (q >= 2 ? d : 1.f);
    d = dpp_mov<0x114>(y); y *= (q >= 4 ? d : 1.f);
    d = dpp_mov<0x118>(y); y *= (q >= 8 ? d : 1.f);
    Q = y;
    d = dpp_mov<0x111>(y);
    P = q >= 1 ? d : 1.f;
  }
  static __device__ __forceinline__ float suffix_excl(float v, int q) {
    float y = v, d;
    d = dpp_mov<0x101>(y); y += (q < 15 ? d : 0.f);   // row_shl:1 (lane + 1)
    d = dpp_mov<0x102>(y); y += (q < 14 ? d : 0.f);
    d = dpp_mov<0x104>(y); y += (q < 12 ? d : 0.f);
    d = dpp_mov<0x108>(y); y += (q < 8 ? d : 0.f);
    d = dpp_mov<0x101>(y);
    return q < 15 ? d : 0.f;
  }
  static __device__ __forceinline__ float next(float v) { return dpp_mov<0x101>(v); }
};

// 8 lanes per pixel (the heavy-tile forward, k_raster_fwd<false, 8, 8>): a half row of DPP
template <>
struct PixGroup<8> {
  static __device__ __forceinline__ int min_i(int v) {
    v = quad_min_i(v);
    return min(v, dpp_i<0x141>(v));   // row_half_mirror: lane i <-> 7 - i of its half row
  }
  static __device__ __forceinline__ int max_i(int v) {
    v = quad_max_i(v);
    return max(v, dpp_i<0x141>(v));
  }
  static __device__ __forceinline__ float sum(float v) {
    v = quad_sum(v);
    return v + dpp_mov<0x141>(v);
  }
  static __device__ __forceinline__ void prefix(float x, int q, float& Q, float& P) {
    float y = x, d;
    d = dpp_mov<0x111>(y); y *= (q >= 1 ? d : 1.f);   // row_shr:1 (lane - 1)
    d = dpp_mov<0x112>(y); y *= (q >= 2 ? d : 1.f);
    d = dpp_mov<0x114>(y); y *= (q >= 4 ? d : 1.f);
    Q = y;
    d = dpp_mov<0x111>(y);
    P = q >= 1 ? d : 1.f;
  }
  static __device__ __forceinline__ float suffix_excl(float v, int q) {
    float y = v, d;
    d = dpp_mov<0x101>(y); y += (q < 7 ? d : 0.f);   // row_shl:1 (lane + 1)
    d = dpp_mov<0x102>(y); y += (q < 6 ? d : 0.f);
    d = dpp_mov<0x104>(y); y += (q < 4 ? d : 0.f);
    d = dpp_mov<0x101>(y);
    return q < 7 ? d : 0.f;
  }
  static __device__ __forceinline__ float next(float v) { return dpp_mov<0x101>(v); }
};

// Forward geometry per lanes-per-pixel and waves per workgroup: LPP 4 -> 4 workgroups per tile
// (8x8 quadrants), waves of 4x4 pixels; LPP 16 -> 16 workgroups per tile (4x4 boxes), waves of
// 2x2 pixels (the latency mode: a quarter of the serial chain, for scenes with few busy tiles);
// LPP 8 with 8 waves (the heavy-tile forward) -> 4 workgroups per tile (8x8 quadrants), waves
// of 4x2 pixels and rounds of 512 list entries (half the rounds of the quad layout).
template <int LPP, int NW = 4>
struct FwdShape {
  static constexpr int G = LPP == 16 ? 16 : 4;         // workgroups per tile
  static constexpr int WB = LPP == 16 ? 4 : 8;         // workgroup box side
  static constexpr int VBX = LPP == 16 ? 2 : 4;        // wave box width
  static constexpr int VBY = 64 / LPP / VBX;           // wave box height
  static constexpr int WPR = WB / VBX;                 // wave boxes per row of the workgroup box
  static_assert(VBX * VBY * LPP == 64, "a wave is VBX x VBY pixels x LPP lanes");
  static_assert(NW * VBX * VBY == WB * WB, "the waves tile the workgroup box");
};
// workgroups for the busy tiles: G per tile, rounded up to whole groups of 8 tiles
template <int LPP, int NW = 4>
__host__ __device__ __forceinline__ int busy_grid(int n_busy) { return 8 * FwdShape<LPP, NW>::G * ((n_busy + 7) / 8); }
// Heavy tiles (gsr_set_fwd_heavy, OFF by default): busy tiles whose lists have at least
// stats->heavy_min_len entries (at most kFwdHeavyMax of them) run the 8-wave forward on a side
// stream (forked and joined inside gsr3d_raster_fwd) while the quad forward takes the others.
// 512-entry rounds halve a walk's rounds, each gathered and culled by 8 waves in parallel.
// Measured (round 5, config 3): serialised, the 8-wave kernel renders the lists >= 4096 in 42 us
// (their walks set the quad forward's ~100 us span), but the quad forward over the rest still
// takes 84 us; run concurrently the two kernels contend for the CUs (quad 105 -> 131 us, step
// 0.383 -> 0.405 ms; with the side stream at the highest priority a captured step took 0.60 ms),
// and every tile in the 8-wave layout is slower (raster fwd 107 -> 120 us, config 5 389 -> 516 us)
// -- the forward is throughput-bound beyond its heaviest walks.


// slot of tile pixel (il, jl) in a chunk record: box-major inside the 8x8 quadrant wv,
// 64 * wv + 16 * box + pos (pos = pixel within its 4x4 box).  The quad forward writes one 4x4
// box per wave, so its 16 records are 256 contiguous bytes (full lines; the backward's
// lane-interleaved order, 64 * wv + 4 * pos + box, put them 64 B apart); a backward or box-
// forward wave (lane = 4 * pos + box) covers its quadrant's 1 KB, permuted, in one access.
__device__ __forceinline__ int ckpt_slot_of(int wv, int box, int pos) { return (wv << 6) | (box << 4) | pos; }
__device__ __forceinline__ int bwd_pixel_slot(int il, int jl) {
  const int wv = ((il >> 3) << 1) | (jl >> 3);
  const int box = (((il >> 2) & 1) << 1) | ((jl >> 2) & 1);
  const int pos = ((il & 3) << 2) | (jl & 3);
  return ckpt_slot_of(wv, box, pos);
}

//
// 2D (IS2D, the reference's index-order compositor, src/gaussian_renderer.py:416-425) runs
// the same kernel with the reference's arithmetic in transmittance form: integer pixel
// centres, alpha = o exp(-q) with no clamp and no skip threshold (entries with alpha below
// eps_cut -- the binning's extent cut -- are the only ones left out, as in every sub-tile
// the binning drops), and the saturation stop of the reference (A reaches 1.0f, after which
// every contribution is exactly 0) becomes "stop AFTER the entry that takes T to <= 2^-25"
// (the half-ulp of 1.0f below which A = 1 - T rounds to 1).  final_T holds (T_final,
// T before the last composited entry) per pixel: the backward's division-free start at a
// pixel's last entry (its 1 - alpha may be exactly 0 when opacity == 1.0f).
constexpr float kT2DMin = 2.98023224e-8f;   // 2^-25

// Lazy depth order (3D; binning.hip LazyArgs): the forward walks each list only to the end of
// its sorted prefix (tile_sorted) and flags the tile when the walk got there -- a pixel still
// live, or one whose last composited entry is the prefix's last (the cut key of the next
// entry must come from a sorted list).  rerun: the second pass over the flagged tiles
// (list[0..count), sorted whole by then), from scratch.

struct FwdLazy {
  const int32_t* tile_sorted;
  int32_t* flag;
  int32_t* list;
  int32_t* count;
  int rerun;
};

__device__ __forceinline__ void lazy_flag_tile(const FwdLazy& lz, int ct) {
  if (atomicExch(&lz.flag[ct], 1) == 0) lz.list[atomicAdd(lz.count, 1)] = ct;
}

#ifdef GSR_FWD_TRACE
// timing build only (tools/fwd_trace.py): per workgroup {start, first round in, walk done, end,
// rounds, list entries, hw id}
__device__ unsigned long long* g_fwd_trace = nullptr;
extern "C" int gsr_debug_fwd_trace(void* buf) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_fwd_trace), &buf, sizeof(buf)) == hipSuccess ? 0 : 1;
}
#define FWD_T(i) if (threadIdx.x == 0) s_ftr[i] = wall_clock64()
// per-round phase accumulators of wave 0 (3D quad layout): 0 gather wait + quadrant cull,
// 1 round barrier, 2 box culls, 3 composites
#define FWD_P(k)                                          \
  if (threadIdx.x == 0) {                                 \
    const unsigned long long now_ = wall_clock64();       \
    f_acc[k] += now_ - f_t;                               \
    f_t = now_;                                           \
  }
#else
#define FWD_T(i)
#define FWD_P(k)
#endif
// minimum workgroups per CU of the 3D quad-layout raster forward (build knob for measurements):
// 6 fit 25.9 KB of LDS (queue entry offsets as bytes) and 79 VGPRs without spills -- config 3
// raster fwd 116.2 -> 111.0 us, config 5 416 -> 408 us (r03s2 A/B on one box); the 16-lane
// layout (few busy tiles: latency, not occupancy) keeps the compiler's choice
#ifndef GSR_FWD_MINB
#define GSR_FWD_MINB 6
#endif
#ifndef GSR_FWD_PRIO
#define GSR_FWD_PRIO 3       // s_setprio of the waves of long-list tiles (0: off; 3: +0.7 % at config 3, r06 A/B)
#endif
#ifndef GSR_FWD_PRIO_LEN
#define GSR_FWD_PRIO_LEN 2048
#endif
#ifndef GSR_BOXM
#define GSR_BOXM 1   // the quad forward writes each chunk's box survivor masks for the backward
#endif
#ifndef GSR_FWD_SLOTPF
#define GSR_FWD_SLOTPF 1   // 0: plain slot reads (folded into one read at the use: measurement knob)
#endif
template <typename T>
__device__ __forceinline__ int fwd_slot(T* p) {
#if GSR_FWD_SLOTPF
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
#else
  return *p;
#endif
}
#ifndef GSR_FWD_PF2
#define GSR_FWD_PF2 0   // 1: 3D quad rounds gather records two rounds ahead (12 more VGPRs)
#endif
// NW: waves per workgroup (4; 8 for the heavy-tile variant, LPP 8).  part: 0 every busy tile,
// 1 the tiles with lists shorter than stats->heavy_min_len, 2 the others (the heavy tiles: a
// first-pass forward finds them at the head of the busy order, a lazy re-render anywhere in its list).
template <bool IS2D, int LPP, int NW = 4>
__global__ __launch_bounds__(NW * 64, NW == 8 ? 6 : (IS2D || LPP != 4) ? 1 : GSR_FWD_MINB) void k_raster_fwd(
    const Splat* __restrict__ rec, const int32_t* __restrict__ ids, const int32_t* __restrict__ kos,
    const int32_t* __restrict__ tile_offset,
    const int32_t* __restrict__ order, int W, int H, int tw, int th, const float* __restrict__ bg,
    float* __restrict__ out_rgb, float* __restrict__ out_alpha, float* __restrict__ out_T,
    int32_t* __restrict__ out_last, int32_t* __restrict__ tile_end, float4* __restrict__ ckpt,
    const int32_t* __restrict__ chunk_base, int n_busy, int64_t CT,
    uint64_t* __restrict__ tile_cut, float cut2d, const FwdLazy lz, const gsr_bin_stats* __restrict__ stats,
    const Sets2D sets, int part = 0, uint4* __restrict__ boxm = nullptr) {
  static_assert(!IS2D || LPP == 4, "2D walks per wave with quads");
  static_assert(NW == 4 || (NW == 8 && !IS2D && LPP == 8), "8 waves: the 3D heavy-tile layout");
  using PG = PixGroup<LPP>;
  using FS = FwdShape<LPP, NW>;
  constexpr int NT = NW * 64;   // threads; a 3D round gathers NT list entries
  __shared__ int s_max;
#ifdef GSR_FWD_TRACE
  __shared__ unsigned long long s_ftr[4];
  int n_rounds = 0;
  unsigned long long f_acc[4] = {0ull, 0ull, 0ull, 0ull}, f_t = wall_clock64();
  unsigned long long f_groups = 0, f_surv = 0;
  FWD_T(0);
#endif
  // n_busy sizes the grid (the read-back busy count or a bound); the tiles come from the device
  // count, which the sort has checked against that bound (GSR_OVF_BUSY)
  const int busy_blocks = busy_grid<LPP, NW>(n_busy);
  // XCD-aware mapping: workgroups are dealt to the 8 XCDs round-robin by id, so the G
  // workgroups of a tile get ids 8G*k + 8*sub + x (same id mod 8): they share one XCD's L2
  // for the tile's records.  Busy tile u = 8k + x, in longest-first order.
  const int u = ((int)blockIdx.x / (8 * FS::G)) * 8 + ((int)blockIdx.x & 7);
  const int sub = ((int)blockIdx.x >> 3) & (FS::G - 1);
  // the device counts and this workgroup's tile are loaded together (one round trip before
  // any work, as with a host count); the tile index is clamped in range and used only if real
  if (lz.rerun) order = lz.list;
  const int ct = order[min(u, (int)CT - 1)];
  const int ovf = stats->overflow;
  const int nb_dev = lz.rerun ? *lz.count : stats->n_busy;
  // (a lazy re-render's list holds only *lz.count tiles: slots past it are stale, never a fault)
  if (ovf | ((ct < 0) & (u < nb_dev))) {
    // (the sticky status is also set here: a forward with no backward skips the finalize)
    if (blockIdx.x == 0 && threadIdx.x == 0 && stats->status != nullptr) atomicOr(stats->status, ovf);
    nan_fill(CT, W, H, tw, th, out_rgb, out_alpha);
    return;
  }
  if (lz.rerun) {
    n_busy = min(n_busy, nb_dev);
  } else {
    n_busy = nb_dev;
    if ((int)blockIdx.x >= busy_blocks) {
      fill_empty<IS2D>(order, tile_offset, n_busy, busy_blocks, CT, W, H, tw, th, bg, out_rgb, out_alpha, out_T,
                       out_last, tile_end, tile_cut, sets, stats->status);
      return;
    }
  }
  if (u >= n_busy) return;

  int c, ty, tx;
  tile_coords(ct, tw, th, c, ty, tx);
  if constexpr (IS2D) rec += rec_offset2d(sets.begin, sets.F, c, sets.N);   // the set's record copy
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int q = lane & (LPP - 1), p = lane / LPP;
  const int sx = (sub % (kTile / FS::WB)) * FS::WB, sy = (sub / (kTile / FS::WB)) * FS::WB;
  const int ox = sx + (wv % FS::WPR) * FS::VBX, oy = sy + (wv / FS::WPR) * FS::VBY;
  const int il = oy + p / FS::VBX, jl = ox + p % FS::VBX;
  const int i = ty * kTile + il, j = tx * kTile + jl;
  const bool inside = i < H && j < W;
  const float off = IS2D ? 0.f : 0.5f;   // 2D: integer centres (src/gaussian_renderer.py:355-358)
  const float px = (float)j + off, py = (float)i + off;
  const float bx0 = (float)(tx * kTile + ox) + off, bx1 = bx0 + (float)(FS::VBX - 1);
  const float by0 = (float)(ty * kTile + oy) + off, by1 = by0 + (float)(FS::VBY - 1);
  const int start = tile_offset[ct], list_end = tile_offset[ct + 1];
  if (part != 0 && (part == 2) != (list_end - start >= stats->heavy_min_len)) return;   // heavy / light split
  const int end = lz.tile_sorted && !lz.rerun ? lz.tile_sorted[ct] : list_end;
#if GSR_FWD_PRIO
  // long lists: the serial round chains that set the forward's span win the CU's issue arbitration
  if (!IS2D && list_end - start >= GSR_FWD_PRIO_LEN) __builtin_amdgcn_s_setprio(GSR_FWD_PRIO);
#endif
  if (threadIdx.x == 0) s_max = -1;
  __syncthreads();
  float T = 1.f, cr = 0.f, cg = 0.f, cb = 0.f;
  float Tl = 1.f;   // 2D: T before this lane's latest composited entry
  int last = -1;
  bool done = !inside;
  // chunk records for the chunk-parallel backward (per pixel, per chunk of stats->chunk_entries
  // list entries, a power-of-two multiple of the 128-entry round half)
  const int cbase = chunk_base[ct];
  const int umask = stats->chunk_entries - 1;
  int kcur = 0;
  float Ts = 1.f, dr = 0.f, dg = 0.f, db = 0.f;   // dr..: this lane's share of the chunk's colour
  if constexpr (!IS2D) {
  // one array (records of slot i at s_q[buf][0..2][i]): one address, immediate offsets
  using QIdx = typename std::conditional<(NT > 256), unsigned short, unsigned char>::type;
  __shared__ float4 s_q[2][3][NT];
  __shared__ QIdx s_qe[2][NT];   // entry - round base (LDS: 6 workgroups per CU at 4 waves)
  __shared__ int s_qn[2][NW];
  __shared__ __attribute__((aligned(16))) int s_live[2][NW];
  __shared__ QIdx s_l[NW][128];
  // box survivor masks for the backward (boxm): per wave, one flag byte per entry of the half
  constexpr bool kBoxMasks = LPP == 4 && NW == 4;   // the quad layout's waves are the 4x4 boxes
  __shared__ __attribute__((aligned(4))) unsigned char s_fl[kBoxMasks ? NW : 1][128];
  const bool wbm = kBoxMasks && boxm != nullptr && ckpt != nullptr && umask == kChunk3 - 1;
  if (wbm && blockIdx.x == 0 && threadIdx.x == 0) atomicOr(const_cast<int32_t*>(&stats->masks), kStatsBoxMasks);
  // 3D -- shared rounds: the quadrant workgroup walks the list in 256-entry rounds; wave w gathers
  // entries 64w..64w+63 of the round (one round ahead), culls them against the 8x8 quadrant
  // and writes its survivors to segment w of a double-buffered LDS queue; after ONE barrier
  // per round every wave culls the queue against its 4x4 box (two halves = two 128-entry
  // chunks) and composites its survivors as below.  Each entry is gathered and 8x8-culled
  // once per quadrant instead of once per wave.
  static_assert(kChunk3 % 128 == 0, "a round half is one 128-entry chunk");
  const int e_last = max(end - 1, start);
  const float qx0 = (float)(tx * kTile + sx) + off, qx1 = qx0 + (float)(FS::WB - 1);
  const float qy0 = (float)(ty * kTile + sy) + off, qy1 = qy0 + (float)(FS::WB - 1);
  float4 c0 = make_float4(0.f, 0.f, 0.f, 0.f), c1 = c0, c2 = c0;
  // quadrant masks (kos: gsr_bin_emit's bits 28..31): an entry whose bit for this workgroup's
  // 8x8 quadrant is clear cannot reach it -- its record is not even gathered (an entry reaches
  // 1.27 of its tile's 4 quadrants at config 3).  Kept entries still take the exact cull.
  const int qbit = kMaskShift + ((sy >> 3) << 1) + (sx >> 3);
  if ((stats->masks & kStatsMasks3D) == 0) kos = nullptr;   // this call's emission stored no masks
  // kn: the raw emission word of the entry two rounds ahead (all bits set without masks), tested
  // only when its record is gathered a round later.  (Testing it at its load made every round
  // wait out that load's full latency: the mask is an SGPR lane mask, so the compiler placed a
  // vmcnt(0) right behind the two loads.)
  int idn = 0, kn = -1;
  bool ucur = false;
  // (without masks kn is read from ids, a word of the same line as idn, and never tested: a
  // conditional load kept the old kn live beside the new one, and the loop's latch then copied
  // the loaded registers -- a vmcnt(0) behind every round's record gather)
  const int32_t* const kptr = kos != nullptr ? kos : ids;
  // rounds of records in flight: 1, or (GSR_FWD_PF2) 2 in two register sets that the rounds use
  // in turn (no copies: a copy of a set waits for its load)
  constexpr int kAhead = GSR_FWD_PF2 ? 2 : 1;
#if GSR_FWD_PF2
  float4 d0 = c0, d1 = c0, d2 = c0;
  bool unext = false;
#endif
  if (end > start) {
    const int e0 = min(start + 64 * wv + lane, e_last), e1 = min(start + NT + 64 * wv + lane, e_last);
    const int id0 = ids[e0];
    ucur = kos == nullptr || ((kos[e0] >> qbit) & 1);
#if GSR_FWD_PF2
    const int e2 = min(start + 2 * NT + 64 * wv + lane, e_last);
    const int id1 = ids[e1];
    unext = kos == nullptr || ((kos[e1] >> qbit) & 1);
    idn = ids[e2];
    kn = kptr[e2];
#else
    idn = ids[e1];
    kn = kptr[e1];
#endif
    if (ucur) {
      const Splat s0 = rec[id0];
      c0 = s0.p0; c1 = s0.p1; c2 = s0.p2;
    }
#if GSR_FWD_PF2
    if (unext) {
      const Splat s1 = rec[id1];
      d0 = s1.p0; d1 = s1.p1; d2 = s1.p2;
    }
#endif
  }
  // one round: cull the set x (this round's records) into the queue, gather into x the records
  // kAhead rounds on and the ids one round further, then the round's walk.  false: every pixel
  // of the workgroup is done.
  auto round = [&](int rb, int buf, float4& x0, float4& x1, float4& x2, bool& ux) -> bool {
#ifdef GSR_FWD_TRACE
    if (threadIdx.x == 0) f_t = wall_clock64();
#endif
    {
      const int e = rb + 64 * wv + lane;
      const bool keep = e < end && ux && cull_keep<IS2D>(x0, x1, x2, qx0, qx1, qy0, qy1);
      const unsigned long long m = __ballot(keep);
      if (keep) {
        const int slot = 64 * wv +
                         __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
        s_q[buf][0][slot] = x0;
        s_q[buf][1][slot] = x1;
        s_q[buf][2][slot] = x2;
        s_qe[buf][slot] = (QIdx)(64 * wv + lane);   // e - rb
      }
      if (lane == 0) s_qn[buf][wv] = __popcll(m);
      // the records kAhead rounds on first, then the ids one round further into the registers the
      // records' addresses have just freed (loaded in place: no copy at the loop's latch)
      ux = kos == nullptr || ((kn >> qbit) & 1) != 0;
      if (ux) {
        const Splat sn = rec[idn];
        x0 = sn.p0; x1 = sn.p1; x2 = sn.p2;
      }
      const int en = min(rb + (kAhead + 1) * NT + 64 * wv + lane, e_last);
      idn = ids[en];
      kn = kptr[en];
    }
    FWD_P(0);
    if (!sync_any<NW>(!done, s_live[buf])) return false;
    FWD_P(1);
#ifdef GSR_FWD_TRACE
    if (n_rounds++ == 0) FWD_T(1);
#endif
    for (int h = 0; h < NT / 128; ++h) {
      const int hb = rb + 128 * h;
      // (a wave whose pixels are all done writes no more box masks: the backward reads a box's
      // masks only up to the box's last composited entry)
      if (hb >= end || __ballot(!done) == 0ull) break;
      if (hb > start && ((hb - start) & umask) == 0) {   // entering chunk kcur+1
        const float Dr = PG::sum(dr), Dg = PG::sum(dg), Db = PG::sum(db);
        if (q == 0 && ckpt) ckpt[(int64_t)(cbase + kcur) * kRasterThreads + bwd_pixel_slot(il, jl)] = make_float4(Ts, Dr, Dg, Db);
        cr += Dr;
        cg += Dg;
        cb += Db;
        dr = dg = db = 0.f;
        Ts = T;
        ++kcur;
      }
      const int na = s_qn[buf][2 * h], nh = na + s_qn[buf][2 * h + 1];
      int n = 0, lastq = -1;
      if (wbm && lane < 32) reinterpret_cast<uint32_t*>(s_fl[wv])[lane] = 0u;
      __builtin_amdgcn_wave_barrier();
      for (int r0 = 0; r0 < nh; r0 += 64) {
        const int ii = r0 + lane;
        const int idx = ii < na ? 128 * h + ii : 128 * h + 64 + (ii - na);
        const bool keep = ii < nh && cull_keep<IS2D>(s_q[buf][0][idx], s_q[buf][1][idx], s_q[buf][2][idx], bx0, bx1, by0, by1);
        const unsigned long long m = __ballot(keep);
        if (keep) {
          s_l[wv][n + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0))] =
              (QIdx)idx;
          if (wbm) s_fl[wv][s_qe[buf][idx] - 128 * h] = 1;   // (entry - hb: this half's 128)
        }
        n += __popcll(m);
      }
      __builtin_amdgcn_wave_barrier();

      FWD_P(2);
#ifdef GSR_FWD_TRACE
      f_groups += (n + LPP - 1) / LPP;
      f_surv += n;
#endif
      // the next group's queue slot is read one group ahead (one LDS round trip less on the
      // serial chain of a group)
      // (relaxed atomic reads: instcombine folds a phi of two plain loads into ONE load at the
      // use, which put the slot read back on the group's chain; atomic loads are not folded)
      QIdx* const lq = s_l[wv];
      int idx_next = fwd_slot(lq + (q < n ? q : max(n - 1, 0)));
      for (int k0 = 0; k0 < n; k0 += LPP) {
        const int k = k0 + q;
        const int idx = idx_next;
        idx_next = fwd_slot(lq + (k + LPP < n ? k + LPP : n - 1));
        const float4 p0 = s_q[buf][0][idx];
        const float4 p1 = s_q[buf][1][idx];
        const float4 p2 = s_q[buf][2][idx];
        const float dx = p0.x - px, dy = p0.y - py;
        const float sg = conic_sigma(p1, dx, dy);
        const float raw = p0.z * gauss_exp<IS2D>(sg);
        const float alpha = IS2D ? raw : fminf(kAlphaMax, raw);
        const bool valid = IS2D ? (k < n && !done && alpha >= cut2d)
                                : (k < n && !done && sg >= 0.f && alpha >= kAlphaThreshold);
        const float xq = valid ? 1.f - alpha : 1.f;
        float Qi, Pe;
        PG::prefix(xq, q, Qi, Pe);
        const float nT = T * Qi;
        const int fs = PG::min_i(valid && nT <= (IS2D ? kT2DMin : kTMin) ? q : LPP);
        const bool con = valid && (IS2D ? q <= fs : q < fs);
        const float Tq = T * Pe;
        const float vis = con ? alpha * Tq : 0.f;
        dr += p2.x * vis;
        dg += p2.y * vis;
        db += p2.z * vis;
        lastq = con ? idx : lastq;
        if (IS2D) Tl = con ? Tq : Tl;
        // the group minimum of non-negative transmittances, on their int32 bit patterns
        T = __int_as_float(PG::min_i(__float_as_int((IS2D ? q <= fs : q < fs) ? nT : T)));
        done = done || fs < LPP;
      }
      if (wbm) {
        // the box's survivors of this 128-entry chunk as a 128-bit mask over its entries (read
        // after the walk: off the walk's serial chain)
        const unsigned long long blo = __ballot(s_fl[wv][lane] != 0), bhi = __ballot(s_fl[wv][64 + lane] != 0);
        if (lane == 0)
          boxm[(int64_t)(cbase + ((hb - start) >> 7)) * 16 + 4 * sub + wv] =
              make_uint4((uint32_t)blo, (uint32_t)(blo >> 32), (uint32_t)bhi, (uint32_t)(bhi >> 32));
      }
      if (lastq >= 0) {   // the entry index of this lane's latest composite, once per half
        last = rb + s_qe[buf][lastq];
        lastq = -1;
      }
      __builtin_amdgcn_wave_barrier();
      FWD_P(3);
    }
    return true;
  };
#if GSR_FWD_PF2
  for (int rb = start; rb < end; rb += 2 * NT) {
    if (!round(rb, 0, c0, c1, c2, ucur)) break;
    if (rb + NT >= end || !round(rb + NT, 1, d0, d1, d2, unext)) break;
  }
#else
  for (int rb = start, buf = 0; rb < end; rb += NT, buf ^= 1)
    if (!round(rb, buf, c0, c1, c2, ucur)) break;
#endif
  } else {
  // 2D (every tile busy and long; the per-wave walk measured faster there): each wave walks
  // the list on its own in 64-entry batches.
  __shared__ float4 s_pw[4][3][64];
  // software pipeline over 64-entry batches (records of b+1, b+2 and ids of b+3 in flight;
  // see the notes of the 2-way unrolled loop below)
  const int e_last = max(end - 1, start);
  const float4 zero4 = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 x0 = zero4, x1 = zero4, x2 = zero4, y0 = zero4, y1 = zero4, y2 = zero4;
  int idp = 0, idq = 0;
  if (end > start) {
    const int ida = ids[min(start + lane, e_last)];
    const int idb = ids[min(start + 64 + lane, e_last)];
    const Splat sa = rec[ida];
    idp = ids[min(start + 128 + lane, e_last)];
    const Splat sb = rec[idb];
    x0 = sa.p0; x1 = sa.p1; x2 = sa.p2;
    y0 = sb.p0; y1 = sb.p1; y2 = sb.p2;
    unpack_rec<IS2D>(x0, x1, x2);   // (2D records are stored packed: pack_rec)
    unpack_rec<IS2D>(y0, y1, y2);
  }
  // One batch: cull + compact c (batch b0), refill c with batch b0+128 (id_use), load the ids
  // of batch b0+192 into id_new (issued BEFORE the record loads, so waiting for an id never
  // waits for younger record loads), composite.  false = every pixel of the wave is done.
  auto step = [&](int b0, float4& c0, float4& c1, float4& c2, int id_use, int& id_new) -> bool {
    if (__ballot(!done) == 0ull) return false;
    if (b0 > start && ((b0 - start) & umask) == 0) {   // entering chunk kcur+1
      const float Dr = quad_sum(dr), Dg = quad_sum(dg), Db = quad_sum(db);
      // 2D: the pixel's T anchor at the chunk start (k_raster2d_bwd_tile)
      if (q == 0 && ckpt)
        reinterpret_cast<float*>(ckpt)[(int64_t)(cbase + kcur + 1) * kRasterThreads + bwd_pixel_slot(il, jl)] = T;
      cr += Dr;
      cg += Dg;
      cb += Db;
      dr = dg = db = 0.f;
      Ts = T;
      ++kcur;
    }
    const bool keep = (b0 + lane < end) && cull_keep<IS2D>(c0, c1, c2, bx0, bx1, by0, by1);
    const unsigned long long m = __ballot(keep);
    const int n = __popcll(m);
    if (keep) {
      const int slot = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
      s_pw[wv][0][slot] = c0;
      s_pw[wv][1][slot] = make_float4(c1.x, c1.y, c1.z, __int_as_float(b0 + lane));
      s_pw[wv][2][slot] = c2;
    }
    id_new = ids[min(b0 + 192 + lane, e_last)];
    const Splat sc = rec[id_use];
    c0 = sc.p0; c1 = sc.p1; c2 = sc.p2;
    unpack_rec<IS2D>(c0, c1, c2);
    __builtin_amdgcn_wave_barrier();
    for (int k0 = 0; k0 < n; k0 += 4) {
      const int k = k0 + q;
      const int kk = k < n ? k : n - 1;
      const float4 p0 = s_pw[wv][0][kk];
      const float4 p1 = s_pw[wv][1][kk];
      const float4 p2 = s_pw[wv][2][kk];
      const float dx = p0.x - px, dy = p0.y - py;
      const float sg = conic_sigma(p1, dx, dy);
      const float raw = p0.z * gauss_exp<IS2D>(sg);
      const float alpha = IS2D ? raw : fminf(kAlphaMax, raw);
      const bool valid = IS2D ? (k < n && !done && alpha >= cut2d)
                              : (k < n && !done && sg >= 0.f && alpha >= kAlphaThreshold);
      const float xq = valid ? 1.f - alpha : 1.f;
      // quad prefix products of x (inclusive Q, exclusive P).  The DPP moves run in every
      // lane (a DPP read of a lane that is switched off returns 0); only the selects depend
      // on the slot.
      const float d1 = dpp_mov<kQuadPrefix1>(xq);
      const float q1 = xq * (q >= 1 ? d1 : 1.f);
      const float d2 = dpp_mov<kQuadPrefix2>(q1);
      const float Qi = q1 * (q >= 2 ? d2 : 1.f);      // prod_{i<=q} x_i
      const float d3 = dpp_mov<kQuadPrefix1>(Qi);
      const float Pe = q >= 1 ? d3 : 1.f;             // prod_{i<q} x_i
      const float nT = T * Qi;
      // first stopping slot: 3D stops BEFORE the entry that takes T to <= 1e-4, 2D after
      // the one that takes it to <= 2^-25 (the reference's A == 1.0f)
      const int fs = quad_min_i(valid && nT <= (IS2D ? kT2DMin : kTMin) ? q : 4);
      const bool con = valid && (IS2D ? q <= fs : q < fs);
      const float Tq = T * Pe;
      const float vis = con ? alpha * Tq : 0.f;
      dr += p2.x * vis;
      dg += p2.y * vis;
      db += p2.z * vis;
      last = con ? __float_as_int(p1.w) : last;
      if (IS2D) Tl = con ? Tq : Tl;
      T = quad_min_nonneg((IS2D ? q <= fs : q < fs) ? nT : T);
      done = done || fs < 4;
    }
    __builtin_amdgcn_wave_barrier();
    return true;
  };
  for (int b0 = start; b0 < end; b0 += 128) {
    if (!step(b0, x0, x1, x2, idp, idq)) break;
    if (b0 + 64 >= end || !step(b0 + 64, y0, y1, y2, idq, idp)) break;
  }
  }
#ifdef GSR_FWD_TRACE
  __syncthreads();
  FWD_T(2);
#endif
  const float Dr = PG::sum(dr), Dg = PG::sum(dg), Db = PG::sum(db);
  cr += Dr;
  cg += Dg;
  cb += Db;
  if (IS2D) {
    // quad arg-max of last, carrying the T before that entry
    int ol = dpp_i<kQuadXor1>(last);
    float oT = dpp_mov<kQuadXor1>(Tl);
    Tl = ol > last ? oT : Tl;
    last = max(last, ol);
    ol = dpp_i<kQuadXor2>(last);
    oT = dpp_mov<kQuadXor2>(Tl);
    Tl = ol > last ? oT : Tl;
    last = max(last, ol);
  } else {
    last = PG::max_i(last);
  }
  // (no chunk records: a forward with no backward to follow; 2D: the T anchors are final)
  if (!IS2D && end > start && ckpt) {
    // Turn this pixel's chunk records {T at chunk start, chunk colour sum} into what the
    // backward needs at each chunk's END: {T_end, suffix colour sum of the later chunks}
    // (positive terms, summed back to front).  The pixel's LPP lanes split the chunks into
    // LPP contiguous ranges: each sums its range's colour, a group suffix sum of the range
    // sums gives each range's starting suffix, then each rewrites its range back to front
    // (records re-read 8 at a time).  1/LPP of the serial chain of one lane.
    float4* ck = ckpt + (int64_t)cbase * kRasterThreads + bwd_pixel_slot(il, jl);
    if (q == 0) ck[(int64_t)kcur * kRasterThreads] = make_float4(T, 0.f, 0.f, 0.f);
    const int per = (kcur + LPP - 1) / LPP;
    const int r0 = min(kcur, q * per), r1 = min(kcur, r0 + per);
    float Rr = 0.f, Rg = 0.f, Rb = 0.f, F = 0.f;
    for (int k0 = r0; k0 < r1; k0 += 8) {
      float4 r[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (k0 + u < r1) r[u] = ck[(int64_t)(k0 + u) * kRasterThreads];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (k0 + u < r1) {
          if (k0 + u == r0) F = r[u].x;
          Rr += r[u].y;
          Rg += r[u].z;
          Rb += r[u].w;
        }
    }
    // suffix of the later ranges (slots q+1..LPP-1) plus the current chunk's own colour
    const float Fn = PG::next(F);   // F of the next range
    float sr = Dr + PG::suffix_excl(Rr, q), sg = Dg + PG::suffix_excl(Rg, q), sb = Db + PG::suffix_excl(Rb, q);
    float Tn = r1 < kcur ? Fn : Ts;
    for (int k0 = r1 - 1; k0 >= r0; k0 -= 8) {
      float4 r[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (k0 - u >= r0) r[u] = ck[(int64_t)(k0 - u) * kRasterThreads];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (k0 - u >= r0) {
          ck[(int64_t)(k0 - u) * kRasterThreads] = make_float4(Tn, sr, sg, sb);
          Tn = r[u].x;
          sr += r[u].y;
          sg += r[u].z;
          sb += r[u].w;
        }
    }
  }
  if (q == 0 && inside) {
    const int64_t pix = ((int64_t)c * H + i) * W + j;
    const float* bgc = bg + c * 3;
    out_rgb[pix * 3 + 0] = cr + T * bgc[0];
    out_rgb[pix * 3 + 1] = cg + T * bgc[1];
    out_rgb[pix * 3 + 2] = cb + T * bgc[2];
    out_alpha[pix] = 1.f - T;
    if (IS2D)
      reinterpret_cast<float2*>(out_T)[pix] = make_float2(T, Tl);
    else
      out_T[pix] = T;
    out_last[pix] = last;
  }
  if (q == 0 && last >= 0) atomicMax(&s_max, last);
  if (end < list_end) {   // lazy: did the walk reach the end of the sorted prefix?
    if (__syncthreads_or(!done || last == end - 1) && threadIdx.x == 0) lazy_flag_tile(lz, ct);
  } else {
    __syncthreads();
  }
  if (threadIdx.x == 0 && s_max >= 0) atomicMax(&tile_end[ct], s_max);   // finalised by k_raster_finalize
#ifdef GSR_FWD_TRACE
  FWD_T(3);
  if (threadIdx.x == 0 && g_fwd_trace != nullptr) {
    ulonglong2* d = reinterpret_cast<ulonglong2*>(g_fwd_trace + 16 * (int64_t)blockIdx.x);
    d[0] = make_ulonglong2(s_ftr[0], s_ftr[1]);
    d[1] = make_ulonglong2(s_ftr[2], s_ftr[3]);
    d[2] = make_ulonglong2((unsigned long long)n_rounds, (unsigned long long)(list_end - start));
    d[3] = make_ulonglong2((unsigned long long)__smid(), (unsigned long long)ct);
    d[4] = make_ulonglong2(f_acc[0], f_acc[1]);
    d[5] = make_ulonglong2(f_acc[2], f_acc[3]);
    d[6] = make_ulonglong2(f_groups, f_surv);
    d[7] = make_ulonglong2(0ull, 0ull);
  }
#endif
}

// ---------------------------------------------------------------- forward, box layout
// The throughput layout (2D; selectable for 3D): ONE workgroup
// per busy tile, ONE lane per pixel, laid out as in the backward (wave = 8x8 quadrant, lane l
// = pixel l>>2 of the 4x4 box l&3), so each pixel composites its entries with gsplat's
// sequential recursion T <- T (1 - a) -- no quad prefix products, no DPP on the serial chain.
// The tile's list is walked in 256-entry rounds: every thread gathers one entry's record
// (one round ahead) into a double-buffered LDS image; per 128-entry half (one chunk) each
// wave culls the half against its 8x8 quadrant (exact test, as everywhere), then the
// quadrant's survivors against each 4x4 box, and every lane walks its box's survivor list in
// order (the wave runs max over its four boxes; a lane past its own list idles).  A wave
// leaves as soon as all its pixels are done, the workgroup as soon as all four waves are.
// Chunk records are written per pixel at thread index = the backward's slot, coalesced.
template <bool IS2D>
__global__ __launch_bounds__(kRasterThreads, 6) void k_raster_fwd_box(
    const Splat* __restrict__ rec, const int32_t* __restrict__ ids, const int32_t* __restrict__ kos,
    const int32_t* __restrict__ tile_offset,
    const int32_t* __restrict__ order, int W, int H, int tw, int th, const float* __restrict__ bg,
    float* __restrict__ out_rgb, float* __restrict__ out_alpha, float* __restrict__ out_T,
    int32_t* __restrict__ out_last, int32_t* __restrict__ tile_end, float4* __restrict__ ckpt,
    const int32_t* __restrict__ chunk_base, int n_busy, int64_t CT,
    uint64_t* __restrict__ tile_cut, float cut2d, const FwdLazy lz, const gsr_bin_stats* __restrict__ stats,
    const Sets2D sets) {
  (void)kos;   // one workgroup per tile: the waves' own quadrant culls decide
  constexpr bool PACK = IS2D && GSR_BOX_PACK;   // 2D walk: records staged packed (pack_rec)
  // round records, part j of entry k of half h at s_r[buf][j][129 h + k]; slot 129 h + 128 of every
  // part is a zero record (opacity 0: never valid), the 2D walk's pad entry
  constexpr int kHS = 129, kRS = 2 * kHS;
  __shared__ float4 s_r[2][3][kRS];
  // ... and each box's survivors, in list order; 2D reads them four at a time (one b32 per four
  // steps, the next word read ahead: +4), the row stride (132 B = 33 banks) puts the two boxes
  // of a 32-lane half in different banks
  __shared__ __attribute__((aligned(16))) unsigned char s_box[4][4][kBoxStride];
  __shared__ int s_max;
  __shared__ __attribute__((aligned(16))) int s_live[2][4];
  static_assert(kChunk3 == 128, "a round half is one chunk");
  const int busy_blocks = (n_busy + 7) & ~7;   // n_busy: the grid's bound (see k_raster_fwd)
  // device counts and this workgroup's tile in one round trip (see k_raster_fwd); 2D: every tile,
  // busy or empty, in the XCD-aware sweep (sweep_tile2d; an empty list just writes the background)
  if (lz.rerun) order = lz.list;
  const int ct = IS2D ? sweep_tile2d(blockIdx.x, CT, tw * th, sets.begin, sets.F) : order[min((int)blockIdx.x, (int)CT - 1)];
  const int ovf = stats->overflow;
  const int nb_dev = lz.rerun ? *lz.count : stats->n_busy;
  // (a lazy re-render's list holds only *lz.count tiles: slots past it are stale, never a fault)
  if (ovf | (!IS2D & (ct < 0) & ((int)blockIdx.x < nb_dev))) {
    // (the sticky status is also set here: a forward with no backward skips the finalize)
    if (blockIdx.x == 0 && threadIdx.x == 0 && stats->status != nullptr) atomicOr(stats->status, ovf);
    nan_fill(CT, W, H, tw, th, out_rgb, out_alpha);
    return;
  }
  if (IS2D) {
    if (ct < 0) return;
  } else if (lz.rerun) {
    n_busy = min(n_busy, nb_dev);
  } else {
    n_busy = nb_dev;
    if ((int)blockIdx.x >= busy_blocks) {
      fill_empty<IS2D>(order, tile_offset, n_busy, busy_blocks, CT, W, H, tw, th, bg, out_rgb, out_alpha, out_T,
                       out_last, tile_end, tile_cut, sets, stats->status);
      return;
    }
  }
  if (!IS2D && (int)blockIdx.x >= n_busy) return;
  int c, ty, tx;
  tile_coords(ct, tw, th, c, ty, tx);
  if constexpr (IS2D) rec += rec_offset2d(sets.begin, sets.F, c, sets.N);   // the set's record copy
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
#if GSR_BOX_LANES
  // box = the lane's ds_read_b128 group ((bit 5, bit 4 ^ bit 3 ^ bit 2), MI355X_MICROARCH.md
  // §LDS): every b128 record read of the walk is one address per lane group, a broadcast, so
  // the four boxes' different entries never meet on a bank (with box = lane & 3 every group
  // held all four boxes: +32 % LDS cycles in bank conflicts at config 4, r03 PMC)
  const int box = ((lane >> 4) & 2) | (((lane >> 4) ^ (lane >> 3) ^ (lane >> 2)) & 1);
  const int pos = (lane & 3) | ((lane >> 1) & 12);
#else
  const int box = lane & 3, pos = lane >> 2;
#endif
  const float off = IS2D ? 0.f : 0.5f;   // 2D: integer centres (src/gaussian_renderer.py:355-358)
  const int qx0 = tx * kTile + (wv & 1) * 8, qy0 = ty * kTile + (wv >> 1) * 8;   // quadrant origin
  const int bx0i = qx0 + (box & 1) * 4, by0i = qy0 + (box >> 1) * 4;             // box origin
  const int i = by0i + (pos >> 2), j = bx0i + (pos & 3);
  const bool inside = i < H && j < W;
  const float px = (float)j + off, py = (float)i + off;
  const int start = tile_offset[ct], list_end = tile_offset[ct + 1];
  if (IS2D && start == list_end && lists2d_missing(tile_offset, sets, c, ct, tw * th)) {
    if (threadIdx.x == 0 && stats->status != nullptr) atomicOr(stats->status, GSR_OVF_LAYOUT);
    nan_tile(c, ty, tx, W, H, out_rgb, out_alpha);
    return;
  }
  const int end = lz.tile_sorted && !lz.rerun ? lz.tile_sorted[ct] : list_end;
  if (threadIdx.x == 0) s_max = -1;
  float T = 1.f, cr = 0.f, cg = 0.f, cb = 0.f;
  float Tl = 1.f;   // 2D: T before the latest composited entry
  int last = -1;
  bool done = !inside;
  const int cbase = chunk_base[ct];
  const int umask = stats->chunk_entries - 1;   // chunk = a power-of-two multiple of 128 entries
  int kcur = 0;
  float Ts = 1.f, dr = 0.f, dg = 0.f, db = 0.f;   // the current chunk's start T and colour
  const int e_last = max(end - 1, start);
  // round prefetch: this thread's entry of the next round (record in registers, id ahead)
  float4 c0 = make_float4(0.f, 0.f, 0.f, 0.f), c1 = c0, c2 = c0;
  int idn = 0;
  if (end > start) {
    const int id0 = ids[min(start + (int)threadIdx.x, e_last)];
    idn = ids[min(start + 256 + (int)threadIdx.x, e_last)];
    c0 = rec[id0].p0;
    c1 = rec[id0].p1;
    c2 = rec[id0].p2;
  }
  if (threadIdx.x < 12) s_r[threadIdx.x / 6][(threadIdx.x / 2) % 3][kHS * (threadIdx.x & 1) + 128] = make_float4(0.f, 0.f, 0.f, 0.f);
  int buf = 0;
  for (int rb = start; rb < end; rb += 256, buf ^= 1) {
    if constexpr (IS2D && !PACK) unpack_rec<true>(c0, c1, c2);   // (2D records are stored packed)
    {
      const int si = (int)(threadIdx.x >> 7) * kHS + (int)(threadIdx.x & 127);
      s_r[buf][0][si] = c0;
      s_r[buf][1][si] = c1;
      s_r[buf][2][si] = c2;
    }
    {
      const int id_use = idn;
      idn = ids[min(rb + 512 + (int)threadIdx.x, e_last)];
      c0 = rec[id_use].p0;
      c1 = rec[id_use].p1;
      c2 = rec[id_use].p2;
    }
    if (!sync_any<4>(!done, s_live[buf])) break;
    // a half's quadrant survivors (slot in the half), kept in this wave's own slots of the other
    // round buffer: dead since the round barrier, and rewritten only by this wave at the next
    // round's start (LDS 27.2 -> 26.6 KB: 6 workgroups per CU)
    // (wave regions of 64 records skip the zero slot at 128)
    unsigned char* const s_list_w = reinterpret_cast<unsigned char*>(&s_r[buf ^ 1][0][64 * wv + (wv >> 1)]);
    for (int h = 0; h < 2; ++h) {
      const int hb = rb + 128 * h;
      if (hb >= end || __ballot(!done) == 0ull) break;
      if (hb > start && ((hb - start) & umask) == 0) {   // entering chunk kcur+1 (every few halves)
        if (IS2D) {   // 2D: the pixel's T anchor at the chunk start (k_raster2d_bwd_tile)
          if (ckpt)
            reinterpret_cast<float*>(ckpt)[(int64_t)(cbase + kcur + 1) * kRasterThreads + ckpt_slot_of(wv, box, pos)] = T;
        } else {
          if (ckpt) ckpt[(int64_t)(cbase + kcur) * kRasterThreads + ckpt_slot_of(wv, box, pos)] = make_float4(Ts, dr, dg, db);
        }
        cr += dr;
        cg += dg;
        cb += db;
        dr = dg = db = 0.f;
        Ts = T;
        ++kcur;
      }
      const int nh = min(128, end - hb);
      // the half against the wave's 8x8 quadrant (two entries per lane), in list order
      int nsurv = 0;
      {
        const float x0 = (float)qx0 + off, y0 = (float)qy0 + off;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int k = q * 64 + lane;
          const int sl = kHS * h + k;
          float4 r0 = s_r[buf][0][sl], r1 = s_r[buf][1][sl], r2 = s_r[buf][2][sl];
          unpack_rec<PACK>(r0, r1, r2);
          const bool keep = k < nh && cull_keep<IS2D>(r0, r1, r2, x0, x0 + 7.f, y0, y0 + 7.f);
          const unsigned long long m = __ballot(keep);
          if (keep)
            s_list_w[nsurv + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                         __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0))] =
                (unsigned char)k;
          nsurv += __popcll(m);
        }
      }
      __builtin_amdgcn_wave_barrier();
      // ... and the quadrant's survivors against each 4x4 box
      int nbx[4];
      box4_cull<IS2D, PACK>(s_list_w, nsurv, &s_r[buf][0][kHS * h], &s_r[buf][1][kHS * h], &s_r[buf][2][kHS * h],
                            (float)qx0 + off, (float)qy0 + off, &s_box[wv][0][0], kBoxStride, nbx);
      const int nb = box == 0 ? nbx[0] : box == 1 ? nbx[1] : box == 2 ? nbx[2] : nbx[3];
      __builtin_amdgcn_wave_barrier();
      // steps walked by the wave: max over its boxes
      const int nmax = max(max(nbx[0], nbx[1]), max(nbx[2], nbx[3]));
      // the sequential walk of the box's survivors (entry index read one step ahead)
      const float4* const rh = &s_r[buf][0][kHS * h];
      if constexpr (IS2D) {
        // 2D walks branch-free (lists are long and rarely saturate; the branchy walk spent as
        // many scalar as vector instructions on exec masks): a box's list is padded to the
        // wave's step count with a real quadrant survivor (finite record), which a step past
        // nb reads and leaves out by select -- the same sums, bit for bit.
        // (reading the survivor slots four per b32 measured slower: 9.55 vs 9.05 ms at config 4)
        unsigned char* const lst = s_box[wv][box];
        for (int s = nb + pos; s < nmax; s += 16) lst[s] = (unsigned char)128;   // the zero record
        __builtin_amdgcn_wave_barrier();
        int k_next = lst[0];
        int lk = -1;
        // (steps in blocks of 32 between the "all pixels done" tests: one loop test per step)
        for (int t0 = 0; t0 < nmax; t0 += 32) {
          if (t0 > 0 && __ballot(!done) == 0ull) break;
          const int t1 = min(t0 + 32, nmax);
#pragma nounroll
        for (int t = t0; t < t1; ++t) {
          const int k = k_next;
          k_next = lst[t + 1];   // past the padded list: read, never used
          __builtin_assume((unsigned)k <= 128u);   // a byte slot (128: the zero record)
          {
            const float4* rk = rh + k;   // the half's records: part j at rk[kRS j]
            float4 p0 = rk[0], p1 = rk[kRS];
            float cb_;
            if constexpr (PACK) {
              cb_ = reinterpret_cast<const float*>(rk + 2 * kRS)[0];   // q2.x: the blue channel (b32)
            } else {
              const float4 p2 = rk[2 * kRS];
              p0.w = p2.x;
              p1.w = p2.y;
              cb_ = p2.z;
            }
            const float dx = p0.x - px, dy = p0.y - py;
            const float sg = conic_sigma(p1, dx, dy);
            const float alpha = p0.z * gauss_exp<true>(sg);
            // (steps past the box's list read the zero record: alpha 0 < cut2d, never valid)
            const bool valid = !done && alpha >= cut2d;
            // an invalid step enters with alpha 0: vis = 0 and T * (1 - 0) = T exactly (one
            // select instead of three); the entry slot of the latest composite is kept per half
            const float av = valid ? alpha : 0.f;
            const float vis = av * T;
            dr += p0.w * vis;
            dg += p1.w * vis;
            db += cb_ * vis;
            Tl = valid ? T : Tl;
            T = T * (1.f - av);
            lk = valid ? k : lk;
            done = done || T <= kT2DMin;   // the reference's A == 1.0f, after this entry
          }
        }
        }
        if (lk >= 0) last = hb + lk;
        __builtin_amdgcn_wave_barrier();
        continue;
      }
      int k_next = s_box[wv][box][0];
      for (int t = 0; t < nmax; ++t) {
        const int k = k_next;
        k_next = s_box[wv][box][t + 1];   // past the list: read, never used
        if (t < nb && !done) {
          __builtin_assume((unsigned)k < 256u);   // a byte: the address is one shift-add
          const float4* rk = rh + k;   // the half's records: part j at rk[kRS j]
          const float4 p0 = rk[0];
          const float4 p1 = rk[kRS];
          const float4 p2 = rk[2 * kRS];
          const float dx = p0.x - px, dy = p0.y - py;
          const float sg = conic_sigma(p1, dx, dy);
          const float raw = p0.z * gauss_exp<IS2D>(sg);
          const float alpha = IS2D ? raw : fminf(kAlphaMax, raw);
          const bool valid = IS2D ? alpha >= cut2d : (sg >= 0.f && alpha >= kAlphaThreshold);
          if (valid) {
            if constexpr (IS2D) {
              const float vis = alpha * T;
              dr += p2.x * vis;
              dg += p2.y * vis;
              db += p2.z * vis;
              Tl = T;
              T *= 1.f - alpha;
              last = hb + k;
              if (T <= kT2DMin) done = true;   // the reference's A == 1.0f, after this entry
            } else {
              const float nT = T * (1.f - alpha);
              if (nT <= kTMin) {
                done = true;   // gsplat: this entry and every later one are not composited
              } else {
                const float vis = alpha * T;
                dr += p2.x * vis;
                dg += p2.y * vis;
                db += p2.z * vis;
                T = nT;
                last = hb + k;
              }
            }
          }
        }
        if ((t & (IS2D ? 31 : 7)) == (IS2D ? 31 : 7) && __ballot(!done) == 0ull) break;
      }
      __builtin_amdgcn_wave_barrier();
    }
  }
  cr += dr;
  cg += dg;
  cb += db;
  if (!IS2D && end > start && ckpt) {   // (2D: the T anchors are final as written)
    // chunk records {T at chunk start, chunk colour} -> what the backward needs at each chunk's
    // END: {T_end, suffix colour sum of the later chunks}, back to front (records re-read 8 at a time)
    float4* ck = ckpt + (int64_t)cbase * kRasterThreads + ckpt_slot_of(wv, box, pos);
    ck[(int64_t)kcur * kRasterThreads] = make_float4(T, 0.f, 0.f, 0.f);
    float sr = dr, sg = dg, sb = db;
    float Tn = Ts;
    for (int k0 = kcur - 1; k0 >= 0; k0 -= 8) {
      float4 r[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (k0 - u >= 0) r[u] = ck[(int64_t)(k0 - u) * kRasterThreads];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (k0 - u >= 0) {
          ck[(int64_t)(k0 - u) * kRasterThreads] = make_float4(Tn, sr, sg, sb);
          Tn = r[u].x;
          sr += r[u].y;
          sg += r[u].z;
          sb += r[u].w;
        }
    }
  }
  if (inside) {
    const int64_t pix = ((int64_t)c * H + i) * W + j;
    const float* bgc = bg + c * 3;
    out_rgb[pix * 3 + 0] = cr + T * bgc[0];
    out_rgb[pix * 3 + 1] = cg + T * bgc[1];
    out_rgb[pix * 3 + 2] = cb + T * bgc[2];
    out_alpha[pix] = 1.f - T;
    if (IS2D)
      reinterpret_cast<float2*>(out_T)[pix] = make_float2(T, Tl);
    else
      out_T[pix] = T;
    out_last[pix] = last;
  }
  if (last >= 0) atomicMax(&s_max, last);
  if (end < list_end) {   // lazy: did the walk reach the end of the sorted prefix?
    if (__syncthreads_or(!done || last == end - 1) && threadIdx.x == 0) lazy_flag_tile(lz, ct);
  } else {
    __syncthreads();
  }
  if (threadIdx.x == 0 && s_max >= 0) tile_end[ct] = s_max;   // one workgroup per tile; finalised by k_raster_finalize
}

// ---------------------------------------------------------------- 2D forward, pixel pairs
// The 2D box forward with TWO pixels per lane: one 2-wave workgroup per tile, wave w the 16x8
// half-tile of rows 8w..8w+7, eight 4x4 boxes per wave.  A lane's pixels are (r, j) and
// (r + 2, j) of its box, so every record read from LDS (2 x b128 + b32) and the step's slot read
// serve two pixels.  Lanes: box = 2 x (the lane's ds_read_b128 group) + (lane bit 4), so a b128
// read of the walk has two addresses per lane group (the box forward's broadcast trick, halved).
// The list is walked in 128-entry rounds (one chunk each; records double-buffered in 12 KB of
// LDS), so 11 workgroups (22 waves) fit a CU.  Per pixel the arithmetic is the box forward's
// (dx = x - px, dy = y - py, conic_sigma, alpha >= cut2d, stop after T <= 2^-25), so
// k_raster2d_bwd_pair's validity tests agree with it exactly -- except that T <- T (1 - a) is one
// fmaf (one rounding, the box forward rounds 1 - a first): the images are not bitwise the box
// layout's (EXPERIMENTS.md §F).
#ifndef GSR_FWD2D_PAIR
#define GSR_FWD2D_PAIR 1
#endif
#ifndef GSR_FWD2P_MINB
#define GSR_FWD2P_MINB 5   // waves per SIMD the compiler aims at
#endif
__global__ __launch_bounds__(128, GSR_FWD2P_MINB) void k_raster2d_fwd_pair(
    const Splat* __restrict__ rec, const int32_t* __restrict__ ids, const int32_t* __restrict__ tile_offset, int W,
    int H, int tw, int th, const float* __restrict__ bg, float* __restrict__ out_rgb, float* __restrict__ out_alpha,
    float* __restrict__ out_T, int32_t* __restrict__ out_last, int32_t* __restrict__ tile_end,
    float* __restrict__ anchors, const int32_t* __restrict__ chunk_base, int64_t CT, float cut2d,
    gsr_bin_stats* __restrict__ stats, const Sets2D sets, int share_lists, int part_colour) {
  constexpr int kHS = kChunk3 + 1;   // part j of round entry k at s_r[buf][j][k]; slot 128 a zero record
  __shared__ float4 s_r[2][3][kHS];
  __shared__ __attribute__((aligned(16))) unsigned char s_box[2][8][kBoxStride];
  __shared__ int s_max;
  __shared__ __attribute__((aligned(8))) int s_live[2][2];
  const int ct = sweep_tile2d(blockIdx.x, CT, tw * th, sets.begin, sets.F);
  const int ovf = stats->overflow;
  if (ovf) {
    if (blockIdx.x == 0 && threadIdx.x == 0 && stats->status != nullptr) atomicOr(stats->status, ovf);
    nan_fill(CT, W, H, tw, th, out_rgb, out_alpha);
    return;
  }
  // the backward's split walks read the colour planes only if this forward wrote them
  if (part_colour && anchors != nullptr && blockIdx.x == 0 && threadIdx.x == 0) atomicOr(&stats->masks, kStatsPlanes2D);
  if (ct < 0) return;
  int c, ty, tx;
  tile_coords(ct, tw, th, c, ty, tx);
  // the set's record copy: entry ids of camera c's own list are c*N + n, of a shared list (the
  // set's first camera's, lists2d_per_set) already cf*N + n
  if (!share_lists) rec += rec_offset2d(sets.begin, sets.F, c, sets.N);
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  const int grp = ((lane >> 4) & 2) | (((lane >> 4) ^ (lane >> 3) ^ (lane >> 2)) & 1);   // b128 lane group
  const int box = 2 * grp + ((lane >> 4) & 1);
  const int pp = (lane & 3) | ((lane >> 1) & 4);   // pixel pair in the box (lane bits 0, 1, 3)
  const int jl = 4 * (box & 3) + (pp & 3), ilA = 8 * wv + 4 * (box >> 2) + (pp >> 2), ilB = ilA + 2;
  const int pj = tx * kTile + jl, piA = ty * kTile + ilA, piB = ty * kTile + ilB;
  const bool inA = piA < H && pj < W, inB = piB < H && pj < W;
  float px = (float)pj, pyA = (float)piA, pyB = (float)piB;   // integer centres
  // (opaque to the compiler: it re-derived pyB from the int with a v_cvt in every walk step)
  asm volatile("" : "+v"(px), "+v"(pyA), "+v"(pyB));
  const int slotA = bwd_pixel_slot(ilA, jl), slotB = bwd_pixel_slot(ilB, jl);
  const int hx0 = tx * kTile, hy0 = ty * kTile + 8 * wv;   // the wave's half-tile origin
  // lists2d_per_set: every camera of the set renders its first camera's list of this tile; only
  // that camera writes the T anchors and tile_end (the others have no chunk rows; theirs would
  // be the same values), and the backward reads that camera's state (k_raster2d_bwd_frame)
  const int T = tw * th;
  const int cfirst = share_lists ? set_first_camera(sets.begin, sets.F, c) : c;
  const int ctl = cfirst * T + (ct - c * T);
  const bool lead = cfirst == c;
  if (!lead) anchors = nullptr;
  const int start = tile_offset[ctl], end = tile_offset[ctl + 1];
  if (!share_lists && start == end && lists2d_missing(tile_offset, sets, c, ct, T)) {
    if (threadIdx.x == 0 && stats->status != nullptr) atomicOr(stats->status, GSR_OVF_LAYOUT);
    nan_tile(c, ty, tx, W, H, out_rgb, out_alpha);
    return;
  }
  if (tid == 0) s_max = -1;
  float TA = 1.f, TlA = 1.f, crA = 0.f, cgA = 0.f, cbA = 0.f, drA = 0.f, dgA = 0.f, dbA = 0.f;
  float TB = 1.f, TlB = 1.f, crB = 0.f, cgB = 0.f, cbB = 0.f, drB = 0.f, dgB = 0.f, dbB = 0.f;
  int lastA = -1, lastB = -1;
  bool doneA = !inA, doneB = !inB;
  const int cbase = chunk_base[ct];
  const int umask = stats->chunk_entries - 1;
  int kcur = 0;
  const int e_last = max(end - 1, start);
  float4 c0 = make_float4(0.f, 0.f, 0.f, 0.f), c1 = c0, c2 = c0;
  int idn = 0;
  if (end > start) {
    const int id0 = ids[min(start + tid, e_last)];
    idn = ids[min(start + kChunk3 + tid, e_last)];
    c0 = rec[id0].p0;
    c1 = rec[id0].p1;
    c2 = rec[id0].p2;
  }
  if (tid < 6) s_r[tid / 3][tid % 3][kChunk3] = make_float4(0.f, 0.f, 0.f, 0.f);
  int buf = 0;
  for (int rb = start; rb < end; rb += kChunk3, buf ^= 1) {
    s_r[buf][0][tid] = c0;
    s_r[buf][1][tid] = c1;
    s_r[buf][2][tid] = c2;
    {
      const int id_use = idn;
      idn = ids[min(rb + 2 * kChunk3 + tid, e_last)];
      c0 = rec[id_use].p0;
      c1 = rec[id_use].p1;
      c2 = rec[id_use].p2;
    }
    if (!sync_any<2>(!(doneA && doneB), s_live[buf])) break;
    if (rb > start && ((rb - start) & umask) == 0) {   // entering unit kcur+1: the pixels' T anchors
      crA += drA;
      cgA += dgA;
      cbA += dbA;
      crB += drB;
      cgB += dgB;
      cbB += dbB;
      drA = dgA = dbA = drB = dgB = dbB = 0.f;
      if (anchors) {
        const int64_t arow = (int64_t)(cbase + kcur + 1) * kRasterThreads;
        anchors[arow + slotA] = TA;
        anchors[arow + slotB] = TB;
        if (part_colour) {   // the colour before the unit (k_raster2d_bwd_frame's parts)
          float* const cp = anchors + arow;
          const int64_t pl = colour_plane2d(stats);
          cp[pl + slotA] = crA;
          cp[2 * pl + slotA] = cgA;
          cp[3 * pl + slotA] = cbA;
          cp[pl + slotB] = crB;
          cp[2 * pl + slotB] = cgB;
          cp[3 * pl + slotB] = cbB;
        }
      }
      ++kcur;
    }
    const int nh = min(kChunk3, end - rb);
    // the round's survivors of the half-tile cull, in this wave's own slots of the idle buffer
    // (dead since the round barrier; rewritten only by this wave's threads at the next round)
    unsigned char* const s_list_w = reinterpret_cast<unsigned char*>(&s_r[buf ^ 1][0][64 * wv]);
    const float4* const r0 = s_r[buf][0];
    const float4* const r1 = s_r[buf][1];
    const float4* const r2 = s_r[buf][2];
    int nsurv = 0;
#pragma unroll
    for (int q = 0; q < kChunk3 / 64; ++q) {
      const int k = q * 64 + lane;
      float4 a = r0[k], b = r1[k], d = r2[k];
      unpack_rec<true>(a, b, d);
      const bool keep = k < nh && cull_keep<true>(a, b, d, (float)hx0, (float)hx0 + 15.f, (float)hy0, (float)hy0 + 7.f);
      const unsigned long long m = __ballot(keep);
      if (keep)
        s_list_w[nsurv + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0))] =
            (unsigned char)k;
      nsurv += __popcll(m);
    }
    __builtin_amdgcn_wave_barrier();
    int nbx[8];
#pragma unroll
    for (int b = 0; b < 8; ++b) nbx[b] = 0;
    {
      const unsigned long long below = (1ull << lane) - 1ull;
      for (int s0 = 0; s0 < nsurv; s0 += 64) {
        const int si = s0 + lane;
        const bool in = si < nsurv;
        const int k = s_list_w[in ? si : 0];
        float4 a = r0[k], b = r1[k], d = r2[k];
        unpack_rec<true>(a, b, d);
#pragma unroll
        for (int bx = 0; bx < 8; ++bx) {
          const float x0 = (float)(hx0 + 4 * (bx & 3)), y0 = (float)(hy0 + 4 * (bx >> 2));
          const bool keep = in && cull_keep<true>(a, b, d, x0, x0 + 3.f, y0, y0 + 3.f);
          const unsigned long long m = __ballot(keep);
          if (keep) s_box[wv][bx][nbx[bx] + __popcll(m & below)] = (unsigned char)k;
          nbx[bx] += __popcll(m);
        }
      }
    }
    int nb = nbx[0], nmax = nbx[0];
#pragma unroll
    for (int b = 1; b < 8; ++b) {
      nb = box == b ? nbx[b] : nb;
      nmax = max(nmax, nbx[b]);
    }
    unsigned char* const lst = s_box[wv][box];
    for (int s = nb + pp; s < nmax; s += 8) lst[s] = (unsigned char)kChunk3;   // the zero record
    __builtin_amdgcn_wave_barrier();
    int k_next = lst[0];
    int lkA = -1, lkB = -1;
    for (int t0 = 0; t0 < nmax; t0 += 32) {
      if (t0 > 0 && __ballot(!(doneA && doneB)) == 0ull) break;
      const int t1 = min(t0 + 32, nmax);
#pragma nounroll
      for (int t = t0; t < t1; ++t) {
        const int k = k_next;
        k_next = lst[t + 1];   // past the padded list: read, never used
        __builtin_assume((unsigned)k <= (unsigned)kChunk3);
        const float4* rk = r0 + k;   // part j at rk[kHS j]
        const float4 p0 = rk[0], p1 = rk[kHS];   // (x, y, o, r), (a, b, c, g)
        const float cbl = reinterpret_cast<const float*>(rk + 2 * kHS)[0];   // blue
        const float dx = p0.x - px;
        {
          const float dy = p0.y - pyA;
          const float alpha = p0.z * gauss_exp<true>(conic_sigma(p1, dx, dy));
          const bool valid = !doneA && alpha >= cut2d;
          const float av = valid ? alpha : 0.f;
          const float vis = av * TA;
          drA += p0.w * vis;
          dgA += p1.w * vis;
          dbA += cbl * vis;
          TlA = valid ? TA : TlA;
          TA = fmaf(-TA, av, TA);   // T (1 - a) in one rounding
          lkA = valid ? k : lkA;
          doneA = doneA || TA <= kT2DMin;
        }
        {
          const float dy = p0.y - pyB;
          const float alpha = p0.z * gauss_exp<true>(conic_sigma(p1, dx, dy));
          const bool valid = !doneB && alpha >= cut2d;
          const float av = valid ? alpha : 0.f;
          const float vis = av * TB;
          drB += p0.w * vis;
          dgB += p1.w * vis;
          dbB += cbl * vis;
          TlB = valid ? TB : TlB;
          TB = fmaf(-TB, av, TB);
          lkB = valid ? k : lkB;
          doneB = doneB || TB <= kT2DMin;
        }
      }
    }
    if (lkA >= 0) lastA = rb + lkA;
    if (lkB >= 0) lastB = rb + lkB;
    __builtin_amdgcn_wave_barrier();
  }
  const float* bgc = bg + c * 3;
  auto store = [&](bool in, int pi, float T, float Tl, float cr, float cg, float cb, int last) {
    if (!in) return;
    const int64_t pix = ((int64_t)c * H + pi) * W + pj;
    out_rgb[pix * 3 + 0] = cr + T * bgc[0];
    out_rgb[pix * 3 + 1] = cg + T * bgc[1];
    out_rgb[pix * 3 + 2] = cb + T * bgc[2];
    out_alpha[pix] = 1.f - T;
    reinterpret_cast<float2*>(out_T)[pix] = make_float2(T, Tl);
    out_last[pix] = last;
  };
  store(inA, piA, TA, TlA, crA + drA, cgA + dgA, cbA + dbA, lastA);
  store(inB, piB, TB, TlB, crB + drB, cgB + dgB, cbB + dbB, lastB);
  if (anchors && part_colour && end > start) {   // row 0 (no anchor there) holds the totals
    float* const cp = anchors + (int64_t)cbase * kRasterThreads;
    const int64_t pl = colour_plane2d(stats);
    cp[pl + slotA] = crA + drA;
    cp[2 * pl + slotA] = cgA + dgA;
    cp[3 * pl + slotA] = cbA + dbA;
    cp[pl + slotB] = crB + drB;
    cp[2 * pl + slotB] = cgB + dgB;
    cp[3 * pl + slotB] = cbB + dbB;
  }
  const int lmax = max(lastA, lastB);
  if (lmax >= 0) atomicMax(&s_max, lmax);
  __syncthreads();
  // one workgroup per tile; finalised by k_raster_finalize
  if (tid == 0 && s_max >= 0 && lead) tile_end[ct] = s_max;
}

// Per busy tile: tile_end = 1 + max last over the tile's four quadrant workgroups (or the
// tile's start), the cut key, and the tile's active chunks appended to the backward's list.
// (A separate launch: finishing it inside the forward by the last-arriving quadrant
// workgroup needs device-scope release fences, which write back the XCD's L2 on gfx950 --
// measured 2x slower forward.)
__global__ __launch_bounds__(kRasterThreads) void k_raster_finalize(
    const float* __restrict__ depth, const int32_t* __restrict__ ids, const int32_t* __restrict__ tile_offset,
    const int32_t* __restrict__ order, int n_busy, const int32_t* __restrict__ chunk_base,
    int32_t* __restrict__ tile_end, uint64_t* __restrict__ tile_cut, gsr_bin_stats* __restrict__ stats,
    int32_t* __restrict__ chunk_list, int key_order, int tile_units, int64_t CT, int T, const Sets2D sets) {
  // the stats words and this thread's tile load together (the tile slot is clamped into the
  // grid's bound; used only when real): one round trip, then the tile's words, then the atomic
  const int ovf = stats->overflow, nb_dev = stats->n_busy;
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  const int ct_busy = tile_units ? 0 : order[min(b, max(n_busy - 1, 0))];
  if (ovf) {   // bounded call over its bounds: report to the caller's sticky status, nothing else
    if (blockIdx.x == 0 && threadIdx.x == 0 && stats->status != nullptr) atomicOr(stats->status, ovf);
    return;
  }
  const int lane = threadIdx.x & 63;
  // tile_units (2D): slot b of the XCD-aware sweep (every tile, busy or empty), one unit each
  const int sct = tile_units && b < sweep_grid2d(CT) ? sweep_tile2d(b, CT, T, sets.begin, sets.F) : -1;
  const bool in = tile_units ? sct >= 0 : b < nb_dev;
  const int ct = tile_units ? max(sct, 0) : in ? ct_busy : 0;
  int start = 0, end = 0, te = 0;
  if (in) {
    start = tile_offset[ct];
    end = tile_offset[ct + 1];
    const int m = tile_end[ct];
    te = m >= 0 ? m + 1 : start;
    tile_end[ct] = te;
  }
  if (tile_units) {
    // the unit of sweep slot b: the tile's whole consumed list [start, te) (empty: a unit of 0
    // entries, which the backward skips); the backward's grid is the sweep's
    if (b == 0) stats->n_active = sweep_grid2d(CT);
    if (b < sweep_grid2d(CT))
      reinterpret_cast<int4*>(chunk_list)[b] = in ? make_int4(start, te - start, chunk_base[ct], ct) : make_int4(0, 0, 0, 0);
    if (in) tile_cut[ct] = te < end ? sort_key(depth, ids[te], key_order) : ~0ull;
    return;
  }
  const int U = stats->chunk_entries;
  const int nact = (te - start + U - 1) / U;
  // one atomic per wave on the active-chunk counter (one per tile serialised ~700 atomics on
  // one address at config 3)
  const int incl = wave_incl_scan_dpp(nact);
  int base = 0;
  if (lane == 63 && incl > 0) base = atomicAdd(&stats->n_active, incl);
  base = __builtin_amdgcn_readlane(base, 63);
  if (in && nact > 0) {
    const int pos = base + incl - nact;
    const int cbase = chunk_base[ct];
    int4* desc = reinterpret_cast<int4*>(chunk_list);
    for (int k = 0; k < nact; ++k) {
      const int b0 = start + k * U;
      desc[pos + k] = make_int4(b0, min(U, te - b0), cbase + k, ct);
    }
  }
  // the cut key (two more dependent loads) after the chunk list: off its chain
  if (in) tile_cut[ct] = te < end ? sort_key(depth, ids[te], key_order) : ~0ull;
}

// Partial rows are stored in EMISSION order (row k_of_s[s] for sorted entry s), 9 floats
// (36 B, no padding) per row, so *_project_bwd reads each Gaussian's rows contiguously.
static_assert(kPartialStride == kPartial, "a partial row is its 9 partials");
__device__ __forceinline__ void store_partial_row(float* __restrict__ partial, int k, const float (&v)[kPartial]) {
  float* dst = partial + (int64_t)k * kPartialStride;
#pragma unroll
  for (int q = 0; q < kPartial; ++q) dst[q] = v[q];
}

// The per-entry sum update of the backward kernels: lane f adds the staged value v[b] of box b
// to its wave's slot Lw[k[b]], for NB boxes, box by box.  A box lists an entry once, but two
// boxes may list the same entry at DIFFERENT group positions, i.e. from different lanes (lane
// (g, q) of box 0 and lane (g', q) of box 1), so the boxes' read-add-writes must stay in box
// order: each box's reads see the previous box's writes.  (Issuing all NB reads first and
// chaining only a lane's own aliased boxes lost those cross-lane updates: measured wrong in the
// fit test, round 5.)
// GSR_BWD_LWPAR=1 rebuilds exactly that broken form (commit 3ec9d20) as the NEGATIVE CONTROL of
// tests/test_race_gpu.py (tools/race_control.sh builds it into build_var/; never the product).
#ifndef GSR_BWD_LWPAR
#define GSR_BWD_LWPAR 0
#endif
template <int NB>
__device__ __forceinline__ void lw_add(float* Lw, const int (&k)[NB], const float (&v)[NB]) {
#if GSR_BWD_LWPAR
  float n[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) n[b] = Lw[k[b]];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    n[b] += v[b];
#pragma unroll
    for (int c = 0; c < b; ++c) n[b] = k[c] == k[b] ? n[c] + v[b] : n[b];
  }
#pragma unroll
  for (int b = 0; b < NB; ++b) Lw[k[b]] = n[b];
#else
#pragma unroll
  for (int b = 0; b < NB; ++b) Lw[k[b]] += v[b];
#endif
}
// GSR_BWD_PF: the walk reads entry g+1's record from LDS before it evaluates entry g (a
// scheduling fence keeps the reads there: left to itself the compiler issued each entry's reads
// at its use, two exposed LDS round trips per entry, 14 per group)
#ifndef GSR_BWD_PF
#define GSR_BWD_PF 1
#endif
__device__ __forceinline__ void walk_fence() {
#if GSR_BWD_PF
  __builtin_amdgcn_sched_barrier(0);
#endif
}

// Cotangent of  g_iou * iou_loss + g_img * img_loss  (+ extra cotangents) at one pixel
// (scripts/training/train_script.py:30-36, 128-130), from the sums of gsr_loss_iou_l1_fwd:
//   d iou_loss / d a = -(1/C) [ m / (U+e) - (I+e) / (U+e)^2 (1 - m) ]       (e = 1e-6)
//   d img_loss / d rgb_k = img_lambda / M * sign(rgb_k - t_k)                 (sign(0) = 0)
// the same association torch's autograd uses for the unfused expressions.
__device__ __forceinline__ void loss_cotangent(const gsr_loss_terms& lt, int C, int c, int64_t pix, int64_t pv,
                                               int64_t HW, float& vr, float& vg, float& vb, float& va) {
  const float g_iou = lt.grad_out[0], g_img = lt.grad_out[1];
  const float Ie = lt.sums[4 * c + 0] + 1e-6f, Ue = lt.sums[4 * c + 1] + 1e-6f;
  const float M = lt.sums[4 * C + 2];
  const float m = lt.target_mask[pix];
  const float d_iou_dI = 1.f / Ue;
  const float d_iou_dU = -Ie / (Ue * Ue);
  const float g = -g_iou / (float)C;
  va = g * (d_iou_dI * m + d_iou_dU * (1.f - m));
  const float s = g_img * lt.img_lambda / M;
  const float* t = lt.target_img + (int64_t)c * 3 * HW + pv;
  const float* r = lt.rgb + pix * 3;
  const float d0 = r[0] - t[0], d1 = r[1] - t[HW], d2 = r[2] - t[2 * HW];
  vr = s * (float)((d0 > 0.f) - (d0 < 0.f));
  vg = s * (float)((d1 > 0.f) - (d1 < 0.f));
  vb = s * (float)((d2 > 0.f) - (d2 < 0.f));
  if (lt.v_rgb_extra) {
    vr += lt.v_rgb_extra[pix * 3 + 0];
    vg += lt.v_rgb_extra[pix * 3 + 1];
    vb += lt.v_rgb_extra[pix * 3 + 2];
  }
  if (lt.v_alpha_extra) va += lt.v_alpha_extra[pix];
}

// ---------------------------------------------------------------- 3D backward
// Chunk-parallel: one workgroup per (tile, GSR_CHUNK-entry chunk of its list), so no
// pixel's back-to-front walk is longer than one chunk.  Workgroup b takes entry b of the
// forward's chunk list (only chunks before their tile's tile_end).  The forward's chunk
// records give each pixel's state at the chunk's END exactly: T_end (the T the forward had
// there) and the suffix colour sum S_end = sum of the later chunks' own colour sums
// (positive terms, no cancellation).  Inside the chunk:
//   T_i recovered as T_{i+1}/(1-a_i) with v_rcp (a <= 0.999);
//   d rgb/d c_i = a_i T_i;  d rgb/d a_i = c_i T_i - (S_i + T_f bg)/(1-a_i);  d alpha/d a_i = T_f/(1-a_i)
//   a = o e^{-sigma} (unclamped only):  d/do = e^{-sigma},  d/dsigma = -a.
//
// Layout: wave w owns the 8x8 quadrant w of the tile; its lane l serves pixel l>>2 of the
// 4x4 BOX l&3 of that quadrant.  The chunk is culled against the quadrant (exact test, as in
// the forward), the quadrant's survivors against each of its four boxes, and every lane
// walks its own box's survivor list back to front in straight-line groups of 7 (the wave
// runs max over its boxes of the group count).  4x4 boxes evaluate ~0.45x the (pixel, entry)
// pairs of 8x8 ones (tools/cull_stats.py: the wave walks 0.64x the groups at config 3).  Each
// group's 7 entries x 9 gradient sums are reduced over the 16 lanes of each box by a
// transposed butterfly over lane bits 5,4,3,2 (reduce_box16: two permlane-swap levels, two
// DPP levels), after which every lane holds 4 of its box's 63 sums.  They are staged in LDS
// and added box by box into the wave's own slot of the per-entry sums with plain
// read-add-writes (distinct addresses inside an instruction, boxes in program order): no LDS
// atomics (one float atomic per lane per group was ~40% of the LDS time), and the fixed-order
// 4-slot sum at the end keeps the result bitwise deterministic.
//
// LOSS: the pixel cotangents are not read from v_rgb / v_alpha images but generated from the
// training loss (loss_cotangent below, gsr3d_raster_bwd_loss).
//
// IS2D: the same walk in "mu" form, mu_{i+1} = (value of everything after entry i) / T_{i+1}:
//   d/d a_i = T_i (c_i.v - mu_{i+1}),   mu_i = a_i c_i.v + (1 - a_i) mu_{i+1},
//   mu after a pixel's last entry = v.bg - v_alpha;  at a chunk end e before it,
//   mu_e = (S_e.v + T_f mu_last) / T_e  (T_e > 2^-25: the pixel had not saturated there).
// T_i = T_{i+1} / (1 - a_i) as in 3D, except at the pixel's last entry, whose T comes from
// the forward (final_T .y) -- the one entry whose 1 - a may be exactly 0.  No clamp: every
// valid pair feeds the sigma / opacity gradients.
// minimum workgroups per CU of the MULTI variant (build knob for measurements; the one-sub-chunk
// variant fits 5 per CU in 84 VGPRs on its own)
#ifndef GSR_BWD_MINB
#define GSR_BWD_MINB 1
#endif
#ifndef GSR_BWD_LDS
#define GSR_BWD_LDS 0   // 1: packed LDS records + grouped survivor slots (PK below); measured slower in 3D (config 5 raster bwd 0.60 -> 0.67 ms)
#endif
#ifndef GSR_BWD_MULTI_MINB
#define GSR_BWD_MULTI_MINB 1
#endif
#ifndef GSR_BWD_PRIO
#define GSR_BWD_PRIO 0   // 1: s_setprio by the wave's walk length (timing experiment)
#endif
#ifdef GSR_BWD_TRACE
// timing build only (tools/bwd_trace.py): per workgroup {wall clock at 7 points, hw id, groups}
__device__ unsigned long long* g_bwd_trace = nullptr;
#define BWD_T(i) if (threadIdx.x == 0) tr[i] = wall_clock64()   // (LDS: registers would cost occupancy)
#else
#define BWD_T(i)
#endif
template <bool LOSS, bool IS2D, bool MULTI>
__global__ __launch_bounds__(kRasterThreads, MULTI ? GSR_BWD_MULTI_MINB : GSR_BWD_MINB) void k_raster_bwd(
    const Splat* __restrict__ rec, const int32_t* __restrict__ ids, const int32_t* __restrict__ tile_offset,
    const int32_t* __restrict__ tile_end, const int32_t* __restrict__ chunk_base,
    const float4* __restrict__ ckpt, int W, int H, int tw, int th,
    const float* __restrict__ bg, const float* __restrict__ final_T, const int32_t* __restrict__ last_in,
    const float* __restrict__ v_rgb, const float* __restrict__ v_alpha, float* __restrict__ partial,
    const int32_t* __restrict__ chunk_list, gsr_bin_stats* __restrict__ stats,
    const int32_t* __restrict__ k_of_s, const gsr_loss_terms lt, int C, float cut2d,
    const uint4* __restrict__ boxm = nullptr) {
  static_assert(!(LOSS && IS2D), "the fused loss is the 3D training loss");
  // slot kNull: a zero-opacity record (never valid) that pads survivor groups to 7
  constexpr int kNull = kChunk3;
#ifndef GSR_BWD_GROUP
#define GSR_BWD_GROUP 7
#endif
  constexpr int kGroup = GSR_BWD_GROUP;
  constexpr int kLen = kChunk3 + kGroup;   // survivor list capacity (padded to whole groups)
  // PK: records staged packed (pack_rec: the walk's nine values in 2 x b128 + b32) and each box's
  // survivor list with a pad byte after every 7 (grouped_slot): a group's seven slots are ONE
  // 8-byte read instead of seven byte reads
  constexpr bool PK = GSR_BWD_LDS;
  constexpr int kLenB = PK ? 8 * ((kLen + kGroup - 1) / kGroup) : kLen;
  __shared__ float4 s_p[3][kChunk3 + 1];   // the chunk's records, part j of entry k at s_p[j][k]
  // gradient sums per entry, one slot per wave (index kNull absorbs the padding's zeros):
  // sum q of entry k in wave w's slot at L[q * kLq + w * (kChunk3 + 1) + k].  The odd q stride
  // (517 = 5 mod 32 banks) keeps the nine q of one entry on nine banks in the read-add-writes
  // below (516 put q = 0 and q = 8 on one bank: a 2-way conflict in every instruction)
  constexpr int kLq = 4 * (kChunk3 + 1) + 1;
  constexpr int kLn = kPartial * kLq;
  __shared__ __attribute__((aligned(16))) float L[(kLn + 3) & ~3];
  __shared__ unsigned char s_list[4][kLen];     // quadrant survivors, back to front
  __shared__ __attribute__((aligned(16))) unsigned char s_box[4][4][kLenB];   // per (wave, box) survivors, back to front
  // per wave: the group's reduced sums, box-major rows of 64 (reduce_grp16's swizzled staging)
  __shared__ __attribute__((aligned(16))) float s_stage[4][4][64];
  __shared__ unsigned char s_mask[kChunk3];   // 3D: each entry's quadrant mask (k_of_s bits 28..31)
  // one workgroup per grid slot; slots past the forward's active-chunk count exit at once
  // the chunk's descriptor {first entry, entries (>= 1), chunk record row, tile} -- one load
  // (read before the bound check: the list has a slot for every grid slot)
  // The descriptor and the three stats words load together and ONE branch tests them (separate
  // tests made the compiler wait for each load in turn: three extra round trips per workgroup).
  // MULTI = false: units of exactly one sub-chunk (no loop: the loop's back-edge keeps ~40 more
  // VGPRs live and costs a wave per SIMD); a forward with longer units is flagged, not half done.
#ifdef GSR_BWD_TRACE
  __shared__ unsigned long long tr[8];
  __shared__ int tr_nb[16];
  BWD_T(0);
#endif
  const int4 cd = reinterpret_cast<const int4*>(chunk_list)[blockIdx.x];
  const int n_act = stats->n_active, ovf = stats->overflow, ce = stats->chunk_entries;
  const int smasks = stats->masks;
  const bool use_masks = !IS2D && (smasks & kStatsMasks3D) != 0;
  const bool unit_bad = !MULTI && ce != kChunk3;
  if ((ovf != 0) | ((int)blockIdx.x >= n_act) | unit_bad | (cd.y <= 0)) {
    if (unit_bad && blockIdx.x == 0 && threadIdx.x == 0) {
      atomicOr(&stats->overflow, GSR_OVF_UNIT);
      // the forward's finalize has already reported to the sticky word: report this one too
      if (stats->status != nullptr) atomicOr(stats->status, GSR_OVF_UNIT);
    }
    return;
  }
  BWD_T(1);
  const int b0 = cd.x, n = cd.y, chunk = cd.z, ct = cd.w;
  int c, ty, tx;
  tile_coords(ct, tw, th, c, ty, tx);
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  // box = the lane's ds_read_b128 group (reduce_grp16): a walk read is one address per group
  const int box = b128_group(lane), pos = grp16_pos(lane);
  const float off = IS2D ? 0.f : 0.5f;   // 2D: integer centres (src/gaussian_renderer.py:355-358)
  const int qx0 = tx * kTile + (wv & 1) * 8, qy0 = ty * kTile + (wv >> 1) * 8;   // quadrant origin
  const int bx0i = qx0 + (box & 1) * 4, by0i = qy0 + (box >> 1) * 4;             // box origin
  const int pi = by0i + (pos >> 2), pj = bx0i + (pos & 3);
  const bool inside = pi < H && pj < W;
  const float px = (float)pj + off, py = (float)pi + off;
  // A work unit ("chunk", stats->chunk_entries list entries) is walked back to front in
  // sub-chunks of kChunk3 entries staged in LDS; the pixel's state (T, and the suffix term: Sv
  // in 3D, mu in 2D) carries from one sub-chunk into the previous one, so the pixel state and
  // the chunk record are read once per unit.
  const int nsub = MULTI ? (n + kChunk3 - 1) / kChunk3 : 1;
  int sb0 = b0 + (nsub - 1) * kChunk3;   // the current sub-chunk [sb0, sb0 + sn)
  int sn = b0 + n - sb0;
  // Every load is issued up front, none waiting for `last` (the per-WG latency chain is what
  // bounds this kernel's fixed part): the pixel's state, its chunk record, the last sub-chunk's
  // ids and sort positions; pixels that stopped before this unit then drop them by select.
  const float4 rck = ckpt[(int64_t)chunk * kRasterThreads + ckpt_slot_of(wv, box, pos)];
  // the forward's survivor masks of this chunk's 4x4 boxes (the same two culls, done there):
  // wave-uniform, scalar loads
  const bool use_bm = !IS2D && !MULTI && boxm != nullptr && (smasks & kStatsBoxMasks) != 0;
  uint4 bm[4] = {};
  if (use_bm) {
    const uint4* bmp = boxm + (int64_t)chunk * 16 + 4 * __builtin_amdgcn_readfirstlane(wv);
#pragma unroll
    for (int b = 0; b < 4; ++b) bm[b] = bmp[b];
  }
  int id_mine = threadIdx.x < sn ? ids[sb0 + threadIdx.x] : 0;
  int kos_mine = threadIdx.x < sn ? k_of_s[sb0 + threadIdx.x] : 0;
  // the records as three float4 registers (a Splat variable assigned under a branch and in the
  // sub-chunk loop went through 48 B of scratch per lane: a store + reload on the load chain),
  // gathered right behind the ids: issued after the pixel-state loads, they waited for `last`
  // as well (one more memory latency on every workgroup's load chain)
  const float4* const rec4 = reinterpret_cast<const float4*>(rec);
  float4 sp0 = make_float4(0.f, 0.f, 0.f, 0.f), sp1 = sp0, sp2 = sp0;
  if (threadIdx.x < sn) {
    sp0 = rec4[3 * (int64_t)id_mine + 0];
    sp1 = rec4[3 * (int64_t)id_mine + 1];
    sp2 = rec4[3 * (int64_t)id_mine + 2];
  }
  float Tf = 1.f, Tl = 1.f, vr = 0.f, vg = 0.f, vb = 0.f, va = 0.f;
  int last = -1;
  if (inside) {
    const int64_t pix = ((int64_t)c * H + pi) * W + pj;
    last = last_in[pix];
    if constexpr (IS2D) {
      const float2 t2 = reinterpret_cast<const float2*>(final_T)[pix];
      Tf = t2.x;
      Tl = t2.y;
    } else {
      Tf = final_T[pix];
    }
    if constexpr (LOSS) {
      loss_cotangent(lt, C, c, pix, (int64_t)pi * W + pj, (int64_t)W * H, vr, vg, vb, va);
    } else {
      vr = v_rgb[pix * 3 + 0];
      vg = v_rgb[pix * 3 + 1];
      vb = v_rgb[pix * 3 + 2];
      va = v_alpha[pix];
    }
  }
  const bool live = last >= b0;
  if (!live) {
    Tf = Tl = 1.f;
    vr = vg = vb = va = 0.f;
  }
  // state at the end of this unit: {T_end, suffix colour sum} (forward epilogue)
  const float T0 = live ? rck.x : Tf, Sr = live ? rck.y : 0.f, Sg = live ? rck.z : 0.f, Sb = live ? rck.w : 0.f;
  float T = T0;
  const float* bgc = bg + c * 3;
  const float bgdot = bgc[0] * vr + bgc[1] * vg + bgc[2] * vb;
  const float vTa = Tf * (va - bgdot);
  // the suffix colour enters only through its dot product with the pixel's colour cotangent
  float Sv = Sr * vr + Sg * vg + Sb * vb;
  float mu = 0.f;   // 2D
  if constexpr (IS2D) {
    const float mu_last = bgdot - va;
    mu = last < b0 + n ? mu_last : (Sv + Tf * mu_last) / T;
  }
  const int wlast = wave_max_i(last);   // wave-uniform (an SGPR across the sub-chunk loop)
  const int fg = lane / kPartial, fq = lane - kPartial * (lane / kPartial);
  const bool fown = lane < kGroup * kPartial;
  float* const Lw = &L[fq * kLq + wv * (kChunk3 + 1)];
  // lane f reads flat sum f of box bx at s_stage[wv][bx][f ^ grp16_swz(bx)]; lane l stages its
  // four sums (box grp16_out_box(l), flat 4 grp16_slot(l) + i) as one b128 store
  const float* const stage_rd0 = &s_stage[wv][0][lane];
  const float* const stage_rd1 = &s_stage[wv][0][lane ^ 16];
  float4* const stage_wr = reinterpret_cast<float4*>(
      &s_stage[wv][grp16_out_box(lane)][(4 * grp16_slot(lane)) ^ grp16_swz(grp16_out_box(lane))]);
  const unsigned char* my_list = s_box[wv][box];
  for (int sub = nsub - 1; sub >= 0; --sub) {
    if (sub != nsub - 1) __syncthreads();   // the previous sub-chunk's LDS is consumed
    if (PK) pack_rec(sp0, sp1, sp2);
    if (threadIdx.x < sn) {
      s_p[0][threadIdx.x] = sp0;
      s_p[1][threadIdx.x] = sp1;
      s_p[2][threadIdx.x] = sp2;
      s_mask[threadIdx.x] = (unsigned char)((unsigned)kos_mine >> kMaskShift);
    }
    for (int i = threadIdx.x; i < ((kLn + 3) >> 2); i += kRasterThreads)   // b128 stores
      reinterpret_cast<float4*>(L)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (threadIdx.x == 0) {
      const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
      s_p[0][kNull] = z;
      s_p[1][kNull] = z;
      s_p[2][kNull] = z;
    }
    __syncthreads();
    BWD_T(2);
    // the pixel's last entry as a slot of this sub-chunk: lastk for the range test (the pad
    // slot kNull is past it), lastq for the 2D equality (never a slot when the last entry is
    // in a later sub-chunk or before this one)
    const int lastk = min(last - sb0, kChunk3 - 1);   // < 0: the pixel stopped before this sub-chunk
    const int lastq = last - sb0 < kChunk3 ? last - sb0 : -1;
    int nbx[4];
    if (use_bm) {
      // each box's list from its mask, back to front, cut at the box's last composited entry
      // (the forward writes a box's masks only while one of its pixels is live): the max of
      // `last` over the box's 16 lanes -- quad xor 1, 2, row_mirror (xor 15), swizzle xor 24
      int bl16 = last;
      bl16 = max(bl16, dpp_row_i<0xB1>(bl16));   // quad_perm [1,0,3,2]
      bl16 = max(bl16, dpp_row_i<0x4E>(bl16));   // quad_perm [2,3,0,1]
      bl16 = max(bl16, dpp_row_i<0x140>(bl16));  // row_mirror
      bl16 = max(bl16, __builtin_amdgcn_ds_swizzle(bl16, (0x18 << 10) | 0x1F));   // lane ^ 24 in 32
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        // box b's lanes: bit 5 = b >> 1, parity of bits 2..4 = b & 1 (b128_group); lane 32 (b >> 1) + 4 (b & 1)
        const int lim = min(sn - 1, __builtin_amdgcn_readlane(bl16, 32 * (b >> 1) + 4 * (b & 1)) - sb0);
        const unsigned long long mlo = lim < 0 ? 0ull : lim >= 63 ? ~0ull : (2ull << lim) - 1ull;
        const unsigned long long mhi = lim < 64 ? 0ull : lim >= 127 ? ~0ull : (2ull << (lim - 64)) - 1ull;
        const unsigned long long lo = (((unsigned long long)bm[b].y << 32) | bm[b].x) & mlo;
        const unsigned long long hi = (((unsigned long long)bm[b].w << 32) | bm[b].z) & mhi;
        const int nhi = __popcll(hi);
        nbx[b] = nhi + __popcll(lo);
        unsigned char* const bl = s_box[wv][b];
        if ((hi >> lane) & 1ull) {
          const int p = __popcll((hi >> lane) >> 1);
          bl[PK ? grouped_slot(p) : p] = (unsigned char)(64 + lane);
        }
        if ((lo >> lane) & 1ull) {
          const int p = nhi + __popcll((lo >> lane) >> 1);
          bl[PK ? grouped_slot(p) : p] = (unsigned char)lane;
        }
      }
    } else {
    // cull the sub-chunk against this wave's 8x8 quadrant; survivors are listed back to front
    int nsurv = 0;
    {
      const float x0 = (float)qx0 + off, y0 = (float)qy0 + off;
#pragma unroll
      for (int q = kChunk3 / 64 - 1; q >= 0; --q) {
        const int k = q * 64 + lane;
        // the quadrant test: the emission's mask bit where it stored masks (the same cull_keep on
        // the same bounds, no record reads), else the test itself
        bool in_q;
        if (use_masks) {
          in_q = ((s_mask[k] >> wv) & 1) != 0;
        } else {
          float4 r0 = s_p[0][k], r1 = s_p[1][k], r2 = s_p[2][k];
          unpack_rec<PK>(r0, r1, r2);
          in_q = cull_keep<IS2D>(r0, r1, r2, x0, x0 + 7.f, y0, y0 + 7.f);
        }
        const bool keep = k < sn && (sb0 + k) <= wlast && in_q;
        const unsigned long long mk = __ballot(keep);
        if (keep) {
          const unsigned long long above = lane == 63 ? 0ull : (mk >> (lane + 1));
          s_list[wv][nsurv + __popcll(above)] = (unsigned char)k;
        }
        nsurv += __popcll(mk);
      }
    }
    __builtin_amdgcn_wave_barrier();
    // ... and the quadrant's survivors against each 4x4 box (one survivor per lane, all four
    // boxes; box4_cull keeps the list order)
    box4_cull<IS2D, PK, PK>(s_list[wv], nsurv, s_p[0], s_p[1], s_p[2], (float)qx0 + off, (float)qy0 + off,
                            &s_box[wv][0][0], kLenB, nbx);
    }
    const int nb = box == 0 ? nbx[0] : box == 1 ? nbx[1] : box == 2 ? nbx[2] : nbx[3];   // this lane's box
    // groups walked by the wave: max over its boxes
    const int ngrp = max(max(nbx[0], nbx[1]), max(nbx[2], nbx[3]));
    const int npad = (ngrp + kGroup - 1) / kGroup * kGroup;
    for (int s = nb + pos; s < npad; s += 16) s_box[wv][box][PK ? grouped_slot(s) : s] = (unsigned char)kNull;
    __builtin_amdgcn_wave_barrier();
#if GSR_BWD_PRIO
    // the chunk's long walks (its slowest waves, which the others wait for at the rows barrier)
    // win the CU's issue arbitration
    if (ngrp > 3 * kGroup) __builtin_amdgcn_s_setprio(2);
    else if (ngrp > 2 * kGroup) __builtin_amdgcn_s_setprio(1);
#endif
#ifdef GSR_BWD_TRACE
    if (pos == 0) tr_nb[wv * 4 + box] = nb;
#endif
    BWD_T(3);
    // after reduce_grp16 lane l holds 4 sums of box grp16_out_box(l), flat indices
    // 4 grp16_slot(l) + i = 9*g + q.  They are staged in LDS (one b128 store per group, box-major
    // and swizzled: conflict-free stores and reads), and lane f < 63 then adds flat index
    // f = 9g + q of every box, box by box, into the wave's slot L[q][wv][entry]: inside one
    // instruction the 63 (q, entry) addresses are distinct (a box lists an entry once), and
    // the boxes follow in program order, so the plain read-add-write is race-free and
    // deterministic -- no LDS atomics.
    // Branch-free groups of 7 survivors: an invalid (entry, pixel) pair contributes zeros and
    // leaves T and S unchanged (ra = 1, fac = 0), so every group is straight-line code.
    for (int g0 = 0, gb = 0; g0 < ngrp; g0 += kGroup, gb += 8) {
      float acc[64];
      acc[63] = 0.f;
      const uint2 w8 = PK ? *reinterpret_cast<const uint2*>(my_list + gb) : make_uint2(0u, 0u);
      int kk[kGroup];
#pragma unroll
      for (int g = 0; g < kGroup; ++g)
        kk[g] = PK ? (int)(((g < 4 ? w8.x : w8.y) >> (8 * (g & 3))) & 0xFFu) : my_list[g0 + g];
      // entry g+1's record is read before entry g is evaluated (GSR_BWD_PF)
      float4 n0 = s_p[0][kk[0]], n1 = s_p[1][kk[0]], n2 = s_p[2][kk[0]];
#pragma unroll
      for (int g = 0; g < kGroup; ++g) {
        const int k = kk[g];
        const float4 p0 = n0;
        const float4 p1 = n1;
        float4 p2;
        if (PK) {
          p2 = make_float4(p0.w, p1.w, n2.x, 0.f);   // the colour (packed: b32 in part 2)
        } else {
          p2 = n2;
        }
        if (g + 1 < kGroup) {
          n0 = s_p[0][kk[g + 1]];
          n1 = s_p[1][kk[g + 1]];
          n2 = s_p[2][kk[g + 1]];
        }
        walk_fence();
        const float dx = p0.x - px, dy = p0.y - py;
        const float sigma = conic_sigma(p1, dx, dy);
        const float vis = gauss_exp<IS2D>(sigma);
        const float raw = p0.z * vis;
        const float alpha = IS2D ? raw : fminf(kAlphaMax, raw);
        // an invalid pair enters with alpha 0: ra = rcp(1) = 1, fac = 0 and (2D) v_sig = -0,
        // mu unchanged, exactly, without a select each.  2D: the pixel's last entry (valid by
        // construction) takes its T from the forward -- its 1 - alpha may be exactly 0.
        const bool valid = IS2D ? k <= lastk && alpha >= cut2d : k <= lastk && sigma >= 0.f && alpha >= kAlphaThreshold;
        const float alpha_v = valid ? alpha : 0.f;
        const float ra = __builtin_amdgcn_rcpf(1.f - alpha_v);
        if (IS2D)
          T = k == lastq ? Tl : T * ra;
        else
          T *= ra;
        const float fac = alpha_v * T;
        acc[g * kPartial + 6] = fac * vr;
        acc[g * kPartial + 7] = fac * vg;
        acc[g * kPartial + 8] = fac * vb;
        const float cv = p2.x * vr + p2.y * vg + p2.z * vb;
        float v_sig;
        if constexpr (IS2D) {
          const float dmu = cv - mu;
          v_sig = -alpha_v * (T * dmu);
          mu = mu + alpha_v * dmu;
        } else {
          const float v_al = T * cv + ra * (vTa - Sv);
          const bool unclamped = valid && raw <= kAlphaMax;
          v_sig = unclamped ? -raw * v_al : 0.f;
        }
        // moments of v_sig: (dx, dy) here; the mean gradient (2a dx + b dy, b dx + 2c dy) is
        // formed from their sums per entry after the reduction
        const float tx_ = v_sig * dx, ty_ = v_sig * dy;
        acc[g * kPartial + 0] = tx_;
        acc[g * kPartial + 1] = ty_;
        acc[g * kPartial + 2] = tx_ * dx;
        acc[g * kPartial + 3] = tx_ * dy;
        acc[g * kPartial + 4] = ty_ * dy;
        acc[g * kPartial + 5] = v_sig;   // v_opacity = vis v_al = -v_sig / o (formed per entry below)
        if (!IS2D) Sv += fac * cv;
      }
      float sum[4];
      reduce_grp16(acc, sum);
      *stage_wr = make_float4(sum[0], sum[1], sum[2], sum[3]);
      __builtin_amdgcn_wave_barrier();
      if (fown) {
        int kb[4];
        float vb4[4];
#pragma unroll
        for (int bx = 0; bx < 4; ++bx) {
          kb[bx] = s_box[wv][bx][PK ? gb + fg : g0 + fg];
          vb4[bx] = (grp16_swz(bx) ? stage_rd1 : stage_rd0)[64 * bx];
        }
        lw_add(Lw, kb, vb4);
      }
      __builtin_amdgcn_wave_barrier();
    }
    // the next (earlier) sub-chunk's ids, sort positions and records, gathered while this
    // one's rows are summed and stored (not during the walk: registers)
    // (assigned on every path: a conditional assignment keeps the old values live across the walk)
    int kos_next = 0;
    if (MULTI) sp0 = sp1 = sp2 = make_float4(0.f, 0.f, 0.f, 0.f);
    if (sub > 0 && threadIdx.x < kChunk3) {
      const int id_next = ids[sb0 - kChunk3 + threadIdx.x];
      kos_next = k_of_s[sb0 - kChunk3 + threadIdx.x];
      sp0 = rec4[3 * (int64_t)id_next + 0];
      sp1 = rec4[3 * (int64_t)id_next + 1];
      sp2 = rec4[3 * (int64_t)id_next + 2];
    }
    BWD_T(4);
    __syncthreads();
    BWD_T(5);
    if (threadIdx.x < sn) {
      const int k = threadIdx.x;
      float v[kPartial];
#pragma unroll
      for (int q = 0; q < kPartial; ++q) {
        const float* Lq = &L[q * kLq + k];
        v[q] = (Lq[0] + Lq[kChunk3 + 1]) + (Lq[2 * (kChunk3 + 1)] + Lq[3 * (kChunk3 + 1)]);
      }
      const float4 p1 = s_p[1][k];
      const float mx = v[0], my = v[1];
      // (records hold the conic times log2(e): the mean's chain takes the unscaled one)
      v[0] = (2.f * p1.x * mx + p1.y * my) * conic_unscale<IS2D>();
      v[1] = (p1.y * mx + 2.f * p1.z * my) * conic_unscale<IS2D>();
      v[5] = -v[5] / s_p[0][k].z;
      // (bits 28..31 hold the 3D quadrant mask only where the emission stored masks: a call
      // without them may have 2^28 entries or more, whose indices must not be cut)
      store_partial_row(partial, use_masks ? kos_mine & kEmitIndexMask : kos_mine, v);
    }
    sb0 -= kChunk3;
    sn = kChunk3;
    kos_mine = kos_next;
#ifdef GSR_BWD_TRACE
    if (threadIdx.x == 0) tr[7] = ((unsigned long long)__smid() << 32) | (unsigned)ngrp;
#endif
  }
#ifdef GSR_BWD_TRACE
  __syncthreads();
  BWD_T(6);
  if (threadIdx.x == 0 && g_bwd_trace != nullptr) {
    ulonglong2* dst = reinterpret_cast<ulonglong2*>(g_bwd_trace + (int64_t)blockIdx.x * 16);
    for (int i = 0; i < 4; ++i) dst[i] = make_ulonglong2(tr[2 * i], tr[2 * i + 1]);
    int4* dn = reinterpret_cast<int4*>(dst + 4);
    for (int i = 0; i < 4; ++i) dn[i] = make_int4(tr_nb[4 * i], tr_nb[4 * i + 1], tr_nb[4 * i + 2], tr_nb[4 * i + 3]);
  }
#endif
}
// ---------------------------------------------------------------- 2D backward, per tile
// The 2D (index-order) lists never terminate early (I_eff = I), so every tile is long and busy:
// config 4 has 55 296 tiles of ~2 090 entries, far more tiles than the chip's workgroup slots,
// and the chunk-parallel backward's price -- per 128-entry chunk a 16-B {T_end, suffix colour}
// record per pixel (written, read back and rewritten by the forward's epilogue, read by the
// backward) and the pixel's 28-B state re-read -- bought no parallelism the tiles did not
// already give.  Here ONE workgroup walks a tile's whole consumed list [start, tile_end) back to
// front in 128-entry sub-chunks (same layout, culls, transposed box reduction and staged LDS sums
// as k_raster_bwd).  The pixel state is read once per tile; mu (mu form: the value of everything
// after the entry over T) carries from one sub-chunk into the previous one -- no suffix colour
// sums; T is re-anchored at every unit boundary (stats->chunk_entries entries) from the
// forward's T record (4 B per pixel per unit, written once), and inside a unit recovered as
// T_{i+1} / (1 - a_i) exactly as in the chunk-parallel kernel.  Partial rows as there.
// 4 workgroups per CU: 128 VGPRs, no spills (at 5: 96 VGPRs and ~110 B of spills per lane outside
// the walk -- config 4 bwd 18.9 vs 18.1 ms, profiles/r04_c4_glds_ab2.txt)
#ifndef GSR_BWD2D_MINB
#define GSR_BWD2D_MINB 4
#endif
// 1: the previous sub-chunk's records gathered straight into a second LDS buffer with
// global_load_lds during the walk (no registers; LDS 38 KB) -- measured 18.5 vs 18.1 ms for the
// register staging after the walk, kept as an option
#ifndef GSR_BWD2D_GLDS
#define GSR_BWD2D_GLDS 0
#endif
__global__ __launch_bounds__(kRasterThreads, GSR_BWD2D_MINB) void k_raster2d_bwd_tile(
    const Splat* __restrict__ rec, const int32_t* __restrict__ ids, const float* __restrict__ anchors, int W, int H,
    int tw, int th, const float* __restrict__ bg, const float* __restrict__ final_T,
    const int32_t* __restrict__ last_in, const float* __restrict__ v_rgb, const float* __restrict__ v_alpha,
    float* __restrict__ partial, const int32_t* __restrict__ units, gsr_bin_stats* __restrict__ stats,
    const int32_t* __restrict__ k_of_s, float cut2d, const Sets2D sets) {
  constexpr int kNull = kChunk3;
  constexpr int kGroup = GSR_BWD_GROUP;
  constexpr int kLen = kChunk3 + kGroup;
  // Records are stored packed (pack_rec: the walk's nine values in 2 x b128 + b32) and each box's
  // survivor list has a pad byte after every 7 (grouped_slot), so a group's seven slots are ONE
  // 8-byte read instead of seven byte reads (19.07 -> 18.64 ms at config 4).
  // GL: the previous sub-chunk's records are gathered straight into the other half of a
  // double-buffered LDS image (global_load_lds, 16 B per lane: no registers, in flight during the
  // walk; the ids are read one sub-chunk earlier); else gathered into registers after the walk.
  constexpr bool GL = GSR_BWD2D_GLDS;
  constexpr int kLenB = 8 * ((kLen + kGroup - 1) / kGroup);
  __shared__ float4 s_p[GL ? 2 : 1][3][kChunk3 + 1];
  __shared__ __attribute__((aligned(16))) float L[kPartial][4][kChunk3 + 1];
  __shared__ unsigned char s_list[4][kLen];
  __shared__ __attribute__((aligned(16))) unsigned char s_box[4][4][kLenB];
  __shared__ float s_stage[4][64][4];
#ifdef GSR_BWD_TRACE
  // timing build (tools/bwd2d_trace.py): {start, end, nsub | cu << 32, wave 0's summed phases:
  // top barrier + staging, culls, groups, pre-rows barrier, rows}
  unsigned long long tr_t = wall_clock64(), tr_acc[5] = {0, 0, 0, 0, 0};
  const unsigned long long tr_start = tr_t;
#define BWD2_P(i)                                     \
  if (threadIdx.x == 0) {                              \
    const unsigned long long now_ = wall_clock64();    \
    tr_acc[i] += now_ - tr_t;                          \
    tr_t = now_;                                       \
  }
#else
#define BWD2_P(i)
#endif
  // the unit {first entry, entries, first record row, tile}, the stats words: one round trip
  const int4 cd = reinterpret_cast<const int4*>(units)[blockIdx.x];
  const int n_act = stats->n_active, ovf = stats->overflow, U = stats->chunk_entries;
  if ((ovf != 0) | ((int)blockIdx.x >= n_act) | (cd.y <= 0)) return;
  const int start = cd.x, n = cd.y, cbase = cd.z, ct = cd.w;
  int c, ty, tx;
  tile_coords(ct, tw, th, c, ty, tx);
  rec += rec_offset2d(sets.begin, sets.F, c, sets.N);   // the set's record copy
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int box = lane & 3, pos = lane >> 2;
  const int qx0 = tx * kTile + (wv & 1) * 8, qy0 = ty * kTile + (wv >> 1) * 8;   // quadrant origin
  const int pi = qy0 + (box >> 1) * 4 + (pos >> 2), pj = qx0 + (box & 1) * 4 + (pos & 3);
  const bool inside = pi < H && pj < W;
  const float px = (float)pj, py = (float)pi;   // 2D: integer centres (src/gaussian_renderer.py:355-358)
  const int slot = ckpt_slot_of(wv, box, pos);
  // the last sub-chunk [sb0, sb0 + sn) first: its ids, emission indices and records
  const int nsub = (n + kChunk3 - 1) / kChunk3;
  int sb0 = start + (nsub - 1) * kChunk3;
  int sn = start + n - sb0;
  const bool loader = threadIdx.x < kChunk3;   // waves 0 and 1 stage a sub-chunk's 128 entries
  const int id_mine = threadIdx.x < sn ? ids[sb0 + threadIdx.x] : 0;
  int kos_mine = threadIdx.x < sn ? k_of_s[sb0 + threadIdx.x] : 0;
  // GL: the ids of the sub-chunk before the last (gathered at the start of the last one's walk)
  int id_pf = GL && nsub > 1 && loader ? ids[sb0 - kChunk3 + threadIdx.x] : 0;
  float Tf = 1.f, Tl = 1.f, vr = 0.f, vg = 0.f, vb = 0.f, va = 0.f;
  int last = -1;
  if (inside) {
    const int64_t pix = ((int64_t)c * H + pi) * W + pj;
    last = last_in[pix];
    const float2 t2 = reinterpret_cast<const float2*>(final_T)[pix];
    Tf = t2.x;
    Tl = t2.y;
    vr = v_rgb[pix * 3 + 0];
    vg = v_rgb[pix * 3 + 1];
    vb = v_rgb[pix * 3 + 2];
    va = v_alpha[pix];
  }
  const float4* const rec4 = reinterpret_cast<const float4*>(rec);
  float4 sp0 = make_float4(0.f, 0.f, 0.f, 0.f), sp1 = sp0, sp2 = sp0;
  if (threadIdx.x < sn) {
    sp0 = rec4[3 * (int64_t)id_mine + 0];
    sp1 = rec4[3 * (int64_t)id_mine + 1];
    sp2 = rec4[3 * (int64_t)id_mine + 2];
  }
  const float* bgc = bg + c * 3;
  // mu after the pixel's last entry; T at the list's end is the final T (tile_end - 1 is the
  // tile's last composited entry, so no pixel has a valid entry after it)
  float mu = bgc[0] * vr + bgc[1] * vg + bgc[2] * vb - va;
  float T = Tf, T_next = Tf;
  const int wlast = wave_max_i(last);
  const int fg = lane / kPartial, fq = lane - kPartial * (lane / kPartial);
  const bool fown = lane < kGroup * kPartial;
  float* const Lw = &L[fq][wv][0];
  const float* const stage_rd = &s_stage[wv][0][0] + 4 * (4 * (lane >> 2)) + (lane & 3);   // + 4*box
  const unsigned char* my_list = s_box[wv][box];
  if (threadIdx.x < 3 * (GL ? 2 : 1)) s_p[threadIdx.x / 3][threadIdx.x % 3][kNull] = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int sub = nsub - 1; sub >= 0; --sub) {
    const int buf = GL ? (nsub - 1 - sub) & 1 : 0;
    float4 (*const sp)[kChunk3 + 1] = s_p[buf];
    if (sub != nsub - 1) {
      __syncthreads();   // the previous sub-chunk's LDS is consumed (and, GL, this one's gathers landed)
      // re-anchor T where this sub-chunk ends on a unit boundary (T_next: read during the
      // previous sub-chunk's rows)
      if (((sb0 + sn - start) & (U - 1)) == 0) T = T_next;
    }
    if (!GL || sub == nsub - 1) {
      if (threadIdx.x < sn) {
        sp[0][threadIdx.x] = sp0;
        sp[1][threadIdx.x] = sp1;
        sp[2][threadIdx.x] = sp2;
      }
    }
    for (int i = threadIdx.x; i < kPartial * (kChunk3 + 1); i += kRasterThreads)   // b128 stores
      reinterpret_cast<float4*>(&L[0][0][0])[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    __syncthreads();
    if (GL && sub > 0 && loader) {
      // the previous sub-chunk's records into the other buffer (in flight during the walk), then
      // the ids of the one before it
      const float4* src = rec4 + 3 * (int64_t)id_pf;
#pragma unroll
      for (int j = 0; j < 3; ++j)
        __builtin_amdgcn_global_load_lds(src + j, (__attribute__((address_space(3))) void*)&s_p[buf ^ 1][j][64 * wv],
                                         16, 0, 0);
      if (sub > 1) id_pf = ids[sb0 - 2 * kChunk3 + threadIdx.x];
    }
    BWD2_P(0);
    const int lastk = min(last - sb0, kChunk3 - 1);   // < 0: the pixel stopped before this sub-chunk
    const int lastq = last - sb0 < kChunk3 ? last - sb0 : -1;
    int nsurv = 0;
    {
      const float x0 = (float)qx0, y0 = (float)qy0;
#pragma unroll
      for (int q = kChunk3 / 64 - 1; q >= 0; --q) {
        const int k = q * 64 + lane;
        float4 r0 = sp[0][k], r1 = sp[1][k], r2 = sp[2][k];
        unpack_rec<true>(r0, r1, r2);
        const bool keep = k < sn && (sb0 + k) <= wlast && cull_keep<true>(r0, r1, r2, x0, x0 + 7.f, y0, y0 + 7.f);
        const unsigned long long mk = __ballot(keep);
        if (keep) {
          const unsigned long long above = lane == 63 ? 0ull : (mk >> (lane + 1));
          s_list[wv][nsurv + __popcll(above)] = (unsigned char)k;
        }
        nsurv += __popcll(mk);
      }
    }
    __builtin_amdgcn_wave_barrier();
    int nbx[4];
    box4_cull<true, true, true>(s_list[wv], nsurv, sp[0], sp[1], sp[2], (float)qx0, (float)qy0, &s_box[wv][0][0],
                                kLenB, nbx);
    const int nb = box == 0 ? nbx[0] : box == 1 ? nbx[1] : box == 2 ? nbx[2] : nbx[3];
    const int ngrp = max(max(nbx[0], nbx[1]), max(nbx[2], nbx[3]));
    const int npad = (ngrp + kGroup - 1) / kGroup * kGroup;
    for (int s = nb + pos; s < npad; s += 16) s_box[wv][box][grouped_slot(s)] = (unsigned char)kNull;
    __builtin_amdgcn_wave_barrier();
    BWD2_P(1);
    // the walk (as k_raster_bwd, IS2D): invalid pairs enter with alpha 0 (ra = 1, no change)
    for (int g0 = 0, gb = 0; g0 < ngrp; g0 += kGroup, gb += 8) {
      float acc[64];
      acc[63] = 0.f;
      const uint2 w8 = *reinterpret_cast<const uint2*>(my_list + gb);
#pragma unroll
      for (int g = 0; g < kGroup; ++g) {
        const int k = (int)(((g < 4 ? w8.x : w8.y) >> (8 * (g & 3))) & 0xFFu);
        const float4 p0 = sp[0][k];   // x, y, o, r
        const float4 p1 = sp[1][k];   // a, b, c, g
        const float cbl = reinterpret_cast<const float*>(&sp[2][k])[0];   // blue
        const float dx = p0.x - px, dy = p0.y - py;
        const float sigma = conic_sigma(p1, dx, dy);
        const float alpha = p0.z * gauss_exp<true>(sigma);
        const bool valid = k <= lastk && alpha >= cut2d;
        const float alpha_v = valid ? alpha : 0.f;
        const float ra = __builtin_amdgcn_rcpf(1.f - alpha_v);
        T = k == lastq ? Tl : T * ra;
        const float fac = alpha_v * T;
        acc[g * kPartial + 6] = fac * vr;
        acc[g * kPartial + 7] = fac * vg;
        acc[g * kPartial + 8] = fac * vb;
        const float cv = p0.w * vr + p1.w * vg + cbl * vb;
        const float dmu = cv - mu;
        const float v_sig = -alpha_v * (T * dmu);
        mu = mu + alpha_v * dmu;
        const float tx_ = v_sig * dx, ty_ = v_sig * dy;
        acc[g * kPartial + 0] = tx_;
        acc[g * kPartial + 1] = ty_;
        acc[g * kPartial + 2] = tx_ * dx;
        acc[g * kPartial + 3] = tx_ * dy;
        acc[g * kPartial + 4] = ty_ * dy;
        acc[g * kPartial + 5] = v_sig;
      }
      float sum[4];
      reduce_box16(acc, sum);
      reinterpret_cast<float4*>(&s_stage[wv][0][0])[lane] = make_float4(sum[0], sum[1], sum[2], sum[3]);
      __builtin_amdgcn_wave_barrier();
      if (fown) {
#pragma unroll
        for (int bx = 0; bx < 4; ++bx) {
          const int k = s_box[wv][bx][gb + fg];
          Lw[k] += stage_rd[4 * bx];
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
    BWD2_P(2);
    // the previous sub-chunk's emission indices (and, !GL, records), read while this one's rows
    // are summed and stored (assigned on every path: a conditional assignment would keep the old
    // values live across the walk)
    const int kos_next = sub > 0 && loader ? k_of_s[sb0 - kChunk3 + threadIdx.x] : 0;
    // T at the previous sub-chunk's end when that is a unit boundary: the forward wrote the
    // pixel's T there if the pixel was still live (its last entry lies beyond), else it is Tf
    // (consumed after the next top barrier, which waits for every load anyway)
    const int ue = sb0 - start;
    T_next = sub > 0 && (ue & (U - 1)) == 0 && last >= sb0 ? anchors[(int64_t)(cbase + ue / U) * kRasterThreads + slot] : Tf;
    if (!GL) {
      sp0 = sp1 = sp2 = make_float4(0.f, 0.f, 0.f, 0.f);
      if (sub > 0 && loader) {
        const int id_next = ids[sb0 - kChunk3 + threadIdx.x];
        sp0 = rec4[3 * (int64_t)id_next + 0];
        sp1 = rec4[3 * (int64_t)id_next + 1];
        sp2 = rec4[3 * (int64_t)id_next + 2];
      }
    }
    __syncthreads();
    BWD2_P(3);
    if (threadIdx.x < sn) {
      const int k = threadIdx.x;
      float v[kPartial];
#pragma unroll
      for (int q = 0; q < kPartial; ++q) v[q] = (L[q][0][k] + L[q][1][k]) + (L[q][2][k] + L[q][3][k]);
      const float4 p1 = sp[1][k];
      const float mx = v[0], my = v[1];
      // (2D records hold the conic times log2(e): the mean's chain takes the unscaled one)
      v[0] = (2.f * p1.x * mx + p1.y * my) * kLn2;
      v[1] = (p1.y * mx + 2.f * p1.z * my) * kLn2;
      v[5] = -v[5] / sp[0][k].z;
      store_partial_row(partial, kos_mine, v);   // (2D emissions store no masks)
    }
    BWD2_P(4);
    sb0 -= kChunk3;
    sn = kChunk3;
    kos_mine = kos_next;
  }
#ifdef GSR_BWD_TRACE
  if (threadIdx.x == 0 && g_bwd_trace != nullptr) {
    unsigned long long* dst = g_bwd_trace + (int64_t)blockIdx.x * 16;
    dst[0] = tr_start;
    dst[1] = wall_clock64();
    dst[2] = ((unsigned long long)__smid() << 32) | (unsigned)nsub;
    for (int i = 0; i < 5; ++i) dst[3 + i] = tr_acc[i];
  }
#endif
}
#undef BWD2_P

// ---------------------------------------------------------------- 2D backward, per tile, pixel pairs
// k_raster2d_bwd_tile's walk with TWO pixels per lane (the same column, rows r and r + 2 of a
// 4x4 box): every record read, list decode and transposed reduction serves two pixels, and
// their contributions are summed in registers before the reduction.  One workgroup of 2 waves
// per tile; wave w owns the 16x8 half-tile of rows 8w..8w+7 (eight 4x4 boxes); lane l serves
// box l & 7 (bits 0-2), pixel pair l >> 3.  The reduction runs over lane bits 5-3 (reduce_box8:
// two permlane-swap levels and one DPP level), so each lane holds 8 of its box's 63 sums.  Same
// sub-chunk walk, T anchors, mu carry and partial rows as k_raster2d_bwd_tile; the per-entry
// sums are two waves' slots (L[q][0][k] + L[q][1][k]).
#ifndef GSR_BWD2D_PAIR
#define GSR_BWD2D_PAIR 1
#endif
#ifndef GSR_BWD2P_MINB
#define GSR_BWD2P_MINB 3   // waves per SIMD the compiler aims at: 3 -> 168 VGPRs, ~no spills (4: 128 VGPRs + 120 B of spills, 18.7 vs 17.5 ms)
#endif
__global__ __launch_bounds__(128, GSR_BWD2P_MINB) void k_raster2d_bwd_pair(
    const Splat* __restrict__ rec, const int32_t* __restrict__ ids, const float* __restrict__ anchors, int W, int H,
    int tw, int th, const float* __restrict__ bg, const float* __restrict__ final_T,
    const int32_t* __restrict__ last_in, const float* __restrict__ v_rgb, const float* __restrict__ v_alpha,
    float* __restrict__ partial, const int32_t* __restrict__ units, gsr_bin_stats* __restrict__ stats,
    const int32_t* __restrict__ k_of_s, float cut2d, const Sets2D sets) {
  constexpr int kNull = kChunk3;
  constexpr int kGroup = GSR_BWD_GROUP;
  static_assert(kGroup == 7 && kPartial == 9, "reduce_box8 sums 7 entries x 9 values in 64 registers");
  constexpr int kLen = kChunk3 + kGroup;
  constexpr int kLenB = 8 * ((kLen + kGroup - 1) / kGroup);
  __shared__ float4 s_p[3][kChunk3 + 1];   // packed records of the sub-chunk (pack_rec layout)
  __shared__ __attribute__((aligned(16))) float L[kPartial][2][kChunk3 + 1];
  __shared__ unsigned char s_list[2][kLen];
  __shared__ __attribute__((aligned(16))) unsigned char s_box[2][8][kLenB];
  // per wave: the group's reduced sums, box-major rows of 64 (reduce_grp8's swizzled staging)
  __shared__ __attribute__((aligned(16))) float s_stage[2][8][64];
  const int4 cd = reinterpret_cast<const int4*>(units)[blockIdx.x];
  const int n_act = stats->n_active, ovf = stats->overflow, U = stats->chunk_entries;
  if ((ovf != 0) | ((int)blockIdx.x >= n_act) | (cd.y <= 0)) return;
  const int start = cd.x, n = cd.y, cbase = cd.z, ct = cd.w;
  int c, ty, tx;
  tile_coords(ct, tw, th, c, ty, tx);
  rec += rec_offset2d(sets.begin, sets.F, c, sets.N);   // the set's record copy
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  // box: two per ds_read_b128 lane group (reduce_grp8), so a walk read is two addresses per group
  const int box = grp8_box(lane), pp = grp8_pos(lane);
  const int hx0 = tx * kTile, hy0 = ty * kTile + 8 * wv;   // the wave's 16x8 half-tile
  const int bjl = 4 * (box & 3), bil = 8 * wv + 4 * (box >> 2);   // box origin in the tile
  const int jl = bjl + (pp & 3), ilA = bil + (pp >> 2), ilB = ilA + 2;
  const int pj = tx * kTile + jl, piA = ty * kTile + ilA, piB = ty * kTile + ilB;
  const bool inA = piA < H && pj < W, inB = piB < H && pj < W;
  const float px = (float)pj, pyA = (float)piA, pyB = (float)piB;   // 2D: integer centres
  const int slotA = bwd_pixel_slot(ilA, jl), slotB = bwd_pixel_slot(ilB, jl);
  const int nsub = (n + kChunk3 - 1) / kChunk3;
  int sb0 = start + (nsub - 1) * kChunk3;
  int sn = start + n - sb0;
  const int id_mine = (int)threadIdx.x < sn ? ids[sb0 + threadIdx.x] : 0;
  int kos_mine = (int)threadIdx.x < sn ? k_of_s[sb0 + threadIdx.x] : 0;
  float TfA = 1.f, TlA = 1.f, vrA = 0.f, vgA = 0.f, vbA = 0.f, vaA = 0.f;
  float TfB = 1.f, TlB = 1.f, vrB = 0.f, vgB = 0.f, vbB = 0.f, vaB = 0.f;
  int lastA = -1, lastB = -1;
  if (inA) {
    const int64_t pix = ((int64_t)c * H + piA) * W + pj;
    lastA = last_in[pix];
    const float2 t2 = reinterpret_cast<const float2*>(final_T)[pix];
    TfA = t2.x;
    TlA = t2.y;
    vrA = v_rgb[pix * 3 + 0];
    vgA = v_rgb[pix * 3 + 1];
    vbA = v_rgb[pix * 3 + 2];
    vaA = v_alpha[pix];
  }
  if (inB) {
    const int64_t pix = ((int64_t)c * H + piB) * W + pj;
    lastB = last_in[pix];
    const float2 t2 = reinterpret_cast<const float2*>(final_T)[pix];
    TfB = t2.x;
    TlB = t2.y;
    vrB = v_rgb[pix * 3 + 0];
    vgB = v_rgb[pix * 3 + 1];
    vbB = v_rgb[pix * 3 + 2];
    vaB = v_alpha[pix];
  }
  const float4* const rec4 = reinterpret_cast<const float4*>(rec);
  float4 sp0 = make_float4(0.f, 0.f, 0.f, 0.f), sp1 = sp0, sp2 = sp0;
  if ((int)threadIdx.x < sn) {
    sp0 = rec4[3 * (int64_t)id_mine + 0];
    sp1 = rec4[3 * (int64_t)id_mine + 1];
    sp2 = rec4[3 * (int64_t)id_mine + 2];
  }
  const float* bgc = bg + c * 3;
  float muA = bgc[0] * vrA + bgc[1] * vgA + bgc[2] * vbA - vaA;
  float muB = bgc[0] * vrB + bgc[1] * vgB + bgc[2] * vbB - vaB;
  float TA = TfA, TB = TfB, TnA = TfA, TnB = TfB;
  const int wlast = wave_max_i(max(lastA, lastB));
  // the L update: lane f < 63 owns flat sum index f = 9 g + q of every box
  const int fg = lane / kPartial, fq = lane - kPartial * (lane / kPartial);
  const bool fown = lane < kGroup * kPartial;
  float* const Lw = &L[fq][wv][0];
  // lane f reads flat sum f of box bx at s_stage[wv][bx][f ^ grp8_swz(bx)]; lane l stages its 8
  // sums (box grp8_out_box(l), flat 8 grp8_slot(l) + i) as two b128 stores
  const float* const stage_rd = &s_stage[wv][0][0];
  const int obox = grp8_out_box(lane);
  float* const stage_wr = &s_stage[wv][obox][0];
  const int wr0 = (8 * grp8_slot(lane)) ^ grp8_swz(obox), wr1 = (8 * grp8_slot(lane) + 4) ^ grp8_swz(obox);
  const unsigned char* my_list = s_box[wv][box];
  if (threadIdx.x < 3) s_p[threadIdx.x][kNull] = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int sub = nsub - 1; sub >= 0; --sub) {
    if (sub != nsub - 1) {
      __syncthreads();   // the previous sub-chunk's LDS is consumed
      if (((sb0 + sn - start) & (U - 1)) == 0) {   // re-anchor T at a unit boundary
        TA = TnA;
        TB = TnB;
      }
    }
    if ((int)threadIdx.x < sn) {
      s_p[0][threadIdx.x] = sp0;
      s_p[1][threadIdx.x] = sp1;
      s_p[2][threadIdx.x] = sp2;
    }
    for (int i = threadIdx.x; i < kPartial * 2 * (kChunk3 + 1) / 4; i += 128)   // b128 stores
      reinterpret_cast<float4*>(&L[0][0][0])[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (threadIdx.x == 0 && (kPartial * 2 * (kChunk3 + 1)) % 4 != 0)
      for (int i = kPartial * 2 * (kChunk3 + 1) / 4 * 4; i < kPartial * 2 * (kChunk3 + 1); ++i) (&L[0][0][0])[i] = 0.f;
    __syncthreads();
    const int lastqA = lastA - sb0 < kChunk3 ? lastA - sb0 : -1, lastqB = lastB - sb0 < kChunk3 ? lastB - sb0 : -1;
    // cull the sub-chunk against the wave's 16x8 half-tile (exact test), survivors back to front
    int nsurv = 0;
    {
      const float x0 = (float)hx0, y0 = (float)hy0;
#pragma unroll
      for (int q = kChunk3 / 64 - 1; q >= 0; --q) {
        const int k = q * 64 + lane;
        float4 r0 = s_p[0][k], r1 = s_p[1][k], r2 = s_p[2][k];
        unpack_rec<true>(r0, r1, r2);
        const bool keep = k < sn && (sb0 + k) <= wlast && cull_keep<true>(r0, r1, r2, x0, x0 + 15.f, y0, y0 + 7.f);
        const unsigned long long mk = __ballot(keep);
        if (keep) {
          const unsigned long long above = lane == 63 ? 0ull : (mk >> (lane + 1));
          s_list[wv][nsurv + __popcll(above)] = (unsigned char)k;
        }
        nsurv += __popcll(mk);
      }
    }
    __builtin_amdgcn_wave_barrier();
    // ... and against the eight 4x4 boxes (one survivor per lane, its record read once)
    int nbx[8];
#pragma unroll
    for (int b = 0; b < 8; ++b) nbx[b] = 0;
    {
      const unsigned long long below = (1ull << lane) - 1ull;
      for (int s0 = 0; s0 < nsurv; s0 += 64) {
        const int si = s0 + lane;
        const bool in = si < nsurv;
        const int k = s_list[wv][in ? si : 0];
        float4 r0 = s_p[0][k], r1 = s_p[1][k], r2 = s_p[2][k];
        unpack_rec<true>(r0, r1, r2);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
          const float x0 = (float)(hx0 + 4 * (b & 3)), y0 = (float)(hy0 + 4 * (b >> 2));
          const bool keep = in && cull_keep<true>(r0, r1, r2, x0, x0 + 3.f, y0, y0 + 3.f);
          const unsigned long long m = __ballot(keep);
          if (keep) s_box[wv][b][grouped_slot(nbx[b] + __popcll(m & below))] = (unsigned char)k;
          nbx[b] += __popcll(m);
        }
      }
    }
    int nb = nbx[0], ngrp = nbx[0];
#pragma unroll
    for (int b = 1; b < 8; ++b) {
      nb = box == b ? nbx[b] : nb;
      ngrp = max(ngrp, nbx[b]);
    }
    const int npad = (ngrp + kGroup - 1) / kGroup * kGroup;
    for (int s = nb + pp; s < npad; s += 8) s_box[wv][box][grouped_slot(s)] = (unsigned char)kNull;
    __builtin_amdgcn_wave_barrier();
    // the walk: both pixels of the lane per entry, their contributions summed in registers
    for (int g0 = 0, gb = 0; g0 < ngrp; g0 += kGroup, gb += 8) {
      float acc[64];
      acc[63] = 0.f;
      const uint2 w8 = *reinterpret_cast<const uint2*>(my_list + gb);
      int kk[kGroup];
#pragma unroll
      for (int g = 0; g < kGroup; ++g) kk[g] = (int)(((g < 4 ? w8.x : w8.y) >> (8 * (g & 3))) & 0xFFu);
      float4 n0 = s_p[0][kk[0]], n1 = s_p[1][kk[0]];
      float n2 = reinterpret_cast<const float*>(&s_p[2][kk[0]])[0];
#pragma unroll
      for (int g = 0; g < kGroup; ++g) {
        const int k = kk[g];
        const float4 p0 = n0;   // x, y, o, r
        const float4 p1 = n1;   // a, b, c, g
        const float cbl = n2;   // blue
        if (g + 1 < kGroup) {   // entry g+1's record read before entry g is evaluated (GSR_BWD_PF)
          n0 = s_p[0][kk[g + 1]];
          n1 = s_p[1][kk[g + 1]];
          n2 = reinterpret_cast<const float*>(&s_p[2][kk[g + 1]])[0];
        }
        walk_fence();
        const float dx = p0.x - px, dyA = p0.y - pyA;
        const int ks = sb0 + k;   // the entry's list position (the zero pad slot is never valid: alpha 0)
        // the entry's 9 sums over the lane's two pixels: pixel A sets them, pixel B adds (a
        // zero start cost 63 "0 + x" adds per group: IEEE keeps them, -0 + 0 = +0)
        float a6, a7, a8, a0, a1, a2, a3, a4, a5;
        auto pixel = [&](const bool first, float dy, int last, int lastq, float Tl, float vr, float vg, float vb,
                         float& T, float& mu) {
          auto add = [first](float& a, float x) { a = first ? x : a + x; };
          const float sigma = conic_sigma(p1, dx, dy);
          const float alpha = p0.z * gauss_exp<true>(sigma);
          // (& not &&: with a short-circuit the compiler wrapped each pixel's exp in a branch)
          const bool valid = (ks <= last) & (alpha >= cut2d);
          const float alpha_v = valid ? alpha : 0.f;
          const float ra = __builtin_amdgcn_rcpf(1.f - alpha_v);
          T = k == lastq ? Tl : T * ra;
          const float fac = alpha_v * T;
          add(a6, fac * vr);
          add(a7, fac * vg);
          add(a8, fac * vb);
          const float cv = p0.w * vr + p1.w * vg + cbl * vb;
          const float dmu = cv - mu;
          const float v_sig = -alpha_v * (T * dmu);
          mu = mu + alpha_v * dmu;
          const float tx_ = v_sig * dx, ty_ = v_sig * dy;
          add(a0, tx_);
          add(a1, ty_);
          add(a2, tx_ * dx);
          add(a3, tx_ * dy);
          add(a4, ty_ * dy);
          add(a5, v_sig);
        };
        pixel(true, dyA, lastA, lastqA, TlA, vrA, vgA, vbA, TA, muA);
        pixel(false, p0.y - pyB, lastB, lastqB, TlB, vrB, vgB, vbB, TB, muB);   // (dy as the forward forms it)
        acc[g * kPartial + 0] = a0;
        acc[g * kPartial + 1] = a1;
        acc[g * kPartial + 2] = a2;
        acc[g * kPartial + 3] = a3;
        acc[g * kPartial + 4] = a4;
        acc[g * kPartial + 5] = a5;
        acc[g * kPartial + 6] = a6;
        acc[g * kPartial + 7] = a7;
        acc[g * kPartial + 8] = a8;
      }
      float sum[8];
      reduce_grp8(acc, sum);
      *reinterpret_cast<float4*>(stage_wr + wr0) = make_float4(sum[0], sum[1], sum[2], sum[3]);
      *reinterpret_cast<float4*>(stage_wr + wr1) = make_float4(sum[4], sum[5], sum[6], sum[7]);
      __builtin_amdgcn_wave_barrier();
      if (fown) {   // two batches of four boxes (lw_add)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          int kb[4];
          float vb4[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int bx = 4 * h + j;
            kb[j] = s_box[wv][bx][gb + fg];
            vb4[j] = stage_rd[64 * bx + (lane ^ grp8_swz(bx))];
          }
          lw_add(Lw, kb, vb4);
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
    // the previous sub-chunk's ids, emission indices, records and T anchors, read while this
    // one's rows are summed and stored (assigned on every path)
    const bool more = sub > 0 && (int)threadIdx.x < kChunk3;
    const int kos_next = more ? k_of_s[sb0 - kChunk3 + threadIdx.x] : 0;
    sp0 = sp1 = sp2 = make_float4(0.f, 0.f, 0.f, 0.f);
    if (more) {
      const int id_next = ids[sb0 - kChunk3 + threadIdx.x];
      sp0 = rec4[3 * (int64_t)id_next + 0];
      sp1 = rec4[3 * (int64_t)id_next + 1];
      sp2 = rec4[3 * (int64_t)id_next + 2];
    }
    {
      const int ue = sb0 - start;
      const bool anch = sub > 0 && (ue & (U - 1)) == 0;
      const int64_t arow = (int64_t)(cbase + ue / U) * kRasterThreads;
      TnA = anch && lastA >= sb0 ? anchors[arow + slotA] : TfA;
      TnB = anch && lastB >= sb0 ? anchors[arow + slotB] : TfB;
    }
    __syncthreads();
    if ((int)threadIdx.x < sn) {
      const int k = threadIdx.x;
      float v[kPartial];
#pragma unroll
      for (int q = 0; q < kPartial; ++q) v[q] = L[q][0][k] + L[q][1][k];
      const float4 p1 = s_p[1][k];
      const float mx = v[0], my = v[1];
      // (2D records hold the conic times log2(e): the mean's chain takes the unscaled one)
      v[0] = (2.f * p1.x * mx + p1.y * my) * kLn2;
      v[1] = (p1.y * mx + 2.f * p1.z * my) * kLn2;
      v[5] = -v[5] / s_p[0][k].z;
      store_partial_row(partial, kos_mine, v);   // (2D emissions store no masks)
    }
    sb0 -= kChunk3;
    sn = kChunk3;
    kos_mine = kos_next;
  }
}

// ---------------------------------------------------------------- 2D backward, a frame's units per tile
// pose-splatter's 2D renderer ignores the view (src/gaussian_renderer.py:280-281): every camera
// of a parameter set renders the same image, from the same list over the same record copy, and
// only its cotangent differs.  k_raster2d_bwd_frame runs ONE workgroup per (set, tile) -- the
// set's first camera's sweep slot; the other cameras' slots exit -- and walks the tile's list
// once for all the set's cameras: the per-(entry, pixel) forward state (sigma, alpha, the
// validity test, T recovered by division, alpha T) is computed once, then every camera's pixel
// is walked with ITS OWN cotangent (its colour dot product, its own mu recursion, its colour
// partials), and the cameras' contributions are summed in registers before the one cross-lane
// reduction per group.  The entry's partial row -- the sum over the set's cameras -- is written
// once, at the set's first camera's emission index, and gsr2d_project_bwd reads only those rows
// (the rows of a set's cameras used to be written per camera and summed there).
//   Same layout, culls, sub-chunk walk, T anchors and reduction as k_raster2d_bwd_pair; the forward
// state read is the first camera's (bitwise equal to every camera's of the set:
// tests/test_multiframe_gpu.py checks it).  GB cameras are walked per pass (registers: 8 per
// camera and lane); a set with more walks its tile again per further GB cameras, adding to its
// rows.  A set of one camera (GB = 1) is k_raster2d_bwd_pair's arithmetic exactly.
// pairwise sum of K values (a tree of independent adds; K = 1: the value itself)
template <int K>
__device__ __forceinline__ float pair_sum(const float* v) {
  if constexpr (K == 1) {
    return v[0];
  } else {
    return pair_sum<K / 2>(v) + pair_sum<K - K / 2>(v + K / 2);
  }
}
#ifndef GSR_BWD2F_MINB
#define GSR_BWD2F_MINB 2   // waves per SIMD the compiler aims at (the per-camera state: 8 x GB VGPRs)
#endif
template <int GB>
__global__ __launch_bounds__(128, GSR_BWD2F_MINB) void k_raster2d_bwd_frame(
    const Splat* __restrict__ rec, const int32_t* __restrict__ ids, const float* __restrict__ anchors, int W, int H,
    int tw, int th, const float* __restrict__ bg, const float* __restrict__ final_T,
    const int32_t* __restrict__ last_in, const float* __restrict__ v_rgb, const float* __restrict__ v_alpha,
    float* __restrict__ partial, const int32_t* __restrict__ tile_offset, const int32_t* __restrict__ tile_end,
    const int32_t* __restrict__ chunk_base, gsr_bin_stats* __restrict__ stats, const int32_t* __restrict__ k_of_s,
    float cut2d, const Sets2D sets, int parts) {
  constexpr int kNull = kChunk3;
  constexpr int kGroup = GSR_BWD_GROUP;
  static_assert(kGroup == 7 && kPartial == 9, "reduce_grp8 sums 7 entries x 9 values in 64 registers");
  constexpr int kLen = kChunk3 + kGroup;
  constexpr int kLenB = 8 * ((kLen + kGroup - 1) / kGroup);
  __shared__ float4 s_p[3][kChunk3 + 1];
  __shared__ __attribute__((aligned(16))) float L[kPartial][2][kChunk3 + 1];
  __shared__ unsigned char s_list[2][kLen];
  __shared__ __attribute__((aligned(16))) unsigned char s_box[2][8][kLenB];
  __shared__ __attribute__((aligned(16))) float s_stage[2][8][64];
  // One workgroup per (set, tile), XCD-aware: workgroup b runs on XCD b % 8 and takes position
  // (b % 8) * S + b / 8 of the (set, tile row, tile column) order, so each XCD walks its eighth
  // of it in order and a set's records come into its L2 about once.  (A grid of every camera's
  // tile slot with the other cameras' workgroups exiting put all the working ones on every
  // other CU -- the slots are dealt to an XCD's CUs in turn: half the chip idle.)
  const int T = tw * th;
  const int64_t FTP = (int64_t)sets.F * T * parts;   // (set, tile, part) slots, parts of a tile adjacent
  const int64_t S = (FTP + 7) / 8;
  const int64_t pos = (int64_t)(blockIdx.x & 7) * S + (blockIdx.x >> 3);
  const int ovf = stats->overflow, U = stats->chunk_entries;
  // split walks start from the colour planes: only if the forward wrote them (ADVICE r5 -- a
  // gsr_set_bwd2d_parts / gsr_set_fwd_lanes change between the calls); else refuse, loudly
  const bool planes_missing = parts > 1 && (stats->masks & kStatsPlanes2D) == 0;
  if (planes_missing) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      atomicOr(&stats->overflow, GSR_OVF_LAYOUT);
      if (stats->status != nullptr) atomicOr(stats->status, GSR_OVF_LAYOUT);
    }
    return;
  }
  if ((ovf != 0) | (pos >= FTP)) return;
  const int64_t tpos = pos / parts;
  const int part = (int)(pos - tpos * parts);
  const int f = (int)(tpos / T), t = (int)(tpos - (int64_t)f * T);
  const int cf = sets.begin != nullptr ? sets.begin[f] : 0;
  const int G = sets.begin != nullptr ? sets.begin[f + 1] - cf : 1;
  if (G <= 0) return;   // a set no camera renders
  const int ct = cf * T + t;
  const int start = tile_offset[ct], te = tile_end[ct], cbase = chunk_base[ct];
  const int n = te - start;   // the consumed list [start, tile_end) (k_raster_finalize)
  if (n <= 0) return;
  // this workgroup's part [pbeg, pend) of it: whole units, `parts` about equal ranges
  int pbeg = start, pend = te;
  if (parts > 1) {   // units [nu p / parts, nu (p + 1) / parts): none empty while nu >= parts
    const int nu = (n + U - 1) / U, u_lo = (int)((int64_t)nu * part / parts),
              u_hi = (int)((int64_t)nu * (part + 1) / parts);
    if (u_lo >= u_hi) return;
    pbeg = start + u_lo * U;
    pend = min(start + u_hi * U, te);
  }
  int c, ty, tx;
  tile_coords(ct, tw, th, c, ty, tx);   // (c = cf: the set's record copy, rec_offset2d = 0)
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int box = grp8_box(lane), pp = grp8_pos(lane);
  const int hx0 = tx * kTile, hy0 = ty * kTile + 8 * wv;
  const int bjl = 4 * (box & 3), bil = 8 * wv + 4 * (box >> 2);
  const int jl = bjl + (pp & 3), ilA = bil + (pp >> 2), ilB = ilA + 2;
  const int pj = tx * kTile + jl, piA = ty * kTile + ilA, piB = ty * kTile + ilB;
  const bool inA = piA < H && pj < W, inB = piB < H && pj < W;
  const float px = (float)pj, pyA = (float)piA, pyB = (float)piB;
  const int slotA = bwd_pixel_slot(ilA, jl), slotB = bwd_pixel_slot(ilB, jl);
  const int64_t HW = (int64_t)H * W;
  const int64_t pvA = (int64_t)piA * W + pj, pvB = (int64_t)piB * W + pj;   // pixel within a camera's image
  // the shared forward state (camera cf's; every camera of the set has the same)
  float TfA = 1.f, TlA = 1.f, TfB = 1.f, TlB = 1.f;
  int lastA = -1, lastB = -1;
  if (inA) {
    lastA = last_in[(int64_t)c * HW + pvA];
    const float2 t2 = reinterpret_cast<const float2*>(final_T)[(int64_t)c * HW + pvA];
    TfA = t2.x;
    TlA = t2.y;
  }
  if (inB) {
    lastB = last_in[(int64_t)c * HW + pvB];
    const float2 t2 = reinterpret_cast<const float2*>(final_T)[(int64_t)c * HW + pvB];
    TfB = t2.x;
    TlB = t2.y;
  }
  // a part before the list's end starts from each live pixel's state there: T from the anchor at
  // pend, and (per camera, below) mu = (S.v + T_f mu_last) / T with S the colour after pend -- the
  // total minus the colour before pend (the forward's colour planes)
  const bool contA = pend < te && lastA >= pend, contB = pend < te && lastB >= pend;
  float T0A = TfA, T0B = TfB, SrA = 0.f, SgA = 0.f, SbA = 0.f, SrB = 0.f, SgB = 0.f, SbB = 0.f;
  if (contA | contB) {
    const int64_t pl = colour_plane2d(stats);
    const float* const ae = anchors + (int64_t)(cbase + (pend - start) / U) * kRasterThreads;
    const float* const a0 = anchors + (int64_t)cbase * kRasterThreads;
    if (contA) {
      T0A = ae[slotA];
      SrA = a0[pl + slotA] - ae[pl + slotA];
      SgA = a0[2 * pl + slotA] - ae[2 * pl + slotA];
      SbA = a0[3 * pl + slotA] - ae[3 * pl + slotA];
    }
    if (contB) {
      T0B = ae[slotB];
      SrB = a0[pl + slotB] - ae[pl + slotB];
      SgB = a0[2 * pl + slotB] - ae[2 * pl + slotB];
      SbB = a0[3 * pl + slotB] - ae[3 * pl + slotB];
    }
  }
  const int wlast = wave_max_i(max(lastA, lastB));
  const int fg = lane / kPartial, fq = lane - kPartial * (lane / kPartial);
  const bool fown = lane < kGroup * kPartial;
  float* const Lw = &L[fq][wv][0];
  const float* const stage_rd = &s_stage[wv][0][0];
  const int obox = grp8_out_box(lane);
  float* const stage_wr = &s_stage[wv][obox][0];
  const int wr0 = (8 * grp8_slot(lane)) ^ grp8_swz(obox), wr1 = (8 * grp8_slot(lane) + 4) ^ grp8_swz(obox);
  const unsigned char* my_list = s_box[wv][box];
  const float4* const rec4 = reinterpret_cast<const float4*>(rec);
  const int nsub = (pend - pbeg + kChunk3 - 1) / kChunk3;
  if (threadIdx.x < 3) s_p[threadIdx.x][kNull] = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int u0 = 0; u0 < G; u0 += GB) {
    // this pass's cameras' cotangents and mu (zero past the set's cameras: exact zero terms)
    float vrA[GB], vgA[GB], vbA[GB], muA[GB], vrB[GB], vgB[GB], vbB[GB], muB[GB];
#pragma unroll
    for (int u = 0; u < GB; ++u) {
      vrA[u] = vgA[u] = vbA[u] = muA[u] = vrB[u] = vgB[u] = vbB[u] = muB[u] = 0.f;
      const int cam = cf + u0 + u;
      if (u0 + u < G) {
        const float* bgc = bg + cam * 3;
        if (inA) {
          const int64_t pix = (int64_t)cam * HW + pvA;
          vrA[u] = v_rgb[pix * 3 + 0];
          vgA[u] = v_rgb[pix * 3 + 1];
          vbA[u] = v_rgb[pix * 3 + 2];
          muA[u] = bgc[0] * vrA[u] + bgc[1] * vgA[u] + bgc[2] * vbA[u] - v_alpha[pix];
        }
        if (inB) {
          const int64_t pix = (int64_t)cam * HW + pvB;
          vrB[u] = v_rgb[pix * 3 + 0];
          vgB[u] = v_rgb[pix * 3 + 1];
          vbB[u] = v_rgb[pix * 3 + 2];
          muB[u] = bgc[0] * vrB[u] + bgc[1] * vgB[u] + bgc[2] * vbB[u] - v_alpha[pix];
        }
      }
      if (contA) muA[u] = (SrA * vrA[u] + SgA * vgA[u] + SbA * vbA[u] + TfA * muA[u]) / T0A;
      if (contB) muB[u] = (SrB * vrB[u] + SgB * vgB[u] + SbB * vbB[u] + TfB * muB[u]) / T0B;
    }
    const float VrA = pair_sum<GB>(vrA), VgA = pair_sum<GB>(vgA), VbA = pair_sum<GB>(vbA);
    const float VrB = pair_sum<GB>(vrB), VgB = pair_sum<GB>(vgB), VbB = pair_sum<GB>(vbB);
    int sb0 = pbeg + (nsub - 1) * kChunk3;
    int sn = pend - sb0;
    const int id_mine = (int)threadIdx.x < sn ? ids[sb0 + threadIdx.x] : 0;
    int kos_mine = (int)threadIdx.x < sn ? k_of_s[sb0 + threadIdx.x] : 0;
    float4 sp0 = make_float4(0.f, 0.f, 0.f, 0.f), sp1 = sp0, sp2 = sp0;
    if ((int)threadIdx.x < sn) {
      sp0 = rec4[3 * (int64_t)id_mine + 0];
      sp1 = rec4[3 * (int64_t)id_mine + 1];
      sp2 = rec4[3 * (int64_t)id_mine + 2];
    }
    float TA = T0A, TB = T0B, TnA = TfA, TnB = TfB;
    for (int sub = nsub - 1; sub >= 0; --sub) {
      if (sub != nsub - 1 || u0 > 0) __syncthreads();   // the previous sub-chunk's (pass's) LDS is consumed
      if (sub != nsub - 1 && ((sb0 + sn - start) & (U - 1)) == 0) {   // re-anchor T at a unit boundary
        TA = TnA;
        TB = TnB;
      }
      if ((int)threadIdx.x < sn) {
        s_p[0][threadIdx.x] = sp0;
        s_p[1][threadIdx.x] = sp1;
        s_p[2][threadIdx.x] = sp2;
      }
      for (int i = threadIdx.x; i < kPartial * 2 * (kChunk3 + 1) / 4; i += 128)
        reinterpret_cast<float4*>(&L[0][0][0])[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (threadIdx.x == 0 && (kPartial * 2 * (kChunk3 + 1)) % 4 != 0)
        for (int i = kPartial * 2 * (kChunk3 + 1) / 4 * 4; i < kPartial * 2 * (kChunk3 + 1); ++i) (&L[0][0][0])[i] = 0.f;
      __syncthreads();
      const int lastqA = lastA - sb0 < kChunk3 ? lastA - sb0 : -1, lastqB = lastB - sb0 < kChunk3 ? lastB - sb0 : -1;
      int nsurv = 0;
      {
        const float x0 = (float)hx0, y0 = (float)hy0;
#pragma unroll
        for (int q = kChunk3 / 64 - 1; q >= 0; --q) {
          const int k = q * 64 + lane;
          float4 r0 = s_p[0][k], r1 = s_p[1][k], r2 = s_p[2][k];
          unpack_rec<true>(r0, r1, r2);
          const bool keep = k < sn && (sb0 + k) <= wlast && cull_keep<true>(r0, r1, r2, x0, x0 + 15.f, y0, y0 + 7.f);
          const unsigned long long mk = __ballot(keep);
          if (keep) {
            const unsigned long long above = lane == 63 ? 0ull : (mk >> (lane + 1));
            s_list[wv][nsurv + __popcll(above)] = (unsigned char)k;
          }
          nsurv += __popcll(mk);
        }
      }
      __builtin_amdgcn_wave_barrier();
      int nbx[8];
#pragma unroll
      for (int b = 0; b < 8; ++b) nbx[b] = 0;
      {
        const unsigned long long below = (1ull << lane) - 1ull;
        for (int s0 = 0; s0 < nsurv; s0 += 64) {
          const int si = s0 + lane;
          const bool in = si < nsurv;
          const int k = s_list[wv][in ? si : 0];
          float4 r0 = s_p[0][k], r1 = s_p[1][k], r2 = s_p[2][k];
          unpack_rec<true>(r0, r1, r2);
#pragma unroll
          for (int b = 0; b < 8; ++b) {
            const float x0 = (float)(hx0 + 4 * (b & 3)), y0 = (float)(hy0 + 4 * (b >> 2));
            const bool keep = in && cull_keep<true>(r0, r1, r2, x0, x0 + 3.f, y0, y0 + 3.f);
            const unsigned long long m = __ballot(keep);
            if (keep) s_box[wv][b][grouped_slot(nbx[b] + __popcll(m & below))] = (unsigned char)k;
            nbx[b] += __popcll(m);
          }
        }
      }
      int nb = nbx[0], ngrp = nbx[0];
#pragma unroll
      for (int b = 1; b < 8; ++b) {
        nb = box == b ? nbx[b] : nb;
        ngrp = max(ngrp, nbx[b]);
      }
      const int npad = (ngrp + kGroup - 1) / kGroup * kGroup;
      for (int s = nb + pp; s < npad; s += 8) s_box[wv][box][grouped_slot(s)] = (unsigned char)kNull;
      __builtin_amdgcn_wave_barrier();
      for (int g0 = 0, gb = 0; g0 < ngrp; g0 += kGroup, gb += 8) {
        float acc[64];
        acc[63] = 0.f;
        const uint2 w8 = *reinterpret_cast<const uint2*>(my_list + gb);
        int kk[kGroup];
#pragma unroll
        for (int g = 0; g < kGroup; ++g) kk[g] = (int)(((g < 4 ? w8.x : w8.y) >> (8 * (g & 3))) & 0xFFu);
        float4 n0 = s_p[0][kk[0]], n1 = s_p[1][kk[0]];
        float n2 = reinterpret_cast<const float*>(&s_p[2][kk[0]])[0];
#pragma unroll
        for (int g = 0; g < kGroup; ++g) {
          const int k = kk[g];
          const float4 p0 = n0;   // x, y, o, r
          const float4 p1 = n1;   // a, b, c, g
          const float cbl = n2;   // blue
          if (g + 1 < kGroup) {
            n0 = s_p[0][kk[g + 1]];
            n1 = s_p[1][kk[g + 1]];
            n2 = reinterpret_cast<const float*>(&s_p[2][kk[g + 1]])[0];
          }
          walk_fence();
          const float dx = p0.x - px, dyA = p0.y - pyA;
          const int ks = sb0 + k;
          float a6, a7, a8, a0, a1, a2, a3, a4, a5;
          auto pixel = [&](const bool first, float dy, int last, int lastq, float Tl, const float (&vr)[GB],
                           const float (&vg)[GB], const float (&vb)[GB], float (&mu)[GB], float& T, float Vr,
                           float Vg, float Vb) {
            auto add = [first](float& a, float x) { a = first ? x : a + x; };
            // the forward state, once for the set's cameras
            const float sigma = conic_sigma(p1, dx, dy);
            const float alpha = p0.z * gauss_exp<true>(sigma);
            const bool valid = (ks <= last) & (alpha >= cut2d);
            const float alpha_v = valid ? alpha : 0.f;
            const float ra = __builtin_amdgcn_rcpf(1.f - alpha_v);
            T = k == lastq ? Tl : T * ra;
            const float fac = alpha_v * T;
            // each camera with its own cotangent: its colour dot product, dL/d(mu) term and mu
            // recursion; the terms summed pairwise (independent chains, not one serial sum)
            float dmu[GB];
#pragma unroll
            for (int u = 0; u < GB; ++u) {
              const float cv = p0.w * vr[u] + p1.w * vg[u] + cbl * vb[u];
              dmu[u] = cv - mu[u];
              mu[u] = mu[u] + alpha_v * dmu[u];
            }
            const float sdmu = pair_sum<GB>(dmu);
            // colour partials: alpha T times the cameras' summed colour cotangent
            add(a6, fac * Vr);
            add(a7, fac * Vg);
            add(a8, fac * Vb);
            const float v_sig = -alpha_v * (T * sdmu);   // sum over the cameras of -alpha T (c.v - mu)
            const float tx_ = v_sig * dx, ty_ = v_sig * dy;
            add(a0, tx_);
            add(a1, ty_);
            add(a2, tx_ * dx);
            add(a3, tx_ * dy);
            add(a4, ty_ * dy);
            add(a5, v_sig);
          };
          pixel(true, dyA, lastA, lastqA, TlA, vrA, vgA, vbA, muA, TA, VrA, VgA, VbA);
          pixel(false, p0.y - pyB, lastB, lastqB, TlB, vrB, vgB, vbB, muB, TB, VrB, VgB, VbB);
          acc[g * kPartial + 0] = a0;
          acc[g * kPartial + 1] = a1;
          acc[g * kPartial + 2] = a2;
          acc[g * kPartial + 3] = a3;
          acc[g * kPartial + 4] = a4;
          acc[g * kPartial + 5] = a5;
          acc[g * kPartial + 6] = a6;
          acc[g * kPartial + 7] = a7;
          acc[g * kPartial + 8] = a8;
        }
        float sum[8];
        reduce_grp8(acc, sum);
        *reinterpret_cast<float4*>(stage_wr + wr0) = make_float4(sum[0], sum[1], sum[2], sum[3]);
        *reinterpret_cast<float4*>(stage_wr + wr1) = make_float4(sum[4], sum[5], sum[6], sum[7]);
        __builtin_amdgcn_wave_barrier();
        if (fown) {
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            int kb[4];
            float vb4[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int bx = 4 * h + j;
              kb[j] = s_box[wv][bx][gb + fg];
              vb4[j] = stage_rd[64 * bx + (lane ^ grp8_swz(bx))];
            }
            lw_add(Lw, kb, vb4);
          }
        }
        __builtin_amdgcn_wave_barrier();
      }
      const bool more = sub > 0 && (int)threadIdx.x < kChunk3;
      const int kos_next = more ? k_of_s[sb0 - kChunk3 + threadIdx.x] : 0;
      sp0 = sp1 = sp2 = make_float4(0.f, 0.f, 0.f, 0.f);
      if (more) {
        const int id_next = ids[sb0 - kChunk3 + threadIdx.x];
        sp0 = rec4[3 * (int64_t)id_next + 0];
        sp1 = rec4[3 * (int64_t)id_next + 1];
        sp2 = rec4[3 * (int64_t)id_next + 2];
      }
      {
        const int ue = sb0 - start;
        const bool anch = sub > 0 && (ue & (U - 1)) == 0;
        const int64_t arow = (int64_t)(cbase + ue / U) * kRasterThreads;
        TnA = anch && lastA >= sb0 ? anchors[arow + slotA] : TfA;
        TnB = anch && lastB >= sb0 ? anchors[arow + slotB] : TfB;
      }
      __syncthreads();
      if ((int)threadIdx.x < sn) {
        const int k = threadIdx.x;
        float v[kPartial];
#pragma unroll
        for (int q = 0; q < kPartial; ++q) v[q] = L[q][0][k] + L[q][1][k];
        const float4 p1 = s_p[1][k];
        const float mx = v[0], my = v[1];
        v[0] = (2.f * p1.x * mx + p1.y * my) * kLn2;
        v[1] = (p1.y * mx + 2.f * p1.z * my) * kLn2;
        v[5] = -v[5] / s_p[0][k].z;
        if (u0 == 0) {
          store_partial_row(partial, kos_mine, v);
        } else {   // a further pass over the set's cameras: this thread wrote the row in the first
          float* dst = partial + (int64_t)kos_mine * kPartialStride;
#pragma unroll
          for (int q = 0; q < kPartial; ++q) dst[q] += v[q];
        }
      }
      sb0 -= kChunk3;
      sn = kChunk3;
      kos_mine = kos_next;
    }
  }
}

// ---------------------------------------------------------------- 3D backward, pixel pairs
// k_raster_bwd (3D, one 128-entry chunk per workgroup, no fused loss, one sub-chunk) with the
// layout of k_raster2d_bwd_pair: TWO waves per chunk, wave w the 16x8 half-tile of rows
// 8w..8w+7, lane l box l & 7 and pixel pair l >> 3 (rows r and r + 2 of the box), both pixels'
// contributions summed in registers before reduce_box8.  A chunk holds half the waves of the
// 4-wave kernel, so more chunks are in flight per CU for the same number of waves.
// The pair layout is the throughput choice: it keeps 7 chunks per CU in flight (the 4-wave
// kernel 5) at a longer chunk latency, so the automatic choice (gsr_set_bwd_layout 0) takes it
// only for calls with many tiles per CU -- config 5 (27 648 tiles, ~35k chunks): raster bwd
// 0.60 -> 0.56 ms; config 3 (6 912 tiles, ~7.4k chunks): 0.136 -> 0.140 ms
// (r04_c35_pair3d_ab.txt).  The rule reads the call's shape (cameras x tiles), not its chunk
// count, so a bounded call and an exact one of the same shape take the same kernel (bitwise).
constexpr int kBwdPairTilesPerCU = 64;
#ifndef GSR_BWD3P_MINB
#define GSR_BWD3P_MINB 3   // waves per SIMD the compiler aims at
#endif
#ifndef GSR_BWD3P_HALFSTAGE
#define GSR_BWD3P_HALFSTAGE 1
#endif
__global__ __launch_bounds__(128, GSR_BWD3P_MINB) void k_raster_bwd_pair3d(
    const Splat* __restrict__ rec, const int32_t* __restrict__ ids, const float4* __restrict__ ckpt, int W, int H,
    int tw, int th, const float* __restrict__ bg, const float* __restrict__ final_T,
    const int32_t* __restrict__ last_in, const float* __restrict__ v_rgb, const float* __restrict__ v_alpha,
    float* __restrict__ partial, const int32_t* __restrict__ chunk_list, gsr_bin_stats* __restrict__ stats,
    const int32_t* __restrict__ k_of_s, const uint4* __restrict__ boxm = nullptr) {
  constexpr int kNull = kChunk3;
  constexpr int kGroup = GSR_BWD_GROUP;
  static_assert(kGroup == 7 && kPartial == 9, "reduce_box8 sums 7 entries x 9 values in 64 registers");
  constexpr int kLen = kChunk3 + kGroup;
  constexpr int kLenB = 8 * ((kLen + kGroup - 1) / kGroup);
  __shared__ float4 s_p[3][kChunk3 + 1];   // the chunk's records (Splat parts)
  __shared__ __attribute__((aligned(16))) float L[kPartial][2][kChunk3 + 1];
  __shared__ unsigned char s_list[2][kLen];
  __shared__ __attribute__((aligned(16))) unsigned char s_box[2][8][kLenB];
  // GSR_BWD3P_HALFSTAGE: stage the reduced sums in two halves (2 KB less LDS: 8 workgroups per CU)
  // (box-major rows of 64 -- 32 in halves -- per wave: reduce_grp8's swizzled staging)
  __shared__ __attribute__((aligned(16))) float s_stage[2][8][GSR_BWD3P_HALFSTAGE ? 32 : 64];
  const int4 cd = reinterpret_cast<const int4*>(chunk_list)[blockIdx.x];
  const int n_act = stats->n_active, ovf = stats->overflow, ce = stats->chunk_entries;
  const int smasks = stats->masks;
  const bool use_masks = (smasks & kStatsMasks3D) != 0;   // k_of_s bits 28..31 hold quadrant masks
  const bool unit_bad = ce != kChunk3;
  if ((ovf != 0) | ((int)blockIdx.x >= n_act) | unit_bad | (cd.y <= 0)) {
    if (unit_bad && blockIdx.x == 0 && threadIdx.x == 0) {
      atomicOr(&stats->overflow, GSR_OVF_UNIT);
      if (stats->status != nullptr) atomicOr(stats->status, GSR_OVF_UNIT);
    }
    return;
  }
  const int b0 = cd.x, sn = cd.y, chunk = cd.z, ct = cd.w;
  int c, ty, tx;
  tile_coords(ct, tw, th, c, ty, tx);
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int box = grp8_box(lane), pp = grp8_pos(lane);   // (two boxes per b128 lane group)
  const int hx0 = tx * kTile, hy0 = ty * kTile + 8 * wv;   // the wave's 16x8 half-tile
  const int bjl = 4 * (box & 3), bil = 8 * wv + 4 * (box >> 2);
  const int jl = bjl + (pp & 3), ilA = bil + (pp >> 2), ilB = ilA + 2;
  const int pj = tx * kTile + jl, piA = ty * kTile + ilA, piB = ty * kTile + ilB;
  const bool inA = piA < H && pj < W, inB = piB < H && pj < W;
  const float px = (float)pj + 0.5f, pyA = (float)piA + 0.5f, pyB = (float)piB + 0.5f;
  // every load up front (see k_raster_bwd): the two pixels' chunk records and state, ids, records
  const float4 rckA = ckpt[(int64_t)chunk * kRasterThreads + bwd_pixel_slot(ilA, jl)];
  const float4 rckB = ckpt[(int64_t)chunk * kRasterThreads + bwd_pixel_slot(ilB, jl)];
  // the forward's box survivor masks (as k_raster_bwd): this wave's 8 boxes are tile boxes
  // (bx, by) = (b & 3, 2 wv + (b >> 2)), mask slots 4 quadrant + box in quadrant = 8 wv + ..
  const bool use_bm = boxm != nullptr && (smasks & kStatsBoxMasks) != 0;
  uint4 bm[8] = {};
  if (use_bm) {
    const uint4* bmp = boxm + (int64_t)chunk * 16 + 8 * __builtin_amdgcn_readfirstlane(wv);
#pragma unroll
    for (int b = 0; b < 8; ++b) bm[b] = bmp[4 * ((b & 3) >> 1) + 2 * (b >> 2) + (b & 1)];
  }
  const int id_mine = (int)threadIdx.x < sn ? ids[b0 + threadIdx.x] : 0;
  const int kos_mine = (int)threadIdx.x < sn ? k_of_s[b0 + threadIdx.x] : 0;
  float TfA = 1.f, vrA = 0.f, vgA = 0.f, vbA = 0.f, vaA = 0.f;
  float TfB = 1.f, vrB = 0.f, vgB = 0.f, vbB = 0.f, vaB = 0.f;
  int lastA = -1, lastB = -1;
  if (inA) {
    const int64_t pix = ((int64_t)c * H + piA) * W + pj;
    lastA = last_in[pix];
    TfA = final_T[pix];
    vrA = v_rgb[pix * 3 + 0];
    vgA = v_rgb[pix * 3 + 1];
    vbA = v_rgb[pix * 3 + 2];
    vaA = v_alpha[pix];
  }
  if (inB) {
    const int64_t pix = ((int64_t)c * H + piB) * W + pj;
    lastB = last_in[pix];
    TfB = final_T[pix];
    vrB = v_rgb[pix * 3 + 0];
    vgB = v_rgb[pix * 3 + 1];
    vbB = v_rgb[pix * 3 + 2];
    vaB = v_alpha[pix];
  }
  const float4* const rec4 = reinterpret_cast<const float4*>(rec);
  if ((int)threadIdx.x < sn) {
    s_p[0][threadIdx.x] = rec4[3 * (int64_t)id_mine + 0];
    s_p[1][threadIdx.x] = rec4[3 * (int64_t)id_mine + 1];
    s_p[2][threadIdx.x] = rec4[3 * (int64_t)id_mine + 2];
  }
  for (int i = threadIdx.x; i < kPartial * 2 * (kChunk3 + 1) / 4; i += 128)   // b128 stores
    reinterpret_cast<float4*>(&L[0][0][0])[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (threadIdx.x == 0 && (kPartial * 2 * (kChunk3 + 1)) % 4 != 0)
    for (int i = kPartial * 2 * (kChunk3 + 1) / 4 * 4; i < kPartial * 2 * (kChunk3 + 1); ++i) (&L[0][0][0])[i] = 0.f;
  if (threadIdx.x < 3) s_p[threadIdx.x][kNull] = make_float4(0.f, 0.f, 0.f, 0.f);
  // the pixels' state at the chunk's end: {T_end, suffix colour sum} (forward epilogue); a pixel
  // that stopped before the chunk contributes nothing
  const bool liveA = lastA >= b0, liveB = lastB >= b0;
  if (!liveA) { TfA = 1.f; vrA = vgA = vbA = vaA = 0.f; }
  if (!liveB) { TfB = 1.f; vrB = vgB = vbB = vaB = 0.f; }
  const float* bgc = bg + c * 3;
  float TA = liveA ? rckA.x : TfA, TB = liveB ? rckB.x : TfB;
  const float vTaA = TfA * (vaA - (bgc[0] * vrA + bgc[1] * vgA + bgc[2] * vbA));
  const float vTaB = TfB * (vaB - (bgc[0] * vrB + bgc[1] * vgB + bgc[2] * vbB));
  float SvA = liveA ? rckA.y * vrA + rckA.z * vgA + rckA.w * vbA : 0.f;
  float SvB = liveB ? rckB.y * vrB + rckB.z * vgB + rckB.w * vbB : 0.f;
  const int wlast = wave_max_i(max(lastA, lastB));
  const int lastkA = min(lastA - b0, kChunk3 - 1), lastkB = min(lastB - b0, kChunk3 - 1);
  const int fg = lane / kPartial, fq = lane - kPartial * (lane / kPartial);
  const bool fown = lane < kGroup * kPartial;
  float* const Lw = &L[fq][wv][0];
  const float* const stage_rd = &s_stage[wv][0][0];
  const int obox = grp8_out_box(lane);
  float* const stage_wr = &s_stage[wv][obox][0];
#if GSR_BWD3P_HALFSTAGE
  // half h: sums 4h..4h+3 of every lane, compressed index 4 grp8_slot(l) + i (flat f -> ((f >> 3) << 2) | (f & 3))
  const int wr0 = (4 * grp8_slot(lane)) ^ grp8h_swz(obox);
  const int rdc = ((lane >> 3) << 2) | (lane & 3);
#else
  const int wr0 = (8 * grp8_slot(lane)) ^ grp8_swz(obox), wr1 = (8 * grp8_slot(lane) + 4) ^ grp8_swz(obox);
#endif
  const unsigned char* my_list = s_box[wv][box];
  __syncthreads();
  int nbx[8];
  if (use_bm) {
    // each box's list from its mask, back to front, cut at the box's last composited entry: the
    // max over its 8 lanes (quad xor 1, row_mirror = xor 15, swizzle xor 24 keep grp8_box)
    int bl8 = max(lastA, lastB);
    bl8 = max(bl8, dpp_row_i<0xB1>(bl8));   // quad_perm [1,0,3,2]
    bl8 = max(bl8, dpp_row_i<0x140>(bl8));  // row_mirror
    bl8 = max(bl8, __builtin_amdgcn_ds_swizzle(bl8, (0x18 << 10) | 0x1F));   // lane ^ 24 in 32
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      // box b's lanes: bit 5 = b >> 2, parity(bits 2,3,4) = (b >> 1) & 1, parity(bits 1,3,4) = b & 1
      const int lim = min(sn - 1, __builtin_amdgcn_readlane(bl8, 32 * (b >> 2) + 4 * ((b >> 1) & 1) + 2 * (b & 1)) - b0);
      const unsigned long long mlo = lim < 0 ? 0ull : lim >= 63 ? ~0ull : (2ull << lim) - 1ull;
      const unsigned long long mhi = lim < 64 ? 0ull : lim >= 127 ? ~0ull : (2ull << (lim - 64)) - 1ull;
      const unsigned long long lo = (((unsigned long long)bm[b].y << 32) | bm[b].x) & mlo;
      const unsigned long long hi = (((unsigned long long)bm[b].w << 32) | bm[b].z) & mhi;
      const int nhi = __popcll(hi);
      nbx[b] = nhi + __popcll(lo);
      unsigned char* const bl = s_box[wv][b];
      if ((hi >> lane) & 1ull) bl[grouped_slot(__popcll((hi >> lane) >> 1))] = (unsigned char)(64 + lane);
      if ((lo >> lane) & 1ull) bl[grouped_slot(nhi + __popcll((lo >> lane) >> 1))] = (unsigned char)lane;
    }
  } else {
  // cull the chunk against the wave's 16x8 half-tile (exact test), survivors back to front
  int nsurv = 0;
  {
    const float x0 = (float)hx0 + 0.5f, y0 = (float)hy0 + 0.5f;
#pragma unroll
    for (int q = kChunk3 / 64 - 1; q >= 0; --q) {
      const int k = q * 64 + lane;
      const bool keep = k < sn && (b0 + k) <= wlast &&
                        cull_keep<false>(s_p[0][k], s_p[1][k], s_p[2][k], x0, x0 + 15.f, y0, y0 + 7.f);
      const unsigned long long mk = __ballot(keep);
      if (keep) {
        const unsigned long long above = lane == 63 ? 0ull : (mk >> (lane + 1));
        s_list[wv][nsurv + __popcll(above)] = (unsigned char)k;
      }
      nsurv += __popcll(mk);
    }
  }
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int b = 0; b < 8; ++b) nbx[b] = 0;
  {
    const unsigned long long below = (1ull << lane) - 1ull;
    for (int s0 = 0; s0 < nsurv; s0 += 64) {
      const int si = s0 + lane;
      const bool in = si < nsurv;
      const int k = s_list[wv][in ? si : 0];
      const float4 r0 = s_p[0][k], r1 = s_p[1][k], r2 = s_p[2][k];
#pragma unroll
      for (int b = 0; b < 8; ++b) {
        const float x0 = (float)(hx0 + 4 * (b & 3)) + 0.5f, y0 = (float)(hy0 + 4 * (b >> 2)) + 0.5f;
        const bool keep = in && cull_keep<false>(r0, r1, r2, x0, x0 + 3.f, y0, y0 + 3.f);
        const unsigned long long m = __ballot(keep);
        if (keep) s_box[wv][b][grouped_slot(nbx[b] + __popcll(m & below))] = (unsigned char)k;
        nbx[b] += __popcll(m);
      }
    }
  }
  }
  int nb = nbx[0], ngrp = nbx[0];
#pragma unroll
  for (int b = 1; b < 8; ++b) {
    nb = box == b ? nbx[b] : nb;
    ngrp = max(ngrp, nbx[b]);
  }
  const int npad = (ngrp + kGroup - 1) / kGroup * kGroup;
  for (int s = nb + pp; s < npad; s += 8) s_box[wv][box][grouped_slot(s)] = (unsigned char)kNull;
  __builtin_amdgcn_wave_barrier();
  for (int g0 = 0, gb = 0; g0 < ngrp; g0 += kGroup, gb += 8) {
    float acc[64];
    acc[63] = 0.f;
    const uint2 w8 = *reinterpret_cast<const uint2*>(my_list + gb);
    int kk[kGroup];
#pragma unroll
    for (int g = 0; g < kGroup; ++g) kk[g] = (int)(((g < 4 ? w8.x : w8.y) >> (8 * (g & 3))) & 0xFFu);
    float4 n0 = s_p[0][kk[0]], n1 = s_p[1][kk[0]], n2 = s_p[2][kk[0]];
#pragma unroll
    for (int g = 0; g < kGroup; ++g) {
      const int k = kk[g];
      const float4 p0 = n0;
      const float4 p1 = n1;
      const float4 p2 = n2;
      if (g + 1 < kGroup) {   // entry g+1's record read before entry g is evaluated (GSR_BWD_PF)
        n0 = s_p[0][kk[g + 1]];
        n1 = s_p[1][kk[g + 1]];
        n2 = s_p[2][kk[g + 1]];
      }
      walk_fence();
      const float dx = p0.x - px;
      // pixel A sets the entry's 9 sums, pixel B adds (no "0 + x" adds: k_raster2d_bwd_pair)
      float a0, a1, a2, a3, a4, a5, a6, a7, a8;
      auto pixel = [&](const bool first, float dy, int lastk, float vr, float vg, float vb, float vTa, float& T,
                       float& Sv) {
        auto add = [first](float& a, float x) { a = first ? x : a + x; };
        const float sigma = conic_sigma(p1, dx, dy);
        const float vis = gauss_exp<false>(sigma);
        const float raw = p0.z * vis;
        const float alpha = fminf(kAlphaMax, raw);
        const bool valid = (k <= lastk) & (sigma >= 0.f) & (alpha >= kAlphaThreshold);
        const float alpha_v = valid ? alpha : 0.f;
        const float ra = __builtin_amdgcn_rcpf(1.f - alpha_v);
        T *= ra;
        const float fac = alpha_v * T;
        add(a6, fac * vr);
        add(a7, fac * vg);
        add(a8, fac * vb);
        const float cv = p2.x * vr + p2.y * vg + p2.z * vb;
        const float v_al = T * cv + ra * (vTa - Sv);
        const bool unclamped = valid & (raw <= kAlphaMax);
        const float v_sig = unclamped ? -raw * v_al : 0.f;
        const float tx_ = v_sig * dx, ty_ = v_sig * dy;
        add(a0, tx_);
        add(a1, ty_);
        add(a2, tx_ * dx);
        add(a3, tx_ * dy);
        add(a4, ty_ * dy);
        add(a5, v_sig);
        Sv += fac * cv;
      };
      pixel(true, p0.y - pyA, lastkA, vrA, vgA, vbA, vTaA, TA, SvA);
      pixel(false, p0.y - pyB, lastkB, vrB, vgB, vbB, vTaB, TB, SvB);
      acc[g * kPartial + 0] = a0;
      acc[g * kPartial + 1] = a1;
      acc[g * kPartial + 2] = a2;
      acc[g * kPartial + 3] = a3;
      acc[g * kPartial + 4] = a4;
      acc[g * kPartial + 5] = a5;
      acc[g * kPartial + 6] = a6;
      acc[g * kPartial + 7] = a7;
      acc[g * kPartial + 8] = a8;
    }
    float sum[8];
    reduce_grp8(acc, sum);
#if GSR_BWD3P_HALFSTAGE
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      *reinterpret_cast<float4*>(stage_wr + wr0) =
          h == 0 ? make_float4(sum[0], sum[1], sum[2], sum[3]) : make_float4(sum[4], sum[5], sum[6], sum[7]);
      __builtin_amdgcn_wave_barrier();
      if (fown && ((lane >> 2) & 1) == h) {   // two batches of four boxes (lw_add)
#pragma unroll
        for (int hb = 0; hb < 2; ++hb) {
          int kb[4];
          float vb4[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int bx = 4 * hb + j;
            kb[j] = s_box[wv][bx][gb + fg];
            vb4[j] = stage_rd[32 * bx + (rdc ^ grp8h_swz(bx))];
          }
          lw_add(Lw, kb, vb4);
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
#else
    *reinterpret_cast<float4*>(stage_wr + wr0) = make_float4(sum[0], sum[1], sum[2], sum[3]);
    *reinterpret_cast<float4*>(stage_wr + wr1) = make_float4(sum[4], sum[5], sum[6], sum[7]);
    __builtin_amdgcn_wave_barrier();
    if (fown) {
#pragma unroll
      for (int hb = 0; hb < 2; ++hb) {
        int kb[4];
        float vb4[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int bx = 4 * hb + j;
          kb[j] = s_box[wv][bx][gb + fg];
          vb4[j] = stage_rd[64 * bx + (lane ^ grp8_swz(bx))];
        }
        lw_add(Lw, kb, vb4);
      }
    }
    __builtin_amdgcn_wave_barrier();
#endif
  }
  __syncthreads();
  if ((int)threadIdx.x < sn) {
    const int k = threadIdx.x;
    float v[kPartial];
#pragma unroll
    for (int q = 0; q < kPartial; ++q) v[q] = L[q][0][k] + L[q][1][k];
    const float4 p1 = s_p[1][k];
    const float mx = v[0], my = v[1];
    v[0] = (2.f * p1.x * mx + p1.y * my) * conic_unscale<false>();   // (records: conic times log2(e))
    v[1] = (p1.y * mx + 2.f * p1.z * my) * conic_unscale<false>();
    v[5] = -v[5] / s_p[0][k].z;
    store_partial_row(partial, use_masks ? kos_mine & kEmitIndexMask : kos_mine, v);
  }
}

#ifdef GSR_BWD_TRACE
extern "C" int gsr_debug_bwd_trace(void* buf) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_bwd_trace), &buf, sizeof(buf)) == hipSuccess ? 0 : 1;
}
#endif

__global__ void k_selftest_reduce64(float* out) {
  float v[64];
#pragma unroll
  for (int i = 0; i < 64; ++i) v[i] = (float)((threadIdx.x * 7 + i * 13) % 97) + 0.25f * (float)i;
  out[threadIdx.x] = reduce64(v);
}

// reduce_box16 on the same pattern: out[4*l + i] = lane l's i-th sum
__global__ void k_selftest_reduce_box16(float* out) {
  float v[64];
#pragma unroll
  for (int i = 0; i < 64; ++i) v[i] = (float)((threadIdx.x * 7 + i * 13) % 97) + 0.25f * (float)i;
  float s[4];
  reduce_box16(v, s);
#pragma unroll
  for (int i = 0; i < 4; ++i) out[4 * threadIdx.x + i] = s[i];
}

// reduce_grp16 / reduce_grp8 on the same pattern: out[G*l + i] = lane l's i-th sum (G = 4 / 8),
// then per lane {walk box, position in it, output box, output slot} as floats at out[64 G + 4 l]
template <int G>
__global__ void k_selftest_reduce_grp(float* out) {
  float v[64];
#pragma unroll
  for (int i = 0; i < 64; ++i) v[i] = (float)((threadIdx.x * 7 + i * 13) % 97) + 0.25f * (float)i;
  float s[G];
  const int l = threadIdx.x;
  int meta[4];
  if constexpr (G == 4) {
    reduce_grp16(v, s);
    meta[0] = b128_group(l); meta[1] = grp16_pos(l); meta[2] = grp16_out_box(l); meta[3] = grp16_slot(l);
  } else {
    reduce_grp8(v, s);
    meta[0] = grp8_box(l); meta[1] = grp8_pos(l); meta[2] = grp8_out_box(l); meta[3] = grp8_slot(l);
  }
#pragma unroll
  for (int i = 0; i < G; ++i) out[G * l + i] = s[i];
#pragma unroll
  for (int i = 0; i < 4; ++i) out[64 * G + 4 * l + i] = (float)meta[i];
}

}  // namespace gsr

using namespace gsr;

extern "C" {

// Self-test of the b128-group-aligned box reductions (reduce_grp16 / reduce_grp8): see gsr.h.
int gsr_selftest_reduce_grp(float* out, int box_lanes, void* stream) {
  GSR_REQUIRE(box_lanes == 16 || box_lanes == 8, "gsr_selftest_reduce_grp: box_lanes must be 16 or 8, got %d",
              box_lanes);
  if (box_lanes == 16)
    hipLaunchKernelGGL(k_selftest_reduce_grp<4>, dim3(1), dim3(64), 0, (hipStream_t)stream, out);
  else
    hipLaunchKernelGGL(k_selftest_reduce_grp<8>, dim3(1), dim3(64), 0, (hipStream_t)stream, out);
  GSR_LAUNCH_CHECK("k_selftest_reduce_grp");
  return GSR_OK;
}


// Self-test of the transposed wave reduction: out[l] = sum over lanes of v_lane[l] for the
// pattern v_lane[i] = ((lane*7 + i*13) % 97) + i/4 (checked on the host by tests/).
int gsr_selftest_reduce64(float* out, void* stream) {
  hipLaunchKernelGGL(k_selftest_reduce64, dim3(1), dim3(64), 0, (hipStream_t)stream, out);
  GSR_LAUNCH_CHECK("k_selftest_reduce64");
  return GSR_OK;
}

// Self-test of the per-box reduction (the raster backward's): out[4*l + i] = sum over the 16
// lanes l' with l' % 4 == l % 4 of v_l'[4*(l/4) + i], same pattern; out holds 256 floats.
int gsr_set_fwd_lanes(int lanes) {
  GSR_REQUIRE(lanes == 0 || lanes == 1 || lanes == 4 || lanes == 16,
              "gsr_set_fwd_lanes: lanes must be 0 (auto), 1, 4 or 16, got %d", lanes);
  gsr::g_fwd_lanes = lanes;
  return GSR_OK;
}

int gsr_set_fwd_heavy(int log2_min_len) {
  GSR_REQUIRE(log2_min_len == 0 || (log2_min_len >= 6 && log2_min_len <= 30),
              "gsr_set_fwd_heavy: log2_min_len must be 0 (off) or 6..30, got %d", log2_min_len);
  gsr::g_fwd_heavy_log2 = log2_min_len;
  return GSR_OK;
}

int gsr_set_bwd2d_parts(int target_workgroups) {
  GSR_REQUIRE(target_workgroups >= 0 && target_workgroups <= (1 << 24),
              "gsr_set_bwd2d_parts: target_workgroups must be in [0, 2^24], got %d", target_workgroups);
  gsr::g_bwd2d_part_wgs = target_workgroups;
  return GSR_OK;
}

int gsr_set_bwd_layout(int layout) {
  GSR_REQUIRE(layout >= 0 && layout <= 2, "gsr_set_bwd_layout: layout must be 0 (auto), 1 or 2, got %d", layout);
  gsr::g_bwd_layout = layout;
  return GSR_OK;
}

int gsr_selftest_reduce_box16(float* out, void* stream) {
  hipLaunchKernelGGL(k_selftest_reduce_box16, dim3(1), dim3(64), 0, (hipStream_t)stream, out);
  GSR_LAUNCH_CHECK("k_selftest_reduce_box16");
  return GSR_OK;
}

}  // extern "C"

namespace gsr {

// Layout of the raster forward.  3D: 16 lanes per pixel and 16 workgroups per tile for calls of
// at most kFwd16MaxTiles tiles (cameras x tiles: few busy tiles, the quad layout would fill
// under half of the chip's ~1 280 workgroup slots, so latency rules; config 2: 288 tiles, 36
// busy), else 4 lanes per pixel, 4 workgroups per tile (the heavy
// tiles' serial walks are a quarter as long as with one lane per pixel: config 3 raster fwd
// 112 us against 287 us for the box layout).  2D (every tile busy, no early termination, so
// throughput rules): the box layout, one lane per pixel (config 4 raster fwd 12.5 ms against
// 15.2 ms with quads).  gsr_set_fwd_lanes forces one (tests run every layout on the same
// scenes).  The rule reads the call's shape, not its busy-tile count: a capacity-bounded call
// knows only a bound on that count, and must run the layout an exact call of the same inputs
// runs (bitwise-equal results; round 4 chose by the count, which a varying Gaussian count moved
// across the threshold in one call and not in the other, tests/test_headline_mode_gpu.py).
constexpr int64_t kFwd16MaxTiles = 320;
bool lists2d_per_set(const int32_t* set_begin, int F, int C) {
  return GSR_FWD2D_PAIR && g_fwd_lanes == 0 && rows2d_per_set(set_begin, F, C);
}
// frame_parts2d: parts per tile so that the per-set backward has about gsr_set_bwd2d_parts'
// target workgroups (at most 16 parts; 1 -- the whole list per workgroup -- from that many (set,
// tile) pairs on, e.g. config 4's eight frames at the binding's 4 608).  Only with the pair
// forward's shared lists, whose lead camera writes the colour planes.
int frame_parts2d(const int32_t* set_begin, int F, int C, int T) {
  const int target = g_bwd2d_part_wgs;
  if (target <= 0 || !lists2d_per_set(set_begin, F, C)) return 1;
  const int64_t ft = std::max<int64_t>(1, (int64_t)F * T);
  return (int)std::min<int64_t>(16, std::max<int64_t>(1, (target + ft - 1) / ft));
}
static int fwd_lanes(bool is2d, int64_t CT) {
  if (g_fwd_lanes == 1 || g_fwd_lanes == 4 || (g_fwd_lanes == 16 && !is2d)) return g_fwd_lanes;
  if (is2d) return 1;
  return CT <= kFwd16MaxTiles ? 16 : 4;
}

// The heavy-tile forward's side stream and its fork / join events, one set per (host thread,
// device): created on first use (before any graph capture: a bounded call, the only kind that
// is captured, always follows an eager call of its shape).  The fork / join
// are stream-ordered event waits, so a captured forward holds the two launches as parallel
// branches of its graph.
struct FwdSide {
  hipStream_t s = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
  bool ok = false, tried = false;
};
static FwdSide* fwd_side() {
  static thread_local FwdSide sides[16];
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess || d < 0 || d >= 16) return nullptr;
  FwdSide& x = sides[d];
  if (!x.tried) {
    x.tried = true;
    // default priority: at the device's highest one a captured step's branches ran pathologically
    // (config 3 step 0.38 -> 0.60 ms; 0.41 ms at the default priority, r05 A/B)
    x.ok = hipStreamCreateWithPriority(&x.s, hipStreamNonBlocking, 0) == hipSuccess &&
           hipEventCreateWithFlags(&x.fork, hipEventDisableTiming) == hipSuccess &&
           hipEventCreateWithFlags(&x.join, hipEventDisableTiming) == hipSuccess;
    if (!x.ok) (void)hipGetLastError();
  }
  return x.ok ? &x : nullptr;
}

// Shared by the 3D and 2D entry points (2D: C = 1, index-order keys, final_T [H,W,2]).
template <bool IS2D>
static int raster_fwd(const char* who, const float* rec, const float* depth, const int32_t* sorted_ids,
                      const int32_t* kos, const int32_t* tile_offset, const int32_t* tile_order, const int32_t* chunk_base, int C,
                      int width, int height, float cut2d, const float* bg, int32_t n_busy, gsr_bin_stats* stats,
                      float* rgb, float* alpha, float* final_T, int32_t* last, int32_t* tile_end,
                      uint64_t* tile_cut, float* chunk_state, int32_t* chunk_list,
                      void* stream, const FwdLazy& lz = FwdLazy{}, int lanes = 0, bool finalize = true,
                      const Sets2D sets = Sets2D{0, nullptr, 1}, uint32_t* box_masks = nullptr) {
  GSR_REQUIRE(C >= 1 && width > 0 && height > 0, "%s: bad C=%d or image %dx%d", who, C, width, height);
  const int tw = ceil_div(width, kTile), th = ceil_div(height, kTile);
  const int64_t CT = (int64_t)C * tw * th;
  GSR_REQUIRE(CT < (1ll << 31), "%s: too many tiles", who);
  GSR_REQUIRE(n_busy >= 0 && n_busy <= CT, "%s: n_busy=%d out of [0, %lld]", who, n_busy, (long long)CT);
  // the lazy second pass covers only its (device-counted) tiles: no empty-tile fill
  // (at least one fill workgroup: with a bounded n_busy the true count may be lower)
  const int64_t n_fill = lz.rerun ? 0 : std::max<int64_t>(1, std::min<int64_t>(CT - n_busy, kFillBlocks));
  hipStream_t s = (hipStream_t)stream;
  // tile_end collects max(last) of the quadrant workgroups (atomicMax from the -1 that
  // gsr_bin_offsets wrote)
  // Dynamic-LDS padding caps the forward at 4 workgroups per CU (measured: 4 and 5 per CU
  // beat 6, whose extra tiles in flight spill each XCD's L2; 3 starves the CU).
  // 3D with few busy tiles (a single small view, a multi-GPU rank's share): 16 lanes per pixel,
  // 16 workgroups per tile -- a quarter of the serial walk per wave, for a chip the quad layout
  // would leave mostly idle
  if (lanes == 0) lanes = fwd_lanes(IS2D, CT);
  if (lz.rerun && n_busy == 0) return GSR_OK;
  if (!IS2D && lanes == 16) {
    hipLaunchKernelGGL((k_raster_fwd<false, 16>), dim3((unsigned)(busy_grid<16>(n_busy) + n_fill)),
                       dim3(kRasterThreads), kFwdLdsPad, s, (const Splat*)rec, sorted_ids, kos, tile_offset, tile_order,
                       width, height, tw, th, bg, rgb, alpha, final_T, last, tile_end, (float4*)chunk_state,
                       chunk_base, (int)n_busy, CT, tile_cut, cut2d, lz, stats, sets);
  } else if (lanes == 4) {
    // 3D: the heavy tiles (lists >= stats->heavy_min_len) on the side stream in the 8-wave layout,
    // the rest here -- with the automatic layout only (a layout forced by gsr_set_fwd_lanes is every
    // tile's).  A first pass finds them among the first kFwdHeavyMax busy tiles; a lazy re-render
    // (lz.rerun) anywhere in its list of n_busy tiles, the same tiles as the pass over a full sort.
    FwdSide* side = !IS2D && g_fwd_lanes == 0 && g_fwd_heavy_log2 > 0 && n_busy > 0 ? fwd_side() : nullptr;
    int part = 0;
    if (side != nullptr && hipEventRecord(side->fork, s) == hipSuccess &&
        hipStreamWaitEvent(side->s, side->fork, 0) == hipSuccess) {
      hipStream_t hs = side->s;
      const int nh = lz.rerun ? (int)n_busy : std::min<int>(n_busy, kFwdHeavyMax);
      hipLaunchKernelGGL((k_raster_fwd<false, 8, 8>), dim3((unsigned)busy_grid<8, 8>(nh)), dim3(512), 0, hs,
                         (const Splat*)rec, sorted_ids, kos, tile_offset, tile_order, width, height, tw, th, bg, rgb,
                         alpha, final_T, last, tile_end, (float4*)chunk_state, chunk_base, nh, CT, tile_cut, cut2d,
                         lz, stats, sets, 2);
      GSR_LAUNCH_CHECK("k_raster_fwd<heavy>");
      part = 1;
    }
    hipLaunchKernelGGL((k_raster_fwd<IS2D, 4>), dim3((unsigned)(busy_grid<4>(n_busy) + n_fill)),
                       dim3(kRasterThreads), IS2D ? kFwdLdsPad2D : kFwdLdsPad, s, (const Splat*)rec, sorted_ids, kos,
                       tile_offset, tile_order, width, height, tw, th, bg, rgb, alpha, final_T, last, tile_end,
                       (float4*)chunk_state, chunk_base, (int)n_busy, CT, tile_cut, cut2d, lz, stats, sets, part,
                       part == 0 && GSR_BOXM ? reinterpret_cast<uint4*>(box_masks) : nullptr);
    if (part) {
      GSR_LAUNCH_CHECK(who);
      GSR_REQUIRE(hipEventRecord(side->join, side->s) == hipSuccess && hipStreamWaitEvent(s, side->join, 0) == hipSuccess,
                  "%s: joining the heavy-tile stream failed", who);
    }
  } else if (IS2D && GSR_FWD2D_PAIR) {
    // 2D: every tile in the XCD-aware sweep, two pixels per lane
    hipLaunchKernelGGL(k_raster2d_fwd_pair, dim3((unsigned)sweep_grid2d(CT)), dim3(128), 0, s, (const Splat*)rec,
                       sorted_ids, tile_offset, width, height, tw, th, bg, rgb, alpha, final_T, last, tile_end,
                       (float*)chunk_state, chunk_base, CT, cut2d, stats, sets,
                       lists2d_per_set(sets.begin, sets.F, C) ? 1 : 0,
                       frame_parts2d(sets.begin, sets.F, C, tw * th) > 1 ? 1 : 0);
  } else {
    // 2D: every tile in the XCD-aware sweep (no separate empty-tile fill)
    const int64_t grid = IS2D ? (int64_t)sweep_grid2d(CT) : ((n_busy + 7) & ~7) + n_fill;
    hipLaunchKernelGGL((k_raster_fwd_box<IS2D>), dim3((unsigned)grid),
                       dim3(kRasterThreads), 0, s, (const Splat*)rec, sorted_ids, kos, tile_offset, tile_order, width,
                       height, tw, th, bg, rgb, alpha, final_T, last, tile_end, (float4*)chunk_state, chunk_base,
                       (int)n_busy, CT, tile_cut, cut2d, lz, stats, sets);
  }
  GSR_LAUNCH_CHECK(who);
  // no chunk list: a forward with no backward to follow (no records, no finalize).  2D: one unit
  // per sweep slot, written even with no busy tile (the backward's grid is the sweep's)
  if (finalize && (n_busy > 0 || IS2D) && chunk_list != nullptr) {
    const int64_t fgrid = IS2D ? (int64_t)sweep_grid2d(CT) : (int64_t)n_busy;
    hipLaunchKernelGGL(k_raster_finalize, dim3((unsigned)ceil_div(fgrid, (int64_t)kRasterThreads)), dim3(kRasterThreads), 0, s,
                       depth, sorted_ids, tile_offset, tile_order, (int)n_busy, chunk_base, tile_end,
                       tile_cut, stats, chunk_list, IS2D ? GSR_ORDER_INDEX : GSR_ORDER_DEPTH, IS2D ? 1 : 0, CT,
                       tw * th, sets);
  }
  GSR_LAUNCH_CHECK("k_raster_finalize");
  return GSR_OK;
}

// compute units of the current device (cached per process: one device type per box)
static int device_cus() {
  static int n = 0;
  if (n <= 0) {
    int d = 0, v = 0;
    if (hipGetDevice(&d) == hipSuccess && hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, d) == hipSuccess && v > 0)
      n = v;
    else
      n = 256;
  }
  return n;
}

// 3D chunk backward layout (gsr_set_bwd_layout): 1 = k_raster_bwd (4 waves, one pixel per
// lane), 2 = k_raster_bwd_pair3d, 0 = automatic by the call's tile count (above)
static bool bwd3d_pair(int64_t tiles) {
  if (g_bwd_layout != 0) return g_bwd_layout == 2;
  return tiles >= (int64_t)kBwdPairTilesPerCU * device_cus();
}

template <bool LOSS, bool IS2D>
static int raster_bwd(const char* who, const float* rec, const int32_t* sorted_ids, const int32_t* tile_offset,
                      const int32_t* tile_end, const int32_t* chunk_base,
                      const float* chunk_state, const int32_t* chunk_list, gsr_bin_stats* stats, int32_t n_chunks,
                      int32_t chunk_entries, int C, int width, int height, float cut2d, const float* bg,
                      const float* final_T, const int32_t* last, const float* v_rgb, const float* v_alpha,
                      const gsr_loss_terms& lt, const int32_t* k_of_s, float* partial, void* stream,
                      const Sets2D sets = Sets2D{0, nullptr, 1}, const uint32_t* box_masks = nullptr) {
  GSR_REQUIRE(C >= 1 && width > 0 && height > 0, "%s: bad C=%d or image %dx%d", who, C, width, height);
  GSR_REQUIRE(n_chunks >= 0, "%s: bad n_chunks", who);
  GSR_REQUIRE(chunk_entries == 0 || (chunk_entries >= kChunk3 && (chunk_entries & (chunk_entries - 1)) == 0),
              "%s: chunk_entries %d is not 0 or a power of two >= %d", who, chunk_entries, kChunk3);
  const int tw = ceil_div(width, kTile), th = ceil_div(height, kTile);
  if (n_chunks == 0 && !IS2D) return GSR_OK;
  // n_chunks bounds the forward's active-chunk count (stats->n_active, device-side)
  if constexpr (IS2D) {   // 2D: one unit per slot of the sweep (k_raster_finalize), n_chunks unused
    (void)tile_offset;
    (void)tile_end;
    (void)chunk_base;
    (void)lt;
    const int64_t CT = (int64_t)C * tw * th;
    if (rows2d_per_set(sets.begin, sets.F, C)) {
      // cameras per pass: the set size (its mean over the call's sets), rounded up to 2, 4, 6, 8
      const int g = (C + sets.F - 1) / sets.F;
      const int parts = frame_parts2d(sets.begin, sets.F, C, tw * th);   // (the forward's rule: its colour planes)
      const int64_t FTP = (int64_t)sets.F * tw * th * parts;
      GSR_REQUIRE(8 * ((FTP + 7) / 8) < (1ll << 31), "%s: too many (set, tile, part) workgroups", who);
#define GSR_LAUNCH_FRAME(GBV)                                                                                       \
  hipLaunchKernelGGL(k_raster2d_bwd_frame<GBV>, dim3((unsigned)(8 * ((FTP + 7) / 8))), dim3(128), 0,                  \
                     (hipStream_t)stream, (const Splat*)rec, sorted_ids, chunk_state, width, height, tw, th, bg,      \
                     final_T, last, v_rgb, v_alpha, partial, tile_offset, tile_end, chunk_base, stats, k_of_s, cut2d, \
                     sets, parts)
      if (g <= 2)
        GSR_LAUNCH_FRAME(2);
      else if (g <= 4)
        GSR_LAUNCH_FRAME(4);
      else if (g <= 6)
        GSR_LAUNCH_FRAME(6);
      else
        GSR_LAUNCH_FRAME(8);
#undef GSR_LAUNCH_FRAME
    } else if (GSR_BWD2D_PAIR)
      hipLaunchKernelGGL(k_raster2d_bwd_pair, dim3((unsigned)sweep_grid2d(CT)), dim3(128), 0,
                         (hipStream_t)stream, (const Splat*)rec, sorted_ids, chunk_state, width, height, tw, th, bg,
                         final_T, last, v_rgb, v_alpha, partial, chunk_list, stats, k_of_s, cut2d, sets);
    else
      hipLaunchKernelGGL(k_raster2d_bwd_tile, dim3((unsigned)sweep_grid2d(CT)), dim3(kRasterThreads), 0,
                         (hipStream_t)stream, (const Splat*)rec, sorted_ids, chunk_state, width, height, tw, th, bg,
                         final_T, last, v_rgb, v_alpha, partial, chunk_list, stats, k_of_s, cut2d, sets);
  } else if (!LOSS && chunk_entries <= kChunk3 && bwd3d_pair((int64_t)C * tw * th)) {
    hipLaunchKernelGGL(k_raster_bwd_pair3d, dim3(n_chunks), dim3(128), 0, (hipStream_t)stream, (const Splat*)rec,
                       sorted_ids, (const float4*)chunk_state, width, height, tw, th, bg, final_T, last, v_rgb,
                       v_alpha, partial, chunk_list, stats, k_of_s, reinterpret_cast<const uint4*>(box_masks));
  } else if (chunk_entries > kChunk3)
    hipLaunchKernelGGL((k_raster_bwd<LOSS, IS2D, true>), dim3(n_chunks), dim3(kRasterThreads), 0, (hipStream_t)stream,
                       (const Splat*)rec, sorted_ids, tile_offset, tile_end, chunk_base,
                       (const float4*)chunk_state, width, height, tw, th, bg, final_T, last, v_rgb, v_alpha, partial,
                       chunk_list, stats, k_of_s, lt, C, cut2d);
  else
    hipLaunchKernelGGL((k_raster_bwd<LOSS, IS2D, false>), dim3(n_chunks), dim3(kRasterThreads), 0, (hipStream_t)stream,
                       (const Splat*)rec, sorted_ids, tile_offset, tile_end, chunk_base,
                       (const float4*)chunk_state, width, height, tw, th, bg, final_T, last, v_rgb, v_alpha, partial,
                       chunk_list, stats, k_of_s, lt, C, cut2d, reinterpret_cast<const uint4*>(box_masks));
  GSR_LAUNCH_CHECK(who);
  return GSR_OK;
}

}  // namespace gsr

extern "C" {

int gsr3d_raster_fwd(const float* rec, const float* depth, const int32_t* sorted_ids, const int32_t* k_of_s,
                     const int32_t* tile_offset,
                     const int32_t* tile_order, const int32_t* chunk_base, int C, int width, int height,
                     const float* bg, int32_t n_busy, gsr_bin_stats* stats, float* rgb, float* alpha,
                     float* final_T, int32_t* last, int32_t* tile_end, uint64_t* tile_cut, float* chunk_state,
                     int32_t* chunk_list, uint32_t* box_masks, void* stream) {
  return raster_fwd<false>("gsr3d_raster_fwd", rec, depth, sorted_ids, k_of_s, tile_offset, tile_order, chunk_base, C, width,
                           height, 0.f, bg, n_busy, stats, rgb, alpha, final_T, last, tile_end, tile_cut,
                           chunk_state, chunk_list, stream, FwdLazy{}, 0, true, Sets2D{0, nullptr, 1}, box_masks);
}

int gsr3d_raster_fwd_lazy(const float* rec, const float* depth, int32_t* sorted_ids, const int32_t* tile_offset,
                          const int32_t* tile_order, const int32_t* chunk_base, int C, int width, int height,
                          const float* bg, int32_t n_busy, gsr_bin_stats* stats, float* rgb, float* alpha,
                          float* final_T, int32_t* last, int32_t* tile_end, uint64_t* tile_cut, float* chunk_state,
                          int32_t* chunk_list, int32_t* lazy, int32_t n_lazy_max, int32_t max_seg,
                          void* sort_workspace, size_t sort_workspace_bytes, int32_t* k_of_s, uint32_t* box_masks,
                          void* stream) {
  GSR_REQUIRE(lazy != nullptr && sort_workspace != nullptr, "gsr3d_raster_fwd_lazy: missing workspace");
  GSR_REQUIRE(n_lazy_max >= 0 && n_lazy_max <= n_busy, "gsr3d_raster_fwd_lazy: bad n_lazy_max %d", n_lazy_max);
  const int64_t CT = (int64_t)C * ceil_div(width, kTile) * ceil_div(height, kTile);
  const int lanes = fwd_lanes(false, CT);
  // pass 1: every tile walks its sorted prefix; tiles that reach its end are listed
  const FwdLazy l1{lazy, lazy + CT, lazy + 2 * CT, lazy + 3 * CT, 0};
  int rc = raster_fwd<false>("gsr3d_raster_fwd_lazy", rec, depth, sorted_ids, k_of_s,
                             tile_offset, tile_order, chunk_base, C,
                             width, height, 0.f, bg, n_busy, stats, rgb, alpha, final_T, last, tile_end, tile_cut,
                             chunk_state, chunk_list, stream, l1, lanes, false, Sets2D{0, nullptr, 1}, box_masks);
  if (rc != GSR_OK) return rc;
  // the listed tiles sorted whole, then rendered again from scratch (same layout)
  rc = bin_sort_rest(tile_offset, CT, max_seg, n_lazy_max, sort_workspace, sort_workspace_bytes, lazy, tile_end,
                     sorted_ids, k_of_s, stats, (hipStream_t)stream);
  if (rc != GSR_OK) return rc;
  const FwdLazy l2{lazy, lazy + CT, lazy + 2 * CT, lazy + 3 * CT, 1};
  rc = raster_fwd<false>("gsr3d_raster_fwd_lazy", rec, depth, sorted_ids, k_of_s,
                         tile_offset, tile_order, chunk_base, C,
                         width, height, 0.f, bg, n_lazy_max, stats, rgb, alpha, final_T, last, tile_end, tile_cut,
                         chunk_state, chunk_list, stream, l2, lanes, false, Sets2D{0, nullptr, 1}, box_masks);
  if (rc != GSR_OK) return rc;
  if (n_busy > 0 && chunk_list != nullptr) {
    hipLaunchKernelGGL(k_raster_finalize, dim3(ceil_div(n_busy, kRasterThreads)), dim3(kRasterThreads), 0,
                       (hipStream_t)stream, depth, sorted_ids, tile_offset, tile_order, (int)n_busy, chunk_base,
                       tile_end, tile_cut, stats, chunk_list, GSR_ORDER_DEPTH, 0, CT, 0, Sets2D{0, nullptr, 1});
    GSR_LAUNCH_CHECK("k_raster_finalize");
  }
  return GSR_OK;
}

int gsr3d_raster_bwd(const float* rec, const int32_t* sorted_ids, const int32_t* tile_offset,
                     const int32_t* tile_end, const int32_t* chunk_base,
                     const float* chunk_state, const int32_t* chunk_list, gsr_bin_stats* stats, int32_t n_chunks,
                     int32_t chunk_entries, int C, int width, int height, const float* bg, const float* final_T,
                     const int32_t* last, const float* v_rgb, const float* v_alpha, const int32_t* k_of_s,
                     float* partial, const uint32_t* box_masks, void* stream) {
  const gsr_loss_terms none{};
  return raster_bwd<false, false>("gsr3d_raster_bwd", rec, sorted_ids, tile_offset, tile_end, chunk_base,
                                  chunk_state, chunk_list, stats, n_chunks, chunk_entries, C, width, height, 0.f, bg,
                                  final_T, last, v_rgb, v_alpha, none, k_of_s, partial, stream, Sets2D{0, nullptr, 1},
                                  box_masks);
}

int gsr3d_raster_bwd_loss(const float* rec, const int32_t* sorted_ids, const int32_t* tile_offset,
                          const int32_t* tile_end, const int32_t* chunk_base,
                          const float* chunk_state, const int32_t* chunk_list, gsr_bin_stats* stats,
                          int32_t n_chunks, int32_t chunk_entries, int C, int width, int height, const float* bg,
                          const float* final_T, const int32_t* last, const gsr_loss_terms* loss,
                          const int32_t* k_of_s, float* partial, const uint32_t* box_masks, void* stream) {
  GSR_REQUIRE(loss != nullptr && loss->rgb && loss->target_img && loss->target_mask && loss->sums && loss->grad_out,
              "gsr3d_raster_bwd_loss: incomplete loss terms");
  return raster_bwd<true, false>("gsr3d_raster_bwd_loss", rec, sorted_ids, tile_offset, tile_end, chunk_base,
                                 chunk_state, chunk_list, stats, n_chunks, chunk_entries, C, width, height, 0.f, bg,
                                 final_T, last, nullptr, nullptr, *loss, k_of_s, partial, stream, Sets2D{0, nullptr, 1},
                                 box_masks);
}

int gsr2d_raster_fwd(const float* rec, const int32_t* sorted_ids, const int32_t* tile_offset,
                     const int32_t* tile_order, const int32_t* chunk_base, int C, int width, int height, float eps_cut,
                     const float* bg, int32_t n_busy, gsr_bin_stats* stats, float* rgb, float* alpha,
                     float* final_T, int32_t* last, int32_t* tile_end, uint64_t* tile_cut, float* chunk_state,
                     int32_t* chunk_list, int64_t N, const int32_t* set_begin, int F, void* stream) {
  GSR_REQUIRE(eps_cut > 0.f && eps_cut < 1.f, "gsr2d_raster_fwd: eps_cut must be in (0,1)");
  GSR_REQUIRE(N >= 0 && F >= 1 && (set_begin != nullptr || F == 1), "gsr2d_raster_fwd: bad N=%lld / F=%d",
              (long long)N, F);
  return raster_fwd<true>("gsr2d_raster_fwd", rec, nullptr, sorted_ids, nullptr, tile_offset, tile_order, chunk_base, C, width,
                          height, eps_cut, bg, n_busy, stats, rgb, alpha, final_T, last, tile_end, tile_cut,
                          chunk_state, chunk_list, stream, FwdLazy{}, 0, true, Sets2D{N, set_begin, F});
}

int gsr2d_raster_bwd(const float* rec, const int32_t* sorted_ids, const int32_t* tile_offset,
                     const int32_t* tile_end, const int32_t* chunk_base,
                     const float* chunk_state, const int32_t* chunk_list, gsr_bin_stats* stats, int32_t n_chunks,
                     int32_t chunk_entries, int C, int width, int height, float eps_cut, const float* bg,
                     const float* final_T, const int32_t* last, const float* v_rgb, const float* v_alpha,
                     const int32_t* k_of_s, float* partial, int64_t N, const int32_t* set_begin, int F,
                     void* stream) {
  GSR_REQUIRE(eps_cut > 0.f && eps_cut < 1.f, "gsr2d_raster_bwd: eps_cut must be in (0,1)");
  GSR_REQUIRE(N >= 0 && F >= 1 && (set_begin != nullptr || F == 1), "gsr2d_raster_bwd: bad N=%lld / F=%d",
              (long long)N, F);
  const gsr_loss_terms none{};
  return raster_bwd<false, true>("gsr2d_raster_bwd", rec, sorted_ids, tile_offset, tile_end, chunk_base,
                                 chunk_state, chunk_list, stats, n_chunks, chunk_entries, C, width, height, eps_cut, bg,
                                 final_T, last, v_rgb, v_alpha, none, k_of_s, partial, stream, Sets2D{N, set_begin, F});
}

}  // extern "C"
