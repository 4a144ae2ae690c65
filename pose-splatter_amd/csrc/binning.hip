// (b) Tile binning: the per-tile scan, emission of (tile, key) pairs into per-tile buckets,
// and a per-tile sort of the keys in LDS.  (The per-Gaussian emission offsets are claimed by
// the projection's workgroups, project.hip alloc_offsets.)
//
// gsplat (isect_tiles + cub DeviceRadixSort over 64-bit (camera|tile|depth) keys) is
// restated as an MSD counting pass on the tile digit (the buckets come from the tile
// histogram written by projection) followed by an LDS-resident LSD radix sort of each
// bucket's (depth-bits << 32 | c*N+n) keys — the same total order a stable radix sort of
// gsplat's keys over emission order produces (ties in depth → ascending c*N+n), without a
// global multi-pass radix sort over HBM.  2D uses key = n (parameter order).
#include "gsr_common.h"

namespace gsr {

constexpr int kTopThreads = 1024;
constexpr int kScanLdsTiles = 32768;   // tile scan: counts staged in LDS up to 128 KB
constexpr int kChunkEntries = GSR_CHUNK;   // backward work unit (list entries)
#ifndef GSR_EMIT_THREADS
#define GSR_EMIT_THREADS 512
#endif
constexpr int kEmitThreads = GSR_EMIT_THREADS;
// Gaussians per emit workgroup.  (Larger workgroups claim fewer per-(workgroup, tile) slot
// ranges with global atomics, but measured slower at config 5: 438 -> 545 us.)
constexpr int kEmitPerBlock = 1024;
constexpr int kHistMaxTiles = 16384;
// Tile sorts come in two workgroup shapes: 1024 threads with LDS keys up to 16384 (128 KB;
// longer lists merge runs), or -- when every list is shorter than 4096 (the tile scan's class
// counts) -- 256 threads with 4096 keys (32 KB: four workgroups per CU, a quarter of the
// counters).
#ifndef GSR_SORT_THREADS
#define GSR_SORT_THREADS 1024
#endif
constexpr int kSortThreads = GSR_SORT_THREADS;    // 16 waves
constexpr int kSortThreadsSmall = 256;
#ifndef GSR_SORT_ROUNDS
#define GSR_SORT_ROUNDS 16
#endif
#ifndef GSR_SORT_LDS_KEYS
#define GSR_SORT_LDS_KEYS (GSR_SORT_ROUNDS * GSR_SORT_THREADS)
#endif
constexpr int kSortLdsKeys = GSR_SORT_LDS_KEYS;   // 128 KB of 64-bit keys at 1024 threads
constexpr int kSortRounds = GSR_SORT_ROUNDS;      // 64-element rounds per wave (LDS keys <= rounds x threads)
constexpr int kSortSmallKeys = 4096;

// Lazy depth order (3D, long lists): the forward reads a short depth prefix of every long list
// before all its pixels stop (config 5: at most 3 627 of the 16k-30k entries of the lists
// longer than 16 384; tools/tile_lengths.py), so those lists are MSD-partitioned by depth as
// before but only the digit buckets covering the first `prefix` entries are LDS-sorted.  A tile
// whose forward reaches the end of its sorted prefix is re-sorted whole and rendered again
// (gsr3d_raster_fwd_lazy), so every entry any kernel reads is in exact gsplat order.
// Workspace (int32): tile_sorted[CT] (end of the sorted prefix), flag[CT], list[CT], count.
struct LazyArgs {
  int32_t* tile_sorted;
  int32_t* flag;
  int32_t* list;
  int32_t* count;
  int32_t* tile_end;   // mode 2: reset to -1 for the re-rendered tiles
  int min_len;         // lists longer than this are sorted lazily
  int prefix;          // sorted prefix target (entries)
  int mode;            // 0 off; 1 first sort (lazy prefixes); 2 full sort of the flagged tiles
};
static int g_lazy_min_len = 16384;
static int g_lazy_prefix = 4096;
static int g_emit_staged = 1;   // gsr_set_emit_staged
static int g_split_sort = 1;    // gsr_set_split_sort

// ---------------------------------------------------------------- tile scan (single block)
// tile_offset[0..CT] (list starts), chunk_base[0..CT] (starts of each tile's GSR_CHUNK-entry chunks,
// for the chunk-parallel backward), the visit order (non-empty tiles longest-first in log2
// buckets, then the empty tiles in ascending order) and the stats.  Order inside a bucket only
// affects scheduling.  Also initialises tile_end to -1 (the raster forward's atomicMax
// target) and zeroes tile_cut.  Each wave owns a contiguous range of tiles and walks it in
// 64-tile rounds (coalesced loads and stores, in-wave scans); the counts are staged in LDS
// when they fit.
__device__ __forceinline__ int wave_incl_scan(int v) { return wave_incl_scan_dpp(v); }

__global__ __launch_bounds__(kTopThreads) void k_tile_scan(int32_t* __restrict__ tile_count, int64_t CT,
                                                          int32_t* __restrict__ tile_offset,
                                                          int32_t* __restrict__ chunk_base,
                                                          int32_t* __restrict__ order,
                                                          int32_t* __restrict__ tile_end,
                                                          uint64_t* __restrict__ tile_cut,
                                                          const gsr_bin_caps caps,
                                                          gsr_bin_stats* __restrict__ stats, int heavy_log2) {
  constexpr int NW = kTopThreads / 64;
  __shared__ int s_w[3][NW];
  __shared__ int s_max;
  __shared__ int s_bucket[33];
  __shared__ int s_n_busy;
  extern __shared__ int s_cnt[];   // the counts, staged with coalesced loads (CT <= kScanLdsTiles)
  const bool staged = CT <= kScanLdsTiles;
  if (staged) {
    // batches of 8 loads in flight per thread (one memory latency per batch, not per load)
    for (int64_t i0 = threadIdx.x; i0 < CT; i0 += 8 * kTopThreads) {
      int v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int64_t i = i0 + (int64_t)j * kTopThreads;
        v[j] = i < CT ? tile_count[i] : 0;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int64_t i = i0 + (int64_t)j * kTopThreads;
        if (i < CT) s_cnt[i] = v[j];
      }
    }
  }
  const int32_t* cnt = staged ? s_cnt : tile_count;
  if (threadIdx.x == 0) {
    s_max = 0;
    tile_count[CT] = 0;   // the projection's emission counter: consumed, reset for the next call
  }
  if (threadIdx.x < 33) s_bucket[threadIdx.x] = 0;
  __syncthreads();
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t R = ((CT + NW - 1) / NW + 63) & ~int64_t(63);
  const int64_t i0 = min<int64_t>(CT, R * wv), i1 = min<int64_t>(CT, i0 + R);
  // backward work units ("chunks") of 2^ushift list entries (caps.chunk_entries, checked on the host)
  const int ushift = 31 - __clz(caps.chunk_entries > 0 ? caps.chunk_entries : kChunkEntries);
  const int umask = (1 << ushift) - 1;
  // pass 1: per-wave totals, log2-length buckets, longest list
  int sc = 0, sk = 0, se = 0, mx = 0;
  for (int64_t i = i0 + lane; i < i1; i += 64) {
    const int v = cnt[i];
    sc += v;
    sk += (v + umask) >> ushift;
    se += v <= 0;   // (never negative: a corrupted count must not index past the visit order)
    mx = max(mx, v);
    if (v > 0) atomicAdd(&s_bucket[31 - __clz(v)], 1);
  }
  sc = wave_sum_i(sc);
  sk = wave_sum_i(sk);
  se = wave_sum_i(se);
  mx = wave_max_i(mx);
  if (lane == 0) {
    s_w[0][wv] = sc;
    s_w[1][wv] = sk;
    s_w[2][wv] = se;
    atomicMax(&s_max, mx);
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    // wave 0: the per-wave totals and the log2 buckets scanned across lanes (one thread walking
    // them serially was ~100 dependent LDS round trips -- the scan's latency at few tiles)
    const int l = threadIdx.x;
    const int a = l < NW ? s_w[0][l] : 0, b = l < NW ? s_w[1][l] : 0, c = l < NW ? s_w[2][l] : 0;
    const int ia = wave_incl_scan(a), ib = wave_incl_scan(b), ic = wave_incl_scan(c);
    if (l < NW) {
      s_w[0][l] = ia - a;
      s_w[1][l] = ib - b;
      s_w[2][l] = ic - c;
    }
    const int tc = __builtin_amdgcn_readlane(ia, 63), tk = __builtin_amdgcn_readlane(ib, 63),
              te = __builtin_amdgcn_readlane(ic, 63);
    // buckets longest first: lane l holds bucket 31 - l; its start = the lists in longer buckets
    const int bk = l < 32 ? s_bucket[31 - l] : 0;
    const int ex = wave_incl_scan(bk) - bk;
    if (l < 32) s_bucket[31 - l] = ex;
    // sort classes: lists >= 8192 (buckets >= 13: lanes < 19) and 4096..8191 (bucket 12: lane 19);
    // lists >= 1024 (kWaveSortKeys, buckets >= 10: lanes < 22) take one workgroup each
    const int n_big = __builtin_amdgcn_readlane(ex, 19), n_mid = __builtin_amdgcn_readlane(bk, 19),
              n_long = __builtin_amdgcn_readlane(ex, 22);
    // heavy tiles of the 3D forward (gsr_set_fwd_heavy): lists >= 2^b, i.e. buckets >= b, whose
    // count is the start of bucket b - 1 (lane 32 - b; non-decreasing in the lane), for the
    // smallest b >= k that leaves at most kFwdHeavyMax tiles (gsr_common.h): a set fixed by the
    // list lengths alone
    const unsigned long long hm = __ballot(l <= 32 - heavy_log2 && l < 32 && ex <= kFwdHeavyMax);
    const int hl = hm ? 63 - __clzll(hm) : 0;   // (lane 0: ex = 0, no heavy tile)
    const int n_heavy = heavy_log2 > 0 ? __builtin_amdgcn_readlane(ex, hl) : 0;
    const int heavy_min = n_heavy > 0 ? (1 << (32 - hl)) : 0x7fffffff;
    if (l == 0) {
      const int n_busy = (int)CT - te;
      s_n_busy = n_busy;
      stats->n_sort_big = n_big;
      stats->n_sort_mid = n_mid;
      stats->n_sort_long = n_long;
      tile_offset[CT] = tc;
      chunk_base[CT] = tk;
      stats->n_isect = tc;
      stats->max_seg = s_max;
      stats->n_busy = n_busy;
      stats->n_chunks = tk;
      stats->n_active = 0;
      stats->masks = 0;   // set by an emission that stores quadrant masks
      stats->n_heavy = n_heavy;
      stats->heavy_min_len = heavy_min;
      // bounded call: the caller sized the intersection / chunk buffers without reading I back
      int ovf = 0;
      if (caps.isect > 0 && (int64_t)tc > caps.isect) ovf |= GSR_OVF_ISECT;
      if (caps.chunks > 0 && (int64_t)tk > caps.chunks) ovf |= GSR_OVF_CHUNKS;
      stats->isect_cap = caps.isect;
      stats->chunk_cap = caps.chunks;
      stats->overflow = ovf;
      stats->status = caps.status;
      stats->chunk_entries = 1 << ushift;
    }
  }
  __syncthreads();
  // pass 2: 64-tile rounds per wave
  int cc = s_w[0][wv], ck = s_w[1][wv], ce = s_w[2][wv];
  const int n_busy = s_n_busy;
  for (int64_t base = i0; base < i1; base += 64) {
    const int64_t i = base + lane;
    const bool in = i < i1;
    const int v = in ? cnt[i] : 0;
    const int kc = (v + umask) >> ushift;
    const int iv = wave_incl_scan(v), ik = wave_incl_scan(kc);
    const unsigned long long empty = __ballot(in && v <= 0);
    if (in) {
      tile_offset[i] = cc + iv - v;
      chunk_base[i] = ck + ik - kc;
      tile_end[i] = -1;
      tile_cut[i] = 0ull;
      if (v > 0) {
        order[atomicAdd(&s_bucket[31 - __clz(v)], 1)] = (int32_t)i;
      } else {
        const int r = __builtin_amdgcn_mbcnt_hi((uint32_t)(empty >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)empty, 0));
        order[n_busy + ce + r] = (int32_t)i;
      }
    }
    cc += __builtin_amdgcn_readlane(iv, 63);
    ck += __builtin_amdgcn_readlane(ik, 63);
    ce += __popcll(empty);
  }
}

// ---------------------------------------------------------------- emission
// Overflow bits set by the tile scan (stable while any later kernel of the call runs, so a
// workgroup's threads all read the same value); the sort kernels add GSR_OVF_BUSY / SEG / LAZY,
// which only the raster and projection backward (later launches) act on.
constexpr int kOvfCapacity = GSR_OVF_ISECT | GSR_OVF_CHUNKS;

// A bounded call over its caps emits nothing; the projection left its per-tile counts in
// tile_count, which the NEXT call's projection relies on finding zero: workgroup x = 0 of each
// camera clears that camera's counts.
__device__ __forceinline__ void emit_skip_counts(int32_t* __restrict__ tile_count, int T) {
  if (blockIdx.x != 0) return;
  int32_t* g = tile_count + (int64_t)blockIdx.y * T;
  for (int t = threadIdx.x; t < T; t += blockDim.x) g[t] = 0;
}

__global__ __launch_bounds__(kEmitThreads) void k_emit(const float* __restrict__ depth, const Splat* __restrict__ rec,
                                                      const uint2* __restrict__ rect,
                                                      const int32_t* __restrict__ isect_offset, int64_t N, int tw,
                                                      int th, int order, int use_lds,
                                                      const int32_t* __restrict__ tile_offset,
                                                      int32_t* __restrict__ tile_count, uint64_t* __restrict__ keys,
                                                      int32_t* __restrict__ k_of_slot, int per_block,
                                                      gsr_bin_stats* __restrict__ stats, int64_t cap) {
  // launched before the host has read I back (gsr_bin_emit): a workspace too small for this
  // call's I makes every workgroup leave at once, and the host emits again with a larger one.
  // A bounded call over its caps emits nothing.  (Both words load together, one branch.)
  const int ovf = stats->overflow & kOvfCapacity;
  const int64_t n_isect = stats->n_isect;
  if (ovf | (n_isect > cap)) {
    if (ovf) emit_skip_counts(tile_count, tw * th);
    return;
  }
  if (rec != nullptr && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) stats->masks |= kStatsMasks3D;
  // Slots are claimed by counting each tile's count down to zero (slot = tile start +
  // remaining count - 1): no separate cursor array, and tile_count is left zeroed.
  extern __shared__ int hist[];
  const int c = blockIdx.y;
  const int T = tw * th;
  int32_t* gcnt = tile_count + (int64_t)c * T;
  const int32_t* toff = tile_offset + (int64_t)c * T;
  const int64_t n0 = (int64_t)blockIdx.x * per_block;
  const int64_t n1 = min(N, n0 + per_block);
  if (use_lds) {
    for (int t = threadIdx.x; t < T; t += blockDim.x) hist[t] = 0;
    __syncthreads();
    for (int64_t n = n0 + threadIdx.x; n < n1; n += blockDim.x) {
      const uint2 r = rect[(int64_t)c * N + n];
      const int x0 = r.x & 0xffff, x1 = r.x >> 16, y0 = r.y & 0xffff, y1 = r.y >> 16;
      for (int ty = y0; ty < y1; ++ty)
        for (int tx = x0; tx < x1; ++tx) atomicAdd(&hist[ty * tw + tx], 1);
    }
    __syncthreads();
    // claim this workgroup's range of every tile it hits: batches of 8 returning atomics in
    // flight per thread (a strided loop waited one atomic round trip per tile)
    for (int t0 = threadIdx.x; t0 < T; t0 += 8 * kEmitThreads) {
      int v[8], base[8], got[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int t = t0 + j * kEmitThreads;
        v[j] = t < T ? hist[t] : 0;
        base[j] = t < T ? toff[t] : 0;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) got[j] = v[j] ? atomicSub(&gcnt[t0 + j * kEmitThreads], v[j]) : 0;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (v[j]) hist[t0 + j * kEmitThreads] = base[j] + got[j] - v[j];
    }
    __syncthreads();
  }
  for (int64_t n = n0 + threadIdx.x; n < n1; n += blockDim.x) {
    const int64_t cn = (int64_t)c * N + n;
    const uint2 r = rect[cn];
    const int x0 = r.x & 0xffff, x1 = r.x >> 16, y0 = r.y & 0xffff, y1 = r.y >> 16;
    if (x1 <= x0 || y1 <= y0) continue;
    const uint64_t key = sort_key(depth, cn, order);
    int k = isect_offset[cn];   // emission entries of (c,n): k = offset + rect row-major index
    Splat sp{};
    if (rec != nullptr) sp = rec[cn];
    for (int ty = y0; ty < y1; ++ty)
      for (int tx = x0; tx < x1; ++tx) {
        const int t = ty * tw + tx;
        const int slot = use_lds ? atomicAdd(&hist[t], 1) : toff[t] + atomicSub(&gcnt[t], 1) - 1;
        // 3D: the entry's quadrant mask in the top bits (gsr_common.h quad_mask)
        const int mk = rec != nullptr ? (int)((unsigned)quad_mask<false>(sp.p0, sp.p1, sp.p2, tx, ty) << kMaskShift) : 0;
        keys[slot] = key;
        k_of_slot[slot] = k++ | mk;
      }
  }
}

// Staged emission: the same slots, but each workgroup first builds its entries in LDS grouped
// by tile (local counting sort) and then writes them out with consecutive lanes on
// consecutive slots.  The direct scatter above stores every 8-byte key and 4-byte emission
// index on its own, so the runs a workgroup gives each tile (~5 entries at config 5) reach
// HBM as partial-line writes: 906 MB written per launch for 306 MB of entries
// (profiles/r02_pmc_traffic_cfg5.csv).  2048 Gaussians per workgroup make the runs longer
// (GPT = 2 per thread, 3D: ~2 entries per Gaussian).  2D Gaussians cover ~5 tiles each (config
// 4), so 2048 of them overflow the stage and fell back to the scattered writes (2.1 ms at
// config 4): index-order (2D) emission takes 1024 per workgroup (GPT = 1).
constexpr int kStageThreads = 1024;
#ifndef GSR_EMIT_GPT
#define GSR_EMIT_GPT 3   // 3D Gaussians per thread of the staged emission (2 or 3)
#endif
constexpr int kStageCap = 6144;          // staged entries (16 B each)
constexpr size_t kStageLds = (size_t)kStageCap * 16;
// cursor + offset per tile (8 B each) in what is left of the 160 KB of LDS after the stage and
// the kernel's static LDS (s_tmp: 17 ints; 256 B reserved) -- 8 160 tiles, so e.g. a 2048x1024
// view (8 192 tiles) takes the direct scatter instead of failing to launch
constexpr int kLdsBytes = 160 * 1024;
constexpr int kStageStaticLds = 256;
constexpr int kStageMaxTiles = (int)((kLdsBytes - kStageLds - kStageStaticLds) / 8);
static_assert(kStageMaxTiles >= 4096, "staged emission needs room for a 4096-tile camera");

template <int GPT>
__global__ __launch_bounds__(kStageThreads) void k_emit_staged(
    const float* __restrict__ depth, const Splat* __restrict__ rec, const uint2* __restrict__ rect,
    const int32_t* __restrict__ isect_offset,
    int64_t N, int tw, int th, int order, const int32_t* __restrict__ tile_offset, int32_t* __restrict__ tile_count,
    uint64_t* __restrict__ keys, int32_t* __restrict__ k_of_slot, gsr_bin_stats* __restrict__ stats,
    int64_t cap, int stage_cap) {
  constexpr int NT = kStageThreads;
  constexpr int kStagePer = GPT * NT;   // Gaussians per workgroup
  extern __shared__ uint64_t s_key[];   // [stage_cap]
  int32_t* s_kos = (int32_t*)(s_key + stage_cap);
  int32_t* s_slot = s_kos + stage_cap;
  int* cur = s_slot + stage_cap;        // [T] local cursor (starts at the tile's local offset)
  const int T = tw * th;
  int* delta = cur + T;                 // [T] global slot - local position
  __shared__ int s_tmp[NT / 64 + 1];
  const int c = blockIdx.y;
  int32_t* gcnt = tile_count + (int64_t)c * T;
  const int32_t* toff = tile_offset + (int64_t)c * T;
  const int64_t n0 = (int64_t)blockIdx.x * kStagePer;
  // Every load that depends on nothing is issued here, in one round trip: the stats words, the
  // camera's list range and this thread's Gaussians' rects, sort keys and emission offsets (the
  // tests below, then the keys' use after the claims, used to wait for each in turn: three
  // memory latencies on every workgroup's chain, round 6)
  const int ovf = stats->overflow & kOvfCapacity;   // see k_emit
  const int64_t n_isect = stats->n_isect;
  const int cam_first = toff[0], cam_end = toff[T];
  uint2 rr[GPT];
  uint64_t key[GPT];
  int k0[GPT];
#pragma unroll
  for (int j = 0; j < GPT; ++j) {
    const int64_t n = n0 + threadIdx.x + j * NT;
    const int64_t cn = (int64_t)c * N + (n < N ? n : 0);
    rr[j] = n < N ? rect[cn] : make_uint2(0u, 0u);
    key[j] = sort_key(depth, cn, order);
    k0[j] = isect_offset[cn];
  }
  if (ovf | (n_isect > cap)) {
    if (ovf) emit_skip_counts(tile_count, tw * th);
    return;
  }
  if (rec != nullptr && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) stats->masks |= kStatsMasks3D;
  // a camera with no entries (2D: a set's other cameras, lists2d_per_set) -- nothing to stage
  if (cam_first == cam_end) return;
  for (int t = threadIdx.x; t < T; t += NT) cur[t] = 0;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < GPT; ++j) {
    const int x0 = rr[j].x & 0xffff, x1 = rr[j].x >> 16, y0 = rr[j].y & 0xffff, y1 = rr[j].y >> 16;
    for (int ty = y0; ty < y1; ++ty)
      for (int tx = x0; tx < x1; ++tx) atomicAdd(&cur[ty * tw + tx], 1);
  }
  __syncthreads();
  // local offsets: thread-contiguous tile ranges, serial sums, one block scan
  const int tpt = (T + NT - 1) / NT;
  const int t0 = min(T, (int)threadIdx.x * tpt), t1 = min(T, t0 + tpt);
  int mine = 0;
  for (int t = t0; t < t1; ++t) mine += cur[t];
  int total;
  int run = block_exclusive_scan<NT>(mine, s_tmp, &total);
  for (int t = t0; t < t1; ++t) {
    const int v = cur[t];
    delta[t] = v;   // the count, until the claim below
    cur[t] = run;
    run += v;
  }
  __syncthreads();
  // claim the global ranges: batches of 8 returning atomics in flight per thread
  for (int b0 = threadIdx.x; b0 < T; b0 += 8 * NT) {
    int v[8], base[8], got[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int t = b0 + j * NT;
      v[j] = t < T ? delta[t] : 0;
      base[j] = t < T ? toff[t] : 0;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) got[j] = v[j] ? atomicSub(&gcnt[b0 + j * NT], v[j]) : 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int t = b0 + j * NT;
      if (t < T) delta[t] = base[j] + got[j] - v[j] - cur[t];
    }
  }
  __syncthreads();
  const bool staged = total <= stage_cap;   // uniform: else scatter directly (huge rects)
#pragma unroll
  for (int j = 0; j < GPT; ++j) {
    const int x0 = rr[j].x & 0xffff, x1 = rr[j].x >> 16, y0 = rr[j].y & 0xffff, y1 = rr[j].y >> 16;
    int k = k0[j];   // emission entries of (c,n): k = offset + rect row-major index
    // 3D: each entry's quadrant mask goes to the top bits of its emission index (quad_mask)
    Splat sp{};
    if (rec != nullptr && x1 > x0 && y1 > y0) sp = rec[(int64_t)c * N + n0 + threadIdx.x + j * NT];
    for (int ty = y0; ty < y1; ++ty)
      for (int tx = x0; tx < x1; ++tx) {
        const int t = ty * tw + tx;
        const int p = atomicAdd(&cur[t], 1);
        const int kk = (int)((unsigned)k | (rec != nullptr ? (unsigned)quad_mask<false>(sp.p0, sp.p1, sp.p2, tx, ty) << kMaskShift : 0u));
        if (staged) {
          s_key[p] = key[j];
          s_kos[p] = kk;
          s_slot[p] = delta[t] + p;
        } else {
          keys[delta[t] + p] = key[j];
          k_of_slot[delta[t] + p] = kk;
        }
        ++k;
      }
  }
  if (!staged) return;
  __syncthreads();
  for (int i = threadIdx.x; i < total; i += NT) {
    const int slot = s_slot[i];
    keys[slot] = s_key[i];
    k_of_slot[slot] = s_kos[i];
  }
}

// ---------------------------------------------------------------- per-tile sort
// Emitted keys are (sort word << 32 | c*N+n); the sort word is the depth's float bits (3D,
// depth > 0 so integer order = float order) or the index itself (2D).  In LDS each element is
// (sort word << 32 | p), p = its pre-sort position in the tile's bucket, so every lookup after
// the sort (c*N+n, and the slot → sorted-position map used by the backward) stays inside the
// bucket's own window of the key array (L2-resident) instead of gathering per-Gaussian data.
// The LDS sort is a stable LSD radix sort on the sort word, 8-bit digits, skipping digit
// positions that do not vary inside the segment; the rank within the wave comes from one
// returning LDS atomic per key (lane-ordered), so a pass is one read, one block scan of
// 16x256 counters and one scatter.  Ties on the sort word (equal depths) are then put in ascending c*N+n order by a
// bounded odd-even fix-up — the order a stable radix sort of gsplat's keys over emission
// order gives.

#ifdef GSR_SORT_TRACE
__shared__ unsigned long long s_sort_ts[8];   // per-phase wall clock of the sort (thread 0)
#define SORT_T(i) if (threadIdx.x == 0) s_sort_ts[i] = wall_clock64()
#else
#define SORT_T(i)
#endif
__device__ __forceinline__ uint32_t sort_word(uint64_t k) { return (uint32_t)(k >> 32); }
__device__ __forceinline__ uint32_t low_word(uint64_t k) { return (uint32_t)(k & 0xffffffffull); }

// Global <-> LDS staging loops, batched so that kBatch loads per thread are in flight at once
// (a plain strided loop waits one memory latency per iteration: ~10 iterations per list).
constexpr int kBatch = 8;

// A sort group: GT consecutive threads of the workgroup (whole waves) that sort one list in
// their own slice of the LDS image.  sync(): __syncthreads() when the group is the whole
// workgroup (ctr == nullptr, uniform over the workgroup), else an arrival counter in LDS -- the
// group's waves are resident together, so spinning on it cannot deadlock, and the release /
// acquire fences order every LDS access of the group around it.
template <int GT>
struct SortGroup {
  int tid;      // thread index in the group
  int* ctr;     // LDS arrival counter (zeroed before the group's first sync), or nullptr
  int phase;    // arrivals of this group's waves so far (uniform)
  __device__ __forceinline__ void sync() {
    if (ctr == nullptr) {
      __syncthreads();
      return;
    }
    phase += GT / 64;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < phase) __builtin_amdgcn_s_sleep(1);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  }
};
// the group's counters in LDS: W waves' digit counters (W x 256 ints), then 64 misc ints
// (varying bits, tie-run count and flags, the scan's wave sums, the barrier counter last)
constexpr int kGroupMisc = 64;
__host__ __device__ constexpr int group_ints(int waves) { return waves * 256 + kGroupMisc; }

// a[i] = (sort word of src[i]) << 32 | (pbase + i), i < n.  Returns this thread's OR of
// (word ^ src[0]'s word): the bits that vary inside the list, once OR-ed over the group.
// (16 loads in flight per thread: a list of up to 16 GT keys arrives in one round trip)
constexpr int kStageBatch = 16;
template <int GT>
__device__ __forceinline__ uint32_t stage_keys(const SortGroup<GT>& g, uint64_t* a, const uint64_t* __restrict__ src,
                                               int n, int pbase) {
  const uint32_t w0 = sort_word(src[0]);
  uint32_t orv = 0;
  for (int i0 = g.tid; i0 < n; i0 += kStageBatch * GT) {
    uint32_t w[kStageBatch];
#pragma unroll
    for (int j = 0; j < kStageBatch; ++j) {
      const int i = i0 + j * GT;
      w[j] = sort_word(src[i < n ? i : 0]);
    }
#pragma unroll
    for (int j = 0; j < kStageBatch; ++j) {
      const int i = i0 + j * GT;
      orv |= w[j] ^ w0;   // (a clamped duplicate of src[0] adds nothing)
      if (i < n) a[i] = ((uint64_t)w[j] << 32) | (uint64_t)(uint32_t)(pbase + i);
    }
  }
  return orv;
}

// The varying bits of the sort words: the group OR of every thread's `orv` (s_misc[0] must be
// zero on entry; it is left holding the result).  One atomic per wave.
template <int GT>
__device__ __forceinline__ uint32_t block_varying(SortGroup<GT>& g, uint32_t orv, int* s_misc) {
  orv = (uint32_t)wave_or_i((int)orv);
  if ((threadIdx.x & 63) == 0 && orv) atomicOr((unsigned*)&s_misc[0], orv);
  g.sync();
  return (uint32_t)s_misc[0];
}

// The same from keys already in LDS
template <int GT>
__device__ __forceinline__ uint32_t lds_varying(SortGroup<GT>& g, const uint64_t* a, int n, int* s_misc) {
  if (g.tid == 0) s_misc[0] = 0;
  g.sync();
  const uint32_t w0 = sort_word(a[0]);
  uint32_t orv = 0;
  for (int i = g.tid; i < n; i += GT) orv |= sort_word(a[i]) ^ w0;
  return block_varying<GT>(g, orv, s_misc);
}

// Group-wide exclusive scan of one int per thread; s_tmp holds GT/64 + 1 ints.
template <int GT>
__device__ __forceinline__ int group_exclusive_scan(SortGroup<GT>& g, int v, int* s_tmp, int* total) {
  const int lane = threadIdx.x & 63;
  const int w = g.tid >> 6;
  const int x = wave_incl_scan_dpp(v);
  if (lane == 63) s_tmp[w] = x;
  g.sync();
  if (g.tid < 64) {   // the group's first wave scans the wave totals (lane k: wave k)
    const int t = lane < GT / 64 ? s_tmp[lane] : 0;
    const int it = wave_incl_scan_dpp(t);
    if (lane < GT / 64) s_tmp[lane] = it - t;
    if (lane == GT / 64 - 1) s_tmp[GT / 64] = it;
  }
  g.sync();
  const int res = x - v + s_tmp[w];
  *total = s_tmp[GT / 64];
  g.sync();
  return res;
}

// a[i] = src[i], i < n
template <int NT>
__device__ __forceinline__ void copy_keys(uint64_t* a, const uint64_t* __restrict__ src, int n, int tid = -1) {
  for (int i0 = tid >= 0 ? tid : (int)threadIdx.x; i0 < n; i0 += kBatch * NT) {
    uint64_t w[kBatch];
#pragma unroll
    for (int j = 0; j < kBatch; ++j) {
      const int i = i0 + j * NT;
      w[j] = src[i < n ? i : 0];
    }
#pragma unroll
    for (int j = 0; j < kBatch; ++j) {
      const int i = i0 + j * NT;
      if (i < n) a[i] = w[j];
    }
  }
}

// sorted element s (word << 32 | p, p indexing the bucket): ids[s] = c*N+n of key seg[p],
// kos[s] = kslot[p] (its emission index)
template <int NT>
__device__ __forceinline__ void write_sorted(const uint64_t* a, int n, const uint64_t* __restrict__ seg,
                                             const int32_t* __restrict__ kslot, int32_t* __restrict__ ids,
                                             int32_t* __restrict__ kos) {
  for (int s0 = threadIdx.x; s0 < n; s0 += kBatch * NT) {
    uint32_t p[kBatch];
    int32_t id[kBatch], ko[kBatch];
#pragma unroll
    for (int j = 0; j < kBatch; ++j) {
      const int s = s0 + j * NT;
      p[j] = s < n ? low_word(a[s]) : 0u;
    }
#pragma unroll
    for (int j = 0; j < kBatch; ++j) {
      id[j] = (int32_t)low_word(seg[p[j]]);
      ko[j] = kslot[p[j]];
    }
#pragma unroll
    for (int j = 0; j < kBatch; ++j) {
      const int s = s0 + j * NT;
      if (s < n) {
        ids[s] = id[j];
        kos[s] = ko[j];
      }
    }
  }
}

// write_sorted for a list held whole in LDS (p indexes a, capacity >= n 64-bit slots, n <= 16
// GT): the sorted p's move to registers, the list's ids (low words of seg) and emission indices
// are then loaded COALESCED into the same LDS (as two n-word arrays), and each sorted entry
// reads its pair there.  A long list's write was two random global gathers per key, all issued
// by the one workgroup that owns the list (~17 us of a 42 us sort at 11 880 keys).
template <int GT>
__device__ __forceinline__ void write_sorted_lds(SortGroup<GT>& g, uint64_t* a, int n,
                                                 const uint64_t* __restrict__ seg, const int32_t* __restrict__ kslot,
                                                 int32_t* __restrict__ ids, int32_t* __restrict__ kos) {
  constexpr int kMaxPer = 16;   // every caller's slice holds at most 16 GT keys
  uint16_t pv[kMaxPer];
#pragma unroll
  for (int j = 0; j < kMaxPer; ++j) {
    const int s = g.tid + j * GT;
    pv[j] = s < n ? (uint16_t)low_word(a[s]) : (uint16_t)0;
  }
  g.sync();
  uint32_t* xid = reinterpret_cast<uint32_t*>(a);
  int32_t* xk = reinterpret_cast<int32_t*>(a) + n;
  for (int i0 = g.tid; i0 < n; i0 += kMaxPer * GT) {   // one round trip
    uint32_t id[kMaxPer];
    int32_t ko[kMaxPer];
#pragma unroll
    for (int j = 0; j < kMaxPer; ++j) {
      const int i = i0 + j * GT;
      id[j] = low_word(seg[i < n ? i : 0]);
      ko[j] = kslot[i < n ? i : 0];
    }
#pragma unroll
    for (int j = 0; j < kMaxPer; ++j) {
      const int i = i0 + j * GT;
      if (i < n) {
        xid[i] = id[j];
        xk[i] = ko[j];
      }
    }
  }
  g.sync();
#pragma unroll
  for (int j = 0; j < kMaxPer; ++j) {
    const int s = g.tid + j * GT;
    if (s < n) {
      ids[s] = (int32_t)xid[pv[j]];
      kos[s] = xk[pv[j]];
    }
  }
}

// a: n <= 16*GT elements (word << 32 | p) in LDS; seg: the bucket's original keys (tie-break
// by their low word); s_hist: the group's group_ints(GT/64) counters (the misc ints follow the
// digit counters).  varying: the bits in which the sort words differ (block_varying /
// lds_varying).
template <int GT>
__device__ __forceinline__ void lds_radix_sort(SortGroup<GT>& g, uint64_t* a, int n, int* s_hist,
                                               const uint64_t* __restrict__ seg, uint32_t varying) {
  constexpr int kSortWaves = GT / 64;
  constexpr int kWaveBits = kSortWaves == 16 ? 4 : (kSortWaves == 8 ? 3 : 2);
  static_assert(kSortWaves == 16 || kSortWaves == 8 || kSortWaves == 4, "16, 8 or 4 waves");
  const int wv = g.tid >> 6, lane = threadIdx.x & 63;
  int* s_misc = s_hist + kSortWaves * 256;
  if (g.tid == 0) {   // tie-run count and long-run flag (the passes' barriers order these)
    s_misc[1] = 0;
    s_misc[2] = 0;
  }
  SORT_T(1);
  const int per_wave = (((n + kSortWaves - 1) / kSortWaves) + 63) & ~63;
  const int rounds = per_wave >> 6;
  for (int shift = 0; shift < 32; shift += 8) {
    if (((varying >> shift) & 0xFFu) == 0u) continue;
    for (int i = lane; i < 256; i += 64) s_hist[wv * 256 + i] = 0;
    __builtin_amdgcn_wave_barrier();
    uint64_t el[kSortRounds];
    int rk[kSortRounds];
    // Stable rank inside the wave's digit bucket from ONE returning LDS atomic per key: the
    // LDS serialises same-address atomics of one wave instruction in lane order (measured on
    // MI355X; gsr_selftest_lds_order checks it), and rounds run in order, so the returned
    // count is the key's position among the wave's equal digits.
#pragma unroll
    for (int r = 0; r < kSortRounds; ++r) {
      if (r < rounds) {
        const int idx = wv * per_wave + r * 64 + lane;
        const bool valid = idx < n;
        el[r] = valid ? a[idx] : 0ull;
        const uint32_t d = (sort_word(el[r]) >> shift) & 0xFFu;
        rk[r] = valid ? (int)((d << 23) | (uint32_t)atomicAdd(&s_hist[wv * 256 + d], 1)) : -1;   // pos < 2^23
      }
    }
    g.sync();
    // digit-major, wave-minor exclusive scan of the W x 256 counters: 4 per thread
    {
      int v[4];
      int sum = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = g.tid * 4 + j;
        v[j] = s_hist[(c & (kSortWaves - 1)) * 256 + (c >> kWaveBits)];
        sum += v[j];
      }
      int total;
      int run = group_exclusive_scan<GT>(g, sum, s_misc + 8, &total);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = g.tid * 4 + j;
        s_hist[(c & (kSortWaves - 1)) * 256 + (c >> kWaveBits)] = run;
        run += v[j];
      }
    }
    g.sync();
#pragma unroll
    for (int r = 0; r < kSortRounds; ++r) {
      if (r < rounds && rk[r] >= 0) {
        const int d = rk[r] >> 23;
        a[s_hist[wv * 256 + d] + (rk[r] & 0x7FFFFF)] = el[r];
      }
    }
    g.sync();
    SORT_T(2 + shift / 8);
  }
  SORT_T(6);
  // equal sort words: order by c*N+n.  One pass lists the runs of equal words (rare: a few per
  // long list), then one thread per run insertion-sorts it by the keys' low words -- one
  // round of gathers for all runs (odd-even transposition until nothing moved needed ~4
  // barrier-separated passes, each waiting on a gather whenever the list had a tie).
  int* s_runs = s_hist;   // the counters are free now
  constexpr int kMaxRuns = kSortWaves * 256;
  constexpr int kMaxRunLen = 32;
  for (int i = g.tid; i < n; i += GT) {
    const uint32_t w = sort_word(a[i]);
    const bool starts = i + 1 < n && sort_word(a[i + 1]) == w && (i == 0 || sort_word(a[i - 1]) != w);
    if (starts) {
      const int r = atomicAdd(&s_misc[1], 1);
      if (r < kMaxRuns) s_runs[r] = i;
    }
  }
  g.sync();
  const int n_runs = s_misc[1];
  if (n_runs <= kMaxRuns) {
    for (int r = g.tid; r < n_runs; r += GT) {
      const int i0 = s_runs[r];
      const uint32_t w = sort_word(a[i0]);
      int i1 = i0 + 1;
      while (i1 < n && i1 - i0 <= kMaxRunLen && sort_word(a[i1]) == w) ++i1;
      if (i1 - i0 > kMaxRunLen) {   // a long run (degenerate depths): the odd-even passes below
        s_misc[2] = 1;
        continue;
      }
      for (int i = i0 + 1; i < i1; ++i) {   // insertion sort of a[i0..i1) by low_word(seg[p])
        const uint64_t x = a[i];
        const uint32_t kx = low_word(seg[low_word(x)]);
        int j = i - 1;
        while (j >= i0 && low_word(seg[low_word(a[j])]) > kx) {
          a[j + 1] = a[j];
          --j;
        }
        a[j + 1] = x;
      }
    }
    g.sync();
    SORT_T(7);
    if (s_misc[2] == 0) return;
  }
  // (more runs than the list can hold, or a run too long for one thread: odd-even passes
  // until nothing moves; s_misc[3] collects "moved" over the group)
  while (true) {
    bool moved = false;
    if (g.tid == 0) s_misc[3] = 0;
#pragma unroll
    for (int ph = 0; ph < 2; ++ph) {
      for (int i = 2 * g.tid + ph; i + 1 < n; i += 2 * GT) {
        const uint64_t x = a[i], y = a[i + 1];
        if (sort_word(x) == sort_word(y) && low_word(seg[low_word(x)]) > low_word(seg[low_word(y)])) {
          a[i] = y;
          a[i + 1] = x;
          moved = true;
        }
      }
      g.sync();
    }
    if (__ballot(moved) != 0ull && lane == 0) atomicOr(&s_misc[3], 1);
    g.sync();
    const bool any = s_misc[3] != 0;
    g.sync();
    if (!any) break;
  }
  SORT_T(7);
}

__device__ __forceinline__ int next_pow2(int v) {
  int p = 1;
  while (p < v) p <<= 1;
  return p;
}

// Merge two sorted runs of unique keys (with payloads) into out (block-cooperative, per-element
// rank by binary search in the other run).
__device__ __forceinline__ void merge_runs(const uint64_t* __restrict__ a, const int32_t* __restrict__ pa, int na,
                           const uint64_t* __restrict__ b, const int32_t* __restrict__ pb, int nb,
                           uint64_t* __restrict__ out, int32_t* __restrict__ pout) {
  for (int i = threadIdx.x; i < na; i += blockDim.x) {
    const uint64_t k = a[i];
    int lo = 0, hi = nb;   // count of b < k
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (b[mid] < k) lo = mid + 1; else hi = mid;
    }
    out[i + lo] = k;
    pout[i + lo] = pa[i];
  }
  for (int i = threadIdx.x; i < nb; i += blockDim.x) {
    const uint64_t k = b[i];
    int lo = 0, hi = na;   // count of a <= k
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (a[mid] <= k) lo = mid + 1; else hi = mid;
    }
    out[i + lo] = k;
    pout[i + lo] = pb[i];
  }
}

// Short lists (< kWaveSortKeys entries) are sorted by ONE wave each, kSortWaves of them per
// workgroup side by side (the tile scan counts the longer lists: stats->n_sort_long; the busy
// order puts them first): the same stable LSD radix sort on the sort word as lds_radix_sort,
// with wave-ordered LDS atomics for the in-round rank, a wave scan of the wave's 256 counters
// and no workgroup barrier -- a 1 024-thread workgroup spent ~10 us of barriers and round trips
// on a list of a few hundred entries (config 3: 233 such lists, 9.4 us of each CU's sort).
constexpr int kWaveSortKeys = 1024;
constexpr int kWaveRounds = kWaveSortKeys / 64;

__device__ __forceinline__ int wave_excl_scan(int v) { return wave_incl_scan_dpp(v) - v; }

// a: this wave's LDS region (>= kWaveSortKeys slots); hist: its 256 counters.  n < kWaveSortKeys.
__device__ __forceinline__ void wave_sort_list(uint64_t* a, int* hist, int n, const uint64_t* __restrict__ seg,
                                               const int32_t* __restrict__ kslot, int32_t* __restrict__ ids,
                                               int32_t* __restrict__ kos) {
  const int lane = threadIdx.x & 63;
  const int rounds = (n + 63) >> 6;
  // stage (all loads in flight at once) and OR the varying bits of the sort words
  const uint32_t w0 = sort_word(seg[0]);
  uint32_t orv = 0;
  {
    uint32_t w[kWaveRounds];
#pragma unroll
    for (int r = 0; r < kWaveRounds; ++r) {
      const int i = r * 64 + lane;
      w[r] = r < rounds ? sort_word(seg[i < n ? i : 0]) : w0;
    }
#pragma unroll
    for (int r = 0; r < kWaveRounds; ++r) {
      const int i = r * 64 + lane;
      orv |= w[r] ^ w0;
      if (r < rounds && i < n) a[i] = ((uint64_t)w[r] << 32) | (uint64_t)(uint32_t)i;
    }
  }
  orv = (uint32_t)wave_or_i((int)orv);
  __builtin_amdgcn_wave_barrier();
  for (int shift = 0; shift < 32; shift += 8) {
    if (((orv >> shift) & 0xFFu) == 0u) continue;
#pragma unroll
    for (int k = 0; k < 4; ++k) hist[lane * 4 + k] = 0;
    __builtin_amdgcn_wave_barrier();
    uint64_t el[kWaveRounds];
    int rk[kWaveRounds];
#pragma unroll
    for (int r = 0; r < kWaveRounds; ++r) {
      if (r < rounds) {
        const int i = r * 64 + lane;
        const bool valid = i < n;
        el[r] = valid ? a[i] : 0ull;
        const uint32_t d = (sort_word(el[r]) >> shift) & 0xFFu;
        // lane-ordered returning atomics (as lds_radix_sort): the rank among equal digits
        rk[r] = valid ? (int)((d << 23) | (uint32_t)atomicAdd(&hist[d], 1)) : -1;
      }
    }
    __builtin_amdgcn_wave_barrier();
    {
      int c[4], sum = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        c[k] = hist[lane * 4 + k];
        sum += c[k];
      }
      int run = wave_excl_scan(sum);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        hist[lane * 4 + k] = run;
        run += c[k];
      }
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int r = 0; r < kWaveRounds; ++r)
      if (r < rounds && rk[r] >= 0) a[hist[rk[r] >> 23] + (rk[r] & 0x7FFFFF)] = el[r];
    __builtin_amdgcn_wave_barrier();
  }
  // equal sort words: each run insertion-sorted by its keys' low words (c*N+n) by the lane
  // that finds its start; a run longer than 32 (degenerate depths): odd-even passes
  bool long_run = false;
  for (int i = lane; i < n; i += 64) {
    const uint32_t w = sort_word(a[i]);
    if (i + 1 < n && sort_word(a[i + 1]) == w && (i == 0 || sort_word(a[i - 1]) != w)) {
      int i1 = i + 1;
      while (i1 < n && i1 - i <= 32 && sort_word(a[i1]) == w) ++i1;
      if (i1 - i > 32) {
        long_run = true;
        continue;
      }
      for (int k = i + 1; k < i1; ++k) {
        const uint64_t x = a[k];
        const uint32_t kx = low_word(seg[low_word(x)]);
        int j = k - 1;
        while (j >= i && low_word(seg[low_word(a[j])]) > kx) {
          a[j + 1] = a[j];
          --j;
        }
        a[j + 1] = x;
      }
    }
  }
  __builtin_amdgcn_wave_barrier();
  if (__ballot(long_run) != 0ull) {
    while (true) {
      bool moved = false;
      for (int ph = 0; ph < 2; ++ph) {
        for (int i = 2 * lane + ph; i + 1 < n; i += 128) {
          const uint64_t x = a[i], y = a[i + 1];
          if (sort_word(x) == sort_word(y) && low_word(seg[low_word(x)]) > low_word(seg[low_word(y)])) {
            a[i] = y;
            a[i + 1] = x;
            moved = true;
          }
        }
        __builtin_amdgcn_wave_barrier();
      }
      if (__ballot(moved) == 0ull) break;
    }
  }
  // write out through the region (as write_sorted_lds): sorted p's to registers, the list's
  // ids / emission indices coalesced into LDS, then each sorted entry reads its pair
  uint16_t pv[kWaveRounds];
#pragma unroll
  for (int r = 0; r < kWaveRounds; ++r) {
    const int s = r * 64 + lane;
    pv[r] = s < n ? (uint16_t)low_word(a[s]) : (uint16_t)0;
  }
  __builtin_amdgcn_wave_barrier();
  uint32_t* xid = reinterpret_cast<uint32_t*>(a);
  int32_t* xk = reinterpret_cast<int32_t*>(a) + n;
  {
    uint32_t id[kWaveRounds];
    int32_t ko[kWaveRounds];
#pragma unroll
    for (int r = 0; r < kWaveRounds; ++r) {
      const int i = r * 64 + lane;
      id[r] = r < rounds ? low_word(seg[i < n ? i : 0]) : 0u;
      ko[r] = r < rounds ? kslot[i < n ? i : 0] : 0;
    }
#pragma unroll
    for (int r = 0; r < kWaveRounds; ++r) {
      const int i = r * 64 + lane;
      if (r < rounds && i < n) {
        xid[i] = id[r];
        xk[i] = ko[r];
      }
    }
  }
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int r = 0; r < kWaveRounds; ++r) {
    const int s = r * 64 + lane;
    if (r < rounds && s < n) {
      ids[s] = (int32_t)xid[pv[r]];
      kos[s] = xk[pv[r]];
    }
  }
}

// MSD partition of a long list (> lds_keys, <= kMsdRegs NT keys) from REGISTERS: the list's
// sort words are loaded once (every load of a thread in flight together: one memory round trip),
// OR-ed for the varying bits, counted into per-wave digit counters, scanned digit-major /
// wave-minor in parallel, and scattered to part[] as (word << 32 | i) with per-wave returning
// atomics.  (The loop form read the list three times, a batch of 8 loads per thread per round
// trip, and scanned the 256 buckets on one thread: ~61 of a long list's ~90 us at config 5,
// profiles/r06_sort_trace_cfg5.txt.)  Order inside a bucket is free: each group of buckets is
// then sorted whole, ties by c*N+n.  Leaves s_dstart[0..256] (bucket starts) and *s_maxb.
#ifndef GSR_MSD_REGS
#define GSR_MSD_REGS 1
#endif
constexpr int kMsdRegs = 32;
template <int NT>
__device__ __forceinline__ void msd_partition_regs(SortGroup<NT>& g, const uint64_t* __restrict__ seg, int len,
                                                   int* s_hist, int* s_dstart, unsigned* s_or, int* s_maxb,
                                                   uint64_t* __restrict__ part, int lds_keys, int lazy_prefix) {
  constexpr int W = NT / 64;
  static_assert(W == 16, "digit totals below: 16 per-wave counters per digit = one lane quad");
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  for (int i = lane; i < 256; i += 64) s_hist[wv * 256 + i] = 0;
  int* const s_cut = s_hist + W * 256 + 40;   // (a free word of the misc ints)
  if (tid == 0) *s_cut = 256;
  const uint32_t w0 = sort_word(seg[0]);
  uint32_t w[kMsdRegs];
#pragma unroll
  for (int j = 0; j < kMsdRegs; ++j) {
    const int i = tid + j * NT;
    w[j] = sort_word(seg[i < len ? i : 0]);
  }
  uint32_t orv = 0;
#pragma unroll
  for (int j = 0; j < kMsdRegs; ++j) orv |= w[j] ^ w0;   // (clamped duplicates of seg[0] add nothing)
  orv = (uint32_t)wave_or_i((int)orv);
  __syncthreads();   // s_or / s_maxb initialised, the counters zeroed
  if (lane == 0 && orv) atomicOr(s_or, orv);
  __syncthreads();
  const uint32_t varying = *s_or;
  const int sh = varying ? max(31 - __clz(varying) - 7, 0) : 0;
#pragma unroll
  for (int j = 0; j < kMsdRegs; ++j)
    if (tid + j * NT < len) atomicAdd(&s_hist[wv * 256 + ((w[j] >> sh) & 0xFFu)], 1);
  __syncthreads();
  int v[4], sum = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = tid * 4 + j;   // counter (wave c & 15, digit c >> 4)
    v[j] = s_hist[(c & 15) * 256 + (c >> 4)];
    sum += v[j];
  }
  // digit tid >> 2's total: the sums of the lane quad that holds its 16 counters
  int dt = sum + dpp_row_i<0xB1>(sum);   // quad_perm [1,0,3,2]
  dt += dpp_row_i<0x4E>(dt);             // quad_perm [2,3,0,1]
  const int mb = wave_max_i(dt);
  int total;
  int run = group_exclusive_scan<NT>(g, sum, s_hist + W * 256 + 8, &total);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = tid * 4 + j;
    s_hist[(c & 15) * 256 + (c >> 4)] = run;
    if ((c & 15) == 0) s_dstart[c >> 4] = run;
    run += v[j];
  }
  if (lane == 0) atomicMax(s_maxb, mb);
  if (tid == 0) s_dstart[256] = len;
  __syncthreads();
  // a lazily sorted list (lazy_prefix > 0): the walk sorts only the buckets up to the one that
  // reaches the prefix, as ONE group when they fit in LDS -- the other keys are never read, so
  // they are not written (config 5: ~5k of a 29k-key list)
  int dlim = 256;
  if (lazy_prefix > 0) {
    if (tid < 256 && s_dstart[tid] < lazy_prefix && s_dstart[tid + 1] >= lazy_prefix) *s_cut = tid + 1;
    __syncthreads();
    const int dn = *s_cut;
    if (s_dstart[dn] <= lds_keys) dlim = dn;
  }
  if (*s_maxb <= lds_keys) {
#pragma unroll
    for (int j = 0; j < kMsdRegs; ++j) {
      const int i = tid + j * NT;
      const int d = (w[j] >> sh) & 0xFFu;
      if (i < len && d < dlim) {
        const int pos = atomicAdd(&s_hist[wv * 256 + d], 1);
        part[pos] = ((uint64_t)w[j] << 32) | (uint64_t)(uint32_t)i;
      }
    }
    __threadfence_block();
    __syncthreads();
  }
}

// Outputs: sorted_ids[s] = c*N+n of sorted entry s; k_of_s[s] = its emission entry index.
#ifdef GSR_SORT_TRACE
// timing build only (tools/sort_trace.py): per workgroup {start, end, list length, hw id}
__device__ unsigned long long* g_sort_trace = nullptr;
extern "C" int gsr_debug_sort_trace(void* buf) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_sort_trace), &buf, sizeof(buf)) == hipSuccess ? 0 : 1;
}
struct SortTrace {
  unsigned long long t0;
  int len;
  __device__ ~SortTrace() {
    __syncthreads();
    if (threadIdx.x == 0 && g_sort_trace != nullptr && len >= 0) {
      ulonglong2* d = reinterpret_cast<ulonglong2*>(g_sort_trace + 12 * (int64_t)blockIdx.x);
      d[0] = make_ulonglong2(t0, wall_clock64());
      d[1] = make_ulonglong2((unsigned long long)len, (unsigned long long)__smid());
      for (int i = 0; i < 4; ++i) d[2 + i] = make_ulonglong2(s_sort_ts[2 * i], s_sort_ts[2 * i + 1]);
    }
  }
};
#endif
template <int NT>
__global__ __launch_bounds__(NT) void k_segsort(
    uint64_t* __restrict__ keys, uint64_t* __restrict__ tmpk, int32_t* __restrict__ tmpp0,
    int32_t* __restrict__ tmpp1, const int32_t* __restrict__ tile_offset, const int32_t* __restrict__ busy,
    const int32_t* __restrict__ k_of_slot, int lds_keys, int32_t* __restrict__ sorted_ids,
    int32_t* __restrict__ k_of_s, const LazyArgs lz, gsr_bin_stats* __restrict__ stats) {
  extern __shared__ uint64_t s_keys[];
  int* s_hist = (int*)(s_keys + lds_keys);
  // the grid covers gridDim.x lists (the busy count read back, or a bound): more lists than
  // that is flagged for the raster (which then writes NaN) instead of leaving lists unsorted.
  // The counts and this workgroup's tile load together (both lists hold a slot per grid slot).
  const int ct = lz.mode == 2 ? lz.list[blockIdx.x] : busy[blockIdx.x];
  const int nb = lz.mode == 2 ? *lz.count : stats->n_busy;
  // List classes (the busy order is by log2 length, longest first; tile scan counts): A
  // (>= 8192 entries, or every list of the 256-thread shape that is >= 1024) one workgroup
  // each; B (4096..8191) two per workgroup, 8 waves and an 8 192-key slice each; C
  // (1024..4095) four per workgroup, 4 waves and 4 096 keys each; D (< 1024) a wave each.
  // The groups of B / C synchronise through LDS counters (SortGroup), not workgroup barriers,
  // so a long list no longer holds 16 waves through every barrier of a short one.  The lazy
  // re-sort's list is not in length order: one list per workgroup.
  constexpr int kSortWaves = NT / 64;
  const bool pack = lz.mode != 2 && lds_keys >= kSortWaves * kWaveSortKeys;
  int n_long = pack ? stats->n_sort_long : nb;
  int nA = !pack ? nb : (NT == 1024 ? stats->n_sort_big : n_long);
  int nAB = !pack ? nb : (NT == 1024 ? nA + stats->n_sort_mid : nA);
  if (lz.mode == 1) {   // a list that may be sorted lazily (longer than min_len) takes class A
    if (lz.min_len < kWaveSortKeys - 1) nA = nAB = n_long = nb;
    else if (lz.min_len < 4095) nA = nAB = n_long;
    else if (lz.min_len < 8191) nA = nAB;
  }
  const int wA = nA, wB = wA + (nAB - nA + 1) / 2, wC = wB + (n_long - nAB + 3) / 4;
  if ((stats->overflow & kOvfCapacity) | (ct < 0)) return;   // bounded call over its caps: nothing to sort
  if (blockIdx.x == 0 && threadIdx.x == 0 && nb > (int)gridDim.x)
    atomicOr(&stats->overflow, lz.mode == 2 ? GSR_OVF_LAZY : GSR_OVF_BUSY);
  if (lz.mode == 1 && blockIdx.x == 0 && threadIdx.x == 0 && nA == 0) *lz.count = 0;
  if ((int)blockIdx.x >= wC) {   // D: a wave per list
    const int wv = threadIdx.x >> 6;
    const int u = n_long + ((int)blockIdx.x - wC) * kSortWaves + wv;
    if (u >= nb) return;
    const int ctw = busy[u];
    const int st = tile_offset[ctw];
    const int ln = tile_offset[ctw + 1] - st;
    if (lz.mode == 1 && (threadIdx.x & 63) == 0) {   // sorted whole (at most a wave's slice)
      lz.tile_sorted[ctw] = st + ln;
      lz.flag[ctw] = 0;
    }
    wave_sort_list(s_keys + wv * kWaveSortKeys, s_hist + wv * 256, ln, keys + st, k_of_slot + st, sorted_ids + st,
                   k_of_s + st);
    return;
  }
  if constexpr (NT == 1024) {
    if ((int)blockIdx.x >= wA) {   // B or C: 2 or 4 lists per workgroup
      const bool is_b = (int)blockIdx.x < wB;
      const int W = is_b ? 8 : 4;   // waves per group
      const int gi = (threadIdx.x >> 6) / W;
      const int u = is_b ? nA + ((int)blockIdx.x - wA) * 2 + gi : nAB + ((int)blockIdx.x - wB) * 4 + gi;
      int* ghist = s_hist + gi * group_ints(W);
      int* gmisc = ghist + W * 256;
      uint64_t* slice = s_keys + gi * (lds_keys / (is_b ? 2 : 4));
      if ((threadIdx.x & (64 * W - 1)) == 0) {
        gmisc[0] = 0;                 // varying bits
        gmisc[kGroupMisc - 1] = 0;    // barrier counter
      }
      __syncthreads();   // the last workgroup-wide barrier of this path
      if (u >= (is_b ? nAB : n_long)) return;
      const int ctg = busy[u];
      const int st = tile_offset[ctg];
      const int ln = tile_offset[ctg + 1] - st;
      if (lz.mode == 1 && (threadIdx.x & (64 * W - 1)) == 0) {   // sorted whole (fits the slice)
        lz.tile_sorted[ctg] = st + ln;
        lz.flag[ctg] = 0;
      }
      if (is_b) {
        SortGroup<512> g{(int)threadIdx.x & 511, gmisc + kGroupMisc - 1, 0};
        const uint32_t varying = block_varying<512>(g, stage_keys<512>(g, slice, keys + st, ln, 0), gmisc);
        lds_radix_sort<512>(g, slice, ln, ghist, keys + st, varying);
        write_sorted_lds<512>(g, slice, ln, keys + st, k_of_slot + st, sorted_ids + st, k_of_s + st);
      } else {
        SortGroup<256> g{(int)threadIdx.x & 255, gmisc + kGroupMisc - 1, 0};
        const uint32_t varying = block_varying<256>(g, stage_keys<256>(g, slice, keys + st, ln, 0), gmisc);
        lds_radix_sort<256>(g, slice, ln, ghist, keys + st, varying);
        write_sorted_lds<256>(g, slice, ln, keys + st, k_of_slot + st, sorted_ids + st, k_of_s + st);
      }
      return;
    }
  }
  const int start = tile_offset[ct];
  const int len = tile_offset[ct + 1] - start;
#ifdef GSR_SORT_TRACE
  __shared__ unsigned long long s_t0;
  if (threadIdx.x == 0) {
    s_t0 = wall_clock64();
    for (int i = 0; i < 8; ++i) s_sort_ts[i] = 0;
  }
  SortTrace st_{0, -1};
  st_.t0 = s_t0;   // (read by thread 0 only)
  st_.len = len;
#endif
  uint64_t* seg = keys + start;
  const bool lazy = lz.mode == 1 && len > lz.min_len;
  if (lz.mode != 0 && threadIdx.x == 0) {
    lz.tile_sorted[ct] = start + len;   // lowered below for a lazily sorted list
    if (lz.mode == 1) {
      lz.flag[ct] = 0;
      if (blockIdx.x == 0) *lz.count = 0;
    } else {
      lz.tile_end[ct] = -1;   // the forward renders this tile again
    }
  }
  SortGroup<NT> g{(int)threadIdx.x, nullptr, 0};   // the whole workgroup
  if (len <= lds_keys && !lazy) {
    int* s_misc = s_hist + (NT / 64) * 256;
    if (threadIdx.x == 0) s_misc[0] = 0;
    __syncthreads();
    // the varying bits are OR-ed while staging (the barrier after the staging is block_varying's)
    const uint32_t varying = block_varying<NT>(g, stage_keys<NT>(g, s_keys, seg, len, 0), s_misc);
    lds_radix_sort<NT>(g, s_keys, len, s_hist, seg, varying);
    write_sorted_lds<NT>(g, s_keys, len, seg, k_of_slot + start, sorted_ids + start, k_of_s + start);
    return;
  }
  // Long list (> lds_keys): MSD partition by the top 8 varying bits of the sort word into
  // 256 digit buckets (through tmpk, as (word << 32 | p)), then LDS-sort groups of consecutive
  // buckets that fit -- each group holds a contiguous key range, so the sorted groups
  // concatenate to the sorted list.  One more pass over the list instead of global merges.
  {
    __shared__ int s_dstart[257];
    __shared__ int s_dcur[256];
    __shared__ unsigned s_or;
    __shared__ int s_maxb;
    if (threadIdx.x == 0) {
      s_or = 0u;
      s_maxb = 0;
    }
    for (int d = threadIdx.x; d < 256; d += blockDim.x) s_dcur[d] = 0;
    bool in_regs = false;
#if GSR_MSD_REGS
    if constexpr (NT == 1024) {
      if (len <= kMsdRegs * NT) {
        msd_partition_regs<NT>(g, seg, len, s_hist, s_dstart, &s_or, &s_maxb, tmpk + start, lds_keys,
                               lazy ? lz.prefix : 0);
        in_regs = true;
      }
    }
#endif
    if (!in_regs) {
    __syncthreads();
    const uint32_t w0 = sort_word(seg[0]);
    uint32_t orv = 0;
    for (int i0 = threadIdx.x; i0 < len; i0 += kBatch * NT) {
      uint32_t w[kBatch];
#pragma unroll
      for (int j = 0; j < kBatch; ++j) {
        const int i = i0 + j * NT;
        w[j] = sort_word(seg[i < len ? i : 0]);
      }
#pragma unroll
      for (int j = 0; j < kBatch; ++j) orv |= w[j] ^ w0;
    }
    if (orv) atomicOr(&s_or, orv);
    __syncthreads();
    const uint32_t varying = s_or;
    const int sh = varying ? max(31 - __clz(varying) - 7, 0) : 0;
    for (int i0 = threadIdx.x; i0 < len; i0 += kBatch * NT) {
      uint32_t w[kBatch];
#pragma unroll
      for (int j = 0; j < kBatch; ++j) {
        const int i = i0 + j * NT;
        w[j] = sort_word(seg[i < len ? i : 0]);
      }
#pragma unroll
      for (int j = 0; j < kBatch; ++j)
        if (i0 + j * NT < len) atomicAdd(&s_dcur[(w[j] >> sh) & 0xFFu], 1);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      int acc = 0, mb = 0;
      for (int d = 0; d < 256; ++d) {
        const int c = s_dcur[d];
        s_dstart[d] = acc;
        s_dcur[d] = acc;
        acc += c;
        mb = max(mb, c);
      }
      s_dstart[256] = acc;
      s_maxb = mb;
    }
    __syncthreads();
    if (s_maxb <= lds_keys) {
      uint64_t* part = tmpk + start;
      for (int i0 = threadIdx.x; i0 < len; i0 += kBatch * NT) {
        uint32_t w[kBatch];
#pragma unroll
        for (int j = 0; j < kBatch; ++j) {
          const int i = i0 + j * NT;
          w[j] = sort_word(seg[i < len ? i : 0]);
        }
#pragma unroll
        for (int j = 0; j < kBatch; ++j) {
          const int i = i0 + j * NT;
          if (i < len) {
            const int pos = atomicAdd(&s_dcur[(w[j] >> sh) & 0xFFu], 1);
            part[pos] = ((uint64_t)w[j] << 32) | (uint64_t)(uint32_t)i;
          }
        }
      }
      __threadfence_block();
      __syncthreads();
    }
    }
    if (s_maxb <= lds_keys) {
      uint64_t* part = tmpk + start;
      int d0 = 0;
      while (d0 < 256) {
        const int g0 = s_dstart[d0];
        int d1 = d0 + 1;
        if (lazy) {   // a group just long enough for the prefix (fewer keys to sort)
          while (d1 < 256 && s_dstart[d1] - g0 < lz.prefix && s_dstart[d1 + 1] - g0 <= lds_keys) ++d1;
        } else {
          while (d1 < 256 && s_dstart[d1 + 1] - g0 <= lds_keys) ++d1;
        }
        const int n = s_dstart[d1] - g0;
        if (n > 0) {
          copy_keys<NT>(s_keys, part + g0, n);
          __syncthreads();
          lds_radix_sort<NT>(g, s_keys, n, s_hist, seg, lds_varying<NT>(g, s_keys, n, s_hist + (NT / 64) * 256));
          write_sorted<NT>(s_keys, n, seg, k_of_slot + start, sorted_ids + start + g0, k_of_s + start + g0);
          __syncthreads();
        }
        d0 = d1;
        if (lazy && s_dstart[d0] >= lz.prefix) break;
      }
      if (lazy && threadIdx.x == 0) lz.tile_sorted[ct] = start + s_dstart[d0];
      return;
    }
  }
  // a digit bucket still exceeds LDS (depths packed into < 2^-8 of their range): sort runs of
  // lds_keys in LDS (elements keep their bucket-local index p), write them back as
  // (word | c*N+n) keys with p as payload, then merge runs pairwise in global memory.
  uint64_t* kA = tmpk + start;
  int32_t* pA = tmpp0 + start;
  uint64_t* kB = seg;   // the original keys are dead once every run is converted
  int32_t* pB = tmpp1 + start;
  for (int r0 = 0; r0 < len; r0 += lds_keys) {
    const int rl = min(lds_keys, len - r0);
    stage_keys<NT>(g, s_keys, seg + r0, rl, r0);
    __syncthreads();
    lds_radix_sort<NT>(g, s_keys, rl, s_hist, seg, lds_varying<NT>(g, s_keys, rl, s_hist + (NT / 64) * 256));
    for (int i = threadIdx.x; i < rl; i += blockDim.x) {
      const uint32_t p = low_word(s_keys[i]);
      kA[r0 + i] = (s_keys[i] & 0xffffffff00000000ull) | (uint64_t)low_word(seg[p]);
      pA[r0 + i] = (int32_t)p;
    }
    __syncthreads();
  }
  __threadfence_block();
  __syncthreads();
  for (int run = lds_keys; run < len; run <<= 1) {
    for (int r0 = 0; r0 < len; r0 += 2 * run) {
      const int na = min(run, len - r0);
      const int nb = max(0, min(run, len - r0 - na));
      merge_runs(kA + r0, pA + r0, na, kA + r0 + na, pA + r0 + na, nb, kB + r0, pB + r0);
    }
    __threadfence_block();
    __syncthreads();
    uint64_t* tk = kA; kA = kB; kB = tk;
    int32_t* tp = pA; pA = pB; pB = tp;
  }
  for (int s = threadIdx.x; s < len; s += blockDim.x) {
    sorted_ids[start + s] = (int32_t)low_word(kA[s]);
    k_of_s[start + s] = k_of_slot[start + pA[s]];
  }
}

// ---------------------------------------------------------------- split sort (few busy tiles)
// With few busy tiles (a single small view, a multi-GPU rank's share) one workgroup per list
// leaves the chip idle and the longest list's LDS sort is the whole binning's latency (config
// 2: 35 us for 8 649 keys).  The lists are then cut into blocks of kSplitBlock keys, each
// sorted by its own workgroup (same LDS radix sort and tie rule), and a second launch places
// every key at its final position: its rank in its own block plus, for every other block of
// the list, the number of keys below it there (binary searches over the list's sorted blocks
// staged in LDS).  The keys (depth word << 32 | c*N+n) of one list are unique, so the ranks
// are exactly the stable order of the one-workgroup sort.
#ifndef GSR_SPLIT_BLOCK
#define GSR_SPLIT_BLOCK 1024
#endif
constexpr int kSplitBlock = GSR_SPLIT_BLOCK;
constexpr int kSplitThreads = 256;
static_assert(kSplitBlock <= 16 * kSplitThreads, "lds_radix_sort<256> sorts at most 4096 keys");
#ifndef GSR_SPLIT_MAX_BUSY
#define GSR_SPLIT_MAX_BUSY 128
#endif
constexpr int kSplitMaxBusy = GSR_SPLIT_MAX_BUSY;
constexpr int kSplitRankThreads = 1024;   // one key per thread (1024-key blocks): the binary searches are serial LDS round trips

__global__ __launch_bounds__(kSplitThreads) void k_split_blocksort(
    const uint64_t* __restrict__ keys, uint64_t* __restrict__ tmpk, int32_t* __restrict__ tmpp,
    const int32_t* __restrict__ tile_offset, const int32_t* __restrict__ busy, const int32_t* __restrict__ k_of_slot,
    int nb_max, int32_t* __restrict__ sorted_ids, int32_t* __restrict__ k_of_s, gsr_bin_stats* __restrict__ stats) {
  __shared__ uint64_t s_keys[kSplitBlock];
  __shared__ int s_hist[(kSplitThreads / 64) * 256 + 64];
  if (stats->overflow & kOvfCapacity) return;
  const int u = blockIdx.x / nb_max, j = blockIdx.x - u * nb_max;
  const int nb = stats->n_busy;
  if (blockIdx.x == 0 && threadIdx.x == 0 && (int64_t)nb * nb_max > (int64_t)gridDim.x)
    atomicOr(&stats->overflow, GSR_OVF_BUSY);
  if (u >= nb) return;
  const int ct = busy[u];
  const int start = tile_offset[ct];
  const int len = tile_offset[ct + 1] - start;
  // the grid gives each list nb_max blocks: a longer list is flagged, not half sorted
  if (j == 0 && threadIdx.x == 0 && len > nb_max * kSplitBlock) atomicOr(&stats->overflow, GSR_OVF_SEG);
  const int b0 = j * kSplitBlock;
  if (b0 >= len) return;
  const int n = min(kSplitBlock, len - b0);
  const uint64_t* seg = keys + start;
  SortGroup<kSplitThreads> g{(int)threadIdx.x, nullptr, 0};
  stage_keys<kSplitThreads>(g, s_keys, seg + b0, n, b0);
  __syncthreads();
  lds_radix_sort<kSplitThreads>(g, s_keys, n, s_hist, seg,
                                lds_varying<kSplitThreads>(g, s_keys, n, s_hist + (kSplitThreads / 64) * 256));
  if (len <= kSplitBlock) {   // one block: final order
    write_sorted<kSplitThreads>(s_keys, n, seg, k_of_slot + start, sorted_ids + start, k_of_s + start);
    return;
  }
  for (int i = threadIdx.x; i < n; i += kSplitThreads) {
    const uint32_t p = low_word(s_keys[i]);
    tmpk[start + b0 + i] = seg[p];   // the full key: (depth word << 32 | c*N+n)
    tmpp[start + b0 + i] = (int32_t)p;
  }
}

__global__ __launch_bounds__(kSplitRankThreads) void k_split_rank(
    const uint64_t* __restrict__ tmpk, const int32_t* __restrict__ tmpp, const int32_t* __restrict__ tile_offset,
    const int32_t* __restrict__ busy, const int32_t* __restrict__ k_of_slot, int nb_max,
    int32_t* __restrict__ sorted_ids, int32_t* __restrict__ k_of_s, const gsr_bin_stats* __restrict__ stats) {
  extern __shared__ uint64_t s_all[];   // the list's sorted blocks (nb_max * kSplitBlock keys)
  if (stats->overflow & kOvfCapacity) return;
  const int u = blockIdx.x / nb_max, j = blockIdx.x - u * nb_max;
  if (u >= stats->n_busy) return;
  const int ct = busy[u];
  const int start = tile_offset[ct];
  const int len = tile_offset[ct + 1] - start;
  const int nb = (len + kSplitBlock - 1) / kSplitBlock;
  // (a list longer than the LDS image was flagged GSR_OVF_SEG by k_split_blocksort)
  if (nb <= 1 || j >= nb || nb > nb_max) return;
  copy_keys<kSplitRankThreads>(s_all, tmpk + start, len);
  __syncthreads();
  const int b0 = j * kSplitBlock;
  const int n = min(kSplitBlock, len - b0);
  for (int i = threadIdx.x; i < n; i += kSplitRankThreads) {
    const uint64_t k = s_all[b0 + i];
    int pos = i;
    for (int jj = 0; jj < nb; ++jj) {
      if (jj == j) continue;
      int lo = jj * kSplitBlock, hi = min(lo + kSplitBlock, len);   // keys of block jj below k
      const int base = lo;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (s_all[mid] < k) lo = mid + 1; else hi = mid;
      }
      pos += lo - base;
    }
    sorted_ids[start + pos] = (int32_t)low_word(k);
    k_of_s[start + pos] = k_of_slot[start + tmpp[start + b0 + i]];
  }
}

__global__ void k_selftest_lds_order(int32_t* violations) {
  __shared__ int hist[4][256];
  __shared__ int got[256];
  __shared__ int dig[256];
  __shared__ int bad;
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 4 * 256; i += blockDim.x) (&hist[0][0])[i] = 0;
  if (threadIdx.x == 0) bad = 0;
  __syncthreads();
  for (int r = 0; r < 48; ++r) {
    // all-equal, few-distinct and spread digit patterns
    const int d = r % 3 == 0 ? 7 : (r % 3 == 1 ? ((lane * 7 + r) >> 4) & 3 : (lane * 37 + r * 11) & 255);
    dig[threadIdx.x] = d;
    got[threadIdx.x] = atomicAdd(&hist[wv][d], 1);
    __syncthreads();
    for (int b = lane + 1; b < 64; ++b)
      if (dig[wv * 64 + b] == d && !(got[wv * 64 + b] > got[threadIdx.x])) atomicAdd(&bad, 1);
    __syncthreads();
  }
  if (threadIdx.x == 0) *violations = bad;
}

}  // namespace gsr

using namespace gsr;

extern "C" {

int gsr_abi_version(void) { return GSR_ABI_VERSION; }

int gsr_bin_offsets(int32_t* tile_count, int64_t CT, int32_t* tile_offset, int32_t* chunk_base,
                    int32_t* busy_tiles, int32_t* tile_end, uint64_t* tile_cut, const gsr_bin_caps* caps,
                    gsr_bin_stats* stats, void* stream) {
  GSR_REQUIRE(CT >= 1 && CT < (1ll << 31), "gsr_bin_offsets: bad CT=%lld", (long long)CT);
  gsr_bin_caps cp{0, 0, nullptr, 0, 0};
  if (caps != nullptr) cp = *caps;
  GSR_REQUIRE(cp.isect >= 0 && cp.isect < (1ll << 31) && cp.chunks >= 0 && cp.chunks < (1ll << 31),
              "gsr_bin_offsets: bad caps (I %lld, chunks %lld)", (long long)cp.isect, (long long)cp.chunks);
  const int ce = cp.chunk_entries;
  GSR_REQUIRE(ce == 0 || (ce >= kChunkEntries && ce <= (1 << 20) && (ce & (ce - 1)) == 0),
              "gsr_bin_offsets: chunk_entries %d is not 0 or a power of two in [%d, 2^20]", ce, kChunkEntries);
  const size_t lds = CT <= kScanLdsTiles ? (size_t)CT * sizeof(int) : 0;
  hipLaunchKernelGGL(k_tile_scan, dim3(1), dim3(kTopThreads), lds, (hipStream_t)stream, tile_count, CT, tile_offset,
                     chunk_base, busy_tiles, tile_end, tile_cut, cp, stats, g_fwd_heavy_log2);
  GSR_LAUNCH_CHECK("k_tile_scan");
  return GSR_OK;
}

size_t gsr_bin_sort_workspace(int64_t n_isect, int64_t CT) {
  // keys [I] + merge keys [I] (u64), two merge payloads [I] + k_of_slot [I] (i32)
  (void)CT;
  return (size_t)(2 * n_isect * sizeof(uint64_t) + 3 * n_isect * sizeof(int32_t) + 256);
}

// The workspace layout is a function of its size only (capacity cap = entries it holds), so
// gsr_bin_emit (before the host knows I) and gsr_bin_sort agree on it.
static int64_t ws_cap(size_t workspace_bytes) {
  return workspace_bytes > 256 ? (int64_t)((workspace_bytes - 256) / (2 * sizeof(uint64_t) + 3 * sizeof(int32_t))) : 0;
}

struct SortWs {
  uint64_t* keys;
  uint64_t* tmpk;
  int32_t* tmpp0;
  int32_t* tmpp1;
  int32_t* k_of_slot;
};

static SortWs sort_ws(void* workspace, int64_t cap) {
  SortWs w;
  w.keys = (uint64_t*)workspace;
  w.tmpk = w.keys + cap;
  w.tmpp0 = (int32_t*)(w.tmpk + cap);
  w.tmpp1 = w.tmpp0 + cap;
  w.k_of_slot = w.tmpp1 + cap;
  return w;
}

int gsr_bin_emit(const float* depth, const float* rec, const uint32_t* rect, const int32_t* isect_offset,
                 const int32_t* tile_offset, int32_t* tile_count, int C, int64_t N, int width, int height, int order,
                 gsr_bin_stats* stats, void* workspace, size_t workspace_bytes, void* stream) {
  GSR_REQUIRE(order == GSR_ORDER_DEPTH || order == GSR_ORDER_INDEX, "gsr_bin_emit: bad order %d", order);
  GSR_REQUIRE(order == GSR_ORDER_INDEX || depth != nullptr, "gsr_bin_emit: depth order needs the depth array");
  GSR_REQUIRE(C >= 1 && N >= 0 && (int64_t)C * N < (1ll << 31), "gsr_bin_emit: bad C=%d or N=%lld", C,
              (long long)N);
  GSR_REQUIRE(width > 0 && height > 0, "gsr_bin_emit: bad image %dx%d", width, height);
  if (N == 0) return GSR_OK;
  const int tw = ceil_div(width, kTile), th = ceil_div(height, kTile);
  const int64_t T = (int64_t)tw * th;
  const int64_t cap = ws_cap(workspace_bytes);
  GSR_REQUIRE(rec == nullptr || (order == GSR_ORDER_DEPTH && cap <= kEmitIndexMask + 1ll),
              "gsr_bin_emit: quadrant masks (rec != NULL) need depth order and a workspace of at most 2^28 entries "
              "(%lld); pass rec = NULL", (long long)cap);
  const SortWs w = sort_ws(workspace, cap);
  const int use_lds = T <= kHistMaxTiles;
  // staged when it fills the chip with its 1024-thread workgroups (config 2's 25 would leave
  // most CUs idle: 7.3 us scattered vs 9.8 us staged; config 3 30 -> 27 us, config 5 450 -> 230 us)
  // 3D: GSR_EMIT_GPT Gaussians per thread, the stage sized by the LDS the camera's tile counters
  // leave (fewer, larger workgroups claim fewer (workgroup, tile) ranges with returning atomics)
  const int gpt = order == GSR_ORDER_INDEX ? 1 : GSR_EMIT_GPT;   // Gaussians per thread (see k_emit_staged)
  const int64_t per = (int64_t)gpt * kStageThreads;
  if (T <= kStageMaxTiles && g_emit_staged && ceil_div(N, per) * C >= 256) {
    const int stage_cap = gpt == 3 ? (int)((kLdsBytes - kStageStaticLds - 8 * T) / 16) : kStageCap;
    const size_t lds = (size_t)stage_cap * 16 + (size_t)2 * T * sizeof(int);
    if (gpt == 1)
      hipLaunchKernelGGL(k_emit_staged<1>, dim3(ceil_div(N, per), C), dim3(kStageThreads), lds, (hipStream_t)stream,
                         depth, (const Splat*)rec, (const uint2*)rect, isect_offset, N, tw, th, order, tile_offset, tile_count, w.keys,
                         w.k_of_slot, stats, cap, stage_cap);
    else if (gpt == 3)
      hipLaunchKernelGGL(k_emit_staged<3>, dim3(ceil_div(N, per), C), dim3(kStageThreads), lds, (hipStream_t)stream,
                         depth, (const Splat*)rec, (const uint2*)rect, isect_offset, N, tw, th, order, tile_offset, tile_count, w.keys,
                         w.k_of_slot, stats, cap, stage_cap);
    else
      hipLaunchKernelGGL(k_emit_staged<2>, dim3(ceil_div(N, per), C), dim3(kStageThreads), lds, (hipStream_t)stream,
                         depth, (const Splat*)rec, (const uint2*)rect, isect_offset, N, tw, th, order, tile_offset, tile_count, w.keys,
                         w.k_of_slot, stats, cap, stage_cap);
    GSR_LAUNCH_CHECK("k_emit_staged");
    return GSR_OK;
  }
  dim3 grid(ceil_div(N, kEmitPerBlock), C);
  hipLaunchKernelGGL(k_emit, grid, dim3(kEmitThreads), use_lds ? T * sizeof(int) : 0, (hipStream_t)stream, depth,
                     (const Splat*)rec, (const uint2*)rect, isect_offset, N, tw, th, order, use_lds, tile_offset, tile_count, w.keys,
                     w.k_of_slot, kEmitPerBlock, stats, cap);
  GSR_LAUNCH_CHECK("k_emit");
  return GSR_OK;
}

static int bin_sort_impl(const char* who, const float* depth, const float* rec, const uint32_t* rect, const int32_t* isect_offset, const int32_t* tile_offset,
                 int32_t* tile_count, const int32_t* busy_tiles, int C, int64_t N, int width, int height, int order, int64_t n_isect,
                 int32_t max_seg, int32_t n_busy, int32_t n_big, int32_t n_mid, int emitted, gsr_bin_stats* stats,
                 void* workspace, size_t workspace_bytes, int32_t* sorted_ids, int32_t* k_of_s, const LazyArgs& lz, void* stream) {
  GSR_REQUIRE(order == GSR_ORDER_DEPTH || order == GSR_ORDER_INDEX, "%s: bad order %d", who, order);
  GSR_REQUIRE(n_isect >= 0 && n_isect < (1ll << 31), "%s: I=%lld out of range", who, (long long)n_isect);
  GSR_REQUIRE((int64_t)C * N < (1ll << 31), "%s: C*N too large for 32-bit ids", who);
  const int tw = ceil_div(width, kTile), th = ceil_div(height, kTile);
  const int64_t T = (int64_t)tw * th;
  const int64_t CT = T * C;
  GSR_REQUIRE(workspace_bytes >= gsr_bin_sort_workspace(n_isect, CT), "%s: workspace too small", who);
  if (n_isect == 0 || N == 0) return GSR_OK;
  hipStream_t s = (hipStream_t)stream;
  const SortWs w = sort_ws(workspace, ws_cap(workspace_bytes));
  uint64_t* keys = w.keys;
  uint64_t* tmpk = w.tmpk;
  int32_t* tmpp0 = w.tmpp0;
  int32_t* tmpp1 = w.tmpp1;
  int32_t* k_of_slot = w.k_of_slot;
  if (!emitted) {
    const int rc = gsr_bin_emit(depth, rec, rect, isect_offset, tile_offset, tile_count, C, N, width, height, order,
                                stats, workspace, workspace_bytes, stream);
    if (rc != GSR_OK) return rc;
  }
  GSR_REQUIRE(n_big >= 0 && n_mid >= 0 && n_big + n_mid <= n_busy, "%s: bad sort classes %d/%d of %d", who,
              n_big, n_mid, n_busy);
  // counters: the 1024-thread shape's largest layout is class C (four 4-wave groups)
  auto hist_bytes = [](int nt) { return (size_t)(nt == 1024 ? 4 * group_ints(4) : group_ints(nt / 64)) * sizeof(int); };
  if (lz.mode == 0 && g_split_sort && n_busy > 0 && n_busy <= kSplitMaxBusy && max_seg > kSplitBlock &&
      max_seg <= kSortLdsKeys) {
    const int nb_max = (max_seg + kSplitBlock - 1) / kSplitBlock;
    hipLaunchKernelGGL(k_split_blocksort, dim3(n_busy * nb_max), dim3(kSplitThreads), 0, s, keys, tmpk, tmpp0,
                       tile_offset, busy_tiles, k_of_slot, nb_max, sorted_ids, k_of_s, stats);
    GSR_LAUNCH_CHECK("k_split_blocksort");
    hipLaunchKernelGGL(k_split_rank, dim3(n_busy * nb_max), dim3(kSplitRankThreads),
                       (size_t)nb_max * kSplitBlock * sizeof(uint64_t), s, tmpk, tmpp0, tile_offset, busy_tiles,
                       k_of_slot, nb_max, sorted_ids, k_of_s, stats);
    GSR_LAUNCH_CHECK("k_split_rank");
    return GSR_OK;
  }
  // ONE launch: separate launches per class serialise (measured slower whenever long lists
  // exist); the small shape only when every list is short (e.g. the 2D configs)
  if (n_big + n_mid > 0) {
    // the full LDS image: the short lists are sorted a wave each in kWaveSortKeys-key slices of
    // it (the kernel's registers allow one workgroup per CU whatever its LDS)
    const int lds_keys = kSortLdsKeys;
    hipLaunchKernelGGL(k_segsort<kSortThreads>, dim3(n_busy), dim3(kSortThreads),
                       lds_keys * sizeof(uint64_t) + hist_bytes(kSortThreads), s, keys, tmpk, tmpp0, tmpp1,
                       tile_offset, busy_tiles, k_of_slot, lds_keys, sorted_ids, k_of_s, lz, stats);
  } else if (n_busy > 0) {
    hipLaunchKernelGGL(k_segsort<kSortThreadsSmall>, dim3(n_busy), dim3(kSortThreadsSmall),
                       kSortSmallKeys * sizeof(uint64_t) + hist_bytes(kSortThreadsSmall), s, keys, tmpk, tmpp0,
                       tmpp1, tile_offset, busy_tiles, k_of_slot, kSortSmallKeys, sorted_ids, k_of_s, lz, stats);
  }
  GSR_LAUNCH_CHECK(who);
  return GSR_OK;
}

int gsr_bin_sort(const float* depth, const float* rec, const uint32_t* rect, const int32_t* isect_offset, const int32_t* tile_offset,
                 int32_t* tile_count, const int32_t* busy_tiles, int C, int64_t N, int width, int height, int order, int64_t n_isect,
                 int32_t max_seg, int32_t n_busy, int32_t n_big, int32_t n_mid, int emitted, gsr_bin_stats* stats,
                 void* workspace, size_t workspace_bytes, int32_t* sorted_ids, int32_t* k_of_s, void* stream) {
  const LazyArgs off{};
  return bin_sort_impl("gsr_bin_sort", depth, rec, rect, isect_offset, tile_offset, tile_count, busy_tiles, C, N, width,
                       height, order, n_isect, max_seg, n_busy, n_big, n_mid, emitted, stats, workspace,
                       workspace_bytes, sorted_ids, k_of_s, off, stream);
}

size_t gsr_lazy_workspace(int64_t CT) { return (size_t)(3 * CT + 4) * sizeof(int32_t); }

int gsr_set_lazy_sort(int min_len, int prefix) {
  GSR_REQUIRE(prefix >= 1, "gsr_set_lazy_sort: prefix must be >= 1, got %d", prefix);
  gsr::g_lazy_min_len = min_len;
  gsr::g_lazy_prefix = prefix;
  return GSR_OK;
}

int gsr_lazy_min_len(void) { return gsr::g_lazy_min_len; }

int gsr_set_split_sort(int on) {
  gsr::g_split_sort = on != 0;
  return GSR_OK;
}

int gsr_set_emit_staged(int on) {
  gsr::g_emit_staged = on != 0;
  return GSR_OK;
}

int gsr_bin_sort_lazy(const float* depth, const float* rec, const uint32_t* rect, const int32_t* isect_offset,
                      const int32_t* tile_offset, int32_t* tile_count, const int32_t* busy_tiles, int C, int64_t N,
                      int width, int height, int64_t n_isect, int32_t max_seg, int32_t n_busy, int32_t n_big,
                      int32_t n_mid, int emitted, gsr_bin_stats* stats, void* workspace,
                      size_t workspace_bytes, int32_t* sorted_ids, int32_t* k_of_s, int32_t* lazy, void* stream) {
  GSR_REQUIRE(lazy != nullptr, "gsr_bin_sort_lazy: no lazy workspace");
  const int64_t CT = (int64_t)C * ceil_div(width, kTile) * ceil_div(height, kTile);
  LazyArgs lz{lazy, lazy + CT, lazy + 2 * CT, lazy + 3 * CT, nullptr, g_lazy_min_len, g_lazy_prefix, 1};
  if (lz.min_len <= 0) lz.min_len = 1 << 30;   // disabled: every list sorted whole
  return bin_sort_impl("gsr_bin_sort_lazy", depth, rec, rect, isect_offset, tile_offset, tile_count, busy_tiles, C, N,
                       width, height, GSR_ORDER_DEPTH, n_isect, max_seg, n_busy, n_big, n_mid, emitted, stats,
                       workspace, workspace_bytes, sorted_ids, k_of_s, lz, stream);
}

// Self-test of the property the sort's ranking relies on: returning LDS atomics of one wave
// instruction to the same address are applied in lane order.  out[64*R] gets each lane's
// returned count for R rounds of digits d(lane, r); returns GSR_OK and writes the number of
// out-of-order pairs to *violations (device int).
int gsr_selftest_lds_order(int32_t* violations, void* stream) {
  hipLaunchKernelGGL(k_selftest_lds_order, dim3(1), dim3(256), 0, (hipStream_t)stream, violations);
  GSR_LAUNCH_CHECK("k_selftest_lds_order");
  return GSR_OK;
}


}  // extern "C"

namespace gsr {
// The second sort of the lazy path: every tile the forward flagged (list[0..count)) sorted
// whole (one workgroup per grid slot, slots past the device-side count leave at once).
int bin_sort_rest(const int32_t* tile_offset, int64_t CT, int32_t max_seg, int32_t n_max, void* workspace,
                  size_t workspace_bytes, int32_t* lazy, int32_t* tile_end, int32_t* sorted_ids, int32_t* k_of_s,
                  gsr_bin_stats* stats, hipStream_t s) {
  if (n_max <= 0) return GSR_OK;
  const SortWs w = sort_ws(workspace, ws_cap(workspace_bytes));
  const LazyArgs lz{lazy, lazy + CT, lazy + 2 * CT, lazy + 3 * CT, tile_end, 1 << 30, 1, 2};
  int lds_keys = 1024;
  while (lds_keys < max_seg && lds_keys < kSortLdsKeys) lds_keys <<= 1;
  lds_keys = min(lds_keys, kSortLdsKeys);
  const size_t hist = (size_t)((kSortThreads / 64) * 256 + 64) * sizeof(int);
  hipLaunchKernelGGL(k_segsort<kSortThreads>, dim3(n_max), dim3(kSortThreads), lds_keys * sizeof(uint64_t) + hist, s,
                     w.keys, w.tmpk, w.tmpp0, w.tmpp1, tile_offset, (const int32_t*)nullptr, w.k_of_slot, lds_keys,
                     sorted_ids, k_of_s, lz, stats);
  GSR_LAUNCH_CHECK("k_segsort (lazy rest)");
  return GSR_OK;
}
}  // namespace gsr
