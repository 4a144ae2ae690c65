/*
 * gsr.h — C ABI of the MI355X (gfx950) Gaussian-splatting rasterizer (libgsr.so).
 *
 * Drop-in boundary: this library replaces the native arithmetic behind
 * pose-splatter's renderer plugin (src/gaussian_renderer.py):
 *
 *   - 3D: the gsplat extension called by GaussianRenderer3D.render
 *         (src/gaussian_renderer.py:196-208 → gsplat.rendering.rasterization, packed=False,
 *         classic mode).  Each entry point below replaces one gsplat stage:
 *           gsr3d_project_fwd   ← fully_fused_projection (fwd)
 *           gsr_bin_offsets     ← isect_tiles (counting) + isect_offset_encode
 *           gsr_bin_sort        ← isect_tiles (key emission) + cub radix sort
 *           gsr3d_raster_fwd    ← rasterize_to_pixels (fwd)
 *           gsr3d_raster_bwd    ← rasterize_to_pixels (bwd)
 *           gsr3d_project_bwd   ← fully_fused_projection (bwd) + the adapter's autograd
 *                                  (exp / quat-normalise / clamp / sigmoid,
 *                                   src/gaussian_renderer.py:190-193)
 *   - 2D: the dense PyTorch compositor GaussianRenderer2D._render_vectorized
 *         (src/gaussian_renderer.py:336-427) and its autograd backward, re-expressed as a
 *         tiled, index-ordered compositor:  gsr2d_project_fwd / gsr_bin_* (index order) /
 *         gsr2d_raster_fwd / gsr2d_raster_bwd / gsr2d_project_bwd.
 *
 * Conventions
 *   - Plain pointers to DEVICE memory; the caller (PyTorch's caching allocator) owns all
 *     memory.  The library allocates nothing and frees nothing.  Inputs are read-only.
 *   - Every call enqueues on the caller's stream (a hipStream_t passed as void*); no call
 *     synchronises the device.  The caller either reads gsr_bin_stats back (filled on the
 *     device by gsr_bin_offsets; the first 32 bytes) to size the intersection buffers
 *     exactly, or -- with NO host read at all -- passes upper bounds (gsr_bin_caps) to
 *     gsr_bin_offsets and sizes every buffer and grid from them.  A bound that does not hold
 *     is detected on the device: stats->overflow gets a GSR_OVF_* bit, every later kernel of
 *     the call writes NaN to its float outputs (rgb, alpha, v_params) instead of computing,
 *     and the bits are OR-ed into the caller's sticky status word.  A bounded call therefore
 *     never returns a silently wrong render ("Threading / streams").
 *   - Return 0 on success; negative on failure (GSR_E*).  gsr_last_error() returns a
 *     thread-local message for the last failure of the calling thread.  No C++ exception
 *     crosses the ABI.
 *   - fp32 arithmetic throughout; 32-bit indices (I < 2^31 intersections per call).
 *
 * Splat record (written by *_project_fwd, read by binning and rasterisation):
 *   12 floats (48 B) per (camera c, Gaussian n), at rec[(c*N + n)*12]:
 *     [0]=x [1]=y  screen-space mean (pixels)      [2]=opacity   [3]=L
 *     [4]=a [5]=b [6]=c  exponent  sigma = a*dx^2 + b*dx*dy + c*dy^2,  d = mean - pixel
 *     [7]=-b/(2c)
 *     [8..10]=rgb (activated colour)                [11]=-b/(2a)
 *   ([3], [7], [11] are the per-Gaussian constants of the rasterizer's sub-tile cull:
 *    L = ln(255*opacity) in 3D (gsplat's 1/255 skip), ln(opacity/eps_cut) in 2D.)
 *   2D records (gsr2d_project_fwd, since ABI 8) are stored PACKED for the compositing walks:
 *     [0]=x [1]=y [2]=opacity [3]=r   [4]=a [5]=b [6]=c [7]=g   [8]=b(blue) [9]=L [10]=-b/(2c)
 *     [11]=-b/(2a); and only for the first camera of each parameter set (ABI 7).
 *   Since ABI 11 (2D) / 12 (3D) a, b, c and L are stored times log2(e) (alpha = opacity *
 *   2^-(a dx^2 + ...), one v_exp_f32 in the walks); the slopes are unchanged.
 *   depth: 1 float per (c,n) (3D camera-space z; the sort key's high word).
 *   rect: 2 uint32 per (c,n): {x0 | x1<<16, y0 | y1<<16}, tiles [x0,x1) x [y0,y1).
 *
 * Per-entry gradient partials (written by *_raster_bwd, reduced by *_project_bwd):
 *   one row of GSR_PARTIAL_STRIDE floats per intersection, in EMISSION order (row
 *   k = isect_offset[c*N+n] + j, j = row-major index of the tile in the Gaussian's rect):
 *   d/dx, d/dy, d/da, d/db, d/dc, d/dopacity, d/drgb[3] (36 B, summed over the 16x16
 *   tile's pixels) — a deterministic replacement for float atomics.  Only entries before
 *   their tile's cut (see tile_cut) are written; the others are never read.
 *   2D with more cameras than parameter sets (C > F, set_begin given; round 5, revision 12
 *   kept): the cameras of a set render the same image (views are ignored), so
 *   gsr2d_raster_bwd walks each (set, tile) once for all the set's cameras, each with its own
 *   cotangent, and writes the set's SUMMED row at its first camera's emission index only;
 *   gsr2d_project_bwd, called with the same C / F / set_begin, reads only those rows.  The
 *   other cameras' rows are left unwritten.  A caller that pairs the two calls sees no change.
 *   With the automatic forward layout (gsr_set_fwd_lanes(0)) the binning is shared the same way:
 *   gsr2d_project_fwd gives only each set's first camera tiles (the other cameras' rect / count
 *   are empty), and gsr2d_raster_fwd renders every camera of the set from that camera's lists.
 */
#ifndef GSR_H
#define GSR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GSR_OK 0
#define GSR_EINVAL -1     /* bad shape / argument                                   */
#define GSR_ELAUNCH -2    /* HIP launch failure                                     */
#define GSR_ECAPACITY -3  /* caller buffer / workspace too small                     */

#define GSR_TILE 16
#define GSR_RADIUS_OPACITY_AABB 0      /* gsplat >= 1.5: per-axis, opacity-aware extent */
#define GSR_RADIUS_ISOTROPIC_3SIGMA 1  /* gsplat <= 1.4: ceil(3*sqrt(lambda_max))       */
#define GSR_ORDER_DEPTH 0              /* 3D: per-tile list ordered by (depth, c*N+n)   */
#define GSR_ORDER_INDEX 1              /* 2D: per-tile list ordered by parameter index  */
#define GSR_INPUT_ADAPTER 0            /* 3D rows: raw pose-splatter params (adapter)   */
#define GSR_INPUT_GSPLAT 1             /* 3D rows: activated gsplat rasterization() inputs */

#ifndef GSR_CHUNK
#define GSR_CHUNK 128                  /* list entries per LDS-staged backward sub-chunk; the work unit
                                          ("chunk", gsr_bin_caps.chunk_entries) is a power-of-two
                                          multiple of it (default GSR_CHUNK) */
#endif
#define GSR_PARTIAL_STRIDE 9           /* floats per partial row (36 B, 4 B aligned; 12 before ABI 10) */

/* stats->overflow bits (capacity-bounded calls; 0 = every bound held) */
#define GSR_OVF_ISECT 1      /* I > caps->isect: intersection buffers too small              */
#define GSR_OVF_CHUNKS 2     /* chunks > caps->chunks: chunk records / descriptors too small */
#define GSR_OVF_BUSY 4       /* more busy tiles than the sort / raster grids cover (n_busy)  */
#define GSR_OVF_SEG 8        /* a list longer than the split sort's geometry (max_seg)       */
#define GSR_OVF_LAZY 16      /* more lazily sorted tiles than the re-render covers            */
#define GSR_OVF_UNIT 32      /* a raster backward given another chunk_entries than gsr_bin_offsets */
#define GSR_OVF_EXCHANGE 64  /* a rank touched more Gaussians than its gradient row block holds */
#define GSR_OVF_LAYOUT 128   /* a 2D call's layout decisions disagree between its calls (a gsr_set_*
                                setting changed between projection, forward and backward): the
                                tiles / gradients concerned are NaN */

typedef struct gsr_bin_stats {
  int64_t n_isect;     /* total (Gaussian, tile) intersections I                     */
  int32_t max_seg;     /* longest per-tile list                                       */
  int32_t n_busy;      /* tiles with a non-empty list                                 */
  int32_t n_chunks;    /* sum over tiles of ceil(list length / chunk_entries)          */
  int32_t n_active;    /* chunks the 3D backward visits (appended by gsr3d_raster_fwd)   */
  int32_t n_sort_big;  /* tiles with lists >= 8192 entries (the first of the busy order)   */
  int32_t n_sort_mid;  /* tiles with 4096..8191 entries (the next ones)                    */
  /* ---- capacity-bounded calls (gsr_bin_caps); zero for exact (read-back) calls ---- */
  int64_t isect_cap;   /* copy of caps->isect (0: unbounded)                          */
  int64_t chunk_cap;   /* copy of caps->chunks (0: unbounded)                         */
  int32_t overflow;    /* GSR_OVF_* bits; nonzero: this call's outputs are NaN        */
  int32_t chunk_entries; /* list entries per backward work unit (copy of caps->chunk_entries) */
  int32_t* status;     /* copy of caps->status (device; may be NULL)                  */
  int32_t n_sort_long; /* tiles with lists >= 1024 entries (the sort's one-workgroup lists) */
  int32_t masks;       /* bit 0: the emission stored 3D quadrant masks in k_of_s (gsr_bin_emit rec);
                          bit 1: the 2D forward wrote the colour planes of the split per-set
                          backward (gsr_set_bwd2d_parts), which checks it;
                          bit 2: the 3D forward wrote box survivor masks (box_masks) */
  int32_t n_heavy;     /* busy tiles with lists >= heavy_min_len entries (gsr_set_fwd_heavy; 0 if
                          off): the first of the busy order, rendered by the 3D forward's
                          heavy-tile layout */
  int32_t heavy_min_len; /* their list-length threshold, a power of two (INT32_MAX: none) */
} gsr_bin_stats;       /* 80 bytes; written by gsr_bin_offsets                         */

/* Upper bounds for a call that does not read stats back (gsr_bin_offsets).  The caller sizes
 * the intersection buffers (sort workspace, sorted_ids, k_of_s, partial rows) for `isect`
 * entries and the chunk buffers for `chunks`, and passes grid bounds (n_busy, max_seg,
 * n_lazy_max, n_chunks) to the later calls instead of read-back values.  status: an optional
 * caller-owned DEVICE int32 that accumulates (OR) the overflow bits of every bounded call that
 * reaches its raster forward (a sticky flag the caller inspects when convenient). */
typedef struct gsr_bin_caps {
  int64_t isect;
  int64_t chunks;
  int32_t* status;
  /* list entries per backward work unit (a "chunk": one chunk record per pixel in the forward,
   * one workgroup in the backward, which walks it back to front in GSR_CHUNK-entry sub-chunks
   * carrying each pixel's state): 0 = GSR_CHUNK, else a power of two >= GSR_CHUNK.  Longer
   * units write fewer chunk records and re-read the pixel state less often; shorter ones give
   * the backward more parallelism (long, early-terminating 3D lists). */
  int32_t chunk_entries;
  int32_t reserved;
} gsr_bin_caps;

int gsr_version(void);
/* ABI revision of this header (bumped whenever a prototype or struct above changes; the
 * Python binding refuses a library whose revision differs).  Revision 3: gsr_bin_stats grew
 * to 80 bytes and gained the bounded-call fields; gsr_bin_offsets takes gsr_bin_caps;
 * gsr3d_project_bwd / gsr2d_project_bwd take the stats (NaN rows on overflow); gsr_bin_sort /
 * gsr_bin_sort_lazy take mutable stats. */
/* Revision 4: gsr_bin_stats.n_sort_long (in the former reserved words; size unchanged). */
/* Revision 5: the sparse gradient row blocks (gsr3d_touched_rows, gsr3d_project_bwd_rows,
 * gsr_rows_scatter_add, GSR_OVF_EXCHANGE); quadrant masks: gsr_bin_emit / gsr_bin_sort /
 * gsr_bin_sort_lazy take `rec` after `depth`, gsr3d_raster_fwd takes `k_of_s` after
 * `sorted_ids`, gsr_bin_stats.masks (the former reserved32) says whether they were stored. */
/* Revision 6: 2D chunk records are T anchors (one float per pixel per chunk: T at the chunk's
 * start, written by gsr2d_raster_fwd), the 2D chunk list holds one unit per tile and
 * gsr2d_raster_bwd's n_chunks bounds the busy tiles (k_raster2d_bwd_tile). */
/* Revision 7: 2D records are stored once per parameter set (gsr2d_project_fwd writes the copy of
 * each set's first camera only); gsr2d_raster_fwd / gsr2d_raster_bwd take N, set_begin, F (the
 * same set CSR as gsr2d_project_fwd) to read it, visit the tiles in an XCD-aware sweep (the
 * cameras of a set render a tile back to back on one XCD), and the 2D chunk list holds one
 * unit per sweep slot: chunk_list needs >= C * tiles + 8 entries. */
/* Revision 8: 2D records are stored packed (layout above): the 2D walks read them as 2 x b128 +
 * b32 from LDS as staged (or gathered straight into LDS). */
/* Revision 9: gsr_set_bwd_layout (the 3D raster backward's layout, process-wide). */
/* Revision 10: partial rows are 9 floats (GSR_PARTIAL_STRIDE 9, was 12: the 3 padding floats cost
 * 25 % of the rows' HBM writes and reads). */
/* Revision 11: 2D records hold the conic and L times log2(e) (layout above). */
/* Revision 12: 3D records too hold the conic and L times log2(e). */
/* Revision 13 (round 6): the 2D contract changes of round 5 and round 6 made explicit -- with more
 * cameras than parameter sets (C > F) gsr2d_project_fwd bins only each set's first camera (the
 * other cameras get no tiles and their forwards render the first camera's lists) and
 * gsr2d_raster_bwd / gsr2d_project_bwd write / read one summed partial row per (set, entry);
 * gsr_bin_stats.masks became a bit field (bit 1: the 2D forward wrote the split backward's
 * colour planes); GSR_OVF_LAYOUT (128) flags a 2D call whose calls disagree on those layout
 * decisions (a gsr_set_* setting changed between them): NaN tiles / gradients, sticky status. */
/* Revision 14 (round 6): gsr3d_raster_fwd, gsr3d_raster_fwd_lazy, gsr3d_raster_bwd and
 * gsr3d_raster_bwd_loss take box_masks (before the stream): the forward's per-chunk box
 * survivor masks, stats->masks bit 2. */
#define GSR_ABI_VERSION 14
int gsr_abi_version(void);
const char* gsr_last_error(void);

/* Self-test of the cross-lane reduction used by the backward kernels (one 64-lane wave):
 * out[l] = sum over lanes L of v_L[l] with v_L[i] = ((L*7 + i*13) % 97) + i/4.  out: 64 floats. */
int gsr_selftest_reduce64(float* out, void* stream);

/* Self-test of the per-box reduction of the raster backward (one 64-lane wave, same pattern):
 * out[4*l + i] = sum over the 16 lanes L with L % 4 == l % 4 of v_L[4*(l/4) + i].  out: 256 floats. */
int gsr_selftest_reduce_box16(float* out, void* stream);

/* Self-test of the b128-group-aligned per-box reductions of the raster backward (one 64-lane
 * wave, same pattern; additive to revision 12).  box_lanes 16 (G = 4 sums per lane) or 8 (G = 8):
 * out[G*l + i] = sum over the lanes L whose walk box equals lane l's output box of
 * v_L[G*slot(l) + i]; then out[64*G + 4*l + {0,1,2,3}] = {walk box, position in it, output box,
 * slot} of lane l as floats.  out: 64 * (G + 4) floats. */
int gsr_selftest_reduce_grp(float* out, int box_lanes, void* stream);

/* Layout of the raster forward (process-wide): 0 = automatic (3D: 16 lanes per pixel and 16
 * workgroups per tile for calls of at most 320 tiles (cameras x tiles), else 4 lanes per pixel and 4 workgroups per
 * tile; 2D: one 2-wave workgroup per tile, two pixels per lane), or 1, 4 or 16 (3D only) to force one.
 * All give the same result up to fp32 regrouping of the transmittance products. */
int gsr_set_fwd_lanes(int lanes);

/* Layout of the 3D raster backward (process-wide): 0 = automatic (two pixels per lane in 2-wave
 * workgroups when the call has at least 64 tiles (cameras x tiles) per compute unit, else one
 * pixel per lane in 4-wave workgroups), 1 = one pixel per lane, 2 = two pixels per lane.  Calls
 * with a fused loss or multi-chunk units always run one pixel per lane.  The layouts sum the
 * pixels' terms in different orders (fp32 regrouping); each is deterministic. */
int gsr_set_bwd_layout(int layout);

/* Heavy-tile split of the 3D raster forward (process-wide; additive to revision 12): busy tiles
 * whose lists have at least 2^log2_min_len entries (at most 64 of them, the first of the busy
 * order) are rendered in an 8-wave, 8-lanes-per-pixel layout with 512-entry rounds on a side
 * stream, forked from and joined into the call's stream, while the quad layout renders the
 * others.  log2_min_len 0 turns it off (the default); 6..30 sets the threshold, raised
 * to the next power of two while more than 64 tiles reach it (a set fixed by the list lengths).
 * Only with the automatic forward layout (gsr_set_fwd_lanes(0)): a forced layout is every tile's.
 * Takes effect at the next gsr_bin_offsets (which counts the tiles, gsr_bin_stats.n_heavy).
 * Same results as the quad layout up to fp32 regrouping of the transmittance products. */
int gsr_set_fwd_heavy(int log2_min_len);

/* Split 2D per-set backward (process-wide; additive to revision 12).  With several cameras per
 * parameter set (the per-set walk, see "Per-entry gradient partials") and fewer than
 * target_workgroups (set, tile) pairs in a call -- a frame owner's one frame of six views --
 * gsr2d_raster_bwd splits each tile's consumed list into P = min(16, ceil(target / (F x tiles)))
 * unit-aligned parts walked by separate workgroups, each starting from the pixels' suffix state
 * at its end.  gsr2d_raster_fwd then also writes, per pixel, its colour sum before every unit
 * and in total into chunk_state as three planes of n_chunks x 256 floats after the T anchors:
 * chunk_state must then hold 4 floats per slot (n_chunks*256*4, as in 3D) instead of the one the
 * 2D contract names.  0 (the default) is off; the Python binding sets 4 608.  Same results up to
 * fp32 regrouping of the suffix terms; each setting is deterministic. */
int gsr_set_bwd2d_parts(int target_workgroups);

/* Self-test of the lane-ordered LDS atomics the tile sort's ranking relies on: writes the
 * number of violations (0 expected) to the device int *violations. */
int gsr_selftest_lds_order(int32_t* violations, void* stream);

/* ---------------------------------------------------------------- (a) projection */

/* 3D projection (+ adapter activations fused).  params: [N, >=14] fp32 rows with
 * row_stride floats (layout src/gaussian_renderer.py:183-187: mean 0:3, scale 3:6, quat
 * 6:10, colour 10:13, opacity 13).  input_mode GSR_INPUT_ADAPTER: raw values through the
 * adapter's activations; GSR_INPUT_GSPLAT: activated values as gsplat's rasterization()
 * takes them (no exp/sigmoid/clamp; the quaternion is only renormalised).  viewmats [C,4,4] world->cam
 * row-major; Ks [C,3,3].  Writes rec [C*N*12], depth [C*N], rect [C*N*2], isect_count [C*N]
 * (optional: NULL writes no counts -- a count is its rect's area, (x1-x0)*(y1-y0), and no 3D
 * kernel reads it; 4 of the 68 bytes written per (c,n)),
 * isect_offset [C*N] (the first emission entry of each (c,n): every workgroup claims one
 * contiguous range for its items with one atomic, so the (c,n) ranges tile [0, I) in
 * workgroup arrival order -- consumers only address rows through isect_offset) and
 * tile_count [C*tiles + 1] (zeroed, then accumulated; element C*tiles ends as I, the
 * emission counter).  tile_count_zeroed != 0: the caller guarantees tile_count is already
 * all zero -- gsr_bin_offsets resets the counter element and gsr_bin_sort counts the tiles
 * back down, so a buffer that went through project -> offsets -> sort needs no memset.
 * Culled Gaussians get count 0.
 * [band_y0, band_y1): the tile rows this call bins, counted over the C cameras' rows laid end
 * to end (row r of camera c is global row c*th + r, th = ceil(height/16); band_y1 = -1: all
 * C*th rows).  Multi-GPU (view, band) sharding gives each rank one
 * contiguous range of (view, row) units; tiles outside it stay empty (background) and their
 * entries contribute nothing, so the ranks' gradients sum to the full gradient. */
int gsr3d_project_fwd(const float* params, int64_t N, int64_t row_stride,
                      const float* viewmats, const float* Ks, int C, int width, int height,
                      float near_plane, float far_plane, float radius_clip, float eps2d,
                      int radius_mode, int input_mode, int band_y0, int band_y1, float* rec, float* depth,
                      uint32_t* rect, int32_t* isect_count, int32_t* isect_offset, int32_t* tile_count,
                      int tile_count_zeroed, void* stream);

/* 2D projection: F parameter sets params [F][N, >=9] (layout src/gaussian_renderer.py:314-318;
 * rows row_stride floats apart, sets set_stride floats apart) rendered as C cameras (units):
 * cameras are grouped by set, set f owning cameras [set_begin[f], set_begin[f+1]) (set_begin:
 * [F+1] DEVICE int32, set_begin[F] = C; NULL means F = 1 and every camera renders set 0).  The
 * 2D renderer ignores the camera (src/gaussian_renderer.py:280-281), so a multi-frame batch
 * (frames x views) is one call with one camera per (frame, view) unit.  The
 * tile rect covers every pixel where opacity*exp(-q) >= eps_cut (the reference is dense;
 * eps_cut bounds the dropped mass).  Same outputs as gsr3d_project_fwd (rec [C*N*12], rect,
 * isect_count / isect_offset [C*N], tile_count [C*tiles + 1]); C*N < 2^31. */
int gsr2d_project_fwd(const float* params, int64_t N, int64_t row_stride, int64_t set_stride,
                      const int32_t* set_begin, int F, int C, int width, int height, float eps_cut,
                      float* rec, uint32_t* rect, int32_t* isect_count, int32_t* isect_offset,
                      int32_t* tile_count, int tile_count_zeroed, void* stream);

/* ---------------------------------------------------------------- (b) binning */

/* One workgroup over the tile histogram: tile_offset [CT+1] (exclusive scan), chunk_base
 * [CT+1] (first GSR_CHUNK-entry chunk of each tile's list), busy_tiles [CT] (rasterizer visit
 * order: the stats.n_busy non-empty tiles first, longest lists first, then the empty tiles),
 * tile_end [CT] (set to -1: the raster forward's atomicMax target), tile_cut [CT] (zeroed;
 * the raster forward writes the cut keys) and stats (device).  Resets the emission counter
 * tile_count[CT] to 0 (the per-tile counts are consumed by gsr_bin_sort).
 * caps (HOST struct, may be NULL): the bounds of a call that will not read stats back; the
 * scan records them in stats and sets GSR_OVF_ISECT / GSR_OVF_CHUNKS when I or the chunk count
 * exceeds them (isect = chunks = 0: an exact call, the caller reads stats back and sizes from
 * it), and the backward work-unit length (chunk_entries).  NULL: exact, GSR_CHUNK. */
int gsr_bin_offsets(int32_t* tile_count, int64_t CT, int32_t* tile_offset,
                    int32_t* chunk_base, int32_t* busy_tiles, int32_t* tile_end,
                    uint64_t* tile_cut, const gsr_bin_caps* caps, gsr_bin_stats* stats, void* stream);

/* Workspace for gsr_bin_sort, bytes (depends on the I read back from stats). */
size_t gsr_bin_sort_workspace(int64_t n_isect, int64_t CT);

/* Emit the (tile, key) pairs into the workspace (the first step of gsr_bin_sort), callable
 * BEFORE the host has read stats back: the workspace layout depends only on
 * workspace_bytes, and if this call's I (stats->n_isect, device) exceeds what the
 * workspace holds, the kernel does nothing -- the caller then sizes a workspace from the
 * read-back I and calls gsr_bin_sort with emitted = 0.  tile_count is consumed (counted
 * down to zero) by an emit that ran.
 * rec (3D, depth order; may be NULL): gsr3d_project_fwd's records.  When given, each entry's
 * emission index carries the entry's QUADRANT MASK in bits 28..31 (k_of_s after the sort):
 * bit q set iff the raster's exact cull keeps the record for 8x8 quadrant q of the tile
 * (q = 2 * row + column), so the raster forward can skip -- not even gather -- entries that
 * cannot reach its quadrant (at config 3 an entry reaches 1.27 of its tile's 4 quadrants).
 * Needs a workspace of at most 2^28 entries; mask the bits (& 0x0FFFFFFF) to use an index.
 * An emission that stores masks sets stats->masks = 1 (gsr_bin_offsets resets it). */
int gsr_bin_emit(const float* depth, const float* rec, const uint32_t* rect, const int32_t* isect_offset,
                 const int32_t* tile_offset, int32_t* tile_count, int C, int64_t N, int width,
                 int height, int order, gsr_bin_stats* stats, void* workspace,
                 size_t workspace_bytes, void* stream);

/* Emit (tile, key) pairs and sort each tile's list in LDS.  depth: gsr3d_project_fwd's
 * depth array (GSR_ORDER_DEPTH; may be null for GSR_ORDER_INDEX).  tile_count (the projection's
 * per-tile counts) is consumed: it is counted down to zero while slots are claimed.  Outputs:
 *   sorted_ids [I]: c*N+n per sorted entry (what the rasterizer reads),
 *   k_of_s     [I]: the emission entry k = isect_offset[cn]+j of each sorted entry (j =
 *                   row-major index of the tile in the Gaussian's rect): where the raster
 *                   backward stores that entry's partial row.
 * Sort key per entry: (sort word << 32) | c*N+n, sort word = depth float bits (3D, order
 * GSR_ORDER_DEPTH) or c*N+n (2D, GSR_ORDER_INDEX).  max_seg, n_busy and the sort classes
 * n_sort_big / n_sort_mid only choose workgroup shapes and grids: the read-back values, or
 * bounds (a bounded call: n_isect = caps->isect, n_busy >= the true busy-tile count, max_seg and
 * the classes from an earlier call).  Every list is sorted correctly for any max_seg / class
 * values; a busy count above n_busy (GSR_OVF_BUSY) or, in the split sort, a list longer than
 * max_seg (GSR_OVF_SEG) is flagged in stats->overflow.
 * emitted != 0: gsr_bin_emit already ran on this workspace (same workspace_bytes) and I fit;
 * otherwise the emit runs here.  stats: the device gsr_bin_stats. */
int gsr_bin_sort(const float* depth, const float* rec, const uint32_t* rect, const int32_t* isect_offset,
                 const int32_t* tile_offset, int32_t* tile_count,
                 const int32_t* busy_tiles, int C, int64_t N,
                 int width, int height, int order, int64_t n_isect, int32_t max_seg,
                 int32_t n_busy, int32_t n_sort_big, int32_t n_sort_mid, int emitted,
                 gsr_bin_stats* stats, void* workspace,
                 size_t workspace_bytes, int32_t* sorted_ids, int32_t* k_of_s, void* stream);

/* Lazy depth order (3D).  The forward of a tile reads its depth-sorted list only until every
 * pixel of the tile has stopped (T < 1e-4) -- at config 5 at most ~3.6k of the 16k-30k entries
 * of its longest lists.  gsr_bin_sort_lazy sorts every list longer than min_len only up to
 * a depth prefix of at least `prefix` entries (whole MSD digit buckets; the rest stays
 * unsorted), and gsr3d_raster_fwd_lazy walks each tile to the end of its sorted prefix; a
 * tile whose walk gets there (a live pixel, or a pixel whose last entry is the prefix's last)
 * is sorted whole and rendered again from scratch inside the same call.  Every entry any
 * kernel reads therefore comes in exact gsplat order: the outputs equal those of
 * gsr_bin_sort + gsr3d_raster_fwd bit for bit; sorted_ids / k_of_s past a tile's tile_end
 * are unspecified.  lazy: caller-owned int32 workspace of gsr_lazy_workspace(CT) bytes.
 * gsr_set_lazy_sort (process-wide; default min_len 16384, prefix 4096; min_len <= 0
 * disables); gsr_lazy_min_len returns the current min_len. */
/* Emission layout (process-wide, for tests and timing): 1 (default) = entries staged in LDS
 * by tile and written out in per-tile runs when the camera has <= 8192 tiles and the call
 * has >= 256 workgroups of 2048 Gaussians (per camera); 0 = every entry
 * scattered from its thread.  Same slots either way. */
int gsr_set_emit_staged(int on);

/* Sort layout (process-wide, default 1): with at most 128 busy tiles and a list longer than
 * 1024 (but <= 16384) entries, lists are sorted in 1024-key blocks by separate workgroups and
 * merged by rank (same order); 0 = one workgroup per list always. */
int gsr_set_split_sort(int on);

size_t gsr_lazy_workspace(int64_t CT);
int gsr_set_lazy_sort(int min_len, int prefix);
int gsr_lazy_min_len(void);
int gsr_bin_sort_lazy(const float* depth, const float* rec, const uint32_t* rect, const int32_t* isect_offset,
                      const int32_t* tile_offset, int32_t* tile_count, const int32_t* busy_tiles, int C,
                      int64_t N, int width, int height, int64_t n_isect, int32_t max_seg, int32_t n_busy,
                      int32_t n_sort_big, int32_t n_sort_mid, int emitted, gsr_bin_stats* stats,
                      void* workspace, size_t workspace_bytes, int32_t* sorted_ids, int32_t* k_of_s,
                      int32_t* lazy, void* stream);

/* ---------------------------------------------------------------- (c) rasterisation */

/* Front-to-back compositing (gsplat classic).  One workgroup per non-empty 16x16 tile,
 * visited in tile_order (the busy_tiles array of gsr_bin_offsets: non-empty tiles
 * longest-first, then the empty ones).  The kernels take the busy-tile count from the device
 * stats; n_busy sizes the grid (and picks the layout): stats.n_busy as read back, or a bound
 * (a bounded call; the sort has flagged GSR_OVF_BUSY if it does not hold).  With
 * stats->overflow set the call writes NaN to rgb / alpha and nothing else.
 * Empty tiles get the background (written by extra fill workgroups).  bg [C,3].
 * Outputs rgb [C,H,W,3], alpha [C,H,W], final_T [C,H,W] (exact transmittance, kept for the
 * backward), last [C,H,W] (index of the last contributing sorted entry, -1 if none),
 * tile_end [CT] (1 + max last over the tile, or the tile's start), tile_cut [CT] (sort key
 * of the tile's entry at tile_end, ~0 if none: an entry has a partial row iff its key is
 * below its tile's cut), and for the
 * chunk-parallel backward (both NULL: a forward with no backward to follow -- no records are
 * written and tile_end keeps the raw maximum of last, -1 for none; tile_cut is not set):
 * chunk_state [n_chunks*256*4] ({T at the chunk's end, the rgb
 * sum of all later chunks} per pixel of the tile, for every GSR_CHUNK-entry chunk the tile's
 * walk reached) and chunk_list [n_chunks][4] (a descriptor {first sorted entry, entry count, chunk_state row, tile} for
 * each chunk before its tile's tile_end, in no particular order; their count is added to
 * stats->n_active).  stats: the device gsr_bin_stats of gsr_bin_offsets.
 * k_of_s (may be NULL): the sort's emission indices; when the emission stored quadrant masks
 * in them (stats->masks, gsr_bin_emit given rec) a quadrant workgroup gathers only the entries
 * whose bit is set.  The outputs are the same bit for bit either way.
 * box_masks (may be NULL; ABI 14): uint32 [chunk rows][16][4], chunk rows as chunk_state.  With
 * 128-entry chunks (chunk_entries 0 or 128) the quad-layout forward writes, per chunk and 4x4
 * pixel box b of the tile (b = 4 * quadrant + box in quadrant, row-major), the 128-bit mask of
 * the chunk's entries that survive both culls for that box (empty once every pixel of the box
 * is done), and sets stats->masks bit 2; gsr3d_raster_bwd given the same buffer then lists
 * each box's entries from the masks instead of culling again.  Results are the same. */
int gsr3d_raster_fwd(const float* rec, const float* depth, const int32_t* sorted_ids, const int32_t* k_of_s,
                     const int32_t* tile_offset,
                     const int32_t* tile_order, const int32_t* chunk_base, int C, int width,
                     int height, const float* bg, int32_t n_busy, gsr_bin_stats* stats,
                     float* rgb, float* alpha, float* final_T, int32_t* last, int32_t* tile_end,
                     uint64_t* tile_cut, float* chunk_state, int32_t* chunk_list, uint32_t* box_masks,
                     void* stream);

/* gsr3d_raster_fwd over the lists of gsr_bin_sort_lazy (same outputs, see above): the tiles
 * that read past their sorted prefix are sorted whole (sort_workspace / k_of_s / max_seg of
 * that gsr_bin_sort_lazy call) and rendered again.  n_lazy_max: an upper bound on the tiles
 * sorted lazily (n_sort_big when min_len >= 8191, else n_busy).  Quadrant masks in k_of_s
 * (stats->masks) are used as in gsr3d_raster_fwd. */
int gsr3d_raster_fwd_lazy(const float* rec, const float* depth, int32_t* sorted_ids, const int32_t* tile_offset,
                          const int32_t* tile_order, const int32_t* chunk_base, int C, int width, int height,
                          const float* bg, int32_t n_busy, gsr_bin_stats* stats, float* rgb, float* alpha,
                          float* final_T, int32_t* last, int32_t* tile_end, uint64_t* tile_cut, float* chunk_state,
                          int32_t* chunk_list, int32_t* lazy, int32_t n_lazy_max, int32_t max_seg,
                          void* sort_workspace, size_t sort_workspace_bytes, int32_t* k_of_s, uint32_t* box_masks,
                          void* stream);

/* Backward of gsr3d_raster_fwd: workgroup b takes chunk_list[b] for b < stats->n_active
 * (n_chunks bounds the grid).  chunk_entries: the caps->chunk_entries given to gsr_bin_offsets
 * (0 = GSR_CHUNK); it selects the one- or the multi-sub-chunk kernel, and a mismatch with the
 * forward is flagged GSR_OVF_UNIT (NaN gradients).  v_rgb [C,H,W,3], v_alpha [C,H,W]
 * (contiguous).  Writes the partial row k_of_s[s] of every sorted entry s in [tile start,
 * tile_end).  box_masks (may be NULL): the buffer given to the forward (used only when
 * stats->masks bit 2 says it wrote it). */
int gsr3d_raster_bwd(const float* rec, const int32_t* sorted_ids, const int32_t* tile_offset,
                     const int32_t* tile_end, const int32_t* chunk_base, const float* chunk_state,
                     const int32_t* chunk_list, gsr_bin_stats* stats, int32_t n_chunks,
                     int32_t chunk_entries, int C, int width, int height, const float* bg, const float* final_T,
                     const int32_t* last, const float* v_rgb, const float* v_alpha,
                     const int32_t* k_of_s, float* partial, const uint32_t* box_masks, void* stream);

/* 2D index-order compositor (src/gaussian_renderer.py:416-425), integer pixel centres, on
 * the 3D kernels' structure (C cameras of gsr2d_project_fwd, index-order keys).  Since ABI 6
 * chunk_state holds T anchors: float [chunks][256], row chunk_base[t] + k = the T of each pixel
 * of tile t at the start of its k-th chunk of chunk_entries entries (k >= 1; written only while
 * the pixel is live), and chunk_list gets ONE unit {start, tile_end - start, chunk_base, tile} per
 * tile with a consumed entry (the per-tile backward).  rgb = canvas + (1-A)*bg, alpha = A.  Arithmetic in
 * transmittance form; a pixel stops after the entry that takes T to <= 2^-25 (the
 * reference's A == 1.0f).  Pairs with alpha < eps_cut (the binning's extent cut) are left
 * out.  bg [C,3]; rgb [C,H,W,3], alpha [C,H,W]; final_T [C,H,W,2] = (T_final, T before the
 * pixel's last composited entry).  N, set_begin, F: the parameter sets of the cameras as given to
 * gsr2d_project_fwd (the record of entry c*N+n is read from the copy of the first camera of
 * c's set).  The tiles are visited in an XCD-aware sweep (tile_order is not used by the default
 * one-lane-per-pixel layout). */
int gsr2d_raster_fwd(const float* rec, const int32_t* sorted_ids, const int32_t* tile_offset,
                     const int32_t* tile_order, const int32_t* chunk_base, int C, int width, int height,
                     float eps_cut, const float* bg, int32_t n_busy, gsr_bin_stats* stats,
                     float* rgb, float* alpha, float* final_T, int32_t* last, int32_t* tile_end,
                     uint64_t* tile_cut, float* chunk_state, int32_t* chunk_list, int64_t N,
                     const int32_t* set_begin, int F, void* stream);

/* Backward of gsr2d_raster_fwd (the reference's autograd of the recursion), same contract
 * as gsr3d_raster_bwd except that the units are whole tiles: the forward's finalize writes one
 * unit per slot of the XCD-aware tile sweep and the backward runs one workgroup per slot
 * (n_chunks is not used); each walks its tile's list back to front, re-anchoring T from
 * chunk_state at every chunk_entries boundary.  N, set_begin, F: as gsr2d_raster_fwd. */
int gsr2d_raster_bwd(const float* rec, const int32_t* sorted_ids, const int32_t* tile_offset,
                     const int32_t* tile_end, const int32_t* chunk_base, const float* chunk_state,
                     const int32_t* chunk_list, gsr_bin_stats* stats, int32_t n_chunks,
                     int32_t chunk_entries, int C, int width, int height, float eps_cut, const float* bg,
                     const float* final_T, const int32_t* last, const float* v_rgb,
                     const float* v_alpha, const int32_t* k_of_s, float* partial, int64_t N,
                     const int32_t* set_begin, int F, void* stream);

/* ---------------------------------------------------------------- projection backward */

/* Reduce the partial rows of each (c,n) (those below their tile's cut, in row order),
 * chain through projection and the adapter activations, sum over cameras: rows
 * [n_begin, n_end) of v_params [N,14] (fully overwritten, deterministic; n_end = -1: N).
 * Gaussian ranges let a multi-GPU caller start the all-reduce of finished rows while later
 * ranges are still being computed.  depth: the projection's depth array (sort keys).
 * stats: the forward's device gsr_bin_stats (may be NULL): with stats->overflow set the rows
 * are written as NaN.  isect_count is not read (each entry count is its rect's area; may be
 * NULL). */
int gsr3d_project_bwd(const float* params, int64_t N, int64_t row_stride,
                      const float* viewmats, const float* Ks, int C, int width, int height,
                      float eps2d, int input_mode, const float* depth, const uint32_t* rect,
                      const int32_t* isect_offset, const int32_t* isect_count,
                      const uint64_t* tile_cut, const float* partial, int64_t n_begin,
                      int64_t n_end, const gsr_bin_stats* stats, float* v_params, void* stream);

/* ---- Sparse gradient rows of a band share (multi-GPU strong layout) ----
 * A (view, tile-row) share of one multi-view job gives a gradient to few Gaussians (config 5
 * at 8 ranks: 2-12 %: the band's walks stop early, so most Gaussians that reach its tiles are
 * never composited).  Instead of the dense [N,14] v_params the share's
 * projection backward writes only their rows, compacted into a caller-owned ROW BLOCK of
 * cap + 1 rows of GSR_ROW_FLOATS floats:
 *   row 0      = header {int32 count (may exceed cap: overflow), int32 cap, 0, ...};
 *   row 1 + i  = {int32 n, 0, v_params[n][0..13]}   for i < min(count, cap), any order.
 * The blocks of all ranks are all-gathered (one equal-size collective, no host read) and
 * summed into the dense result in rank order by gsr_rows_scatter_add, so every rank ends
 * with the same bits.  Each call is stream-ordered and sized by cap: a whole step, exchange
 * included, can be captured in a HIP graph. */
#define GSR_ROW_FLOATS 16

/* After the forward (its finalize set tile_end): zero the header, then list the Gaussians n that
 * own a list entry before their tile's cut in any of the call's busy tiles (tile_order, the
 * device busy count in stats; n_busy bounds it) -- exactly those the raster backward gives a
 * partial row.  header count := their number, rows 1 + i := {n, 0, 0...} for the first cap.
 * stats->overflow set (the forward's bounds did not hold): header count := cap + 1, so the
 * exchange (gsr_rows_scatter_add) NaN-fills and reports GSR_OVF_EXCHANGE.
 * flags: caller workspace of N bytes (rounded up to 4).  N == 0 or n_busy == 0: the header only. */
int gsr3d_touched_rows(const int32_t* sorted_ids, const int32_t* tile_offset, const int32_t* tile_end,
                       const int32_t* tile_order, const gsr_bin_stats* stats, int32_t n_busy, int64_t N,
                       int64_t cap, uint8_t* flags, float* block, void* stream);

/* gsr3d_project_bwd for the Gaussians listed in `block` (gsr3d_touched_rows): their 14
 * gradients go to words 2..15 of their rows (deterministic per row; stats->overflow set: NaN
 * rows, and the header gsr3d_touched_rows left past the cap poisons the exchange). */
int gsr3d_project_bwd_rows(const float* params, int64_t N, int64_t row_stride,
                           const float* viewmats, const float* Ks, int C, int width, int height,
                           float eps2d, int input_mode, const float* depth, const uint32_t* rect,
                           const int32_t* isect_offset, const int32_t* isect_count,
                           const uint64_t* tile_cut, const float* partial, const gsr_bin_stats* stats,
                           int64_t cap, float* block, void* stream);

/* v_params [N,14] += the rows of `world` gathered blocks (blocks[r] at r * (cap + 1) rows),
 * rank 0 first (one stream-ordered launch per rank; a block lists an n at most once).  A header
 * whose count exceeds cap: v_params is written all NaN and *status (device, may be NULL) gets
 * GSR_OVF_EXCHANGE. */
int gsr_rows_scatter_add(const float* blocks, int world, int64_t cap, float* v_params, int64_t N,
                         int32_t* status, void* stream);

/* 2D: v_params [F,N,9] (fully overwritten): set f's gradient sums the partial rows of all its
 * cameras (set_begin as in gsr2d_project_fwd, NULL: F = 1) in camera order, then chains
 * through the activations once.  stats as in gsr3d_project_bwd. */
int gsr2d_project_bwd(const float* params, int64_t N, int64_t row_stride, int64_t set_stride,
                      const int32_t* set_begin, int F, int C, int width, int height,
                      const uint32_t* rect, const int32_t* isect_offset,
                      const int32_t* isect_count, const uint64_t* tile_cut,
                      const float* partial, const gsr_bin_stats* stats, float* v_params, void* stream);

/* ---- Loss-fused backward ------------------------------------------
 * The reference training step (scripts/training/train_script.py:30-36, 128-133) takes
 *   iou_loss = 1 - mean_c[(I_c + 1e-6) / (U_c + 1e-6)],  I_c = sum a m,  U_c = sum (a + m - a m)
 *   img_loss = img_lambda * sum |target - rgb| / sum m
 * of the rendered views (a = alpha [C,H,W], rgb [C,H,W,3]) against target_img [C,3,H,W]
 * (planar, the loader's layout) and target_mask [C,H,W].  gsr_loss_iou_l1_fwd evaluates both
 * in one pass (deterministic fixed-order reduction) and gsr3d_raster_bwd_loss generates the
 * per-pixel cotangents of  g_iou * iou_loss + g_img * img_loss (+ optional extra cotangents,
 * e.g. an SSIM term's) inside the raster backward, so no v_rgb / v_alpha image is written. */
size_t gsr_loss_workspace(int C, int width, int height);

/* sums [(C+1)*4]: per view {I_c, U_c, sum m, sum |t-rgb|}, row C = {0, 0, total m, total L1};
 * iou_loss, img_loss: one float each.  ws: gsr_loss_workspace bytes. */
int gsr_loss_iou_l1_fwd(const float* rgb, const float* alpha, const float* target_img,
                        const float* target_mask, int C, int width, int height, float img_lambda,
                        void* ws, size_t ws_bytes, float* sums, float* iou_loss, float* img_loss,
                        void* stream);

typedef struct gsr_loss_terms {
  const float* rgb;            /* [C,H,W,3] forward output */
  const float* target_img;     /* [C,3,H,W] */
  const float* target_mask;    /* [C,H,W] */
  const float* sums;           /* [(C+1)*4] from gsr_loss_iou_l1_fwd */
  const float* grad_out;       /* [2] = {g_iou, g_img}: d(total)/d(iou_loss), d(total)/d(img_loss) */
  const float* v_rgb_extra;    /* optional [C,H,W,3] added to the fused cotangent (NULL: none) */
  const float* v_alpha_extra;  /* optional [C,H,W] */
  float img_lambda;
  int32_t reserved;
} gsr_loss_terms;

/* gsr3d_raster_bwd with the cotangents generated from `loss` instead of read from images. */
int gsr3d_raster_bwd_loss(const float* rec, const int32_t* sorted_ids, const int32_t* tile_offset,
                          const int32_t* tile_end, const int32_t* chunk_base,
                          const float* chunk_state, const int32_t* chunk_list, gsr_bin_stats* stats,
                          int32_t n_chunks, int32_t chunk_entries, int C, int width, int height, const float* bg,
                          const float* final_T, const int32_t* last, const gsr_loss_terms* loss,
                          const int32_t* k_of_s, float* partial, const uint32_t* box_masks, void* stream);

/* ---- Parameter head + pose transform ----------------------------
 * Replace the post-MLP part of PoseSplatter.get_gaussian_params_from_volume_unified
 * (src/model.py:185-254) and apply_pose_transform_3d (src/model.py:258-298, with the
 * quaternion helpers at :378-421, whose float64 eigh runs here as in-register Jacobi). */

size_t gsr_head_select_workspace(int64_t M);

/* Mask-threshold search + ordered selection (src/model.py:185-197) over v0 = volume[0] [M]:
 * mt starts at mask_threshold, rises by delta while more than max_n voxels pass
 * sigmoid(v0 - mt) > prob_threshold, then falls while fewer than min_n pass (at most
 * max_iter steps in total).  Writes *mt_out (float64), info[0] = final count, info[1] =
 * steps taken, info[2] = 1 if max_iter was hit, and idx[0..count) = the passing voxel
 * indices in increasing order (idx needs M entries of room).  No host synchronisation. */
int gsr_head_select(const float* v0, int64_t M, double mask_threshold, float prob_threshold, double delta,
                    int32_t min_n, int32_t max_n, int32_t max_iter, void* ws, size_t ws_bytes, int32_t* info,
                    double* mt_out, int64_t* idx, void* stream);

/* net [N, >=14] (row stride net_stride): the MLP output (quats, scales, opacity, colours,
 * delta_means); v0 [N] = volume[0] at the selected voxels; grid [N,3] their grid points;
 * scale: device pointer to the model's scalar log-scale offset.  out [N,14] in the renderer
 * layout (means, log_scales, quats, colours, logit opacity); pose = 1 also applies the pose
 * transform for the rotation angle (host) and translation p3d[3] (device pointer). */
int gsr_head3d_fwd(const float* net, int64_t N, int64_t net_stride, const float* v0, const float* grid,
                   const float* scale, float mt, float prob_threshold, float clip_lo, float clip_hi,
                   float voxel_size, int pose, double angle, const float* p3d, float* out, void* stream);

/* g_out [N,14] -> g_net [N,14] (column 7, the discarded opacity, gets 0) and g_v0 [N].
 * The gradient of the scale offset is the sum of g_out[:,3:6] (left to the caller). */
int gsr_head3d_bwd(const float* net, int64_t N, int64_t net_stride, const float* v0, const float* grid,
                   float mt, float prob_threshold, float clip_lo, float clip_hi, float voxel_size, int pose,
                   double angle, const float* g_out, float* g_net, float* g_v0, void* stream);

/* apply_pose_transform_3d alone on renderer-layout rows [N, >=14]; out / g_params [N,14]. */
int gsr_pose3d_fwd(const float* params, int64_t N, int64_t row_stride, double angle, const float* p3d,
                   float* out, void* stream);
int gsr_pose3d_bwd(const float* params, int64_t N, int64_t row_stride, double angle, const float* g_out,
                   float* g_params, void* stream);

/* ---- SSIM loss term (scripts/training/train_script.py:129) ----------
 * torchmetrics StructuralSimilarityIndexMeasure(data_range=1.0) of C image pairs (the batch
 * mean): x = the target [C,3,H,W] and y = the render, each given as (data, strides[4] in
 * elements for (view, channel, row, column)) so planar and channels-last images are read in
 * place.  x_strides / y_strides: HOST int64 arrays (read on the host when the call is made;
 * the exception to the device-pointer convention, like taps11).
 * taps11: HOST array, the normalised 1-D Gaussian (11 taps, sigma 1.5) the caller
 * computes as torchmetrics does.  Needs H, W > 10.  fwd writes the scalar *ssim (device) and,
 * when factors != NULL (device, gsr_ssim_factors_size floats), each window's backward factors
 * (dS/dmu_y, dS/dE[y^2], dS/dE[xy]); bwd blurs those onto the pixels and writes
 * d(g_out * ssim)/dy into grad_y (device, y's strides), g_out a device scalar.  Both are
 * deterministic (fixed-order sums). */
size_t gsr_ssim_workspace(int C, int width, int height);
size_t gsr_ssim_factors_size(int C, int width, int height);
int gsr_ssim_fwd(const float* x, const int64_t* x_strides, const float* y, const int64_t* y_strides, int C, int width,
                 int height, const float* taps11, void* ws, size_t ws_bytes, float* ssim, float* factors,
                 void* stream);
int gsr_ssim_bwd(const float* x, const int64_t* x_strides, const float* y, const int64_t* y_strides, int C, int width,
                 int height, const float* taps11, const float* factors, const float* g_out, float* grad_y,
                 void* stream);

/* ---- Shape carving -----------------------------------------------
 * ShapeCarver.forward (src/shape_carver.py:322-366): the [4, n_voxels] volume (mask
 * occupancy, then rgb) from C masks [C,1,H,W] and images [C,3,H,W], with the scatter-min
 * visibility of ray_cast_visibility_torch (:132-204) done as 64-bit atomicMin.
 * grid [n_voxels,3] = the model's un-posed grid points; center [3] (device) and angle pose
 * it (get_grid_points :369-374); Ks [C,3,3] and Es [C,4,4] are HOST arrays (fixed model
 * cameras).  Ks_mask (host, or NULL = Ks) are the intrinsics of the mask volume: the adaptive
 * path (:328-335) projects the masks with principal points moved to the triangulated seed and
 * samples colours with the carver's own Ks.  Ties in the per-pixel minimum distance go to the
 * lower voxel index. */
size_t gsr_carve_workspace(int64_t n_voxels, int C, int height);
int gsr_carve_volume(const float* grid, int64_t n_voxels, const float* center, double angle, const float* Ks,
                     const float* Ks_mask, const float* Es, int C, const float* mask, const float* rgb, int height,
                     int width, float fill, float nonvisible_weight, void* ws, size_t ws_bytes, float* out,
                     void* stream);

/* Adaptive cameras, step 1 of adjust_principal_points_to_seed (src/shape_carving.py:173-245):
 * for each of C masks [C,H,W] (float, nonzero = inside; device), medoid[c] = the flat index
 * y*W+x of the mask pixel nearest the mask centroid (float64 means and squared distances as
 * numpy computes them; ties to the lowest index), or INT32_MAX for an empty mask (the
 * reference raises).  medoid: device int32 [C]; ws: device, gsr_carve_medoids_workspace(C). */
size_t gsr_carve_medoids_workspace(int C);
int gsr_carve_medoids(const float* masks, int C, int height, int width, void* ws, size_t ws_bytes, int32_t* medoid,
                      void* stream);

#ifdef __cplusplus
}
#endif
#endif /* GSR_H */
