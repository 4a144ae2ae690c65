// FETCH_SIZE calibration for the raster kernels' access widths (MI355X_MICROARCH.md §HBM: the
// x2 correction is calibrated for 16-B/lane streaming reads only; other widths must be
// calibrated on a known byte count).  Three kernels, each over a working set far beyond the
// 256 MiB Infinity Cache so every byte comes from HBM:
//   stream16 : lane i reads float4 a[i]                        known = 16 B x n
//   gather48 : lane i reads ids[i] then the 48-B record rec[ids[i]] (3 x float4), ids a random
//              permutation (each record read once)               known = (4 + 48) B x n
//   gather48r: the raster backward's pattern: 128-entry chunks, chunk k reads ids of its range
//              and their records; every record is referenced by 3 chunks (tiles) at random
//                                                                known = 4 B x n + 48 B x distinct
// Each kernel writes 4 B per 64 lanes (a checksum, to keep the loads alive).
// Build: hipcc -O3 --offload-arch=gfx950 tools/fetch_probe.hip -o build_var/fetch_probe
// Run:   rocprofv3 --pmc FETCH_SIZE --output-format csv -d DIR -o run -- build_var/fetch_probe
//        then bytes per launch = FETCH_SIZE(KB) x 1024 vs the "known" line printed per kernel.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
#include <vector>

#define CHECK(x)                                                                      \
  do {                                                                                \
    hipError_t e = (x);                                                               \
    if (e != hipSuccess) {                                                            \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));   \
      std::exit(1);                                                                   \
    }                                                                                 \
  } while (0)

__device__ __forceinline__ void wave_store(float v, float* out) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if ((threadIdx.x & 63) == 0) out[(blockIdx.x * blockDim.x + threadIdx.x) >> 6] = v;
}

__global__ void stream16(const float4* __restrict__ a, long n, float* out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  float s = 0.f;
  if (i < n) {
    const float4 v = a[i];
    s = v.x + v.y + v.z + v.w;
  }
  wave_store(s, out);
}

struct __align__(16) Rec {
  float4 p0, p1, p2;
};

__global__ void gather48(const Rec* __restrict__ rec, const int* __restrict__ ids, long n, float* out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  float s = 0.f;
  if (i < n) {
    const Rec r = rec[ids[i]];
    s = r.p0.x + r.p1.y + r.p2.z;
  }
  wave_store(s, out);
}

int main() {
  const long M = 8l << 20;              // 8 Mi records = 384 MiB (> 256 MiB Infinity Cache)
  const long nS = 32l << 20;            // 32 Mi float4 = 512 MiB streamed
  const long nR = 3 * M;                // gather48r: 3 references per record
  std::vector<int> perm(M);
  std::iota(perm.begin(), perm.end(), 0);
  std::mt19937 rng(7);
  std::shuffle(perm.begin(), perm.end(), rng);
  std::vector<int> rep(nR);
  for (long i = 0; i < nR; ++i) rep[i] = perm[i % M];
  // chunks of 128 consecutive references, chunk order shuffled (tiles visit records in depth order)
  {
    std::vector<long> chunks(nR / 128);
    std::iota(chunks.begin(), chunks.end(), 0);
    std::shuffle(chunks.begin(), chunks.end(), rng);
    std::vector<int> tmp(nR);
    for (size_t c = 0; c < chunks.size(); ++c)
      std::copy(rep.begin() + chunks[c] * 128, rep.begin() + chunks[c] * 128 + 128, tmp.begin() + c * 128);
    rep.swap(tmp);
  }
  float4* a;
  Rec* rec;
  int *ids, *ids_r;
  float* out;
  CHECK(hipMalloc(&a, nS * sizeof(float4)));
  CHECK(hipMalloc(&rec, M * sizeof(Rec)));
  CHECK(hipMalloc(&ids, M * sizeof(int)));
  CHECK(hipMalloc(&ids_r, nR * sizeof(int)));
  CHECK(hipMemset(a, 0, nS * sizeof(float4)));
  CHECK(hipMemset(rec, 0, M * sizeof(Rec)));
  CHECK(hipMemcpy(ids, perm.data(), M * sizeof(int), hipMemcpyHostToDevice));
  CHECK(hipMemcpy(ids_r, rep.data(), nR * sizeof(int), hipMemcpyHostToDevice));
  // flush: stream a buffer beyond the Infinity Cache between launches
  float4* flush;
  const long nF = 48l << 20;   // 768 MiB
  CHECK(hipMalloc(&flush, nF * sizeof(float4)));
  CHECK(hipMemset(flush, 0, nF * sizeof(float4)));
  // one checksum per wave of the largest launch
  CHECK(hipMalloc(&out, (std::max({nS, nR, nF, M}) / 64 + 64) * sizeof(float)));
  const int B = 256;
  for (int rep_i = 0; rep_i < 3; ++rep_i) {
    hipLaunchKernelGGL(stream16, dim3((nF + B - 1) / B), dim3(B), 0, 0, flush, nF, out);   // flush (ignore)
    hipLaunchKernelGGL(stream16, dim3((nS + B - 1) / B), dim3(B), 0, 0, a, nS, out);
    hipLaunchKernelGGL(stream16, dim3((nF + B - 1) / B), dim3(B), 0, 0, flush, nF, out);
    hipLaunchKernelGGL(gather48, dim3((M + B - 1) / B), dim3(B), 0, 0, rec, ids, M, out);
    hipLaunchKernelGGL(stream16, dim3((nF + B - 1) / B), dim3(B), 0, 0, flush, nF, out);
    hipLaunchKernelGGL(gather48, dim3((nR + B - 1) / B), dim3(B), 0, 0, rec, ids_r, nR, out);
  }
  CHECK(hipDeviceSynchronize());
  std::printf("launch order per repetition: flush, stream16, flush, gather48 (perm), flush, gather48 (3 refs)\n");
  std::printf("known stream16  bytes/launch: %ld\n", nS * 16);
  std::printf("known gather48  bytes/launch: %ld (ids %ld + records %ld)\n", M * 52, M * 4, M * 48);
  std::printf("known gather48r bytes/launch: %ld (ids %ld + distinct records %ld; %ld if every reference refetched)\n",
              nR * 4 + M * 48, nR * 4, M * 48, nR * 52);
  std::printf("flush stream16 bytes/launch: %ld\n", nF * 16);
  return 0;
}
