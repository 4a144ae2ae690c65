// Workgroup-dispatch probe (tools only): how long does a launch of many short workgroups take
// on MI355X, against the same work done by a persistent grid pulling items from an atomic
// counter?  Each item: one dependent pair of global loads and one store (the shape of the
// raster backward's per-chunk skeleton).  Usage: dispatch_probe [items] [lds_bytes]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ __launch_bounds__(256) void k_items(const int* __restrict__ idx, const float* __restrict__ src,
                                               float* __restrict__ dst, int n_items) {
  extern __shared__ float lds[];
  const int it = blockIdx.x;
  if (it >= n_items) return;
  const int j = idx[it * 256 + threadIdx.x];
  lds[threadIdx.x] = src[j];
  __syncthreads();
  dst[it * 256 + threadIdx.x] = lds[255 - threadIdx.x];
}

__global__ __launch_bounds__(256) void k_queue(const int* __restrict__ idx, const float* __restrict__ src,
                                               float* __restrict__ dst, int n_items, int* counter) {
  extern __shared__ float lds[];
  __shared__ int s_it;
  while (true) {
    if (threadIdx.x == 0) s_it = atomicAdd(counter, 1);
    __syncthreads();
    const int it = s_it;
    if (it >= n_items) break;
    const int j = idx[it * 256 + threadIdx.x];
    lds[threadIdx.x] = src[j];
    __syncthreads();
    dst[it * 256 + threadIdx.x] = lds[255 - threadIdx.x];
    __syncthreads();
  }
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

int main(int argc, char** argv) {
  const int n_items = argc > 1 ? atoi(argv[1]) : 7740;
  const int lds = argc > 2 ? atoi(argv[2]) : 31564;
  const size_t n = (size_t)n_items * 256;
  int* idx;
  float *src, *dst;
  int* counter;
  CK(hipMalloc(&idx, n * sizeof(int)));
  CK(hipMalloc(&src, n * sizeof(float)));
  CK(hipMalloc(&dst, n * sizeof(float)));
  CK(hipMalloc(&counter, sizeof(int)));
  int* h = (int*)malloc(n * sizeof(int));
  for (size_t i = 0; i < n; ++i) h[i] = (int)((i * 2654435761ull) % n);
  CK(hipMemcpy(idx, h, n * sizeof(int), hipMemcpyHostToDevice));
  CK(hipMemset(src, 0, n * sizeof(float)));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  int dev_cus = 0;
  CK(hipDeviceGetAttribute(&dev_cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int per_cu = 163840 / (lds + 1024);
  for (int rep = 0; rep < 3; ++rep) {
    float t1, t2;
    CK(hipEventRecord(a));
    for (int k = 0; k < 20; ++k) hipLaunchKernelGGL(k_items, dim3(n_items), dim3(256), lds, 0, idx, src, dst, n_items);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&t1, a, b));
    const int grid = dev_cus * (per_cu < 1 ? 1 : per_cu);
    CK(hipEventRecord(a));
    for (int k = 0; k < 20; ++k) {
      hipMemsetAsync(counter, 0, sizeof(int), 0);
      hipLaunchKernelGGL(k_queue, dim3(grid), dim3(256), lds, 0, idx, src, dst, n_items, counter);
    }
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&t2, a, b));
    printf("items %d lds %d: one workgroup per item %.1f us; persistent queue (%d workgroups) %.1f us\n", n_items,
           lds, 1000.f * t1 / 20, grid, 1000.f * t2 / 20);
  }
  return 0;
}
