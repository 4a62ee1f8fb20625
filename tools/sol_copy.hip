// Copy speed-of-light for xdp_stage's traffic (diagnostic): 840 MB read + 840 MB written (a 1 Mi
// mixed 64/1500-byte batch's ctx-prefixed images), as
//   grid   - a grid-stride float4 copy (every CU sweeping the buffer together), 4 loads in flight
//   ranges - xdp_stage's shape: 4096 workgroups of 256 threads, each copying its own contiguous
//            205 KB range (thread t: chunks t, t + 256, ..., four in flight)
// HIP events around 10 launches each.  hipcc --offload-arch=gfx950 -O3 tools/sol_copy.hip -o build/sol_copy
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ __launch_bounds__(256) void copy_grid(const uint4* __restrict__ s, uint4* __restrict__ d, uint64_t n) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += 4 * stride) {
    uint4 v[4];
#pragma unroll
    for (int u = 0; u < 4; u++) v[u] = i + u * stride < n ? s[i + u * stride] : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int u = 0; u < 4; u++) if (i + u * stride < n) d[i + u * stride] = v[u];
  }
}

__global__ __launch_bounds__(256) void copy_ranges(const uint4* __restrict__ s, uint4* __restrict__ d, uint64_t n,
                                                   uint64_t per) {
  const uint64_t b0 = (uint64_t)blockIdx.x * per, e = b0 + per < n ? b0 + per : n;
  for (uint64_t i = b0 + threadIdx.x; i < e; i += 4 * 256) {
    uint4 v[4];
#pragma unroll
    for (int u = 0; u < 4; u++) v[u] = i + u * 256 < e ? s[i + u * 256] : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int u = 0; u < 4; u++) if (i + u * 256 < e) d[i + u * 256] = v[u];
  }
}

int main() {
  const uint64_t bytes = 839647040ull, n = bytes / 16;
  uint4 *s, *d;
  if (hipMalloc(&s, bytes) != hipSuccess || hipMalloc(&d, bytes) != hipSuccess) return 1;
  (void)hipMemset(s, 1, bytes);
  (void)hipMemset(d, 0, bytes);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int grid : {1024, 2048, 4096, 8192, 0}) {
    for (int w = 0; w < 3; w++) {
      if (grid) hipLaunchKernelGGL(copy_grid, dim3(grid), dim3(256), 0, 0, s, d, n);
      else hipLaunchKernelGGL(copy_ranges, dim3(4096), dim3(256), 0, 0, s, d, n, (n + 4095) / 4096);
    }
    (void)hipEventRecord(e0, 0);
    for (int w = 0; w < 10; w++) {
      if (grid) hipLaunchKernelGGL(copy_grid, dim3(grid), dim3(256), 0, 0, s, d, n);
      else hipLaunchKernelGGL(copy_ranges, dim3(4096), dim3(256), 0, 0, s, d, n, (n + 4095) / 4096);
    }
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double us = ms * 1e3 / 10;
    printf("%s grid %d: %.1f us, %.2f TB/s (read + write)\n", grid ? "grid-stride" : "ranges", grid ? grid : 4096,
           us, 2.0 * bytes / us / 1e6);
  }
  return 0;
}
