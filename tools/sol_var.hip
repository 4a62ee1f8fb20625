// sol_var.hip -- speed-of-light reference for the var kernels' memory traffic (measurement tool,
// not part of the product): an offsets + lens batch (u32 offsets[n], u16 lens[n], 64-byte windows
// gathered by offset, one verdict byte per packet) with the var kernel's tiling (one wave per 64
// packets), as
//   (a) one tile per wave: offsets + lens by LDS-DMA, wait, the 64 windows by LDS-DMA, wait;
//   (b) as (a) with the metadata read into VGPRs (one offset / length per lane) and each window
//       round's addresses taken from the owning lane by ds_bpermute;
//   (c) persistent waves (k tiles each, balanced) with the next tile's metadata prefetched into a
//       second LDS buffer while this tile's windows are in flight (the var kernel's scheme);
//   (d) as (c) with double-buffered windows: tile i+1's windows and tile i+2's metadata in flight
//       while tile i is "run";
//   (e) the fixed-slot reference: (a) without the metadata (windows at i * 64).
// Prints microseconds per batch (one HIP event pair around 200 back-to-back launches, as
// bench.py) and GB/s of the algorithmic 71 B per packet (64 + 4 + 2 + 1), for 1 Mi and 8 Mi
// packets per batch.
//   hipcc --offload-arch=gfx950 -O3 -o sol_var tools/sol_var.hip && ./sol_var
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

constexpr int kWave = 64;

__device__ __forceinline__ void dma4(uintptr_t src, uint32_t lds) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(src), "s"(lds) : "memory");
}
__device__ __forceinline__ void dma1(uintptr_t src, uint32_t lds) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(src), "s"(lds) : "memory");
}
__device__ __forceinline__ void wait_all() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ uint32_t lds_of(const void* p) {
  return __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const void*)p);
}

struct Batch {
  const uint8_t* frames;
  const uint32_t* offs;
  const uint16_t* lens;
  uint64_t n;
  uint8_t* verdict;
};

// metadata of tile t into meta (offsets u32[64], lens u16[64] packed: lanes 0..31 one dword)
__device__ __forceinline__ void meta_dma(const Batch& b, uint64_t t, uint32_t* meta, uint32_t lane) {
  const uint64_t p = t * kWave + lane;
  dma1(p < b.n ? (uintptr_t)(b.offs + p) : (uintptr_t)b.offs, lds_of(meta));
  if (lane < 32) dma1(p < b.n ? (uintptr_t)(b.lens + t * kWave) + 4 * lane : (uintptr_t)b.lens, lds_of(meta + 64));
}

// the 64 windows of tile t (metadata in meta) into win: round r moves packets 16r .. 16r + 15
__device__ __forceinline__ void win_dma(const Batch& b, uint64_t t, const uint32_t* meta, uint8_t* win,
                                        uint32_t lane) {
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const uint32_t j = r * 16 + lane / 4;
    const uint64_t p = t * kWave + j;
    const uint32_t len = ((const uint16_t*)(meta + 64))[j];
    const uint32_t c = lane & 3;
    const uintptr_t src = p < b.n && c * 16 < len ? (uintptr_t)(b.frames + meta[j] + c * 16) : (uintptr_t)b.frames;
    dma4(src, lds_of(win + r * 1024));
  }
}

__device__ __forceinline__ void verdict_of(const Batch& b, uint64_t t, const uint8_t* win, uint32_t lane) {
  const uint32_t v = *(const uint32_t*)(win + lane * 64 + 12);
  const uint64_t p = t * kWave + lane;
  if (p < b.n) b.verdict[p] = (uint8_t)(1 + (v == 0x12345678u));
}

// (a)
__global__ __launch_bounds__(256) void var_one(Batch b) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x / 64);
  const uint64_t t = (uint64_t)blockIdx.x * 4 + wv;
  uint8_t* win = smem + wv * 4608;
  uint32_t* meta = (uint32_t*)(win + 4096);
  meta_dma(b, t, meta, lane);
  wait_all();
  win_dma(b, t, meta, win, lane);
  wait_all();
  verdict_of(b, t, win, lane);
}

// (b)
__global__ __launch_bounds__(256) void var_one_vgpr(Batch b) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x / 64);
  const uint64_t t = (uint64_t)blockIdx.x * 4 + wv;
  uint8_t* win = smem + wv * 4096;
  const uint64_t p = t * kWave + lane;
  const uint32_t off = p < b.n ? b.offs[p] : 0u;
  const uint32_t len = p < b.n ? b.lens[p] : 0u;
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const int j = r * 16 + lane / 4;
    const uint32_t oj = __builtin_amdgcn_ds_bpermute(j * 4, off);
    const uint32_t lj = __builtin_amdgcn_ds_bpermute(j * 4, len);
    const uint32_t c = lane & 3;
    const uintptr_t src = t * kWave + j < b.n && c * 16 < lj ? (uintptr_t)(b.frames + oj + c * 16) : (uintptr_t)b.frames;
    dma4(src, lds_of(win + r * 1024));
  }
  wait_all();
  verdict_of(b, t, win, lane);
}

// (c) persistent, metadata prefetched one tile ahead
__global__ __launch_bounds__(256) void var_persist(Batch b) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x / 64);
  uint8_t* win = smem + wv * (4096 + 768);
  uint32_t* meta0 = (uint32_t*)(win + 4096);
  const uint64_t tiles = (b.n + 63) / 64, waves = (uint64_t)gridDim.x * 4;
  uint64_t t = (uint64_t)blockIdx.x * 4 + wv;
  uint32_t mb = 0;
  if (t < tiles) meta_dma(b, t, meta0, lane);
  for (; t < tiles; t += waves) {
    uint32_t* meta = meta0 + mb * 96;
    wait_all();
    win_dma(b, t, meta, win, lane);
    if (t + waves < tiles) {  // the next tile's metadata stays in flight (two instructions)
      meta_dma(b, t + waves, meta0 + (mb ^ 1) * 96, lane);
      asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    } else {
      wait_all();
    }
    verdict_of(b, t, win, lane);
    mb ^= 1;
  }
}

// (d) persistent, double-buffered windows
__global__ __launch_bounds__(256) void var_db(Batch b) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x / 64);
  uint8_t* win0 = smem + wv * (8192 + 3 * 384);
  uint32_t* meta0 = (uint32_t*)(win0 + 8192);
  const uint64_t tiles = (b.n + 63) / 64, waves = (uint64_t)gridDim.x * 4;
  uint64_t t = (uint64_t)blockIdx.x * 4 + wv;
  if (t >= tiles) return;
  meta_dma(b, t, meta0, lane);
  wait_all();
  win_dma(b, t, meta0, win0, lane);
  if (t + waves < tiles) meta_dma(b, t + waves, meta0 + 96, lane);
  uint32_t m = 0, w = 0;
  for (; t < tiles; t += waves) {
    wait_all();  // tile t's windows, tile t + W's metadata
    const uint64_t t1 = t + waves;
    const uint32_t m1 = m == 2 ? 0 : m + 1, m2 = m1 == 2 ? 0 : m1 + 1;
    if (t1 < tiles) {
      win_dma(b, t1, meta0 + m1 * 96, win0 + (w ^ 1) * 4096, lane);
      if (t1 + waves < tiles) meta_dma(b, t1 + waves, meta0 + m2 * 96, lane);
    }
    verdict_of(b, t, win0 + w * 4096, lane);
    m = m1;
    w ^= 1;
  }
}

// (e) fixed slots, one tile per wave
__global__ __launch_bounds__(256) void fixed_one(Batch b) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x / 64);
  const uint64_t t = (uint64_t)blockIdx.x * 4 + wv;
  uint8_t* win = smem + wv * 4608;
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const uint64_t p = t * kWave + r * 16 + lane / 4;
    dma4(p < b.n ? (uintptr_t)(b.frames + p * 64 + (lane & 3) * 16) : (uintptr_t)b.frames, lds_of(win + r * 1024));
  }
  wait_all();
  verdict_of(b, t, win, lane);
}

#define CK(x)                                                       \
  do {                                                              \
    hipError_t e_ = (x);                                            \
    if (e_ != hipSuccess) {                                         \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));       \
      return 1;                                                     \
    }                                                               \
  } while (0)

int main() {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  for (uint64_t n : {1ull << 20, 8ull << 20}) {
    uint8_t *frames, *verdict;
    uint32_t* offs;
    uint16_t* lens;
    const int pool = n == (1ull << 20) ? 8 : 1;  // distinct batches (> the 256 MiB MALL at 1 Mi)
    CK(hipMalloc(&frames, pool * n * 64));
    CK(hipMemset(frames, 1, pool * n * 64));
    CK(hipMalloc(&offs, pool * n * 4));
    CK(hipMalloc(&lens, pool * n * 2));
    CK(hipMalloc(&verdict, n));
    std::vector<uint32_t> ho(n);
    std::vector<uint16_t> hl(n, 64);
    for (int q = 0; q < pool; q++) {
      for (uint64_t i = 0; i < n; i++) ho[i] = (uint32_t)(i * 64);
      CK(hipMemcpy(offs + q * n, ho.data(), n * 4, hipMemcpyHostToDevice));
      CK(hipMemcpy(lens + q * n, hl.data(), n * 2, hipMemcpyHostToDevice));
    }
    const uint64_t tiles = (n + 63) / 64;
    auto run = [&](const char* name, auto kern, uint32_t grid, uint32_t lds) -> int {
      hipEvent_t e0, e1;
      CK(hipEventCreate(&e0));
      CK(hipEventCreate(&e1));
      auto launch = [&](int i) {
        const int q = i % pool;
        Batch b{frames + (uint64_t)q * n * 64, offs + (uint64_t)q * n, lens + (uint64_t)q * n, n, verdict};
        hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, 0, b);
      };
      for (int i = 0; i < 20; i++) launch(i);
      CK(hipEventRecord(e0, 0));
      const int K = 200;
      for (int i = 0; i < K; i++) launch(i);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double us = ms * 1000.0 / K;
      printf("%-34s n=%8llu grid=%6u  %8.2f us  %7.1f GB/s\n", name, (unsigned long long)n, grid,
             us, n * 71.0 / us / 1e3);
      return 0;
    };
    const uint32_t one = (uint32_t)((tiles + 3) / 4);
    if (run("(a) one tile/wave, LDS meta", var_one, one, 4 * 4608)) return 1;
    if (run("(b) one tile/wave, VGPR meta", var_one_vgpr, one, 4 * 4096)) return 1;
    for (int per_cu : {6, 7, 8}) {
      const uint64_t resident = (uint64_t)cus * per_cu * 4;
      const uint64_t per_wave = (tiles + resident - 1) / resident;
      const uint64_t waves = (tiles + per_wave - 1) / per_wave;
      char nm[64];
      snprintf(nm, sizeof nm, "(c) persist+meta pf, %d WG/CU", per_cu);
      if (run(nm, var_persist, (uint32_t)((waves + 3) / 4), 163840 / per_cu - 80)) return 1;
    }
    for (int per_cu : {3, 4}) {
      const uint64_t resident = (uint64_t)cus * per_cu * 4;
      const uint64_t per_wave = (tiles + resident - 1) / resident;
      const uint64_t waves = (tiles + per_wave - 1) / per_wave;
      char nm[64];
      snprintf(nm, sizeof nm, "(d) persist DB, %d WG/CU", per_cu);
      if (run(nm, var_db, (uint32_t)((waves + 3) / 4), 163840 / per_cu - 80)) return 1;
    }
    if (run("(e) fixed slots, one tile/wave", fixed_one, one, 4 * 4608)) return 1;
    CK(hipFree(frames));
    CK(hipFree(offs));
    CK(hipFree(lens));
    CK(hipFree(verdict));
  }
  return 0;
}
