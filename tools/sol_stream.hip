// sol_stream.hip -- speed-of-light reference for the tile kernel's memory traffic (measurement
// tool, not part of the product): read 64 bytes per packet of a fixed-slot batch and write one
// verdict byte per packet, with the tile kernel's tiling (one wave per 64 packets), as
//   (a) plain global_load_dwordx4 into VGPRs, one tile per wave;
//   (b) LDS-DMA (global_load_lds_dwordx4) into a 4 KiB per-wave window, one tile per wave;
//   (c) as (b) with 8 waves per SIMD forced by 4.5 KiB of LDS per wave (the tile kernel's);
//   (d) as (c) on the tile kernel's balanced persistent grid (each wave k tiles);
//   (e) a streaming read: persistent grid, every lane 4 x 16 B loads in flight per round.
// Prints microseconds per batch (one HIP event pair around 200 back-to-back launches, as
// bench.py) and the HBM GB/s of 65 B per packet, for 1 Mi and 8 Mi packets per batch.
//   hipcc --offload-arch=gfx950 -O3 -o sol_stream tools/sol_stream.hip && ./sol_stream
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

constexpr int kWave = 64;

__global__ __launch_bounds__(256) void sol_vgpr(const uint8_t* frames, uint64_t n, uint8_t* verdict) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t tile = (uint64_t)blockIdx.x * 4 + threadIdx.x / 64;
  uint32_t acc = 0;
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const uint64_t p = tile * kWave + r * 16 + lane / 4;
    if (p < n) {
      const uint4 v = *(const uint4*)(frames + p * 64 + (lane & 3) * 16);
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  const uint64_t pkt = tile * kWave + lane;
  if (pkt < n) verdict[pkt] = (uint8_t)(1 + (acc == 0x12345678u));
}

template <int PAD>
__global__ __launch_bounds__(256) void sol_lds(const uint8_t* frames, uint64_t n, uint8_t* verdict) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x / 64);
  const uint64_t tile = (uint64_t)blockIdx.x * 4 + wv;
  uint8_t* win = smem + wv * (4096 + PAD);
  const uint32_t lds = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)win;
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const uint64_t p = tile * kWave + r * 16 + lane / 4;
    const uintptr_t src = p < n ? (uintptr_t)(frames + p * 64 + (lane & 3) * 16) : (uintptr_t)frames;
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(lds + r * 1024) : "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const uint32_t v = *(const uint32_t*)(win + lane * 64 + 12);
  const uint64_t pkt = tile * kWave + lane;
  if (pkt < n) verdict[pkt] = (uint8_t)(1 + (v == 0x12345678u));
}

// (d): balanced persistent waves, each `per` consecutive... grid-stride tiles
__global__ __launch_bounds__(256, 8) void sol_lds_persist(const uint8_t* frames, uint64_t n,
                                                         uint8_t* verdict) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x / 64);
  uint8_t* win = smem + wv * 4608;
  const uint32_t lds = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)win;
  const uint64_t tiles = (n + 63) / 64, waves = (uint64_t)gridDim.x * 4;
  for (uint64_t tile = (uint64_t)blockIdx.x * 4 + wv; tile < tiles; tile += waves) {
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const uint64_t p = tile * kWave + r * 16 + lane / 4;
      const uintptr_t src = p < n ? (uintptr_t)(frames + p * 64 + (lane & 3) * 16) : (uintptr_t)frames;
      uint32_t keep;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep) : "v"(src), "s"(lds + r * 1024) : "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t v = *(const uint32_t*)(win + lane * 64 + 12);
    const uint64_t pkt = tile * kWave + lane;
    if (pkt < n) verdict[pkt] = (uint8_t)(1 + (v == 0x12345678u));
  }
}

// (e): streaming read, grid-stride over 64-packet tiles, 4 x dwordx4 per lane per round
__global__ __launch_bounds__(256) void sol_stream(const uint8_t* frames, uint64_t n,
                                                  uint8_t* verdict) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wv = threadIdx.x / 64;
  const uint64_t tiles = (n + 63) / 64, waves = (uint64_t)gridDim.x * 4;
  for (uint64_t tile = (uint64_t)blockIdx.x * 4 + wv; tile < tiles; tile += waves) {
    uint4 v[4];
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const uint64_t p = tile * kWave + r * 16 + lane / 4;
      v[r] = p < n ? *(const uint4*)(frames + p * 64 + (lane & 3) * 16) : uint4{0, 0, 0, 0};
    }
    uint32_t acc = 0;
#pragma unroll
    for (int r = 0; r < 4; r++) acc ^= v[r].x ^ v[r].y ^ v[r].z ^ v[r].w;
    const uint64_t pkt = tile * kWave + lane;
    if (pkt < n) verdict[pkt] = (uint8_t)(1 + (acc == 0x12345678u));
  }
}

// (f): (c) + a returning agent-scope atomic per workgroup at the end (the counter flush's round trip)
__global__ __launch_bounds__(256) void sol_lds_atomic(const uint8_t* frames, uint64_t n,
                                                      uint8_t* verdict, unsigned long long* ctr) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x / 64);
  const uint64_t tile = (uint64_t)blockIdx.x * 4 + wv;
  uint8_t* win = smem + wv * 4608;
  const uint32_t lds = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)win;
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const uint64_t p = tile * kWave + r * 16 + lane / 4;
    const uintptr_t src = p < n ? (uintptr_t)(frames + p * 64 + (lane & 3) * 16) : (uintptr_t)frames;
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(lds + r * 1024) : "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const uint32_t v = *(const uint32_t*)(win + lane * 64 + 12);
  const uint64_t pkt = tile * kWave + lane;
  if (pkt < n) verdict[pkt] = (uint8_t)(1 + (v == 0x12345678u));
  if (wv == 0 && lane < 8) {
    const unsigned long long old = __hip_atomic_fetch_add(&ctr[(blockIdx.x % 64) * 8 + lane], 1ull,
                                                          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == 0xFFFFFFFFFFFFull) ctr[lane] = 0;  // (never: keeps the returned value live)
  }
}

template <typename K>
static float time_it(K launch, int reps = 200) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 20; i++) launch(i);
  hipEventRecord(a);
  for (int i = 0; i < reps; i++) launch(i);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float t;
  hipEventElapsedTime(&t, a, b);
  return t * 1000.f / reps;
}

int main() {
  int cus = 256;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  for (uint64_t n : {1ull << 12, 1ull << 16, 1ull << 20, 1ull << 23}) {
    const int pool = n <= (1ull << 20) ? 8 : 2;  // distinct batches (> the 256 MiB Infinity Cache at 1 Mi)
    std::vector<uint8_t*> fr(pool);
    for (auto& f : fr) {
      hipMalloc(&f, n * 64);
      hipMemset(f, 1, n * 64);
    }
    uint8_t* verdict;
    hipMalloc(&verdict, n);
    const int grid = (int)((n / 64 + 3) / 4);
    const double bytes = (double)n * 65;
    // the tile kernel's balanced persistent grid: resident waves, k tiles each
    const uint64_t tiles = n / 64, resident = (uint64_t)cus * 32;
    const uint64_t per = (tiles + resident - 1) / resident;
    const int pgrid = (int)(((tiles + per - 1) / per + 3) / 4);
    const int sgrid = cus * 8;
    printf("n = %llu packets (grid %d, persistent %d)\n", (unsigned long long)n, grid, pgrid);
    auto report = [&](const char* name, float us) {
      printf("  %-40s %8.2f us  %7.1f GB/s  %6.2f Gpkt/s\n", name, us, bytes / us / 1e3, n / us / 1e3);
    };
    report("(a) global_load_dwordx4 -> VGPR", time_it([&](int i) {
             sol_vgpr<<<grid, 256>>>(fr[i % pool], n, verdict);
           }));
    report("(b) LDS-DMA, 4 KiB per wave", time_it([&](int i) {
             sol_lds<0><<<grid, 256, 4 * 4096>>>(fr[i % pool], n, verdict);
           }));
    report("(c) LDS-DMA, 4.5 KiB per wave", time_it([&](int i) {
             sol_lds<512><<<grid, 256, 4 * 4608>>>(fr[i % pool], n, verdict);
           }));
    unsigned long long* ctr;
    hipMalloc(&ctr, 64 * 8 * 8);
    hipMemset(ctr, 0, 64 * 8 * 8);
    report("(f) as (c) + a returning atomic per WG", time_it([&](int i) {
             sol_lds_atomic<<<grid, 256, 4 * 4608>>>(fr[i % pool], n, verdict, ctr);
           }));
    hipFree(ctr);
    report("(d) LDS-DMA, 4.5 KiB, balanced persistent", time_it([&](int i) {
             sol_lds_persist<<<pgrid, 256, 4 * 4608>>>(fr[i % pool], n, verdict);
           }));
    report("(e) streaming read, persistent", time_it([&](int i) {
             sol_stream<<<sgrid, 256>>>(fr[i % pool], n, verdict);
           }));
    for (auto& f : fr) hipFree(f);
    hipFree(verdict);
  }
  return 0;
}
