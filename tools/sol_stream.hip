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

// (c) with s_memrealtime stamps per wave (entry, exit) into tr[2 * wave]: the waves' span vs
// the kernel's time shows the launch's own start/end cost
template <bool UNUSED>
__global__ __launch_bounds__(256) void sol_lds_trace(const uint8_t* frames, uint64_t n,
                                                     uint8_t* verdict, uint64_t* tr) {
  uint64_t t0;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
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
  uint64_t t1;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  if (lane == 0) {
    tr[2 * tile] = t0;
    tr[2 * tile + 1] = t1;
  }
}

// (g): the traced (c) with the compiled fixed-slot kernel's resources: 32 KiB LDS per workgroup,
// 82 VGPRs, 100 SGPRs (clobbers), to see whether they change the launch's start/end cost
template <bool BIG>
__global__ __launch_bounds__(256) void sol_lds_res(const uint8_t* frames, uint64_t n,
                                                   uint8_t* verdict, uint64_t* tr) {
  uint64_t t0;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  if (BIG)
    asm volatile("" ::: "v40", "v50", "v60", "v70", "v75", "v80", "v81", "s40", "s50", "s60",
                 "s70", "s80", "s90", "s95", "s99");
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x / 64);
  const uint64_t tile = (uint64_t)blockIdx.x * 4 + wv;
  uint8_t* win = smem + wv * (BIG ? 8192 : 4608);
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
  uint64_t t1;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  if (lane == 0) {
    tr[2 * tile] = t0;
    tr[2 * tile + 1] = t1;
  }
}

// (h): the traced (c) with a 208-byte by-value argument struct and gridDim (hidden kernel
// arguments: a 464-byte kernarg segment, as the compiled kernel's LaunchArgs)
struct BigArgs {
  const uint8_t* frames;
  uint64_t n;
  uint8_t* verdict;
  uint64_t* tr;
  uint64_t pad[22];
};
__global__ __launch_bounds__(256) void sol_lds_bigargs(BigArgs a) {
  uint64_t t0;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x / 64);
  const uint64_t tile = ((uint64_t)blockIdx.x * 4 + wv) % ((uint64_t)gridDim.x * 4);
  uint8_t* win = smem + wv * 4608;
  const uint32_t lds = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)win;
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const uint64_t p = tile * kWave + r * 16 + lane / 4;
    const uintptr_t src = p < a.n ? (uintptr_t)(a.frames + p * 64 + (lane & 3) * 16) : (uintptr_t)a.frames;
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(lds + r * 1024) : "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const uint32_t v = *(const uint32_t*)(win + lane * 64 + 12);
  const uint64_t pkt = tile * kWave + lane;
  if (pkt < a.n) a.verdict[pkt] = (uint8_t)(1 + (v == 0x12345678u) + a.pad[lane % 22]);
  uint64_t t1;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  if (lane == 0) {
    a.tr[2 * tile] = t0;
    a.tr[2 * tile + 1] = t1;
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
    if (n == (1ull << 20)) {  // waves' span (stamps) vs kernel time, consecutive launches
      uint64_t* tr;
      const size_t tb = (n / 64) * 2 * sizeof(uint64_t);
      hipMalloc(&tr, 2 * tb);
      const float us = time_it([&](int i) {
        sol_lds_trace<false><<<grid, 256, 4 * 4608>>>(fr[i % pool], n, verdict, tr + (i & 1) * (tb / 8));
      });
      std::vector<uint64_t> h(2 * tb / 8);
      hipMemcpy(h.data(), tr, 2 * tb, hipMemcpyDeviceToHost);
      uint64_t lo[2] = {~0ull, ~0ull}, hi[2] = {0, 0};
      for (int k = 0; k < 2; k++)
        for (size_t w = 0; w < n / 64; w++) {
          lo[k] = std::min(lo[k], h[k * tb / 8 + 2 * w]);
          hi[k] = std::max(hi[k], h[k * tb / 8 + 2 * w + 1]);
        }
      printf("  (c) traced: %.2f us per launch, waves' span %.2f / %.2f us, gap between launches %.2f us\n",
             us, (hi[0] - lo[0]) / 100.0, (hi[1] - lo[1]) / 100.0,
             (lo[0] > hi[1] ? (double)(lo[0] - hi[1]) : (double)(lo[1] - hi[0])) / 100.0);
      {
        BigArgs ba{};
        ba.n = n;
        ba.verdict = verdict;
        const float us3 = time_it([&](int i) {
          ba.frames = fr[i % pool];
          ba.tr = tr + (i & 1) * (tb / 8);
          sol_lds_bigargs<<<grid, 256, 4 * 4608>>>(ba);
        });
        hipMemcpy(h.data(), tr, 2 * tb, hipMemcpyDeviceToHost);
        uint64_t l3[2] = {~0ull, ~0ull}, h3[2] = {0, 0};
        for (int k = 0; k < 2; k++)
          for (size_t w = 0; w < n / 64; w++) {
            l3[k] = std::min(l3[k], h[k * tb / 8 + 2 * w]);
            h3[k] = std::max(h3[k], h[k * tb / 8 + 2 * w + 1]);
          }
        printf("  (h) traced, 464-byte kernarg segment: %.2f us per launch, span %.2f us, gap %.2f us\n",
               us3, (h3[0] - l3[0]) / 100.0,
               (l3[0] > h3[1] ? (double)(l3[0] - h3[1]) : (double)(l3[1] - h3[0])) / 100.0);
      }
      {  // (c) traced, launched from a code object with hipModuleLaunchKernel (as compiled programs)
        hipModule_t mod;
        hipFunction_t fn;
        if (hipModuleLoad(&mod, "tools/bin/sol_stream.co") == hipSuccess &&
            hipModuleGetFunction(&fn, mod, "_Z13sol_lds_traceILb0EEvPKhmPhPm") == hipSuccess) {
          struct {
            const uint8_t* f;
            uint64_t n;
            uint8_t* v;
            uint64_t* t;
          } ka;
          ka.n = n;
          ka.v = verdict;
          const float us4 = time_it([&](int i) {
            ka.f = fr[i % pool];
            ka.t = tr + (i & 1) * (tb / 8);
            size_t sz = sizeof(ka);
            void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &ka, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz,
                           HIP_LAUNCH_PARAM_END};
            hipModuleLaunchKernel(fn, grid, 1, 1, 256, 1, 1, 4 * 4608, nullptr, nullptr, cfg);
          });
          hipMemcpy(h.data(), tr, 2 * tb, hipMemcpyDeviceToHost);
          uint64_t l4[2] = {~0ull, ~0ull}, h4[2] = {0, 0};
          for (int k = 0; k < 2; k++)
            for (size_t w = 0; w < n / 64; w++) {
              l4[k] = std::min(l4[k], h[k * tb / 8 + 2 * w]);
              h4[k] = std::max(h4[k], h[k * tb / 8 + 2 * w + 1]);
            }
          printf("  (m) traced (c) via hipModuleLaunchKernel: %.2f us per launch, span %.2f us, gap %.2f us\n",
                 us4, (h4[0] - l4[0]) / 100.0,
                 (l4[0] > h4[1] ? (double)(l4[0] - h4[1]) : (double)(l4[1] - h4[0])) / 100.0);
        } else {
          printf("  (m) no tools/bin/sol_stream.co\n");
        }
      }
      for (int big = 0; big < 2; big++) {
        const float us2 = time_it([&](int i) {
          if (big)
            sol_lds_res<true><<<grid, 256, 4 * 8192>>>(fr[i % pool], n, verdict, tr + (i & 1) * (tb / 8));
          else
            sol_lds_res<false><<<grid, 256, 4 * 4608>>>(fr[i % pool], n, verdict, tr + (i & 1) * (tb / 8));
        });
        hipMemcpy(h.data(), tr, 2 * tb, hipMemcpyDeviceToHost);
        uint64_t l2[2] = {~0ull, ~0ull}, h2[2] = {0, 0};
        for (int k = 0; k < 2; k++)
          for (size_t w = 0; w < n / 64; w++) {
            l2[k] = std::min(l2[k], h[k * tb / 8 + 2 * w]);
            h2[k] = std::max(h2[k], h[k * tb / 8 + 2 * w + 1]);
          }
        printf("  (g%d) traced, %s: %.2f us per launch, span %.2f us, gap %.2f us\n", big,
               big ? "32 KiB LDS/WG, 82 VGPR, 100 SGPR" : "as (c)", us2, (h2[0] - l2[0]) / 100.0,
               (l2[0] > h2[1] ? (double)(l2[0] - h2[1]) : (double)(l2[1] - h2[0])) / 100.0);
      }
      hipFree(tr);
    }
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
