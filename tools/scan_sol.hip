// scan_sol.hip -- speed-of-light for the loop kernel's refill pattern (measurement tool, not part
// of the product): every wave scans the 1500 bytes of each of its 64 packets (1536-byte slots,
// 512 Ki packets = config 5's long half), transposed as the refills are, with the next step's loads
// in flight while the current one is consumed (v_sad_u8 into a per-lane sum). The step width W
// sets how many lanes read one packet per load instruction:
//   W =   64: 4 lanes x 16 B per packet, 16 packets per instruction (today's refills);
//   W =  128: 8 lanes per packet -- one full 128-byte line per packet per instruction;
//   W =  256: 16 lanes per packet (no prefetch: the registers of one step only);
//   W = 1024: 64 lanes per packet, one packet per instruction.
// Also at 6 / 5 / 4 / 3 waves per SIMD (occupancy capped with dynamic LDS).
// Prints microseconds per batch (one event pair around 20 launches) and the GB/s of packet bytes.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/scan_sol tools/scan_sol.hip && /tmp/scan_sol
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

constexpr uint32_t kLen = 1500, kSlot = 1536;

__device__ __forceinline__ uint32_t sad4(uint4 v, uint32_t acc) {
  acc = __builtin_amdgcn_sad_u8(v.x, 0, acc);
  acc = __builtin_amdgcn_sad_u8(v.y, 0, acc);
  acc = __builtin_amdgcn_sad_u8(v.z, 0, acc);
  return __builtin_amdgcn_sad_u8(v.w, 0, acc);
}

// W-byte steps, R = W / 64 * 4 load instructions per step (lanes per packet = W / 16)
template <uint32_t W, bool PREFETCH>
__global__ __launch_bounds__(256) void scan(const uint8_t* frames, uint64_t n, uint32_t* out) {
  constexpr uint32_t LPP = W / 16;          // lanes per packet
  constexpr uint32_t PPI = 64 / LPP;        // packets per instruction
  constexpr uint32_t R = 64 / PPI;          // instructions per step (64 packets)
  constexpr uint32_t STEPS = (kLen + W - 1) / W;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t tile = (uint64_t)blockIdx.x * 4 + threadIdx.x / 64;
  if (tile * 64 >= n) return;
  const uint32_t sub = lane % LPP, pk = lane / LPP;
  const uint8_t* base[R];
#pragma unroll
  for (uint32_t r = 0; r < R; r++) base[r] = frames + (tile * 64 + r * PPI + pk) * kSlot + sub * 16;
  uint32_t acc = 0;
  uint4 cur[R], nxt[R];
#pragma unroll
  for (uint32_t r = 0; r < R; r++)
    cur[r] = sub * 16 < kLen ? *(const uint4*)base[r] : make_uint4(0, 0, 0, 0);
  for (uint32_t s = 0; s < STEPS; s++) {
    const uint32_t o = (s + 1) * W + sub * 16;
    if (PREFETCH) {
#pragma unroll
      for (uint32_t r = 0; r < R; r++)
        nxt[r] = o < kLen ? *(const uint4*)(base[r] + (s + 1) * W) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (uint32_t r = 0; r < R; r++) acc = sad4(cur[r], acc);
    if (PREFETCH) {
#pragma unroll
      for (uint32_t r = 0; r < R; r++) cur[r] = nxt[r];
    } else {
#pragma unroll
      for (uint32_t r = 0; r < R; r++)
        cur[r] = o < kLen ? *(const uint4*)(base[r] + (s + 1) * W) : make_uint4(0, 0, 0, 0);
    }
  }
  out[tile * 64 + lane] = acc;
}

// one packet per instruction: 64 lanes x 16 B = 1 KiB contiguous, the next packet in flight
__global__ __launch_bounds__(256) void scan_packet(const uint8_t* frames, uint64_t n, uint32_t* out) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t tile = (uint64_t)blockIdx.x * 4 + threadIdx.x / 64;
  if (tile * 64 >= n) return;
  const uint8_t* b = frames + tile * 64 * kSlot + lane * 16;
  uint32_t acc = 0, mine = 0;
  const bool two = 1024 + lane * 16 < kLen;
  uint4 c0 = *(const uint4*)b, c1 = two ? *(const uint4*)(b + 1024) : make_uint4(0, 0, 0, 0);
  for (uint32_t p = 0; p < 64; p++) {
    const uint8_t* nb = b + (p + 1) * kSlot;
    uint4 n0 = make_uint4(0, 0, 0, 0), n1 = n0;
    if (p + 1 < 64) {
      n0 = *(const uint4*)nb;
      if (two) n1 = *(const uint4*)(nb + 1024);
    }
    uint32_t s = sad4(c1, sad4(c0, 0));
    for (int m = 32; m; m >>= 1) s += __shfl_xor(s, m);
    if (lane == p) mine = s;
    acc += s;
    c0 = n0;
    c1 = n1;
  }
  out[tile * 64 + lane] = mine ^ (acc & 1);
}

// The same scan over config 5's layout: 50/50 64/1500-byte frames in 64-byte aligned slots, each
// tile the next 64 long packets in index order (length-binned), offsets read per lane.
__global__ __launch_bounds__(256) void scan_mixed(const uint8_t* frames, const uint64_t* offs,
                                                  uint64_t n, uint32_t* out) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t tile = (uint64_t)blockIdx.x * 4 + threadIdx.x / 64;
  if (tile * 64 >= n) return;
  const uint32_t sub = lane % 4, pk = lane / 4;
  const uint8_t* base[4];
#pragma unroll
  for (uint32_t r = 0; r < 4; r++) base[r] = frames + offs[tile * 64 + r * 16 + pk] + sub * 16;
  uint32_t acc = 0;
  for (uint32_t s = 0; s < (kLen + 63) / 64; s++) {
    uint4 c[4];
    const uint32_t o = s * 64 + sub * 16;
#pragma unroll
    for (uint32_t r = 0; r < 4; r++) c[r] = o < kLen ? *(const uint4*)(base[r] + s * 64) : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (uint32_t r = 0; r < 4; r++) acc = sad4(c[r], acc);
  }
  out[tile * 64 + lane] = acc;
}

// scan_mixed behind the loop kernel's tile prologue: the binned order's index (perm), the
// offset through it, the first 64-byte window of every packet (four transposed loads), each level
// waiting for the one before -- three dependent HBM round trips before the scan starts.
__global__ __launch_bounds__(256) void scan_mixed_prologue(const uint8_t* frames, const uint64_t* offs,
                                                           const uint32_t* perm, uint64_t n,
                                                           uint32_t* out) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t tile = (uint64_t)blockIdx.x * 4 + threadIdx.x / 64;
  if (tile * 64 >= n) return;
  const uint32_t src = perm[tile * 64 + lane];
  const uint64_t my = offs[src];
  const uint32_t sub = lane % 4, pk = lane / 4;
  uint32_t acc = 0;
  const uint8_t* base[4];
#pragma unroll
  for (uint32_t r = 0; r < 4; r++)
    base[r] = frames + __shfl(my, (int)(r * 16 + pk)) + sub * 16;
  {
    uint4 w[4];
#pragma unroll
    for (uint32_t r = 0; r < 4; r++) w[r] = *(const uint4*)base[r];
#pragma unroll
    for (uint32_t r = 0; r < 4; r++) acc = sad4(w[r], acc) & 1;
  }
  for (uint32_t s = 0; s < (kLen + 63) / 64; s++) {
    uint4 c[4];
    const uint32_t o = s * 64 + sub * 16;
#pragma unroll
    for (uint32_t r = 0; r < 4; r++) c[r] = o < kLen ? *(const uint4*)(base[r] + s * 64) : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (uint32_t r = 0; r < 4; r++) acc = sad4(c[r], acc);
  }
  out[tile * 64 + lane] = acc;
}

template <typename K>
static float time_it(K kernel, const uint8_t* f, uint64_t n, uint32_t* o, uint32_t lds = 0) {
  const int grid = (int)((n / 64 + 3) / 4);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int i = 0; i < 3; i++) hipLaunchKernelGGL(kernel, dim3(grid), dim3(256), lds, 0, f, n, o);
  (void)hipEventRecord(a);
  for (int i = 0; i < 20; i++) hipLaunchKernelGGL(kernel, dim3(grid), dim3(256), lds, 0, f, n, o);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms * 1000.f / 20.f;
}

int main() {
  const uint64_t n = 512 * 1024;
  uint8_t* f;
  uint32_t* o;
  if (hipMalloc(&f, n * kSlot) != hipSuccess || hipMalloc(&o, n * 4) != hipSuccess) return 1;
  (void)hipMemset(f, 1, n * kSlot);
  const double bytes = (double)n * kLen;
  struct {
    const char* name;
    float us;
  } r[] = {
      {"W=64 prefetch", time_it(scan<64, true>, f, n, o)},
      {"W=64 no prefetch", time_it(scan<64, false>, f, n, o)},
      {"W=128 prefetch", time_it(scan<128, true>, f, n, o)},
      {"W=128 no prefetch", time_it(scan<128, false>, f, n, o)},
      {"W=256 no prefetch", time_it(scan<256, false>, f, n, o)},
      {"W=1024 (packet per instruction)", time_it(scan_packet, f, n, o)},
      // occupancy capped by dynamic LDS (blocks of 4 waves per CU: 160 KiB / bytes)
      {"W=64 prefetch, 6 waves/SIMD", time_it(scan<64, true>, f, n, o, 26 * 1024)},
      {"W=64 prefetch, 5 waves/SIMD", time_it(scan<64, true>, f, n, o, 31 * 1024)},
      {"W=64 prefetch, 4 waves/SIMD", time_it(scan<64, true>, f, n, o, 39 * 1024)},
      {"W=64 prefetch, 3 waves/SIMD", time_it(scan<64, true>, f, n, o, 52 * 1024)},
      {"W=128 prefetch, 5 waves/SIMD", time_it(scan<128, true>, f, n, o, 31 * 1024)},
      {"W=128 prefetch, 4 waves/SIMD", time_it(scan<128, true>, f, n, o, 39 * 1024)},
  };
  for (auto& x : r) printf("%-34s %9.1f us  %7.0f GB/s\n", x.name, x.us, bytes / (x.us * 1e3));
  // config 5's layout: 1 Mi packets, half long, 64-byte aligned slots
  {
    const uint64_t np = 1 << 20;
    std::vector<uint64_t> off_long;
    uint64_t pos = 0, x = 0x5EED0005ull;
    for (uint64_t i = 0; i < np; i++) {
      x = x * 6364136223846793005ull + 1442695040888963407ull;
      const bool lng = (x >> 33) & 1;
      if (lng) off_long.push_back(pos);
      pos += lng ? 1536 : 64;
    }
    const uint64_t nl = off_long.size() / 64 * 64;
    uint8_t* mf;
    uint64_t* mo;
    if (hipMalloc(&mf, pos) != hipSuccess || hipMalloc(&mo, nl * 8) != hipSuccess) return 1;
    (void)hipMemset(mf, 1, pos);
    (void)hipMemcpy(mo, off_long.data(), nl * 8, hipMemcpyHostToDevice);
    const int grid = (int)((nl / 64 + 3) / 4);
    std::vector<uint32_t> idp(nl);
    for (uint64_t i = 0; i < nl; i++) idp[i] = (uint32_t)i;
    uint32_t* pm;
    if (hipMalloc(&pm, nl * 4) != hipSuccess) return 1;
    (void)hipMemcpy(pm, idp.data(), nl * 4, hipMemcpyHostToDevice);
    for (uint32_t lds : {0u, 31u * 1024}) {
      hipEvent_t a, b;
      (void)hipEventCreate(&a);
      (void)hipEventCreate(&b);
      for (int i = 0; i < 3; i++)
        hipLaunchKernelGGL(scan_mixed_prologue, dim3(grid), dim3(256), lds, 0, mf, mo, pm, nl, o);
      (void)hipEventRecord(a);
      for (int i = 0; i < 20; i++)
        hipLaunchKernelGGL(scan_mixed_prologue, dim3(grid), dim3(256), lds, 0, mf, mo, pm, nl, o);
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, a, b);
      const float us = ms * 1000.f / 20.f;
      printf("mixed layout + tile prologue, %s %9.1f us\n", lds ? "5 waves/SIMD" : "full occupancy", us);
    }
    for (uint32_t lds : {0u, 31u * 1024}) {
      hipEvent_t a, b;
      (void)hipEventCreate(&a);
      (void)hipEventCreate(&b);
      for (int i = 0; i < 3; i++) hipLaunchKernelGGL(scan_mixed, dim3(grid), dim3(256), lds, 0, mf, mo, nl, o);
      (void)hipEventRecord(a);
      for (int i = 0; i < 20; i++) hipLaunchKernelGGL(scan_mixed, dim3(grid), dim3(256), lds, 0, mf, mo, nl, o);
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, a, b);
      const float us = ms * 1000.f / 20.f;
      printf("mixed layout, %u long packets, %s %9.1f us  %7.0f GB/s\n", (unsigned)nl,
             lds ? "5 waves/SIMD" : "full occupancy", us, (double)nl * kLen / (us * 1e3));
    }
  }
  return 0;
}
