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

// Config 5 whole, unbinned: every wave takes 64 consecutive packets of the 50/50 mix (no length
// order). Short packets (< 128 B): each lane reads its own 64 bytes (four dwordx4). Long ones: the
// whole wave walks them one packet at a time, 64 lanes x 16 B per load instruction (1 KiB
// contiguous, two loads for 1500 B), with D packets' loads in flight; the per-packet sum is reduced
// across the wave and lands in the packet's lane.
template <uint32_t D>
__global__ __launch_bounds__(256) void scan_unbinned(const uint8_t* frames, const uint32_t* offs,
                                                     const uint16_t* lens, uint64_t n, uint32_t* out) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t tile = (uint64_t)blockIdx.x * 4 + threadIdx.x / 64;
  if (tile * 64 >= n) return;
  const uint64_t me = tile * 64 + lane;
  const uint32_t my_off = me < n ? offs[me] : 0, my_len = me < n ? lens[me] : 0;
  uint32_t mine = 0;
  const bool lng = my_len >= 128;
  if (!lng && my_len) {
    const uint4* p = (const uint4*)(frames + my_off);
    for (uint32_t c = 0; c < 4; c++) {
      uint4 v = p[c];
      mine = sad4(v, mine);
    }
  }
  uint64_t mask = __ballot(lng);
  // ring of D packets in flight: lane reads 16 B at +16*lane and +1024+16*lane
  uint4 b0[D], b1[D];
  uint32_t who[D];
  auto issue = [&](uint32_t s) {
    if (mask) {
      const uint32_t l = __builtin_ctzll(mask);
      mask &= mask - 1;
      who[s] = l;
      const uint32_t o = __shfl(my_off, (int)l), ln = __shfl(my_len, (int)l);
      const uint8_t* p = frames + o + lane * 16;
      b0[s] = lane * 16 < ln ? *(const uint4*)p : make_uint4(0, 0, 0, 0);
      b1[s] = 1024 + lane * 16 < ln ? *(const uint4*)(p + 1024) : make_uint4(0, 0, 0, 0);
    } else {
      who[s] = 64;
    }
  };
#pragma unroll
  for (uint32_t s = 0; s < D; s++) issue(s);
  for (;;) {
    bool any = false;
#pragma unroll
    for (uint32_t s = 0; s < D; s++) {
      if (who[s] == 64) continue;
      any = true;
      uint32_t v = sad4(b1[s], sad4(b0[s], 0));
      for (int m = 32; m; m >>= 1) v += __shfl_xor(v, m);
      if (lane == who[s]) mine = v;
      issue(s);
    }
    if (!any) break;
  }
  if (me < n) out[me] = mine;
}

// Config 5 whole, unbinned, the long packets compacted: lanes whose packet has >= 128 bytes get
// ranks 0..C-1; groups of 32 of them are walked 128 bytes per packet per round (8 lanes x 16 B
// per packet, 8 packets per load instruction, four instructions per round, full 128-byte lines),
// with the next round's loads in flight (PF). Short packets: each lane reads its 64 bytes.
template <bool PF>
__global__ __launch_bounds__(256) void scan_unbinned_c128(const uint8_t* frames, const uint32_t* offs,
                                                          const uint16_t* lens, uint64_t n,
                                                          uint32_t* out) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t tile = (uint64_t)blockIdx.x * 4 + threadIdx.x / 64;
  if (tile * 64 >= n) return;
  const uint64_t me = tile * 64 + lane;
  const uint32_t my_off = me < n ? offs[me] : 0, my_len = me < n ? lens[me] : 0;
  uint32_t mine = 0;
  const bool lng = my_len >= 128;
  if (!lng && my_len) {
    const uint4* p = (const uint4*)(frames + my_off);
    for (uint32_t c = 0; c < 4; c++) {
      uint4 v = p[c];
      mine = sad4(v, mine);
    }
  }
  const uint64_t mask = __ballot(lng);
  const uint32_t C = __popcll(mask);
  const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                                  __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0));
  // srcl[r] = the lane of rank r (a full permutation: the short lanes take ranks C..63)
  const uint32_t srank = lng ? rank : C + (lane - rank);
  const int srcl = __builtin_amdgcn_ds_permute((int)(srank * 4), (int)lane);
  const uint32_t sub = (lane & 7) * 16;
  for (uint32_t g = 0; g * 32 < C; g++) {
    uint32_t o[4], hi[4], acc[4];
    uint32_t mx = 0;
#pragma unroll
    for (uint32_t k = 0; k < 4; k++) {
      const uint32_t r = 32 * g + 8 * k + lane / 8;
      const int s = __builtin_amdgcn_ds_bpermute((int)(r * 4), srcl);
      o[k] = (uint32_t)__builtin_amdgcn_ds_bpermute(s * 4, (int)my_off) + sub;
      hi[k] = r < C ? (uint32_t)__builtin_amdgcn_ds_bpermute(s * 4, (int)my_len) : 0u;
      acc[k] = 0;
      mx = max(mx, hi[k]);
    }
    for (int m = 32; m; m >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, m));
    uint4 cur[4], nxt[4];
#pragma unroll
    for (uint32_t k = 0; k < 4; k++)
      cur[k] = sub < hi[k] ? *(const uint4*)(frames + o[k]) : make_uint4(0, 0, 0, 0);
    for (uint32_t W = 0; W < mx; W += 128) {
      if (PF) {
#pragma unroll
        for (uint32_t k = 0; k < 4; k++)
          nxt[k] = W + 128 + sub < hi[k] ? *(const uint4*)(frames + o[k] + W + 128)
                                         : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (uint32_t k = 0; k < 4; k++) {
        if (W + sub + 16 <= hi[k]) acc[k] = sad4(cur[k], acc[k]);
        else if (W + sub < hi[k]) {  // a partial last chunk
          const uint32_t b = hi[k] - W - sub;
          uint32_t w[4] = {cur[k].x, cur[k].y, cur[k].z, cur[k].w};
          for (uint32_t d = 0; d < 4; d++) {
            const int keep = (int)b - (int)(4 * d);
            const uint32_t m = keep >= 4 ? 0xffffffffu : keep <= 0 ? 0u : (1u << (8 * keep)) - 1;
            acc[k] = __builtin_amdgcn_sad_u8(w[d] & m, 0, acc[k]);
          }
        }
      }
      if (PF) {
#pragma unroll
        for (uint32_t k = 0; k < 4; k++) cur[k] = nxt[k];
      } else {
#pragma unroll
        for (uint32_t k = 0; k < 4; k++)
          cur[k] = W + 128 + sub < hi[k] ? *(const uint4*)(frames + o[k] + W + 128)
                                         : make_uint4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (uint32_t k = 0; k < 4; k++) {
      acc[k] += __shfl_xor((int)acc[k], 1);
      acc[k] += __shfl_xor((int)acc[k], 2);
      acc[k] += __shfl_xor((int)acc[k], 4);
    }
    // the lane of rank r (group g) takes slot k = (r % 32) / 8, lane 8 * (r % 8)
    const uint32_t kk = (rank % 32) / 8, from = 8 * (rank % 8);
    const uint32_t v0 = (uint32_t)__shfl((int)acc[0], (int)from), v1 = (uint32_t)__shfl((int)acc[1], (int)from),
                   v2 = (uint32_t)__shfl((int)acc[2], (int)from), v3 = (uint32_t)__shfl((int)acc[3], (int)from);
    if (lng && rank / 32 == g) mine = kk == 0 ? v0 : kk == 1 ? v1 : kk == 2 ? v2 : v3;
  }
  if (me < n) out[me] = mine;
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
    {  // the whole mixed batch, unbinned, packet per instruction, D packets in flight
      std::vector<uint32_t> offs(np);
      std::vector<uint16_t> lens(np);
      uint64_t p2 = 0, y = 0x5EED0005ull, tot = 0;
      for (uint64_t i = 0; i < np; i++) {
        y = y * 6364136223846793005ull + 1442695040888963407ull;
        const bool lng = (y >> 33) & 1;
        offs[i] = (uint32_t)p2;
        lens[i] = lng ? 1500 : 64;
        tot += lens[i];
        p2 += lng ? 1536 : 64;
      }
      uint32_t *d_off, *o2;
      uint16_t* d_len;
      if (hipMalloc(&d_off, np * 4) != hipSuccess || hipMalloc(&d_len, np * 2) != hipSuccess ||
          hipMalloc(&o2, np * 4) != hipSuccess)
        return 1;
      (void)hipMemcpy(d_off, offs.data(), np * 4, hipMemcpyHostToDevice);
      (void)hipMemcpy(d_len, lens.data(), np * 2, hipMemcpyHostToDevice);
      const int g2 = (int)((np / 64 + 3) / 4);
      auto run = [&](auto kern, const char* name, uint32_t lds) {
        hipEvent_t a, b;
        (void)hipEventCreate(&a);
        (void)hipEventCreate(&b);
        for (int i = 0; i < 3; i++)
          hipLaunchKernelGGL(kern, dim3(g2), dim3(256), lds, 0, mf, d_off, d_len, np, o2);
        (void)hipEventRecord(a);
        for (int i = 0; i < 20; i++)
          hipLaunchKernelGGL(kern, dim3(g2), dim3(256), lds, 0, mf, d_off, d_len, np, o2);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        const float us = ms * 1000.f / 20.f;
        printf("unbinned mixed 1 Mi, packet/instr, %-22s lds %6u %9.1f us  %7.0f GB/s\n", name, lds,
               us, (double)(tot + np * 7) / (us * 1e3));
      };
      for (uint32_t lds : {0u, 31u * 1024, 39u * 1024}) {
        run(scan_unbinned<1>, "D=1", lds);
        run(scan_unbinned<2>, "D=2", lds);
        run(scan_unbinned<4>, "D=4", lds);
        run(scan_unbinned_c128<true>, "c128 prefetch", lds);
        run(scan_unbinned_c128<false>, "c128 no prefetch", lds);
        std::vector<uint32_t> got(np);
        (void)hipMemcpy(got.data(), o2, np * 4, hipMemcpyDeviceToHost);
        uint64_t bad = 0;
        for (uint64_t i = 0; i < np; i++) bad += got[i] != lens[i];  // (every byte is 1)
        printf("c128 sums wrong: %llu of %llu\n", (unsigned long long)bad, (unsigned long long)np);
      }
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
