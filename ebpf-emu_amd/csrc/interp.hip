// interp.hip — the batched eBPF/XDP interpreter for MI355X (gfx950 / CDNA4).
//
// Replaces the reference's fetch-decode-execute loop (src/emu.rs:48-458) and flat memory
// (src/mmu.rs:1-31). One lane interprets the program over one packet; one wave64 holds 64
// packets (a "tile"). Design:
//   * the pre-decoded micro-op table (uop.h) is staged ONCE per workgroup in LDS; a fetch is a
//     wave-uniform LDS broadcast read whose fields go to SGPRs (readfirstlane), so dispatch is a
//     scalar branch and register indices are scalar (s_set_gpr_idx VGPR indexing, no scratch);
//   * re-convergence by min-pc: lanes whose pc equals the wave's minimum pc execute the step;
//     the all-lanes-agree case is one readfirstlane + one compare-ballot, the divergent case a
//     DPP wave-min. Lanes that are done (exit, fall-off, fault) park at pc = 0xFFFFFFFF;
//   * memory tier 0 (programs without stores/calls): the first 64 bytes of each packet (its
//     "header window") are copied HBM -> LDS by LDS-DMA (global_load_lds_dwordx4: 16 packets x
//     64 contiguous bytes per wave instruction, no VGPR destination), double-buffered so that
//     the windows of the wave's next tile land while the current tile is interpreted; reads
//     beyond the window go to HBM with dword-aligned loads; bytes past the packet read as
//     zero, exactly as the reference's zeroed image does;
//   * memory tier 1 (stores, atomics or calls present): each lane owns a lane-interleaved copy
//     of the reference's whole memory image plus a frame stack in device scratch;
//   * every mmu.rs bounds check is inlined; faults become per-packet status codes.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdlib>
#include <map>
#include <mutex>
#include <tuple>

#include "../../include/ebpf_emu.h"
#include "dag_asm.h"
#include "launch.h"
#include "uop.h"

namespace ebpfemu {

__device__ __forceinline__ uint32_t rfl(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t rfl64(uint64_t v) {
  return (uint64_t)rfl((uint32_t)v) | ((uint64_t)rfl((uint32_t)(v >> 32)) << 32);
}
__device__ __forceinline__ uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }

// Minimum over the 64 lanes (all lanes active) — DPP row shifts + row broadcasts (gfx9 DPP).
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x111, 0xf, 0xf, false));
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x112, 0xf, 0xf, false));
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x114, 0xf, 0xf, false));
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x118, 0xf, 0xf, false));
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x142, 0xa, 0xf, false));
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x143, 0xc, 0xf, false));
  return __builtin_amdgcn_readlane(v, 63);
}

// Sum over the 64 lanes (all lanes active), 64-bit: the same DPP pattern as wave_min_u32 (row
// prefix sums, then rows 1/3 take row 0/2's total, rows 2/3 take lanes 0-31's), lane 63's value.
#define WAVE_SUM_STEP(ctrl, rows)                                                              \
  do {                                                                                         \
    const uint32_t lo_ = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, ctrl, rows, \
                                                               0xf, true);                      \
    const uint32_t hi_ = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v >> 32),    \
                                                               ctrl, rows, 0xf, true);          \
    v += (uint64_t)lo_ | ((uint64_t)hi_ << 32);                                                \
  } while (0)
__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
  WAVE_SUM_STEP(0x111, 0xf);
  WAVE_SUM_STEP(0x112, 0xf);
  WAVE_SUM_STEP(0x114, 0xf);
  WAVE_SUM_STEP(0x118, 0xf);
  WAVE_SUM_STEP(0x142, 0xa);
  WAVE_SUM_STEP(0x143, 0xc);
  return (uint64_t)__builtin_amdgcn_readlane((uint32_t)v, 63) |
         ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(v >> 32), 63) << 32);
}
#undef WAVE_SUM_STEP

// 32-bit: one DPP add per step
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, true);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, true);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, true);
  return __builtin_amdgcn_readlane(v, 63);
}

// Explicit global (address space 1) accesses: pointers carried in LaunchArgs would otherwise be
// generic and lower to flat_* instructions (which also count against lgkmcnt).
typedef __attribute__((address_space(1))) const uint8_t g_u8;
typedef __attribute__((address_space(1))) const uint32_t g_u32;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 g_u4;
__device__ __forceinline__ uint32_t gld8(uintptr_t p) { return *(g_u8*)p; }
__device__ __forceinline__ uint32_t gld32(uintptr_t p) { return *(g_u32*)p; }
__device__ __forceinline__ uint4 gld128(uintptr_t p) {
  const u32x4 v = *(g_u4*)p;
  return make_uint4(v.x, v.y, v.z, v.w);
}

// Set of pcs at which some lane of the wave is parked, for programs of up to 64 * NW micro-ops:
// the next pc to run is its lowest member (s_ff1), replacing a per-step wave-wide min.
template <int NW>
struct PcSet {  // NW in {0 (unused), 1, 4}; words are named scalars (SGPRs), never an array
  uint64_t w0, w1, w2, w3;
  __device__ __forceinline__ void init(bool any) {
    w0 = any ? 1ull : 0ull;  // every lane starts at pc 0
    w1 = w2 = w3 = 0;
  }
  __device__ __forceinline__ uint32_t first() const {
    if (w0) return (uint32_t)__builtin_ctzll(w0);
    if (NW > 1) {
      if (w1) return 64u + (uint32_t)__builtin_ctzll(w1);
      if (w2) return 128u + (uint32_t)__builtin_ctzll(w2);
      if (w3) return 192u + (uint32_t)__builtin_ctzll(w3);
    }
    return PC_DONE;
  }
  __device__ __forceinline__ void add(uint32_t p) {
    const uint64_t bit = 1ull << (p & 63);
    if (NW == 1 || p < 64) w0 |= bit;
    else if (p < 128) w1 |= bit;
    else if (p < 192) w2 |= bit;
    else w3 |= bit;
  }
  __device__ __forceinline__ void del(uint32_t p) {
    const uint64_t bit = ~(1ull << (p & 63));
    if (NW == 1 || p < 64) w0 &= bit;
    else if (p < 128) w1 &= bit;
    else if (p < 192) w2 &= bit;
    else w3 &= bit;
  }
};

__device__ __forceinline__ uint64_t wmask(uint32_t w) {
  return w >= 8 ? ~0ull : ((1ull << (8 * w)) - 1);
}

__device__ __forceinline__ uint32_t bswap32(uint32_t v) { return __builtin_bswap32(v); }

// Bytes [a, a+w) of a packet at `base` whose length is len, with a < len; bytes at or past len
// read as zero (the zeroed image, main.rs:16). Only dwords holding at least one packet byte
// are loaded, so no access leaves the page of a valid byte.
__device__ __forceinline__ uint64_t pkt_read(const uint8_t* base, uint32_t a, uint32_t w,
                                             uint32_t len) {
  if (w == 1) return gld8((uintptr_t)base + a);
  const uintptr_t p = (uintptr_t)base + a;
  const uintptr_t end = (uintptr_t)base + len;
  const uintptr_t p4 = p & ~(uintptr_t)3;
  const uint32_t s = (uint32_t)(p & 3);
  const uint32_t d0 = gld32(p4);
  const uint32_t d1 = (p4 + 4 < end) ? gld32(p4 + 4) : 0u;
  uint64_t v = __builtin_amdgcn_alignbyte(d1, d0, s);
  if (w == 8) {
    const uint32_t d2 = (p4 + 8 < end) ? gld32(p4 + 8) : 0u;
    v |= (uint64_t)__builtin_amdgcn_alignbyte(d2, d1, s) << 32;
  }
  const uint32_t valid = len - a;
  if (valid < w) v &= wmask(valid);
  return v & wmask(w);
}

// Header window layout (per wave, per buffer): packet j's 64 bytes at j * 64, its 16-byte
// chunk c stored at chunk slot c ^ swz(j), swz(j) = (j >> 2) & 3. The XOR is applied on the
// DMA's SOURCE addresses (the LDS side of an LDS-DMA is lane-linear), and spreads the 16 packets
// of each ds_read_b128 lane group over all 16 four-bank groups.
__device__ __forceinline__ uint32_t win_swz(uint32_t j) { return (j >> 2) & 3; }

// LDS byte offset of logical window byte b (multiple of 4) of the packet whose window starts at
// pw (swz = win_swz of that packet).
__device__ __forceinline__ uint32_t win_off(uint32_t b, uint32_t swz) {
  return ((((b >> 4) ^ swz) << 4) | (b & 15)) & 63;
}

// Bytes [a, a+w) of the lane's window, a < len, a + w <= kWin; bytes at or past len are 0.
__device__ __forceinline__ uint64_t win_read(const uint8_t* pw, uint32_t swz, uint32_t a, uint32_t w,
                                             uint32_t len) {
  const uint32_t b0 = a & ~3u, s = a & 3;
  const uint32_t d0 = *(const uint32_t*)(pw + win_off(b0, swz));
  const uint32_t d1 = *(const uint32_t*)(pw + win_off(b0 + 4, swz));  // in-window wrap if unused
  uint64_t v = __builtin_amdgcn_alignbyte(d1, d0, s);
  if (w == 8) {
    const uint32_t d2 = *(const uint32_t*)(pw + win_off(b0 + 8, swz));
    v |= (uint64_t)__builtin_amdgcn_alignbyte(d2, d1, s) << 32;
  }
  const uint32_t valid = len - a;
  if (valid < w) v &= wmask(valid);
  return v & wmask(w);
}

// ---- LDS-DMA (global_load_lds_*): lane i's data lands at lds_dst + i * max(size, 4) ----
// Hand-written per MI355X guide §5.7: M0 is written in the same statement that reads it, and the
// transfer is invisible to hipcc's s_waitcnt bookkeeping, so completion is waited for explicitly
// (dma_wait) before the wave reads the buffer.
__device__ __forceinline__ void dma_x4(uintptr_t gsrc, uint32_t lds_dst) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds_dst) : "memory");
}
__device__ __forceinline__ void dma_x1(uintptr_t gsrc, uint32_t lds_dst) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds_dst) : "memory");
}
__device__ __forceinline__ void dma_u16(uintptr_t gsrc, uint32_t lds_dst) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_ushort %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds_dst) : "memory");
}
__device__ __forceinline__ void dma_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return rfl((uint32_t)(uintptr_t)(__attribute__((address_space(3))) const void*)p);
}

// Dword d of a final image (mem_out row of mem_size bytes, any length): one dword store when the
// row is dword-aligned, else its in-bounds bytes one by one (the reference's Mmu.memory is a Vec<u8>
// of any length, mmu.rs:2-4).
__device__ __forceinline__ void put_image(uint8_t* row, uint32_t d, uint32_t v, uint32_t mem_size) {
  if ((mem_size & 3) == 0) {
    ((uint32_t*)row)[d] = v;
    return;
  }
  for (uint32_t i = 0; i < 4 && d * 4 + i < mem_size; i++) row[d * 4 + i] = (uint8_t)(v >> (8 * i));
}

// ---- tier-1 image: lane-interleaved dwords, dword d of this lane at img[d * 64] (materialised
// lazily, interp_kernel: lazy_read / lazy_write) ----
__device__ __forceinline__ void img_write(uint32_t* img, uint32_t a, uint32_t w, uint64_t v) {
  uint32_t* p = img + (size_t)(a >> 2) * kWave;
  const uint32_t s = a & 3;
  if (w == 1) {
    ((uint8_t*)p)[s] = (uint8_t)v;
    return;
  }
  const uint64_t m = wmask(w);
  const uint64_t vm = v & m;
  const uint64_t m01 = m << (8 * s), v01 = vm << (8 * s);
  const uint32_t mlo = (uint32_t)m01, mhi = (uint32_t)(m01 >> 32);
  if (mlo) p[0] = (p[0] & ~mlo) | (uint32_t)v01;
  if (mhi) p[kWave] = (p[kWave] & ~mhi) | (uint32_t)(v01 >> 32);
  if (s && w == 8) {
    const uint32_t m2 = (uint32_t)(m >> (64 - 8 * s)), v2 = (uint32_t)(vm >> (64 - 8 * s));
    p[2 * kWave] = (p[2 * kWave] & ~m2) | v2;
  }
}

// ---- tier-0 header-window pipeline ----
// Per-wave LDS region: win[2][64 packets][64 B] + meta_off[2][64] u32 + meta_len[2][64] u32.
// (A sub-dword LDS-DMA such as global_load_lds_ushort still fills one zero-extended DWORD slot
// per lane, so the 16-bit lengths land in 4-byte slots.)
constexpr uint32_t kWinBytes = kWave * kWin;                          // one buffer, 4 KiB
constexpr uint32_t kMetaBytes = 2 * kWave * 4 + 2 * kWave * 4;             // 1 KiB
// per-wave LDS bytes of the general interpreter's tier 0: one window buffer + metadata
constexpr uint32_t kWaveLds0 = kWinBytes + kMetaBytes;

struct WaveLds {
  uint8_t* win;        // [2][kWinBytes]
  uint32_t* meta_off;  // [2][64]
  uint32_t* meta_len;  // [2][64], low 16 bits
};

__device__ __forceinline__ uint32_t stride_len(const LaunchArgs& a) {
  return (uint32_t)(a.stride > 0xFFFFFFFFull ? 0xFFFFFFFFull : a.stride);
}

// DMA the offsets / lengths of tile t into meta buffer b (lanes past the batch read a dummy).
// PK (the compiled forward var kernels, tile_body PLEN): the buffer holds the offsets, then the
// lengths packed as u16[64] (128 bytes instead of 64 zero-extended dword slots); b must be 0 (L
// names the buffer). A whole tile of 4-byte aligned lengths moves as 32 dwords (lanes 0..31);
// the batch's partial last tile and unaligned length arrays store them lane by lane.
template <bool PK = false>
__device__ __forceinline__ void dma_meta(const LaunchArgs& a, const WaveLds& L, uint32_t b,
                                         uint64_t t, uint32_t lane) {
  const uint64_t pkt = t * kWave + lane;
  const bool ok = t < a.n_tiles && pkt < a.n;
  if (a.offsets)
    dma_x1(ok ? (uintptr_t)(a.offsets + pkt) : (uintptr_t)a.prog, lds_addr(L.meta_off + b * kWave));
  if (!a.lens) return;
  if (!PK) {
    dma_u16(ok ? (uintptr_t)(a.lens + pkt) : (uintptr_t)a.prog, lds_addr(L.meta_len + b * kWave));
  } else if (t < a.n_tiles && (t + 1) * kWave <= a.n && ((uintptr_t)a.lens & 3) == 0) {
    if (lane < kWave / 2) dma_x1((uintptr_t)(a.lens + t * kWave) + 4 * lane, lds_addr(L.meta_len));
  } else {
    ((uint16_t*)L.meta_len)[lane] = ok ? a.lens[pkt] : (uint16_t)0;
  }
}

// Packet j of tile t, from meta buffer b: base address and length (0 for j past the batch).
template <bool PK = false>
__device__ __forceinline__ void meta_of(const LaunchArgs& a, const WaveLds& L, uint32_t b,
                                        uint64_t t, uint32_t j, uintptr_t& base, uint32_t& len) {
  const uint64_t pkt = t * kWave + j;
  const bool ok = pkt < a.n;
  base = (uintptr_t)a.frames + (a.offsets ? (uint64_t)L.meta_off[b * kWave + j] : pkt * a.stride);
  const uint32_t ml = PK ? (uint32_t)((const uint16_t*)L.meta_len)[j] : L.meta_len[b * kWave + j];
  len = ok ? (a.lens ? (ml & 0xffffu) : stride_len(a)) : 0u;
}

// DMA tile t's 64 header windows (metadata in buffer mb) into window buffer wb: round r moves
// packets 16r..16r+15, lane l filling chunk slot (l & 3) of packet 16r + l/4 from logical chunk
// (l & 3) ^ swz. Chunks wholly past the packet's end read a dummy address instead (never a byte
// past a valid 16-byte chunk).
template <bool PK = false>
__device__ __forceinline__ void dma_window(const LaunchArgs& a, const WaveLds& L, uint32_t mb,
                                           uint32_t wb, uint64_t t, uint32_t lane) {
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const uint32_t j = r * 16 + (lane >> 2);
    uintptr_t bj;
    uint32_t lj;
    meta_of<PK>(a, L, mb, t, j, bj, lj);
    const uint32_t c = (lane & 3) ^ win_swz(j);
    const uintptr_t src = (c * 16 < lj) ? bj + c * 16 : (uintptr_t)a.prog;
    dma_x4(src, lds_addr(L.win + wb * kWinBytes + r * 1024));
  }
}

// The same for packets at any 4-byte aligned address (the var tile loop, gen_tile.py
// jit_statement_varl): chunk c straight from packet + 16c, except a chunk that would read past the
// 16-byte block holding the packet's last byte (16c + 16 + m > ceil16(m + len), m = packet & 15),
// which moves the aligned block below, (packet + 16c) & ~15 -- the statement shifts that slot into
// place at the tile's top (its tailfix, %[mis] bit 0).
__device__ __forceinline__ void dma_window_any(const LaunchArgs& a, const WaveLds& L, uint64_t t,
                                               uint32_t lane) {
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const uint32_t j = r * 16 + (lane >> 2);
    uintptr_t bj;
    uint32_t lj;
    meta_of<true>(a, L, 0, t, j, bj, lj);
    const uint32_t c = (lane & 3) ^ win_swz(j), m = (uint32_t)(bj & 15);
    uintptr_t src = bj + c * 16;
    if (c * 16 + 16 + m > ((m + lj + 15) & ~15u)) src &= ~(uintptr_t)15;
    dma_x4(c * 16 < lj ? src : (uintptr_t)a.prog, lds_addr(L.win + r * 1024));
  }
}

// Stride layout with 16-byte aligned slots of >= kWin bytes: every packet's whole window is
// inside its slot (the C ABI requires n * stride bytes of frames), so tile t's windows can be
// DMA'd without its lengths -- i.e. in the same HBM round trip as the lengths. Bytes past a
// packet's length are masked when read.
__device__ __forceinline__ bool stride_windows(const LaunchArgs& a) {
  return a.offsets == nullptr && a.stride >= (uint64_t)kWin &&
         (((uintptr_t)a.frames | (uintptr_t)a.stride) & 15) == 0;
}
__device__ __forceinline__ void dma_window_stride(const LaunchArgs& a, uint8_t* win, uint64_t t,
                                                  uint32_t lane) {
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const uint32_t j = r * 16 + (lane >> 2);
    const uint64_t pkt = t * kWave + j;
    const uint32_t c = (lane & 3) ^ win_swz(j);
    const uintptr_t src =
        pkt < a.n ? (uintptr_t)a.frames + pkt * a.stride + c * 16 : (uintptr_t)a.prog;
    dma_x4(src, lds_addr(win + r * 1024));
  }
}

// The xdp_md convention in place (xdp.rs:16-20, main.rs:14-31 handed [ctx][packet]): the lane's
// window holds packet bytes [0, 64); make it image bytes [0, 64) = {u32 data = 8, u32 data_end =
// 8 + len} + packet bytes [0, 56). The statement then sees the image exactly as if the packet
// had been staged behind its ctx (its BASE is the packet - 8, its LEN 8 + len).
// (8-byte halves, from the top down in two groups: every half is read before it is overwritten;
// LDS operations of one wave complete in order)
__device__ __forceinline__ void xdp_window(uint8_t* pw, uint32_t swz, uint32_t len) {
  // (the lane's own window: no readfirstlane, unlike lds_addr)
  const uint32_t win = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const void*)pw;
  const uint32_t swz16 = swz << 4;
  const uint64_t ctx = 8ull | ((uint64_t)(min(len, 0xffffu) + 8u) << 32);
  uint32_t a0, a1, a2, a3;
  uint64_t q0, q1, q2, q3;
  asm volatile(
      "v_xad_u32 %[a0], %[swz], 0, %[win]\n\t"
      "v_xad_u32 %[a1], %[swz], 16, %[win]\n\t"
      "v_xad_u32 %[a2], %[swz], 32, %[win]\n\t"
      "v_xad_u32 %[a3], %[swz], 48, %[win]\n\t"
      "ds_read_b64 %[q0], %[a3]\n\t"
      "ds_read_b64 %[q1], %[a2] offset:8\n\t"
      "ds_read_b64 %[q2], %[a2]\n\t"
      "ds_read_b64 %[q3], %[a1] offset:8\n\t"
      "s_waitcnt lgkmcnt(0)\n\t"
      "ds_write_b64 %[a3], %[q0] offset:8\n\t"
      "ds_write_b64 %[a3], %[q1]\n\t"
      "ds_write_b64 %[a2], %[q2] offset:8\n\t"
      "ds_write_b64 %[a2], %[q3]\n\t"
      "ds_read_b64 %[q0], %[a1]\n\t"
      "ds_read_b64 %[q1], %[a0] offset:8\n\t"
      "ds_read_b64 %[q2], %[a0]\n\t"
      "s_waitcnt lgkmcnt(0)\n\t"
      "ds_write_b64 %[a1], %[q0] offset:8\n\t"
      "ds_write_b64 %[a1], %[q1]\n\t"
      "ds_write_b64 %[a0], %[q2] offset:8\n\t"
      "ds_write_b64 %[a0], %[ctx]\n\t"
      "s_waitcnt lgkmcnt(0)"
      : [a0] "=&v"(a0), [a1] "=&v"(a1), [a2] "=&v"(a2), [a3] "=&v"(a3), [q0] "=&v"(q0),
        [q1] "=&v"(q1), [q2] "=&v"(q2), [q3] "=&v"(q3)
      : [win] "v"(win), [swz] "v"(swz16), [ctx] "v"(ctx)
      : "memory");
}

// The 16-byte aligned source block at a, or zeros when it holds no byte of [src, end): a block
// holding a packet byte lies in that byte's page, so no load leaves the packet's pages.
__device__ __forceinline__ u32x4 blk16(uintptr_t a, uintptr_t src, uintptr_t end) {
  if (a + 16 <= src || a >= end) return u32x4{0u, 0u, 0u, 0u};
  return *(g_u4*)a;
}

// Synchronous per-lane staging for tiles whose packet bases are not all 16-byte aligned: the
// five 16-byte aligned blocks that cover the window's bytes (each only where it holds one of
// them), funnel-shifted into place (v_alignbyte), bytes at or past min(len, 64) zero. Five load
// instructions per wave, each over its 64 packets' lines (round 4 read the window as 16
// bounds-checked dwords, two loads each: 32 such instructions).
__device__ __forceinline__ void stage_window_lane(uint8_t* pw, uint32_t swz, const uint8_t* base,
                                                  uint32_t len, bool valid) {
  const uint32_t m = valid ? min(len, (uint32_t)kWin) : 0u;
  const uintptr_t s0 = (uintptr_t)base, end = s0 + m, a0 = s0 & ~(uintptr_t)15;
  const uint32_t sh = (uint32_t)(s0 & 15), q = sh >> 2;
  uint32_t d[20];
#pragma unroll
  for (int k = 0; k < 5; k++) {
    const u32x4 b = m ? blk16(a0 + 16 * k, s0, end) : u32x4{0u, 0u, 0u, 0u};
    d[4 * k] = b.x, d[4 * k + 1] = b.y, d[4 * k + 2] = b.z, d[4 * k + 3] = b.w;
  }
#pragma unroll
  for (uint32_t c = 0; c < 4; c++) {
    uint32_t w[4];
#pragma unroll
    for (uint32_t e = 0; e < 4; e++) {
      const uint32_t j = 4 * c + e;  // window dword j = bytes [4j + sh, 4j + sh + 4) of the blocks
      const uint32_t l0 = (q & 1) ? d[j + 1] : d[j], l1 = (q & 1) ? d[j + 3] : d[j + 2];
      const uint32_t h0 = (q & 1) ? d[j + 2] : d[j + 1], h1 = (q & 1) ? d[j + 4] : d[j + 3];
      const uint32_t v = __builtin_amdgcn_alignbyte((q & 2) ? h1 : h0, (q & 2) ? l1 : l0, sh & 3);
      const uint32_t valid_b = m > 4 * j ? min(m - 4 * j, 4u) : 0u;
      w[e] = valid_b >= 4 ? v : v & ((1u << (8 * valid_b)) - 1u);
    }
    *(uint4*)(pw + win_off(16 * c, swz)) = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// ---- counters ----
// Per-workgroup accumulator in static LDS (separate from each kernel's dynamic LDS, which other
// waves may still be using when one wave finishes). Zeroed by counters_init() at kernel start.
struct WgCounters {
  uint64_t acc[8];
  uint32_t arrived;
  uint32_t next;  // the compiled fixed-slot kernel's tile hand-out (tile_body)
};
__device__ __forceinline__ WgCounters* wg_counters() {
  __shared__ WgCounters c;
  return &c;
}
// Every kernel calls this first; the barrier makes the zeroed accumulator visible to all waves.
__device__ __forceinline__ void counters_init() {
  WgCounters* w = wg_counters();
  if (threadIdx.x < 8) w->acc[threadIdx.x] = 0;
  if (threadIdx.x == 0) w->arrived = 0;
  if (threadIdx.x == 1) w->next = 0;
  __syncthreads();
}

// Per-wave counter epilogue; no workgroup barrier, so a finished wave retires at once.
//   * each wave adds its sums to the workgroup accumulator in LDS and takes an LDS arrival ticket;
//   * the workgroup's last wave adds the 8 sums to shard g = blockIdx % 64 (blockIdx -> XCD is
//     round-robin, so a shard is only ever hit from one XCD), 8 lanes, one 8-byte agent-scope
//     atomic each;
//   * fold_kernel = 0 (default): every shard word carries its own arrival count in bits 48..63 --
//     a workgroup adds (1 << 48) + sum with a RETURNING atomic, and the one whose add completes
//     the word (count == the shard's workgroups - 1; atomics on one word are serialized, so the
//     old value holds every other member's sum) forwards the word's total to the caller's
//     counter and clears the word. One round trip for the last wave of each workgroup, no
//     ticket chain, no second kernel. Needs every per-shard sum < 2^48 (the host checks the
//     launch's bound: packets x steps per packet);
//   * fold_kernel = 1: plain adds, folded by fold_counters launched next on the stream.
// cnt[] is wave-uniform, retired per lane.
constexpr uint64_t kShardCountShift = 48;
constexpr uint64_t kShardSumMask = (1ull << kShardCountShift) - 1;

// (REDUCED: `retired` is already the wave's total)
template <uint32_t WPB = kWavesPerBlock, bool REDUCED = false>
__device__ __forceinline__ void flush_counters(const LaunchArgs& a, const uint64_t (&cnt)[7],
                                               uint64_t retired, uint8_t*, uint32_t lane,
                                               uint32_t) {
  if (a.counters == nullptr) return;
  if (!REDUCED) retired = wave_sum_u64(retired);
  WgCounters* w = wg_counters();
  uint64_t mine = retired;
#pragma unroll
  for (int b = 0; b < 7; b++) mine = lane == (uint32_t)b ? cnt[b] : mine;
  if (lane < 8 && mine) atomicAdd((unsigned long long*)&w->acc[lane], (unsigned long long)mine);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  uint32_t old = 0;
  if (lane == 0) old = atomicAdd(&w->arrived, 1u);
  old = __builtin_amdgcn_readfirstlane(old);
  if (old != WPB - 1) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  // the workgroup's last wave
  const uint32_t g = blockIdx.x % kCounterShards;
  if (lane >= 8) return;
  const uint64_t sum = w->acc[lane];
  uint64_t* word = &a.shards[g * 8 + lane];
  if (a.fold_kernel) {  // fold_counters runs next on the stream
    if (sum) __hip_atomic_fetch_add(word, sum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  const uint32_t members = (gridDim.x - g + kCounterShards - 1) / kCounterShards;
  const uint64_t add = (1ull << kShardCountShift) + sum;
  const uint64_t before =
      __hip_atomic_fetch_add(word, add, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if ((before >> kShardCountShift) != members - 1) return;
  const uint64_t total = (before + add) & kShardSumMask;
  __hip_atomic_store(word, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (total) atomicAdd((unsigned long long*)&a.counters[lane], (unsigned long long)total);
}

// The eBPF register file r0..r10 (emu.rs:15), as two 11-entry u32 arrays (low and high words):
// each maps to an 11-VGPR tuple indexed with s_set_gpr_idx by the scalar register number, where a
// uint64_t[11] would occupy a 32-VGPR tuple (10 registers wasted).
#define RF_GET(i) ((uint64_t)rlo[i] | ((uint64_t)rhi[i] << 32))
#define RF_SET(i, v)                     \
  do {                                   \
    const uint64_t v_ = (v);             \
    rlo[i] = (uint32_t)v_;               \
    rhi[i] = (uint32_t)(v_ >> 32);       \
  } while (0)

template <int TIER, bool LDSP, int NW>
__global__ __launch_bounds__(kBlock) void interp_kernel(LaunchArgs a) {
  // the deopt pass with an empty list (the usual case): every workgroup leaves at once -- no
  // program staging, no counter flush, nothing to clear (the list cannot grow during the pass)
  if (TIER == 1 && a.deopt_pass &&
      rfl(__hip_atomic_load(a.deopt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == 0) {
    if (blockIdx.x == 0 && threadIdx.x == 0)  // (deopt[2]: packets the last pass re-ran, tests)
      __hip_atomic_store(a.deopt + 2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  counters_init();
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t nu = a.n_uops;
  const uint32_t prog_bytes = LDSP ? nu * (uint32_t)sizeof(Uop) : 0u;
  Uop* sprog = (Uop*)smem;
  uint8_t* const wave_region = smem + prog_bytes;  // tier 0: kWaveLds0 per wave

  // stage the program once per workgroup (emu.instructions, emu.rs:24)
  if (LDSP) {
    const uint4* src = (const uint4*)a.prog;
    uint4* dst = (uint4*)sprog;
    for (uint32_t i = threadIdx.x; i < nu; i += kBlock) dst[i] = src[i];
  }
  __syncthreads();

  const uint32_t lane = threadIdx.x & (kWave - 1);
  const uint32_t wv = threadIdx.x / kWave;
  WaveLds L;
  L.win = wave_region + (size_t)wv * kWaveLds0;
  L.meta_off = (uint32_t*)(L.win + kWinBytes);
  L.meta_len = L.meta_off + 2 * kWave;
  const uint32_t my_swz = win_swz(lane);
  const uint64_t wave_slot = (uint64_t)blockIdx.x * kWavesPerBlock + wv;
  const uint64_t total_waves = (uint64_t)gridDim.x * kWavesPerBlock;
  const uint32_t mem_size = a.mem_size;
  const uint32_t max_steps = (uint32_t)(a.max_steps > 0xFFFFFFFFull ? 0xFFFFFFFFull : a.max_steps);

  uint32_t* const img = TIER == 1
      ? (uint32_t*)(a.image_ws + wave_slot * tier1_slot_bytes(mem_size)) + lane
      : nullptr;
  uint32_t* const cstack = TIER == 1 ? img + (size_t)((mem_size + 3) / 4) * kWave : nullptr;

  uint64_t cnt[7] = {0, 0, 0, 0, 0, 0, 0};  // wave-uniform verdict buckets + faults
  uint64_t retired = 0;                     // per lane

  // Tier 0 pipeline (W = total waves; metadata buffers alternate per tile of this wave): the
  // windows of t are DMA'd and waited for at the top of t; the metadata of t + W is in flight
  // during t. (Double-buffered windows -- the next tile's windows in flight as well -- were an
  // opt-in A/B variant until round 5: half the resident waves, not faster.)
  uint32_t b = 0;
  bool co_cur = false;  // tile t's windows were DMA'd (all packet bases 16-byte aligned)
  if (TIER == 0 && wave_slot < a.n_tiles) {
    dma_meta(a, L, 0, wave_slot, lane);
    dma_wait();
  }

  // the deopt pass (tier 1, LaunchArgs::deopt_pass): the packets the compiled store-mode kernel
  // listed, idx[0 .. count), each run from the start with its outputs at its own index
  const bool dpass = TIER == 1 && a.deopt_pass != 0;
  uint64_t n_run = a.n, tiles_run = a.n_tiles;
  if (dpass) {
    n_run = rfl(__hip_atomic_load(a.deopt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    tiles_run = (n_run + kWave - 1) / kWave;
  }
  for (uint64_t tile = wave_slot; tile < tiles_run; tile += total_waves) {
    const uint64_t slot = tile * kWave + lane;
    const bool valid = slot < n_run;
    const uint64_t pkt = !dpass ? slot : valid ? (uint64_t)a.deopt_idx[slot] : 0ull;
    const uint8_t* base = nullptr;
    uint32_t len = 0;
    uint8_t* const my_win = L.win + lane * kWin;
    if (TIER == 0) {
      dma_wait();  // this tile's metadata
      uintptr_t mb;
      uint32_t ml;
      meta_of(a, L, b, tile, lane, mb, ml);
      base = (const uint8_t*)mb;
      len = valid ? ml : 0u;
      co_cur = ballot(valid && ml != 0 && (mb & 15) != 0) == 0;
      if (co_cur) {
        dma_window(a, L, b, 0, tile, lane);
        dma_wait();
      }
      if (!co_cur) stage_window_lane(my_win, my_swz, base, len, valid);
    } else if (valid) {
      base = a.frames + (a.offsets ? (uint64_t)a.offsets[pkt] : pkt * a.stride);
      len = a.lens ? (uint32_t)a.lens[pkt] : stride_len(a);
    }
    // the xdp_md convention in place (tier 1): the image is [u32 data = 8][u32 data_end =
    // 8 + len][packet] (xdp.rs:16-20), r2 = its length 8 + len -- built below, no staging copy
    const uint32_t plen = len;  // (the packet's own length)
    if (TIER == 1 && a.xdp && valid) len = min(plen, 0xffffu) + 8u;

    // ---- Emu::default() + main.rs:14-31 register/memory layout ----
    uint32_t rlo[11], rhi[11];
    if (a.init_regs) {  // caller-set Emu.state.regs (emu.rs:14-17)
#pragma unroll
      for (int i = 0; i < 11; i++) RF_SET(i, a.init_regs[i]);
    } else {            // main.rs:28-31
#pragma unroll
      for (int i = 0; i < 11; i++) RF_SET(i, 0);
      RF_SET(2, len);
      RF_SET(10, a.r10);
    }
    uint32_t pc = valid ? 0u : PC_DONE;
    uint32_t st = EBPF_ST_OK;
    uint32_t nsteps = 0;
    uint32_t csp = 0;
    if (valid && len > mem_size) {  // main.rs:20-21 index panic
      st = EBPF_ST_BADPKT;
      pc = PC_DONE;
    }
    // tier 1: the image (main.rs:16-27: the packet, then zeros to mem_size) is materialised in
    // the lane's scratch lazily, a block at a time (32 blocks of 2^bsh dwords cover it: 32 bytes
    // for the 1 KiB default): a block is written from the packet / zeros by the first store into
    // it (bit b of `ib`), and reads of a block never stored to compute the initial bytes instead.
    // The eager copy wrote mem_size bytes per packet (1 GiB per 1 Mi-packet batch at 1 KiB) where
    // a program typically stores into one or two blocks.
    const uint32_t m_img = (TIER == 1 && pc != PC_DONE) ? len : 0u;
    uint32_t ib = 0;
    if (TIER == 1) {
      // the caller's initial frame stack (Emu.fp, emu.rs:26): an EXIT pops it (emu.rs:273-279)
      csp = a.init_fp_len;
      for (uint32_t i = 0; i < csp; i++) cstack[(size_t)i * kWave] = a.init_fp[i];
    }

    if (TIER == 0) {
      // vmcnt(0) as a builtin: hipcc's wait-count pass then knows that none of ITS loads (e.g.
      // init_regs into the register file) is pending, so it puts no wait at the interpreter's
      // indexed register accesses -- such a wait would also drain the LDS-DMA issued next,
      // which hipcc does not see.
      __builtin_amdgcn_s_waitcnt(0x0F70);
      const uint64_t tn = tile + total_waves;
      if (tn < a.n_tiles) {
        dma_meta(a, L, b ^ 1, tn, lane);  // lands while this tile is interpreted
      }
    }

    // ---- Emu::run (emu.rs:452-458) with min-pc re-convergence ----
    // Each iteration executes the instruction at the wave's minimum pc for the lanes parked
    // there ("act"). The step is computed by all lanes and COMMITTED through selects on act,
    // so the eBPF register file (22 VGPRs, indexed by the scalar dst/src via s_set_gpr_idx)
    // is never inside divergent control flow; only memory accesses are predicated on act.
    // (tier 1) dword d of the initial image; whether dword d is in a materialised block; a block
    // materialised; the lazy image's reads and writes (img_read / img_write's layout)
    const uint32_t img_md = (mem_size + 3) / 4;
    const uint32_t bsh = img_md <= 32 ? 0u : 32u - __builtin_clz((img_md + 31) / 32 - 1);
    auto vdw = [&](uint32_t d) -> uint32_t {
      if (d * 4 >= m_img) return 0u;
      if (a.xdp) return d == 0 ? 8u : d == 1 ? len : (uint32_t)pkt_read(base, d * 4 - 8, 4, plen);
      return (uint32_t)pkt_read(base, d * 4, 4, len);
    };
    auto rdw = [&](uint32_t d) -> uint32_t {
      return (ib >> (d >> bsh)) & 1u ? img[(size_t)d * kWave] : vdw(d);
    };
    auto own = [&](uint32_t d) {  // (d < img_md: the access was bounds-checked)
      const uint32_t b = d >> bsh;
      if ((ib >> b) & 1u) return;
      const uint32_t e1 = min((b + 1) << bsh, img_md);
      for (uint32_t e = b << bsh; e < e1; e++) img[(size_t)e * kWave] = vdw(e);
      ib |= 1u << b;
    };
    auto lazy_read = [&](uint32_t a0, uint32_t w) -> uint64_t {
      const uint32_t d = a0 >> 2, sft = a0 & 3;
      const uint32_t d0 = rdw(d);
      const uint32_t d1 = (sft + w > 4) ? rdw(d + 1) : 0u;
      uint64_t v = __builtin_amdgcn_alignbyte(d1, d0, sft);
      if (w == 8) {
        const uint32_t d2 = sft ? rdw(d + 2) : 0u;
        v |= (uint64_t)__builtin_amdgcn_alignbyte(d2, d1, sft) << 32;
      }
      return v & wmask(w);
    };
    auto lazy_write = [&](uint32_t a0, uint32_t w, uint64_t v) {
      const uint32_t d = a0 >> 2, dl = (a0 + w - 1) >> 2;
      own(d);
      if (dl != d) own(dl);
      if (dl > d + 1) own(d + 1);
      img_write(img, a0, w, v);
    };
    uint32_t wsteps = 0;
    // Termination guard: every iteration retires >= 1 lane-step and a lane retires at most
    // max_steps, so 64 * max_steps + 64 iterations bound a correct run; the guard only turns a
    // re-convergence bug into EBPF_ST_STEPS instead of a hung wave.
    uint32_t witer = 0;
    const uint64_t cap64 = (uint64_t)kWave * max_steps + kWave;
    const uint32_t witer_cap = cap64 > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)cap64;
    PcSet<NW> live;
    if (NW > 0) live.init(nu > 0 && ballot(pc == 0) != 0);
    for (;;) {
      uint32_t pcs;
      if (NW > 0) {
        pcs = live.first();
      } else {
        pcs = rfl(pc);
        if (ballot(pc != pcs) != 0) pcs = wave_min_u32(pc);
      }
      if (pcs >= nu) break;  // every lane exited, fell off the end or faulted
      if (++witer > witer_cap) {
        if (pc != PC_DONE) { st = EBPF_ST_STEPS; pc = PC_DONE; }
        break;
      }
      if (++wsteps > max_steps) {  // exact per-lane budget only once it can bind
        const bool over = pc == pcs && nsteps >= max_steps;
        st = over ? EBPF_ST_STEPS : st;
        pc = over ? PC_DONE : pc;  // an iteration with no active lane commits nothing
      }
      // fetch (wave-uniform): emu.rs:49
      uint4 q;
      if (LDSP) q = *(const uint4*)(sprog + pcs);
      else q = *(const uint4*)(a.prog + pcs);
      const uint32_t w0 = rfl(q.x), x = rfl(q.y), w2 = rfl(q.z), w3 = rfl(q.w);
      const uint32_t op = w0 & 0xff, dst = (w0 >> 8) & 0xff, src = (w0 >> 16) & 0xff;
      const uint32_t aux = w0 >> 24;
      const uint64_t k = (uint64_t)w2 | ((uint64_t)w3 << 32);

      const bool act = pc == pcs;
      const uint64_t A = RF_GET(dst);
      const uint64_t S = RF_GET(src);
      const uint64_t B = (aux & F_SRC) ? S : k;
      const uint32_t a32 = (uint32_t)A, b32 = (uint32_t)B;
      uint64_t R = A;             // dst value to commit
      uint32_t npc = pcs + 1;     // emu.rs:63
      bool fault = false;
      uint32_t fst = 0;
      bool w_r0 = false, w_src = false;  // atomic side writes (emu.rs:418,435)
      uint64_t side = 0;
      switch (op) {
        // ---- ALU64 ----
        case U_ADD64: R = A + B; break;
        case U_SUB64: R = A - B; break;
        case U_MUL64: R = A * B; break;
        case U_DIV64: R = B ? A / B : 0; break;
        case U_OR64: R = A | B; break;
        case U_AND64: R = A & B; break;
        case U_LSH64: R = A << (b32 & 63); break;
        case U_RSH64: R = A >> (b32 & 63); break;
        case U_NEG64: R = 0 - A; break;
        case U_MOD64: R = B ? A % B : A; break;
        case U_XOR64: R = A ^ B; break;
        case U_MOV64: R = B; break;
        case U_ARSH64: {  // rotate, then multiply by the sign (Q4, emu.rs:142-164)
          const uint32_t sh = b32 & 63;
          const uint64_t rot = sh ? ((A >> sh) | (A << (64 - sh))) : A;
          const bool neg = (int64_t)A < 0;
          fault = neg && rot == 0x8000000000000000ull;  // i64::MIN * -1 (emu.rs:162)
          fst = EBPF_ST_ARITH;
          R = neg ? 0 - rot : rot;
          break;
        }
        // ---- ALU32 (Q6/Q25) ----
        case U_ADD32: R = (uint32_t)(a32 + b32); break;
        case U_SUB32: R = (uint32_t)(a32 - b32); break;
        case U_MUL32: R = (uint32_t)(a32 * b32); break;
        case U_DIV32: R = b32 ? a32 / b32 : 0u; break;
        case U_OR32: R = a32 | b32; break;
        case U_AND32: R = a32 & b32; break;
        case U_LSH32: R = (uint32_t)(a32 << (b32 & 31)); break;
        case U_RSH32: R = a32 >> (b32 & 31); break;
        case U_NEG32: R = (uint32_t)(0u - a32); break;
        case U_MOD32: R = b32 ? a32 % b32 : a32; break;
        case U_XOR32: R = a32 ^ b32; break;
        case U_MOV32: R = b32; break;
        case U_ARSH32: {
          const uint32_t rot = __builtin_amdgcn_alignbit(a32, a32, b32 & 31);
          R = (int32_t)a32 < 0 ? (uint32_t)(0u - rot) : rot;
          break;
        }
        // ---- END (Q7) ----
        case U_ZX16: R = A & 0xffffull; break;
        case U_ZX32: R = A & 0xffffffffull; break;
        case U_NOP: break;
        case U_BSWAP16: R = ((A & 0xff) << 8) | ((A >> 8) & 0xff); break;
        case U_BSWAP32: R = bswap32(a32); break;
        case U_BSWAP64: R = ((uint64_t)bswap32(a32) << 32) | bswap32((uint32_t)(A >> 32)); break;
        // ---- JMP: signed orderings (Q2) ----
        case U_JA: npc = x; break;
        case U_JEQ: npc = A == B ? x : npc; break;
        case U_JGT: npc = (int64_t)A > (int64_t)B ? x : npc; break;
        case U_JGE: npc = (int64_t)A >= (int64_t)B ? x : npc; break;
        case U_JSET: npc = (A & B) ? x : npc; break;
        case U_JNE: npc = A != B ? x : npc; break;
        case U_JLT: npc = (int64_t)A < (int64_t)B ? x : npc; break;
        case U_JLE: npc = (int64_t)A <= (int64_t)B ? x : npc; break;
        // ---- JMP32: sign-extended low words (Q3) ----
        case U_JEQ32: npc = a32 == b32 ? x : npc; break;
        case U_JGT32: npc = (int32_t)a32 > (int32_t)b32 ? x : npc; break;
        case U_JGE32: npc = (int32_t)a32 >= (int32_t)b32 ? x : npc; break;
        case U_JSET32: npc = (a32 & b32) ? x : npc; break;  // == (sext(a) & sext(b)) != 0
        case U_JNE32: npc = a32 != b32 ? x : npc; break;
        case U_JLT32: npc = (int32_t)a32 < (int32_t)b32 ? x : npc; break;
        case U_JLE32: npc = (int32_t)a32 <= (int32_t)b32 ? x : npc; break;
        case U_CALL:  // emu.rs:265-272
          if (TIER == 1) {
            fault = csp >= (uint32_t)kCallDepth;
            fst = EBPF_ST_CALLDEPTH;
            if (act && !fault) {
              cstack[(size_t)csp * kWave] = x + 1;
              csp++;
            }
            npc = x;
          } else {
            fault = true;  // unreachable: the loader routes calls to tier 1
            fst = EBPF_ST_INSN;
          }
          break;
        case U_EXIT:  // emu.rs:273-279
          npc = PC_DONE;
          if (TIER == 1 && act && csp > 0) {
            csp--;
            npc = cstack[(size_t)csp * kWave];
          }
          break;
        // ---- loads / stores (emu.rs:311-444) ----
        case U_LDIMM: R = k; break;
        case U_LDX: {
          int64_t sum;
          const bool ovf = __builtin_add_overflow((int64_t)S, (int64_t)(int32_t)x, &sum);
          const uint64_t ua = (uint64_t)sum;
          const bool oob = ovf || ua >= mem_size;
          const bool ub = !oob && ua + aux > mem_size;
          fault = oob || ub;
          fst = oob ? EBPF_ST_MEM : EBPF_ST_MEM_UB;
          const uint32_t a0 = (uint32_t)ua;
          uint64_t v = 0;
          if (act && !fault) {
            if (TIER == 1) v = lazy_read(a0, aux);
            else if (a0 >= len) v = 0;
            else if (a0 + aux <= (uint32_t)kWin) v = win_read(my_win, my_swz, a0, aux, len);
            else v = pkt_read(base, a0, aux, len);
          }
          const uint64_t m = wmask(aux);
          R = (A & ~m) | v;  // upper bytes preserved (Q1)
          break;
        }
        case U_ST:
        case U_STX: {
          if (TIER == 1) {
            int64_t sum;
            const bool ovf = __builtin_add_overflow((int64_t)A, (int64_t)(int32_t)x, &sum);
            const uint64_t ua = (uint64_t)sum;
            const bool oob = ovf || ua >= mem_size;
            const bool ub = !oob && ua + aux > mem_size;
            fault = oob || ub;
            fst = oob ? EBPF_ST_MEM : EBPF_ST_MEM_UB;
            if (act && !fault) lazy_write((uint32_t)ua, aux, op == U_ST ? k : S);
          } else {
            fault = true;
            fst = EBPF_ST_INSN;
          }
          break;
        }
        case U_ATOMIC: {  // emu.rs:373-437
          if (TIER == 1) {
            int64_t sum;
            const bool ovf = __builtin_add_overflow((int64_t)A, (int64_t)(int32_t)x, &sum);
            const uint64_t ua = (uint64_t)sum;
            fault = ovf || ua >= mem_size || ua + 8 > mem_size;
            fst = EBPF_ST_MEM;
            const bool go = act && !fault;
            uint64_t orig = go ? lazy_read((uint32_t)ua, 8) : 0;
            const bool fetch = aux & F_FETCH;
            const bool is32 = aux & F_ATOMIC32;
            uint64_t bak = fetch ? orig : 0;
            uint64_t high = 0, sv = S, r0v = RF_GET(0);
            if (is32) {
              sv = (uint32_t)sv;
              high = orig >> 32;
              orig = (uint32_t)orig;
              r0v = (uint32_t)r0v;
              bak = (uint32_t)bak;
            }
            bool f2 = false;
            uint32_t fst2 = EBPF_ST_ARITH;
            if (k == 0x00) {
              int64_t t;
              f2 = __builtin_add_overflow((int64_t)orig, (int64_t)sv, &t);
              orig = (uint64_t)t;
            } else if (k == 0x40) orig |= sv;
            else if (k == 0x50) orig &= sv;
            else if (k == 0xa0) orig ^= sv;
            else if (k == 0xe0) { bak = orig; orig = sv; }
            else if (k == 0xf0) {
              if (orig == r0v) orig = sv;
              w_r0 = true;
            } else { f2 = true; fst2 = EBPF_ST_INSN; }
            int64_t t;
            const bool f3 = __builtin_add_overflow((int64_t)orig, (int64_t)(high << 32), &t);
            if (!fault && (f2 || f3)) { fault = true; fst = f2 ? fst2 : EBPF_ST_ARITH; }
            if (act && !fault) lazy_write((uint32_t)ua, 8, (uint64_t)t);
            w_src = fetch;
            side = bak;
          } else {
            fault = true;
            fst = EBPF_ST_INSN;
          }
          break;
        }
        default:  // U_FAULT
          fault = true;
          fst = aux;
          break;
      }
      // ---- commit (active lanes only) ----
      const bool ok = act && !fault;
      if (TIER == 1) {
        if (w_r0) RF_SET(0, ok ? side : RF_GET(0));        // cmpxchg: regs[0] = old (emu.rs:418)
        if (w_src) RF_SET(src, ok ? side : RF_GET(src));  // fetch: regs[src] = old (emu.rs:435)
      }
      RF_SET(dst, ok ? R : A);  // dst snapshot write-back for ST/STX/ATOMIC (Q14, emu.rs:443)
      nsteps += ok ? 1u : 0u;
      st = (act && fault) ? fst : st;
      pc = act ? (fault || npc >= nu ? PC_DONE : npc) : pc;
      if (NW > 0) {  // successors of this step: pcs + 1, the jump/call target, popped returns
        live.del(pcs);
        const uint32_t f = pcs + 1;
        if (f < nu && ballot(act && pc == f) != 0) live.add(f);
        const bool jumps = op >= U_JA && op <= U_CALL;
        if (jumps && x < nu && x != f && ballot(act && pc == x) != 0) live.add(x);
        if (TIER == 1 && op == U_EXIT) {
          uint64_t m = ballot(act && pc < nu);
          while (m) {
            const uint32_t p = __builtin_amdgcn_readlane(pc, __builtin_ctzll(m));
            live.add(p);
            m &= ~ballot(pc == p);
          }
        }
      }
    }

    // ---- outputs: r0 (main.rs:43), status, verdict (xdp.rs:3-9), final image ----
    const uint64_t r0v = RF_GET(0);
    if (a.mem_out && valid) {
      uint8_t* mo = a.mem_out + pkt * (uint64_t)mem_size;
      const uint32_t m = min(len, mem_size);
      for (uint32_t d = 0; d < (mem_size + 3) / 4; d++) {
        uint32_t v;
        if (TIER == 1) v = rdw(d);
        else if (d * 4 >= m) v = 0u;
        else if (d * 4 < (uint32_t)kWin) v = (uint32_t)win_read(my_win, my_swz, d * 4, 4, len);
        else v = (uint32_t)pkt_read(base, d * 4, 4, len);
        put_image(mo, d, v, mem_size);
      }
    }
    if (TIER == 1 && valid && (a.fp_len_out || a.fp_out)) {  // the final frame stack (Emu.fp);
      if (a.fp_len_out) a.fp_len_out[pkt] = (uint8_t)csp;     // either output may come alone
      if (a.fp_out)
        for (uint32_t i = 0; i < csp; i++) a.fp_out[pkt * kCallDepth + i] = cstack[(size_t)i * kWave];
    }
    if (a.regs_out && valid) {
#pragma unroll
      for (int i = 0; i < 11; i++) a.regs_out[pkt * 11 + i] = RF_GET(i);
    }
    if (valid) {
      if (a.r0) a.r0[pkt] = r0v;
      if (a.status) a.status[pkt] = (uint8_t)st;
      if (a.verdict) a.verdict[pkt] = st ? (uint8_t)EBPF_VERDICT_FAULT
                                         : (r0v < 5 ? (uint8_t)r0v : (uint8_t)EBPF_VERDICT_OTHER);
    }
    const bool okv = valid && st == EBPF_ST_OK;
#pragma unroll
    for (int b = 0; b < 5; b++) cnt[b] += __builtin_popcountll(ballot(okv && r0v == (uint64_t)b));
    cnt[5] += __builtin_popcountll(ballot(okv && r0v >= 5));
    cnt[6] += __builtin_popcountll(ballot(valid && st != EBPF_ST_OK));
    retired += valid ? nsteps : 0u;
    b ^= 1;
  }
  if (TIER == 0) dma_wait();  // no LDS-DMA may still target this workgroup's LDS at exit

  flush_counters(a, cnt, retired, smem, lane, wv);
  if (dpass) {  // the last workgroup to finish clears the list for the next batch on the stream
    __syncthreads();
    if (threadIdx.x == 0 &&
        __hip_atomic_fetch_add(a.deopt + 1, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) ==
            gridDim.x - 1) {
      __hip_atomic_store(a.deopt + 2, (uint32_t)n_run, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(a.deopt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(a.deopt + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ============================================================================================
// dag_kernel — tier-0 programs whose jumps all go forward (the verifier-era XDP shape), run with
// max_steps >= n_uops. Same semantics as interp_kernel<0, ...> (bit-exact, tested against each
// other and the oracle), shaped around the CU's ONE scalar unit, which interp_kernel saturates:
//   * the register file lives in LDS ([11][64] u64 per wave), so a register access is a VALU
//     address add + ds_read/ds_write instead of an s_set_gpr_idx_on/off pair per 32-bit half;
//   * the micro-op is ONE s_load_dwordx16 of a DUop whose fields are pre-scaled on the host
//     (register byte offsets, next pc, jump target, pc-set bits), so no readfirstlane/bit-field
//     extraction;
//   * lanes only move forward, so no step budget can bind (a lane retires <= n_uops steps) and
//     the scheduler is just "lowest pc with a parked lane" over a pc set whose every member has
//     a lane parked at it: no step counters, no termination guard, no empty iterations.
// Each step is computed by all lanes and committed through selects on `act`, as in
// interp_kernel, so uniform state (the pc set) is never written under divergent control flow.
// ============================================================================================
constexpr uint32_t kRegBytes = 11 * kRegStride;                           // 5.5 KiB per wave
constexpr uint32_t kDagMetaBytes = 2 * kWave * 4;                         // offsets + lengths
constexpr uint32_t kDagWaveLds = kRegBytes + kWinBytes + kDagMetaBytes;  // 10 KiB per wave

typedef uint32_t u32x16 __attribute__((ext_vector_type(16)));

// The C++ step's half of a DUop (dwords 32..47) from the device table.
__device__ __forceinline__ u32x16 load_duop(const DUop* prog, uint32_t pc) {
  u32x16 v;
  asm volatile("s_load_dwordx16 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)"
      : "=s"(v) : "s"(prog), "s"(pc * (uint32_t)sizeof(DUop) + (uint32_t)offsetof(DUop, opaux)));
  return v;
}

__device__ __forceinline__ uint64_t rget(const uint8_t* rl, uint32_t off) {
  return *(const uint64_t*)(rl + off);
}
__device__ __forceinline__ void rset(uint8_t* rl, uint32_t off, uint64_t v) {
  *(uint64_t*)(rl + off) = v;
}

template <int NW>
__global__ __launch_bounds__(kBlock) void dag_kernel(LaunchArgs a) {
  counters_init();
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t lane = threadIdx.x & (kWave - 1);
  const uint32_t wv = threadIdx.x / kWave;
  uint8_t* const wreg = smem + wv * kDagWaveLds;
  uint8_t* const rl = wreg + lane * 8;  // this lane's regs[0]; regs[r] at + r * kRegStride
  WaveLds L;
  L.win = wreg + kRegBytes;
  L.meta_off = (uint32_t*)(L.win + kWinBytes);
  L.meta_len = L.meta_off + kWave;
  const uint32_t my_swz = win_swz(lane);
  uint8_t* const my_win = L.win + lane * kWin;
  const uint64_t wave_slot = (uint64_t)blockIdx.x * kWavesPerBlock + wv;
  const uint64_t total_waves = (uint64_t)gridDim.x * kWavesPerBlock;
  const uint32_t mem_size = a.mem_size;

  uint64_t cnt[7] = {0, 0, 0, 0, 0, 0, 0};
  uint64_t retired = 0;

  for (uint64_t tile = wave_slot; tile < a.n_tiles; tile += total_waves) {
    const uint64_t pkt = tile * kWave + lane;
    const bool valid = pkt < a.n;
    // ---- header windows: with stride slots, windows and lengths in one round trip; else as
    //      interp_kernel's single-buffered tier 0 (lengths/offsets first) ----
    const bool sw = stride_windows(a);
    dma_meta(a, L, 0, tile, lane);
    if (sw) dma_window_stride(a, L.win, tile, lane);
    dma_wait();
    uintptr_t mb;
    uint32_t ml;
    meta_of(a, L, 0, tile, lane, mb, ml);
    const uint8_t* const base = (const uint8_t*)mb;
    const uint32_t len = valid ? ml : 0u;
    const bool co = sw || ballot(valid && ml != 0 && (mb & 15) != 0) == 0;
    if (co && !sw) dma_window(a, L, 0, 0, tile, lane);

    // ---- Emu::default() + main.rs:14-31 register layout (or caller-set regs) ----
    if (a.init_regs) {
#pragma unroll
      for (int i = 0; i < 11; i++) rset(rl, i * kRegStride, a.init_regs[i]);
    } else {
#pragma unroll
      for (int i = 0; i < 11; i++)
        rset(rl, i * kRegStride, i == 2 ? (uint64_t)len : i == 10 ? a.r10 : 0ull);
    }
    uint32_t lpc = valid ? 0u : PC_DONE;
    uint32_t st = EBPF_ST_OK;
    uint32_t nsteps = 0;
    if (valid && len > mem_size) {  // main.rs:20-21 index panic
      st = EBPF_ST_BADPKT;
      lpc = PC_DONE;
    }
    if (co) {
      if (!sw) dma_wait();
    } else {
      stage_window_lane(my_win, my_swz, base, len, valid);
    }

    // ---- Emu::run (emu.rs:452-458): lowest parked pc first ----
    PcSet<NW> live;
    live.init(ballot(lpc == 0) != 0);
    for (;;) {
      const uint32_t P = live.first();
      if (P == PC_DONE) break;
      live.del(P);
      const u32x16 q = load_duop(a.dprog, P);
      const uint32_t op = q[0] & 0xff, aux = q[0] >> 8, doff = q[1], soff = q[2], npc = q[3];
      const uint32_t x = q[4];
      const uint64_t k = (uint64_t)q[6] | ((uint64_t)q[7] << 32);
      const uint64_t nbit = (uint64_t)q[8] | ((uint64_t)q[9] << 32);
      const uint64_t tbit = (uint64_t)q[10] | ((uint64_t)q[11] << 32);
      const bool act = lpc == P;
      const uint64_t A = rget(rl, doff);
      const uint64_t S = rget(rl, soff);
      // operand B and the low words are formed inside each handler, after the dispatch, so the
      // register reads above are in flight while the scalar unit walks the dispatch tree
#define B ((aux & F_SRC) ? S : k)
#define a32 ((uint32_t)A)
#define b32 ((uint32_t)B)
      uint64_t R;
      bool cnd;
      switch (op) {
        // ---- ALU64 ----
        case U_ADD64: R = A + B; goto alu;
        case U_SUB64: R = A - B; goto alu;
        case U_MUL64: R = A * B; goto alu;
        case U_DIV64: R = B ? A / B : 0; goto alu;
        case U_OR64: R = A | B; goto alu;
        case U_AND64: R = A & B; goto alu;
        case U_LSH64: R = A << (b32 & 63); goto alu;
        case U_RSH64: R = A >> (b32 & 63); goto alu;
        case U_NEG64: R = 0 - A; goto alu;
        case U_MOD64: R = B ? A % B : A; goto alu;
        case U_XOR64: R = A ^ B; goto alu;
        case U_MOV64: R = B; goto alu;
        case U_ARSH64: {  // rotate, then multiply by the sign (Q4, emu.rs:142-164)
          const uint32_t sh = b32 & 63;
          const uint64_t rot = sh ? ((A >> sh) | (A << (64 - sh))) : A;
          const bool neg = (int64_t)A < 0;
          const bool fault = neg && rot == 0x8000000000000000ull;  // i64::MIN * -1 (emu.rs:162)
          R = neg ? 0 - rot : rot;
          const bool ok = act && !fault;
          rset(rl, doff, ok ? R : A);
          st = (act && fault) ? (uint32_t)EBPF_ST_ARITH : st;
          lpc = act ? (fault ? PC_DONE : npc) : lpc;
          nsteps += ok ? 1u : 0u;
          if (ballot(ok) != 0) {
            if (NW == 1) live.w0 |= nbit;
            else if (npc != PC_DONE) live.add(npc);
          }
          continue;
        }
        // ---- ALU32 (Q6/Q25) ----
        case U_ADD32: R = (uint32_t)(a32 + b32); goto alu;
        case U_SUB32: R = (uint32_t)(a32 - b32); goto alu;
        case U_MUL32: R = (uint32_t)(a32 * b32); goto alu;
        case U_DIV32: R = b32 ? a32 / b32 : 0u; goto alu;
        case U_OR32: R = a32 | b32; goto alu;
        case U_AND32: R = a32 & b32; goto alu;
        case U_LSH32: R = (uint32_t)(a32 << (b32 & 31)); goto alu;
        case U_RSH32: R = a32 >> (b32 & 31); goto alu;
        case U_NEG32: R = (uint32_t)(0u - a32); goto alu;
        case U_MOD32: R = b32 ? a32 % b32 : a32; goto alu;
        case U_XOR32: R = a32 ^ b32; goto alu;
        case U_MOV32: R = b32; goto alu;
        case U_ARSH32: {
          const uint32_t rot = __builtin_amdgcn_alignbit(a32, a32, b32 & 31);
          R = (int32_t)a32 < 0 ? (uint32_t)(0u - rot) : rot;
          goto alu;
        }
        // ---- END (Q7) ----
        case U_ZX16: R = A & 0xffffull; goto alu;
        case U_ZX32: R = A & 0xffffffffull; goto alu;
        case U_NOP: R = A; goto alu;
        case U_BSWAP16: R = ((A & 0xff) << 8) | ((A >> 8) & 0xff); goto alu;
        case U_BSWAP32: R = bswap32(a32); goto alu;
        case U_BSWAP64: R = ((uint64_t)bswap32(a32) << 32) | bswap32((uint32_t)(A >> 32)); goto alu;
        case U_LDIMM: R = k; goto alu;
        // ---- JMP: signed orderings (Q2); JMP32 on sign-extended low words (Q3). The host
        //      rewrote JNE/JGE/JLE as JEQ/JLT/JGT with swapped successors (build_dag). ----
        case U_JA: cnd = true; goto jump;
        case U_JEQ: cnd = A == B; goto jump;
        case U_JGT: cnd = (int64_t)A > (int64_t)B; goto jump;
        case U_JSET: cnd = (A & B) != 0; goto jump;
        case U_JLT: cnd = (int64_t)A < (int64_t)B; goto jump;
        case U_JEQ32: cnd = a32 == b32; goto jump;
        case U_JGT32: cnd = (int32_t)a32 > (int32_t)b32; goto jump;
        case U_JSET32: cnd = (a32 & b32) != 0; goto jump;
        case U_JLT32: cnd = (int32_t)a32 < (int32_t)b32; goto jump;
        case U_EXIT:  // emu.rs:273-279 with an empty frame stack: stop
          lpc = act ? PC_DONE : lpc;
          nsteps += act ? 1u : 0u;
          continue;
        case U_LDX: {  // emu.rs:341-349 + mmu.rs bounds (Q1 upper bytes kept, Q20 first byte)
          int64_t sum;
          const bool ovf = __builtin_add_overflow((int64_t)S, (int64_t)(int32_t)x, &sum);
          const uint64_t ua = (uint64_t)sum;
          const bool oob = ovf || ua >= mem_size;
          const bool ub = !oob && ua + aux > mem_size;
          const bool fault = oob || ub;
          const uint32_t a0 = (uint32_t)ua;
          const bool ok = act && !fault;
          const bool in_pkt = a0 < len;
          const bool in_win = a0 + aux <= (uint32_t)kWin;
          // the window read is harmless for every lane (address kept inside the window)
          uint64_t v = win_read(my_win, my_swz, in_win ? a0 : 0u, aux, len);
          v = (in_pkt && in_win) ? v : 0ull;
          const bool far = ok && in_pkt && !in_win;
          if (ballot(far) != 0) {
            if (far) v = pkt_read(base, a0, aux, len);
          }
          R = (A & ~k) | v;  // k = width mask
          rset(rl, doff, ok ? R : A);
          st = (act && fault) ? (oob ? (uint32_t)EBPF_ST_MEM : (uint32_t)EBPF_ST_MEM_UB) : st;
          lpc = act ? (fault ? PC_DONE : npc) : lpc;
          nsteps += ok ? 1u : 0u;
          if (ballot(ok) != 0) {
            if (NW == 1) live.w0 |= nbit;
            else if (npc != PC_DONE) live.add(npc);
          }
          continue;
        }
        case U_LDXK: {  // LDX at a load-time constant address (host.cpp fold_const_loads)
          const uint64_t ua = (uint64_t)q[12] | ((uint64_t)q[13] << 32);  // DUop::addr
          const bool oob = ua >= mem_size;
          if (oob || ua + aux > mem_size) {  // uniform: every active lane faults alike
            st = act ? (oob ? (uint32_t)EBPF_ST_MEM : (uint32_t)EBPF_ST_MEM_UB) : st;
            lpc = act ? PC_DONE : lpc;
            continue;
          }
          const uint32_t a0 = (uint32_t)ua;
          uint64_t v = 0;
          if (a0 + aux <= (uint32_t)kWin) {
            v = win_read(my_win, my_swz, a0, aux, len);
            v = a0 < len ? v : 0ull;
          } else {
            const bool far = act && a0 < len;
            if (ballot(far) != 0) {
              if (far) v = pkt_read(base, a0, aux, len);
            }
          }
          R = (A & ~k) | v;
          goto alu;
        }
        default:  // U_FAULT (static faults; tier-1 kinds never reach this kernel)
          st = act ? (op == U_FAULT ? aux : (uint32_t)EBPF_ST_INSN) : st;
          lpc = act ? PC_DONE : lpc;
          continue;
      }
#undef B
#undef a32
#undef b32
    alu:
      rset(rl, doff, act ? R : A);
      lpc = act ? npc : lpc;
      nsteps += act ? 1u : 0u;
      if (NW == 1) live.w0 |= nbit;
      else if (npc != PC_DONE) live.add(npc);
      continue;
    jump: {
      const uint64_t tk = ballot(act && cnd), nt = ballot(act && !cnd);
      lpc = act ? (cnd ? x : npc) : lpc;
      nsteps += act ? 1u : 0u;
      if (NW == 1) {
        live.w0 |= (tk ? tbit : 0ull) | (nt ? nbit : 0ull);
      } else {
        if (tk && x != PC_DONE) live.add(x);
        if (nt && npc != PC_DONE) live.add(npc);
      }
    }
    }

    // ---- outputs: r0 (main.rs:43), status, verdict (xdp.rs:3-9), final image/registers ----
    const uint64_t r0v = rget(rl, 0);
    if (a.mem_out && valid) {
      uint8_t* mo = a.mem_out + pkt * (uint64_t)mem_size;
      const uint32_t m = min(len, mem_size);
      for (uint32_t d = 0; d < (mem_size + 3) / 4; d++) {
        uint32_t v;
        if (d * 4 >= m) v = 0u;
        else if (d * 4 < (uint32_t)kWin) v = (uint32_t)win_read(my_win, my_swz, d * 4, 4, len);
        else v = (uint32_t)pkt_read(base, d * 4, 4, len);
        put_image(mo, d, v, mem_size);
      }
    }
    if (a.regs_out && valid) {
#pragma unroll
      for (int i = 0; i < 11; i++) a.regs_out[pkt * 11 + i] = rget(rl, i * kRegStride);
    }
    if (valid) {
      if (a.r0) a.r0[pkt] = r0v;
      if (a.status) a.status[pkt] = (uint8_t)st;
      if (a.verdict) a.verdict[pkt] = st ? (uint8_t)EBPF_VERDICT_FAULT
                                         : (r0v < 5 ? (uint8_t)r0v : (uint8_t)EBPF_VERDICT_OTHER);
    }
    const bool okv = valid && st == EBPF_ST_OK;
#pragma unroll
    for (int b = 0; b < 5; b++) cnt[b] += __builtin_popcountll(ballot(okv && r0v == (uint64_t)b));
    cnt[5] += __builtin_popcountll(ballot(okv && r0v >= 5));
    cnt[6] += __builtin_popcountll(ballot(valid && st != EBPF_ST_OK));
    retired += valid ? nsteps : 0u;
  }
  flush_counters(a, cnt, retired, smem, lane, wv);
}

#ifndef EBPFEMU_JIT_TEMPLATE  // (the JIT template build: the tile kernels only)
// ============================================================================================
// Length-binned lane packing (loop mode, offsets + lens layouts). Lanes of a tile run until its
// longest packet is done, so a tile mixing 64- and 1500-byte frames idles half its lanes in a
// per-byte loop. A counting sort by class ceil(len / 128) (capped) groups similar lengths:
// bin_hist counts the classes per workgroup (LDS histogram, wave-aggregated), bin_scatter
// derives each workgroup's range per class from those counts and writes the indices, longest
// class first.
// The order within a class is arbitrary; every output stays indexed by the original packet.
// ============================================================================================
constexpr int kBinBlock = 1024;

__device__ __forceinline__ uint32_t bin_class(uint32_t len) {
  const uint32_t c = (len + 127) >> 7;
  return c < (uint32_t)kBinClasses ? c : (uint32_t)kBinClasses - 1;
}

// The lanes of a wave that hold class c add their count with one LDS atomic (its lowest lane);
// returns this lane's slot: the class's count before the wave's add plus the lane's rank among
// the wave's lanes of its class. A mixed 64/1500-byte batch has two classes per wave, so two
// atomics instead of 64 serialized on two LDS words.
__device__ __forceinline__ uint32_t wave_class_slot(uint32_t c, uint32_t* h) {
  const uint32_t lane = __lane_id();
  const uint64_t below = (1ull << lane) - 1;
  uint64_t todo = __ballot(1);
  uint32_t slot = 0;
  while (todo) {
    const int lead = __ffsll((unsigned long long)todo) - 1;
    const uint32_t cc = __shfl(c, lead);
    const uint64_t m = __ballot(c == cc) & todo;
    uint32_t b = 0;
    if ((int)lane == lead) b = atomicAdd(&h[cc], (uint32_t)__popcll(m));
    b = __shfl(b, lead);
    if (c == cc) slot = b + (uint32_t)__popcll(m & below);
    todo &= ~m;
  }
  return slot;
}

// Per-workgroup class counts (wgc[block][class], plain stores: no device atomics, which on two
// class words serialized 256 workgroups' adds in each kernel).
__global__ __launch_bounds__(kBinBlock) void bin_hist(const uint16_t* lens, uint64_t n,
                                                      uint32_t* wgc) {
  __shared__ uint32_t h[kBinClasses];
  if (threadIdx.x < kBinClasses) h[threadIdx.x] = 0;
  __syncthreads();
  for (uint64_t i = (uint64_t)blockIdx.x * kBinBlock + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * kBinBlock)
    (void)wave_class_slot(bin_class(lens[i]), h);
  __syncthreads();
  if (threadIdx.x < kBinClasses) wgc[blockIdx.x * kBinClasses + threadIdx.x] = h[threadIdx.x];
}

// Each workgroup sums the class totals and the counts of the workgroups before it (thread t
// reads class t % 16 of every 64th workgroup), then writes its packets' indices from
// base(class) = packets of longer classes + earlier workgroups' packets of the class.
__global__ __launch_bounds__(kBinBlock) void bin_scatter(const uint16_t* lens, uint64_t n,
                                                         const uint32_t* wgc, uint32_t* perm) {
  static_assert(kBinBlock % kBinClasses == 0, "class of a thread fixed across the sum");
  __shared__ uint32_t h[kBinClasses], tot[kBinClasses], pre[kBinClasses], base[kBinClasses];
  const uint32_t t = threadIdx.x;
  if (t < kBinClasses) h[t] = tot[t] = pre[t] = 0;
  __syncthreads();
  uint32_t my_tot = 0, my_pre = 0;
  for (uint32_t j = t; j < gridDim.x * kBinClasses; j += kBinBlock) {
    const uint32_t v = wgc[j];
    my_tot += v;
    if (j / kBinClasses < blockIdx.x) my_pre += v;
  }
  if (my_tot) atomicAdd(&tot[t % kBinClasses], my_tot);
  if (my_pre) atomicAdd(&pre[t % kBinClasses], my_pre);
  __syncthreads();
  if (t < kBinClasses) {
    // classes in descending order (longest packets first): the hardware dispatches tiles in
    // order, so the long tiles start first and the short ones fill the launch's tail
    uint32_t start = pre[t];
    for (int c = (int)t + 1; c < kBinClasses; c++) start += tot[c];
    base[t] = start;
  }
  __syncthreads();
  for (uint64_t i = (uint64_t)blockIdx.x * kBinBlock + t; i < n; i += (uint64_t)gridDim.x * kBinBlock) {
    const uint32_t c = bin_class(lens[i]);
    perm[base[c] + wave_class_slot(c, h)] = (uint32_t)i;
  }
}

hipError_t launch_binning(const uint16_t* lens, uint64_t n, uint32_t* wgc, uint32_t* perm,
                          hipStream_t stream) {
  uint64_t g = (n + 4ull * kBinBlock - 1) / (4ull * kBinBlock);  // ~4 packets per thread
  const int grid = (int)(g < 1 ? 1 : g > kBinMaxWgs ? kBinMaxWgs : g);
  hipLaunchKernelGGL(bin_hist, dim3(grid), dim3(kBinBlock), 0, stream, lens, n, wgc);
  hipLaunchKernelGGL(bin_scatter, dim3(grid), dim3(kBinBlock), 0, stream, lens, n, wgc, perm);
  return hipGetLastError();
}

// ============================================================================================
// xdp_md calling convention (xdp.rs:16-20): image i = [u32 data = 8][u32 data_end = 8 + len]
// [packet bytes] -- the bytes main.rs would be handed for a standard XDP program. One workgroup
// stages 256 packets: it sizes their 16-byte aligned slots, reserves its range with one device
// atomic (workgroups pack in arrival order; every packet keeps its index through the offsets),
// then writes the range's 16-byte chunks: each wave a quarter of the range, its lanes on
// consecutive chunks (each mapped to its packet through the slot prefix sums in LDS), so a wave
// stores 1 KB of contiguous chunks per instruction whatever the packets' lengths. An image
// longer than mem_size is not copied: its length alone makes the batch fault it ST_BADPKT
// (main.rs:20-21).
// (Round 4 copied short images a thread each and long ones a wave each, every chunk from four
// bounds-checked dword loads: 675 us for a 1 Mi mixed 64/1500-byte batch.)

// Image chunk c (image bytes [16c, 16c + 16)) of a packet of len bytes at src: the ctx {data = 8,
// data_end = 8 + len} in its first 8 bytes, packet byte b at image byte 8 + b, zeros at or past
// 8 + len. A chunk inside the packet is one 16-byte load at its (unaligned) address; the first
// and the last: two aligned 16-byte source blocks and a funnel shift (v_alignbyte) per dword.
// (any address: tools/probe_dma_align.hip; a clang vector, not HIP_vector_type, whose 16-byte
// aligned copy constructor would be handed the 1-byte aligned lvalue)
typedef uint32_t u32x4_any __attribute__((ext_vector_type(4), aligned(1)));
__device__ __forceinline__ uint4 xdp_image_chunk(const uint8_t* src, uint32_t len, uint32_t c) {
  // a chunk wholly inside the packet (packet bytes [16c - 8, 16c + 8)): one load, as it lies
  if (c != 0 && 16 * c + 8 <= len) {
    const u32x4_any v = *(const u32x4_any*)(src + 16 * c - 8);
    return make_uint4(v.x, v.y, v.z, v.w);
  }
  const uintptr_t s0 = (uintptr_t)src, end = s0 + len;
  const uintptr_t p = s0 + 16ull * c - 8;  // the source address of image byte 16c
  const uintptr_t a0 = p & ~(uintptr_t)15;
  const uint32_t sh = (uint32_t)(p & 15), q = sh >> 2;
  const u32x4 b0 = blk16(a0, s0, end);
  const u32x4 b1 = sh ? blk16(a0 + 16, s0, end) : u32x4{0u, 0u, 0u, 0u};
  const uint32_t d[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
  uint32_t w[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    // d[k + q] and d[k + q + 1] by selects (q per thread: no dynamic register indexing)
    const uint32_t l0 = (q & 1) ? d[k + 1] : d[k], l1 = (q & 1) ? d[k + 3] : d[k + 2];
    const uint32_t h0 = (q & 1) ? d[k + 2] : d[k + 1];
    const uint32_t h1 = (q & 1) ? (k + 4 < 8 ? d[k + 4] : 0u) : d[k + 3];
    const uint32_t lo = (q & 2) ? l1 : l0, hi = (q & 2) ? h1 : h0;
    w[k] = __builtin_amdgcn_alignbyte(hi, lo, sh & 3);
    const uint32_t b = 16 * c + 4 * k;  // image byte of the dword
    const uint32_t valid = 8 + len > b ? min(8 + len - b, 4u) : 0u;
    w[k] = b == 0 ? 8u : b == 4 ? 8u + len : valid >= 4 ? w[k] : w[k] & ((1u << (8 * valid)) - 1u);
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

__global__ __launch_bounds__(256) void xdp_stage(const uint8_t* __restrict__ frames,
                                                 const uint32_t* __restrict__ offsets,
                                                 const uint16_t* __restrict__ lens, uint64_t stride,
                                                 uint64_t n, uint32_t mem_size,
                                                 uint8_t* __restrict__ dst, uint32_t* doffs,
                                                 uint16_t* dlens, unsigned long long* cursor) {
  __shared__ uint32_t pre[256], len_s[256];
  __shared__ const uint8_t* src_s[256];
  __shared__ unsigned long long base;
  const uint32_t t = threadIdx.x;
  const uint64_t i = (uint64_t)blockIdx.x * 256 + t;
  uint32_t len = 0, copy = 0, slot = 0;
  if (i < n) {
    len = lens ? lens[i] : (uint32_t)(stride < 0xFFFF ? stride : 0xFFFF);
    copy = len + 8 <= mem_size ? len + 8 : 0u;
    slot = ((copy ? copy : 8u) + 15u) & ~15u;
    src_s[t] = frames + (offsets ? (uint64_t)offsets[i] : i * stride);
  }
  pre[t] = slot;
  len_s[t] = copy ? len : 0xFFFFFFFFu;  // (not copied: ST_BADPKT)
  __syncthreads();
  for (uint32_t d = 1; d < 256; d <<= 1) {  // inclusive scan of the slot sizes
    const uint32_t v = t >= d ? pre[t - d] : 0u;
    __syncthreads();
    pre[t] += v;
    __syncthreads();
  }
  if (t == 255) base = atomicAdd(cursor, (unsigned long long)pre[255]);
  __syncthreads();
  if (i < n) {
    doffs[i] = (uint32_t)(base + pre[t] - slot);
    dlens[i] = (uint16_t)(len + 8 < 0xFFFF ? len + 8 : 0xFFFF);
  }
  uint8_t* const o = dst + base;
  const uint32_t chunks = pre[255] / 16;
  // wave w writes the w-th quarter of the range, lane l the chunks l, l + 64, ... of it, four in
  // flight before any store (each chunk's packet: the first j with pre[j] > 16k, found by a binary
  // search for the lane's first chunk, then walked forward -- k grows by 64 chunks, about one
  // packet of the mixed batch)
  const uint32_t wv = t >> 6, ln = t & 63, q = (chunks + 3) / 4;
  const uint32_t kb = min(wv * q, chunks), ke = min(kb + q, chunks);
  uint32_t j = 0;
  if (kb + ln < ke) {
    uint32_t lo = 0, hi = 255;  // (pre[255] > 16 k for every k < chunks)
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (pre[mid] <= 16 * (kb + ln)) lo = mid + 1;
      else hi = mid;
    }
    j = lo;
  }
  for (uint32_t k0 = kb + ln; k0 < ke; k0 += 4 * 64) {
    uint4 v[4];
    uint32_t kk[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const uint32_t k = k0 + 64 * u;
      kk[u] = k;
      v[u] = make_uint4(0u, 0u, 0u, 0u);
      if (k >= ke) continue;
      while (pre[j] <= 16 * k) j++;
      const uint32_t lj = len_s[j];
      if (lj == 0xFFFFFFFFu) {
        kk[u] = 0xFFFFFFFFu;  // (not copied: ST_BADPKT)
        continue;
      }
      v[u] = xdp_image_chunk(src_s[j], lj, (16 * k - (j ? pre[j - 1] : 0u)) / 16);
    }
#pragma unroll
    for (int u = 0; u < 4; u++)
      if (kk[u] < ke) *(uint4*)(o + 16ull * kk[u]) = v[u];
  }
}

hipError_t launch_xdp_stage(const uint8_t* frames, const uint32_t* offsets, const uint16_t* lens,
                            uint64_t stride, uint64_t n, uint32_t mem_size, uint8_t* dst,
                            uint32_t* doffs, uint16_t* dlens, unsigned long long* cursor,
                            hipStream_t stream) {
  const uint64_t grid = (n + 255) / 256;
  hipLaunchKernelGGL(xdp_stage, dim3((unsigned)grid), dim3(256), 0, stream, frames, offsets, lens,
                     stride, n, mem_size, dst, doffs, dlens, cursor);
  return hipGetLastError();
}

#endif  // EBPFEMU_JIT_TEMPLATE

// ============================================================================================
// tile_kernel -- the forward-only fast path for programs of <= 63 micro-ops. The C++ part only
// moves each tile's header windows HBM -> LDS (LDS-DMA) and turns the per-lane counter bucket
// into ballots; everything in between is ONE hand-written asm statement (tile.inc, generated by
// gen_tile.py): per-lane packet address/length, the register file in VGPRs with in-place indexed
// access, min-pc dispatch with basic-block chaining, every tier-0 micro-op, mmu.rs faults, and the
// verdict / r0 / status / register outputs. No per-lane C++ value lives across the statement, so
// the kernel fits 64 VGPRs: 8 waves per SIMD.
// FIXED: the stride layout with 16-byte aligned slots of >= 64 bytes, no lens array and no
// final-image output (a NIC ring of fixed slots): no packet metadata at all.
// ============================================================================================
constexpr uint32_t kTileWaveLds = kWinBytes + kDagMetaBytes;  // window + metadata, 4.5 KiB
constexpr uint32_t kTileWaveLdsPipe = kWinBytes + 2 * kDagMetaBytes;  // two metadata buffers, 5 KiB
// the compiled forward var kernels (tile_body PLEN): metadata buffers with packed u16 lengths
// (dma_meta<true>), 384 bytes each -- a wave's window and two buffers take 4864 bytes, so eight
// 4-wave workgroups and their 80 bytes of static counters fit a CU's 160 KiB of LDS (5 KiB buffers
// left room for seven)
constexpr uint32_t kVarMetaBytes = kWave * 4 + kWave * 2;
constexpr uint32_t kVarWaveLds = kWinBytes + 2 * kVarMetaBytes;       // 4.75 KiB
// ebpf_tile_jit_varl: two windows and two packed metadata buffers per wave, 8.75 KiB (4 workgroups
// of 4 waves per CU)
constexpr uint32_t kVarlWaveLds = 2 * kWinBytes + 2 * kVarMetaBytes;


#define TILE_ASM_OUT [bkt] "=&v"(bkt), [nst] "=&v"(nst)
#define TILE_ASM_IN \
          [ka] "s"(ka), [tile] "s"(t), [winb] "s"(winb), [metab] "s"(metab), \
          [fixed] "i"(FIXED ? 1 : 0), [loops] "i"(LOOPS ? 1 : 0), [aligned] "s"(rfl(aligned)), \
          [plen] "i"(PLEN ? 1 : 0), \
          [o_xdp] "i"(offsetof(LaunchArgs, xdp)), \
          [o_tprog] "i"(offsetof(LaunchArgs, tprog)), \
          [o_tprog_exact] "i"(offsetof(LaunchArgs, tprog_exact)), \
          [o_maxs] "i"(offsetof(LaunchArgs, max_steps)), [o_perm] "i"(offsetof(LaunchArgs, perm)), \
          [o_frames] "i"(offsetof(LaunchArgs, frames)), [o_stride] "i"(offsetof(LaunchArgs, stride)), \
          [o_n] "i"(offsetof(LaunchArgs, n)), [o_mem] "i"(offsetof(LaunchArgs, mem_size)), \
          [o_offsets] "i"(offsetof(LaunchArgs, offsets)), [o_lens] "i"(offsetof(LaunchArgs, lens)), \
          [o_init] "i"(offsetof(LaunchArgs, init_regs)), [o_r10] "i"(offsetof(LaunchArgs, r10)), \
          [o_verdict] "i"(offsetof(LaunchArgs, verdict)), [o_r0] "i"(offsetof(LaunchArgs, r0)), \
          [o_status] "i"(offsetof(LaunchArgs, status)), [o_regs] "i"(offsetof(LaunchArgs, regs_out))
#define TILE_ASM_CLOBBER "s33", "s34", "s35", "s36", "s37", "s38", "s39", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53", "s54", "s55", "s56", "s57", "s58", "s59", "s60", "s61", "s62", "s63", "s64", "s65", "s66", "s67", "s68", "s69", "s70", "s71", "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "vcc", "scc", "memory"
#define TILE_ASM_OPERANDS : TILE_ASM_OUT : TILE_ASM_IN : TILE_ASM_CLOBBER
// the fixed-slot statements' (marker pm=1) pending masks of compiled forward programs (jit.cpp pm_assign)
#define TILE_ASM_CLOBBER_PM "s72", "s73", "s74", "s75", "s76", "s77", "s78", "s79"
// the compiled programs' preloaded window dwords (jit.cpp ldxk_fast): v[64:79]
// and the stack window of memory tier 0.5 (jit.h kStackVgpr, kStackMax / 4 dwords): v[80:95]
// compiled loop programs: the next 64 bytes of each lane's packet, prefetched by every window
// refill (jit.cpp refill_prefetch), in v[56:71]
#define TILE_ASM_CLOBBER_PREFETCH "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", \
    "v65", "v66", "v67", "v68", "v69", "v70", "v71"
#define TILE_ASM_CLOBBER_WINDOW_HI "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79", "v80", \
    "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94", \
    "v95"
// the deep-prefetch loop kernel (jit.cpp refill_prefetch, pf_depth > 1): prefetch stages 1 and 2
// in v[72:87] and v[88:103], their window tags in v104, v105
#define TILE_ASM_CLOBBER_DEEP "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81", \
    "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94", \
    "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105"
#define TILE_ASM_CLOBBER_WINDOW "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", \
    "v73", "v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81", "v82", "v83", "v84", "v85", \
    "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94", "v95"


// JIT: the statement of the compiled-program template kernels (tile_jit.inc; jit.cpp fills in the
// program's code at load time). The compiled fixed-slot kernel (ebpf_tile_jit_fixed, below) has a
// statement of its own that loops over the wave's tiles, with two window buffers per wave (the
// next tile's DMA in flight while the current one runs).
constexpr uint32_t kTileWaveLdsDb = 2 * kWinBytes;

// STACK (with JIT, !FIXED, !LOOPS): the statement of stack-window programs, which also owns
// v[64:95] (the preloaded header window and the stack window, jit.cpp body)
// DEEP (with JIT, LOOPS): the loop statement whose refills prefetch two or three windows ahead
template <bool FIXED, bool LOOPS, bool JIT, bool STACK = false, bool DEEP = false>
__device__ __forceinline__ void tile_body(LaunchArgs& a) {
  constexpr uint32_t WPB = kWavesPerBlock;
  counters_init();
  // the length bins of this batch were consumed by bin_scatter (earlier on the stream): re-zero
  if (LOOPS && a.perm && blockIdx.x == 0 && threadIdx.x < 2 * kBinClasses)
    a.bin_counts[threadIdx.x] = 0;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t wv = rfl(threadIdx.x / kWave);  // wave-uniform: keeps LDS addresses scalar
  // PIPE (the compiled kernels on offsets / lens batches): two metadata buffers per wave, the
  // next tile's offsets and lengths DMA'd while this tile runs, so a tile waits for one HBM round
  // trip (its windows) instead of two (metadata, then windows). Loop kernels: only in batch order
  // (no perm; one tile per wave, so only a wave whose grid slot recurs has a next tile). The
  // statement reads the metadata in its prologue only, and a DMA older than its own loads only
  // makes its vmcnt waits stricter. (Double-buffered windows as well, with three metadata
  // buffers, were measured slower: 9.5 KiB of LDS per wave leaves 4 waves per SIMD instead of 7,
  // profiles/r03_ab_var_db.json; removed in round 5.)
  constexpr bool PIPE = JIT && !FIXED;
  // PLEN: the compiled forward var kernels' packed-length metadata buffers (dma_meta<true>; the
  // statement's prologue reads the lengths as u16, gen_tile.py %[plen])
  constexpr bool PLEN = JIT && !FIXED && !LOOPS;
  const bool pipe = PIPE && !(LOOPS && a.perm);
  constexpr uint32_t kMetaStride = PLEN ? kVarMetaBytes / 4 : 2 * kWave;  // (u32 units)
  WaveLds L;
  L.win = smem + wv * (PLEN ? kVarWaveLds : PIPE ? kTileWaveLdsPipe : kTileWaveLds);
  L.meta_off = (uint32_t*)(L.win + kWinBytes);
  L.meta_len = L.meta_off + kWave;
  // window buffer w and metadata buffer m of this wave (offsets, then lengths: 512 bytes each, or
  // 384 with PLEN)
  auto bufs = [&](uint32_t w, uint32_t m) {
    WaveLds x;
    x.win = L.win + w * kWinBytes;
    x.meta_off = L.meta_off + m * kMetaStride;
    x.meta_len = x.meta_off + kWave;
    return x;
  };
  uint32_t mb = 0;  // PIPE: the metadata buffer of the current tile (0 or 1)
  const uint64_t wave_slot = (uint64_t)blockIdx.x * WPB + wv;
  const uint64_t total_waves = (uint64_t)gridDim.x * WPB;
  const auto ka = __builtin_amdgcn_kernarg_segment_ptr();

  uint32_t cnt[7] = {0, 0, 0, 0, 0, 0, 0};  // per wave: < 2^32 packets
  uint32_t retired = 0;                      // per lane: <= 63 steps per tile
  // diagnostics (EBPFEMU_TRACE=1, tools/trace_loop.py; the JIT loop kernels only): s_memrealtime stamps of
  // the wave's first tile -- entry, window ready, statement done, counters flushed -- its lane 0's
  // packet length and the hardware ids
  // (the forward var kernels, tools/trace_var.py: window ready / statement done of each of the
  // wave's first five tiles in slots 1 + 2i / 2 + 2i, its tile count in slot 15)
  // (the var kernels' stamps cost registers: built only with -DEBPFEMU_VAR_TRACE, tools/trace_var.py)
#ifdef EBPFEMU_VAR_TRACE
  constexpr bool kTraceHere = JIT;
#else
  constexpr bool kTraceHere = JIT && LOOPS;
#endif
  uint64_t* const trace =
      kTraceHere && a.trace && wave_slot < kTraceWaves ? a.trace + wave_slot * kTraceSlots : nullptr;
  uint32_t ti = 0;  // (var trace: the wave's tile ordinal)
  auto stamp = [&](uint32_t slot) {
    uint64_t ts;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(ts)::"memory");
    if (threadIdx.x % kWave == 0) trace[slot] = ts;
  };
  if (trace) stamp(0);

  if (pipe && wave_slot < a.n_tiles) {  // the first tile's metadata
    uint32_t lane;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane));
    dma_meta<PLEN>(a, L, 0, wave_slot, lane);
  }
  for (uint64_t tile = wave_slot; tile < a.n_tiles;) {
    // the lane index is re-derived inside the loop (volatile: not hoistable), so no per-lane
    // address of the window DMA stays live across the asm statement
    uint32_t aligned = 1;  // every packet base of the tile 16-byte aligned (loop-mode refills)
    // this tile's window and metadata buffers (without PIPE: buffer 0)
    const WaveLds Lc = bufs(0u, PIPE ? mb : 0u);
    const uint32_t winb = lds_addr(Lc.win);
    const uint32_t metab = lds_addr(Lc.meta_off);
    if (!FIXED) {  // (FIXED: the asm statement DMAs the windows itself)
      uint32_t lane;
      asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane));
      const uint64_t pkt = tile * kWave + lane;
      const bool valid = pkt < a.n;
      const bool sw = stride_windows(a);
      if (pipe) {
        // (metadata already in flight: issued for this tile by the previous iteration)
      } else if (LOOPS && a.perm) {  // length-binned order: gather this tile's packet metadata
        const uint64_t src = valid ? (uint64_t)a.perm[pkt] : 0ull;
        if (a.offsets)
          dma_x1(valid ? (uintptr_t)(a.offsets + src) : (uintptr_t)a.prog, lds_addr(L.meta_off));
        if (a.lens)
          dma_u16(valid ? (uintptr_t)(a.lens + src) : (uintptr_t)a.prog, lds_addr(L.meta_len));
      } else {
        dma_meta<PLEN>(a, L, 0, tile, lane);
      }
      if (sw) dma_window_stride(a, L.win, tile, lane);
      dma_wait();
      uintptr_t pb;
      uint32_t ml;
      meta_of<PLEN>(a, Lc, 0, tile, lane, pb, ml);
      const bool co = sw || ballot(valid && ml != 0 && (pb & 15) != 0) == 0;
      aligned = co ? 1u : 0u;
      if (co) {
        if (!sw) {
          dma_window<PLEN>(a, Lc, 0, 0, tile, lane);
          dma_wait();
        }
      } else {
        stage_window_lane(L.win + lane * kWin, win_swz(lane), (const uint8_t*)pb,
                          valid ? ml : 0u, valid);
      }
      if (!LOOPS && a.xdp) xdp_window(L.win + lane * kWin, win_swz(lane), ml);
      __builtin_amdgcn_s_waitcnt(0xc07f);  // the window's LDS writes / metadata reads: done
      // PIPE: the next tile's metadata into the other buffer (last read by the previous tile's
      // statement, which has finished), landing while this tile runs
      const uint64_t ntl = rfl64(tile) + total_waves;
      if (pipe && ntl < a.n_tiles) dma_meta<PLEN>(a, bufs(0, mb ^ 1u), 0, ntl, lane);
    }
    const uint64_t t = rfl64(tile);
    const uint64_t nt = t + total_waves;
    uint32_t bkt, nst;
    if (trace && !LOOPS && ti < 5) stamp(1 + 2 * ti);
    if (trace && LOOPS && t == wave_slot) {
      stamp(1);
      if (!FIXED && threadIdx.x % kWave == 0) {
        uintptr_t mb;
        uint32_t ml;
        meta_of<PLEN>(a, Lc, 0, tile, 0, mb, ml);
        trace[4] = ml;
      }
    }
    if constexpr (JIT && LOOPS && STACK) {  // stack-window loop programs: v[56:95] too
      asm volatile(
#include "tile_jit_stack.inc"
          TILE_ASM_OPERANDS, TILE_ASM_CLOBBER_PREFETCH, TILE_ASM_CLOBBER_WINDOW_HI);
    } else if constexpr (JIT && LOOPS && DEEP) {  // + the deeper prefetch's stages
      asm volatile(
#include "tile_jit_deep.inc"
          TILE_ASM_OPERANDS, TILE_ASM_CLOBBER_PREFETCH, TILE_ASM_CLOBBER_DEEP);
    } else if constexpr (JIT && LOOPS) {  // + the refill prefetch registers of compiled loop programs
      asm volatile(
#include "tile_jit.inc"
          TILE_ASM_OPERANDS, TILE_ASM_CLOBBER_PREFETCH);
    } else if constexpr (JIT && STACK) {
      asm volatile(
#include "tile_jit_stack.inc"
          TILE_ASM_OPERANDS, TILE_ASM_CLOBBER_WINDOW);
    } else if constexpr (JIT) {
      asm volatile(
#include "tile_jit.inc"
          TILE_ASM_OPERANDS);
    } else {
      asm volatile(
#include "tile.inc"
          TILE_ASM_OPERANDS);
    }

    // ---- final image (Emu.state.mmu.memory): the window, then the packet, then zeros ----
    if (!FIXED && a.mem_out) {
      uint32_t ln;
      asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
      const uint64_t slot = tile * kWave + ln;
      const uint64_t pk = slot < a.n && LOOPS && a.perm ? (uint64_t)a.perm[slot] : slot;
      if (slot < a.n) {
        uintptr_t mb;
        uint32_t ml;
        meta_of<PLEN>(a, Lc, 0, tile, ln, mb, ml);
        // (xdp_md in place: the image is the packet 8 bytes further on, behind its ctx)
        const uint32_t len = a.xdp ? min(ml, 0xffffu) + 8u : ml;
        const uint8_t* base = (const uint8_t*)mb - (a.xdp ? 8 : 0);
        const uint32_t mem_size = a.mem_size;
        uint8_t* mo = a.mem_out + pk * (uint64_t)mem_size;
        const uint32_t m = min(len, mem_size);
        for (uint32_t d = 0; d < (mem_size + 3) / 4; d++) {
          uint32_t v;
          if (d * 4 >= m) v = 0u;
          else if (!LOOPS && d * 4 < (uint32_t)kWin)  // (loop mode may have moved the window)
            v = (uint32_t)win_read(Lc.win + ln * kWin, win_swz(ln), d * 4, 4, len);
          else v = (uint32_t)pkt_read(base, d * 4, 4, len);
          put_image(mo, d, v, mem_size);
        }
      }
    }
    if (JIT && a.deopt) {  // store mode: lanes that left for the general interpreter (bucket 8)
      const uint64_t dm = ballot(bkt == 8u);
      if (dm) {
        uint32_t ln;
        asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(dm >> 32),
                                                        __builtin_amdgcn_mbcnt_lo((uint32_t)dm, 0u));
        const uint32_t first = (uint32_t)__builtin_ctzll(dm);
        uint32_t base = 0;
        if (ln == first)
          base = __hip_atomic_fetch_add(a.deopt, (uint32_t)__builtin_popcountll(dm),
                                        __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        base = __builtin_amdgcn_readlane(base, first);
        const uint64_t slot = t * kWave + ln;
        if (bkt == 8u)
          a.deopt_idx[base + rank] =
              (uint32_t)(LOOPS && a.perm ? (uint64_t)a.perm[slot] : slot);
      }
    }
#pragma unroll
    for (int b = 0; b < 7; b++) cnt[b] += __builtin_popcountll(ballot(bkt == (uint32_t)b));
    retired += nst;
    if (trace && LOOPS && t == wave_slot) stamp(2);
    if (trace && !LOOPS && ti < 5) stamp(2 + 2 * ti);
    ti++;
    tile = nt;
    if (pipe) mb ^= 1u;  // (without the prefetch: buffer 0 always)
  }
  uint64_t cnt64[7];
#pragma unroll
  for (int b = 0; b < 7; b++) cnt64[b] = cnt[b];
  uint32_t ln;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
  if (trace) {
    stamp(12);
    uint32_t xcc, hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)\n\ts_getreg_b32 %1, hwreg(HW_REG_HW_ID)"
                 : "=s"(xcc), "=s"(hw));
    if (ln == 0) trace[14] = ((uint64_t)xcc << 32) | hw;
    if (!LOOPS && ln == 0) trace[15] = ti;
  }
  flush_counters<WPB>(a, cnt64, retired, smem, ln, wv);
  if (trace) stamp(13);
}

#ifndef EBPFEMU_JIT_TEMPLATE
template <bool FIXED, bool LOOPS>
__global__ __launch_bounds__(kBlock, 8) void tile_kernel(LaunchArgs a) {
  tile_body<FIXED, LOOPS, false>(a);
}
#else
// The JIT template kernels (build/tile_jit.s, embedded in the library): jit.cpp inserts each
// program's compiled code at the marker of their statement and assembles the result.
// (one workgroup of 16 waves per CU: its two window buffers per wave take the LDS, so 128 VGPRs
// are free)
//
// ebpf_tile_jit_fixed: the wave's whole run of tiles in one asm statement (tile_jit_loop.inc,
// gen_tile.py jit_statement_loop), re-entered only every 511 tiles to unpack the per-lane packed
// counter buckets. Launch conditions (jit_fixed_ok): the fixed-slot layout, n_tiles < 2^31 and
// 64 * stride < 2^32, so tile indices and tile byte offsets are 32-bit scalars.
//
// SINGLE (ebpf_tile_jit_fixed_occ, WAVES = kOccWaves): the occupancy variant for issue-bound
// programs (a long rule chain: hundreds of steps per packet for 64 bytes of HBM) -- one window
// buffer per wave (tile_jit_loop1.inc claims and DMAs the next tile when the current one is done),
// and a statement that owns only v[0:55] (the compiled code has no preloaded window, jit.cpp
// Compiler::body occ): under 80 VGPRs, so 3 workgroups of 8 waves fit a CU -- 6 waves per SIMD
// (its ~100 SGPRs allow no more) instead of 4, to hide the min-pc scheme's exec / vcc chains.
template <uint32_t WAVES, bool SINGLE>
__device__ __forceinline__ void fixed_body(LaunchArgs& a) {
  constexpr uint32_t kWaveLds = SINGLE ? kWinBytes : kTileWaveLdsDb;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t wv = rfl(threadIdx.x / kWave);
  // the wave's first tile's windows go out before the workgroup's start barrier (counters_init:
  // the 16 waves of a workgroup do not start together), the statement then skips that DMA
  // (A/B, round 4: 14.17 vs 14.72 us one launch, profiles/r04_ab_fixed_early_dma.log)
  uint32_t first = 1;
  {
    const uint32_t t0 = blockIdx.x + wv * gridDim.x;
    if (t0 < a.n_tiles) {
      uint32_t ln;
      asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
      dma_window_stride(a, smem + wv * kWaveLds, t0, ln);
      first = 0;
    }
  }
  counters_init();
  uint32_t winb = lds_addr(smem + wv * kWaveLds), nwinb = SINGLE ? winb : winb + kWinBytes;
  const uint32_t wx = winb ^ nwinb;
  uint32_t lane;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane));
  // lane l's window-DMA source offset within a tile (fixed_dma_db in gen_tile.py), its packet's
  // offset, its LDS window offset and chunk swizzle -- loop-invariant
  const uint64_t dmaoff =
      (uint64_t)(lane >> 2) * a.stride + (uint64_t)(((lane & 3u) ^ ((lane >> 4) & 3u)) * 16u);
  // (xdp_md in place: BASE = the packet - 8, LEN = 8 + len, the ctx synthesised by the program's
  // code, jit.cpp xdp_shift)
  const uint64_t laneoff = (uint64_t)lane * a.stride - (a.xdp ? 8u : 0u);
  const uint32_t lane64 = lane << 6, swz = ((lane >> 2) & 3u) << 4;
  const uint64_t lanep = lane;
  const uint32_t nxa = lds_addr(&wg_counters()->next), one = 1;
  const uint32_t grid = gridDim.x, wg = blockIdx.x;
  // (scalars computed with selects go through readfirstlane: an "s" operand left in a VGPR by the
  // compiler would be printed as one)
  const uint32_t ntiles = rfl((uint32_t)a.n_tiles), nfull = rfl((uint32_t)(a.n / kWave));
  const uint32_t nfast = rfl(a.stride == (uint64_t)kWin ? nfull : 0u);
  const uint32_t tbytes = rfl((uint32_t)(a.stride * kWave));
  const uint32_t lenc = rfl(a.xdp ? (uint32_t)min(a.stride, (uint64_t)0xffff) + 8u
                                 : a.stride >> 32 ? 0xffffffffu : (uint32_t)a.stride);
  const uint32_t xdpf = rfl(a.xdp);
  const uint32_t kflags = rfl((a.init_regs ? 1u : 0u) | (a.r0 ? 2u : 0u) | (a.status ? 4u : 0u) |
                              (a.regs_out ? 8u : 0u));
  const uint32_t initx = rfl(kflags & 9u), oflags = rfl(kflags & 14u);
  const uint64_t ka = (uint64_t)__builtin_amdgcn_kernarg_segment_ptr();
  uint64_t* const trace = a.trace && (uint64_t)wg * WAVES + wv < kTraceWaves
                              ? a.trace + ((uint64_t)wg * WAVES + wv) * kTraceSlots : nullptr;
  auto stamp = [&](uint32_t slot) {
    uint64_t ts;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(ts)::"memory");
    if (lane == 0) trace[slot] = ts;
  };
  if (trace) stamp(0);

  uint32_t cnt[7] = {0, 0, 0, 0, 0, 0, 0};
  uint32_t ret = 0, ordv = 0, tile = wg + wv * grid, rounds = 0;
  uint64_t retired = 0;
  while (tile < ntiles) {
    uint64_t acc = 0;
    uint32_t cdn, ntile;
#define FIXED_OPERANDS \
        : [tile] "+s"(tile), [winb] "+s"(winb), [nwinb] "+s"(nwinb), [ordv] "+v"(ordv), \
          [acc] "+v"(acc), [ret] "+v"(ret), [cdn] "=&s"(cdn), [ntile] "=&s"(ntile) \
        : [first] "s"(first), [ka] "s"(ka), [k_tprog] "s"(a.tprog), [k_frames] "s"(a.frames), \
          [fr_lo] "s"((uint32_t)(uintptr_t)a.frames), [fr_hi] "s"((uint32_t)((uintptr_t)a.frames >> 32)), \
          [k_stride] "s"(a.stride), [k_n] "s"(a.n), [k_mem] "s"(a.mem_size), [k_r10] "s"(a.r10), \
          [k_verdict] "s"(a.verdict), [vd_lo] "s"((uint32_t)(uintptr_t)a.verdict), \
          [vd_hi] "s"((uint32_t)((uintptr_t)a.verdict >> 32)), [k_flags] "s"(kflags), \
          [initx] "s"(initx), [oflags] "s"(oflags), [grid] "s"(grid), [wg] "s"(wg), \
          [wpb] "i"(WAVES), [ntiles] "s"(ntiles), [nfull] "s"(nfull), [nfast] "s"(nfast), \
          [tbytes] "s"(tbytes), [lenc] "s"(lenc), [wx] "s"(wx), \
          [dmaoff] "v"(dmaoff), [laneoff] "v"(laneoff), [lane64] "v"(lane64), [swz] "v"(swz), \
          [lanep] "v"(lanep), [nxa] "v"(nxa), [one] "v"(one), [aligned] "s"(one), \
          [fixed] "i"(1), [loops] "i"(0), [xdpf] "s"(xdpf), \
          [o_init] "i"(offsetof(LaunchArgs, init_regs)), \
          [o_r0] "i"(offsetof(LaunchArgs, r0)), [o_status] "i"(offsetof(LaunchArgs, status)), \
          [o_regs] "i"(offsetof(LaunchArgs, regs_out))
    if constexpr (SINGLE) {
      asm volatile(
#include "tile_jit_loop1.inc"
          FIXED_OPERANDS
          : TILE_ASM_CLOBBER, TILE_ASM_CLOBBER_PM);
    } else {
      // (+ store mode's deopt list and overflow images: gen_tile.py STORE_DEOPT_FIXED)
      const uint32_t dfl = rfl((a.deopt ? 1u : 0u) | (a.deopt_pass == 2 ? 2u : 0u));
      asm volatile(
#include "tile_jit_loop.inc"
          FIXED_OPERANDS, [k_deopt] "s"(a.deopt), [k_dix] "s"(a.deopt_idx), [k_ovf] "s"(a.ovf),
          [dfl] "s"(dfl)
          : TILE_ASM_CLOBBER, TILE_ASM_CLOBBER_WINDOW, TILE_ASM_CLOBBER_PM);
    }
#undef FIXED_OPERANDS
    // (an asm statement with VGPR outputs is divergent as a whole to the compiler: the scalar
    // loop state goes back through readfirstlane, which is free on an SGPR)
    tile = rfl(tile);
    winb = rfl(winb);
    nwinb = rfl(nwinb);
    first = 0;
    rounds++;
    // the packed buckets (seven 9-bit fields per lane) summed over the wave two at a time, as
    // 16-bit fields (<= 64 x 511), and this round's retired steps (<= 64 x 511 x 62 < 2^32)
#pragma unroll
    for (int b = 0; b < 7; b += 2) {
      const uint32_t q = (uint32_t)(acc >> (9 * b)) & 511u;
      const uint32_t s =
          wave_sum_u32(b < 6 ? q | ((uint32_t)(acc >> (9 * b + 9)) & 511u) << 16 : q);
      cnt[b] += s & 0xffffu;
      if (b < 6) cnt[b + 1] += s >> 16;
    }
    retired += wave_sum_u32(ret);
    ret = 0;
  }
  if (trace) {
    stamp(12);
    uint32_t xcc, hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)\n\ts_getreg_b32 %1, hwreg(HW_REG_HW_ID)"
                 : "=s"(xcc), "=s"(hw));
    if (lane == 0) {
      trace[14] = ((uint64_t)xcc << 32) | hw;
      trace[15] = rounds;
    }
  }
  uint64_t cnt64[7];
#pragma unroll
  for (int b = 0; b < 7; b++) cnt64[b] = cnt[b];
  flush_counters<WAVES, true>(a, cnt64, retired, smem, lane, wv);
  if (trace) stamp(13);
}
extern "C" __global__ __launch_bounds__(kDbBlock, 1) void ebpf_tile_jit_fixed(LaunchArgs a) {
  fixed_body<kDbWaves, false>(a);
}
extern "C" __global__ __launch_bounds__(kOccBlock, kOccWgsPerCu) void ebpf_tile_jit_fixed_occ(LaunchArgs a) {
  fixed_body<kOccWaves, true>(a);
}
extern "C" __global__ __launch_bounds__(kOccWideBlock, kOccWideWgsPerCu) void ebpf_tile_jit_fixed_occw(
    LaunchArgs a) {
  fixed_body<kOccWideWaves, true>(a);
}
extern "C" __global__ __launch_bounds__(kBlock, 7) void ebpf_tile_jit_var(LaunchArgs a) {
  tile_body<false, false, true>(a);
}
// ebpf_tile_jit_varl: offsets + lens batches (varl_ok in launch_interp: offsets present, lengths
// 4-byte aligned or absent, no final images, n_tiles < 2^31) -- the wave's tiles tile, tile + W,
// ... in one asm statement (tile_jit_varl.inc, gen_tile.py jit_statement_varl) with two window
// buffers and two packed metadata buffers per wave (kVarlWaveLds; 4 workgroups of 4 waves per
// CU), so a tile's windows are in flight while the one before it runs. Tiles whose packets are
// not all 16-byte aligned (a capture's records) are DMA'd straight from the packets (the last
// chunk of a short packet from the aligned block below, shifted into place at the tile's top).
// The C++ here only starts the wave's first tile, stages the windows of a tile the statement
// hands back (the batch's partial last tile) and unpacks the per-lane packed counter buckets.
#define VARL_OPERANDS \
        : [tile] "+s"(tile), [winb] "+s"(winb), [nwinb] "+s"(nwinb), [metab] "+s"(metab), \
          [nmetab] "+s"(nmetab), [acc] "+v"(acc), [ret] "+v"(ret), [cdn] "=&s"(cdn), \
          [stage] "=&s"(stg), [mis] "+s"(mis), [dmask] "=&s"(dmask) \
        : [ka] "s"(ka), [k_frames] "s"(a.frames), [fr_lo] "s"((uint32_t)(uintptr_t)a.frames), \
          [of_lo] "s"((uint32_t)(uintptr_t)a.offsets), \
          [of_hi] "s"((uint32_t)((uintptr_t)a.offsets >> 32)), \
          [ln_lo] "s"((uint32_t)(uintptr_t)a.lens), [ln_hi] "s"((uint32_t)((uintptr_t)a.lens >> 32)), \
          [fc] "v"(fc), [lb] "v"(lb), [db] "v"(db), \
          [tbytes] "s"(rfl(tbytes)), [s16] "s"(rfl(s16)), [lane] "v"(lane), \
          [k_deopt] "s"(a.deopt), [k_dix] "s"(a.deopt_idx), [k_ovf] "s"(a.ovf), \
          [k_n] "s"(a.n), [k_mem] "s"(a.mem_size), [k_r10] "s"(a.r10), \
          [vd_lo] "s"((uint32_t)(uintptr_t)a.verdict), \
          [vd_hi] "s"((uint32_t)((uintptr_t)a.verdict >> 32)), [fl] "s"(rfl(fl)), \
          [W] "s"(W), [ntiles] "s"(ntiles), [nfull] "s"(rfl(nfull)), [lenc] "s"(rfl(lenc)), \
          [xdpf] "s"(rfl(xdpf)), \
          [wx] "s"(wx), [mx] "s"(mx), [lane4] "v"(lane4), [lane2] "v"(lane2), [moff] "v"(moff), \
          [loff] "v"(loff), [c16] "v"(c16), [lane64] "v"(lane64), [swz] "v"(swz), \
          [lanep] "v"(lanep), [aligned] "s"(rfl(one)), [fixed] "i"(0), [loops] "i"(0), \
          [o_init] "i"(offsetof(LaunchArgs, init_regs)), [o_r0] "i"(offsetof(LaunchArgs, r0)), \
          [o_status] "i"(offsetof(LaunchArgs, status)), \
          [o_regs] "i"(offsetof(LaunchArgs, regs_out)) \
        : TILE_ASM_CLOBBER, TILE_ASM_CLOBBER_WINDOW
template <bool STACK>
__device__ __forceinline__ void varl_body(LaunchArgs& a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t wv = rfl(threadIdx.x / kWave);
  uint8_t* const wbase = smem + wv * kVarlWaveLds;  // [window 0][window 1][metadata 0][metadata 1]
  uint32_t winb = lds_addr(wbase), nwinb = winb + kWinBytes;
  uint32_t metab = lds_addr(wbase + 2 * kWinBytes), nmetab = metab + kVarMetaBytes;
  const uint32_t win0 = winb, meta0 = metab;
  const uint32_t wx = winb ^ nwinb, mx = metab ^ nmetab;
  uint32_t lane;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane));
  // per-lane constants of the statement: its own metadata (offset, packed length), the window
  // DMA's (packet 16r + l/4's offset and length at +64r / +32r, the chunk it moves), its window
  const uint32_t lane4 = lane * 4, lane2 = 256 + lane * 2, moff = lane & ~3u;
  const uint32_t loff = 256 + ((lane >> 2) << 1), c16 = ((lane & 3u) ^ ((lane >> 4) & 3u)) * 16u;
  const uint32_t lane64 = lane << 6, swz = ((lane >> 2) & 3u) << 4;
  const uint64_t lanep = lane;
  const uint64_t fc = (uint64_t)(uintptr_t)a.frames + c16;  // (the window DMA: frames + chunk)
  // the stride layout (no offsets, 16-byte aligned slots of 64 bytes or more): lane l's packet at
  // lb + tile * 64 * stride, round r's DMA source at db + tile * 64 * stride + r * 16 * stride
  const uint64_t lb = (uint64_t)(uintptr_t)a.frames + (uint64_t)lane * a.stride;
  const uint64_t db = (uint64_t)(uintptr_t)a.frames + (uint64_t)(lane >> 2) * a.stride + c16;
  const uint32_t tbytes = (uint32_t)(a.stride * kWave), s16 = (uint32_t)(a.stride * 16);
  const uint32_t W = gridDim.x * kWavesPerBlock;
  const uint32_t ntiles = rfl((uint32_t)a.n_tiles), nfull = rfl((uint32_t)(a.n / kWave));
  const uint32_t haslen = rfl(a.lens ? 1u : 0u), xdpf = rfl(a.xdp);
  const uint32_t lenc = rfl(stride_len(a));
  const uint32_t kflags = rfl((a.init_regs ? 1u : 0u) | (a.r0 ? 2u : 0u) | (a.status ? 4u : 0u) |
                              (a.regs_out ? 8u : 0u));
  const uint32_t initx = rfl(kflags & 9u), oflags = rfl(kflags & 14u), one = 1;
  // the statement's flags (gen_tile.py jit_statement_varl)
  const uint32_t fl = kflags | (initx ? 16u : 0u) | (oflags ? 32u : 0u) | (haslen ? 64u : 0u) |
                      (xdpf ? 128u : 0u) | (a.offsets ? 0u : 256u) | (a.verdict ? 512u : 0u) |
                      (a.deopt_pass == 2 ? 1024u : 0u);
  const uint64_t ka = (uint64_t)__builtin_amdgcn_kernarg_segment_ptr();
  // the wave's current window / metadata buffers as generic pointers (staging)
  auto buf = [&](uint32_t wb, uint32_t mb) {
    WaveLds x;
    x.win = wbase + (wb == win0 ? 0u : kWinBytes);
    x.meta_off = (uint32_t*)(wbase + 2 * kWinBytes + (mb == meta0 ? 0u : kVarMetaBytes));
    x.meta_len = x.meta_off + kWave;
    return x;
  };
  // tile t's windows into X, lane by lane (its metadata in X; a partial tile's is fetched here)
  auto stage = [&](uint32_t t, const WaveLds& X) {
    if ((uint64_t)(t + 1) * kWave > a.n) {
      dma_meta<true>(a, X, 0, t, lane);
      dma_wait();
    }
    uintptr_t pb;
    uint32_t ml;
    meta_of<true>(a, X, 0, t, lane, pb, ml);
    const bool valid = (uint64_t)t * kWave + lane < a.n;
    stage_window_lane(X.win + lane * kWin, win_swz(lane), (const uint8_t*)pb, valid ? ml : 0u,
                      valid);
  };

  uint32_t cnt[7] = {0, 0, 0, 0, 0, 0, 0};
  uint64_t retired = 0;
  uint32_t tile = blockIdx.x * kWavesPerBlock + wv;
  uint32_t mis = 0;  // bit 0: the current tile's windows came from unaligned packets (tailfix)
  // the first two tiles' metadata at once, before the workgroup's start barrier (as the
  // fixed-slot kernel's first DMA); then the first tile's windows (DMA'd when whole and aligned):
  // the statement's first wait is for those windows alone. (Tried: both first tiles' windows in
  // flight from the start, as the fixed-slot kernel's opening burst -- 17.6 vs 16.6 us per 1
  // Mi-packet 5-tuple batch, A/B on one box.)
  const WaveLds X = buf(winb, metab);
  if (tile < ntiles) {
    dma_meta<true>(a, X, 0, tile, lane);
    if (tile + W < ntiles) dma_meta<true>(a, buf(nwinb, nmetab), 0, tile + W, lane);
  }
  counters_init();
  if (tile < ntiles) {
    dma_wait();
    uintptr_t pb;
    uint32_t ml;
    meta_of<true>(a, X, 0, tile, lane, pb, ml);
    const bool whole = (uint64_t)(tile + 1) * kWave <= a.n;
    if (whole) {
      mis = ballot(ml != 0 && (pb & 15) != 0) != 0 ? 1u : 0u;
      if (mis) dma_window_any(a, X, tile, lane);
      else dma_window<true>(a, X, 0, 0, tile, lane);
    } else {
      stage(tile, X);
    }
  }
  while (tile < ntiles) {
    uint64_t acc = 0;
    uint32_t ret = 0, cdn, stg;
    uint64_t dmask;  // (store mode: the lanes whose overflow image is live, per tile)
    if constexpr (STACK) {
      asm volatile(
#include "tile_jit_varl_stack.inc"
          VARL_OPERANDS);
    } else {
      asm volatile(
#include "tile_jit_varl.inc"
          VARL_OPERANDS);
    }
    // (scalar loop state back through readfirstlane: the statement has VGPR outputs)
    tile = rfl(tile);
    winb = rfl(winb);
    nwinb = rfl(nwinb);
    metab = rfl(metab);
    nmetab = rfl(nmetab);
    stg = rfl(stg);
#pragma unroll
    for (int b = 0; b < 7; b += 2) {
      const uint32_t q = (uint32_t)(acc >> (9 * b)) & 511u;
      const uint32_t s =
          wave_sum_u32(b < 6 ? q | ((uint32_t)(acc >> (9 * b + 9)) & 511u) << 16 : q);
      cnt[b] += s & 0xffffu;
      if (b < 6) cnt[b + 1] += s >> 16;
    }
    retired += wave_sum_u32(ret);
    mis = rfl(mis);
    if (tile < ntiles && stg) {  // a tile the statement hands back: stage its windows
      dma_wait();                // (the next tile's metadata)
      stage(tile, buf(winb, metab));
      mis = 0;
    }
  }
  uint64_t cnt64[7];
#pragma unroll
  for (int b = 0; b < 7; b++) cnt64[b] = cnt[b];
  flush_counters<kWavesPerBlock, true>(a, cnt64, retired, smem, lane, wv);
}
#undef VARL_OPERANDS
extern "C" __global__ __launch_bounds__(kBlock, 4) void ebpf_tile_jit_varl(LaunchArgs a) {
  varl_body<false>(a);
}
// stack-window programs (memory tier 0.5, not store mode): the stack window in v[80:95] too
extern "C" __global__ __launch_bounds__(kBlock, 4) void ebpf_tile_jit_varl_stack(LaunchArgs a) {
  varl_body<true>(a);
}
// stack-window programs (memory tier 0.5) on offsets + lens, stride + lens and xdp_md batches:
// the var kernel with the preloaded header window and the stack window in v[64:95]
extern "C" __global__ __launch_bounds__(kBlock, 4) void ebpf_tile_jit_var_stack(LaunchArgs a) {
  tile_body<false, false, true, true>(a);
}
// loop programs (back edges, or a step budget that can bind): the exact budget and refillable
// windows as tile_kernel<false, true>
// (6 waves per SIMD: the prefetch registers take the kernel past 64 VGPRs)
extern "C" __global__ __launch_bounds__(kBlock, 5) void ebpf_tile_jit_loop(LaunchArgs a) {
  tile_body<false, true, true>(a);
}
// loop programs whose refills prefetch two or three windows ahead (jit.cpp refill_prefetch,
// EBPFEMU_PF_DEPTH): 32 more prefetch VGPRs, 4 waves per SIMD
extern "C" __global__ __launch_bounds__(kBlock, 4) void ebpf_tile_jit_loop_deep(LaunchArgs a) {
  tile_body<false, true, true, false, true>(a);
}
// stack-window loop programs (memory tier 0.5 with back edges or a binding budget): the stack
// window in v[80:95]
extern "C" __global__ __launch_bounds__(kBlock, 4) void ebpf_tile_jit_loop_stack(LaunchArgs a) {
  tile_body<false, true, true, true>(a);
}
#endif

#ifndef EBPFEMU_JIT_TEMPLATE

// Folds the shards into the caller's counters (EBPFEMU_FOLD=kernel A/B mode): one workgroup,
// launched after the interpreter on the same stream.
__global__ __launch_bounds__(kCounterShards * 8) void fold_counters(uint64_t* shards,
                                                                     uint64_t* counters) {
  __shared__ uint64_t fold[kCounterShards * 8];
  fold[threadIdx.x] =
      __hip_atomic_exchange(&shards[threadIdx.x], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  if (threadIdx.x < 8) {
    uint64_t t = 0;
    for (int i = threadIdx.x; i < kCounterShards * 8; i += 8) t += fold[i];
    if (t) atomicAdd((unsigned long long*)&counters[threadIdx.x], (unsigned long long)t);
  }
}

// Adds src[0..7] into dst[0..7] (ebpf_run_batch_multi: the all-reduced totals of one call into the
// caller's counters, which are accumulated, never overwritten).
__global__ __launch_bounds__(64) void counters_add(const uint64_t* src, uint64_t* dst) {
  if (threadIdx.x < EBPF_NCOUNTERS && src[threadIdx.x])
    atomicAdd((unsigned long long*)&dst[threadIdx.x], (unsigned long long)src[threadIdx.x]);
}

hipError_t launch_counters_add(const uint64_t* src, uint64_t* dst, hipStream_t stream) {
  hipLaunchKernelGGL(counters_add, dim3(1), dim3(64), 0, stream, src, dst);
  return hipGetLastError();
}

// Counter fold: in-kernel with counted shard words (default), or fold_counters after the launch
// (EBPFEMU_FOLD=kernel: fold_counters for every launch -- the test of the path that launches whose
// per-shard sums could reach 2^48 take, tests/test_knobs.py)
static bool g_fold_kernel = [] {
  const char* e = getenv("EBPFEMU_FOLD");
  return e && e[0] == 'k';
}();

static uint32_t lds_bytes_for(int kind, uint32_t n_uops, bool jit_loop = false) {
  if (kind == kKindLoop)  // (the compiled loop kernels: + the second metadata buffer)
    return kWavesPerBlock * (jit_loop ? kTileWaveLdsPipe : kTileWaveLds);
  if (kind == kKindDag)  // the program is fetched by SMEM
    return kWavesPerBlock * (n_uops <= kTileMaxUops ? kTileWaveLds : kDagWaveLds);
  const uint32_t prog = n_uops <= (uint32_t)kMaxLdsUops ? n_uops * (uint32_t)sizeof(Uop) : 0u;
  uint32_t rest = kind == kKindTier0 ? kWavesPerBlock * kWaveLds0 : 0u;
  return prog + rest;
}

// Kernel variant for a program: tier (memory model), LDS-staged program, scheduler width.
template <int TIER>
static const void* variant(uint32_t n_uops) {
  if (n_uops <= 64) return (const void*)interp_kernel<TIER, true, 1>;
  if (n_uops <= 256) return (const void*)interp_kernel<TIER, true, 4>;
  if (n_uops <= (uint32_t)kMaxLdsUops) return (const void*)interp_kernel<TIER, true, 0>;
  return (const void*)interp_kernel<TIER, false, 0>;
}



// Programs that run on tile_kernel (kKindLoop always does).
static bool tile_kernel_for(int kind, uint32_t n_uops) {
  return kind == kKindLoop || (kind == kKindDag && n_uops <= kTileMaxUops);
}

// The tile kernel's lean variant serves the fixed-slot stride layout without image output.
static bool fixed_layout(const LaunchArgs* a) {
  return a && a->offsets == nullptr && a->lens == nullptr && a->mem_out == nullptr &&
         a->stride >= (uint64_t)kWin && (((uintptr_t)a->frames | (uintptr_t)a->stride) & 15) == 0;
}

bool launch_fixed_layout(const LaunchArgs& a) { return fixed_layout(&a); }

// The compiled fixed-slot kernel keeps tile indices and tile byte offsets in 32-bit scalars.
static bool jit_fixed_layout(const LaunchArgs* a) {
  return fixed_layout(a) && a->n_tiles < (1ull << 31) && a->stride < (1ull << 26);
}

static const void* kernel_for(int kind, uint32_t n_uops, const LaunchArgs* a = nullptr) {
  if (kind == kKindDag) {
    if (tile_kernel_for(kind, n_uops))
      return fixed_layout(a) ? (const void*)tile_kernel<true, false>
                             : (const void*)tile_kernel<false, false>;
    return n_uops > 64 ? (const void*)dag_kernel<4> : (const void*)dag_kernel<1>;
  }
  if (kind == kKindLoop) return (const void*)tile_kernel<false, true>;
  if (kind == kKindTier1) return variant<1>(n_uops);
  return variant<0>(n_uops);
}

int interp_grid(int kind, uint32_t n_uops, bool tiny, uint64_t n_tiles, int* grid_out) {
  int dev = 0, cus = 256, per_cu = 1;
  if (hipGetDevice(&dev) != hipSuccess) return -1;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return -1;
  const uint32_t lds = lds_bytes_for(kind, n_uops);
  const void* k = kernel_for(kind, n_uops);
  {
    static std::mutex mu;
    static std::map<std::tuple<int, const void*, uint32_t>, int> cache;
    std::lock_guard<std::mutex> lk(mu);
    auto key = std::make_tuple(dev, k, lds);
    auto it = cache.find(key);
    if (it != cache.end()) {
      per_cu = it->second;
    } else {
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, kBlock, lds) != hipSuccess ||
          per_cu < 1)
        per_cu = 1;
      cache[key] = per_cu;
    }
  }
  if (kind == kKindTier1 && per_cu > 4) per_cu = 4;  // bounds the tier-1 image scratch
  const uint64_t resident = (uint64_t)cus * (uint64_t)per_cu * kWavesPerBlock;
  const uint64_t tiles = n_tiles ? n_tiles : 1;
  uint64_t waves;
  // tile_kernel: balanced persistent waves (few workgroups: cheap in-kernel counter fold)
  const int policy = kind == kKindLoop ? 2  // divergent tiles: one per wave
                     : kind == kKindTier1 || tile_kernel_for(kind, n_uops) ? 0
                     : tiny ? 1 : 2;
  if (policy == 1) {
    waves = tiles < resident ? tiles : resident;  // every resident slot, grid-stride
  } else if (policy == 2 && kind != kKindTier1) {
    waves = tiles;  // one tile per wave, hardware dispatch
  } else {
    // Persistent waves, each owning the same number of tiles (+-1): k = ceil(tiles / resident
    // waves), then just enough waves for k tiles each.
    const uint64_t per_wave = (tiles + resident - 1) / resident;
    waves = (tiles + per_wave - 1) / per_wave;
  }
  *grid_out = (int)((waves + kWavesPerBlock - 1) / kWavesPerBlock);
  return 0;
}

// Balanced persistent grid of a compiled kernel (its own occupancy: the DB kernel holds two
// window buffers per wave).
// handout: the fixed-slot kernels, whose waves take tiles within their workgroup (one workgroup
// per resident slot, capped by the tiles)
static int jit_grid(hipFunction_t f, uint32_t lds, uint64_t n_tiles, int block = kBlock,
                    bool handout = false, int max_per_cu = 0) {
  const uint64_t wpb = (uint64_t)block / kWave;
  static std::mutex mu;
  static std::map<std::tuple<int, hipFunction_t, uint32_t>, std::pair<int, int>> cache;
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::pair<int, int> occ;  // (CUs, workgroups per CU)
  {
    std::lock_guard<std::mutex> lk(mu);
    auto key = std::make_tuple(dev, f, lds);
    auto it = cache.find(key);
    if (it != cache.end()) {
      occ = it->second;
    } else {
      int cus = 256, per_cu = 1;
      (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
      if (hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, f, block, lds) !=
              hipSuccess ||
          per_cu < 1)
        per_cu = 1;
      // (the occupancy API over-reports by a workgroup for SGPR-heavy kernels, MI355X guide
      // 'Residency': the caller's hardware bound)
      if (max_per_cu > 0 && per_cu > max_per_cu) per_cu = max_per_cu;
      occ = cache[key] = {cus, per_cu};
    }
  }
  const uint64_t tiles = n_tiles ? n_tiles : 1;
  const uint64_t wgs = (uint64_t)occ.first * occ.second;
  if (handout) {  // tiles handed out within the workgroup: >= 1 tile each
    // (tests: EBPFEMU_FIXED_WGS caps the workgroups, so a moderate batch gives each wave more
    // than the 511 tiles one entry of the tile-loop statement runs)
    const char* cap = getenv("EBPFEMU_FIXED_WGS");
    const uint64_t lim = cap && atoi(cap) > 0 ? (uint64_t)atoi(cap) : wgs;
    const uint64_t g = wgs < lim ? wgs : lim;
    return (int)(tiles < g ? tiles : g);
  }
  const uint64_t resident = wgs * wpb;
  const uint64_t per_wave = (tiles + resident - 1) / resident;
  const uint64_t waves = (tiles + per_wave - 1) / per_wave;
  return (int)((waves + wpb - 1) / wpb);
}

// The compiled forward-only program runs where tile_kernel would, and instead of dag_kernel for
// programs of 63..kJitMaxUops micro-ops.
static bool jit_forward_for(int kind, uint32_t n_uops) {
  return kind == kKindDag && (n_uops > kTileMaxUops || tile_kernel_for(kind, n_uops));
}

// The var tile loop (ebpf_tile_jit_varl) takes a compiled forward program's var-kernel batches:
// offsets (4-byte aligned) or 16-byte aligned slots of >= 64 bytes, lengths 4-byte aligned or
// absent, no final images, tile indices in 31 bits (store-mode programs with their deopt list
// included).
static bool varl_ok(int kind, const LaunchArgs& a, const JitFns* jit, bool stack) {
  const bool layout = a.offsets ? ((uintptr_t)a.offsets & 3) == 0
                                : a.stride >= (uint64_t)kWin && a.stride < (1ull << 26) &&
                                      (((uintptr_t)a.frames | (uintptr_t)a.stride) & 15) == 0;
  // (the fixed-slot layout's programs keep ebpf_tile_jit_fixed; store-mode programs, which run
  // on the var kernels only, are stack-window programs)
  return jit && jit->varl && kind == kKindDag && jit_forward_for(kind, a.n_uops) &&
         layout && ((uintptr_t)a.lens & 3) == 0 && !a.mem_out && !a.perm &&
         a.n_tiles < (1ull << 31) && (!jit_fixed_layout(&a) || jit->var_only) &&
         (!jit->var_only || stack);
}

// The fixed-slot kernel's occupancy variant takes a compiled issue-bound program's fixed-slot
// batches (jit_compile's *occ; not stack-window programs, not xdp_md in place: its code has no
// preloaded window to shift the ctx into).
static bool fixed_occ_ok(int kind, const LaunchArgs& a, const JitFns* jit, bool stack) {
  return jit && jit->fixed_occ && !stack && !jit->var_only && !a.xdp && kind == kKindDag &&
         jit_forward_for(kind, a.n_uops) && jit_fixed_layout(&a);
}

int launch_kernel_id(int kind, const LaunchArgs& a, const JitFns* jit, bool stack) {
  if (jit && jit->loop && kind == kKindLoop)
    return stack ? EBPF_KERNEL_JIT_LOOP_STACK : EBPF_KERNEL_JIT_LOOP;
  if (varl_ok(kind, a, jit, stack))
    return stack ? EBPF_KERNEL_JIT_VARL_STACK : EBPF_KERNEL_JIT_VARL;
  if (fixed_occ_ok(kind, a, jit, stack)) return EBPF_KERNEL_JIT_FIXED_OCC;
  if (jit && jit->fixed && jit_forward_for(kind, a.n_uops))
    return jit_fixed_layout(&a) && !jit->var_only
               ? (stack ? EBPF_KERNEL_JIT_STACK : EBPF_KERNEL_JIT_FIXED)
                                : (stack ? EBPF_KERNEL_JIT_VAR_STACK : EBPF_KERNEL_JIT_VAR);
  if (kind == kKindDag)
    return tile_kernel_for(kind, a.n_uops) ? EBPF_KERNEL_TILE : EBPF_KERNEL_DAG;
  if (kind == kKindLoop) return EBPF_KERNEL_TILE_LOOP;
  return kind == kKindTier1 ? EBPF_KERNEL_GENERAL_T1 : EBPF_KERNEL_GENERAL_T0;
}

hipError_t launch_interp(int kind, const LaunchArgs& a, int grid, hipStream_t stream,
                         const JitFns* jit, bool stack) {
  const uint32_t lds = lds_bytes_for(kind, a.n_uops, jit && jit->loop);
  // the compiled var kernels: balanced persistent waves at their own occupancy (interp_grid sizes
  // for tile_kernel's, which is higher: its extra workgroups would run in a second round)
  const bool var = jit && jit->fixed && kind != kKindLoop && jit_forward_for(kind, a.n_uops) &&
                   (!jit_fixed_layout(&a) || jit->var_only);
  const uint32_t vlds = kWavesPerBlock * kVarWaveLds;
  if (var) grid = jit_grid(stack ? jit->var_stack : jit->var, vlds, a.n_tiles);
  const bool vl = varl_ok(kind, a, jit, stack);
  const uint32_t llds = kWavesPerBlock * kVarlWaveLds;
  if (vl) {
    grid = jit_grid(stack ? jit->varl_stack : jit->varl, llds, a.n_tiles);
    // (tests: EBPFEMU_VARL_WGS caps the workgroups, so a moderate batch gives each wave more than
    // the 511 tiles of one statement entry)
    const char* cap = getenv("EBPFEMU_VARL_WGS");
    if (cap && atoi(cap) > 0 && atoi(cap) < grid) grid = atoi(cap);
  }
  LaunchArgs b = a;
  // a shard word's sum must stay below 2^48: bound it by packets x steps per packet; and its
  // arrival count (16 bits) must reach the shard's workgroups - 1: at most 65535 members (the
  // compiled fixed-slot kernel's grid is one workgroup per CU, every other grid is `grid`)
  const uint64_t steps = kind == kKindDag ? (uint64_t)a.n_uops : a.max_steps;
  const uint64_t members = ((uint64_t)grid + kCounterShards - 1) / kCounterShards;
  const bool fits = a.n < (1ull << 40) && steps < (1ull << 47) / (a.n + 1) &&
                    members < (1ull << (64 - kShardCountShift));
  const bool fold_kernel = g_fold_kernel || !fits;
  b.fold_kernel = fold_kernel ? 1u : 0u;
  void* bargs[] = {(void*)&b};
  hipError_t e;
  if (jit && jit->loop && kind == kKindLoop) {  // the compiled loop program
    e = hipModuleLaunchKernel(stack ? jit->loop_stack : jit->loop, grid, 1, 1, kBlock, 1, 1, lds,
                              stream, bargs, nullptr);
  } else if (vl) {  // offsets + lens batches: the var tile loop
    e = hipModuleLaunchKernel(stack ? jit->varl_stack : jit->varl, grid, 1, 1, kBlock, 1, 1, llds,
                              stream, bargs, nullptr);
  } else if (fixed_occ_ok(kind, a, jit, stack)) {  // one window buffer, 6 waves per SIMD
    const bool wide = a.n_uops >= kOccWideUops;  // (jit.cpp compiled the code into that one)
    hipFunction_t f = wide ? jit->fixed_occw : jit->fixed_occ;
    const uint32_t ob = wide ? kOccWideBlock : kOccBlock;
    const uint32_t olds = (wide ? kOccWideWaves : kOccWaves) * kWinBytes;
    e = hipModuleLaunchKernel(f, jit_grid(f, olds, a.n_tiles, ob, true,
                                          wide ? kOccWideWgsPerCu : kOccWgsPerCu), 1, 1,
                              ob, 1, 1, olds, stream, bargs, nullptr);
  } else if (jit && jit->fixed && jit_forward_for(kind, a.n_uops)) {
    if (jit_fixed_layout(&a) && !jit->var_only) {  // double-buffered windows: its own LDS size and grid
      const uint32_t dlds = kDbWaves * kTileWaveLdsDb;
      e = hipModuleLaunchKernel(jit->fixed, jit_grid(jit->fixed, dlds, a.n_tiles, kDbBlock, true),
                                1, 1, kDbBlock, 1, 1, dlds, stream, bargs, nullptr);
    } else {  // (the tile kernel's window LDS + a second metadata buffer, also for programs
              // past kTileMaxUops)
      e = hipModuleLaunchKernel(stack ? jit->var_stack : jit->var, grid, 1, 1, kBlock, 1, 1, vlds,
                                stream, bargs, nullptr);
    }
  } else
    e = hipLaunchKernel(kernel_for(kind, a.n_uops, &a), dim3(grid), dim3(kBlock), bargs, lds,
                        stream);
  if (e != hipSuccess || a.counters == nullptr || !fold_kernel) return e;
  uint64_t* shards = a.shards;
  uint64_t* counters = a.counters;
  void* fargs[] = {(void*)&shards, (void*)&counters};
  return hipLaunchKernel((const void*)fold_counters, dim3(1), dim3(kCounterShards * 8), fargs, 0,
                         stream);
}

#endif  // EBPFEMU_JIT_TEMPLATE

}  // namespace ebpfemu
