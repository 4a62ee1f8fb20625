// launch.h — host <-> device-launcher interface inside libebpfemu.so (not part of the C ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "jit.h"
#include "uop.h"

namespace ebpfemu {

constexpr int kWave = 64;
constexpr int kBlock = 256;           // 4 waves per workgroup
constexpr int kWavesPerBlock = kBlock / kWave;
// the compiled fixed-slot kernel: one workgroup of 16 waves per CU, its tiles handed out to
// the waves by an LDS counter (interp.hip tile_body)
constexpr int kDbWaves = 16;
constexpr int kDbBlock = kDbWaves * kWave;
// ebpf_tile_jit_fixed_occ (issue-bound programs): one window buffer per wave, 3 workgroups of 8
// waves per CU (6 waves per SIMD, the limit of its ~103 SGPRs)
constexpr int kOccWaves = 8;
constexpr int kOccBlock = kOccWaves * kWave;
constexpr int kOccWgsPerCu = 3;
// its wide form (ebpf_tile_jit_fixed_occw): 2 workgroups of 12 waves per CU -- the same 6 waves per
// SIMD in fewer, larger workgroups -- for programs of at least kOccWideUops micro-ops (the rule
// chains: 53 -> 57 Gpkt/s at two streams for acl_rules, while the 5-tuple's line drops 106 -> 101
// on it: DESIGN 3.35). jit.cpp gives each program's code to the one of the two its length picks.
constexpr int kOccWideWaves = 12;
constexpr int kOccWideBlock = kOccWideWaves * kWave;
constexpr int kOccWideWgsPerCu = 2;
constexpr uint32_t kOccWideUops = 256;
constexpr int kWin = 64;              // packet bytes staged in LDS per lane (header window)
constexpr int kWinStride = kWin + 4;  // padded per-lane LDS stride: 17 dwords, conflict-free b32
constexpr int kMaxLdsUops = 4096;     // programs up to this many micro-ops are staged in LDS
constexpr int kCallDepth = 64;        // EBPF_MAX_CALL_DEPTH
constexpr int kCounterShards = 64;    // device-atomic counter shards (spread contention)
// workspace layout: [deopt count, done u32[2] @0 | (unused) | multi-GPU counter sums u64[8] @256 | xdp_md cursor u64 @320 |
// length-bin counts u32[16] @384 | bin cursors u32[16] @448, 512 B][shards u64[64][8]][tier-1
// wave slots, or the length-binned packet order u32[n]]; bin counts/cursors and shards are zero
// between batches
constexpr uint64_t kWsBinCountsOff = 384;
constexpr uint64_t kWsBinCursorOff = 448;
constexpr int kBinClasses = 16;  // packets are binned by ceil(len / 128), capped
constexpr int kBinMaxWgs = 1024;  // binning grid cap; per-workgroup class counts follow the order
constexpr uint64_t kWsDeoptOff = 0;  // u32 count, done: the deopt list (LaunchArgs::deopt); u32
                                     // at +8: how many packets the last deopt pass re-ran
constexpr uint64_t kWsXdpCursorOff = 320;  // u64: bytes staged by xdp_stage (reset per batch)
constexpr uint64_t kWsMultiOff = 256;  // u64[8]: ebpf_run_batch_multi's per-shard counter sums
constexpr uint64_t kWsShardsOff = 512;
constexpr uint64_t kWsSlotsOff = kWsShardsOff + kCounterShards * 8 * 8;

// Kernel kinds: the two memory tiers of interp_kernel, and dag_kernel (tier-0 programs whose
// jumps all go forward, run with max_steps >= n_uops so no step budget can bind).
enum KernelKind : int { kKindTier0 = 0, kKindTier1 = 1, kKindDag = 2, kKindLoop = 3 };
constexpr uint32_t kMaxDagUops = 256;

struct LaunchArgs {
  const Uop* prog;      // device micro-ops
  const DUop* dprog;    // device DAG micro-ops (kKindDag)
  const TUop* tprog;    // device tile micro-ops (kKindDag / kKindLoop, <= 62 micro-ops), else null
  const TUop* tprog_exact;  // kKindLoop: the one-micro-op-per-block table (exact step budget)
  uint32_t n_uops;
  uint32_t mem_size;
  const uint8_t* frames;
  const uint32_t* offsets;
  const uint16_t* lens;
  uint64_t stride;
  uint64_t n;
  uint64_t r10;
  uint64_t max_steps;
  uint8_t* verdict;
  uint64_t* r0;
  uint8_t* status;
  uint64_t* counters;   // optional caller counters [8] (added to)
  uint64_t* shards;     // workspace: [kCounterShards][8] partial counters (left zeroed)
  uint8_t* image_ws;    // tier 1: per-wave-slot images + call stacks
  uint64_t n_tiles;     // ceil(n / 64)
  const uint64_t* init_regs;  // optional [11] initial registers (else main.rs layout)
  uint8_t* mem_out;           // optional [n][mem_size] final images
  uint64_t* regs_out;         // optional [n][11] final registers
  uint32_t fold_kernel;       // 1: shards are folded by fold_counters after the launch, 0:
                              //    in-kernel (counted shard words, flush_counters)
  const uint32_t* perm;       // loop mode: packet index of tile slot i (length-binned), else null
  uint32_t* bin_counts;       // with perm: bin counts + cursors, zeroed again by the tile kernel
  uint64_t* trace;            // diagnostics (EBPFEMU_TRACE=1): per-wave s_memrealtime stamps of
                              // the compiled fixed-slot kernel, kTraceSlots per wave; else null
  const uint32_t* init_fp;    // tier-1 kernel: initial frame stack (Emu.fp, emu.rs:26), bottom first
  uint32_t init_fp_len;       //   its depth (<= kCallDepth)
  uint32_t* fp_out;           // tier-1 kernel: optional [n][kCallDepth] final frame stacks
  uint8_t* fp_len_out;        //   optional [n] their depths
  uint32_t xdp;               // 1: the xdp_md convention run in place (xdp.rs:16-20): image =
                              //   [u32 data = 8][u32 data_end = 8 + len][packet]; the window is
                              //   shifted by 8 bytes in LDS and the ctx synthesised per lane, BASE
                              //   = packet - 8 and LEN = 8 + len (no staging copy)
  // store-mode programs (jit.h StackPlan::any_dyn): the deopt list in the workspace -- u32
  // [count, done] at kWsDeoptOff (zero between batches), idx[n] past the tier-1 slots. The
  // compiled kernel appends the packet index of every lane that deoptimized (status kStDeopt: no
  // outputs, not counted); then the general interpreter runs with deopt_pass = 1 over
  // idx[0 .. count) (outputs at those indices), and its last workgroup zeroes count and done.
  // deopt_pass = 2 on a compiled store-mode launch that no pass follows (StackPlan::no_deopt): a
  // lane that still leaves is not listed but gets status EBPF_ST_JIT (the proof failed).
  uint32_t* deopt;
  uint32_t* deopt_idx;
  uint32_t deopt_pass;
  // store mode on the var tile loop: per packet its image's bytes [64, 128) once it stores there
  // (u8[n][64] + 16 in the workspace past deopt_idx; jit.cpp ovf_fill), else null
  uint8_t* ovf;
};

constexpr int kTraceSlots = 16;
constexpr uint64_t kTraceWaves = 1 << 16;
constexpr int kTraceRing = 4;  // launches kept (consecutive launches' gaps)

// Bytes of tier-1 scratch per wave slot: lane-interleaved image dwords + call stack.
__host__ __device__ inline uint64_t tier1_slot_bytes(uint32_t mem_size) {
  return (uint64_t)((mem_size + 3) / 4 + kCallDepth) * kWave * 4;
}

// Programs this short with no back edge do a fixed, tiny amount of work per tile.
constexpr uint32_t kTinyUops = 8;

// Grid size on the current device. Tier 0 and DAG: one tile (64 packets) per wave, so the hardware
// dispatcher balances divergent tiles, except `tiny` programs, which get every resident wave
// slot once (grid-stride) so per-workgroup fixed costs are paid once per slot. Tier 1:
// balanced persistent waves (bounds the per-wave image scratch).
int interp_grid(int kind, uint32_t n_uops, bool tiny, uint64_t n_tiles, int* grid_out);

// Length-binned lane packing for the loop-mode tile kernel (offsets + lens layouts): fills
// perm[n] with the packet indices grouped by ceil(len / 128), so a tile's lanes run loops of
// similar trip counts. Two kernels on `stream` (histogram, scatter); bins start zeroed.
hipError_t launch_binning(const uint16_t* lens, uint64_t n, uint32_t* wgc, uint32_t* perm,
                          hipStream_t stream);

// xdp_md calling convention: stage image i = [xdp_md {8, 8 + len}][packet][...] for every packet
// into dst (16-byte aligned slots, packed in workgroup order); writes the staged offsets and
// lengths (8 + len). Images longer than mem_size are not copied (the batch faults them
// ST_BADPKT from the length alone). cursor: a zeroed u64.
hipError_t launch_xdp_stage(const uint8_t* frames, const uint32_t* offsets, const uint16_t* lens,
                            uint64_t stride, uint64_t n, uint32_t mem_size, uint8_t* dst,
                            uint32_t* doffs, uint16_t* dlens, unsigned long long* cursor,
                            hipStream_t stream);

// Whether a launch runs the fixed-slot kernels (stride layout, 16-byte aligned slots of >= 64
// bytes, no lengths, no image output; EBPFEMU_FIXED=0 disables them).
bool launch_fixed_layout(const LaunchArgs& a);

// The EBPF_KERNEL_* id of the kernel launch_interp runs for (kind, a, jit); stack: a memory
// tier 0.5 batch.
int launch_kernel_id(int kind, const LaunchArgs& a, const JitFns* jit, bool stack);

// dst[0..7] += src[0..7] on `stream` (one tiny kernel).
hipError_t launch_counters_add(const uint64_t* src, uint64_t* dst, hipStream_t stream);

// Enqueue the interpreter on `stream`; with counters, its last workgroup folds the shards into them.
// jit: the program's compiled kernels, launched instead of the tile interpreter where it would run.
hipError_t launch_interp(int kind, const LaunchArgs& a, int grid, hipStream_t stream,
                         const JitFns* jit = nullptr, bool stack = false);

}  // namespace ebpfemu
