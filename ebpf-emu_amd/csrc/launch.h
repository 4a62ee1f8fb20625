// launch.h — host <-> device-launcher interface inside libebpfemu.so (not part of the C ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "uop.h"

namespace ebpfemu {

constexpr int kWave = 64;
constexpr int kBlock = 256;           // 4 waves per workgroup
constexpr int kWavesPerBlock = kBlock / kWave;
constexpr int kWin = 64;              // packet bytes staged in LDS per lane (header window)
constexpr int kWinStride = kWin + 4;  // padded per-lane LDS stride: 17 dwords, conflict-free b32
constexpr int kMaxLdsUops = 4096;     // programs up to this many micro-ops are staged in LDS
constexpr int kCallDepth = 64;        // EBPF_MAX_CALL_DEPTH
constexpr int kCounterShards = 64;    // device-atomic counter shards (spread contention)
// workspace layout: [ticket u32 | pad to 256][shards u64[64][8]][tier-1 wave slots]
constexpr uint64_t kWsShardsOff = 256;
constexpr uint64_t kWsSlotsOff = 256 + kCounterShards * 8 * 8;

struct LaunchArgs {
  const Uop* prog;      // device micro-ops
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
  uint32_t* ticket;     // workspace: workgroups finished (reset by the last one)
  uint64_t* shards;     // workspace: [kCounterShards][8] partial counters (left zeroed)
  uint8_t* image_ws;    // tier 1: per-wave-slot images + call stacks
  uint64_t n_tiles;     // ceil(n / 64)
  const uint64_t* init_regs;  // optional [11] initial registers (else main.rs layout)
  uint8_t* mem_out;           // optional [n][mem_size] final images
  uint64_t* regs_out;         // optional [n][11] final registers
};

// Bytes of tier-1 scratch per wave slot: lane-interleaved image dwords + call stack.
__host__ __device__ inline uint64_t tier1_slot_bytes(uint32_t mem_size) {
  return (uint64_t)(mem_size / 4 + kCallDepth) * kWave * 4;
}

// Persistent grid size for a tier / LDS footprint on the current device.
int interp_grid(int tier, uint32_t n_uops, uint64_t n_tiles, int* grid_out);

// Enqueue the interpreter (one kernel; counters folded in by its last workgroup).
hipError_t launch_interp(int tier, const LaunchArgs& a, int grid, hipStream_t stream);

}  // namespace ebpfemu
