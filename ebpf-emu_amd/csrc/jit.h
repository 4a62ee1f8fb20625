// jit.h — the eBPF -> gfx950 compiler of the tile fast path (jit.cpp).
#pragma once
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>
#include <string>
#include <vector>

#include "uop.h"

namespace ebpfemu {

// The compiled kernels of one program on one device: the fixed-slot stride layout and every
// other layout (the two template kernels of build/tile_jit.s, ebpf_tile_jit_fixed / _var).
struct JitFns {
  hipFunction_t fixed = nullptr;
  hipFunction_t var = nullptr;
  hipFunction_t loop = nullptr;  // loop programs (ebpf_tile_jit_loop)
  hipFunction_t var_stack = nullptr;  // stack-window programs, other layouts (ebpf_tile_jit_var_stack)
  hipFunction_t loop_stack = nullptr;  // stack-window loop programs (ebpf_tile_jit_loop_stack)
  hipFunction_t loop_deep = nullptr;  // loop programs with the deep refill prefetch
  hipFunction_t varl = nullptr;  // offsets + lens batches: the var tile loop (ebpf_tile_jit_varl)
  hipFunction_t varl_stack = nullptr;  // ... for stack-window programs (ebpf_tile_jit_varl_stack)
  // the fixed-slot layout's occupancy variant (ebpf_tile_jit_fixed_occ: issue-bound programs, one
  // window buffer per wave); null unless this program's code went there (jit_compile *occ)
  hipFunction_t fixed_occ = nullptr;
  hipFunction_t fixed_occw = nullptr;  // its wide form (launch.h kOccWideUops)
  // the program's code exists for the var kernels only (store mode: register-address stores into
  // the packet, StackPlan::any_dyn), whatever the batch layout
  bool var_only = false;
};

// Stack-window programs (memory tier 0.5, host.cpp analyze_stack): every store or atomic writes
// the window [r10 - k, r10) at an offset known at load time, so the window lives in VGPRs of the
// compiled fixed-slot kernel (v[kStackVgpr : kStackVgpr + k/4]); stores may also write the
// packet's header window at constant addresses (the preloaded window dwords v[64 : 79]).
// compiled variants of a program: 0 init_regs batches, 1 the main.rs layout (constant-address
// loads resolved), 2 the loop kernel, 3 xdp_md batches (the ctx's data field known, host.cpp
// fold_const_loads), 4 the stack-slot promoted loop program (host.cpp promote_slots), 5 the loop
// program for xdp_md batches (staged images: the ctx's data and data_end known to the range
// analysis, jit.cpp Compiler::xdp_ctx), 6 the same program for xdp_md batches in place (rebased:
// the packet loads 8 bytes lower, the batch run as the main.rs layout over the packets,
// Compiler::xdp_rebase)
constexpr int kJitVariants = 7;
// Store mode (the var tile loop): the overflow image holds image bytes [64, min(mem_size rounded
// up to 64, kOvfEnd)) per packet, in 64-byte blocks filled on first use (jit.cpp ovf_fill); a
// store ending past it (or past the stack window's start) deoptimizes.
constexpr uint32_t kOvfEnd = 2048;
// bytes of the overflow image per packet for a batch's mem_size (host.cpp workspace)
inline uint64_t ovf_stride(uint32_t mem_size) {
  uint64_t e = ((uint64_t)mem_size + 63) & ~63ull;
  e = e < kOvfEnd ? e : kOvfEnd;
  return e > 64 ? e - 64 : 0;
}
constexpr uint32_t kStackMax = 64;    // window bytes
constexpr uint32_t kStackVgpr = 80;   // first VGPR of the window (ebpf_tile_jit_fixed)
constexpr int32_t kNoStack = INT32_MIN;
struct StackPlan {
  uint32_t k = 0;            // window bytes (multiple of 4, <= kStackMax); 0 = no plan
  std::vector<int32_t> off;  // per micro-op: ST/STX, ATOMIC (8 bytes, 4-aligned) and LDX inside
                             // the window: the access's offset from r10 (-k <= off,
                             // off + width <= 0); else kNoStack
  std::vector<int32_t> pw;   // per micro-op: ST/STX into the packet's header window at a constant
                             // image address [0, kWin - width] (r1 = 0, main.rs:28); else kNoStack
  bool any_pw = false;
  // store mode: ST/STX through a register whose value is not known at load time (a packet
  // pointer: a TTL / port / checksum rewrite behind a variable-length header). The packet's header
  // window then lives in LDS only (every packet load and store goes through it, bytes at or past
  // LEN zeroed); a lane whose store leaves the window [0, 64) -- or whose load straddles its end
  // -- deoptimizes: its packet is re-run from the start by the general interpreter (tier 1) after
  // the compiled launch (host.cpp, the deopt list). Forward programs on the var kernels only.
  std::vector<char> dyn;     // per micro-op: a register-address ST/STX
  bool any_dyn = false;
  bool no_deopt = false;     // store_mode_no_deopt: no lane of a main.rs-layout batch can leave
  // per micro-op: an LDX the proof took as constant-address (its range analysis found one value).
  // Codegen checks that every load it compiles as a constant-address far load (whose dirty lanes
  // deoptimize) is one of these, so the proof and the code cannot disagree silently.
  std::vector<char> kld;
  uint64_t st_bound = 128;   // (no_deopt) every register-address store ends at or below this
  bool len_bound = false;    // (no_deopt) ... or inside the packet (LEN <= mem_size)
};

// Store mode on the var tile loop: whether no lane of a main.rs-layout batch can deoptimize
// (jit.cpp, a range analysis of every access; the host also needs the stack window at or past
// byte 128). Then the deopt pass after the launch is not needed.
// *st_bound: every register-address store ends at or below it (>= 128); the host runs a batch
// without the pass when its stack window starts at or past it. *len_bound: some access is bounded
// by the packet's length instead (then also mem_size <= kOvfEnd and the stack window past it).
bool store_mode_no_deopt(const std::vector<Uop>& uops, const StackPlan& stk, uint32_t* why = nullptr,
                         std::vector<char>* kld = nullptr, uint64_t* st_bound = nullptr,
                         bool* len_bound = nullptr);

// Status of a lane that leaves the compiled kernel for the general interpreter (never reported:
// the tile epilogue lists the packet instead of writing its outputs, tile bucket 8).
constexpr uint32_t kStDeopt = 0x80;

// Compiles a forward-only program of <= kTileMaxUops micro-ops (its tile table `t`, built by
// build_tile) into the assembly of the two template kernels, then assembles and links it
// (amd_comgr) into a gfx950 code object. Returns false with a reason in *err on failure.
// stk: a stack-window program (only the fixed-slot kernel and the var kernel's stack variant
// get its code).
// *occ (if given): the code also went into ebpf_tile_jit_fixed_occ (an issue-bound program whose
// code fits that statement's registers).
// main_layout: the table of the main.rs register layout (variant 1): its compare narrowing may use
// the load-time value ranges.
bool jit_compile(const std::vector<Uop>& uops, const std::vector<TUop>& t,
                 std::vector<char>& code_object, std::string* err, std::string* asm_out = nullptr,
                 const StackPlan* stk = nullptr, bool* occ = nullptr, bool main_layout = false);

// Loop programs (back edges, or budgets that can bind; tile tables of build_tile: `t` the block
// table, `tx` the exact one-micro-op-per-block table) for ebpf_tile_jit_loop. *deep (if given):
// the code went into ebpf_tile_jit_loop_deep instead (a loop with a cooperative byte sum).
// guard_k > 0 (a stack-slot promoted program, host.cpp promote_slots): every packet load must be
// a one-byte load proven inside the packet (prove_loads; else the compile fails), and lanes whose
// packet reaches the window (LEN > r10 - guard_k) deoptimize at the start (jit.h kStDeopt).
bool jit_compile_loop(const std::vector<Uop>& uops, const std::vector<TUop>& t,
                      const std::vector<TUop>& tx, std::vector<char>& code_object,
                      std::string* err, std::string* asm_out = nullptr,
                      const StackPlan* stk = nullptr, bool* deep = nullptr, uint32_t guard_k = 0,
                      bool xdp_ctx = false, bool xdp_rebase = false);

// Windows the refills of byte-scanning loop programs prefetch ahead: 1 (ebpf_tile_jit_loop, 5
// waves per SIMD) or 2-3 (ebpf_tile_jit_loop_deep, 4 waves); EBPFEMU_PF_DEPTH overrides.

// Loads a code object on the current device (the functions it does not hold stay null).
bool jit_load(const std::vector<char>& code_object, hipModule_t* mod, JitFns* fns);

}  // namespace ebpfemu
