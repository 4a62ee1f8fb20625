// jit.h — the eBPF -> gfx950 compiler of the tile fast path (jit.cpp).
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "uop.h"

namespace ebpfemu {

// The compiled kernels of one program on one device: the fixed-slot stride layout and every
// other layout (the two template kernels of build/tile_jit.s, ebpf_tile_jit_fixed / _var).
struct JitFns {
  hipFunction_t fixed = nullptr;
  hipFunction_t var = nullptr;
};

// Compiles a forward-only program of <= kTileMaxUops micro-ops (its tile table `t`, built by
// build_tile) into the assembly of the two template kernels, then assembles and links it
// (amd_comgr) into a gfx950 code object. Returns false with a reason in *err on failure.
bool jit_compile(const std::vector<Uop>& uops, const std::vector<TUop>& t,
                 std::vector<char>& code_object, std::string* err, std::string* asm_out = nullptr);

// Loads a code object on the current device.
bool jit_load(const std::vector<char>& code_object, hipModule_t* mod, JitFns* fns);

}  // namespace ebpfemu
