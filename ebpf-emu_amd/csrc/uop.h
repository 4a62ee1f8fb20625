// uop.h — device micro-op format produced by the host pre-decoder (decode.cpp) and
// interpreted by the gfx950 kernel (interp.hip).
//
// One 16-byte micro-op per DECODED reference instruction (a wide lddw is one entry, as
// ins.rs:107-116 folds it), so jump targets keep the reference's decoded-entry indexing
// (quirk Q9). Everything that can be resolved at load time is: operand source, ALU width,
// the sign-extended immediate, absolute jump targets, static runtime faults (reg 11, END imm,
// callx, illegal mode/class combinations). The kernel therefore never indexes register 11.
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace ebpfemu {

struct alignas(16) Uop {
  uint8_t op;   // UopKind
  uint8_t dst;  // 0..10
  uint8_t src;  // 0..10
  uint8_t aux;  // kind-specific: F_SRC, access width, atomic flags, fault status
  int32_t x;    // jump/call target (u32 bits) or memory offset (sign-extended i16)
  int64_t k;    // immediate: sign-extended imm (ALU/JMP), imm64 (LDIMM), zext imm (ST), atomic op
};
static_assert(sizeof(Uop) == 16, "Uop must be 16 bytes");

enum UopAux : uint8_t {
  F_SRC = 1,        // ALU/JMP: operand is regs[src] (code bit 3), else k
  F_ATOMIC32 = 2,   // ATOMIC: 32-bit form (size bits == 0, emu.rs:382)
  F_FETCH = 4,      // ATOMIC: imm & 1 (emu.rs:376)
};

enum UopKind : uint8_t {
  // ALU64 (emu.rs:80-209, class ALU64): dst = f(dst, b)
  U_ADD64 = 0, U_SUB64, U_MUL64, U_DIV64, U_OR64, U_AND64, U_LSH64, U_RSH64, U_NEG64, U_MOD64,
  U_XOR64, U_MOV64, U_ARSH64,
  // ALU32 (class ALU, operands truncated to u32 before and after, emu.rs:76-79,214-216)
  U_ADD32, U_SUB32, U_MUL32, U_DIV32, U_OR32, U_AND32, U_LSH32, U_RSH32, U_NEG32, U_MOD32,
  U_XOR32, U_MOV32, U_ARSH32,
  // END (emu.rs:165-209), either ALU class (Q7)
  U_ZX16, U_ZX32, U_NOP, U_BSWAP16, U_BSWAP32, U_BSWAP64,
  // JMP: all orderings signed (Q2); 32-bit forms compare sign-extended low words (Q3)
  U_JA, U_JEQ, U_JGT, U_JGE, U_JSET, U_JNE, U_JLT, U_JLE,
  U_JEQ32, U_JGT32, U_JGE32, U_JSET32, U_JNE32, U_JLT32, U_JLE32,
  U_CALL,   // pc = x; push x + 1 (emu.rs:265-272)
  U_EXIT,   // pop or stop (emu.rs:273-279)
  // load/store
  U_LDIMM,  // dst = k (emu.rs:332-334)
  U_LDX,    // low aux bytes of dst <- mem[src + x] (Q1, emu.rs:341-349)
  U_ST,     // mem[dst + x] <- low aux bytes of k (Q8)
  U_STX,    // mem[dst + x] <- low aux bytes of src
  U_ATOMIC, // 8-byte RMW at dst + x; k = imm & 0xfe (or 0xff = unknown -> fault after the read)
  U_FAULT,  // aux = EBPF_ST_* raised when executed
  U_NKINDS,
  // dag_kernel only: LDX whose base register holds the same known constant on every path
  // (load-time dataflow, default register layout); DUop::addr = that constant + offset
  U_LDXK = U_NKINDS
};

constexpr uint32_t PC_DONE = 0xFFFFFFFFu;

// Per-lane register file of the DAG kernel in LDS: regs[r] of lane l at r * kRegStride + l * 8.
constexpr uint32_t kRegStride = 64 * 8;

// Micro-op of the DAG kernel (tier-0 programs whose jumps all go forward, dag_kernel in
// interp.hip): a Uop with everything the kernel would otherwise compute per step resolved at
// load time, fetched by scalar loads straight into SGPRs. Two halves: dwords 0..23 hold the
// hand-written handlers' view (dag_asm.h ids, from which build_tile makes the tile kernel's TUop)
// and dwords 32..47 dag_kernel's C++ step.
struct alignas(256) DUop {
  // ---- the hand-written loop ----
  uint32_t hoff;    // d0: handler slot offset (dag_asm.h id * DAG_SLOT)
  uint32_t dst2;    // d1: 2 * dst (register pair index in the loop's VGPR register file)
  uint32_t src2;    // d2: 2 * src
  uint32_t anpc;    // d3: pc + 1, or PC_DONE (canonical jumps: the not-taken successor)
  uint32_t ax;      // d4: jump target, or PC_DONE past the end
  uint32_t a0;      // d5: H_LDXK: the image address
  uint64_t kmask;   // d6-7: H_LDX/H_LDXK: mask of the access width's low bytes
  uint64_t anbit;   // d8-9: 1 << anpc (0 for PC_DONE)
  uint64_t atbit;   // d10-11: 1 << ax
  uint64_t imm;     // d12-13: the immediate as the handler consumes it (negated for SUB, masked
                    //         shift count); H_LDX: the sign-extended offset
  uint32_t width;   // d14: H_LDX/H_LDXK access width
  uint32_t end;     // d15: H_LDXK: a0 + width (scalar bounds check)
  uint32_t win[6];  // d16-21: H_LDXK window dwords i = 0..2 of the access: {chunk bits (b & 0x30),
                    //         byte-in-chunk (b & 15)} of dword address b, for the lane swizzle
  uint32_t apad[10];
  // ---- the C++ step (d32..47) ----
  uint32_t opaux;   // UopKind | aux << 8
  uint32_t doff;    // dst * kRegStride (LDS register file)
  uint32_t soff;    // src * kRegStride
  uint32_t npc;     // pc + 1, or PC_DONE when that falls off the end (a normal stop)
  uint32_t x;       // jump target (PC_DONE past the end) or LDX offset (sign-extended i16)
  uint32_t cpad;
  uint64_t k;       // immediate (ALU/JMP/LDIMM); LDX/LDXK: mask of the access width
  uint64_t nbit;    // 1 << npc in the pc set of programs of <= 64 micro-ops (0 for PC_DONE)
  uint64_t tbit;    // 1 << x likewise, for jumps
  uint64_t addr;    // U_LDXK: the absolute image address
  uint32_t cpad2[16];
};
static_assert(sizeof(DUop) == 256, "DUop must be 256 bytes");

// Micro-op of the tile interpreter (tile_kernel in interp.hip, tile.inc generated by gen_tile.py):
// one s_load_dwordx16 per dispatch, dword i in s[64 + i]. Built from the DUop of the same pc
// (build_tile in host.cpp); entries 62 and 63 of every table are DONE sentinels.
struct alignas(64) TUop {
  uint32_t hoff;   // d0: handler slot offset (tile_ids.h id * TILE_SLOT): chained or block-end form
  uint32_t dst2;   // d1: 2 * dst
  uint32_t src2;   // d2: 2 * src; LDXK: byte offset of window dword 0 (a0 & ~3)
  uint32_t npc;    // d3: pc + 1, or PC_DONE (canonical jumps: the not-taken successor)
  uint32_t x;      // d4: jump target, or PC_DONE past the end; LDXK: a0 + width
  uint32_t a0;     // d5: LDXK: the image address; LDX / ARSH64: steps not retired on a fault
  uint64_t kmask;  // d6-7: LDX/LDXK: mask of the access width's low bytes
  uint64_t nbit;   // d8-9: 1 << npc (0 for PC_DONE)
  uint64_t tbit;   // d10-11: 1 << x; LDXK: byte offsets of window dwords 1, 2
  uint64_t imm;    // d12-13: the immediate as the handler consumes it; LDX: the offset;
                   //         one-dword LDXK: the bit shift (a0 % 4) * 8
  uint32_t width;  // d14: LDX access width; LDXK: steps not retired on a fault
  uint32_t blen;   // d15: block start: length of its basic block (steps retired at dispatch)
};
static_assert(sizeof(TUop) == 64, "TUop must be 64 bytes");
constexpr uint32_t kTileUops = 64;     // table entries: micro-ops, then the DONE sentinels 62, 63
constexpr uint32_t kTileMaxUops = 62;  // programs the tile kernels run
// programs the compiler takes (jit.cpp; flatten_calls' copies likewise). Past kMaxDagUops
// (launch.h, dag_kernel's LDS table) a forward program runs compiled or on the general interpreter.
constexpr uint32_t kJitMaxUops = 4096;
static_assert(offsetof(DUop, opaux) == 128, "the C++ half starts at dword 32");

}  // namespace ebpfemu
