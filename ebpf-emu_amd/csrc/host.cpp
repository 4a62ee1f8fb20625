// host.cpp — the C ABI of libebpfemu.so (include/ebpf_emu.h): program load (the reference's
// decoder, ins.rs), the load-time pre-decoder to device micro-ops, batch launch, and the
// multi-GPU counter all-reduce over RCCL.
//
// This file has no interpreter: execution happens only in the gfx950 kernel (interp.hip).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include <map>
#include <mutex>
#include <thread>
#include <set>
#include <string>
#include <vector>

#include "../../include/ebpf_emu.h"
#include "dag_asm.h"
#include "tile_ids.h"
#include "launch.h"
#include "jit.h"
#include "uop.h"

using namespace ebpfemu;

namespace {

// The reference's decoded Instruction (ins.rs:37-45); `code` kept as the raw opcode byte.
struct RefInsn {
  int32_t imm;
  int64_t imm64;
  int16_t off;
  uint8_t src, dst, code;
};

constexpr int kMaxDevices = 64;

uint64_t le64(const uint8_t* p) {
  uint64_t v = 0;
  for (int i = 7; i >= 0; i--) v = (v << 8) | p[i];
  return v;
}

bool is_ls(uint8_t code) { return (code & 7) <= 3; }  // ins.rs:163

// u64s_to_instructions (ins.rs:96-119) over the LE image; Instruction::from (ins.rs:121-132)
// with the panics of Register::from (ins.rs:32), AOp/JOp::from (ins.rs:251,257) and
// Mode::from (ins.rs:187; 0x80/0xa0 are invalid discriminants) turned into error codes.
int decode_image(const uint8_t* code, size_t nbytes, std::vector<RefInsn>& out, size_t* bad) {
  out.clear();
  if (nbytes % 8) {
    if (bad) *bad = nbytes / 8;
    return EBPF_ELEN;
  }
  const size_t nw = nbytes / 8;
  for (size_t i = 0; i < nw; i++) {
    const uint64_t w = le64(code + 8 * i);
    RefInsn ins;
    ins.imm = (int32_t)(uint32_t)(w >> 32);
    ins.imm64 = (int64_t)(w >> 32);
    ins.off = (int16_t)(uint16_t)(w >> 16);
    ins.src = (uint8_t)((w >> 12) & 0xf);
    ins.dst = (uint8_t)((w >> 8) & 0xf);
    ins.code = (uint8_t)w;
    if (bad) *bad = i;
    if (ins.src >= 12 || ins.dst >= 12) return EBPF_EREG;
    const uint8_t cls = ins.code & 7;
    if (cls >= 4) {
      if ((ins.code >> 4) > 0xd) return EBPF_EOP;
    } else {
      const uint8_t mode = ins.code & 0xe0;
      if (mode > 0xc0 || mode == 0x80 || mode == 0xa0) return EBPF_EMODE;
      if (mode == 0x00) {  // wide: fold the next word (ins.rs:107-114)
        if (++i >= nw) return EBPF_ELDDW;
        int64_t sum;
        if (__builtin_add_overflow((int64_t)(uint32_t)ins.imm, (int64_t)le64(code + 8 * i), &sum))
          return EBPF_ELDDW_OVF;
        ins.imm64 = sum;
        ins.imm = 0;
      }
    }
    out.push_back(ins);
  }
  return EBPF_OK;
}

Uop fault_uop(uint8_t status) {
  Uop u{};
  u.op = U_FAULT;
  u.aux = status;
  return u;
}

// Load-time lowering of one decoded instruction at index pc to a device micro-op
// (the static half of emu.rs:48-451).
Uop lower(const RefInsn& in, uint32_t pc) {
  const uint8_t code = in.code, cls = code & 7;
  Uop u{};
  u.dst = in.dst;
  u.src = in.src;
  if (!is_ls(code)) {
    const uint8_t op = code >> 4, source = (code >> 3) & 1;
    // registers read before any op-specific behaviour (emu.rs:66-72,75,220): index 11 panics
    if ((source && in.src >= 11) || in.dst >= 11) return fault_uop(EBPF_ST_INSN);
    u.aux = source ? F_SRC : 0;
    u.k = (int64_t)in.imm;  // `imm as i64`, emu.rs:67
    if (!source) u.src = 0;
    if (cls == 4 || cls == 7) {
      const bool alu32 = cls == 4;
      if (op == 13) {  // END (emu.rs:165-209)
        u.aux = 0;
        u.src = 0;
        if (in.imm == 16) u.op = source ? U_BSWAP16 : U_ZX16;
        else if (in.imm == 32) u.op = source ? U_BSWAP32 : U_ZX32;
        else if (in.imm == 64) u.op = source ? U_BSWAP64 : U_NOP;
        else return fault_uop(EBPF_ST_INSN);  // unreachable! emu.rs:206
        return u;
      }
      u.op = (uint8_t)((alu32 ? U_ADD32 : U_ADD64) + op);
      return u;
    }
    // JMP / JMP32 (emu.rs:218-304)
    const uint32_t target = (pc + 1) + (uint32_t)(int32_t)in.off;  // wrapping_add_signed
    u.x = (int32_t)target;
    const bool j32 = cls == 6;
    switch (op) {
      case 0: u.op = U_JA; u.aux = 0; u.src = 0; return u;  // JA, also in JMP32 (Q26)
      case 1: u.op = j32 ? U_JEQ32 : U_JEQ; return u;
      case 2: case 6: u.op = j32 ? U_JGT32 : U_JGT; return u;   // JGT == JSGT (Q2)
      case 3: case 7: u.op = j32 ? U_JGE32 : U_JGE; return u;
      case 4: u.op = j32 ? U_JSET32 : U_JSET; return u;
      case 5: u.op = j32 ? U_JNE32 : U_JNE; return u;
      case 10: case 12: u.op = j32 ? U_JLT32 : U_JLT; return u;
      case 11: case 13: u.op = j32 ? U_JLE32 : U_JLE; return u;
      case 8:  // CALL
        if (source) return fault_uop(EBPF_ST_INSN);          // callx: todo!() emu.rs:270
        if (target == 0xFFFFFFFFu) return fault_uop(EBPF_ST_ARITH);  // pc + 1 overflow
        u.op = U_CALL; u.aux = 0; u.src = 0;
        return u;
      case 9: u.op = U_EXIT; u.aux = 0; u.src = 0; return u;
      default: return fault_uop(EBPF_ST_INSN);
    }
  }
  // LS (emu.rs:311-444): src, r0 and dst are read first (emu.rs:320-322)
  if (in.src >= 11 || in.dst >= 11) return fault_uop(EBPF_ST_INSN);
  const uint8_t mode = code & 0xe0, size = code & 0x18;
  const uint8_t w = size == 0x00 ? 4 : size == 0x08 ? 2 : size == 0x10 ? 1 : 8;
  u.x = (int32_t)in.off;
  if (cls == 0 || cls == 1) {
    if (mode == 0x00) { u.op = U_LDIMM; u.k = in.imm64; u.src = 0; return u; }
    if (mode == 0x60 && cls == 1) { u.op = U_LDX; u.aux = w; return u; }
    return fault_uop(EBPF_ST_INSN);  // ABS/IND (:336), LD+MEM (:339), ATOMIC (:351)
  }
  if (mode == 0x60) {
    u.aux = w;
    if (cls == 2) { u.op = U_ST; u.k = in.imm64; u.src = 0; }  // zero-extended imm (Q8)
    else u.op = U_STX;
    return u;
  }
  if (mode == 0xc0) {  // ATOMIC (emu.rs:373-437), ST class behaves like STX here
    u.op = U_ATOMIC;
    u.aux = (uint8_t)((size == 0 ? F_ATOMIC32 : 0) | ((in.imm64 & 1) ? F_FETCH : 0));
    const int64_t aop = in.imm64 & 0xfe;
    const bool known = aop == 0x00 || aop == 0x40 || aop == 0x50 || aop == 0xa0 || aop == 0xe0 ||
                       aop == 0xf0;
    u.k = known ? aop : 0xff;  // unknown op faults only after the 8-byte read (emu.rs:375,421)
    return u;
  }
  return fault_uop(EBPF_ST_INSN);  // ST/STX with IMM/ABS/IND (emu.rs:438)
}

int parse_hex_u64s(const char* hex, std::vector<uint8_t>& image) {
  // hexs_to_u64s (ins.rs:60-74): trim, drop spaces, 16-digit chunks, u64::from_str_radix
  std::string s(hex ? hex : "");
  size_t b = 0, e = s.size();
  while (b < e && isspace((unsigned char)s[b])) b++;
  while (e > b && isspace((unsigned char)s[e - 1])) e--;
  std::string t;
  for (size_t i = b; i < e; i++)
    if (s[i] != ' ') t.push_back(s[i]);
  image.clear();
  for (size_t i = 0; i < t.size(); i += 16) {
    if (i + 16 > t.size()) return EBPF_ELEN;  // "invalid hex format for u64"
    uint64_t v = 0;
    for (size_t j = 0; j < 16; j++) {
      const char c = t[i + j];
      int d;
      if (c >= '0' && c <= '9') d = c - '0';
      else if (c >= 'a' && c <= 'f') d = c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') d = c - 'A' + 10;
      else if (c == '+' && j == 0) continue;  // from_str_radix accepts a leading '+'
      else return EBPF_EHEX;
      v = (v << 4) | (uint64_t)d;
    }
    for (int k = 7; k >= 0; k--) image.push_back((uint8_t)(v >> (8 * k)));  // BE text -> LE image
  }
  return EBPF_OK;
}

struct DevWorkspace {
  void* ptr = nullptr;
  uint64_t bytes = 0;
  // buffers outgrown by a larger batch: kept, not freed -- another host thread may have taken
  // the old pointer for a batch on the same (device, stream) it has not launched yet (the growth
  // doubles, so these add at most the current size)
  std::vector<void*> retired;
};

std::mutex g_ws_mu;
std::map<std::pair<int, void*>, DevWorkspace> g_ws;  // (device, stream) -> library scratch

int device_of_current() {
  int d = 0;
  hipGetDevice(&d);
  return d;
}

}  // namespace

struct ebpf_prog {
  std::vector<RefInsn> insns;
  std::vector<Uop> uops;  // one per decoded instruction: the general interpreter's (interp_kernel)
  int tier = 0;
  // the micro-ops every other kernel runs: uops, or for a program with CALL the copies of
  // flatten_calls (no CALL, no EXIT with a frame stack); xtier: their memory tier
  std::vector<Uop> xuops;
  int xtier = 0;
  bool flattened = false;  // xuops are flatten_calls' copies
  bool tiny = false;  // straight-line and <= kTinyUops: persistent grid (see interp_grid)
  std::vector<DUop> duops;   // tier 0, forward jumps only, <= kMaxDagUops: dag_kernel's table
  std::vector<DUop> duopsk;  // the same with constant-address loads resolved (no init_regs)
  std::mutex mu;
  Uop* dev_uops[kMaxDevices] = {};
  DUop* dev_duops[kMaxDevices] = {};
  DUop* dev_duopsk[kMaxDevices] = {};
  // memory tier 0.5 (analyze_stack): the stack window, and the constant-address loads the compiled
  // code reads from the header window without a run-time window check: (address, width)
  StackPlan stack;
  std::vector<std::pair<uint64_t, uint32_t>> kloads;
  std::vector<TUop> tuops, tuopsk;  // tile_kernel's tables (forward-only, <= 62 micro-ops)
  TUop* dev_tuops[kMaxDevices] = {};
  TUop* dev_tuopsk[kMaxDevices] = {};
  // tile_kernel in loop mode (any tier-0 program of <= 62 micro-ops): block and exact tables
  std::vector<TUop> ltuops, ltuopsx;
  TUop* dev_ltuops[kMaxDevices] = {};
  TUop* dev_ltuopsx[kMaxDevices] = {};
  // the compiled program (jit.cpp), per variant of tuops / tuopsk: code object, and its module on
  // each device. Variants: 0 tuops (init_regs batches), 1 tuopsk (the main.rs layout), 2 the loop
  // program (ltuops + ltuopsx). jit_state: 0 not compiled yet, 1 compiled, 2 not a compiled
  // program, < 0 failed
  int jit_state = 0;
  bool jit_has[kJitVariants] = {};
  bool jit_occ[kJitVariants] = {};  // the variant's code also went into ebpf_tile_jit_fixed_occ
  std::vector<char> jit_co[kJitVariants];
  bool jit_deep = false;  // variant 2 compiled into ebpf_tile_jit_loop_deep
  std::string jit_asm[kJitVariants];
  std::string jit_err;
  hipModule_t jit_mod[kMaxDevices][kJitVariants] = {};
  JitFns jit_fn[kMaxDevices][kJitVariants];
  // xdp_md batches: the forward table with the ctx's data field (8) known at load time, so a
  // standard XDP program's `ldxw rD, [r1 + 0]` (ctx->data) is the constant 8 and its packet
  // loads through rD are constant-address loads (fold_const_loads xdp); variant 3 when it
  // differs from tuopsk
  std::vector<TUop> tuopsk_xdp;
  // stack-slot promotion (promote_slots): a stack-window loop program whose window holds whole
  // 8-byte slots becomes a tier-0 loop program with each slot in a free register (variant 4 of
  // the compiled program, the loop kernels' full byte-loop machinery); its lanes whose packet
  // reaches the window (LEN > r10 - k) deoptimize to the general interpreter
  std::vector<Uop> puops;
  std::vector<TUop> pltuops, pltuopsx;
  TUop* dev_pltuops[kMaxDevices] = {};
  TUop* dev_pltuopsx[kMaxDevices] = {};
  uint32_t pguard_k = 0;
  bool pjit_deep = false;  // variant 4 compiled into ebpf_tile_jit_loop_deep
  bool xjit_deep = false;  // variant 5 likewise
  bool rjit_deep = false;  // variant 6 likewise
};

// Diagnostics: EBPFEMU_TRACE=1 gives the compiled fixed-slot kernel a per-device stamp buffer
// (LaunchArgs::trace, kTraceWaves x kTraceSlots u64), zeroed before each launch;
// ebpf_debug_trace() returns it.
static const bool g_trace = [] {
  const char* e = getenv("EBPFEMU_TRACE");
  return e && e[0] == '1';
}();
static uint64_t* g_trace_buf[kMaxDevices] = {};
static uint32_t g_trace_launch[kMaxDevices] = {};

// EBPFEMU_TEST_FAIL_STACK_JIT=1 (tests): every stack-window program's compilation fails, so
// that the fallback to the general interpreter is exercised.
static const bool g_fail_stack_jit = [] {
  const char* e = getenv("EBPFEMU_TEST_FAIL_STACK_JIT");
  return e && e[0] == '1';
}();

// The compiled variants of recently compiled programs: a program loaded again (the same
// instructions, the same compile-time switches) takes copies of them instead of compiling.
// Bounded by the code objects' bytes (oldest out first).
struct JitRes {
  bool ok = false, deep = false, occ = false;
  std::string err, text;
  std::vector<char> co;
};
struct JitCacheEnt {
  std::string key;
  std::vector<JitRes> r;
  size_t bytes = 0;
};
static constexpr size_t kJitCacheBytes = 96u << 20;
static std::mutex g_jit_cache_mu;
static std::vector<JitCacheEnt> g_jit_cache;  // oldest first
static size_t g_jit_cache_bytes = 0;

static std::string jit_cache_key(const ebpf_prog* p) {
  std::string k;
  k.reserve(p->insns.size() * 16 + 16);
  for (const RefInsn& i : p->insns) {
    char b[16];
    std::memcpy(b, &i.imm64, 8);  // (imm is imm64's low half)
    std::memcpy(b + 8, &i.imm, 4);
    std::memcpy(b + 12, &i.off, 2);
    b[14] = (char)i.code;
    b[15] = (char)(i.dst | (i.src << 4));
    k.append(b, 16);
  }
  for (int v = 0; v < kJitVariants; v++) k += p->jit_has[v] ? '1' : '0';
  const char* e = getenv("EBPFEMU_FIXED_OCC");
  k += std::string("|") + (e ? e : "-") + (g_fail_stack_jit ? "F" : "");
  return k;
}

static bool jit_cache_get(const std::string& key, JitRes* r) {
  std::lock_guard<std::mutex> g(g_jit_cache_mu);
  for (const JitCacheEnt& c : g_jit_cache)
    if (c.key == key) {
      for (int v = 0; v < kJitVariants; v++) r[v] = c.r[v];
      return true;
    }
  return false;
}

static void jit_cache_put(const std::string& key, const JitRes* r) {
  JitCacheEnt c;
  c.key = key;
  c.r.assign(r, r + kJitVariants);
  for (const JitRes& q : c.r) c.bytes += q.co.size() + q.text.size();
  if (c.bytes > kJitCacheBytes / 4) return;
  std::lock_guard<std::mutex> g(g_jit_cache_mu);
  for (const JitCacheEnt& o : g_jit_cache)
    if (o.key == key) return;
  while (!g_jit_cache.empty() && g_jit_cache_bytes + c.bytes > kJitCacheBytes) {
    g_jit_cache_bytes -= g_jit_cache.front().bytes;
    g_jit_cache.erase(g_jit_cache.begin());
  }
  g_jit_cache_bytes += c.bytes;
  g_jit_cache.push_back(std::move(c));
}

// Compile both table variants (caller holds p->mu). Returns the C ABI code of ebpf_prog_compile.
static int jit_compile_locked(ebpf_prog* p) {
  if (p->jit_state == 0) {
    p->jit_has[0] = p->jit_has[1] = !p->tuops.empty() && !p->tuopsk.empty();
    p->jit_has[2] = !p->ltuops.empty() && !p->ltuopsx.empty();
    p->jit_has[3] = !p->tuopsk_xdp.empty() && !p->stack.k;
    p->jit_has[4] = !p->pltuops.empty() && !p->pltuopsx.empty();
    // variant 5: a loop program that reads a 4-byte word at offset 0 or 4 of a register (an
    // xdp_md program's ctx loads, through r1 or a copy of it: jit.cpp ctx_load) gets a copy for
    // xdp_md batches, whose staged images' ctx the range analysis knows
    p->jit_has[5] = false;
    if (p->jit_has[2] && !p->stack.k)
      for (const Uop& u : p->xuops)
        p->jit_has[5] = p->jit_has[5] || (u.op == U_LDX && u.aux == 4 && (u.x == 0 || u.x == 4));
    // variant 6: the same program for xdp_md batches in place (rebased, jit.cpp
    // Compiler::xdp_rebase) when every packet load is proven past the ctx
    p->jit_has[6] = p->jit_has[5];
    if (p->stack.k) p->jit_has[1] = !p->tuopsk.empty();  // (the main.rs layout only)
    if (!p->jit_has[0] && !p->jit_has[1] && !p->jit_has[2]) {
      p->jit_state = 2;
    } else {
      p->jit_state = 1;
      // the variants are independent compiles (own Compiler, own code object; the program's
      // tables are read-only here): all at once, one thread each, then their results in order
      JitRes r[kJitVariants];
      const std::string key = jit_cache_key(p);
      const bool cached = jit_cache_get(key, r);
      std::vector<std::thread> th;
      for (int v = 0; v < kJitVariants && !cached; v++) {
        if (!p->jit_has[v]) continue;
        th.emplace_back([p, v, &r] {
          JitRes& q = r[v];
          if (v == 5 || v == 6)
            q.ok = jit_compile_loop(p->xuops, p->ltuops, p->ltuopsx, q.co, &q.err, &q.text, nullptr,
                                    &q.deep, 0, true, v == 6);
          else if (v == 4)
            q.ok = jit_compile_loop(p->puops, p->pltuops, p->pltuopsx, q.co, &q.err, &q.text,
                                    nullptr, &q.deep, p->pguard_k);
          else
            q.ok = !(g_fail_stack_jit && p->stack.k) &&
                   (v == 2 ? jit_compile_loop(p->xuops, p->ltuops, p->ltuopsx, q.co, &q.err, &q.text,
                                              p->stack.k ? &p->stack : nullptr, &q.deep)
                           : jit_compile(p->xuops, v == 3 ? p->tuopsk_xdp : v ? p->tuopsk : p->tuops,
                                         q.co, &q.err, &q.text, p->stack.k ? &p->stack : nullptr,
                                         &q.occ, v == 1));
        });
      }
      for (std::thread& t : th) t.join();
      if (!cached) jit_cache_put(key, r);
      auto take = [&](int v) {
        p->jit_co[v] = std::move(r[v].co);
        p->jit_asm[v] = std::move(r[v].text);
        p->jit_occ[v] = r[v].occ;
        bool* deep = v == 2 ? &p->jit_deep : v == 4 ? &p->pjit_deep : v == 5 ? &p->xjit_deep
                     : v == 6 ? &p->rjit_deep : nullptr;
        if (deep) *deep = r[v].deep;
      };
      for (int v = 0; v < kJitVariants && p->jit_state == 1; v++) {
        if (!p->jit_has[v]) continue;
        take(v);
        if (v == 5 || v == 6) {  // the xdp_md copies: dropped (staged / the plain loop program
                                 // runs) if they fail
          if (!r[v].ok) {
            p->jit_has[v] = false;
            p->jit_co[v].clear();
          }
          continue;
        }
        if (v == 4) {  // the promoted program: dropped (the stack loop kernel stays) if it fails
          if (!r[4].ok) {
            p->jit_err = r[4].err;
            p->jit_has[4] = false;
            p->jit_co[4].clear();
            p->puops.clear();
            p->pltuops.clear();
            p->pltuopsx.clear();
          }
          continue;
        }
        const bool ok = r[v].ok;
        if (!ok) p->jit_err = r[v].err;
        if (!ok && v >= 1 && p->stack.k && !p->jit_has[0]) {
          // a stack-window program whose code does not assemble (e.g. branches past the
          // assembler's reach in a huge program): it stays on the general interpreter. Its
          // stack tables are dropped too (batch_kind also routes tier-1 programs only there:
          // the tables may already be on a device, and tile_kernel runs no stores)
          p->stack = StackPlan();
          p->kloads.clear();
          p->tuopsk.clear();
          p->ltuops.clear();
          p->ltuopsx.clear();
          p->jit_has[4] = false;  // (the promoted program needs the stack plan's launch checks)
          p->puops.clear();
          p->pltuops.clear();
          p->pltuopsx.clear();
          p->jit_has[1] = p->jit_has[2] = false;
          p->jit_co[1].clear();
          p->jit_co[2].clear();
          for (int w = v + 1; w < kJitVariants; w++) {  // (compiled alongside, never used)
            p->jit_has[w] = false;
            p->jit_co[w].clear();
          }
          break;
        }
        if (!ok) p->jit_state = EBPF_EJIT;
      }
      if (p->jit_state == 1 && !p->jit_has[0] && !p->jit_has[1] && !p->jit_has[2])
        p->jit_state = 2;
    }
  }
  return p->jit_state == 1 ? 1 : p->jit_state == 2 ? 0 : p->jit_state;
}

// Length-binned lane packing for the loop-mode tile kernel (EBPFEMU_BIN=0|1 forces it off/on;
// default: offsets + lens layouts of >= kBinMinPackets packets).
static const int g_bin = [] {
  const char* e = getenv("EBPFEMU_BIN");
  return e ? (e[0] == '1' ? 1 : 0) : -1;
}();
constexpr uint64_t kBinMinPackets = 16384;

// EBPFEMU_XDP_STAGE=1 (A/B): every xdp_md batch goes through xdp_stage (xdp_in_place). (Outside the
// extern "C" block below: a lambda initializer there was given the same closure as g_trace's by
// the host compiler, so the flag read EBPFEMU_TRACE.)
static const bool g_xdp_stage = [] {
  const char* e = getenv("EBPFEMU_XDP_STAGE");
  return e && e[0] == '1';
}();

// Width mask of an access of w bytes.
static uint64_t width_mask(uint32_t w) { return w >= 8 ? ~0ull : ((1ull << (8 * w)) - 1); }

// dag_kernel's table: every per-step quantity that depends only on the micro-op (uop.h DUop).
// The asm loop's handler for a (canonical) micro-op, and the immediate it consumes (d16-17).
static uint32_t asm_handler(uint32_t op, uint32_t aux, uint64_t k, uint64_t& imm) {
  const bool reg = aux & F_SRC;
  imm = k;
  auto pick = [&](uint32_t h_imm, uint32_t h_reg) { return reg ? h_reg : h_imm; };
  switch (op) {
    case U_EXIT: return H_EXIT;
    case U_LDIMM: return H_MOV64_IMM;
    case U_MOV64: return pick(H_MOV64_IMM, H_MOV64_REG);
    case U_ADD64: return pick(H_ADD64_IMM, H_ADD64_REG);
    case U_SUB64:
      if (!reg) imm = 0 - k;  // a - k == a + (-k) mod 2^64
      return pick(H_ADD64_IMM, H_SUB64_REG);
    case U_AND64: return pick(H_AND64_IMM, H_AND64_REG);
    case U_OR64: return pick(H_OR64_IMM, H_OR64_REG);
    case U_XOR64: return pick(H_XOR64_IMM, H_XOR64_REG);
    case U_LSH64: imm = k & 63; return pick(H_LSH64_IMM, H_LSH64_REG);
    case U_RSH64: imm = k & 63; return pick(H_RSH64_IMM, H_RSH64_REG);
    case U_MOV32: imm = (uint32_t)k; return pick(H_MOV32_IMM, H_MOV32_REG);
    case U_ADD32: return pick(H_ADD32_IMM, H_ADD32_REG);
    case U_SUB32:
      if (!reg) imm = (uint32_t)(0u - (uint32_t)k);
      return pick(H_ADD32_IMM, H_SUB32_REG);
    case U_AND32: return pick(H_AND32_IMM, H_AND32_REG);
    case U_OR32: return pick(H_OR32_IMM, H_OR32_REG);
    case U_XOR32: return pick(H_XOR32_IMM, H_XOR32_REG);
    case U_LSH32: imm = k & 31; return pick(H_LSH32_IMM, H_LSH32_REG);
    case U_RSH32: imm = k & 31; return pick(H_RSH32_IMM, H_RSH32_REG);
    case U_ZX16: return H_ZX16;
    case U_ZX32: return H_ZX32;
    case U_NOP: return H_NOP;
    case U_BSWAP16: return H_BSWAP16;
    case U_BSWAP32: return H_BSWAP32;
    case U_BSWAP64: return H_BSWAP64;
    case U_JA: return H_JA;
    case U_JEQ: return pick(H_JEQ_IMM, H_JEQ_REG);
    case U_JGT: return pick(H_JGT_IMM, H_JGT_REG);
    case U_JLT: return pick(H_JLT_IMM, H_JLT_REG);
    case U_JSET: return pick(H_JSET_IMM, H_JSET_REG);
    case U_JEQ32: return pick(H_JEQ32_IMM, H_JEQ32_REG);
    case U_JGT32: return pick(H_JGT32_IMM, H_JGT32_REG);
    case U_JLT32: return pick(H_JLT32_IMM, H_JLT32_REG);
    case U_JSET32: return pick(H_JSET32_IMM, H_JSET32_REG);
    case U_LDX: imm = k; return H_LDX;  // k: the sign-extended offset (set by the caller)
    // the self-contained tile loop only (the hybrid loop hands these to its C++ step)
    case U_MUL64: return pick(H_MUL64_IMM, H_MUL64_REG);
    case U_MUL32: imm = (uint32_t)k; return pick(H_MUL32_IMM, H_MUL32_REG);
    case U_NEG64: return H_NEG64;
    case U_NEG32: return H_NEG32;
    case U_ARSH64: imm = k & 63; return pick(H_ARSH64_IMM, H_ARSH64_REG);
    case U_ARSH32: imm = k & 31; return pick(H_ARSH32_IMM, H_ARSH32_REG);
    case U_DIV64: return pick(H_DIV64_IMM, H_DIV64_REG);
    case U_MOD64: return pick(H_MOD64_IMM, H_MOD64_REG);
    case U_DIV32: imm = (uint32_t)k; return pick(H_DIV32_IMM, H_DIV32_REG);
    case U_MOD32: imm = (uint32_t)k; return pick(H_MOD32_IMM, H_MOD32_REG);
    case U_FAULT: imm = aux; return H_FAULT;  // aux: the status it raises
    default: return H_SLOW;
  }
}

static std::vector<DUop> build_dag(const std::vector<Uop>& uops) {
  const uint32_t n = (uint32_t)uops.size();
  std::vector<DUop> d(n);
  auto bit = [&](uint32_t pc) -> uint64_t { return pc < n && n <= 64 ? 1ull << pc : 0ull; };
  for (uint32_t i = 0; i < n; i++) {
    const Uop& u = uops[i];
    DUop& o = d[i];
    std::memset(&o, 0, sizeof o);
    uint32_t op = u.op;
    o.doff = (uint32_t)u.dst * kRegStride;
    o.soff = (uint32_t)u.src * kRegStride;
    o.npc = i + 1 < n ? i + 1 : PC_DONE;
    o.nbit = bit(i + 1);
    o.k = (uint64_t)u.k;
    if (u.op >= U_JA && u.op <= U_JLE32) {
      const uint32_t t = (uint32_t)u.x;
      o.x = t < n ? t : PC_DONE;
      o.tbit = bit(t);
      // canonical conditions: "jump if not C" = "jump if C" with the two successors swapped
      switch (u.op) {
        case U_JNE: op = U_JEQ; break;
        case U_JGE: op = U_JLT; break;
        case U_JLE: op = U_JGT; break;
        case U_JNE32: op = U_JEQ32; break;
        case U_JGE32: op = U_JLT32; break;
        case U_JLE32: op = U_JGT32; break;
        default: break;
      }
      if (op != u.op) {
        std::swap(o.x, o.npc);
        std::swap(o.tbit, o.nbit);
      }
    } else {
      o.x = (uint32_t)u.x;
    }
    o.opaux = op | ((uint32_t)u.aux << 8);
    if (u.op == U_LDX) {
      o.k = width_mask(u.aux);
      o.width = u.aux;
      o.kmask = o.k;
    }
    // the hand-written loop's half
    o.dst2 = 2u * u.dst;
    o.src2 = 2u * u.src;
    o.anpc = o.npc;
    o.ax = o.x;
    o.anbit = o.nbit;
    o.atbit = o.tbit;
    const uint64_t kk = u.op == U_LDX ? (uint64_t)(int64_t)u.x : (uint64_t)u.k;
    o.hoff = asm_handler(op, u.aux, kk, o.imm) * DAG_SLOT;
  }
  return d;
}

// tile_kernel's table (uop.h TUop) from the DUop table. A micro-op whose successor no jump can
// reach (and that is not itself a jump, exit or fault) gets the CHAINED handler form: the tile loop
// runs its successor next on the same lanes without touching the pc set (basic-block chaining).
// exact: every micro-op its own block (the loop mode's exact-budget table).
static std::vector<TUop> build_tile(const std::vector<Uop>& uops, const std::vector<DUop>& d,
                                    bool exact = false, bool stack = false) {
  const uint32_t n = (uint32_t)uops.size();
  // (programs above kTileMaxUops: a table for the compiler only; tile_kernel never runs them)
  std::vector<TUop> t(std::max<size_t>(kTileUops, n + 2));
  std::memset(t.data(), 0, t.size() * sizeof(TUop));
  // block starts: 0, jump targets, successors of block-ending micro-ops
  std::vector<char> start(n + 1, 0);
  start[0] = 1;
  std::vector<char> term(n, 0);  // jumps, exits, faults: always the end of their block
  for (uint32_t i = 0; i < n; i++) {
    const uint32_t h = d[i].hoff / DAG_SLOT;
    const bool is_jump = uops[i].op >= U_JA && uops[i].op <= U_JLE32;
    if (is_jump && (uint32_t)uops[i].x < n) start[(uint32_t)uops[i].x] = 1;
    // (a stack-window program's stores and atomics are compiled in line: jit.cpp, not block ends)
    const bool stack_store =
        stack && (uops[i].op == U_ST || uops[i].op == U_STX || uops[i].op == U_ATOMIC);
    term[i] = exact || is_jump || h == H_EXIT || h == H_FAULT || (h == H_SLOW && !stack_store);
    if (term[i]) start[i + 1] = 1;
  }
  // rem[i]: micro-ops from i to the end of its block (steps not retired when i faults);
  // blen[i] = rem[i] for a block start (the steps its lanes retire unless one faults)
  std::vector<uint32_t> rem(n + 1, 0);
  for (uint32_t i = n; i-- > 0;) rem[i] = (term[i] || start[i + 1]) ? 1 : rem[i + 1] + 1;
  for (uint32_t i = 0; i < n; i++) {
    const DUop& o = d[i];
    TUop& u = t[i];
    uint32_t h = o.hoff / DAG_SLOT;
    const bool chained = !term[i] && i + 1 < n && !start[i + 1];
    uint32_t id = chained ? kTileIdChained[h] : kTileIdEnd[h];
    u.dst2 = o.dst2;
    u.src2 = o.src2;
    u.npc = o.anpc;
    u.x = o.ax;
    u.a0 = o.a0;
    u.kmask = o.kmask;
    u.nbit = o.anbit;
    u.tbit = o.atbit;
    u.imm = o.imm;
    u.width = o.width;
    u.blen = start[i] ? rem[i] : 0;
    if (h == H_LDX || h == H_ARSH64_IMM || h == H_ARSH64_REG ||
        (stack && (uops[i].op == U_ATOMIC || uops[i].op == U_ST || uops[i].op == U_STX)))
      u.a0 = rem[i];  // REMX
    if (h == H_LDX && o.width == 1) id = chained ? T_LDX1_C : T_LDX1_E;  // one byte: one dword
    if (h == H_LDXK || h == H_LDXK_FAR) {
      const uint32_t a0 = o.a0, w = o.end - o.a0;
      u.x = o.end;      // KEND
      u.width = rem[i]; // REMK
      if (h == H_LDXK) {
        const uint32_t b0 = a0 & ~3u;
        u.src2 = b0;                                     // W0
        const uint32_t b1 = std::min(b0 + 4, (uint32_t)kWin - 4), b2 = std::min(b0 + 8, (uint32_t)kWin - 4);
        u.tbit = (uint64_t)b1 | ((uint64_t)b2 << 32);    // W1, W2
        if ((a0 & 3) + w <= 4) {
          id = chained ? T_LDXK1_C : T_LDXK1_E;
          u.imm = (a0 & 3) * 8;                          // KSHIFT
        } else if (w <= 4) {
          id = chained ? T_LDXK2_C : T_LDXK2_E;
        }
      }
    }
    u.hoff = id * TILE_SLOT;
  }
  t[t.size() - 1].hoff = T_DONE * TILE_SLOT;
  t[t.size() - 2].hoff = T_DONE * TILE_SLOT;  // exact-mode marker bit (loop mode)
  return t;
}

// Load-time constant propagation over a forward-only program, from the main.rs:28-31 register
// layout (r1 = 0 = the packet's image address, r0 and r3..r9 = 0; r2 = len and r10 are
// per-batch). Every LDX whose base register holds one known constant on all paths into it
// becomes U_LDXK with its address resolved, so the kernel neither reads that register nor
// waits on it before reading the packet window. Only used for batches without init_regs.
// xdp: the image starts with the xdp_md ctx (xdp.rs:16-20), whose data field is 8 on every lane:
// a 4-byte load of image address 0 into a register whose upper half is known zero (the loaded
// bytes replace only the low four, Q1) leaves the constant 8 -- r2 = 8 + len starts below 2^32.
static std::vector<DUop> fold_const_loads(const std::vector<Uop>& uops, std::vector<DUop> d,
                                          bool xdp = false) {
  const uint32_t n = (uint32_t)uops.size();
  struct Regs {
    bool reached = false;
    bool known[11] = {};
    bool hz[11] = {};  // the upper 32 bits are known to be zero
    uint64_t v[11] = {};
  };
  std::vector<Regs> in(n + 1);
  in[0].reached = true;
  for (int r = 0; r < 11; r++) in[0].known[r] = (r != 2 && r != 10), in[0].hz[r] = r != 10;
  auto flow = [&](uint32_t to, const Regs& s) {
    if (to >= n) return;
    Regs& t = in[to];
    if (!t.reached) {
      t = s;
      return;
    }
    for (int r = 0; r < 11; r++) {
      if (t.known[r] && !(s.known[r] && s.v[r] == t.v[r])) t.known[r] = false;
      t.hz[r] = t.hz[r] && s.hz[r];
    }
  };
  for (uint32_t i = 0; i < n; i++) {
    if (!in[i].reached) continue;
    const Uop& u = uops[i];
    Regs s = in[i];
    const bool src = u.aux & F_SRC;
    const bool ctx_data = xdp && u.op == U_LDX && u.aux == 4 && s.known[u.src] &&
                          s.v[u.src] + (uint64_t)(int64_t)u.x == 0 && s.hz[u.dst];
    const bool dst_hz = s.hz[u.dst];
    if (u.op == U_LDX && s.known[u.src]) {
      int64_t a;
      DUop& o = d[i];
      const bool ovf = __builtin_add_overflow((int64_t)s.v[u.src], (int64_t)u.x, &a);
      if (ovf || (uint64_t)a > 0xFFFFFFF0ull) {
        // address overflow (emu.rs:344 debug panic) or past any image (mem_size <= 2^24)
        o.opaux = U_FAULT | (EBPF_ST_MEM << 8);
        o.hoff = H_FAULT * DAG_SLOT;
        o.imm = EBPF_ST_MEM;
      } else {
        const uint64_t ua = (uint64_t)a;
        o.opaux = U_LDXK | ((uint32_t)u.aux << 8);
        o.addr = ua;
        o.a0 = (uint32_t)ua;
        o.end = (uint32_t)ua + u.aux;
        o.hoff = H_LDXK_FAR * DAG_SLOT;  // outside the window: global loads (tile loop only)
        // inside the header window (ua < kWin first: ua + width must not wrap): the asm loop
        // reads it; an address past the window or the image runs in the C++ step
        if (ua < (uint64_t)kWin && ua + u.aux <= (uint64_t)kWin) {
          const uint32_t b0 = (uint32_t)ua & ~3u;
          for (uint32_t w = 0; w < 3; w++) {
            const uint32_t b = std::min(b0 + 4 * w, (uint32_t)kWin - 4);  // unused dwords: any
            o.win[2 * w] = b & 0x30;
            o.win[2 * w + 1] = b & 15;
          }
          o.hoff = H_LDXK * DAG_SLOT;
        }
      }
    }
    switch (u.op) {
      case U_JA: case U_JEQ: case U_JGT: case U_JGE: case U_JSET: case U_JNE: case U_JLT:
      case U_JLE: case U_JEQ32: case U_JGT32: case U_JGE32: case U_JSET32: case U_JNE32:
      case U_JLT32: case U_JLE32:
        flow((uint32_t)u.x, s);
        if (u.op != U_JA) flow(i + 1, s);
        continue;
      case U_EXIT: case U_FAULT:
        continue;
      case U_MOV64:
        s.known[u.dst] = !src || s.known[u.src];
        s.v[u.dst] = src ? s.v[u.src] : (uint64_t)u.k;
        break;
      case U_MOV32:
        s.known[u.dst] = !src || s.known[u.src];
        s.v[u.dst] = (uint32_t)(src ? s.v[u.src] : (uint64_t)u.k);
        break;
      case U_LDIMM:
        s.known[u.dst] = true;
        s.v[u.dst] = (uint64_t)u.k;
        break;
      case U_ADD64:
        s.known[u.dst] = s.known[u.dst] && (!src || s.known[u.src]);
        s.v[u.dst] += src ? s.v[u.src] : (uint64_t)u.k;  // wrapping, emu.rs:81-83
        break;
      case U_NOP:
        break;
      case U_ST: case U_STX:  // registers unchanged (the dst write-back of emu.rs:443)
        break;
      case U_ATOMIC:  // (a stack-window program's) fetch writes src, CMPXCHG r0 (emu.rs:409-436)
        s.known[u.src] = s.known[0] = s.known[u.dst] = false;
        break;
      default:  // every other micro-op of tier 0 writes dst with a value not tracked here
        s.known[u.dst] = false;
        break;
    }
    // the upper halves: constants; 32-bit results (zero-extended, emu.rs:214-216); loads of at
    // most 4 bytes into a register whose upper half was zero
    if (u.op == U_LDX) {
      s.hz[u.dst] = dst_hz && u.aux <= 4;
      if (ctx_data) s.known[u.dst] = true, s.v[u.dst] = 8;
    } else if (u.op == U_MOV64) {
      s.hz[u.dst] = src ? s.hz[u.src] : (uint64_t)u.k >> 32 == 0;
    } else if ((u.op >= U_ADD32 && u.op <= U_ARSH32) || u.op == U_ZX16 || u.op == U_ZX32 ||
               u.op == U_BSWAP16 || u.op == U_BSWAP32) {
      s.hz[u.dst] = true;
    } else if (u.op == U_ATOMIC) {
      s.hz[u.src] = s.hz[0] = false;
    } else if (u.op != U_NOP && u.op != U_ST && u.op != U_STX) {
      s.hz[u.dst] = false;
    }
    for (int r = 0; r < 11; r++)
      if (s.known[r]) s.hz[r] = s.v[r] >> 32 == 0;
    flow(i + 1, s);
  }
  return d;
}

// CALL / EXIT without a frame stack (emu.rs:265-279, Q12). A CALL at pc p jumps to t = p + 1 + off
// and pushes t + 1; an EXIT pops the pc, or stops the program on an empty stack. The pushed
// return address is a load-time constant of the call site, so a program that does not recurse
// reaches a finite set of frame stacks, and the pair (pc, frame stack) is all the control state
// there is (no registers are saved, emu.rs:265-272). The reachable pairs become the micro-ops of
// a program without CALL: a CALL a jump to (t, stack + [t + 1]), an EXIT with a non-empty stack a
// jump to (popped pc, the rest), a push past EBPF_MAX_CALL_DEPTH a ST_CALLDEPTH fault, a jump or
// return past the end a jump past the program (a normal stop, Q11). Every instruction is still one
// micro-op, so steps, faults and the step budget are the reference's. Layout: the pairs in chains
// of fall-through successors (same stack, pc + 1), the chains in topological order of their jumps
// where there is one (then the program is forward-only again), the chain that falls off the end
// last. Fails (the general interpreter's frame stack runs the program) on recursion, more than
// kJitMaxUops pairs, or two chains falling off the end.
// Loop-invariant bound loads peeled (load time, every kernel but the general interpreter's):
//   H: ldx rN, [rB + off]      H+1: j<cc> rI, rN -> X      B: ...      J: ja H      X: (J + 1)
// -- a loop testing its bound at the top and reloading it every iteration, as an XDP program
// re-reading ctx->data_end -- becomes
//   H: ldx rN, [rB + off]      H+1: j<cc> rI, rN -> X      B: ...      nop      nop
//   j<!cc> rI, rN -> B         X
// when B holds no jump, store, call or exit and writes neither rN nor rB (rB != rN), and nothing
// else jumps into H+1 .. J. The reload rewrote rN with the value it held (same address, memory
// unchanged; a narrow load keeps rN's high bytes either way), so every step leaves the registers
// exactly as the original's step did -- the two nops retire the ja and the reload, the back edge
// the test -- while the loop becomes one block with its test at the bottom: a counted loop for the
// compiler (jit.cpp counted_entry: byte passes, the cooperative sums). Step counts are unchanged.
static void peel_invariant_loads(std::vector<Uop>& u) {
  auto neg = [](uint8_t op) -> int {
    switch (op) {
      case U_JGE: return U_JLT; case U_JLT: return U_JGE; case U_JGT: return U_JLE;
      case U_JLE: return U_JGT; case U_JEQ: return U_JNE; case U_JNE: return U_JEQ;
      case U_JGE32: return U_JLT32; case U_JLT32: return U_JGE32; case U_JGT32: return U_JLE32;
      case U_JLE32: return U_JGT32; case U_JEQ32: return U_JNE32; case U_JNE32: return U_JEQ32;
      default: return -1;
    }
  };
  for (const Uop& o : u)
    if (o.op == U_CALL) return;
  for (uint32_t J = 2; J < u.size(); J++) {
    const uint32_t n = (uint32_t)u.size();
    if (u[J].op != U_JA || (uint32_t)u[J].x >= J) continue;
    const uint32_t H = (uint32_t)u[J].x;
    if (H + 2 > J) continue;
    const Uop &ld = u[H], &jt = u[H + 1];
    if (ld.op != U_LDX || ld.dst == ld.src || ld.dst > 10 || ld.src > 10) continue;
    if (neg(jt.op) < 0 || !(jt.aux & F_SRC) || (uint32_t)jt.x != J + 1) continue;
    const uint8_t rN = ld.dst, rB = ld.src;
    if (!((jt.src == rN && jt.dst != rN) || (jt.dst == rN && jt.src != rN))) continue;
    bool ok = true;
    for (uint32_t i = H + 2; i < J && ok; i++) {
      const Uop& b = u[i];
      const bool writes = (b.op <= U_BSWAP64 && b.op != U_NOP) || b.op == U_LDIMM || b.op == U_LDX;
      ok = b.op <= U_BSWAP64 || b.op == U_LDIMM || b.op == U_LDX;
      if (writes && (b.dst == rN || b.dst == rB)) ok = false;
    }
    for (uint32_t i = 0; i < n && ok; i++) {  // no other way into H+1 .. J
      const Uop& b = u[i];
      if (b.op < U_JA || b.op > U_JLE32 || i == J) continue;
      const uint32_t x = (uint32_t)b.x;
      if (x > H && x <= J) ok = false;
    }
    if (!ok) continue;
    // the shift: every jump target past J moves 2 on
    for (Uop& b : u)
      if (b.op >= U_JA && b.op <= U_JLE32 && (uint32_t)b.x > J) b.x = (int32_t)((uint32_t)b.x + 2);
    Uop nop{};
    nop.op = U_NOP;
    Uop back = u[H + 1];
    back.op = (uint8_t)neg(back.op);
    back.x = (int32_t)(H + 2);
    u[J] = nop;
    u.insert(u.begin() + J + 1, {nop, back});
    J += 2;
  }
}

static bool flatten_calls(const std::vector<Uop>& u, std::vector<Uop>& out) {
  const uint32_t n = (uint32_t)u.size();
  if (n == 0) return false;
  std::map<std::vector<uint32_t>, uint32_t> id;
  std::vector<std::vector<uint32_t>> ctx;
  auto ctx_of = [&](const std::vector<uint32_t>& st) -> uint32_t {
    auto it = id.find(st);
    if (it != id.end()) return it->second;
    id.emplace(st, (uint32_t)ctx.size());
    ctx.push_back(st);
    return (uint32_t)ctx.size() - 1;
  };
  // explore the reachable (stack, pc) pairs; succ: the jump-like successor of each (or none)
  std::map<std::pair<uint32_t, uint32_t>, int64_t> state;  // -> the pair's index in `order`
  std::vector<std::pair<uint32_t, uint32_t>> order, work;
  auto visit = [&](uint32_t c, uint32_t pc) -> bool {
    if (pc >= n || state.count({c, pc})) return true;
    if (state.size() >= kJitMaxUops) return false;
    state[{c, pc}] = (int64_t)order.size();
    order.push_back({c, pc});
    work.push_back({c, pc});
    return true;
  };
  // the jump-like successor of a pair: (context, pc), pc >= n for a stop; kind 0 none
  auto jump_of = [&](uint32_t c, uint32_t pc, std::pair<uint32_t, uint32_t>& to) -> bool {
    const Uop& o = u[pc];
    if (o.op == U_CALL) {
      if (ctx[c].size() >= EBPF_MAX_CALL_DEPTH) return false;  // (a ST_CALLDEPTH fault)
      std::vector<uint32_t> st = ctx[c];
      st.push_back((uint32_t)o.x + 1);
      to = {ctx_of(st), (uint32_t)o.x};
      return true;
    }
    if (o.op == U_EXIT) {
      if (ctx[c].empty()) return false;
      std::vector<uint32_t> st = ctx[c];
      const uint32_t r = st.back();
      st.pop_back();
      to = {ctx_of(st), r};
      return true;
    }
    if (o.op >= U_JA && o.op <= U_JLE32) {
      to = {c, (uint32_t)o.x};
      return true;
    }
    return false;
  };
  auto falls = [&](uint32_t pc) {  // the pair continues at pc + 1 (taken or not)
    const uint8_t op = u[pc].op;
    return op != U_JA && op != U_EXIT && op != U_FAULT && op != U_CALL;
  };
  ctx_of({});
  visit(0, 0);
  while (!work.empty()) {
    const auto w = work.back();
    work.pop_back();
    std::pair<uint32_t, uint32_t> to;
    if (jump_of(w.first, w.second, to) && !visit(to.first, to.second)) return false;
    if (falls(w.second) && !visit(w.first, w.second + 1)) return false;
  }
  // chains of fall-through successors
  const size_t S = order.size();
  std::vector<int64_t> chain_of(S, -1);
  std::vector<std::vector<uint32_t>> chains;
  for (size_t i = 0; i < S; i++) {
    const auto [c, pc] = order[i];
    if (pc > 0 && falls(pc - 1) && state.count({c, pc - 1})) continue;  // inside another chain
    std::vector<uint32_t> ch;
    for (uint32_t q = pc;; q++) {
      const int64_t k = state.at({c, q});
      chain_of[k] = (int64_t)chains.size();
      ch.push_back((uint32_t)k);
      if (!falls(q) || q + 1 >= n) break;
    }
    chains.push_back(std::move(ch));
  }
  const size_t C = chains.size();
  int64_t tail = -1;  // the chain whose last pair falls off the end
  for (size_t k = 0; k < C; k++) {
    const uint32_t last = order[chains[k].back()].second;
    if (falls(last) && last + 1 >= n) {
      if (tail >= 0) return false;
      tail = (int64_t)k;
    }
  }
  // topological order of the chains by their jumps (Kahn), the falling-off chain last; with a
  // cycle (a loop, or a return to an earlier pair), discovery order: a loop program
  std::vector<std::set<uint32_t>> to_ch(C);
  std::vector<uint32_t> indeg(C, 0);
  bool cyclic = false;
  for (size_t k = 0; k < C; k++)
    for (size_t j = 0; j < chains[k].size(); j++) {
      const auto [c, pc] = order[chains[k][j]];
      std::pair<uint32_t, uint32_t> to;
      if (!jump_of(c, pc, to) || to.second >= n) continue;
      const int64_t t = state.at(to), tc = chain_of[t];
      if (tc == (int64_t)k) {
        const size_t pos = std::find(chains[k].begin(), chains[k].end(), (uint32_t)t) -
                           chains[k].begin();
        cyclic = cyclic || pos <= j;
      } else if (to_ch[k].insert((uint32_t)tc).second) {
        indeg[tc]++;
      }
    }
  std::vector<uint32_t> seq;
  if (!cyclic) {
    std::vector<uint32_t> ready;
    for (size_t k = C; k-- > 0;)
      if (!indeg[k] && (int64_t)k != tail) ready.push_back((uint32_t)k);
    while (!ready.empty()) {
      const uint32_t k = ready.back();
      ready.pop_back();
      seq.push_back(k);
      for (uint32_t t : to_ch[k])
        if (--indeg[t] == 0 && (int64_t)t != tail) ready.push_back(t);
    }
    if (tail >= 0 && indeg[tail] == 0) seq.push_back((uint32_t)tail);
  }
  if (seq.size() != C) {
    seq.clear();
    for (size_t k = 0; k < C; k++)
      if ((int64_t)k != tail) seq.push_back((uint32_t)k);
    if (tail >= 0) seq.push_back((uint32_t)tail);
  }
  std::vector<uint32_t> at(S);
  uint32_t N = 0;
  for (uint32_t k : seq)
    for (uint32_t s2 : chains[k]) at[s2] = N++;
  const uint32_t kPast = 0xFFFFFFFEu;  // a jump target past the program: a normal stop
  out.assign(N, Uop{});
  for (size_t i = 0; i < S; i++) {
    const auto [c, pc] = order[i];
    Uop o = u[pc];
    std::pair<uint32_t, uint32_t> to;
    const bool j = jump_of(c, pc, to);
    const uint32_t x = j && to.second < n ? at[state.at(to)] : kPast;
    if (o.op == U_CALL) {
      if (!j) {
        o = fault_uop(EBPF_ST_CALLDEPTH);
      } else {
        o.op = U_JA;
        o.x = (int32_t)x;
      }
    } else if (o.op == U_EXIT && j) {
      o.op = U_JA;
      o.x = (int32_t)x;
      o.dst = 0;  // (JA reads dst, emu.rs:220: r0 is always valid)
    } else if (o.op >= U_JA && o.op <= U_JLE32) {
      o.x = (int32_t)x;
    }
    out[at[i]] = o;
  }
  return true;
}

// Memory tier 0.5 (stack-window programs): a program of <= kJitMaxUops micro-ops (loops included:
// the compiled loop kernel's stack variant) whose only memory writes are ST/STX at r10 + c for a
// c known at load time (the XDP spill / key
// pattern: `stxdw [r10-8], r3`, also through a copy such as `mov r2, r10; add r2, -16`), with no
// ATOMIC or CALL. A load-time dataflow over the main.rs register layout (main.rs:28-31) tracks
// each register as unknown, a constant, or r10 + c; every store must be r10 + c on all paths, with
// all its bytes in [r10 - k, r10) for the window size k <= kStackMax (emu.rs:354-372; the
// reference has no separate stack -- r10 is just a register into the flat image, which is why the
// launch also checks that the window lies inside the image, past the packet, and away from every
// constant-address load). Loads whose base is r10 + c and whose bytes lie in the window read it
// directly; loads partly inside it make the program ineligible; every other load is checked
// against the window at run time (a store-forwarding overlay).
struct StackAnalysis {
  StackPlan plan;  // k = 0: not a stack-window program
};

static StackAnalysis analyze_stack(const std::vector<Uop>& uops) {
  StackAnalysis res;
  const uint32_t n = (uint32_t)uops.size();
  if (n == 0 || n > kJitMaxUops) return res;
  bool any_store = false, loops = false;
  for (uint32_t i = 0; i < n; i++) {
    const Uop& u = uops[i];
    if (u.op == U_CALL) return res;
    loops = loops || (u.op >= U_JA && u.op <= U_JLE32 && (uint32_t)u.x <= i);  // back edges
    // atomics: the operations emu.rs:391-419 implements (others panic: the general interpreter)
    if (u.op == U_ATOMIC && !(u.k == 0x00 || u.k == 0x40 || u.k == 0x50 || u.k == 0xa0 ||
                              u.k == 0xe0 || u.k == 0xf0))
      return res;
    any_store = any_store || u.op == U_ST || u.op == U_STX || u.op == U_ATOMIC;
  }
  if (!any_store) return res;
  enum Kind : uint8_t { TOP, CONST, FP };
  struct Val { Kind k = TOP; int64_t v = 0; };
  struct Regs { bool reached = false; Val r[11]; };
  std::vector<Regs> in(n + 1);
  in[0].reached = true;
  for (int r = 0; r < 11; r++) in[0].r[r] = Val{CONST, 0};
  in[0].r[2] = Val{TOP, 0};   // len
  in[0].r[10] = Val{FP, 0};   // r10 itself
  auto same = [](const Val& a, const Val& b) { return a.k == b.k && (a.k == TOP || a.v == b.v); };
  bool changed = false;
  auto flow = [&](uint32_t to, const Regs& st) {
    if (to >= n) return;
    Regs& t = in[to];
    if (!t.reached) { t = st; changed = true; return; }
    for (int r = 0; r < 11; r++)
      if (!same(t.r[r], st.r[r]) && t.r[r].k != TOP) t.r[r] = Val{TOP, 0}, changed = true;
  };
  std::vector<int32_t> off(n, kNoStack), pw(n, kNoStack);
  std::vector<char> dyn(n, 0);  // LDX with an unknown base
  std::vector<char> dyns(n, 0);  // ST/STX with an unknown base (store mode)
  bool any_pw = false, any_dyn = false;
  int64_t lo = 0, hi = INT64_MIN;  // store bytes relative to r10: [lo, hi)
  // passes in pc order until the states stop changing (one pass without back edges; with them
  // each join only moves a register towards unknown, so this ends), the last one collecting
  for (int pass = 0;; pass++) {
  changed = false;
  std::fill(off.begin(), off.end(), kNoStack);
  std::fill(pw.begin(), pw.end(), kNoStack);
  std::fill(dyn.begin(), dyn.end(), 0);
  std::fill(dyns.begin(), dyns.end(), 0);
  any_pw = any_dyn = false;
  lo = 0, hi = INT64_MIN;
  for (uint32_t i = 0; i < n; i++) {
    if (!in[i].reached) continue;
    const Uop& u = uops[i];
    Regs st = in[i];
    const bool src = u.aux & F_SRC;
    const Val S = st.r[u.src], D = st.r[u.dst];
    if (u.op == U_ST || u.op == U_STX || u.op == U_ATOMIC) {
      const int64_t w = u.op == U_ATOMIC ? 8 : u.aux;  // (an atomic reads and writes 8 bytes)
      if (D.k == CONST && u.op != U_ATOMIC) {  // into the packet's header window (r1 = 0)
        const int64_t c = D.v + (int64_t)u.x;
        if (c < 0 || c + w > (int64_t)kWin) return res;
        pw[i] = (int32_t)c;
        any_pw = true;
      } else if (D.k == TOP && u.op != U_ATOMIC) {  // through a packet pointer: store mode
        dyns[i] = 1;
        any_dyn = true;
      } else {
        if (D.k != FP) return res;
        const int64_t d = D.v + (int64_t)u.x;
        if (d < -(int64_t)kStackMax || d + w > 0) return res;
        if (u.op == U_ATOMIC && (d & 3)) return res;
        off[i] = (int32_t)d;
        lo = std::min(lo, d);
        hi = std::max(hi, d + w);
      }
    }
    if (u.op == U_LDX) {
      if (S.k == FP) off[i] = (int32_t)std::max<int64_t>(INT32_MIN + 1, std::min<int64_t>(INT32_MAX, S.v + u.x));
      else if (S.k != CONST) dyn[i] = 1;
    }
    switch (u.op) {
      case U_JA: case U_JEQ: case U_JGT: case U_JGE: case U_JSET: case U_JNE: case U_JLT:
      case U_JLE: case U_JEQ32: case U_JGT32: case U_JGE32: case U_JSET32: case U_JNE32:
      case U_JLT32: case U_JLE32:
        flow((uint32_t)u.x, st);
        if (u.op != U_JA) flow(i + 1, st);
        continue;
      case U_EXIT: case U_FAULT:
        continue;
      case U_ST: case U_STX: case U_NOP:
        break;  // the destination register keeps its value (emu.rs:443)
      case U_ATOMIC:  // fetch: src = the old value; CMPXCHG: r0 = it; dst restored (Q14)
        if (u.aux & F_FETCH) st.r[u.src] = Val{TOP, 0};
        if (u.k == 0xf0) st.r[0] = Val{TOP, 0};
        st.r[u.dst] = D;
        break;
      case U_MOV64: st.r[u.dst] = src ? S : Val{CONST, u.k}; break;
      case U_LDIMM: st.r[u.dst] = Val{CONST, u.k}; break;
      case U_ADD64: case U_SUB64: {
        const Val B = src ? S : Val{CONST, u.k};
        const bool sub = u.op == U_SUB64;
        Val r{TOP, 0};
        if (B.k == CONST && (D.k == CONST || D.k == FP))
          r = Val{D.k, (int64_t)((uint64_t)D.v + (sub ? 0 - (uint64_t)B.v : (uint64_t)B.v))};
        else if (!sub && D.k == CONST && B.k == FP)
          r = Val{FP, (int64_t)((uint64_t)D.v + (uint64_t)B.v)};
        st.r[u.dst] = r;
        break;
      }
      default: st.r[u.dst] = Val{TOP, 0}; break;
    }
    flow(i + 1, st);
  }
  if (!changed || !loops) break;
  if (pass > 4 * (int)n + 16) return res;
  }
  // (loop programs run on the loop kernel, whose loads are not constant-folded: no packet-window
  // stores there)
  if (loops && (any_pw || any_dyn)) return res;
  // store mode (register-address stores): the header window lives in LDS, where every packet
  // load reads it; a constant-address load straddling the window's end would read its low bytes
  // from HBM (register-address ones deoptimize their lane at run time)
  if (any_dyn)
    for (uint32_t i = 0; i < n; i++) {
      const Uop& u = uops[i];
      if (u.op != U_LDX || !in[i].reached || off[i] != kNoStack || dyn[i]) continue;
      const Val S = in[i].r[u.src];
      if (S.k != CONST) continue;
      const int64_t a = S.v + (int64_t)u.x;
      if (a < (int64_t)kWin && a + u.aux > (int64_t)kWin) return res;
    }
  // packet-window stores: every load must be a constant-address one (fold_const_loads reads the
  // stored bytes from the window registers) or a stack-window one, none straddling the window's
  // end (its bytes below kWin would come from HBM)
  if (any_pw && !any_dyn)
    for (uint32_t i = 0; i < n; i++) {
      const Uop& u = uops[i];
      if (u.op != U_LDX || !in[i].reached || off[i] != kNoStack) continue;
      const Val S = in[i].r[u.src];
      const int64_t a = S.v + (int64_t)u.x;
      if (dyn[i] || S.k != CONST || (a < (int64_t)kWin && a + u.aux > (int64_t)kWin)) return res;
    }
  // (a plan with packet-window stores only keeps a 4-byte stack window)
  const uint32_t k = std::max<uint32_t>((uint32_t)((-lo + 3) & ~3), any_pw || any_dyn ? 4u : 0u);
  if (hi > 0 || k == 0 || k > kStackMax) return res;
  for (uint32_t i = 0; i < n; i++) {
    const Uop& u = uops[i];
    if (u.op != U_LDX || off[i] == kNoStack) continue;
    const int64_t d = off[i];
    if (d >= -(int64_t)k && d + u.aux <= 0) continue;       // inside the window
    if (d + u.aux <= -(int64_t)k || d >= 0) {                 // disjoint: an ordinary load at a
      if (any_pw && !any_dyn) return res;                     // uniform address, checked at run
      off[i] = kNoStack;                                      // time like any other (not with
      continue;                                               // packet stores: LDS is stale)
    }
    return res;                                               // straddles the window's edge
  }
  res.plan.k = k;
  res.plan.off = std::move(off);
  res.plan.pw = std::move(pw);
  res.plan.any_pw = any_pw;
  res.plan.dyn = std::move(dyns);
  res.plan.any_dyn = any_dyn;
  // (store mode: whether the deopt pass can be left out for main.rs-layout batches, jit.cpp)
  res.plan.no_deopt = any_dyn && store_mode_no_deopt(uops, res.plan, nullptr, &res.plan.kld,
                                                     &res.plan.st_bound, &res.plan.len_bound);
  return res;
}

// Stack-slot promotion: a stack-window loop program (analyze_stack's plan, no packet stores, no
// atomics) whose window accesses are all whole 8-byte slots -- a spilled accumulator, as
// compiled C keeps one (`ldxdw rT, [r10-8]; add rT, rD; stxdw [r10-8], rT`) -- becomes a tier-0
// loop program with each slot in a register the program never names: `stdw [slot], imm` ->
// `lddw rS, imm`, `stxdw [slot], rX` -> `mov rS, rX`, `ldxdw rX, [slot]` -> `mov rX, rS`. One
// micro-op each, so steps, faults and budgets are the reference's (emu.rs:354-372 on a slot the
// loads then read back, emu.rs:341-349). The accumulator triple `mov rT, rS; add rT, rD;
// mov rS, rT` with rT dead after it becomes `nop; add rS, rD; nop` (the loop kernel's byte-sum
// idiom then applies, jit.cpp counted_group). It is exact for the lanes whose packet loads
// cannot read the slots' bytes (the slots start as the image's zeros and only the slots hold the
// stores): the compiled code requires every packet load proven inside the packet (jit.cpp
// all_loads_proven) and deoptimizes lanes with LEN > r10 - k (promo_guard); the final registers
// and image differ (the slot registers, the slots' bytes), so batches that ask for them, or set
// init_regs, run the stack loop kernel instead (promo_ok). Returns false if not applicable.
static bool promote_slots(const std::vector<Uop>& xu, const StackPlan& plan, std::vector<Uop>& out) {
  const uint32_t n = (uint32_t)xu.size();
  if (!plan.k || plan.any_pw || plan.any_dyn || plan.off.size() != n) return false;
  std::vector<int32_t> slots;
  uint32_t used = 1u << 2 | 1u << 10 | 1u;  // r2 = LEN and r10 never; r0 always named
  for (uint32_t i = 0; i < n; i++) {
    const Uop& u = xu[i];
    used |= 1u << (u.dst & 15) | 1u << (u.src & 15);
    if (u.op == U_ATOMIC || u.op == U_CALL) return false;
    const bool acc = u.op == U_ST || u.op == U_STX || (u.op == U_LDX && plan.off[i] != kNoStack);
    if (!acc) continue;
    if (plan.off[i] == kNoStack || u.aux != 8) return false;
    if (std::find(slots.begin(), slots.end(), plan.off[i]) == slots.end()) slots.push_back(plan.off[i]);
  }
  std::sort(slots.begin(), slots.end());
  for (size_t j = 1; j < slots.size(); j++)
    if (slots[j] - slots[j - 1] < 8) return false;  // (partly overlapping slots)
  std::vector<uint8_t> reg(slots.size());
  uint32_t r = 9;
  for (size_t j = 0; j < slots.size(); j++) {
    while (r >= 1 && ((used >> r) & 1)) r--;
    if (r < 1) return false;  // no free register left
    reg[j] = (uint8_t)r--;
  }
  auto slot_reg = [&](int32_t off) {
    return reg[std::find(slots.begin(), slots.end(), off) - slots.begin()];
  };
  out = xu;
  for (uint32_t i = 0; i < n; i++) {
    const Uop& u = xu[i];
    const bool acc = u.op == U_ST || u.op == U_STX || (u.op == U_LDX && plan.off[i] != kNoStack);
    if (!acc) continue;
    Uop v{};
    if (u.op == U_ST) {
      v.op = U_LDIMM, v.dst = slot_reg(plan.off[i]), v.k = u.k;
    } else if (u.op == U_STX) {
      v.op = U_MOV64, v.dst = slot_reg(plan.off[i]), v.src = u.src, v.aux = F_SRC;
    } else {
      v.op = U_MOV64, v.dst = u.dst, v.src = slot_reg(plan.off[i]), v.aux = F_SRC;
    }
    out[i] = v;
  }
  // the accumulator triple, inside one basic block, rT dead after it
  std::vector<char> tgt(n + 1, 0);
  for (uint32_t i = 0; i < n; i++)
    if (out[i].op >= U_JA && out[i].op <= U_JLE32 && (uint32_t)out[i].x <= n) tgt[(uint32_t)out[i].x] = 1;
  // liveness of r0..r10 (r0 live at exits and faults; conservative for calls: none here)
  std::vector<uint32_t> lin(n + 1, 0);
  lin[n] = 1u;
  auto rw = [&](const Uop& u, uint32_t& rd, uint32_t& wr) {
    const uint32_t d = 1u << u.dst, sr = (u.aux & F_SRC) ? 1u << u.src : 0u;
    rd = wr = 0;
    if (u.op <= U_ARSH32) { wr = d; rd = sr | ((u.op == U_MOV64 || u.op == U_MOV32) ? 0u : d); }
    else if (u.op <= U_BSWAP64) { rd = wr = d; }
    else if (u.op >= U_JA && u.op <= U_JLE32) { rd = u.op == U_JA ? 0u : (d | sr); }
    else if (u.op == U_LDIMM) { wr = d; }
    else if (u.op == U_LDX) { rd = d | (1u << u.src); wr = d; }
    else if (u.op == U_EXIT || u.op == U_FAULT) { rd = 1u; }
    else { rd = 0x7ffu; }  // (anything else: everything live)
  };
  for (bool ch = true; ch;) {
    ch = false;
    for (uint32_t i = n; i-- > 0;) {
      const Uop& u = out[i];
      uint32_t rd, wr, o = 0;
      rw(u, rd, wr);
      if (u.op == U_EXIT || u.op == U_FAULT) o = 0;
      else if (u.op >= U_JA && u.op <= U_JLE32) {
        o = lin[std::min<uint32_t>((uint32_t)u.x, n)];
        if (u.op != U_JA) o |= lin[i + 1];
      } else o = lin[i + 1];
      const uint32_t v = rd | (o & ~wr);
      if (v != lin[i]) lin[i] = v, ch = true;
    }
  }
  for (uint32_t i = 0; i + 2 < n; i++) {
    const Uop &a = out[i], &b = out[i + 1], &c = out[i + 2];
    if (a.op != U_MOV64 || !(a.aux & F_SRC) || b.op != U_ADD64 || !(b.aux & F_SRC) ||
        c.op != U_MOV64 || !(c.aux & F_SRC))
      continue;
    const uint32_t rT = a.dst, rS = a.src, rD = b.src;
    if (std::find(reg.begin(), reg.end(), (uint8_t)rS) == reg.end() || rT == rS || b.dst != rT ||
        rD == rT || rD == rS || c.dst != rS || c.src != rT || tgt[i + 1] || tgt[i + 2] ||
        ((lin[i + 3] >> rT) & 1))
      continue;
    Uop nop{};
    nop.op = U_NOP, nop.dst = (uint8_t)rS;
    Uop add = b;
    add.dst = (uint8_t)rS;
    out[i] = nop, out[i + 1] = add, out[i + 2] = nop;
    i += 2;
  }
  return true;
}

extern "C" {

void ebpf_batch_init(ebpf_batch* b) {
  if (!b) return;
  std::memset(b, 0, sizeof *b);
  b->mem_size = EBPF_DEFAULT_MEM;
  b->r10 = EBPF_DEFAULT_R10;
  b->max_steps = EBPF_DEFAULT_STEPS;
}

int ebpf_prog_load(const uint8_t* code, size_t nbytes, ebpf_prog** out, size_t* bad_word) {
  if (!out || (!code && nbytes)) return EBPF_EINVAL;
  *out = nullptr;
  std::vector<RefInsn> insns;
  int rc = decode_image(code, nbytes, insns, bad_word);
  if (rc) return rc;
  if (insns.size() > EBPF_MAX_INSNS) return EBPF_ETOOBIG;
  ebpf_prog* p = new (std::nothrow) ebpf_prog;
  if (!p) return EBPF_ENOMEM;
  p->insns = std::move(insns);
  p->uops.reserve(p->insns.size());
  for (size_t i = 0; i < p->insns.size(); i++) {
    Uop u = lower(p->insns[i], (uint32_t)i);
    if (u.op == U_FAULT) { u.dst = 0; u.src = 0; }  // the kernel never indexes a bad register
    if (u.op == U_ST || u.op == U_STX || u.op == U_ATOMIC || u.op == U_CALL) p->tier = 1;
    p->uops.push_back(u);
  }
  // CALL / EXIT: the frame stacks as program copies (flatten_calls) for every kernel but the
  // general interpreter, unless the program does not flatten
  p->xuops = p->uops;
  if (std::any_of(p->uops.begin(), p->uops.end(), [](const Uop& u) { return u.op == U_CALL; })) {
    std::vector<Uop> f;
    if (flatten_calls(p->uops, f)) {
      p->xuops = std::move(f);
      p->flattened = true;
    }
  }
  if (p->xuops.size() + 2 <= kJitMaxUops) peel_invariant_loads(p->xuops);
  const std::vector<Uop>& xu = p->xuops;
  for (const Uop& u : xu)
    if (u.op == U_ST || u.op == U_STX || u.op == U_ATOMIC || u.op == U_CALL) p->xtier = 1;
  bool forward = true;  // no back edge: every lane's pc only grows (a DAG)
  for (size_t i = 0; i < xu.size(); i++) {
    const Uop& u = xu[i];
    if (u.op >= U_JA && u.op <= U_CALL && (uint32_t)u.x <= (uint32_t)i) forward = false;
  }
  p->tiny = forward && xu.size() <= kTinyUops;
  // (past kMaxDagUops the tables serve the compiler only: batch_kind)
  if (forward && p->xtier == 0 && !xu.empty() && xu.size() <= kJitMaxUops) {
    p->duops = build_dag(xu);
    p->duopsk = fold_const_loads(xu, p->duops);
    if (xu.size() <= kJitMaxUops) {  // tile_kernel's (<= 62) and the compiler's tables
      p->tuops = build_tile(xu, p->duops);
      p->tuopsk = build_tile(xu, p->duopsk);
      std::vector<TUop> tx = build_tile(xu, fold_const_loads(xu, p->duops, true));
      if (tx.size() != p->tuopsk.size() ||
          std::memcmp(tx.data(), p->tuopsk.data(), tx.size() * sizeof(TUop)) != 0)
        p->tuopsk_xdp = std::move(tx);
    }
  }
  // (past kTileMaxUops: tables for the compiled loop program only, batch_kind)
  if (p->xtier == 0 && !xu.empty() && xu.size() <= kJitMaxUops) {
    const std::vector<DUop> d = p->duops.empty() ? build_dag(xu) : p->duops;
    p->ltuops = build_tile(xu, d);
    p->ltuopsx = build_tile(xu, d, true);
  }
  if (p->xtier == 1) {  // memory tier 0.5: the compiled fixed-slot kernel only
    StackAnalysis sa = analyze_stack(xu);
    const std::vector<DUop> dk =
        sa.plan.k && forward ? fold_const_loads(xu, build_dag(xu)) : std::vector<DUop>();
    // packet-window stores: every load outside the stack window must be a constant-address one
    // (read from the window registers the stores update)
    for (size_t i = 0; sa.plan.k && sa.plan.any_pw && !sa.plan.any_dyn && forward && i < xu.size(); i++)
      if (xu[i].op == U_LDX && sa.plan.off[i] == kNoStack && (dk[i].opaux & 0xff) != U_LDXK)
        sa.plan.k = 0;
    if (sa.plan.k) {
      if (forward) {  // the forward kernels' table, constant-address loads resolved
        for (const DUop& o : dk)
          if ((o.opaux & 0xff) == U_LDXK) p->kloads.push_back({o.addr, o.opaux >> 8});
        p->tuopsk = build_tile(xu, dk, false, true);
      }
      // the loop kernel's stack variant (back edges, or a step budget that can bind; not with
      // packet-window stores, which need the forward kernels' preloaded window)
      if (!sa.plan.any_pw && !sa.plan.any_dyn) {
        const std::vector<DUop> d = build_dag(xu);
        p->ltuops = build_tile(xu, d, false, true);
        p->ltuopsx = build_tile(xu, d, true, true);
        // loops with whole-slot accumulators: also the promoted tier-0 program (variant 4)
        std::vector<Uop> pu;
        if (!forward && promote_slots(xu, sa.plan, pu)) {
          const std::vector<DUop> pd = build_dag(pu);
          p->pltuops = build_tile(pu, pd);
          p->pltuopsx = build_tile(pu, pd, true);
          p->puops = std::move(pu);
          p->pguard_k = sa.plan.k;
        }
      }
      p->stack = std::move(sa.plan);
    }
  }
  *out = p;
  return EBPF_OK;
}

int ebpf_prog_load_hex(const char* hex, ebpf_prog** out, size_t* bad_word) {
  std::vector<uint8_t> image;
  int rc = parse_hex_u64s(hex, image);
  if (rc) {
    if (bad_word) *bad_word = 0;
    return rc;
  }
  return ebpf_prog_load(image.data(), image.size(), out, bad_word);
}

void ebpf_prog_free(ebpf_prog* p) {
  if (!p) return;
  int cur = device_of_current();
  for (int d = 0; d < kMaxDevices; d++) {
    if (p->dev_uops[d] || p->dev_duops[d]) {
      hipSetDevice(d);
      if (p->dev_uops[d]) hipFree(p->dev_uops[d]);
      if (p->dev_duops[d]) hipFree(p->dev_duops[d]);
      if (p->dev_duopsk[d]) hipFree(p->dev_duopsk[d]);
      if (p->dev_tuops[d]) hipFree(p->dev_tuops[d]);
      if (p->dev_tuopsk[d]) hipFree(p->dev_tuopsk[d]);
      if (p->dev_ltuops[d]) hipFree(p->dev_ltuops[d]);
      if (p->dev_ltuopsx[d]) hipFree(p->dev_ltuopsx[d]);
      if (p->dev_pltuops[d]) hipFree(p->dev_pltuops[d]);
      if (p->dev_pltuopsx[d]) hipFree(p->dev_pltuopsx[d]);
    }
    for (int v = 0; v < kJitVariants; v++)
      if (p->jit_mod[d][v]) {
        hipSetDevice(d);
        (void)hipModuleUnload(p->jit_mod[d][v]);
      }
  }
  hipSetDevice(cur);
  delete p;
}

size_t ebpf_prog_len(const ebpf_prog* p) { return p ? p->insns.size() : 0; }

int ebpf_prog_insn(const ebpf_prog* p, size_t i, int32_t* imm, int64_t* imm64, int16_t* off,
                   uint8_t* src, uint8_t* dst, uint8_t* code) {
  if (!p || i >= p->insns.size()) return EBPF_EINVAL;
  const RefInsn& r = p->insns[i];
  if (imm) *imm = r.imm;
  if (imm64) *imm64 = r.imm64;
  if (off) *off = r.off;
  if (src) *src = r.src;
  if (dst) *dst = r.dst;
  if (code) *code = r.code;
  return EBPF_OK;
}

int ebpf_prog_tier(const ebpf_prog* p) { return p ? p->tier : -1; }

static_assert(kJitMaxUops == EBPF_MAX_COMPILED_UOPS, "include/ebpf_emu.h names the compiler's limit");
int ebpf_prog_forward_only(const ebpf_prog* p) {
  if (!p) return -1;
  if (p->duops.empty()) return 0;
  if (p->uops.size() <= (size_t)kMaxDagUops) return 1;
  // past dag_kernel's table only the compiled forward kernels run it (batch_kind dag_ok): 1 only
  // when they compiled (a compiler failure leaves every batch on the general interpreter)
  ebpf_prog* q = const_cast<ebpf_prog*>(p);
  std::lock_guard<std::mutex> lk(q->mu);
  (void)jit_compile_locked(q);
  return q->jit_state == 1 && (q->jit_has[0] || q->jit_has[1]) ? 1 : 0;
}

int ebpf_prog_stack_window(const ebpf_prog* p) { return p ? (int)p->stack.k : -1; }

int ebpf_prog_store_mode(const ebpf_prog* p) {
  if (!p) return -1;
  return !p->stack.any_dyn ? 0 : p->stack.no_deopt ? 2 : 1;
}

int ebpf_prog_compile(ebpf_prog* p) {
  if (!p) return EBPF_EINVAL;
  std::lock_guard<std::mutex> lk(p->mu);
  return jit_compile_locked(p);
}

int ebpf_prog_jit_asm(ebpf_prog* p, int variant, char* buf, size_t cap, size_t* len) {
  if (!p || variant < 0 || variant >= kJitVariants) return EBPF_EINVAL;
  std::lock_guard<std::mutex> lk(p->mu);
  if (jit_compile_locked(p) != 1 || !p->jit_has[variant]) return EBPF_EINVAL;
  const std::string& a = p->jit_asm[variant];
  if (len) *len = a.size();
  if (buf && cap) {
    const size_t k = std::min(cap - 1, a.size());
    std::memcpy(buf, a.data(), k);
    buf[k] = 0;
  }
  return EBPF_OK;
}

int ebpf_prog_jit_error(ebpf_prog* p, char* buf, size_t cap, size_t* len) {
  if (!p) return EBPF_EINVAL;
  std::lock_guard<std::mutex> lk(p->mu);
  const int rc = jit_compile_locked(p);
  std::string m;
  if (rc < 0 || !p->jit_err.empty()) {
    m = p->jit_err.empty() ? "the compiler failed" : p->jit_err;
  } else if (rc == 0) {
    const size_t n = p->xuops.size();
    if (n > kJitMaxUops)
      m = "not compiled: " + std::to_string(n) + " micro-ops (after flattening calls) past "
          "EBPF_MAX_COMPILED_UOPS (" + std::to_string(kJitMaxUops) + ")";
    else if (p->xtier == 1)
      m = "not compiled: memory writes outside the stack window, a constant-address packet store "
          "past the header window or an atomic outside the stack (the general interpreter's tier 1)";
    else
      m = "not compiled";
  }
  if (len) *len = m.size();
  if (buf && cap) {
    const size_t k = std::min(cap - 1, m.size());
    std::memcpy(buf, m.data(), k);
    buf[k] = 0;
  }
  return EBPF_OK;
}

int ebpf_prog_upload(ebpf_prog* p, int device) {
  if (!p || device < 0 || device >= kMaxDevices) return EBPF_EINVAL;
  std::lock_guard<std::mutex> lk(p->mu);
  if (p->dev_uops[device]) return EBPF_OK;
  int cur = device_of_current();
  if (hipSetDevice(device) != hipSuccess) return EBPF_EHIP;
  const size_t bytes = std::max<size_t>(1, p->uops.size()) * sizeof(Uop);
  Uop* d = nullptr;
  int rc = EBPF_OK;
  if (hipMalloc(&d, bytes) != hipSuccess) rc = EBPF_EHIP;
  else if (!p->uops.empty() &&
           hipMemcpy(d, p->uops.data(), p->uops.size() * sizeof(Uop), hipMemcpyHostToDevice) !=
               hipSuccess)
    rc = EBPF_EHIP;
  // dag_kernel tables, each with one zeroed padding entry past the end (the kernel prefetches
  // the micro-op after each one)
  auto put = [&](const std::vector<DUop>& t, DUop** dst) {
    const size_t nb = t.size() * sizeof(DUop);
    if (rc != EBPF_OK || t.empty()) return;
    if (hipMalloc(dst, nb + sizeof(DUop)) != hipSuccess ||
        hipMemset(*dst, 0, nb + sizeof(DUop)) != hipSuccess ||
        hipMemcpy(*dst, t.data(), nb, hipMemcpyHostToDevice) != hipSuccess)
      rc = EBPF_EHIP;
  };
  auto putt = [&](const std::vector<TUop>& t, TUop** dst) {
    const size_t nb = t.size() * sizeof(TUop);
    if (rc != EBPF_OK || t.empty()) return;
    if (hipMalloc(dst, nb) != hipSuccess ||
        hipMemcpy(*dst, t.data(), nb, hipMemcpyHostToDevice) != hipSuccess)
      rc = EBPF_EHIP;
  };
  DUop* dd = nullptr;
  DUop* ddk = nullptr;
  TUop* td = nullptr;
  TUop* tdk = nullptr;
  TUop* tl = nullptr;
  TUop* tlx = nullptr;
  put(p->duops, &dd);
  put(p->duopsk, &ddk);
  putt(p->tuops, &td);
  putt(p->tuopsk, &tdk);
  putt(p->ltuops, &tl);
  putt(p->ltuopsx, &tlx);
  // the compiled program's modules on this device (a compiler failure leaves the interpreter)
  if (rc == EBPF_OK && jit_compile_locked(p) == 1) {
    for (int v = 0; v < kJitVariants && rc == EBPF_OK; v++)
      if (p->jit_has[v]) {
        if (!jit_load(p->jit_co[v], &p->jit_mod[device][v], &p->jit_fn[device][v]))
          rc = EBPF_EHIP;
        else if ((v == 2 && p->jit_deep) || (v == 4 && p->pjit_deep) ||
                 (v == 5 && p->xjit_deep) || (v == 6 && p->rjit_deep))  // (the code is in the
          p->jit_fn[device][v].loop = p->jit_fn[device][v].loop_deep;     // deep-prefetch kernel)
        // (store mode runs on the fixed-slot statement too since round 6: gen_tile.py st=1)
        p->jit_fn[device][v].var_only = false;
        if (!p->jit_occ[v]) p->jit_fn[device][v].fixed_occ = p->jit_fn[device][v].fixed_occw = nullptr;
      }
  }
  TUop* tp = nullptr;
  TUop* tpx = nullptr;
  if (rc == EBPF_OK && p->jit_has[4]) {  // (the promoted tables: known once compiled)
    putt(p->pltuops, &tp);
    putt(p->pltuopsx, &tpx);
  }
  if (rc == EBPF_OK) {
    p->dev_pltuops[device] = tp;
    p->dev_pltuopsx[device] = tpx;
    p->dev_uops[device] = d;
    p->dev_duops[device] = dd;
    p->dev_duopsk[device] = ddk;
    p->dev_tuops[device] = td;
    p->dev_tuopsk[device] = tdk;
    p->dev_ltuops[device] = tl;
    p->dev_ltuopsx[device] = tlx;
  } else {
    for (void* q : {(void*)d, (void*)dd, (void*)ddk, (void*)td, (void*)tdk, (void*)tl, (void*)tlx,
                    (void*)tp, (void*)tpx})
      if (q) hipFree(q);
  }
  hipSetDevice(cur);
  return rc;
}

// Whether a loop-mode batch runs in length-binned order (an xdp_md batch is staged as offsets +
// lens).
// deep: the loop program that runs is compiled into the deep kernel (its variant's *jit_deep flag;
// false sizes the workspace for any variant)
static bool use_binning(const ebpf_prog* p, const ebpf_batch* b, bool deep = false) {
  const bool ol = (b->offsets && b->lens) || (b->flags & EBPF_BATCH_XDP_MD);
  if (p->ltuops.empty() || !ol || (b->flags & EBPF_BATCH_GENERIC) || b->init_fp_len) return false;
  // (a program on the deep loop kernel -- its long byte sums cooperative, coop_sum_compact -- runs
  // in batch order: a tile's short packets need no binning away from its long ones, and spreading
  // the long packets over every tile balances the waves; config 5, A/B on one box: 169.7 us
  // unbinned vs 191.3 binned per 1 Mi batch)
  if (deep && g_bin < 0) return false;
  return g_bin >= 0 ? g_bin == 1 : b->n >= kBinMinPackets;
}

static uint64_t align16(uint64_t v) { return (v + 15) & ~15ull; }

// xdp_md staging region (at the end of the workspace): offsets u32[n], lengths u16[n], then the
// images, each in a 16-byte aligned slot of at most round16(min(8 + max len, mem_size)) bytes.
static uint64_t xdp_image_bytes(const ebpf_batch* b) {
  const uint64_t maxlen = b->lens ? 0xFFFFull : std::min<uint64_t>(b->stride, 0xFFFFull);
  return b->n * align16(std::min<uint64_t>(maxlen + 8, b->mem_size)) + 64;
}
static uint64_t xdp_region_bytes(const ebpf_batch* b) {
  return align16(b->n * 4) + align16(b->n * 2) + xdp_image_bytes(b);
}

// The memory tier a batch runs at: a caller-set frame stack needs the general interpreter's call
// stack (an EXIT pops it), whatever the program.
static int batch_tier(const ebpf_prog* p, const ebpf_batch* b) {
  return p->tier == 1 || b->init_fp_len ? 1 : 0;
}

// Memory tier 0.5 (analyze_stack) on this batch: the compiled fixed-slot kernel with the main.rs
// register layout, and a window [r10 - k, r10) that lies in the image, past every packet byte (so
// it starts as zeros) and away from every constant-address load; else the general interpreter.
static bool stack_common_ok(const ebpf_prog* p, const ebpf_batch* b, const ebpf_batch_out* out) {
  if (!p->stack.k) return false;
  if (b->flags & (EBPF_BATCH_GENERIC | EBPF_BATCH_NO_JIT)) return false;
  if (b->init_regs || b->init_fp_len || out->mem) return false;
  const uint64_t k = p->stack.k, r10 = b->r10;
  return r10 % 4 == 0 && r10 >= k && r10 <= b->mem_size;
}

// The stack window on the other layouts (ebpf_tile_jit_var_stack, ebpf_tile_jit_loop_stack):
// lanes whose packet reaches into it load those bytes at the start, which needs the window past
// the header window (and the xdp_md ctx).
static bool stack_var_ok(const ebpf_prog* p, const ebpf_batch* b) {
  return b->r10 - p->stack.k >= (uint64_t)kWin;
}

// Forward stack-window programs on the compiled forward kernels (fixed slots: the window must lie
// past every packet byte, so it starts as zeros; other layouts: stack_var_ok).
static bool stack_launch_ok(const ebpf_prog* p, const ebpf_batch* b, const ebpf_batch_out* out,
                            int device) {
  if (!stack_common_ok(p, b, out) || !p->jit_mod[device][1] || b->max_steps < p->xuops.size())
    return false;
  const uint64_t k = p->stack.k, r10 = b->r10;
  LaunchArgs la{};
  la.frames = b->frames;
  la.offsets = b->offsets;
  la.lens = b->lens;
  la.stride = b->stride;
  la.mem_out = out->mem;
  // (store mode runs on the var kernel whatever the layout: its window init covers any packet;
  // its header-window loads read LDS without a bounds check, so the image must cover the window)
  const bool fixed = launch_fixed_layout(la) && !p->stack.any_dyn;
  const uint64_t img_len = b->stride + ((b->flags & EBPF_BATCH_XDP_MD) ? 8 : 0);
  if (fixed ? r10 - k < img_len : !stack_var_ok(p, b)) return false;
  if (p->stack.any_dyn && b->mem_size < (uint64_t)kWin) return false;
  for (const auto& kl : p->kloads) {
    if (kl.first < r10 && kl.first + kl.second > r10 - k) return false;
    // packet-window stores: the compiled code has only the copy whose window loads read the
    // preloaded (and stored-to) registers, which runs when mem_size covers every such load
    if (p->stack.any_pw && kl.first + kl.second <= (uint64_t)kWin &&
        kl.first + kl.second > b->mem_size)
      return false;
  }
  return true;
}

// Stack-window programs with back edges (or a binding step budget) on the loop kernel's stack
// variant.
static bool stack_loop_ok(const ebpf_prog* p, const ebpf_batch* b, const ebpf_batch_out* out,
                          int device) {
  return stack_common_ok(p, b, out) && p->jit_mod[device][2] && stack_var_ok(p, b);
}

// The stack-slot promoted program (variant 4, promote_slots) on this batch: the production
// outputs only (verdict, r0, status, counters: the final registers and image differ) and the
// main.rs layout; the window's launch checks of the stack kernels (stack_common_ok).
static bool promo_ok(const ebpf_prog* p, const ebpf_batch* b, const ebpf_batch_out* out,
                     int device) {
  if (p->puops.empty() || !p->jit_mod[device][4] || !p->dev_pltuops[device]) return false;
  if (!stack_common_ok(p, b, out) || out->regs || out->fp || out->fp_len) return false;
  return true;
}

// The kernel kind of a batch (uploaded program): dag_kernel needs no step budget (a lane of a
// forward-only program retires <= n_uops steps); the tile kernel in loop mode runs loops, or a
// step budget that can bind (exact budget); a stack-window batch runs the compiled stack kernels
// (forward, or the loop kernel's) or the general interpreter.
static int batch_kind(const ebpf_prog* p, const ebpf_batch* b, const ebpf_batch_out* out,
                      int device, bool* stk) {
  // (the final frame stacks of a flattened program are its copies' stacks: the general
  // interpreter's frame stack writes them)
  const bool generic = (b->flags & EBPF_BATCH_GENERIC) || b->init_fp_len ||
                       (p->flattened && (out->fp || out->fp_len));
  *stk = false;
  if (p->stack.k && !generic) {
    if (stack_launch_ok(p, b, out, device)) return *stk = true, kKindDag;
    if (promo_ok(p, b, out, device)) return kKindLoop;  // (stk false: the promoted program)
    if (stack_loop_ok(p, b, out, device)) return *stk = true, kKindLoop;
    return batch_tier(p, b);
  }
  // (a forward program past dag_kernel's kMaxDagUops runs only compiled)
  const bool dag_ok = p->xuops.size() <= kMaxDagUops ||
                      (p->jit_mod[device][0] && !(b->flags & EBPF_BATCH_NO_JIT));
  return (p->dev_duops[device] && b->max_steps >= p->xuops.size() && !generic && dag_ok) ? kKindDag
         : (p->dev_ltuops[device] && !generic && !p->stack.k && p->xtier == 0 &&
            (p->xuops.size() <= kTileMaxUops ||  // tile_kernel's loop mode, or compiled only
             (p->jit_mod[device][2] && !(b->flags & EBPF_BATCH_NO_JIT))))          ? kKindLoop
                                                                         : batch_tier(p, b);
}

// The compiled program, where it applies (tile-kernel programs; same tables, same results).
static const JitFns* batch_jit(ebpf_prog* p, const ebpf_batch* b, int kind, bool stk, int device) {
  if (stk) return &p->jit_fn[device][kind == kKindLoop ? 2 : 1];
  // (batch_kind routes a stack-window program to the loop kind without the stack flag only for
  // its promoted program)
  if (kind == kKindLoop && p->stack.k) return &p->jit_fn[device][4];
  if (b->flags & EBPF_BATCH_NO_JIT) return nullptr;
  if (kind == kKindDag && p->jit_mod[device][0])
    return &p->jit_fn[device][b->init_regs ? 0
                              : (b->flags & EBPF_BATCH_XDP_MD) && p->jit_mod[device][3] ? 3 : 1];
  if (kind == kKindLoop && p->jit_mod[device][2]) return &p->jit_fn[device][2];
  return nullptr;
}

// The micro-ops a kernel kind runs: the general interpreter the decoded program's, every other
// kernel the flattened copies (flatten_calls; the same micro-ops for a program without CALL).
static uint32_t kind_uops(const ebpf_prog* p, int kind) {
  return (uint32_t)(kind == kKindTier0 || kind == kKindTier1 ? p->uops.size() : p->xuops.size());
}

// The xdp_md convention in place (no staging copy): the compiled forward kernels and the tile
// interpreter on the general layouts synthesise each packet's ctx in its window (interp.hip
// xdp_window, jit.cpp xdp_shift) and read the packet 8 bytes further on; every other kernel runs
// the images xdp_stage writes into the workspace. EBPFEMU_XDP_STAGE=1 stages always (A/B runs:
// g_xdp_stage, defined outside this extern "C" block).

static bool xdp_in_place(ebpf_prog* p, const ebpf_batch* b, bool mem_out, int device, int kind,
                         bool stk) {
  if (!(b->flags & EBPF_BATCH_XDP_MD) || g_xdp_stage) return false;
  // the general interpreter's tier 1 builds each lane's image [ctx][packet] itself (interp.hip);
  // so does its deopt pass after a store-mode launch
  if (kind == kKindTier1) return true;
  if (kind != kKindDag) return false;
  LaunchArgs a{};
  a.n_uops = kind_uops(p, kind);
  a.frames = b->frames;
  a.offsets = b->offsets;
  a.lens = b->lens;
  a.stride = b->stride;
  a.n_tiles = (b->n + 63) / 64;
  a.mem_out = mem_out ? (uint8_t*)16 : nullptr;
  a.xdp = 1;  // (the route of an xdp_md batch in place: not the occupancy variant)
  const int id = launch_kernel_id(kind, a, batch_jit(p, b, kind, stk, device), stk);
  return id == EBPF_KERNEL_JIT_FIXED || id == EBPF_KERNEL_JIT_VAR ||
         id == EBPF_KERNEL_JIT_STACK || id == EBPF_KERNEL_JIT_VAR_STACK ||
         id == EBPF_KERNEL_JIT_VARL || id == EBPF_KERNEL_JIT_VARL_STACK ||
         (id == EBPF_KERNEL_TILE && !launch_fixed_layout(a));
}

// An xdp_md batch of a loop program in place (no staging copy): variant 6, the program rebased
// (jit.cpp Compiler::xdp_rebase; compiled only when every packet load is proven past the ctx),
// runs the batch as the main.rs layout over the packets with mem_size - 8 (rebased_batch). Not
// with final images (they hold the ctx) or caller-set registers (the proofs assume r1 = the ctx).
static bool xdp_rebased(ebpf_prog* p, const ebpf_batch* b, const ebpf_batch_out* out, int device,
                        int kind, bool stk) {
  if (!(b->flags & EBPF_BATCH_XDP_MD) || g_xdp_stage || kind != kKindLoop || stk) return false;
  if (!p->jit_mod[device][6] || out->mem || b->init_regs || b->mem_size < 8) return false;
  return batch_jit(p, b, kind, stk, device) == &p->jit_fn[device][2];
}
static ebpf_batch rebased_batch(const ebpf_batch* b) {
  ebpf_batch r = *b;
  r.flags &= ~EBPF_BATCH_XDP_MD;
  r.mem_size -= 8;
  return r;
}

// The general interpreter's tier-1 grid for a batch (its wave slots' images: the workspace).
static int tier1_grid(const ebpf_prog* p, const ebpf_batch* b, int device) {
  int cur = device_of_current();
  hipSetDevice(device);
  int grid = 0;
  interp_grid(kKindTier1, (uint32_t)p->uops.size(), p->tiny, (b->n + 63) / 64, &grid);
  hipSetDevice(cur);
  return grid;
}

// The deopt pass of a store-mode batch: at most this many workgroups (the pass usually finds an
// empty list; each of its workgroups stages the program and flushes its counters)
constexpr int kDeoptMaxGrid = 256;

// Bytes of the tier-1 wave slots (workspace, from kWsSlotsOff).
static uint64_t tier1_slots_bytes(const ebpf_prog* p, const ebpf_batch* b, int device) {
  if (batch_tier(p, b) != 1) return 0;
  return (uint64_t)tier1_grid(p, b, device) * kWavesPerBlock * tier1_slot_bytes(b->mem_size);
}

uint64_t ebpf_workspace_bytes(const ebpf_prog* p, const ebpf_batch* b, int device) {
  if (!p || !b) return 0;
  const uint64_t x = (b->flags & EBPF_BATCH_XDP_MD) ? xdp_region_bytes(b) : 0;
  uint64_t bytes = kWsSlotsOff + x;
  // the binned packet order, then the per-workgroup class counts (either loop program of a
  // promoted stack program may run)
  if (use_binning(p, b))
    bytes += align16(b->n * 4 + 4ull * kBinMaxWgs * kBinClasses);
  bytes += align16(tier1_slots_bytes(p, b, device));
  if (p->stack.any_dyn || !p->puops.empty())  // the deopt list's indices (past the slots)
    bytes += align16(b->n * 4);
  if (p->stack.any_dyn)  // store mode: the overflow images (past the indices; jit.h ovf_stride)
    bytes += b->n * ovf_stride(b->mem_size) + 16;
  return bytes;  // (the xdp_md region, when present, is the last x bytes)
}

// The batch's workspace of `need` bytes on `device` (current): the caller's, or the library-owned
// one of (device, stream), grown as needed (its first kWsSlotsOff bytes zeroed on allocation).
static int batch_workspace(const ebpf_batch* b, uint64_t need, int device, hipStream_t s,
                           uint8_t** out) {
  if (b->workspace) {
    if (b->workspace_bytes < need) return EBPF_EINVAL;
    *out = (uint8_t*)b->workspace;
    return EBPF_OK;
  }
  std::lock_guard<std::mutex> lk(g_ws_mu);
  DevWorkspace& w = g_ws[{device, (void*)s}];
  if (w.bytes < need) {
    const uint64_t grow = std::max(need, 2 * w.bytes);
    void* np = nullptr;
    if (hipMalloc(&np, grow) != hipSuccess) return EBPF_ENOMEM;
    if (hipMemset(np, 0, kWsSlotsOff) != hipSuccess) {  // shards start at zero
      hipFree(np);
      return EBPF_EHIP;
    }
    if (w.ptr) w.retired.push_back(w.ptr);
    w.ptr = np;
    w.bytes = grow;
  }
  *out = (uint8_t*)w.ptr;
  return EBPF_OK;
}

static int check_batch(const ebpf_batch* b) {
  if (!b) return EBPF_EINVAL;
  if (b->mem_size > (1u << 24)) return EBPF_EINVAL;
  if (b->init_fp_len > EBPF_MAX_CALL_DEPTH || (b->init_fp_len && !b->init_fp)) return EBPF_EINVAL;
  if (b->max_steps == 0) return EBPF_EINVAL;
  if (b->n && !b->frames) return EBPF_EINVAL;
  if (!b->offsets && b->stride == 0 && !b->lens) return EBPF_EINVAL;
  if (b->flags & ~(EBPF_BATCH_GENERIC | EBPF_BATCH_XDP_MD | EBPF_BATCH_NO_JIT)) return EBPF_EINVAL;
  if ((b->flags & EBPF_BATCH_XDP_MD) &&
      (b->mem_size > 65528 || xdp_image_bytes(b) > 0xFFFFFFFFull))
    return EBPF_EINVAL;  // 8 + len must fit the u16 lengths; staged offsets are u32
  return EBPF_OK;
}

int ebpf_run_batch(ebpf_prog* p, const ebpf_batch* bin, const ebpf_batch_out* out,
                   ebpf_stream_t stream) {
  if (!p || !out) return EBPF_EINVAL;
  int rc = check_batch(bin);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  int device = 0;
  if (s) {
    if (hipStreamGetDevice(s, &device) != hipSuccess) return EBPF_EHIP;
  } else {
    device = device_of_current();
  }
  if (bin->n == 0) return EBPF_OK;
  ebpf_batch staged = *bin;  // an xdp_md batch runs as the staged offsets + lens batch
  const ebpf_batch* b = bin;
  rc = ebpf_prog_upload(p, device);
  if (rc) return rc;
  int cur = device_of_current();
  if (cur != device) hipSetDevice(device);

  const uint64_t n_tiles = (b->n + 63) / 64;
  bool stk = false;
  const int kind = batch_kind(p, b, out, device, &stk);
  int grid = 0;
  if (interp_grid(kind, kind_uops(p, kind), p->tiny, n_tiles, &grid) != 0) {
    if (cur != device) hipSetDevice(cur);
    return EBPF_EHIP;
  }
  const bool xdp_direct = xdp_in_place(p, bin, out->mem != nullptr, device, kind, stk);
  const bool xdp_rb = !xdp_direct && xdp_rebased(p, bin, out, device, kind, stk);
  if (xdp_rb) {  // (the batch run as the main.rs layout: no staging region)
    staged = rebased_batch(bin);
    b = &staged;
  }
  // scratch: caller-provided or library-owned per (device, stream)
  const uint64_t need = ebpf_workspace_bytes(p, b, device);
  uint8_t* ws = nullptr;
  rc = batch_workspace(bin, need, device, s, &ws);
  if (rc) {
    if (cur != device) hipSetDevice(cur);
    return rc;
  }
  if ((bin->flags & EBPF_BATCH_XDP_MD) && !xdp_direct && !xdp_rb) {
    uint8_t* x = ws + need - xdp_region_bytes(bin);
    uint32_t* doffs = (uint32_t*)x;
    uint16_t* dlens = (uint16_t*)(x + align16(bin->n * 4));
    uint8_t* dst = x + align16(bin->n * 4) + align16(bin->n * 2);
    unsigned long long* cursor = (unsigned long long*)(ws + kWsXdpCursorOff);
    if (hipMemsetAsync(cursor, 0, 8, s) != hipSuccess ||
        launch_xdp_stage(bin->frames, bin->offsets, bin->lens, bin->stride, bin->n, bin->mem_size,
                         dst, doffs, dlens, cursor, s) != hipSuccess) {
      if (cur != device) hipSetDevice(cur);
      return EBPF_EHIP;
    }
    staged.frames = dst;
    staged.offsets = doffs;
    staged.lens = dlens;
    staged.stride = 0;
    staged.flags &= ~EBPF_BATCH_XDP_MD;
    b = &staged;
  }
  LaunchArgs a{};
  a.prog = p->dev_uops[device];
  // constant-address loads are resolved for the main.rs register layout only
  a.dprog = b->init_regs ? p->dev_duops[device] : p->dev_duopsk[device];
  // (the stack-slot promoted program: batch_kind's loop kind without the stack flag)
  const bool promo = kind == kKindLoop && !stk && p->stack.k;
  a.tprog = promo ? p->dev_pltuops[device]
           : kind == kKindLoop ? p->dev_ltuops[device]
           : b->init_regs      ? p->dev_tuops[device] : p->dev_tuopsk[device];
  a.tprog_exact = promo ? p->dev_pltuopsx[device] : p->dev_ltuopsx[device];
  a.n_uops = kind_uops(p, kind);
  a.mem_size = b->mem_size;
  a.frames = b->frames;
  a.offsets = b->offsets;
  a.lens = b->lens;
  a.stride = b->stride;
  a.n = b->n;
  a.r10 = b->r10;
  a.max_steps = b->max_steps;
  a.verdict = out->verdict;
  a.r0 = out->r0;
  a.status = out->status;
  a.counters = out->counters;
  a.shards = (uint64_t*)(ws + kWsShardsOff);
  a.image_ws = ws + kWsSlotsOff;
  a.n_tiles = n_tiles;
  a.init_regs = b->init_regs;
  a.mem_out = out->mem;
  if (g_trace) {  // a ring of kTraceRing launches' stamps
    const size_t tb = kTraceWaves * kTraceSlots * sizeof(uint64_t);
    if (!g_trace_buf[device] && (hipMalloc(&g_trace_buf[device], tb * kTraceRing) != hipSuccess ||
                                 hipMemset(g_trace_buf[device], 0, tb * kTraceRing) != hipSuccess))
      g_trace_buf[device] = nullptr;
    // (no per-launch clearing: a memset between launches would sit in the gaps being measured;
    // every wave rewrites its slots, so only the stamps of tiles it did not run are stale)
    if (g_trace_buf[device])
      a.trace = g_trace_buf[device] + (g_trace_launch[device]++ % kTraceRing) *
                                          (kTraceWaves * kTraceSlots);
  }
  a.regs_out = out->regs;
  a.xdp = xdp_direct ? 1u : 0u;
  a.init_fp = b->init_fp;
  a.init_fp_len = b->init_fp_len;
  a.fp_out = out->fp;
  a.fp_len_out = out->fp_len;
  // only the tier-1 kernel has a frame stack; every other kernel runs programs without CALL and
  // with an empty initial stack, whose final stack is empty
  if (kind != kKindTier1 && out->fp_len && hipMemsetAsync(out->fp_len, 0, b->n, s) != hipSuccess) {
    if (cur != device) hipSetDevice(cur);
    return EBPF_EHIP;
  }
  // the compiled variant that runs: variant 4 for the promoted program, 6 for an xdp_md batch in
  // place (rebased), 5 for a staged one (its range analysis knows the staged images' ctx)
  const JitFns* jit = xdp_rb ? &p->jit_fn[device][6] : batch_jit(p, b, kind, stk, device);
  // (variant 5 compiles ctx loads through r1 as the ctx's constants: only with the main.rs
  // registers, r1 = the image start)
  if (jit == &p->jit_fn[device][2] && (bin->flags & EBPF_BATCH_XDP_MD) && !xdp_direct &&
      !b->init_regs && p->jit_mod[device][5])
    jit = &p->jit_fn[device][5];
  const bool deep = jit == &p->jit_fn[device][2]   ? p->jit_deep
                    : jit == &p->jit_fn[device][4] ? p->pjit_deep
                    : jit == &p->jit_fn[device][5] ? p->xjit_deep
                    : jit == &p->jit_fn[device][6] ? p->rjit_deep
                                                   : false;
  if (kind == kKindLoop && use_binning(p, b, deep)) {
    a.perm = (const uint32_t*)(ws + kWsSlotsOff);
    a.bin_counts = (uint32_t*)(ws + kWsBinCountsOff);
    if (launch_binning(b->lens, b->n, (uint32_t*)a.perm + b->n, (uint32_t*)a.perm, s) !=
        hipSuccess) {
      if (cur != device) hipSetDevice(cur);
      return EBPF_EHIP;
    }
  }
  // store mode (register-address packet stores, StackPlan::any_dyn): lanes the compiled kernel
  // cannot finish are listed, then re-run from the start by the general interpreter (tier 1)
  // (the promoted program: lanes whose packet reaches the slots, jit.cpp promo_guard)
  const int kid = jit ? launch_kernel_id(kind, a, jit, stk) : -1;
  const bool deopt = (stk && p->stack.any_dyn && kind == kKindDag && jit &&
                      (kid == EBPF_KERNEL_JIT_VAR_STACK || kid == EBPF_KERNEL_JIT_VARL_STACK ||
                       kid == EBPF_KERNEL_JIT_STACK)) ||
                     (promo && jit);
  // store mode on the var tile loop with no lane able to leave (StackPlan::no_deopt: the main.rs
  // registers, the stack window at or past the overflow image's end): no deopt pass
  const uint64_t s0 = b->r10 >= p->stack.k ? b->r10 - p->stack.k : 0;  // the stack window's start
  // (the longest image a lane can have: the slot of a batch without lengths, else mem_size --
  // an access bounded by LEN must end before the stack window)
  const uint64_t len_max = std::min<uint64_t>(
      b->mem_size, !b->lens && !b->offsets ? b->stride + (a.xdp ? 8 : 0) : b->mem_size);
  // (a store ending past mem_size faults before it could deoptimize: bounded by mem_size too)
  const bool pass = deopt && !((kid == EBPF_KERNEL_JIT_VARL_STACK || kid == EBPF_KERNEL_JIT_STACK) &&
                               p->stack.no_deopt &&
                               !b->init_regs &&
                               s0 >= std::min<uint64_t>(p->stack.st_bound, b->mem_size) &&
                               (!p->stack.len_bound ||
                                (b->mem_size <= kOvfEnd && s0 >= len_max)));
  if (deopt) {
    a.deopt = (uint32_t*)(ws + kWsDeoptOff);
    // (past the tier-1 slots, or the binned order and its class counts when the batch is binned)
    const uint64_t bin_bytes = a.perm ? b->n * 4 + 4ull * kBinMaxWgs * kBinClasses : 0;
    a.deopt_idx = (uint32_t*)(ws + kWsSlotsOff +
                              align16(std::max<uint64_t>(tier1_slots_bytes(p, b, device), bin_bytes)));
    if (p->stack.any_dyn) a.ovf = (uint8_t*)a.deopt_idx + align16(b->n * 4);
    if (!pass) a.deopt_pass = 2;  // (no pass follows: a lane that leaves faults EBPF_ST_JIT)
  }
  hipError_t e = launch_interp(kind, a, grid, s, jit, stk);
  if (pass && e == hipSuccess) {
    LaunchArgs d = a;
    d.deopt_pass = 1;
    d.n_uops = (uint32_t)p->uops.size();
    d.tprog = d.tprog_exact = nullptr;
    d.dprog = nullptr;
    d.xdp = a.xdp;  // (in place: tier 1 builds the ctx-prefixed images itself)
    const int g1 = std::min(tier1_grid(p, b, device), kDeoptMaxGrid);
    e = launch_interp(kKindTier1, d, g1, s, nullptr, false);
    // a failed pass leaves the list's count behind: the next batch's pass would re-run its stale
    // indices (the pass's last workgroup clears count and done)
    if (e != hipSuccess) (void)hipMemsetAsync(a.deopt, 0, 8, s);
  }
  if (cur != device) hipSetDevice(cur);
  return e == hipSuccess ? EBPF_OK : EBPF_EHIP;
}

int ebpf_batch_kernel(ebpf_prog* p, const ebpf_batch* bin, const ebpf_batch_out* out, int device) {
  if (!p || !out || device < 0 || device >= kMaxDevices) return EBPF_EINVAL;
  int rc = check_batch(bin);
  if (rc) return rc;
  rc = ebpf_prog_upload(p, device);
  if (rc) return rc;
  bool stk = false;
  const int kind = batch_kind(p, bin, out, device, &stk);
  ebpf_batch staged = *bin;  // xdp_md batches not run in place run as offsets + lens batches
  const bool rb = xdp_rebased(p, bin, out, device, kind, stk);
  if (rb) {
    staged = rebased_batch(bin);
  } else if ((bin->flags & EBPF_BATCH_XDP_MD) &&
             !xdp_in_place(p, bin, out->mem != nullptr, device, kind, stk)) {
    staged.offsets = (const uint32_t*)16;
    staged.lens = (const uint16_t*)16;
    staged.stride = 0;
    staged.flags &= ~EBPF_BATCH_XDP_MD;
  }
  LaunchArgs a{};
  a.n_uops = kind_uops(p, kind);
  a.frames = staged.frames;
  a.offsets = staged.offsets;
  a.lens = staged.lens;
  a.stride = staged.stride;
  a.mem_out = out->mem;
  a.xdp = (staged.flags & EBPF_BATCH_XDP_MD) && !rb ? 1u : 0u;  // (in place: as ebpf_run_batch)
  return launch_kernel_id(kind, a, rb ? &p->jit_fn[device][6] : batch_jit(p, &staged, kind, stk, device),
                          stk);
}

int ebpf_batch_staged(ebpf_prog* p, const ebpf_batch* bin, const ebpf_batch_out* out, int device) {
  if (!p || !out || device < 0 || device >= kMaxDevices) return EBPF_EINVAL;
  int rc = check_batch(bin);
  if (rc) return rc;
  rc = ebpf_prog_upload(p, device);
  if (rc) return rc;
  if (!(bin->flags & EBPF_BATCH_XDP_MD)) return 0;
  bool stk = false;
  const int kind = batch_kind(p, bin, out, device, &stk);
  return xdp_in_place(p, bin, out->mem != nullptr, device, kind, stk) ||
                 xdp_rebased(p, bin, out, device, kind, stk)
             ? 0
             : 1;
}

int ebpf_run_batch_multi(ebpf_prog* p, int nshards, const int* devices, const ebpf_batch* batches,
                         const ebpf_batch_out* outs, ebpf_stream_t const* streams) {
  if (!p || nshards <= 0 || nshards > kMaxDevices || !devices || !batches || !outs || !streams)
    return EBPF_EINVAL;
  for (int s = 0; s < nshards; s++) {
    // (a NULL stream is the device's null stream)
    if (!outs[s].counters || devices[s] < 0 || devices[s] >= kMaxDevices)
      return EBPF_EINVAL;
    for (int t = 0; t < s; t++)
      if (devices[t] == devices[s]) return EBPF_EINVAL;  // one communicator rank per device
  }
  int cur = device_of_current();
  // Each shard's counters go to a u64[8] in its batch's workspace (kWsMultiOff, zeroed on the
  // shard's stream), those words are all-reduced, and the global totals are then ADDED to every
  // outs[s].counters: the caller's counters accumulate, as ebpf_run_batch's do (the header's
  // contract). A failing shard leaves every caller counter untouched.
  std::vector<ebpf_batch_out> o(outs, outs + nshards);
  for (int s = 0; s < nshards; s++) {
    const int d = devices[s];
    if (hipSetDevice(d) != hipSuccess) { hipSetDevice(cur); return EBPF_EHIP; }
    int rc = check_batch(&batches[s]);
    if (!rc) rc = ebpf_prog_upload(p, d);
    uint8_t* ws = nullptr;
    if (!rc)
      rc = batch_workspace(&batches[s], ebpf_workspace_bytes(p, &batches[s], d), d,
                           (hipStream_t)streams[s], &ws);
    if (rc) { hipSetDevice(cur); return rc; }
    uint64_t* sc = (uint64_t*)(ws + kWsMultiOff);
    o[s].counters = sc;
    if (hipMemsetAsync(sc, 0, EBPF_NCOUNTERS * sizeof(uint64_t), (hipStream_t)streams[s]) != hipSuccess) {
      hipSetDevice(cur);
      return EBPF_EHIP;
    }
  }
  // per-shard launches: independent, no data-path exchange
  for (int s = 0; s < nshards; s++) {
    hipSetDevice(devices[s]);
    int rc = ebpf_run_batch(p, &batches[s], &o[s], streams[s]);
    if (rc) { hipSetDevice(cur); return rc; }
  }
  // the one exchange step: sum the counters across GPUs over RCCL / xGMI
  static std::mutex mu;
  static std::map<std::vector<int>, std::vector<ncclComm_t>> comms;
  std::vector<int> key(devices, devices + nshards);
  std::vector<ncclComm_t>* cs;
  {
    std::lock_guard<std::mutex> lk(mu);
    auto it = comms.find(key);
    if (it == comms.end()) {
      std::vector<ncclComm_t> c(nshards);
      if (ncclCommInitAll(c.data(), nshards, devices) != ncclSuccess) {
        hipSetDevice(cur);
        return EBPF_ERCCL;
      }
      it = comms.emplace(key, std::move(c)).first;
    }
    cs = &it->second;
  }
  if (ncclGroupStart() != ncclSuccess) { hipSetDevice(cur); return EBPF_ERCCL; }
  for (int s = 0; s < nshards; s++) {
    hipSetDevice(devices[s]);
    if (ncclAllReduce(o[s].counters, o[s].counters, EBPF_NCOUNTERS, ncclUint64, ncclSum, (*cs)[s],
                      (hipStream_t)streams[s]) != ncclSuccess) {
      ncclGroupEnd();
      hipSetDevice(cur);
      return EBPF_ERCCL;
    }
  }
  if (ncclGroupEnd() != ncclSuccess) { hipSetDevice(cur); return EBPF_ERCCL; }
  int rc = EBPF_OK;
  for (int s = 0; s < nshards && rc == EBPF_OK; s++) {
    hipSetDevice(devices[s]);
    if (launch_counters_add(o[s].counters, outs[s].counters, (hipStream_t)streams[s]) != hipSuccess)
      rc = EBPF_EHIP;
  }
  hipSetDevice(cur);
  return rc;
}

int ebpf_pcap_index(const uint8_t* buf, size_t nbytes, uint32_t* offsets, uint16_t* lens,
                    size_t cap, size_t* n, uint32_t* linktype) {
  if (!buf || !n || (cap && (!offsets || !lens))) return EBPF_EINVAL;
  *n = 0;
  if (nbytes < 24) return EBPF_EPCAP;
  auto rd32 = [&](size_t at, bool swap) {
    uint32_t v;
    std::memcpy(&v, buf + at, 4);
    return swap ? __builtin_bswap32(v) : v;
  };
  const uint32_t magic = rd32(0, false);
  bool swap;
  if (magic == 0xa1b2c3d4u || magic == 0xa1b23c4du) swap = false;       // micro / nanosecond
  else if (magic == 0xd4c3b2a1u || magic == 0x4d3cb2a1u) swap = true;   // written byte-swapped
  else return EBPF_EPCAP;
  if (linktype) *linktype = rd32(20, swap) & 0x0fffffffu;  // upper bits: FCS flags
  if (nbytes > 0xFFFFFFFFull) return EBPF_ETOOBIG;
  size_t at = 24, count = 0;
  int rc = EBPF_OK;
  while (at < nbytes) {
    if (nbytes - at < 16) return EBPF_EPCAP;  // truncated record header
    const uint32_t incl = rd32(at + 8, swap);
    if (incl > nbytes - at - 16) return EBPF_EPCAP;  // truncated packet data
    if (incl > 0xFFFF) return EBPF_ETOOBIG;
    if (count < cap) {
      offsets[count] = (uint32_t)(at + 16);
      lens[count] = (uint16_t)incl;
    } else if (cap) {
      rc = EBPF_EINVAL;
    }
    count++;
    at += 16 + (size_t)incl;
  }
  *n = count;
  return rc;
}

const char* ebpf_strerror(int err) {
  switch (err) {
    case EBPF_OK: return "ok";
    case EBPF_EINVAL: return "invalid argument";
    case EBPF_ELEN: return "invalid hex format for u64";  // ins.rs:67
    case EBPF_EREG: return "register index >= 12 (ins.rs:32)";
    case EBPF_EOP: return "ALU/JMP operation > 0xd (ins.rs:251,257)";
    case EBPF_EMODE: return "invalid load/store mode (ins.rs:187)";
    case EBPF_ELDDW: return "wide instruction without second word (ins.rs:112)";
    case EBPF_ELDDW_OVF: return "wide immediate overflows i64 (ins.rs:112)";
    case EBPF_EHEX: return "invalid hex digit";
    case EBPF_ENOMEM: return "out of device memory";
    case EBPF_EHIP: return "HIP runtime error";
    case EBPF_ETOOBIG: return "program too large";
    case EBPF_ERCCL: return "RCCL error";
    case EBPF_EPCAP: return "not a classic pcap capture, or a truncated record";
    default: return "unknown error";
  }
}

int ebpf_debug_trace(int device, void** dev_ptr, size_t* bytes) {
  if (device < 0 || device >= kMaxDevices || !dev_ptr || !bytes) return EBPF_EINVAL;
  *dev_ptr = g_trace_buf[device];
  *bytes = g_trace_buf[device] ? kTraceRing * kTraceWaves * kTraceSlots * sizeof(uint64_t) : 0;
  return EBPF_OK;
}

const char* ebpf_version(void) { return "ebpfemu 0.1 gfx950"; }

}  // extern "C"
