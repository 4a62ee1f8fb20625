// jit.cpp — compiles a forward-only eBPF program into gfx950 code for the tile kernel.
//
// The tile interpreter (gen_tile.py -> tile.inc) spends most of its issue slots on interpretation:
// a scalar load of every micro-op and a wait for it, the pc-set search, the jump into the handler
// slot, and s_set_gpr_idx pairs around every register access. For a program that runs on the
// tile kernel (tier 0, forward jumps only, <= 62 micro-ops, the reference's whole XDP use case),
// all of that is known at load time. This compiler emits the program as straight-line code in pc
// order, built from the very same handler bodies (gen_tile.py -> jit_tmpl.h):
//   * register operands direct (v[2r : 2r+1] for eBPF register r), no index mode;
//   * micro-op fields as inline constants where they are one, else an s_mov into the SGPR the
//     handler reads;
//   * min-pc re-convergence without a pc set: exec holds the lanes running the current block;
//     a jump parks its leaving lanes at the target (LPC = target) and every jump target's entry
//     re-admits the lanes parked there, so blocks run in pc order as the interpreter runs them
//     (forward jumps only: each block once per tile);
//   * retired steps counted per block as before (TUop::blen), faults taking back the rest.
// The code is inserted into the assembly of the template kernels (interp.hip built with
// EBPFEMU_JIT_TEMPLATE, embedded as kJitTemplateAsm: the tile kernel's C++ prologue, the
// statement's prologue and epilogue around a marker), assembled and linked in process with
// amd_comgr, and loaded with hipModuleLoadData. Results are bit-identical to the interpreter's
// (the same instruction sequences); tests/test_gpu_jit.py checks both against the oracle.
#include "jit.h"
#include "launch.h"  // (kOccWideWaves, kOccWideUops)

#include <amd_comgr/amd_comgr.h>

#include <algorithm>
#include <array>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cctype>
#include <cstring>
#include <set>
#include <map>
#include <string>
#include <vector>

#include "jit_template.h"  // build/: kJitTemplateAsm
#include "tile_ids.h"
#include "jit_tmpl.h"

namespace ebpfemu {

namespace {

constexpr uint32_t kFieldSgpr = 36;  // TUop dword d lives in s[36 + d] (gen_tile.py UB)
// far mode: an island of out-of-line code at the first block start past this many lines (a line
// is at most 12 bytes: 36 KiB and the island's own code stay well inside s_branch's reach)
constexpr size_t kIslandLines = 3000;
// far mode: a block entry's empty-exec skip past more micro-ops than this is a long jump
constexpr uint32_t kFarSkipUops = 48;
// forward programs of at least this many micro-ops get the fixed-slot kernel's occupancy variant
// (occ_wanted). 96 until late round 6; 0 since: with two streams its smaller workgroups overlap
// consecutive launches better, the 5-tuple 98 -> 106 Gpkt/s (profiles/r06_occ_short_programs.log)
constexpr uint32_t kOccMinUops = 0;
// store mode's overflow image covers image bytes [64, min(mem_size rounded up to 64, this))
// (jit.h kOvfEnd)

struct Marker {
  size_t begin = 0, end = 0;  // the marker line ";@@JIT@@" (replaced)
  size_t init_begin = 0, init_end = 0;  // ";@@JITINIT@@" of the same statement (replaced)
  std::string n;              // the statement's %= number
  std::string fixed = "0";
  std::string loops = "0";
  std::string aligned;
  std::string xdp;  // the SGPR holding LaunchArgs::xdp (the xdp_md convention in place)
  bool stack = false;  // the var kernel's statement for stack-window programs
  bool deep = false;   // the deep-prefetch loop kernel's statement
  bool occ = false;    // the fixed-slot kernel's occupancy variant (ebpf_tile_jit_fixed_occ): no
                       // preloaded window, only v[0:55] for the program's code
  bool pm = false;     // the statement gives the body s[72:79] (the pending masks, pm_assign)
  bool st = false;     // the fixed-slot statement's store mode (body_store, with ovf / tile / dm)
  std::string waves;   // the occupancy statements' waves per workgroup (8: _occ, 12: _occw)
  bool varl = false;   // the var tile loop's statement (ebpf_tile_jit_varl): the var flavour of
                       // loads with the preloaded window, as the stack statement's
  // the var tile loop's store-mode state (gen_tile.py jit_statement_varl): the SGPR pair of
  // LaunchArgs::ovf, the tile index's SGPR and the SGPR pair of the lanes' overflow-dirty mask
  std::string ovf, tile, dm;
};

bool inline_const(int64_t v) { return v >= -16 && v <= 64; }

// A jump to `label` from anywhere in the code object (s_branch reaches +-128 KiB), for far mode
// (compile_into_template): through s[60:61] (the statement's T0, dead wherever a body is entered
// or left and at every block entry) and SCC (s_add sets it). `tag` makes its label unique.
std::string long_jump(const std::string& label, const std::string& tag) {
  const std::string g = ".Lgp" + tag, d = "(" + label + "-" + g + ")";
  return "s_getpc_b64 s[60:61]\n" + g + ":\ns_add_u32 s60, s60, " + d + "&4294967295\n"
         "s_addc_u32 s61, s61, " + d + ">>32\ns_setpc_b64 s[60:61]\n";
}

std::string hex32(uint32_t v) {
  char b[16];
  snprintf(b, sizeof b, "0x%x", v);
  return b;
}

std::string vreg(uint32_t base, uint32_t a) { return "v" + std::to_string(base + a); }
std::string vpair(uint32_t base, uint32_t a, uint32_t b) {
  return "v[" + std::to_string(base + a) + ":" + std::to_string(base + b) + "]";
}

// Find the markers of the template kernels' statements.
bool find_markers(const std::string& s, std::vector<Marker>& out) {
  size_t pos = 0;
  while ((pos = s.find("; JIT N=", pos)) != std::string::npos) {
    Marker m;
    const size_t eol = s.find('\n', pos);
    const std::string line = s.substr(pos, eol - pos);
    auto field = [&](const char* key) {
      const size_t k = line.find(key);
      if (k == std::string::npos) return std::string();
      const size_t v = k + strlen(key);
      return line.substr(v, line.find(' ', v) - v);
    };
    m.n = field("N=");
    m.fixed = field("fixed=");
    m.loops = field("loops=");
    m.aligned = field("aligned=");
    m.xdp = field("xdp=");
    m.stack = field("stack=") == "1";
    m.deep = field("deep=") == "1";
    m.varl = field("varl=") == "1";
    m.occ = field("occ=") == "1";
    m.pm = field("pm=") == "1";
    m.waves = field("waves=");
    m.st = field(" st=") == "1";
    m.ovf = field("ovf=");
    m.tile = field("tile=");
    m.dm = field("dm=");
    const size_t mk = s.find(";@@JIT@@", eol);
    if (mk == std::string::npos || m.n.empty()) return false;
    const size_t ik = s.rfind(";@@JITINIT@@", pos);
    if (ik == std::string::npos || (!out.empty() && ik < out.back().end)) return false;
    m.init_begin = ik;
    m.init_end = s.find('\n', ik);
    m.begin = mk;
    m.end = s.find('\n', mk);
    out.push_back(m);
    pos = m.end;
  }
  return !out.empty();
}

// Peephole on one micro-op's code: the handlers copy a source register pair into a temporary
// first (READ_S into v[24:25], READ_A into v[54:55]) because the interpreter indexes it; compiled,
// the instructions can read the register itself. Done when no instruction of the micro-op writes
// the source pair or the temporary after the copy (so both hold the same value throughout).
std::string dest_of(const std::string& line) {
  const size_t sp = line.find(' ');
  if (sp == std::string::npos || line.compare(0, 2, "v_") != 0 || line.compare(0, 5, "v_cmp") == 0)
    return "";
  const size_t c = line.find(',', sp);
  return line.substr(sp + 1, (c == std::string::npos ? line.size() : c) - sp - 1);
}

bool reg_overlap(const std::string& op, uint32_t lo, uint32_t hi) {
  uint32_t a, b;
  if (sscanf(op.c_str(), "v[%u:%u]", &a, &b) == 2) return !(b < lo || a > hi);
  if (sscanf(op.c_str(), "v%u", &a) == 1) return a >= lo && a <= hi;
  return false;
}

void replace_token(std::string& s, const std::string& from, const std::string& to) {
  size_t q = 0;
  while ((q = s.find(from, q)) != std::string::npos) {
    const bool left_ok = q == 0 || !(isalnum((unsigned char)s[q - 1]) || s[q - 1] == '_');
    const size_t e = q + from.size();
    const bool right_ok = e >= s.size() || !(isalnum((unsigned char)s[e]) || s[e] == '_');
    if (left_ok && right_ok) {
      s.replace(q, from.size(), to);
      q += to.size();
    } else {
      q = e;
    }
  }
}

// Resolve the assembler conditionals of an expanded handler (".if 1", ".if 0 == 0", ...; the
// statement's %[fixed] / %[loops] are known here), so only the live branch is emitted (and the
// peepholes see straight-line code). Text with any other condition is returned unchanged.
std::string resolve_ifs(const std::string& text) {
  std::string out;
  std::vector<std::pair<bool, bool>> st;  // (this branch active, enclosing active)
  size_t p = 0;
  while (p < text.size()) {
    size_t e = text.find('\n', p);
    if (e == std::string::npos) e = text.size();
    const std::string ln = text.substr(p, e - p);
    p = e + 1;
    const bool live = st.empty() || (st.back().first && st.back().second);
    if (ln.compare(0, 4, ".if ") == 0) {
      long a = 0, b = 0;
      char op[3] = {0};
      bool v;
      if (sscanf(ln.c_str() + 4, "%ld %2s %ld", &a, op, &b) == 3 && std::string(op) == "==")
        v = a == b;
      else if (sscanf(ln.c_str() + 4, "%ld", &a) == 1 && ln.find_first_not_of("0123456789 ", 4) == std::string::npos)
        v = a != 0;
      else
        return text;
      st.push_back({v, live});
      continue;
    }
    if (ln == ".else") {
      if (st.empty()) return text;
      st.back().first = !st.back().first;
      continue;
    }
    if (ln == ".endif") {
      if (st.empty()) return text;
      st.pop_back();
      continue;
    }
    if (live) out += ln + "\n";
  }
  return st.empty() ? out : text;
}

std::string fold_copy(const std::string& text, uint32_t tmp) {
  std::vector<std::string> lines;
  size_t p = 0;
  while (p < text.size()) {
    size_t e = text.find('\n', p);
    if (e == std::string::npos) e = text.size();
    lines.push_back(text.substr(p, e - p));
    p = e + 1;
  }
  const std::string tpair = "v[" + std::to_string(tmp) + ":" + std::to_string(tmp + 1) + "]";
  const std::string head = "v_mov_b64 " + tpair + ", ";
  size_t l0 = lines.size();
  for (size_t i = 0; i < lines.size(); i++)
    if (lines[i].compare(0, head.size(), head) == 0) {
      l0 = i;
      break;
    }
  if (l0 == lines.size()) return text;
  uint32_t a, b;
  if (sscanf(lines[l0].c_str() + head.size(), "v[%u:%u]", &a, &b) != 2 || b != a + 1) return text;
  for (size_t i = l0 + 1; i < lines.size(); i++) {
    const std::string d = dest_of(lines[i]);
    if (reg_overlap(d, a, b) || reg_overlap(d, tmp, tmp + 1)) return text;
    if (lines[i].compare(0, 4, "s_se") == 0) return text;  // (no index mode here, but be safe)
  }
  std::string out;
  for (size_t i = 0; i < lines.size(); i++) {
    if (i == l0) continue;
    std::string ln = lines[i];
    if (i > l0) {
      replace_token(ln, tpair, "v[" + std::to_string(a) + ":" + std::to_string(b) + "]");
      replace_token(ln, "v" + std::to_string(tmp), "v" + std::to_string(a));
      replace_token(ln, "v" + std::to_string(tmp + 1), "v" + std::to_string(b));
    }
    out += ln + "\n";
  }
  return out;
}

struct Compiler {
  const std::vector<Uop>& uops;
  const std::vector<TUop>& t;
  uint32_t n;
  // loops: a loop program (ebpf_tile_jit_loop): back edges, the step budget checked at every
  // block entry; exact: the one-micro-op-per-block copy of the exact step budget
  bool loops = false, exact = false;
  std::vector<char> start, target;
  std::string err;

  static bool is_jump(const Uop& o) { return o.op >= U_JA && o.op <= U_JLE32; }

  const StackPlan* stk = nullptr;  // a stack-window program (memory tier 0.5)
  // loop programs: the qword cache's v[50:55] named by other compiled code (compiled again
  // without the cache)
  bool cache_conflict = false;
  bool zwin = false;  // zero-past-len windows (ldx1_zero_window)
  bool qcache = false;  // with the 8-byte per-lane cache (ldx1_qword_cache)
  bool prefetch = false;  // zwin refills take the prefetched next window (refill_prefetch)
  bool deep_regs = false;  // compiled for ebpf_tile_jit_loop_deep: v[72:105] are the program's
  uint32_t guard_k = 0;  // a stack-slot promoted program (host.cpp promote_slots): the guard
  uint32_t dma_chunks = 4;  // the fixed-slot window DMA's chunks (compile_into_template)
  // xdp_md batches of loop programs run on their staged images (interp.hip xdp_stage): image
  // dwords 0 and 4 are the ctx, data = 8 and data_end = 8 + len = LEN (xdp.rs:16-20), so the
  // range analysis gives `ldxw rX, [ctx + 0]` the constant 8 and `ldxw rX, [ctx + 4]` LEN -- the
  // loop over data .. data_end is then a loop below LEN, as the main.rs layout's over r2
  bool xdp_ctx = false;
  // (xdp_ctx) the ctx loads: `ldxw rX, [r1 + 0 / 4]` with r1 still the initial r1 (the image's
  // start) on every path -- the value is the staged ctx's data (8) or data_end (LEN), a 4-byte
  // load that cannot fault in an image of >= 8 bytes; compiled as one move into rX's low word
  // (the load's merge, Q1), and not a load for the byte-loop machinery (zero windows, prefetch)
  mutable std::vector<int> ctx_off;  // per micro-op: 0 / 4, or -1
  int ctx_load(uint32_t i) const {
    if (!xdp_ctx) return -1;
    if (ctx_off.empty()) {
      // init[i]: the registers (bit r) holding the initial r1 -- the image start, the ctx -- on
      // every path to i: r1 unmodified, or a copy of it (mov rX, r1 / mov32: the start is 0)
      std::vector<char> seen(n, 0);
      std::vector<uint16_t> init(n, 0);
      std::vector<uint32_t> work{0};
      seen[0] = 1;
      init[0] = 1u << 1;
      auto flow = [&](uint32_t to, uint16_t v) {
        if (to >= n) return;
        if (!seen[to]) {
          seen[to] = 1, init[to] = v, work.push_back(to);
        } else if ((init[to] & v) != init[to]) {
          init[to] &= v, work.push_back(to);
        }
      };
      while (!work.empty()) {
        const uint32_t i = work.back();
        work.pop_back();
        const Uop& u = uops[i];
        const bool writes = u.op != U_ST && u.op != U_STX && !is_jump(u) && u.op != U_EXIT &&
                            u.op != U_FAULT && u.op != U_ATOMIC && u.op != U_NOP && u.dst <= 10;
        uint16_t v = init[i];
        if (u.op == U_CALL) v = 0;
        if (u.op == U_ATOMIC) {  // (fetch forms write src, CMPXCHG r0)
          if (u.aux & F_FETCH) v &= (uint16_t)~(1u << u.src);
          if (u.k == 0xf0) v &= (uint16_t)~1u;
        }
        if (writes) {
          const bool copy = (u.op == U_MOV64 || u.op == U_MOV32) && (u.aux & F_SRC) && u.src <= 10 &&
                            ((init[i] >> u.src) & 1);
          v = copy ? (uint16_t)(v | (1u << u.dst)) : (uint16_t)(v & ~(1u << u.dst));
        }
        if (u.op == U_EXIT || u.op == U_FAULT) continue;
        if (u.op == U_JA) {
          flow((uint32_t)u.x, v);
          continue;
        }
        if (is_jump(u)) flow((uint32_t)u.x, v);
        flow(i + 1, v);
      }
      ctx_off.assign(n, -1);
      for (uint32_t i = 0; i < n; i++) {
        const Uop& u = uops[i];
        if (seen[i] && u.op == U_LDX && u.aux == 4 && u.src <= 10 && ((init[i] >> u.src) & 1) &&
            (u.x == 0 || u.x == 4))
          ctx_off[i] = u.x;
      }
    }
    return ctx_off[i];
  }
  // (xdp_ctx) xdp_md in place, rebased (variant 6): the batch runs as the main.rs layout over
  // the packets themselves -- BASE the packet, LEN = len, mem_size - 8 (host.cpp) -- and every
  // packet load's offset is 8 lower (t / tx rebased by jit_compile_loop): image byte a (>= 8, the
  // range analysis proved it for every load) is packet byte a - 8, its bounds a + w <= 8 + len
  // are a - 8 + w <= len, and mem_size's likewise. The registers keep the image's values: r2 and
  // the ctx's data_end are 8 + LEN, data 8 (xdp.rs:16-20).
  bool xdp_rebase = false;
  mutable bool coop_emitted = false;  // a coop_sum entry was emitted (compile_into_template:
                                      // such programs go to the deep kernel, unbinned)

  Compiler(const std::vector<Uop>& u, const std::vector<TUop>& tt, bool lp = false, bool ex = false,
           const StackPlan* sp = nullptr)
      : uops(u), t(tt), n((uint32_t)u.size()), loops(lp), exact(ex), stk(sp) {
    back_in.assign(n + 1, 0);
    addr_src.assign(n + 1, -1);
    start.assign(n + 1, 0);
    target.assign(n + 1, 0);
    target[0] = 1;
    for (uint32_t i = 0; i < n; i++) {
      if (t[i].blen) start[i] = 1;
      const Uop& o = uops[i];
      if (is_jump(o)) {
        const uint32_t x = t[i].x;  // the canonical taken target (PC_DONE past the end)
        const uint32_t np = t[i].npc;
        // (a successor at i + 1 keeps its lanes in exec -- jtail, ja -- and parks none there: no
        // re-admission unless another jump targets it; a back edge parks both, below)
        if (x < n && x != i + 1) target[x] = 1;
        if (np < n && np != i + 1) target[np] = 1;
        // a back edge parks both successors (the fall-through one at i + 1)
        if (loops && ((x <= i && x < n) || (np <= i && np < n)) && i + 1 < n) target[i + 1] = 1;
        if (x <= i && x < n) back_in[x]++;
        if (o.op != U_JA && np <= i && np < n) back_in[np]++;
      }
    }
    start[n] = 1;
    // single-block loops (a head with one back edge, the jump at the end of the head's own
    // block): every lane leaving through that jump parks at the same successor F, so its parked
    // pc is written once when lanes enter the head (they all stay in exec until they leave)
    hoist.assign(n + 1, -2);
    if (loops)
      for (uint32_t i = 0; i < n; i++) {
        const Uop& o = uops[i];
        if (!is_jump(o) || o.op == U_JA) continue;
        const uint32_t x = t[i].x, np = t[i].npc;
        const bool xb = x <= i && x < n, nb = np <= i && np < n;
        if (xb == nb) continue;
        const uint32_t L = xb ? x : np, F = xb ? np : x;
        if (L >= back_in.size() || back_in[L] != 1) continue;
        bool one_block = true;
        for (uint32_t j = L + 1; j <= i; j++) one_block = one_block && !start[j];
        if (one_block) hoist[L] = F >= n ? -1 : (int64_t)F;
      }
  }

  // hoist[L] (loop programs): the parked pc written at the entry of single-block loop head L, or
  // -2 (none)
  std::vector<int64_t> hoist;

  // ---- load-time value ranges: one-byte loads proven in bounds (loop programs) ----
  // The abstract value of a register in the main.rs layout (main.rs:28-31): an unsigned interval
  // [lo, hi]; slack d >= 0 when 0 <= r and r + d <= LEN, the packet's length (LEN <= mem_size for
  // every lane that runs, main.rs:20-21, and <= 2^24), else -1; is_len: r == LEN. Jumps compare
  // signed (emu.rs:230-290, Q2), so a bound is taken from a compare only for a value known
  // non-negative. A one-byte load [r + off] with off + 1 <= slack(r) reads a packet byte: it can
  // neither fault (mmu.rs:16) nor read past the packet, whatever mem_size is.
  struct AbsVal {
    uint64_t lo = 0, hi = ~0ull;
    int64_t slack = -1;
    bool is_len = false;
  };
  using AbsRegs = std::array<AbsVal, 11>;
  static constexpr uint64_t kLenMax = 1ull << 24;  // mem_size bound (include/ebpf_emu.h)
  std::vector<char> inb;   // inb[i]: the one-byte LDX i is proven in bounds
  std::vector<char> reached;  // prove_loads' fixpoint: the micro-ops some path reaches
  std::vector<AbsRegs> ranges;  // the registers' abstract values at each reached micro-op
  // counted loops: a one-byte load's base read from this register instead (-1: its own)
  std::vector<int> addr_src = std::vector<int>(64, -1);
  bool proven = false;     // emitting the proven copy (ldx1_loop drops inb[i] loads' checks)
  // far mode (compile_into_template): the body's long branches as long jumps, and its
  // out-of-line code in islands between blocks (copy) so that every short branch stays in reach
  bool far_mode = false;
  bool occ_ok = false;  // the occupancy variant's body compiled (compile_into_template)
  bool main_layout = false;  // the main.rs register layout (variant 1): the ranges hold for it
  mutable uint32_t wcache = 0;  // store mode: window chunks cached in v[64:79] here (ldxk_lds)
  // pending masks (forward programs, statements with pm=1): pm_of[T] = the SGPR pair s[72+2k:73+2k]
  // k holding the lanes parked at target T, or -1 (parked through LPC, v28, as everywhere else)
  std::vector<int> pm_of;
  static constexpr int kPmPairs = 4;

  // Lanes that jump to a forward target T park in an SGPR mask instead of LPC when every edge into
  // T is a jump's (jtail, ja) and one of kPmPairs pairs is free over [T's first source, T]: the jump
  // ORs its leaving lanes into the mask (SALU) where it wrote LPC with a select (VALU), and T's entry
  // takes exec from the mask where it compared LPC (VALU) -- a rule chain's per-rule VALU chain
  // loses its select and its re-admission compare. Min-pc order is unchanged: code order is
  // execution order in a forward program and every empty-exec skip lands on a target entry (the
  // mask's lanes re-admitted there). A lane's LPC keeps its last parked value, below every later
  // entry, so no LPC compare re-admits it.
  // Complement targets (cm_assign): cm_of[T] = 1 when T's region [R, T) -- R the target before
  // it -- holds only register ALU work, jumps and exits, and every jump into T comes from inside
  // it. Then the lanes reaching T are exactly the region's entry set minus the lanes that left it
  // for elsewhere: kept in P = s[72:73] (set at R's entry, lanes subtracted where they leave for
  // another target or exit), and a test whose leaving lanes go to T only drops them from exec
  // (one v_cmpx: cmpx_pass). A rule chain's tests lose their SALU mask updates.
  std::vector<char> cm_of, cm_start;
  bool cm_any = false;
  void cm_assign(const std::vector<uint32_t>& first) {
    cm_of.assign(n + 1, 0);
    cm_start.assign(n + 1, 0);
    cm_any = false;
    uint32_t R = 0;
    for (uint32_t T = 1; T < n; T++) {
      if (!target[T]) continue;
      bool ok = first[T] != UINT32_MAX && first[T] >= R;
      for (uint32_t i = R; i < T && ok; i++) {
        const Uop& u = uops[i];
        const bool div = u.op == U_DIV64 || u.op == U_MOD64 || u.op == U_DIV32 || u.op == U_MOD32;
        ok = (u.op <= U_BSWAP64 && !div) || u.op == U_LDIMM || is_jump(u) || u.op == U_EXIT;
      }
      if (ok) {
        cm_of[T] = 1;
        if (!cm_of[R]) cm_start[R] = 1;
        cm_any = true;
      }
      R = T;
    }
  }
  // micro-op i lies in a complement target's region: that target (else 0)
  uint32_t cm_region(uint32_t i) const {
    if (!cm_any || i >= n) return 0;
    const uint32_t T = next_target(i);
    return T < n && cm_of[T] ? T : 0;
  }
  static constexpr const char* kCmP = "s[72:73]";

  void pm_assign(const Marker& m) {
    pm_of.assign(n + 1, -1);
    cm_of.assign(n + 1, 0);
    cm_start.assign(n + 1, 0);
    cm_any = false;
    if (!m.pm || loops || stk) return;
    std::vector<uint32_t> first(n + 1, UINT32_MAX);
    for (uint32_t i = 0; i < n; i++) {
      if (!is_jump(uops[i])) continue;
      const uint32_t x = t[i].x, np = t[i].npc;
      if ((x <= i && x < n) || (uops[i].op != U_JA && np <= i && np < n)) return;  // (a back edge)
      if (x < n && x != i + 1) first[x] = std::min(first[x], i);
      if (uops[i].op != U_JA && np < n && np != i + 1) first[np] = std::min(first[np], i);
    }
    cm_assign(first);
    std::vector<uint32_t> busy_until(kPmPairs, 0);  // a pair is free after its target's entry
    std::vector<uint32_t> order;
    for (uint32_t T = 1; T < n; T++)
      if (target[T] && first[T] != UINT32_MAX && !cm_of[T]) order.push_back(T);
    std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return first[a] < first[b]; });
    for (uint32_t T : order)
      for (int k = cm_any ? 1 : 0; k < kPmPairs; k++)
        if (busy_until[k] <= first[T]) {
          busy_until[k] = T;
          pm_of[T] = k;
          break;
        }
  }
  // Block i (a block start) holds only register ALU micro-ops (no division: its fault path)
  // and ends in a jump: code that does nothing with an empty exec.
  bool alu_block(uint32_t i) const {
    for (uint32_t j = i; j < n; j++) {
      const Uop& u = uops[j];
      if (j > i && start[j]) return false;
      if (is_jump(u)) return j + 1 >= n || start[j + 1];
      const bool div = u.op == U_DIV64 || u.op == U_MOD64 || u.op == U_DIV32 || u.op == U_MOD32;
      if (!((u.op <= U_ARSH32 && !div) || u.op == U_LDIMM)) return false;
    }
    return false;
  }
  std::string pm_reg(uint32_t T) const {
    if (T >= pm_of.size() || pm_of[T] < 0) return "";
    const int b = 72 + 2 * pm_of[T];
    return "s[" + std::to_string(b) + ":" + std::to_string(b + 1) + "]";
  }
  std::string pm_zero() const {
    std::string s;
    std::vector<char> used(kPmPairs, 0);
    for (int k : pm_of)
      if (k >= 0 && !used[k]) {
        used[k] = 1;
        s += "s_mov_b64 s[" + std::to_string(72 + 2 * k) + ":" + std::to_string(73 + 2 * k) + "], 0\n";
      }
    return s;
  }
  mutable uint32_t far_tag = 0;
  size_t island_from = 0;  // main's length after the last island
  // A branch whose target may lie past s_branch's reach in far mode: `cond` "" for s_branch, else
  // the s_cbranch_ condition (scc0, scc1, vccz, vccnz, execz, execnz).
  std::string jmp(const std::string& cond, const std::string& label) const {
    if (!far_mode) return (cond.empty() ? "s_branch " : "s_cbranch_" + cond + " ") + label + "\n";
    const std::string t = "f" + ovl_tag + "_" + std::to_string(far_tag++);
    if (cond.empty()) return long_jump(label, t);
    static const char* inv[][2] = {{"scc0", "scc1"}, {"scc1", "scc0"}, {"vccz", "vccnz"},
                                   {"vccnz", "vccz"}, {"execz", "execnz"}, {"execnz", "execz"}};
    std::string ic;
    for (const auto& p : inv)
      if (cond == p[0]) ic = p[1];
    return "s_cbranch_" + ic + " .Lfs" + t + "\n" + long_jump(label, t) + ".Lfs" + t + ":\n";
  }

  static AbsVal av_const(uint64_t c) {
    AbsVal v;
    v.lo = v.hi = c;
    v.slack = c == 0 ? 0 : -1;
    return v;
  }
  static void av_norm(AbsVal& v) {
    if (v.slack >= 0) v.hi = std::min(v.hi, kLenMax), v.lo = std::min(v.lo, v.hi);
  }
  static AbsVal av_meet(const AbsVal& a, const AbsVal& b) {
    AbsVal v;
    v.lo = std::min(a.lo, b.lo);
    v.hi = std::max(a.hi, b.hi);
    v.slack = (a.slack < 0 || b.slack < 0) ? -1 : std::min(a.slack, b.slack);
    v.is_len = a.is_len && b.is_len;
    return v;
  }
  static bool av_eq(const AbsVal& a, const AbsVal& b) {
    return a.lo == b.lo && a.hi == b.hi && a.slack == b.slack && a.is_len == b.is_len;
  }
  // r + c (c as a two's complement 64-bit constant)
  static AbsVal av_add_const(const AbsVal& r, uint64_t c) {
    AbsVal v;  // (full range unless proven free of wrap-around)
    const int64_t sc = (int64_t)c;
    if (sc >= 0 && sc < (1ll << 40) && r.hi < (1ull << 62)) {
      v.lo = r.lo + c, v.hi = r.hi + c;
      if (r.slack >= sc) v.slack = r.slack - sc;
    } else if (sc < 0 && sc > -(1ll << 40) && r.lo >= (uint64_t)-sc) {
      v.lo = r.lo + c, v.hi = r.hi + c;
      if (r.slack >= 0) v.slack = r.slack - sc;
    }
    av_norm(v);
    return v;
  }

  // Transfer of micro-op u over s; jumps also give the taken successor's state (tk).
  static void av_step(const Uop& u, const AbsRegs& s, AbsRegs& nt, AbsRegs& tk,
                      bool xdp_ctx = false) {
    nt = s;
    tk = s;
    const bool reg = (u.aux & F_SRC) != 0;
    const AbsVal b = reg ? s[u.src] : av_const((uint64_t)u.k);
    const bool bconst = b.lo == b.hi;
    AbsVal& d = nt[u.dst];
    const AbsVal a = s[u.dst];
    auto full32 = [] { AbsVal v; v.hi = 0xffffffffull; return v; };
    switch (u.op) {
      case U_MOV64: d = b; return;
      case U_ADD64: {  // (both facts hold when both operands are constants: keep the stronger)
        AbsVal x, y;
        if (bconst) x = av_add_const(a, b.lo);
        if (a.lo == a.hi) y = av_add_const(b, a.lo);
        d.lo = std::max(x.lo, y.lo), d.hi = std::min(x.hi, y.hi);
        d.slack = std::max(x.slack, y.slack);
        d.is_len = (a.is_len && bconst && b.lo == 0) || (b.is_len && a.lo == 0 && a.hi == 0);
        return;
      }
      case U_SUB64:
        d = bconst ? av_add_const(a, 0 - b.lo) : AbsVal();
        d.is_len = a.is_len && bconst && b.lo == 0;
        return;
      case U_AND64:
        d = AbsVal();
        if (b.hi < (1ull << 63)) d.hi = b.hi;
        if (a.hi < (1ull << 63)) d.hi = std::min(d.hi, a.hi), d.slack = a.slack;  // r & c <= r
        if (a.lo == a.hi && bconst) d = av_const(a.lo & b.lo);
        return;
      case U_RSH64:
        if (bconst && b.lo < 64) {
          d = AbsVal();
          d.lo = a.lo >> b.lo, d.hi = a.hi >> b.lo, d.slack = a.slack;  // r >> c <= r
          return;
        }
        d = AbsVal();
        return;
      case U_LSH64:
        d = AbsVal();
        if (bconst && b.lo < 63 && a.hi < (1ull << (62 - b.lo))) d.lo = a.lo << b.lo, d.hi = a.hi << b.lo;
        return;
      case U_MOV32:
        d = bconst ? av_const(b.lo & 0xffffffffull) : full32();
        return;
      case U_AND32:
        d = full32();
        if (bconst) d.hi = b.lo & 0xffffffffull;
        return;
      case U_ZX16: case U_BSWAP16: d = AbsVal(); d.hi = 0xffff; return;
      case U_ZX32: case U_BSWAP32: d = full32(); return;
      case U_BSWAP64: d = AbsVal(); return;
      case U_NOP: return;
      case U_LDIMM: d = av_const((uint64_t)u.k); return;
      case U_LDX: {  // the loaded bytes replace the low aux bytes; the rest of dst stays (Q1)
        d = AbsVal();
        if (u.aux < 8 && a.hi < (1ull << (8 * u.aux))) d.hi = (1ull << (8 * u.aux)) - 1;
        // (xdp_ctx: a 4-byte load of image dword 0 or 4 into a register whose upper half is
        // zero is the ctx's data = 8 or data_end = LEN)
        const AbsVal& base = s[u.src];
        if (xdp_ctx && u.aux == 4 && a.hi < (1ull << 32) && base.lo == base.hi) {
          const uint64_t addr = base.lo + (uint64_t)(int64_t)(int32_t)u.x;
          if (addr == 0) {
            d = av_const(8);
          } else if (addr == 4) {
            d = AbsVal();
            d.hi = kLenMax, d.slack = 0, d.is_len = true;
          }
        }
        return;
      }
      default: break;
    }
    if (u.op <= U_ARSH32) {  // the other ALU operations
      d = u.op >= U_ADD32 ? full32() : AbsVal();
      return;
    }
    if (u.op < U_JEQ || u.op > U_JLE) return;  // JA, 32-bit jumps, EXIT, ...: no refinement
    // signed compares of dst with b (Q2); refinements only for a non-negative dst
    AbsVal& dt = tk[u.dst];
    AbsVal& dn = nt[u.dst];
    const bool nn = a.hi < (1ull << 63);
    const int64_t K = (int64_t)b.lo;
    auto below = [&](AbsVal& v, int64_t lim) {  // v < lim
      if (nn && lim >= 1) v.hi = std::min(v.hi, (uint64_t)lim - 1), v.lo = std::min(v.lo, v.hi);
    };
    auto atleast = [&](AbsVal& v, int64_t lim) {  // v >= lim
      if (nn && lim >= 0 && (uint64_t)lim <= v.hi) v.lo = std::max(v.lo, (uint64_t)lim);
    };
    auto lt_len = [&](AbsVal& v, int64_t sl) {  // 0 <= v and v + sl <= LEN
      if (v.hi < (1ull << 63)) v.slack = std::max(v.slack, sl), av_norm(v);
    };
    if (bconst && !b.is_len) {
      switch (u.op) {
        case U_JEQ:
          if (nn && b.lo <= a.hi && b.lo >= a.lo) dt = av_const(b.lo), dt.slack = std::max(dt.slack, a.slack);
          break;
        case U_JNE:
          if (nn && b.lo <= a.hi && b.lo >= a.lo) dn = av_const(b.lo), dn.slack = std::max(dn.slack, a.slack);
          break;
        case U_JGT: atleast(dt, K + 1); below(dn, K + 1); break;
        case U_JGE: atleast(dt, K); below(dn, K); break;
        case U_JLT: below(dt, K); atleast(dn, K); break;
        case U_JLE: below(dt, K + 1); atleast(dn, K + 1); break;
        default: break;
      }
    }
    if (!reg) return;
    AbsVal& st = tk[u.src];
    AbsVal& sn = nt[u.src];
    if (b.is_len) {  // dst ? LEN
      switch (u.op) {
        case U_JLT: lt_len(dt, 1); break;
        case U_JGE: lt_len(dn, 1); break;
        case U_JLE: lt_len(dt, 0); break;
        case U_JGT: lt_len(dn, 0); break;
        default: break;
      }
    } else if (a.is_len) {  // LEN ? src
      switch (u.op) {
        case U_JGT: lt_len(st, 1); break;
        case U_JLE: lt_len(sn, 1); break;
        case U_JGE: lt_len(st, 0); break;
        case U_JLT: lt_len(sn, 0); break;
        default: break;
      }
    }
  }

  // Forward dataflow to a fixpoint over the micro-ops (meet at joins, bounds widened after a few
  // changes at a loop head); fills inb[]. Programs with stores, atomics or calls prove nothing.
  void prove_loads() {
    inb.assign(n, 0);
    for (const Uop& u : uops)
      if (u.op == U_ST || u.op == U_STX || u.op == U_ATOMIC || u.op == U_CALL) return;
    std::vector<AbsRegs> in(n);
    std::vector<char> seen(n, 0);
    std::vector<uint32_t> changes(n, 0);
    AbsRegs init;
    for (int r = 0; r < 11; r++) init[r] = av_const(0);
    init[2] = AbsVal();
    init[2].hi = kLenMax, init[2].slack = 0, init[2].is_len = true;  // r2 = LEN (main.rs:29)
    init[10] = AbsVal();                                              // r10: a launch value
    std::vector<char> head(n, 0);  // targets of back edges
    for (uint32_t i = 0; i < n; i++)
      if (is_jump(uops[i]) && (uint32_t)uops[i].x <= i) head[(uint32_t)uops[i].x] = 1;
    // widening thresholds: a bound that grows at a loop head jumps to the next of these (the
    // program's non-negative constants and their neighbours, LEN's bound, then no bound), so a
    // counter compared against a constant keeps that bound; a finite ladder, so it terminates
    std::vector<uint64_t> ladder{kLenMax, ~0ull};
    // (xdp_ctx: also INT64_MAX, so a pointer stepping by more than one byte under a signed
    // compare with data_end can settle non-negative -- the compare then bounds it below LEN -- and
    // keep its lower bound past the ctx, which a bound of 2^64 - 1 loses to the add's wrap)
    if (xdp_ctx) ladder.push_back((uint64_t)INT64_MAX);
    for (const Uop& u : uops)
      if (!(u.aux & F_SRC) && u.k >= 0 && (uint64_t)u.k < (1ull << 62))
        for (int64_t d = -1; d <= 1; d++)
          if ((int64_t)u.k + d >= 0) ladder.push_back((uint64_t)(u.k + d));
    std::sort(ladder.begin(), ladder.end());
    auto widen_hi = [&](uint64_t h) { return *std::lower_bound(ladder.begin(), ladder.end(), h); };
    std::vector<uint32_t> work{0};
    in[0] = init;
    seen[0] = 1;
    auto flow = [&](uint32_t to, const AbsRegs& s) {
      if (to >= n) return;
      if (!seen[to]) {
        in[to] = s, seen[to] = 1, work.push_back(to);
        return;
      }
      AbsRegs m;
      bool ch = false;
      for (int r = 0; r < 11; r++) {
        m[r] = av_meet(in[to][r], s[r]);
        if (head[to] && changes[to] > 4) {  // widen at loop heads
          if (m[r].hi != in[to][r].hi)
            m[r].hi = m[r].slack >= 0 ? std::min(widen_hi(m[r].hi), kLenMax) : widen_hi(m[r].hi);
          if (m[r].lo != in[to][r].lo) m[r].lo = 0;
        }
        ch = ch || !av_eq(m[r], in[to][r]);
      }
      if (ch) in[to] = m, changes[to]++, work.push_back(to);
    };
    for (size_t steps = 0; !work.empty() && steps < 100000; steps++) {
      const uint32_t i = work.back();
      work.pop_back();
      const Uop& u = uops[i];
      AbsRegs nt, tk;
      av_step(u, in[i], nt, tk, xdp_ctx);
      if (u.op == U_EXIT || u.op == U_FAULT) continue;
      if (u.op == U_JA) {
        flow((uint32_t)u.x, tk);
        continue;
      }
      if (is_jump(u)) flow((uint32_t)u.x, tk);
      flow(i + 1, nt);
    }
    if (!work.empty()) return;  // (no fixpoint within the bound: prove nothing)
    reached = seen;
    ranges.assign(n, AbsRegs());
    for (uint32_t i = 0; i < n; i++)
      if (seen[i]) ranges[i] = in[i];
    for (uint32_t i = 0; i < n; i++) {
      const Uop& u = uops[i];
      if (!seen[i] || u.op != U_LDX || u.aux != 1) continue;
      const int64_t off = (int64_t)(int32_t)u.x;
      const AbsVal& b = in[i][u.src];
      inb[i] = b.slack >= 0 && off >= 0 && off + 1 <= b.slack;
    }
  }

  // back edges into each pc: a loop head with exactly one lets that jump's taken lanes run the
  // head's block straight away (no lane can be parked there but them)
  std::vector<uint32_t> back_in = std::vector<uint32_t>(64, 0);

  // a jump whose taken or not-taken successor is at or before it
  bool back_edge(uint32_t i) const {
    return loops && is_jump(uops[i]) &&
           ((t[i].x <= i && t[i].x < n) || (uops[i].op != U_JA && t[i].npc <= i && t[i].npc < n));
  }

  // Registers the program may read before writing them (backward liveness over the forward
  // jumps; conservative: LDX reads its base and, merging, its destination, Q1).
  uint32_t live_in() const { return live()[0]; }

  // Registers live at each micro-op's entry (bit r), for live_in and the counted loops.
  std::vector<uint32_t> live() const {
    // r0 is always an output (the return value and the verdict): live past the end, at EXIT and
    // at a fault
    std::vector<uint32_t> in(n + 1, 0);
    in[n] = 1u;
    auto rw = [&](const Uop& u, uint32_t& rd, uint32_t& wr) {
      const uint32_t d = 1u << u.dst, s = (u.aux & F_SRC) ? 1u << u.src : 0u;
      rd = wr = 0;
      if (u.op <= U_ARSH32) {  // ALU64 / ALU32
        wr = d;
        rd = s | ((u.op == U_MOV64 || u.op == U_MOV32) ? 0u : d);
      } else if (u.op <= U_BSWAP64) {  // END
        rd = wr = d;
      } else if (u.op >= U_JA && u.op <= U_JLE32) {
        rd = u.op == U_JA ? 0u : (d | s);
      } else if (u.op == U_LDIMM) {
        wr = d;
      } else if (u.op == U_LDX) {
        rd = d | (1u << u.src);
        wr = d;
      } else if (u.op == U_STX) {
        rd = 1u << u.src;  // (the address r10 + c is resolved at load time)
      } else if (u.op == U_ATOMIC) {  // (stack atomics, emu.rs:373-437) the operand, the dst
        rd = (1u << u.src) | d | (u.k == 0xf0 ? 1u : 0u);  // snapshot written back, CMPXCHG's r0;
      }                                                     // its writes kill nothing here
    };
    for (bool changed = true; changed;) {  // one pass without back edges; to a fixpoint with
      changed = false;                     // them
      for (uint32_t i = n; i-- > 0;) {
        const Uop& u = uops[i];
        uint32_t rd, wr;
        rw(u, rd, wr);
        uint32_t out = 0;
        const bool ends = u.op == U_EXIT || u.op == U_FAULT;
        if (is_jump(u)) {
          out |= in[std::min<uint32_t>(t[i].x, n)];
          if (u.op != U_JA) out |= in[std::min<uint32_t>(t[i].npc, n)];
        } else {
          out = ends ? 1u : in[i + 1];
        }
        const uint32_t v = (rd | (out & ~wr)) & 0x7ffu;
        if (v != in[i]) {
          in[i] = v;
          changed = true;
        }
      }
    }
    return in;
  }

  // ;@@JITINIT@@: r0 and the live-in registers in the main.rs layout
  std::string init_code() const {
    const uint32_t live = live_in() | 1u;
    std::string s = "; registers read before written: " + std::to_string(live) + "\n";
    for (int r = 0; r < 11; r++)
      if (live & (1u << r)) s += r == 2 && xdp_rebase ? std::string("v_add_u32 v4, 8, v31\nv_mov_b32 v5, 0\n")
                                                      : std::string(kJitInitReg[r]);
    return s;
  }

  uint32_t next_start(uint32_t i) const {
    uint32_t j = i + 1;
    while (j < n && !start[j]) j++;
    return j;
  }

  // Whether micro-op j leaves no lane running into j + 1 in a forward program: an exit or fault
  // (@EXIT@), a ja elsewhere, a conditional jump whose successors both lie elsewhere (jtail: both
  // leave). Every branch to a block entry carries an empty exec too (s_cbranch_execz, the fault
  // tails, KFAULT's exit), so a target there re-admits with exec = the parked lanes directly.
  bool clears_exec(uint32_t j) const {
    const Uop& o = uops[j];
    if (o.op == U_EXIT || o.op == U_FAULT) return true;
    if (!is_jump(o)) return false;
    if (o.op == U_JA) return t[j].x != j + 1;
    return t[j].x != j + 1 && t[j].npc != j + 1;
  }

  // The next block after i whose entry can re-admit parked lanes (a jump target), or n: with no
  // lane running, the blocks before it have nothing to do (a rule chain whose first test sent every
  // lane to the next rule skips the rule's other blocks in one branch).
  uint32_t next_target(uint32_t i) const {
    uint32_t j = i + 1;
    while (j < n && !target[j]) j++;
    return j;
  }

  // park the lanes of `mask` ("vcc" or "exec") at pc x (x >= n: they are done, their last
  // entry's LPC is below every later entry)
  std::string park(const std::string& lpc_val, bool done) const {
    if (done) return loops ? "v_mov_b32 v28, -1\n" : std::string();
    return "v_mov_b32 v28, " + lpc_val + "\n";
  }

  // the LPC value of lanes parked at pc x ("" = no write: done lanes of a forward program)
  std::string lpc_of(uint32_t x, bool done) const {
    if (done) return loops ? "-1" : std::string();
    return std::to_string(x);
  }

  std::string entry_label(const std::string& P, uint32_t i) const {
    return ".L" + P + "b" + std::to_string(i);
  }

  // Tail of a jump with a successor at or before it (loop programs): both successors' lanes
  // park (taken: vcc), then the code continues at the lowest backward successor's entry, whose
  // lanes run first (min-pc order; the other successor's lanes are re-admitted on the way).
  std::string back_tail(uint32_t i, const std::string& P) const {
    const uint32_t x = t[i].x, np = t[i].npc;
    const bool ja = uops[i].op == U_JA;
    const bool xb = x <= i && x < n, nb = !ja && np <= i && np < n;
    // one backward successor whose only back edge this is: its lanes continue into the loop
    // head's block directly; the others park at their (forward or done) successor
    if (xb != nb) {
      const uint32_t L = xb ? x : np, F = xb ? np : x;
      if (L < back_in.size() && back_in[L] == 1) {
        if (ja) return "s_branch .L" + P + "body" + std::to_string(L) + "\n";
        if (hoist[L] != -2)  // the leaving lanes' parked pc was set at the head's entry
          return std::string(xb ? "s_and_b64 exec, exec, vcc\n" : "s_andn2_b64 exec, exec, vcc\n") +
                 "s_cbranch_scc1 .L" + P + "body" + std::to_string(L) + "\n";
        // the leaving lanes' parked pc by one select on vcc (a VOP3 write touches only the active
        // lanes), then exec keeps the staying lanes; SCC = some lane stays
        std::string s;  // (loop programs: "-1" for done lanes; pcs above 64 from a VGPR)
        const std::string F_lpc = vop3_lpc(lpc_of(F, F >= n), "v37", s);
        s += xb ? "v_cndmask_b32_e64 v28, " + F_lpc + ", v28, vcc\n"
                : "v_cndmask_b32_e64 v28, v28, " + F_lpc + ", vcc\n";
        s += (xb ? "s_and_b64 exec, exec, vcc\n" : "s_andn2_b64 exec, exec, vcc\n");
        return s + "s_cbranch_scc1 .L" + P + "body" + std::to_string(L) + "\n";
      }
    }
    std::string s;
    if (ja) {
      s += park(std::to_string(x), x >= n);
    } else {
      const std::string lx = vop3_lpc(lpc_of(x, x >= n), "v37", s),
                        ln = vop3_lpc(lpc_of(np, np >= n), "v38", s);
      if (!lx.empty() || !ln.empty())
        s += "v_cndmask_b32_e64 v28, " + (ln.empty() ? "v28" : ln) + ", " +
             (lx.empty() ? "v28" : lx) + ", vcc\n";
    }
    uint32_t back = n;
    if (x <= i && x < n) back = x;
    if (!ja && np <= i && np < n) back = std::min(back, np);
    return s + "s_mov_b64 exec, 0\ns_branch " + entry_label(P, back) + "\n";
  }

  // The 16-byte chunks of the header window the compiled fixed-slot code can read: 4 with any
  // register-address load (its address is a run-time value), else enough to cover every
  // constant-address load and packet-window store ending inside the window (loads past it read
  // HBM directly), at least one. The fixed-slot kernel's window DMA moves only those chunks.
  uint32_t window_chunks() const {
    if (stk && stk->any_dyn) return 4;  // (store mode reads and writes the whole window)
    uint32_t maxend = 0;
    for (uint32_t i = 0; i < n; i++) {
      const uint32_t id = t[i].hoff / TILE_SLOT;
      if (uops[i].op == U_LDX && stk && stk->off[i] != kNoStack) continue;  // (the stack window)
      if (id == T_LDX_C || id == T_LDX_E || id == T_LDX1_C || id == T_LDX1_E) return 4;
      if (is_ldxk(id)) maxend = std::max<uint32_t>(maxend, t[i].x);
      else if (uops[i].op == U_LDX && id != T_LDXK_FAR_C && id != T_LDXK_FAR_E) return 4;
      if (stk && i < stk->pw.size() && stk->pw[i] != kNoStack)
        maxend = std::max<uint32_t>(maxend, (uint32_t)stk->pw[i] + uops[i].aux);
    }
    return std::max<uint32_t>(1, std::min<uint32_t>(4, (maxend + 15) / 16));
  }

  // Every reachable packet load is a one-byte load proven inside the packet (prove_loads).
  // (xdp_ctx) Whether the program runs rebased (xdp_rebase): its range analysis reaches a fixpoint
  // and every load it reaches, but the ctx loads, is a register-address load (T_LDX / T_LDX1, the
  // offset in TUop::imm) whose address is >= 8 on every path -- so it never reads the ctx, which
  // is not in memory there.
  bool rebase_ok(const std::vector<TUop>& tx) {
    prove_loads();
    if (reached.size() != n) return false;
    for (uint32_t i = 0; i < n; i++) {
      if (!reached[i] || uops[i].op != U_LDX || ctx_load(i) >= 0) continue;
      for (const std::vector<TUop>* tt : {&t, &tx}) {
        const uint32_t id = (*tt)[i].hoff / TILE_SLOT;
        if (id != T_LDX_C && id != T_LDX_E && id != T_LDX1_C && id != T_LDX1_E) return false;
        if ((int64_t)(*tt)[i].imm != (int64_t)(int32_t)uops[i].x) return false;
      }
      // a = r + off >= 8 on every path: r >= 8 - off, and r + off does not wrap
      const AbsVal& b = ranges[i][uops[i].src];
      const int64_t off = (int64_t)(int32_t)uops[i].x;
      if (b.lo >= (1ull << 62) || (int64_t)b.lo + off < 8 || (off > 0 && b.hi > ~0ull - (uint64_t)off))
        return false;
    }
    return true;
  }

  bool all_loads_proven() {
    prove_loads();
    if (reached.size() != n) return false;
    for (uint32_t i = 0; i < n; i++)
      if (reached[i] && uops[i].op == U_LDX && !inb[i]) return false;
    return true;
  }

  // A VOP3 operand for an LPC value: an inline constant, or (programs above 64 micro-ops) a
  // VGPR loaded in `pre` (v37 / v38: temporaries free at a jump's tail; an SGPR beside vcc would
  // be a second constant-bus read).
  static std::string vop3_lpc(const std::string& v, const char* vreg_, std::string& pre) {
    if (v.empty() || v == "-1" || std::stoul(v) <= 64) return v;
    pre += std::string("v_mov_b32 ") + vreg_ + ", " + v + "\n";
    return vreg_;
  }

  // Conditional jump tail: vcc = taken among the active lanes.
  // The eBPF registers live on entry to each micro-op (bit r; a backward dataflow to a fixpoint,
  // loops included). Conservative: an exit, a fault or a call reads every register (the final
  // registers are an output), a load merges into its destination (Q1).
  mutable std::vector<uint16_t> live_in_;
  uint16_t live_in(uint32_t pc) const {
    constexpr uint16_t kAll = 0x7ff;
    if (pc >= n) return kAll;
    if (live_in_.empty()) {
      std::vector<uint16_t> li(n, 0);
      for (bool ch = true; ch;) {
        ch = false;
        for (uint32_t j = n; j-- > 0;) {
          const Uop& u = uops[j];
          const uint16_t D = (uint16_t)(u.dst <= 10 ? 1u << u.dst : 0);
          const uint16_t S = (uint16_t)(u.src <= 10 ? 1u << u.src : 0);
          const bool reg = (u.aux & F_SRC) != 0;
          uint16_t use = 0, def = 0, out = 0;
          auto at = [&](uint32_t q) -> uint16_t { return q >= n ? kAll : li[q]; };
          bool next = true;
          if (u.op <= U_ARSH32) {
            const bool mov = u.op == U_MOV64 || u.op == U_MOV32;
            use = (uint16_t)((mov ? 0 : D) | (reg ? S : 0));
            def = D;
          } else if (u.op <= U_BSWAP64) {
            use = D, def = u.op == U_NOP ? 0 : D;
          } else if (u.op == U_JA) {
            next = false;
            out = at((uint32_t)u.x);
          } else if (is_jump(u)) {
            use = (uint16_t)(D | (reg ? S : 0));
            out = at((uint32_t)u.x);
          } else if (u.op == U_LDIMM) {
            def = D;
          } else if (u.op == U_LDX) {
            use = (uint16_t)(S | (u.aux < 8 ? D : 0)), def = D;
          } else if (u.op == U_ST) {
            use = D;
          } else if (u.op == U_STX) {
            use = (uint16_t)(D | S);
          } else if (u.op == U_ATOMIC) {
            use = (uint16_t)(D | S | 1u);
          } else {  // CALL, EXIT, FAULT
            use = kAll, next = false;
          }
          if (next) out |= at(j + 1);
          const uint16_t v = (uint16_t)(use | (out & ~def));
          if (v != li[j]) li[j] = v, ch = true;
        }
      }
      live_in_ = li;
    }
    return live_in_[pc];
  }
  // A marker for the jump tail's sinking pass (sink_high_zero): the high-half VGPRs of the
  // registers dead where this jump's leaving lanes go.
  std::string dead_marker(uint32_t leave) const {
    if (leave >= n) return "";
    const uint16_t dead = (uint16_t)(~live_in(leave) & 0x7ff);
    if (!dead) return "";
    std::string m = "; dead@leave";
    for (uint32_t r = 0; r <= 10; r++)
      if (dead & (1u << r)) m += " v" + std::to_string(2 * r + 1);
    return m + "\n";
  }

  std::string jtail(uint32_t i, const std::string& P) const {
    if (back_edge(i)) return back_tail(i, P);
    const uint32_t x = t[i].x, np = t[i].npc;
    const bool x_next = x == i + 1, n_next = np == i + 1;
    const bool x_done = x >= n, n_done = np >= n;
    if (x_next && n_next) return "";
    if (n_next != x_next) return dead_marker(n_next ? x : np) + jtail_code(i);
    return jtail_code(i);
  }
  std::string jtail_code(uint32_t i) const {
    const uint32_t x = t[i].x, np = t[i].npc;
    const bool x_next = x == i + 1, n_next = np == i + 1;
    const bool x_done = x >= n, n_done = np >= n;
    // the leaving lanes' LPC by one select on vcc (the pcs are inline constants, or VGPRs above
    // 64), then exec
    std::string pre;
    const std::string mx = x_done ? "" : pm_reg(x), mn = n_done ? "" : pm_reg(np);
    if (const uint32_t CT = cm_region(i)) {
      // complement region: lanes leaving for CT are only dropped from exec; lanes leaving for
      // another target or finishing are recorded there (mask or LPC) and taken out of P
      const bool xl = !x_next, nl = !n_next;  // which side leaves
      std::string s;
      if (xl && x != CT) {
        if (!mx.empty()) s += "s_or_b64 " + mx + ", " + mx + ", vcc\n";
        s += std::string("s_andn2_b64 ") + kCmP + ", " + kCmP + ", vcc\n";
      }
      if (nl && np != CT) {
        s += "s_andn2_b64 s[64:65], exec, vcc\n";
        if (!mn.empty()) s += "s_or_b64 " + mn + ", " + mn + ", s[64:65]\n";
        s += std::string("s_andn2_b64 ") + kCmP + ", " + kCmP + ", s[64:65]\n";
      }
      const std::string lx = xl && x != CT && mx.empty() ? vop3_lpc(lpc_of(x, x_done), "v37", pre) : "",
                        ln = nl && np != CT && mn.empty() ? vop3_lpc(lpc_of(np, n_done), "v38", pre) : "";
      if (!lx.empty() || !ln.empty())
        s += pre + "v_cndmask_b32_e64 v28, " + (ln.empty() ? "v28" : ln) + ", " +
             (lx.empty() ? "v28" : lx) + ", vcc\n";
      if (xl && nl) return s + "s_mov_b64 exec, 0\n";
      // (`; cmx`: cmpx_pass may fold the compare and this update into one v_cmpx -- only here,
      // where nothing reads vcc after it: a negated v_cmpx leaves vcc negated)
      return s + (s.empty() ? "; cmx\n" : "") +
             (xl ? "s_andn2_b64 exec, exec, vcc\n" : "s_and_b64 exec, exec, vcc\n");
    }
    if (n_next && !mx.empty())  // taken lanes leave into their target's mask
      return "s_or_b64 " + mx + ", " + mx + ", vcc\n"  // (a VOPC result: 0 in inactive lanes)
             "s_andn2_b64 exec, exec, vcc\n";
    if (x_next && !mn.empty())  // not-taken lanes leave into theirs
      return "s_andn2_b64 s[64:65], exec, vcc\ns_or_b64 " + mn + ", " + mn + ", s[64:65]\n"
             "s_and_b64 exec, exec, vcc\n";
    if (!n_next && !x_next && (!mx.empty() || !mn.empty())) {  // both leave, one or both masked
      std::string s;
      if (!mx.empty()) s += "s_or_b64 " + mx + ", " + mx + ", vcc\n";
      if (!mn.empty()) s += "s_andn2_b64 s[64:65], exec, vcc\ns_or_b64 " + mn + ", " + mn + ", s[64:65]\n";
      const std::string lx = mx.empty() ? vop3_lpc(lpc_of(x, x_done), "v37", pre) : "",
                        ln = mn.empty() ? vop3_lpc(lpc_of(np, n_done), "v38", pre) : "";
      if (!lx.empty() || !ln.empty())
        s += pre + "v_cndmask_b32_e64 v28, " + (ln.empty() ? "v28" : ln) + ", " +
             (lx.empty() ? "v28" : lx) + ", vcc\n";
      return s + "s_mov_b64 exec, 0\n";
    }
    if (n_next) {  // taken lanes leave
      const std::string lx = vop3_lpc(lpc_of(x, x_done), "v37", pre);
      return pre + (lx.empty() ? "" : "v_cndmask_b32_e64 v28, v28, " + lx + ", vcc\n") +
             "s_andn2_b64 exec, exec, vcc\n";
    }
    if (x_next) {  // not-taken lanes leave (a literal pc cannot go in: vcc is the select's one
                   // constant-bus read)
      const std::string ln = vop3_lpc(lpc_of(np, n_done), "v38", pre);
      return pre + (ln.empty() ? "" : "v_cndmask_b32_e64 v28, " + ln + ", v28, vcc\n") +
             "s_and_b64 exec, exec, vcc\n";
    }
    // both leave
    const std::string lx = vop3_lpc(lpc_of(x, x_done), "v37", pre),
                      ln = vop3_lpc(lpc_of(np, n_done), "v38", pre);
    std::string s = pre;
    if (!lx.empty() || !ln.empty())
      s += "v_cndmask_b32_e64 v28, " + (ln.empty() ? "v28" : ln) + ", " +
           (lx.empty() ? "v28" : lx) + ", vcc\n";
    return s + "s_mov_b64 exec, 0\n";
  }

  std::string ja(uint32_t i, const std::string& P) const {
    if (back_edge(i)) return back_tail(i, P);
    const uint32_t x = t[i].x;
    if (x == i + 1) return "";
    const std::string mx = x >= n ? "" : pm_reg(x);
    std::string out = "";
    if (const uint32_t CT = cm_region(i)) {
      if (x == CT) return "s_mov_b64 exec, 0\n";
      out = std::string("s_andn2_b64 ") + kCmP + ", " + kCmP + ", exec\n";
    }
    if (!mx.empty()) return out + "s_or_b64 " + mx + ", " + mx + ", exec\ns_mov_b64 exec, 0\n";
    return out + park(std::to_string(x), x >= n) + "s_mov_b64 exec, 0\n";
  }

  // Expand the tokens of one template text for micro-op i.
  bool expand(const char* tmpl, uint32_t i, const Marker& m, const std::string& P,
              std::set<uint32_t>& sg, std::string& out) {
    const TUop& u = t[i];
    const uint32_t* w = (const uint32_t*)&u;
    const std::string lab = P + "u" + std::to_string(i);
    const std::string next = ".L" + P + "b" + std::to_string(next_start(i));
    std::string text(tmpl);
    size_t ls = 0;
    while (ls < text.size()) {
      size_t le = text.find('\n', ls);
      if (le == std::string::npos) le = text.size();
      const std::string line = text.substr(ls, le - ls);
      ls = le + 1;
      const bool salu = line.compare(0, 2, "s_") == 0;
      int literals = 0;
      std::string o;
      size_t p = 0;
      while (p < line.size()) {
        const size_t a = line.find('@', p);
        if (a == std::string::npos) {
          o += line.substr(p);
          break;
        }
        const size_t b = line.find('@', a + 1);
        if (b == std::string::npos) {
          err = "unterminated token: " + line;
          return false;
        }
        o += line.substr(p, a - p);
        const std::string tok = line.substr(a + 1, b - a - 1);
        p = b + 1;
        if (tok == "U") {
          o += lab;
        } else if (tok == "NEXT") {
          o += next;
        } else if (tok == "JTAIL") {
          o += jtail(i, P);
        } else if (tok == "JA") {
          o += ja(i, P);
        } else if (tok == "EXIT") {
          o += loops ? "v_mov_b32 v28, -1\ns_mov_b64 exec, 0\n"
               : cm_region(i) ? std::string("s_andn2_b64 ") + kCmP + ", " + kCmP +
                                    ", exec\ns_mov_b64 exec, 0\n"
                              : "s_mov_b64 exec, 0\n";
        } else if (tok[0] == 'D' || tok[0] == 'S') {
          const uint32_t base = tok[0] == 'D' ? u.dst2 : u.src2;
          if (base > 20) {
            err = "register index out of range";
            return false;
          }
          const size_t c = tok.find(':');
          if (c == std::string::npos)
            o += vreg(base, (uint32_t)std::stoul(tok.substr(1)));
          else
            o += vpair(base, (uint32_t)std::stoul(tok.substr(1, c - 1)),
                       (uint32_t)std::stoul(tok.substr(c + 1)));
        } else if (tok[0] == 'K') {
          const size_t c = tok.find(':');
          if (c == std::string::npos) {
            const uint32_t d = (uint32_t)std::stoul(tok.substr(1));
            const uint32_t v = w[d];
            if (inline_const((int32_t)v)) {
              o += std::to_string((int32_t)v);
            } else if (salu && literals == 0) {
              o += hex32(v);
              literals++;
            } else {
              sg.insert(d);
              o += "s" + std::to_string(kFieldSgpr + d);
            }
          } else {
            const uint32_t d0 = (uint32_t)std::stoul(tok.substr(1, c - 1));
            const uint32_t d1 = (uint32_t)std::stoul(tok.substr(c + 1));
            const int64_t v = (int64_t)((uint64_t)w[d0] | ((uint64_t)w[d1] << 32));
            if (d1 == d0 + 1 && inline_const(v)) {
              o += std::to_string(v);
            } else {
              for (uint32_t d = d0; d <= d1; d++) sg.insert(d);
              o += "s[" + std::to_string(kFieldSgpr + d0) + ":" + std::to_string(kFieldSgpr + d1) +
                   "]";
            }
          }
        } else {
          err = "unknown token @" + tok + "@";
          return false;
        }
      }
      // the statement's own operands
      for (const auto& kv : {std::make_pair(std::string("%[fixed]"), m.fixed),
                             std::make_pair(std::string("%[loops]"), m.loops),
                             std::make_pair(std::string("%[aligned]"), m.aligned)}) {
        size_t q;
        while ((q = o.find(kv.first)) != std::string::npos) o.replace(q, kv.first.size(), kv.second);
      }
      if (o.find("%[") != std::string::npos) {
        err = "unresolved operand: " + o;
        return false;
      }
      out += o;
      if (!o.empty() && o.back() != '\n') out += '\n';
    }
    return true;
  }

  // The program's code for the statement behind marker m.
  // Constant-address window loads (the LDXK handlers) of the fixed-slot layout.
  static bool is_ldxk(uint32_t id) {
    return id == T_LDXK_C || id == T_LDXK_E || id == T_LDXK1_C || id == T_LDXK1_E ||
           id == T_LDXK2_C || id == T_LDXK2_E;
  }

  // A window load from the registers the fast copy preloaded: window dword k of the lane is
  // v[64 + k] (the fixed-slot layout: every packet >= 64 bytes, so no length masking; the caller
  // checked mem_size against every such load's end). The access's bytes are merged into dst as
  // the handlers do (Q1): v_perm_b32 picks bytes of the window dword for the low `width` bytes
  // and keeps dst's other bytes.
  std::string ldxk_fast(uint32_t i) const {
    const TUop& u = t[i];
    const uint32_t a0 = u.a0, width = u.x - u.a0, sh = a0 & 3, d = a0 >> 2;
    auto W = [](uint32_t k) { return "v" + std::to_string(64 + k); };
    const std::string D0 = "v" + std::to_string(u.dst2), D1 = "v" + std::to_string(u.dst2 + 1);
    std::string s;
    if (width == 8) {
      if (sh == 0)
        return "v_mov_b32 " + D0 + ", " + W(d) + "\nv_mov_b32 " + D1 + ", " + W(d + 1) + "\n";
      return "v_alignbyte_b32 " + D0 + ", " + W(d + 1) + ", " + W(d) + ", " + std::to_string(sh) +
             "\nv_alignbyte_b32 " + D1 + ", " + W(d + 2) + ", " + W(d + 1) + ", " +
             std::to_string(sh) + "\n";
    }
    std::string src = W(d);
    uint32_t off = sh;
    if (sh + width > 4 && width == 4)
      return "v_alignbyte_b32 " + D0 + ", " + W(d + 1) + ", " + W(d) + ", " + std::to_string(sh) +
             "\n";
    if (sh + width > 4) {  // spans two dwords: align into v26 first
      s += "v_alignbyte_b32 v26, " + W(d + 1) + ", " + W(d) + ", " + std::to_string(sh) + "\n";
      src = "v26";
      off = 0;
    }
    if (width == 4) return s + "v_mov_b32 " + D0 + ", " + src + "\n";
    uint32_t sel = 0;
    for (uint32_t b = 0; b < 4; b++) sel |= (b < width ? 4 + off + b : b) << (8 * b);
    return s + "s_mov_b32 s36, " + hex32(sel) + "\nv_perm_b32 " + D0 + ", " + src + ", " + D0 +
           ", s36\n";
  }

  // A one-byte register-address load in a loop program (the per-byte loops): the handler's
  // semantics (ldx1 in gen_tile.py, loop form) with its checks merged -- in bounds is a < mem
  // as one 64-bit compare against s[52:53] = mem (mem < 2^24, so a nonzero high word fails it);
  // a < len is computed once into s[60:61] (a VOPC result is 0 for inactive lanes), and the
  // window offset a - WB is zeroed for lanes at or past len, so one unsigned compare finds the
  // lanes that need a refill (vcc, branched on directly) and the LDS address needs no clamp; the
  // byte is read with ds_read_u8 at its swizzled window address, zeroed past len by the same
  // mask, and merged with the 0xff in s56 (set once per program). The window refill (or, in
  // tiles with unaligned packets, the packet dword's load) is out of line.
  // ---- memory tier 0.5: the stack window [r10 - k, r10) in v[kStackVgpr + j] (dword j) ----
  std::string sv(uint32_t j) const { return "v" + std::to_string(kStackVgpr + j); }

  // LDX from the window at byte p = k + off (static): the bytes merged into dst as the handlers
  // do (Q1, emu.rs:341-349) -- ldxk_fast's code over the window registers.
  std::string stack_load(uint32_t i) const {
    const Uop& o = uops[i];
    const uint32_t p = (uint32_t)((int32_t)stk->k + stk->off[i]), width = o.aux, sh = p & 3, d = p >> 2;
    const std::string D0 = "v" + std::to_string(2 * o.dst), D1 = "v" + std::to_string(2 * o.dst + 1);
    auto W = [&](uint32_t q) { return sv(q); };
    if (width == 8) {
      if (sh == 0) return "v_mov_b32 " + D0 + ", " + W(d) + "\nv_mov_b32 " + D1 + ", " + W(d + 1) + "\n";
      return "v_alignbyte_b32 " + D0 + ", " + W(d + 1) + ", " + W(d) + ", " + std::to_string(sh) +
             "\nv_alignbyte_b32 " + D1 + ", " + W(d + 2) + ", " + W(d + 1) + ", " +
             std::to_string(sh) + "\n";
    }
    std::string s, src = W(d);
    uint32_t off = sh;
    if (sh + width > 4 && width == 4)
      return "v_alignbyte_b32 " + D0 + ", " + W(d + 1) + ", " + W(d) + ", " + std::to_string(sh) + "\n";
    if (sh + width > 4) {
      s += "v_alignbyte_b32 v26, " + W(d + 1) + ", " + W(d) + ", " + std::to_string(sh) + "\n";
      src = "v26";
      off = 0;
    }
    if (width == 4) return s + "v_mov_b32 " + D0 + ", " + src + "\n";
    uint32_t sel = 0;
    for (uint32_t b = 0; b < 4; b++) sel |= (b < width ? 4 + off + b : b) << (8 * b);
    return s + "s_mov_b32 s36, " + hex32(sel) + "\nv_perm_b32 " + D0 + ", " + src + ", " + D0 + ", s36\n";
  }

  // ST / STX into the window at byte p = k + off (static): the low `width` bytes of the value
  // (STX: src register; ST: the zero-extended immediate, Q8) written little-endian
  // (emu.rs:354-372). Per window dword the bytes it takes, by a move (whole dword) or a v_perm.
  std::string stack_store(uint32_t i) const {
    return store_bytes(i, (uint32_t)((int32_t)stk->k + stk->off[i]), kStackVgpr);
  }

  // ST / STX into the packet's header window at the constant image address pw[i]: the window
  // dwords the fast copy preloaded into v[64 + j] (every later load of those bytes is a
  // constant-address one reading them, host.cpp analyze_stack)
  std::string pw_store(uint32_t i) const { return store_bytes(i, (uint32_t)stk->pw[i], 64); }

  // The store of micro-op i at byte p of a window held in v[base + j] (dword j).
  std::string store_bytes(uint32_t i, uint32_t p, uint32_t base) const {
    const Uop& o = uops[i];
    const uint32_t w = o.aux;
    auto sv = [&](uint32_t j) { return "v" + std::to_string(base + j); };
    const bool imm = o.op == U_ST;
    const uint64_t kv = (uint64_t)o.k;  // ST: imm64 (zero-extended imm)
    const std::string V0 = "v" + std::to_string(2 * o.src), V1 = "v" + std::to_string(2 * o.src + 1);
    std::string s;
    for (uint32_t j = p >> 2; j <= (p + w - 1) >> 2; j++) {
      const uint32_t lo = std::max(p, 4 * j), hi = std::min(p + w, 4 * j + 4);
      const int32_t sft = (int32_t)(4 * j) - (int32_t)p;  // value byte at this dword's byte 0
      // t: a dword whose byte q is value byte q + sft (where that byte is used)
      std::string t;
      uint32_t tc = 0;  // (ST) the constant t
      if (imm) {
        for (uint32_t q = 0; q < 4; q++) {
          const int32_t vb = (int32_t)q + sft;
          if (vb >= 0 && vb < 8) tc |= (uint32_t)((kv >> (8 * vb)) & 0xff) << (8 * q);
        }
      } else if (sft == 0) {
        t = V0;
      } else if (sft == 4) {
        t = V1;
      } else if (sft > 0 && sft < 4) {
        s += "v_alignbyte_b32 v42, " + V1 + ", " + V0 + ", " + std::to_string(sft) + "\n";
        t = "v42";
      } else if (sft > 4) {
        s += "v_alignbyte_b32 v42, 0, " + V1 + ", " + std::to_string(sft - 4) + "\n";
        t = "v42";
      } else {  // sft < 0: the first dword of a misaligned store
        s += "v_lshlrev_b32 v42, " + std::to_string(-sft * 8) + ", " + V0 + "\n";
        t = "v42";
      }
      if (lo == 4 * j && hi == 4 * j + 4) {  // the whole dword
        s += imm ? "v_mov_b32 " + sv(j) + ", " + hex32(tc) + "\n" : "v_mov_b32 " + sv(j) + ", " + t + "\n";
        continue;
      }
      uint32_t sel = 0;
      for (uint32_t q = 0; q < 4; q++)
        sel |= (4 * j + q >= lo && 4 * j + q < hi ? 4 + q : q) << (8 * q);
      if (imm) {
        s += "v_mov_b32 v42, " + hex32(tc) + "\n";
        t = "v42";
      }
      s += "s_mov_b32 s36, " + hex32(sel) + "\nv_perm_b32 " + sv(j) + ", " + t + ", " + sv(j) +
           ", s36\n";
    }
    return s;
  }

  // ---- store mode (StackPlan::any_dyn): the lane's header window in LDS is the image's bytes
  // [0, 64) -- packet bytes, zeros at or past LEN, and whatever the program stored there. Window
  // byte b of the lane is at LDS address (b ^ SWZ) + WIN (v35 = SWZ, v34 = WIN: the 16-byte chunks
  // swizzled per lane, interp.hip win_off), so a run of bytes inside one chunk is contiguous. ----

  // The value register pair of a store (STX: src) or, for ST, "" (constant bytes of o.k, Q8).
  // The low `nb` bytes of value bytes [q, q + nb) in a VGPR: a source register itself, or v42
  // (shifted / materialized). hi16: the bytes sit in bits 16.. of the returned register instead.
  std::string store_value(const Uop& o, uint32_t q, uint32_t nb, std::string& s, bool* hi16) const {
    *hi16 = false;
    if (o.op == U_ST) {
      uint32_t c = 0;
      for (uint32_t b = 0; b < nb; b++) c |= (uint32_t)((((uint64_t)o.k) >> (8 * (q + b))) & 0xff) << (8 * b);
      s += "v_mov_b32 v42, " + hex32(c) + "\n";
      return "v42";
    }
    const std::string V = "v" + std::to_string(2 * o.src + (q >= 4 ? 1 : 0));
    const uint32_t r = q & 3;
    if (r == 0) return V;
    if (r == 2 && nb <= 2) {
      *hi16 = true;
      return V;
    }
    if (r + nb <= 4) {
      s += "v_lshrrev_b32 v42, " + std::to_string(8 * r) + ", " + V + "\n";
    } else {  // (crosses into the high word: q < 4 < q + nb)
      s += "v_alignbyte_b32 v42, v" + std::to_string(2 * o.src + 1) + ", v" +
           std::to_string(2 * o.src) + ", " + std::to_string(r) + "\n";
    }
    return "v42";
  }

  // ST / STX at the constant image address p = pw[i] (inside the window): LDS writes of the
  // widest naturally aligned pieces inside each 16-byte chunk (emu.rs:354-372, little-endian).
  std::string lds_store_const(uint32_t i) const {
    const Uop& o = uops[i];
    const uint32_t p = (uint32_t)stk->pw[i], w = o.aux;
    std::string s = "; store [" + std::to_string(p) + ", +" + std::to_string(w) + ") into the window\n";
    int32_t chunk = -1;
    for (uint32_t b = p; b < p + w;) {
      if ((int32_t)(b >> 4) != chunk) {
        chunk = (int32_t)(b >> 4);
        s += "v_xad_u32 v43, v35, " + std::to_string(16 * chunk) + ", v34\n";
      }
      const uint32_t q = b - p, left = std::min(p + w - b, 16 - (b & 15));
      uint32_t nb = 1;
      if ((b & 3) == 0 && (q & 3) == 0 && left >= 4) nb = 4;
      else if ((b & 1) == 0 && (q & 1) == 0 && left >= 2) nb = 2;
      bool hi = false;
      const std::string V = store_value(o, q, nb, s, &hi);
      const std::string op = nb == 4 ? "ds_write_b32" : nb == 2 ? (hi ? "ds_write_b16_d16_hi" : "ds_write_b16")
                                                                : (hi ? "ds_write_b8_d16_hi" : "ds_write_b8");
      s += op + " v43, " + V + " offset:" + std::to_string(b & 15) + "\n";
      b += nb;
    }
    return s;
  }

  // ---- the overflow image (store mode on the var tile loop): image bytes [64, E) of the lane's
  // packet in the workspace, E = min(mem_size rounded up to 64, kOvfEnd = 2048) (LaunchArgs::ovf
  // + packet index * (E - 64)), kept per 64-byte block b (bytes [64 + 64b, 128 + 64b)): a block
  // is filled from the packet (zeros at or past LEN) by the lane's first store into it -- or by
  // a load that spans it and a filled one -- and its bit b set in v23 (the lane's filled
  // blocks; the dirty mask dm: the lanes with any, cleared per tile). Loads of filled blocks read
  // the image (sc1: from L2, where the stores went), of the others the packet. So a rewrite of
  // a 1500-byte frame's payload stays on the compiled kernel, and costs the blocks it touches.
  // s48 = E (from the mem_size in s52).
  static std::string ovf_end() {
    return "s_add_u32 s48, s52, 63\ns_and_b32 s48, s48, 0xffffffc0\n"
           "s_min_u32 s48, s48, " + std::to_string(kOvfEnd) + "\ns_max_u32 s48, s48, 64\n";
  }
  // v[44:45] = the lane's overflow image: ovf + (tile * 64 + lane) * (E - 64). Uses v40, v41,
  // s[48:49], vcc.
  std::string ovf_addr() const {
    return ovf_end() + "s_sub_u32 s48, s48, 64\nv_mov_b32 v41, s48\n"
           "s_lshl_b32 s48, " + tile_s + ", 6\n"
           "v_mbcnt_lo_u32_b32 v40, -1, 0\nv_mbcnt_hi_u32_b32 v40, -1, v40\n"
           "v_add_u32 v40, s48, v40\n"
           "s_mov_b32 s48, " + ovf_lo + "\ns_mov_b32 s49, " + ovf_hi + "\n"
           "v_mad_u64_u32 v[44:45], vcc, v40, v41, s[48:49]\n";
  }
  // The fill routine (one per body, behind its code: ovf_routine; called with s_swappc, return
  // address in s[62:63]): the lanes of exec (some) get block v39 of their overflow image filled
  // from the packet's dwords (those before LEN; the bytes at or past it zero), all 16 in flight
  // through v[64:79]; bit v39 set in v23, the lanes added to dm. Keeps v36-v39, v42, v43,
  // s[60:61], s[66:69]; uses v40, v41, v44-v48, v50, v51, v64-v79, s[48:49], s[64:65], vcc.
  mutable bool ovf_used = false;
  std::string ovf_label() const { return ".Lovf" + ovl_tag; }
  std::string ovf_routine() const {
    if (!ovf_used) return "";
    std::string r = ovf_label() + ":\ns_mov_b64 s[64:65], exec\ns_or_b64 " + dm + ", " + dm + ", exec\n" +
                    ovf_addr() +
                    "v_lshlrev_b32 v40, 6, v39\nv_mov_b32 v41, 0\n"
                    "v_lshl_add_u64 v[44:45], v[44:45], 0, v[40:41]\n"
                    "v_add_u32 v40, 64, v40\n"  // the block's image offset o
                    "v_lshl_add_u64 v[46:47], v[32:33], 0, v[40:41]\n"
                    "v_sub_u32 v48, v31, v40\n";  // LEN - o (signed)
    // the block's 16 dwords in flight at once, into v[64:79] (free in store mode: the chunk
    // cache is invalidated around every call, ldxk_lds)
    for (uint32_t k = 0; k < 16; k++) r += "v_mov_b32 v" + std::to_string(64 + k) + ", 0\n";
    // a chunk wholly before LEN: one 16-byte load; the chunk LEN falls in: its dwords that start
    // before LEN (the rest stay 0; nothing at or past the dword holding LEN - 1 is read)
    for (uint32_t c = 0; c < 4; c++) {
      const std::string C = std::to_string(c), Q = "v[" + std::to_string(64 + 4 * c) + ":" +
                                                    std::to_string(67 + 4 * c) + "]";
      // (every compare under the routine's whole exec: a VOPC result is 0 in inactive lanes)
      r += "s_mov_b64 exec, s[64:65]\n"
           "v_cmp_le_i32 vcc, " + std::to_string(16 * c + 16) + ", v48\n"
           "s_and_b64 exec, s[64:65], vcc\n"
           "global_load_dwordx4 " + Q + ", v[46:47], off offset:" + std::to_string(16 * c) + "\n"
           "s_mov_b64 exec, s[64:65]\n"
           "v_cmp_gt_i32 vcc, " + std::to_string(16 * c + 16) + ", v48\n"
           "s_and_b64 exec, s[64:65], vcc\n"
           "v_cmp_lt_i32 vcc, " + std::to_string(16 * c) + ", v48\n"
           "s_and_b64 exec, exec, vcc\n"
           "s_cbranch_execz .Lovc" + C + "_" + ovl_tag + "\n"
           "s_mov_b64 s[48:49], exec\n";  // (s[48:49]: free once ovf_addr has used it)
      for (uint32_t k = 4 * c; k < 4 * c + 4; k++)
        r += "v_cmp_lt_i32 vcc, " + std::to_string(4 * k) + ", v48\ns_and_b64 exec, s[48:49], vcc\n"
             "global_load_dword v" + std::to_string(64 + k) + ", v[46:47], off offset:" +
             std::to_string(4 * k) + "\n";
      r += ".Lovc" + C + "_" + ovl_tag + ":\n";
    }
    r += "s_mov_b64 exec, s[64:65]\ns_waitcnt vmcnt(0)\n";
    for (uint32_t k = 0; k < 16; k++)
      r += "v_subrev_u32 v50, " + std::to_string(4 * k) + ", v48\n"
           "v_med3_i32 v50, v50, 0, 4\nv_lshlrev_b32 v50, 3, v50\n"
           "v_lshlrev_b64 v[50:51], v50, 1\nv_add_u32 v50, -1, v50\n"
           "v_and_b32 v" + std::to_string(64 + k) + ", v50, v" + std::to_string(64 + k) + "\n";
    for (uint32_t c = 0; c < 4; c++)
      r += "global_store_dwordx4 v[44:45], v[" + std::to_string(64 + 4 * c) + ":" +
           std::to_string(67 + 4 * c) + "], off offset:" + std::to_string(16 * c) + "\n";
    // (the wait also covers the stores' reads of their data VGPRs)
    return r + "s_waitcnt vmcnt(0)\nv_lshlrev_b32 v40, v39, 1\nv_or_b32 v23, v23, v40\n"
               "s_setpc_b64 s[62:63]\n";
  }
  // The lanes of `lanes` whose block v39 is not filled yet: filled by the routine (exec is
  // `lanes` after).
  std::string ovf_ensure(const std::string& lanes, const std::string& tag) const {
    ovf_used = true;
    wcache = 0;  // (the routine uses v[64:79])
    const std::string P = ".Lfp" + tag, L = ovf_label(), d = "(" + L + "-" + P + ")";
    return "v_lshrrev_b32 v40, v39, v23\nv_and_b32 v40, 1, v40\nv_cmp_eq_u32 vcc, 0, v40\n"
           "s_and_b64 exec, " + lanes + ", vcc\ns_cbranch_execz .Lfe" + tag + "\n"
           "s_getpc_b64 s[48:49]\n" + P + ":\ns_add_u32 s48, s48, " + d + "&4294967295\n"
           "s_addc_u32 s49, s49, " + d + ">>32\ns_swappc_b64 s[62:63], s[48:49]\n"
           ".Lfe" + tag + ":\ns_mov_b64 exec, " + lanes + "\n";
  }
  // A constant-address load of [a, a + w) past the window: lanes of exec that filled a block it
  // reads deoptimize first (the load reads the packet).
  std::string ovf_dirty_deopt(const std::string& U, const std::string& next, uint32_t a,
                              uint32_t w) const {
    uint32_t bm = 0;
    for (uint32_t b = std::max(a, 64u); b < a + w && b < kOvfEnd; b++) bm |= 1u << ((b - 64) >> 6);
    if (!bm) return "";
    return "s_and_b64 vcc, exec, " + dm + "\ns_cbranch_vccz .Ldk" + U + "\n"
           "v_and_b32 v40, " + hex32(bm) + ", v23\nv_cmp_ne_u32 vcc, 0, v40\n"
           "s_and_b64 vcc, vcc, exec\ns_cbranch_vccz .Ldk" + U + "\n"
           "s_mov_b64 s[66:67], exec\ns_mov_b64 exec, vcc\nv_mov_b32 v30, 0x80\nv_mov_b32 v28, -1\n"
           "s_andn2_b64 exec, s[66:67], vcc\ns_cbranch_execz " + next + "\n.Ldk" + U + ":\n";
  }

  // ST / STX through a register (StackPlan::dyn): the address a = dst + off with the reference's
  // bounds (a >= mem -> ST_MEM, a + w > mem -> ST_MEM_UB: only the first byte is checked, Q16,
  // mmu.rs:23-30); lanes storing past the window [0, 64) deoptimize (status kStDeopt: the
  // general interpreter re-runs their packets); the rest write their bytes into LDS one by one.
  std::string lds_store_dyn(uint32_t i, const std::string& P, std::string& ool) const {
    const Uop& o = uops[i];
    const uint32_t w = o.aux;
    const std::string U = P + "u" + std::to_string(i), next = entry_label(P, next_start(i));
    const int64_t off = (int64_t)(int32_t)o.x;
    std::string s = "; store through r" + std::to_string(o.dst) + " (store mode)\n", offs;
    if (inline_const(off)) {
      offs = std::to_string(off);
    } else {
      s += "s_mov_b32 s48, " + hex32((uint32_t)off) + "\ns_mov_b32 s49, " +
           hex32((uint32_t)((uint64_t)off >> 32)) + "\n";
      offs = "s[48:49]";
    }
    s += "v_lshl_add_u64 v[36:37], " + vpair(2 * o.dst, 0, 1) + ", 0, " + offs + "\n"
         "v_cmp_gt_u64_e64 s[60:61], s[52:53], v[36:37]\n"
         "v_add_u32 v38, " + std::to_string(w) + ", v36\n"
         "v_cmp_ge_u32_e64 s[62:63], s52, v38\n"
         "s_and_b64 vcc, s[60:61], s[62:63]\n"
         "s_andn2_b64 s[64:65], exec, vcc\n"
         "s_cbranch_scc0 .Lsok" + U + "\n"
         "s_mov_b64 s[66:67], exec\ns_mov_b64 exec, s[64:65]\n"
         "v_cndmask_b32_e64 v30, 1, 2, s[60:61]\n"
         "v_mov_b32 v28, -1\n"
         "v_subrev_u32 v29, " + std::to_string(t[i].a0) + ", v29\n"
         "s_andn2_b64 exec, s[66:67], s[64:65]\n"
         "s_cbranch_execz " + next + "\n"
         ".Lsok" + U + ":\n"
         "v_cmp_lt_u32 vcc, 64, v38\n"
         "s_and_b64 vcc, vcc, exec\n";
    if (!ovf_lo.empty()) {
      s += "s_cbranch_vccnz .Lsov" + U + "\n";
    } else {
      s += "s_cbranch_vccz .Lsin" + U + "\n"
           "s_mov_b64 s[66:67], exec\ns_mov_b64 exec, vcc\n"
           "v_mov_b32 v30, 0x80\nv_mov_b32 v28, -1\n"
           "s_andn2_b64 exec, s[66:67], vcc\n"
           "s_cbranch_execz " + next + "\n";
    }
    s += ".Lsin" + U + ":\n";
    for (uint32_t j = 0; j < w; j++) {
      std::string A = "v36";
      if (j) {
        s += "v_add_u32 v39, " + std::to_string(j) + ", v36\n";
        A = "v39";
      }
      s += "v_xad_u32 v40, " + A + ", v35, v34\n";
      bool hi = false;
      const std::string V = store_value(o, j, 1, s, &hi);
      s += std::string(hi ? "ds_write_b8_d16_hi" : "ds_write_b8") + " v40, " + V + "\n";
    }
    if (ovf_lo.empty()) return s;
    s += ".Lsdn" + U + ":\n";
    // out of line: some lane's store ends past byte 64 (vcc). Lanes ending past min(E, S0 = the
    // stack window's start, s57) deoptimize; the others fill the blocks of their overflow image
    // the store reaches (its first and last byte's: w <= 8) if not yet filled, then write each
    // byte to the window (< 64) or the overflow image.
    std::string o2 = ".Lsov" + U + ":\n" + ovf_end() +
        "v_mov_b32 v39, s48\nv_min_u32 v39, s57, v39\n"
        "v_cmp_lt_u32_e64 s[60:61], v39, v38\n"
        "s_and_b64 s[60:61], s[60:61], vcc\n"
        "s_cbranch_scc0 .Lsnd" + U + "\n"
        "s_mov_b64 s[66:67], exec\ns_mov_b64 exec, s[60:61]\n"
        "v_mov_b32 v30, 0x80\nv_mov_b32 v28, -1\n"
        "s_andn2_b64 exec, s[66:67], s[60:61]\n"
        "s_andn2_b64 vcc, vcc, s[60:61]\n"
        "s_cbranch_execz " + next + "\n"
        ".Lsnd" + U + ":\n"
        "s_mov_b64 s[68:69], vcc\ns_mov_b64 s[66:67], exec\n"
        "v_max_u32 v39, 64, v36\nv_subrev_u32 v39, 64, v39\nv_lshrrev_b32 v39, 6, v39\n" +
        ovf_ensure("s[68:69]", "f" + U) +
        "v_add_u32 v39, -65, v38\nv_lshrrev_b32 v39, 6, v39\n" + ovf_ensure("s[68:69]", "l" + U) +
        "s_mov_b64 exec, s[66:67]\n" + ovf_addr() + "v_mov_b32 v41, 0\n";
    for (uint32_t j = 0; j < w; j++) {
      const std::string J = std::to_string(j);
      o2 += (j ? "v_add_u32 v39, " + J + ", v36\n" : std::string("v_mov_b32 v39, v36\n")) +
            "v_cmp_gt_u32_e64 s[60:61], 64, v39\n"
            "s_mov_b64 s[66:67], exec\ns_and_b64 exec, s[66:67], s[60:61]\n"
            "s_cbranch_execz .Lsw" + J + U + "\n"
            "v_xad_u32 v40, v39, v35, v34\n";
      bool hi = false;
      std::string V = store_value(o, j, 1, o2, &hi);
      o2 += std::string(hi ? "ds_write_b8_d16_hi" : "ds_write_b8") + " v40, " + V + "\n"
            ".Lsw" + J + U + ":\n"
            "s_andn2_b64 exec, s[66:67], s[60:61]\n"
            "s_cbranch_execz .Lsg" + J + U + "\n"
            "v_add_u32 v40, -64, v39\n"
            "v_lshl_add_u64 v[46:47], v[44:45], 0, v[40:41]\n";
      V = store_value(o, j, 1, o2, &hi);
      o2 += std::string(hi ? "global_store_byte_d16_hi" : "global_store_byte") + " v[46:47], " + V +
            ", off\n.Lsg" + J + U + ":\ns_mov_b64 exec, s[66:67]\n";
    }
    o2 += "s_waitcnt vmcnt(0)\ns_branch .Lsdn" + U + "\n";
    ool += o2;
    return s;
  }

  // A constant-address load inside the window (LDXK) in store mode: the window dwords from LDS
  // (no LEN mask: the bytes at or past LEN are zeros there, or stored ones), merged into dst (Q1).
  // Store mode's constant-address loads read the window through a chunk cache in v[64:79] (the
  // preloaded-window registers, free in store mode): a chunk's 16 bytes come from LDS with one
  // ds_read_b128 at its first use and serve every later constant load of it. Every lane of a wave
  // reading the same window byte with ds_read_b32 hit only 16 distinct banks (64-byte windows,
  // chunk-swizzled: a 4-way conflict, PMC round 5: 3.4 conflict cycles per LDS instruction on
  // NAT); a b128 read covers all 64 banks per 16 lanes. Validity (wcache, one bit per chunk) is
  // known at compile time: cleared at every jump target (lanes parked elsewhere re-join, their
  // registers never filled), after every register-address store (any byte may have changed; its
  // overflow fill also uses v[64:79]); a constant-address store writes LDS and merges into the
  // cached dwords (store_bytes).
  std::string ldxk_lds(uint32_t i) const {
    const TUop& u = t[i];
    const uint32_t a0 = u.a0, w = u.x - u.a0, sh = a0 & 3;
    const uint32_t last = w == 8 && sh ? (a0 >> 2) + 2 : (a0 + w - 1) >> 2;
    if (last < 16) {
      std::string s;
      bool fill = false;
      for (uint32_t c = a0 >> 4; c <= last >> 2; c++) {
        if (wcache & (1u << c)) continue;
        s += "v_xad_u32 v43, v35, " + std::to_string(16 * c) + ", v34\nds_read_b128 v[" +
             std::to_string(64 + 4 * c) + ":" + std::to_string(67 + 4 * c) + "], v43\n";
        wcache |= 1u << c;
        fill = true;
      }
      if (fill) s += "s_waitcnt lgkmcnt(0)\n";
      return s + ldxk_fast(i);
    }
    const uint32_t d = a0 & ~3u;
    const uint32_t nd = (sh + w + 3) / 4;
    std::string s;
    for (uint32_t k = 0; k < nd; k++)
      s += "v_xad_u32 v" + std::to_string(43 + k) + ", v35, " + std::to_string(d + 4 * k) +
           ", v34\nds_read_b32 v" + std::to_string(49 + k) + ", v" + std::to_string(43 + k) + "\n";
    s += "s_waitcnt lgkmcnt(0)\n";
    if (nd == 1) s += "v_lshrrev_b32 v26, " + std::to_string(8 * sh) + ", v49\n";
    else s += "v_alignbyte_b32 v26, v50, v49, " + std::to_string(sh) + "\n";
    if (w == 8) s += nd == 3 ? "v_alignbyte_b32 v27, v51, v50, " + std::to_string(sh) + "\n"
                             : std::string("v_mov_b32 v27, v50\n");
    const std::string D0 = "v" + std::to_string(u.dst2);
    if (w == 1 || w == 2)
      s += "s_mov_b32 s42, " + std::string(w == 1 ? "0xff" : "0xffff") + "\nv_bfi_b32 " + D0 +
           ", s42, v26, " + D0 + "\n";
    else if (w == 4)
      s += "v_mov_b32 " + D0 + ", v26\n";
    else
      s += "v_mov_b64 " + vpair(u.dst2, 0, 1) + ", v[26:27]\n";
    return s;
  }

  // The store-mode program (the var kernel's stack statement only; every other statement is
  // never launched for it, host.cpp JitFns::var_only): the stack window in VGPRs as before; the
  // header window's bytes at or past LEN zeroed in LDS once (lanes with LEN < 64 only), so loads
  // and stores address one image; then the program's one (checked) copy.
  bool body_store(const Marker& m, std::string& out) {
    pm_of.clear();  // (LPC parking only)
    const std::string P = "J" + m.n + "_";
    ovl_tag = m.n;
    overlay_widths = 0;
    island_from = 0;
    // (the var tile loop's statement: stores past byte 64 into the overflow image)
    ovf_lo = ovf_hi = tile_s = dm = "";
    unsigned a0 = 0, a1 = 0;
    if (((m.varl && m.stack) || m.st) && !m.tile.empty() && !m.dm.empty() &&
        sscanf(m.ovf.c_str(), "s[%u:%u]", &a0, &a1) == 2 && a1 == a0 + 1) {
      ovf_lo = "s" + std::to_string(a0);
      ovf_hi = "s" + std::to_string(a1);
      tile_s = m.tile;
      dm = m.dm;
    }
    if (!m.stack && !m.st) {
      out = "s_mov_b64 exec, 0  ; (store mode: the var kernels' stack statements and the "
            "fixed-slot statement only)\n";
      return true;
    }
    std::string ool;
    std::string main = "; compiled eBPF program (store mode): " + std::to_string(n) + " micro-ops\n"
                       "s_mov_b32 s52, s33\ns_mov_b32 s53, 0\n";
    if (stk->no_deopt) main += "; store mode: no lane can deoptimize (store_mode_no_deopt)\n";
    if (!dm.empty())  // (no overflow block filled yet: v23, the lanes' block bits, and dm)
      main += "s_mov_b64 " + dm + ", 0\ns_mov_b64 s[64:65], exec\ns_mov_b64 exec, -1\n"
              "v_mov_b32 v23, 0\ns_mov_b64 exec, s[64:65]\n";
    // (the var tile loop's windows hold packet bytes [0, 64): the xdp_md ctx shifted in first, as
    // body does; the var kernel's C++ shifts them itself)
    if ((m.varl || m.st) && !m.xdp.empty())
      main += "s_cmp_lg_u32 " + m.xdp + ", 0\ns_cbranch_scc0 .L" + P + "noxdp\n" + xdp_shift() +
              ".L" + P + "noxdp:\n";
    main += stack_zero() + stack_init(P, ool);
    const std::string Z = ".L" + P + "zdone";
    main += "s_mov_b64 s[64:65], exec\ns_mov_b64 exec, -1\n"
            "v_cmp_gt_u32 vcc, 64, v31\ns_cbranch_vccz " + Z + "\n";
    for (uint32_t c = 0; c < 4; c++)
      main += "v_xad_u32 v" + std::to_string(36 + c) + ", v35, " + std::to_string(16 * c) +
              ", v34\nds_read_b128 v[" + std::to_string(64 + 4 * c) + ":" + std::to_string(67 + 4 * c) +
              "], v" + std::to_string(36 + c) + "\n";
    main += "s_waitcnt lgkmcnt(0)\n";
    for (uint32_t j = 0; j < 16; j++)  // dword j keeps its bytes below LEN
      main += "v_subrev_u32 v40, " + std::to_string(4 * j) + ", v31\n"
              "v_med3_i32 v40, v40, 0, 4\nv_lshlrev_b32 v40, 3, v40\n"
              "v_lshlrev_b64 v[40:41], v40, 1\nv_add_u32 v40, -1, v40\n"
              "v_and_b32 v" + std::to_string(64 + j) + ", v40, v" + std::to_string(64 + j) + "\n";
    for (uint32_t c = 0; c < 4; c++)
      main += "ds_write_b128 v" + std::to_string(36 + c) + ", v[" + std::to_string(64 + 4 * c) + ":" +
              std::to_string(67 + 4 * c) + "]\n";
    main += Z + ":\ns_mov_b64 exec, s[64:65]\ns_mov_b64 exec, 0\n";
    ovf_used = false;
    if (!copy(m, P, false, main, ool)) return false;
    main += ".L" + P + "end:\n";
    ool += overlay_routines() + ovf_routine();
    if (!ool.empty()) main += "s_branch .Ldone" + m.n + "\n" + ool;
    out = peephole(main);
    return true;
  }

  // ATOMIC on the stack window at byte p = k + off (static, 4-aligned; 8 bytes read and written,
  // emu.rs:373-437 as oracle/ebpf_oracle.c restates it): orig = the window qword; the 32-bit form
  // works on its low word, the operand's and r0's low words, and adds the high word back after
  // the operation (a 32-bit ADD's carry leaks into it, Q13); ADD and the recombination fault
  // ST_ARITH on signed overflow (the debug build's checks, Q21); XCHG and CMPXCHG as the
  // reference (CMPXCHG: r0 = the fetched value, 0 without fetch); fetch writes the old value to
  // src; dst is written back from its snapshot last (Q14). Faulting lanes stop with the steps of
  // this micro-op and the rest of its block not retired.
  std::string stack_atomic(uint32_t i, const std::string& P) const {
    const Uop& o = uops[i];
    const uint32_t p = (uint32_t)((int32_t)stk->k + stk->off[i]), j = p >> 2;
    const bool w32 = o.aux & F_ATOMIC32, fetch = o.aux & F_FETCH;
    const uint32_t op = (uint32_t)o.k;
    const std::string W0 = sv(j), W1 = sv(j + 1);
    const std::string S0 = "v" + std::to_string(2 * o.src), S1 = "v" + std::to_string(2 * o.src + 1);
    const std::string D = vpair(2 * o.dst, 0, 1), S = vpair(2 * o.src, 0, 1);
    const std::string U = P + "u" + std::to_string(i), next = entry_label(P, next_start(i));
    // v[36:37] orig, v[38:39] operand, v[40:41] fetched, v[42:43] result, v[44:45] dst snapshot
    std::string s = "v_mov_b64 v[44:45], " + D + "\nv_mov_b32 v36, " + W0 + "\n" +
                    (w32 ? "v_mov_b32 v37, 0\n" : "v_mov_b32 v37, " + W1 + "\n") +
                    "v_mov_b32 v38, " + S0 + "\n" +
                    (w32 ? "v_mov_b32 v39, 0\n" : "v_mov_b32 v39, " + S1 + "\n") +
                    (fetch ? "v_mov_b64 v[40:41], v[36:37]\n" : "v_mov_b64 v[40:41], 0\n");
    std::string ovf;  // lanes that overflow (vcc), from the operation and the recombination
    switch (op) {
      case 0x00:  // ADD
        s += "v_lshl_add_u64 v[42:43], v[36:37], 0, v[38:39]\n";
        if (!w32)  // signed overflow: both operands' signs differ from the sum's
          s += "v_xor_b32 v46, v37, v43\nv_xor_b32 v47, v39, v43\nv_and_b32 v46, v46, v47\n"
               "v_cmp_gt_i32 vcc, 0, v46\n";
        break;
      case 0x40: s += "v_or_b32 v42, v36, v38\nv_or_b32 v43, v37, v39\n"; break;
      case 0x50: s += "v_and_b32 v42, v36, v38\nv_and_b32 v43, v37, v39\n"; break;
      case 0xa0: s += "v_xor_b32 v42, v36, v38\nv_xor_b32 v43, v37, v39\n"; break;
      case 0xe0: s += "v_mov_b64 v[42:43], v[38:39]\nv_mov_b64 v[40:41], v[36:37]\n"; break;
      default:  // 0xf0 CMPXCHG: compare with r0 (its low word in the 32-bit form)
        s += std::string("v_mov_b32 v46, v0\n") + (w32 ? "v_mov_b32 v47, 0\n" : "v_mov_b32 v47, v1\n") +
             "v_cmp_eq_u64 vcc, v[36:37], v[46:47]\n"
             "v_cndmask_b32 v42, v36, v38, vcc\nv_cndmask_b32 v43, v37, v39, vcc\n";
        break;
    }
    const bool add_ovf = op == 0x00 && !w32;
    if (w32) {  // + (high << 32): overflows when the high word is non-negative and the sum is not
      s += "v_add_u32 v43, v43, " + W1 + "\nv_not_b32 v46, " + W1 + "\nv_and_b32 v46, v46, v43\n"
           "v_cmp_gt_i32 vcc, 0, v46\n";
      ovf = "vcc";
    } else if (add_ovf) {
      ovf = "vcc";
    }
    if (!ovf.empty())
      s += "s_cbranch_vccz .Lnf" + U + "\n"
           "s_mov_b64 s[66:67], exec\ns_mov_b64 exec, vcc\n"
           "v_mov_b32 v30, 4\nv_mov_b32 v28, -1\n"
           "v_subrev_u32 v29, " + std::to_string(t[i].a0) + ", v29\n"
           "s_andn2_b64 exec, s[66:67], vcc\n"
           "s_cbranch_execz " + next + "\n"
           ".Lnf" + U + ":\n";
    s += "v_mov_b32 " + W0 + ", v42\nv_mov_b32 " + W1 + ", v43\n";
    if (op == 0xf0) s += "v_mov_b64 v[0:1], v[40:41]\n";
    if (fetch) s += "v_mov_b64 " + S + ", v[40:41]\n";
    return s + "v_mov_b64 " + D + ", v[44:45]\n";
  }

  // A register-address load of a stack-window program: the lanes whose bytes [a, a + w) overlap
  // the window (a - S0 < k or a + w - 1 - S0 < k, u32, S0 = r10 - k in s57) take the window's bytes
  // instead of the image's (store forwarding); the value v[26:27] is patched byte by byte, each
  // byte's window dword picked by a compare/select chain. The patch is one shared subroutine per
  // access width (overlay_routines, called with s_swappc: return address in s[62:63]), out of
  // line; returns the check and the call.
  mutable uint32_t overlay_widths = 0;  // bit w: the width-w routine is needed
  std::string stack_overlay(const std::string& U, uint32_t w, std::string&) const {
    const uint32_t k = stk->k;
    overlay_widths |= 1u << w;
    return "v_subrev_u32 v44, s57, v36\n"
           "v_add_u32 v45, " + std::to_string(w - 1) + ", v44\n"
           "v_cmp_gt_u32 vcc, " + std::to_string(k) + ", v44\n"
           "v_cmp_gt_u32 s[60:61], " + std::to_string(k) + ", v45\n"
           "s_or_b64 vcc, vcc, s[60:61]\n"
           "s_cbranch_vccz .Lovd" + U + "\n"
           "s_getpc_b64 s[60:61]\n.Lovp" + U + ":\n"
           "s_add_u32 s60, s60, " + overlay_label(w) + "-.Lovp" + U + "\n"
           "s_addc_u32 s61, s61, 0\n"
           "s_swappc_b64 s[62:63], s[60:61]\n"
           ".Lovd" + U + ":\n";
  }
  std::string overlay_label(uint32_t w) const { return ".Lovr" + ovl_tag + "_" + std::to_string(w); }
  std::string ovl_tag;  // unique per statement (set by body)
  // store mode on the var tile loop (body_store, marker fields ovf / tile / dm): stores into the
  // image's bytes [64, 128) go to the packet's overflow image in the workspace instead of
  // deoptimizing the lane; empty on the other statements
  std::string ovf_lo, ovf_hi, tile_s, dm;

  // The overlay routines the statement's loads call (vcc = the lanes to patch).
  std::string overlay_routines() const {
    const uint32_t k = stk ? stk->k : 0;
    std::string o;
    for (uint32_t w = 1; w <= 8; w++) {
      if (!(overlay_widths & (1u << w))) continue;
      o += overlay_label(w) + ":\ns_mov_b64 s[66:67], exec\ns_mov_b64 exec, vcc\n";
      for (uint32_t j = 0; j < w; j++) {
        const std::string T = j < 4 ? "v26" : "v27";
        const uint32_t q = j & 3;
        o += "v_add_u32 v46, " + std::to_string(j) + ", v44\n"
             "v_cmp_gt_u32 s[68:69], " + std::to_string(k) + ", v46\n"
             "v_lshrrev_b32 v47, 2, v46\nv_mov_b32 v48, 0\n";
        for (uint32_t d = 0; d < k / 4; d++)
          o += "v_cmp_eq_u32 vcc, " + std::to_string(d) + ", v47\nv_cndmask_b32 v48, v48, " + sv(d) +
               ", vcc\n";
        uint32_t sel = 0;
        for (uint32_t b = 0; b < 4; b++) sel |= (b == q ? 4u : b) << (8 * b);
        o += "v_and_b32 v49, 3, v46\nv_lshlrev_b32 v49, 3, v49\nv_bfe_u32 v48, v48, v49, 8\n"
             "s_mov_b32 s36, " + hex32(sel) + "\nv_perm_b32 v49, v48, " + T + ", s36\n"
             "v_cndmask_b32_e64 " + T + ", " + T + ", v49, s[68:69]\n";
      }
      o += "s_mov_b64 exec, s[66:67]\ns_setpc_b64 s[62:63]\n";
    }
    return o;
  }

  // kJitRefill with the address's low word in register A instead of v36
  static std::string refill(const std::string& A) {
    std::string r(kJitRefill);
    replace_token(r, "v36", A);
    return r;
  }

  std::string ldx1_loop(uint32_t i, const Marker& m, const std::string& P, std::string& ool) const {
    const TUop& u = t[i];
    const std::string U = P + "u" + std::to_string(i), next = entry_label(P, next_start(i));
    const int64_t off = (int64_t)u.imm;
    std::string s;
    std::string offs;
    if (inline_const(off)) {
      offs = std::to_string(off);
    } else {
      s += "s_mov_b32 s48, " + hex32((uint32_t)u.imm) + "\ns_mov_b32 s49, " +
           hex32((uint32_t)(u.imm >> 32)) + "\n";
      offs = "s[48:49]";
    }
    const std::string D0 = "v" + std::to_string(u.dst2);
    // the address a = src + off in v[36:37]; with off = 0 the source pair itself (the refill
    // reads only its low word and uses v37 as a temporary). A counted loop may name another
    // register holding the same value (addr_src, counted_entry).
    const uint32_t src2 = addr_src[i] >= 0 ? 2 * (uint32_t)addr_src[i] : u.src2;
    std::string A = "v36", AP = "v[36:37]";
    if (off == 0) {
      A = vreg(src2, 0);
      AP = vpair(src2, 0, 1);
    } else {
      s += "v_lshl_add_u64 v[36:37], " + vpair(src2, 0, 1) + ", 0, " + offs + "\n";
    }
    if (!(proven && inb[i]))  // (a load proven to read a packet byte cannot fault)
      s += "v_cmp_gt_u64 vcc, s[52:53], " + AP + "\n"
           "s_andn2_b64 s[64:65], exec, vcc\n"
           "s_cbranch_scc0 .Lok" + U + "\n"
           "s_mov_b64 s[66:67], exec\ns_mov_b64 exec, s[64:65]\n"
           "v_mov_b32 v30, 1\nv_mov_b32 v28, -1\n"
           "v_subrev_u32 v29, " + std::to_string(u.a0) + ", v29\n"
           "s_andn2_b64 exec, s[66:67], s[64:65]\n"
           "s_cbranch_execz " + next + "\n"
           ".Lok" + U + ":\n";
    if (zwin && qcache) return s + ldx1_qword_cache(U, A, D0, m, ool);
    if (zwin) return s + ldx1_zero_window(U, A, D0, m, ool);
    s += "v_sub_u32 v42, " + A + ", v22\n"
         "v_cmp_lt_u32_e64 s[60:61], " + A + ", v31\n"
         "v_cndmask_b32_e64 v43, 0, v42, s[60:61]\n"
         "v_cmp_le_u32 vcc, 64, v43\n"
         "s_cbranch_vccnz .Lrf" + U + "\n"
         ".Lrfb" + U + ":\n"
         "v_xad_u32 v42, v35, v43, v34\n"
         "ds_read_u8 v26, v42\n"
         "s_waitcnt lgkmcnt(0)\n"
         "v_cndmask_b32_e64 v26, 0, v26, s[60:61]\n"
         ".Lfarb" + U + ":\n";
    if (stk)  // store forwarding from the stack window
      s += (A == "v36" ? std::string() : "v_mov_b32 v36, " + A + "\n") + "v_mov_b32 v27, 0\n" +
           stack_overlay(U, 1, ool);
    s += "v_bfi_b32 " + D0 + ", s56, v26, " + D0 + "\n";
    ool += ".Lrf" + U + ":\n"
           "s_mov_b64 s[68:69], vcc\n"
           "s_cmp_eq_u32 " + m.aligned + ", 0\n"
           "s_cbranch_scc1 .Lfar" + U + "\n" + refill(A) +
           "v_sub_u32 v42, " + A + ", v22\n"
           "v_cndmask_b32_e64 v43, 0, v42, s[60:61]\n"
           "s_branch .Lrfb" + U + "\n"
           ".Lfar" + U + ":\n"
           "v_min_u32 v43, 63, v43\n"
           "v_xad_u32 v42, v35, v43, v34\n"
           "ds_read_u8 v26, v42\n"
           "s_mov_b64 s[66:67], exec\ns_mov_b64 exec, s[68:69]\n"
           "v_and_b32 v46, -4, " + A + "\nv_mov_b32 v47, 0\n"
           "v_lshl_add_u64 v[44:45], v[32:33], 0, v[46:47]\n"
           "global_load_dword v49, v[44:45], off\n"
           "s_waitcnt vmcnt(0) lgkmcnt(0)\n"
           "v_and_b32 v48, 3, " + A + "\nv_lshlrev_b32 v48, 3, v48\n"
           "v_bfe_u32 v26, v49, v48, 8\n"
           "s_mov_b64 exec, s[66:67]\n"
           "v_cndmask_b32_e64 v26, 0, v26, s[60:61]\n"
           "s_branch .Lfarb" + U + "\n";
    return s;
  }

  // Zero-past-len windows (zwin: loop programs whose register-address loads are all one byte
  // wide, so this handler is the only reader and refiller of the LDS windows): every window byte
  // at or past the packet's length is kept zero -- the prologue clears them after the DMA
  // (window_zero_prologue), each refill before its LDS writes (refill_zero) -- so the load needs
  // no a < len test: it refills when a - WB >= 64 (u32; a lane past its packet refills a window
  // of zeros) and reads its byte. 4 VALU per byte fewer than the masked form.
  std::string ldx1_zero_window(const std::string& U, const std::string& A, const std::string& D0,
                               const Marker& m, std::string& ool) const {
    std::string s = "v_sub_u32 v42, " + A + ", v22\n"
                    "v_cmp_le_u32 vcc, 64, v42\n"
                    "s_cbranch_vccnz .Lrf" + U + "\n"
                    ".Lrfb" + U + ":\n"
                    "v_xad_u32 v42, v35, v42, v34\n"
                    "ds_read_u8 v26, v42\n"
                    "s_waitcnt lgkmcnt(0)\n"
                    ".Lfarb" + U + ":\n"
                    "v_bfi_b32 " + D0 + ", s56, v26, " + D0 + "\n";
    ool += ".Lrf" + U + ":\n"
           "s_mov_b64 s[68:69], vcc\n"
           "s_cmp_eq_u32 " + m.aligned + ", 0\n"
           "s_cbranch_scc1 .Lfar" + U + "\n" + refill_zero(A, U) +
           "v_sub_u32 v42, " + A + ", v22\n"
           "s_branch .Lrfb" + U + "\n"
           // unaligned tile: its window [0, 64) was staged with zeros past len and is never
           // refilled; lanes outside it read the packet's dword from HBM (a < len) or zero
           ".Lfar" + U + ":\n"
           "s_mov_b64 s[66:67], exec\n"
           "v_min_u32 v43, 63, v42\n"
           "v_xad_u32 v42, v35, v43, v34\n"
           "ds_read_u8 v26, v42\n"
           "s_waitcnt lgkmcnt(0)\n"
           "s_mov_b64 exec, s[68:69]\n"
           "v_mov_b32 v26, 0\n"
           "v_cmp_lt_u32 vcc, " + A + ", v31\n"
           "s_and_b64 exec, exec, vcc\n"
           "s_cbranch_execz .Lfz" + U + "\n"
           "v_and_b32 v46, -4, " + A + "\nv_mov_b32 v47, 0\n"
           "v_lshl_add_u64 v[44:45], v[32:33], 0, v[46:47]\n"
           "global_load_dword v49, v[44:45], off\n"
           "s_waitcnt vmcnt(0)\n"
           "v_and_b32 v48, 3, " + A + "\nv_lshlrev_b32 v48, 3, v48\n"
           "v_bfe_u32 v26, v49, v48, 8\n"
           ".Lfz" + U + ":\n"
           "s_mov_b64 exec, s[66:67]\n"
           "s_branch .Lfarb" + U + "\n";
    return s;
  }

  // zwin: the DMA'd windows of an aligned tile hold whatever follows a packet shorter than 64
  // bytes; clear those bytes once per tile (lanes with len - WB < 64; skipped when none).
  std::string window_zero_prologue(const Marker& m, const std::string& P) const {
    if (!zwin) return "";
    const std::string L = ".L" + P + "pz";
    std::string z = "s_cmp_eq_u32 " + m.aligned + ", 0\ns_cbranch_scc1 " + L + "\n"
                    "v_sub_u32 v37, v31, v22\n"
                    "v_cmp_gt_i32 vcc, 64, v37\n"
                    "s_cbranch_vccz " + L + "\n"
                    "s_mov_b64 exec, vcc\n";
    for (uint32_t c = 0; c < 4; c++) {
      z += "v_xad_u32 v43, v35, " + std::to_string(16 * c) + ", v34\n"
           "ds_read_b128 v[44:47], v43\ns_waitcnt lgkmcnt(0)\n";
      for (uint32_t d = 0; d < 4; d++) z += zero_dword("v" + std::to_string(44 + d), 16 * c + 4 * d);
      z += "ds_write_b128 v43, v[44:47]\n";
    }
    return z + "s_waitcnt lgkmcnt(0)\ns_mov_b64 exec, -1\n" + L + ":\n";
  }

  // zwin + an 8-byte per-lane cache: the lane keeps window bytes [TAG, TAG + 8) (TAG 8-aligned,
  // in v55; 0x80000000 = empty) in v[52:53], so seven of eight bytes of a scan are one 64-bit
  // shift with no LDS access; a miss reads the qword with one ds_read_b64 (refilling the window
  // first if the qword is outside it). Bytes past len read as zero from the zeroed windows. Tiles
  // with unaligned packets (no refills) take ldx1_zero_window's far path every time.
  std::string ldx1_qword_cache(const std::string& U, const std::string& A, const std::string& D0,
                               const Marker& m, std::string& ool) const {
    // (a VOPC result is 0 for inactive lanes, so vcc is exactly the missing lanes; the byte at
    // cache offset x = a - TAG < 8 is selector x of v_perm over {v53, v52}; its other selector
    // bytes are 0, and only the low byte is merged)
    std::string s = "v_sub_u32 v42, " + A + ", v55\n"
                    "v_cmp_le_u32 vcc, 8, v42\n"
                    "s_cbranch_vccnz .Lqm" + U + "\n"
                    ".Lqh" + U + ":\n"
                    "v_perm_b32 v26, v53, v52, v42\n"
                    ".Lqd" + U + ":\n"
                    "v_bfi_b32 " + D0 + ", s56, v26, " + D0 + "\n";
    ool += ".Lqm" + U + ":\n"
           "s_mov_b64 s[68:69], vcc\n"
           "s_mov_b64 s[64:65], exec\n"
           "s_cmp_eq_u32 " + m.aligned + ", 0\n"
           "s_cbranch_scc1 .Lqf" + U + "\n"
           "s_mov_b64 exec, s[68:69]\n"
           "v_and_b32 v55, -8, " + A + "\n"
           "v_sub_u32 v42, v55, v22\n"
           "v_cmp_lt_u32 vcc, 56, v42\n"
           "s_cbranch_vccz .Lqn" + U + "\n"
           "s_mov_b64 s[68:69], vcc\n" + refill_zero(A, U) +
           "v_and_b32 v55, -8, " + A + "\n"
           "v_sub_u32 v42, v55, v22\n"
           ".Lqn" + U + ":\n"
           "v_xad_u32 v42, v35, v42, v34\n"
           "ds_read_b64 v[52:53], v42\n"
           "s_waitcnt lgkmcnt(0)\n"
           "s_mov_b64 exec, s[64:65]\n"
           "v_sub_u32 v42, " + A + ", v55\n"
           "s_branch .Lqh" + U + "\n"
           // unaligned tile: the window [0, 64) or the packet's dword in HBM, byte by byte
           ".Lqf" + U + ":\n"
           "v_sub_u32 v42, " + A + ", v22\n"
           "v_cmp_le_u32 s[68:69], 64, v42\n"
           "s_mov_b64 s[66:67], exec\n"
           "v_min_u32 v43, 63, v42\n"
           "v_xad_u32 v42, v35, v43, v34\n"
           "ds_read_u8 v26, v42\n"
           "s_waitcnt lgkmcnt(0)\n"
           "s_and_b64 exec, exec, s[68:69]\n"
           "s_cbranch_execz .Lqz" + U + "\n"
           "v_mov_b32 v26, 0\n"
           "v_cmp_lt_u32 vcc, " + A + ", v31\n"
           "s_and_b64 exec, exec, vcc\n"
           "s_cbranch_execz .Lqz" + U + "\n"
           "v_and_b32 v46, -4, " + A + "\nv_mov_b32 v47, 0\n"
           "v_lshl_add_u64 v[44:45], v[32:33], 0, v[46:47]\n"
           "global_load_dword v49, v[44:45], off\n"
           "s_waitcnt vmcnt(0)\n"
           "v_and_b32 v48, 3, " + A + "\nv_lshlrev_b32 v48, 3, v48\n"
           "v_bfe_u32 v26, v49, v48, 8\n"
           ".Lqz" + U + ":\n"
           "s_mov_b64 exec, s[66:67]\n"
           "s_branch .Lqd" + U + "\n";
    return s;
  }

  // Zero the bytes at or past the packet's length in dword register R holding window bytes
  // [o, o + 4) of a window starting at packet offset WB, given v37 = len - WB (signed):
  // clamp(len - WB - o, 0, 4) bytes stay. Temporaries v26, v27, v42; vcc.
  static std::string zero_dword(const std::string& R, uint32_t o) {
    return "v_subrev_u32 v26, " + std::to_string(o) + ", v37\n"
           "v_med3_i32 v26, v26, 0, 4\n"
           "v_lshlrev_b32 v27, 3, v26\n"
           "v_bfe_u32 v42, " + R + ", 0, v27\n"
           "v_cmp_eq_u32 vcc, 4, v26\n"
           "v_cndmask_b32 " + R + ", v42, " + R + ", vcc\n";
  }

  // kJitRefill with the bytes past the packet's length zeroed before the LDS writes (only for
  // lanes whose new window passes the packet's end: a uniform branch skips it otherwise).
  std::string refill_zero(const std::string& A, const std::string& U) const {
    if (prefetch) return refill_prefetch(A, U);
    std::string r = refill(A);
    const size_t w = r.find("v_xad_u32 v37, v35, 0, v34\nds_write_b128");
    if (w == std::string::npos) return "; (refill layout changed)\ns_trap 2\n";
    static const char* regs[4][4] = {{"v44", "v45", "v46", "v47"}, {"v48", "v49", "v50", "v51"},
                                     {"v52", "v53", "v54", "v55"}, {"v38", "v39", "v40", "v41"}};
    std::string z = "v_sub_u32 v37, v31, v22\n"
                    "v_cmp_gt_i32 vcc, 64, v37\n"
                    "s_cbranch_vccz .Lrz" + U + "\n"
                    "s_mov_b64 s[62:63], exec\ns_mov_b64 exec, vcc\n";
    for (uint32_t c = 0; c < 4; c++)
      for (uint32_t d = 0; d < 4; d++) z += zero_dword(regs[c][d], 16 * c + 4 * d);
    z += "s_mov_b64 exec, s[62:63]\n.Lrz" + U + ":\n";
    r.insert(w, z);
    return r;
  }

  // ---- window refills with a prefetch (zwin loop programs in aligned tiles) ----
  // A forward scan refills each lane's window every 64 bytes. Per-lane refills (kJitRefill: four
  // 16-byte loads per lane, each wave instruction touching 64 packets' lines, then a wait) cost
  // the checksum batch 214 of its 331 us (diagnostics: 117 us with the loads removed, 200 with
  // every refill reading one resident line). So the refills here are transposed and prefetched:
  //  * transposed: in wave instruction k, lane L loads 16 bytes of packet q = 16k + L/4 -- four
  //    lanes read one packet's 64 contiguous bytes, 16 lines per instruction instead of 64 (the
  //    layout of the tile's first window DMA); the lane holding that chunk writes it to q's
  //    window slot (address WIN - 48 L + 1024 k: lane-linear, and the chunk it loads is the one
  //    the window swizzle puts in that slot, (L ^ L/16) & 3). q's refill flag, hit flag, bytes
  //    left and window address come from lane q by ds_bpermute;
  //  * prefetched: each refill also loads every refilled packet's next 64 bytes [WB + 64,
  //    WB + 128) into v[56:71] (held transposed); the next refill waits for them (they have had
  //    the whole window's scan to arrive) and uses them where the new window is that one (a
  //    forward scan: v23 = the prefetched window's offset); lanes whose window moved elsewhere
  //    load theirs first, as does each lane's first refill. The statement's end waits for loads
  //    still in flight.
  // Chunks wholly past the packet are not loaded; bytes at or past len are zeroed before the
  // window writes (zwin). Clobbers v22 (the new WB of the refilled lanes), v23, v26, v27,
  // v37-v51, v54, v[56:71], s[60:63], s[66:67], vcc; exec restored (s[68:69]: the refilled lanes).
  static constexpr uint32_t kRemBias = 1u << 25;  // bytes left (signed, |.| < 2^24) + bias

  // Lane constants (exec = all lanes): v38 = L, v39 = 4 (L / 4) (bpermute index of packet q for
  // k = 0), v40 = the chunk offset 16 ((L ^ L/16) & 3), v54 = v40 + kRemBias, v41 = WIN - 48 L.
  static std::string transpose_consts() {
    return "v_mbcnt_lo_u32_b32 v38, -1, 0\nv_mbcnt_hi_u32_b32 v38, -1, v38\n"
           "v_and_b32 v39, -4, v38\n"
           "v_lshrrev_b32 v40, 4, v38\nv_xor_b32 v40, v38, v40\nv_and_b32 v40, 3, v40\n"
           "v_lshlrev_b32 v40, 4, v40\n"
           "v_add_u32 v54, " + hex32(kRemBias) + ", v40\n"
           "v_mul_u32_u24 v41, 48, v38\nv_sub_u32 v41, v34, v41\n";
  }

  // Slot k of this lane: v48 = packet q's packed word (bit 30 refill, bit 31 hit, low 30 bits
  // bytes left + kRemBias), v[50:51] = q's window address (with_addr), s[62:63] = slots whose
  // packet refills. exec = all lanes.
  static std::string slot_of(uint32_t k, bool with_addr) {
    const std::string o = " offset:" + std::to_string(64 * k) + "\n";
    std::string r = "ds_bpermute_b32 v48, v39, v44" + o;
    if (with_addr) r += "ds_bpermute_b32 v50, v39, v46" + o + "ds_bpermute_b32 v51, v39, v47" + o;
    return r + "s_waitcnt lgkmcnt(0)\n"
               "v_lshrrev_b32 v37, 30, v48\n"
               "v_cmp_ne_u32 s[62:63], 0, v37\n"
               "v_and_b32 v49, 0x3fffffff, v48\n";
  }

  // Transposed loads of every slot (packet refilling, chunk start + extra < bytes left; with
  // miss_only, only packets that missed the prefetch) into v[56+4k : 59+4k], from q's window
  // address + chunk offset + extra. exec = all lanes, and again after.
  static std::string transposed_loads(uint32_t extra, bool miss_only, uint32_t base = 56) {
    std::string r;
    for (uint32_t k = 0; k < 4; k++) {
      r += slot_of(k, true);
      if (miss_only) r += "v_cmp_eq_u32 s[62:63], 1, v37\n";  // refill, not hit
      r += (extra ? "v_add_u32 v37, " + std::to_string(extra) + ", v54\n"
                    "v_cmp_lt_u32 vcc, v37, v49\n"
                  : std::string("v_cmp_lt_u32 vcc, v54, v49\n")) +
           "s_and_b64 exec, vcc, s[62:63]\n"
           "v_add_co_u32 v42, vcc, v50, v40\nv_addc_co_u32 v43, vcc, 0, v51, vcc\n"
           "global_load_dwordx4 v[" + std::to_string(base + 4 * k) + ":" +
           std::to_string(base + 3 + 4 * k) + "], v[42:43], off" +
           (extra ? " offset:" + std::to_string(extra) : std::string()) + "\n"
           "s_mov_b64 exec, -1\n";
    }
    return r;
  }

  // Per-lane words for the slots (exec = the lanes in s[68:69] for the refill values, all lanes
  // before): v44 = packed word (0 for lanes not refilling), v[46:47] = BASE + v22.
  static std::string pack_lane(bool hit_in_vcc) {
    return std::string(hit_in_vcc ? "v_cndmask_b32_e64 v37, 0, 1, vcc\nv_lshlrev_b32 v37, 31, v37\n"
                                  : "v_mov_b32 v37, 0\n") +
           "v_sub_u32 v44, v31, v22\n"
           "v_add_u32 v44, " + hex32(kRemBias) + ", v44\n"
           "v_or_b32 v44, 0x40000000, v44\n"
           "v_or_b32 v44, v44, v37\n"
           // (v22 is -64 after a budget restart: sign-extended)
           "v_mov_b32 v46, v22\n"
           "v_ashrrev_i32 v47, 31, v46\n"
           "v_lshl_add_u64 v[46:47], v[32:33], 0, v[46:47]\n";
  }

  // No window prefetched yet (v23, the packet offset of the window held in v[56:71], is a value
  // no window base takes): the first refill of each lane loads its window and starts the
  // prefetching, so a loop program that never leaves its first window reads nothing more.
  std::string prefetch_prologue(const Marker&, const std::string&) const {
    if (!prefetch) return "";
    std::string r;
    r += "v_mov_b32 v23, 0x80000001\n";
    return r;
  }

  std::string refill_prefetch(const std::string& A, const std::string& U) const {
    std::string r = "s_mov_b64 s[66:67], exec\ns_mov_b64 exec, -1\n" + transpose_consts() +
                    "v_mov_b32 v44, 0\n"
                    "s_mov_b64 exec, s[68:69]\n"
                    "v_and_b32 v22, -16, " + A + "\n"
                    "v_cmp_eq_u32 vcc, v22, v23\n"
                    "s_andn2_b64 s[60:61], s[68:69], vcc\n" + pack_lane(true) +
                    "v_add_u32 v23, 64, v22\n"  // the window this refill prefetches
                    "s_mov_b64 exec, -1\n"
                    "s_waitcnt vmcnt(0)\n"
                    "s_cmp_eq_u64 s[60:61], 0\n"
                    "s_cbranch_scc1 .Lpfh" + U + "\n" + transposed_loads(0, true) +
                    "s_waitcnt vmcnt(0)\n"
                    ".Lpfh" + U + ":\n";
    // per slot: bytes at or past len zeroed, the window slot written, and the packet's next 64
    // bytes loaded into the same registers (a DS write reads its data VGPRs at issue)
    for (uint32_t k = 0; k < 4; k++) {
      const std::string K = std::to_string(k), R0 = std::to_string(56 + 4 * k),
                        R3 = std::to_string(59 + 4 * k);
      r += slot_of(k, true) +
           "v_sub_u32 v37, v49, v54\n"   // bytes left past this chunk's start
           "s_mov_b64 exec, s[62:63]\n"
           "v_cmp_gt_i32 vcc, 16, v37\n"
           "s_cbranch_vccz .Lnz" + K + U + "\n"
           "s_mov_b64 exec, vcc\n";
      for (uint32_t d = 0; d < 4; d++) r += zero_dword("v" + std::to_string(56 + 4 * k + d), 4 * d);
      r += "s_mov_b64 exec, s[62:63]\n"
           ".Lnz" + K + U + ":\n"
           "ds_write_b128 v41, v[" + R0 + ":" + R3 + "] offset:" + std::to_string(1024 * k) + "\n"
           "v_add_u32 v37, 64, v54\n"
           "v_cmp_lt_u32 vcc, v37, v49\n"
           "s_and_b64 exec, exec, vcc\n"
           "v_add_co_u32 v42, vcc, v50, v40\nv_addc_co_u32 v43, vcc, 0, v51, vcc\n"
           "global_load_dwordx4 v[" + R0 + ":" + R3 + "], v[42:43], off offset:64\n"
           "s_mov_b64 exec, -1\n";
    }
    return r + "s_mov_b64 exec, s[66:67]\n";
  }

  // Whether code text names any of v[lo..hi] (single registers or ranges).
  static bool touches(const std::string& text, uint32_t lo, uint32_t hi) {
    for (size_t q = 0; (q = text.find('v', q)) != std::string::npos; q++) {
      if (q > 0 && (isalnum((unsigned char)text[q - 1]) || text[q - 1] == '_')) continue;
      uint32_t a, b;
      if (sscanf(text.c_str() + q, "v[%u:%u]", &a, &b) == 2) {
        if (!(b < lo || a > hi)) return true;
      } else if (isdigit((unsigned char)text[q + 1]) && sscanf(text.c_str() + q, "v%u", &a) == 1) {
        if (a >= lo && a <= hi) return true;
      }
    }
    return false;
  }

  // A register-address load in the fixed-slot layout (ldx in gen_tile.py, non-loop form; every
  // packet a multiple of 16 bytes >= 64 long, the window its first 64 bytes): in bounds is
  // a < mem (64-bit, so a nonzero high word fails) and a + width <= mem; window accesses read the
  // one to three dwords they span (ds_read_u8 for one byte); accesses past the window read the
  // packet's dwords from HBM (zeros past its end) out of line.
  // var (the var kernel's stack statement): packets of any length, so the bytes at or past LEN
  // read as zero (main.rs:16) -- masked after either path, before the stack overlay.
  // loop (the loop kernel's stack statement): the window holds packet bytes [WB, WB + 64) (v22,
  // moved by the one-byte loads' refills); this load reads it at a - WB and never refills.
  std::string ldx_fixed(uint32_t i, bool one, const std::string& P, std::string& ool,
                        bool var = false, bool loop = false) const {
    // store mode: the window's bytes at or past LEN are zeros in LDS and may have been stored to,
    // so only bytes read from the packet past the window are masked by LEN; an access that starts
    // inside the window and ends past it deoptimizes its lane (its low bytes may be stored ones)
    const bool smode = stk && stk->any_dyn && !loop;
    const TUop& u = t[i];
    const uint32_t w = one ? 1u : u.width;
    const std::string U = P + "u" + std::to_string(i), next = entry_label(P, next_start(i));
    const int64_t off = (int64_t)u.imm;
    std::string s, offs;
    if (inline_const(off)) {
      offs = std::to_string(off);
    } else {
      s += "s_mov_b32 s48, " + hex32((uint32_t)u.imm) + "\ns_mov_b32 s49, " +
           hex32((uint32_t)(u.imm >> 32)) + "\n";
      offs = "s[48:49]";
    }
    const std::string D0 = "v" + std::to_string(u.dst2);
    s += "v_lshl_add_u64 v[36:37], " + vpair(u.src2, 0, 1) + ", 0, " + offs + "\n"
         "v_cmp_gt_u64_e64 s[60:61], s[52:53], v[36:37]\n"
         "v_add_u32 v38, " + std::to_string(w) + ", v36\n"
         "v_cmp_ge_u32_e64 s[62:63], s52, v38\n"
         "s_and_b64 vcc, s[60:61], s[62:63]\n"
         "s_andn2_b64 s[64:65], exec, vcc\n"
         "s_cbranch_scc0 .Lok" + U + "\n"
         "s_mov_b64 s[66:67], exec\ns_mov_b64 exec, s[64:65]\n"
         "v_cndmask_b32_e64 v30, 1, 2, s[60:61]\n"
         "v_mov_b32 v28, -1\n"
         "v_subrev_u32 v29, " + std::to_string(u.a0) + ", v29\n"
         "s_andn2_b64 exec, s[66:67], s[64:65]\n"
         "s_cbranch_execz " + next + "\n"
         ".Lok" + U + ":\n" +
         (loop ? "v_sub_u32 v41, v36, v22\nv_cmp_lt_u32_e64 s[62:63], " + std::to_string(64 - w) +
                     ", v41\n"
               : std::string("v_cmp_lt_u32_e64 s[62:63], 64, v38\n")) +
         "s_and_b64 s[68:69], s[62:63], exec\n"
         "s_cbranch_scc1 .Lfar" + U + "\n";
    // the window bytes a .. a + w - 1 (at window offset O: inside [0, 64) here) into v26 (v27)
    const std::string O = loop ? "v41" : "v36";
    std::string win;
    if (w == 1) {
      win = "v_xad_u32 v42, v35, " + O + ", v34\nds_read_u8 v26, v42\ns_waitcnt lgkmcnt(0)\n";
    } else {
      win = "v_and_b32 v42, -4, " + O + "\nv_xad_u32 v43, v35, v42, v34\nds_read_b32 v49, v43\n"
            "v_add_u32 v44, 4, v42\nv_min_u32 v44, 60, v44\nv_xad_u32 v44, v35, v44, v34\n"
            "ds_read_b32 v50, v44\n";
      if (w == 8)
        win += "v_add_u32 v45, 8, v42\nv_min_u32 v45, 60, v45\nv_xad_u32 v45, v35, v45, v34\n"
               "ds_read_b32 v51, v45\n";
      win += "s_waitcnt lgkmcnt(0)\nv_alignbyte_b32 v26, v50, v49, v36\n";
      if (w == 8) win += "v_alignbyte_b32 v27, v51, v50, v36\n";
    }
    s += win + ".Lmrg" + U + ":\n";
    // the valid bytes: min(8, LEN - a) (0 when a >= LEN), the rest shifted out
    const std::string lenmask =
        std::string(w <= 4 ? "v_mov_b32 v27, 0\n" : "") +
        "v_sub_u32 v46, v31, v36\nv_cmp_lt_u32 vcc, v36, v31\nv_cndmask_b32 v46, 0, v46, vcc\n"
        "v_min_u32 v46, 8, v46\nv_lshlrev_b32 v46, 3, v46\nv_sub_u32 v46, 64, v46\n"
        "v_lshlrev_b64 v[26:27], v46, v[26:27]\nv_lshrrev_b64 v[26:27], v46, v[26:27]\n"
        // (a shift by 64 is one by 0: an access at or past LEN is zeroed by the select)
        "v_cndmask_b32 v26, 0, v26, vcc\nv_cndmask_b32 v27, 0, v27, vcc\n";
    if (var && !smode) s += lenmask;
    if (stk) s += stack_overlay(U, w, ool);
    if (w == 1 || w == 2)
      s += "s_mov_b32 s42, " + std::string(w == 1 ? "0xff" : "0xffff") + "\nv_bfi_b32 " + D0 +
           ", s42, v26, " + D0 + "\n";
    else if (w == 4)
      s += "v_mov_b32 " + D0 + ", v26\n";
    else
      s += "v_mov_b64 " + vpair(u.dst2, 0, 1) + ", v[26:27]\n";
    // out of line: lanes whose access ends past the window (in bounds: their bytes come from
    // the packet's dwords that hold a packet byte, zeros past its end)
    std::string far = ".Lfar" + U + ":\n" + (loop ? "v_min_u32 v41, 63, v41\n" : "") + win +
                      "s_mov_b64 s[66:67], exec\ns_mov_b64 exec, s[68:69]\n";
    if (smode && dm.empty())  // straddling the window's end: deoptimize (they leave both lane sets)
      far += "v_cmp_gt_u32 vcc, 64, v36\ns_and_b64 vcc, vcc, exec\ns_cbranch_vccz .Lnd" + U + "\n"
             "s_andn2_b64 s[66:67], s[66:67], vcc\ns_andn2_b64 s[68:69], s[68:69], vcc\n"
             "s_mov_b64 exec, vcc\nv_mov_b32 v30, 0x80\nv_mov_b32 v28, -1\n"
             "s_mov_b64 exec, s[68:69]\n.Lnd" + U + ":\n";
    if (smode && !dm.empty() && w > 1) {
      // straddling the window's end (a < 64 < a + w, so 57 <= a <= 63): bytes [a, 64) from the
      // window in LDS (stored ones included), bytes [64, a + w) from the overflow image (lanes
      // that stored there: the dirty mask) or the packet (zeros at or past LEN); the value is the
      // bytes [56, 72) shifted down by a - 56
      far += "v_cmp_gt_u32 vcc, 64, v36\ns_and_b64 s[60:61], vcc, exec\n"
             "s_cbranch_scc0 .Lnd" + U + "\n"
             "s_mov_b64 exec, s[60:61]\n"
             // (s[62:63]: the lanes whose overflow block 0 is filled)
             "v_and_b32 v40, 1, v23\nv_cmp_ne_u32_e64 s[62:63], 0, v40\n"
             "v_mov_b32 v42, 56\nv_xad_u32 v43, v35, v42, v34\nds_read_b32 v49, v43\n"
             "v_mov_b32 v42, 60\nv_xad_u32 v43, v35, v42, v34\nds_read_b32 v50, v43\n"
             "v_mov_b32 v46, 0\nv_mov_b32 v47, 0\n"
             // clean lanes: the packet's dwords at 64 and 68 that start before LEN
             "s_andn2_b64 exec, s[60:61], s[62:63]\n"
             "s_cbranch_execz .Lsc" + U + "\n"
             "s_mov_b64 s[64:65], exec\n"
             "v_cmp_lt_u32 vcc, 64, v31\ns_and_b64 exec, s[64:65], vcc\n"
             "global_load_dword v46, v[32:33], off offset:64\n"
             "v_cmp_lt_u32 vcc, 0x44, v31\ns_and_b64 exec, s[64:65], vcc\n"
             "global_load_dword v47, v[32:33], off offset:68\n"
             "s_mov_b64 exec, s[64:65]\ns_waitcnt vmcnt(0)\n"
             // (the bytes at or past LEN: min(8, LEN - 64) valid, 0 when LEN <= 64)
             "v_subrev_u32 v42, 64, v31\nv_cmp_lt_u32 vcc, 64, v31\nv_cndmask_b32 v42, 0, v42, vcc\n"
             "v_min_u32 v42, 8, v42\nv_lshlrev_b32 v42, 3, v42\nv_sub_u32 v42, 64, v42\n"
             "v_lshlrev_b64 v[46:47], v42, v[46:47]\nv_lshrrev_b64 v[46:47], v42, v[46:47]\n"
             "v_cndmask_b32 v46, 0, v46, vcc\nv_cndmask_b32 v47, 0, v47, vcc\n"
             ".Lsc" + U + ":\n"
             // dirty lanes: the overflow image's first two dwords
             "s_and_b64 exec, s[60:61], s[62:63]\n"
             "s_cbranch_execz .Lsd" + U + "\n" + ovf_addr() +
             "global_load_dword v46, v[44:45], off sc1\n"
             "global_load_dword v47, v[44:45], off offset:4 sc1\n"
             "s_waitcnt vmcnt(0)\n"
             ".Lsd" + U + ":\n"
             "s_mov_b64 exec, s[60:61]\n"
             "s_waitcnt lgkmcnt(0)\n"
             // dwords [56, 72) = v49 v50 v46 v47; a - 56 = 4q + (a & 3)
             "v_cmp_gt_u32 vcc, 60, v36\n"
             "v_cndmask_b32 v42, v50, v49, vcc\nv_cndmask_b32 v43, v46, v50, vcc\n"
             "v_cndmask_b32 v48, v47, v46, vcc\n"
             "v_alignbyte_b32 v26, v43, v42, v36\nv_alignbyte_b32 v27, v48, v43, v36\n"
             // (these lanes are done: out of the far set; back with the others at the merge)
             "s_andn2_b64 s[68:69], s[68:69], s[60:61]\n"
             "s_mov_b64 exec, s[68:69]\n.Lnd" + U + ":\n";
    } else if (smode && !dm.empty()) {
      far += ".Lnd" + U + ":\n";
    }
    if (smode && !dm.empty()) {
      // lanes that filled a block of their overflow image (the dirty mask) whose access touches
      // one (the blocks bf = v39 and bl = v43 of its first and last byte): the other block filled
      // too if it is not, then the bytes read from the image; an access ending past the image (E,
      // mem_size > kOvfEnd) deoptimizes. The rest read the packet below.
      far += "s_and_b64 s[60:61], s[68:69], " + dm + "\n"
             "s_cbranch_scc0 .Lnv" + U + "\n"
             "s_mov_b64 exec, s[60:61]\n"
             "v_subrev_u32 v39, 64, v36\nv_lshrrev_b32 v39, 6, v39\n"
             "v_add_u32 v43, -65, v38\nv_lshrrev_b32 v43, 6, v43\n"
             "v_lshrrev_b32 v40, v39, v23\nv_lshrrev_b32 v42, v43, v23\nv_or_b32 v40, v40, v42\n"
             "v_and_b32 v40, 1, v40\nv_cmp_ne_u32 vcc, 0, v40\n"
             "s_and_b64 s[60:61], s[60:61], vcc\n"
             "s_cbranch_scc0 .Lnv" + U + "\n" + ovf_end() +
             "v_mov_b32 v42, s48\nv_cmp_lt_u32 vcc, v42, v38\n"
             "s_and_b64 vcc, vcc, s[60:61]\n"
             "s_cbranch_vccz .Lnq" + U + "\n"
             "s_andn2_b64 s[60:61], s[60:61], vcc\n"
             "s_andn2_b64 s[66:67], s[66:67], vcc\n"
             "s_andn2_b64 s[68:69], s[68:69], vcc\n"
             "s_mov_b64 exec, vcc\nv_mov_b32 v30, 0x80\nv_mov_b32 v28, -1\n"
             ".Lnq" + U + ":\n"
             "s_mov_b64 exec, s[60:61]\n"
             "s_cbranch_execz .Lnv" + U + "\n" + ovf_ensure("s[60:61]", "f" + U) +
             "v_mov_b32 v39, v43\n" + ovf_ensure("s[60:61]", "l" + U) + ovf_addr() +
             "v_add_u32 v46, -64, v36\nv_and_b32 v46, -4, v46\nv_mov_b32 v47, 0\n"
             "v_lshl_add_u64 v[44:45], v[44:45], 0, v[46:47]\n"
             "global_load_dword v49, v[44:45], off sc1\n";
      if (w > 1) far += "global_load_dword v50, v[44:45], off offset:4 sc1\n";
      if (w == 8) far += "global_load_dword v51, v[44:45], off offset:8 sc1\n";
      far += "s_waitcnt vmcnt(0)\nv_mov_b32 v27, 0\n";
      if (w == 1)
        far += "v_and_b32 v48, 3, v36\nv_lshlrev_b32 v48, 3, v48\nv_bfe_u32 v26, v49, v48, 8\n";
      else
        far += "v_alignbyte_b32 v26, v50, v49, v36\n" +
               std::string(w == 8 ? "v_alignbyte_b32 v27, v51, v50, v36\n" : "");
      far += "s_andn2_b64 s[68:69], s[68:69], s[60:61]\n"
             ".Lnv" + U + ":\n"
             "s_mov_b64 exec, s[68:69]\n";
    }
    far += "v_mov_b32 v26, 0\nv_mov_b32 v27, 0\n"
                      "v_cmp_lt_u32 vcc, v36, v31\ns_and_b64 exec, s[68:69], vcc\n"
                      "s_cbranch_execz .Lfd" + U + "\n"
                      "v_and_b32 v46, -4, v36\nv_mov_b32 v47, 0\n"
                      "v_lshl_add_u64 v[44:45], v[32:33], 0, v[46:47]\n"
                      "s_mov_b64 s[64:65], exec\n"
                      "global_load_dword v49, v[44:45], off\n"
                      "v_mov_b32 v50, 0\nv_mov_b32 v47, 0\n";
    // (the packet's dwords in v49, v50, v47 -- v47 is free once the address is formed -- so the
    // code stays inside v[0:50], the occupancy variant's registers)
    const int nd = w == 8 ? 3 : (w == 1 ? 1 : 2);
    for (int k = 1; k < nd; k++)
      far += "v_add_u32 v48, " + std::to_string(4 * k) + ", v46\nv_cmp_lt_u32 vcc, v48, v31\n"
             "s_and_b64 exec, s[64:65], vcc\n"
             "global_load_dword v" + std::string(k == 1 ? "50" : "47") + ", v[44:45], off offset:" +
             std::to_string(4 * k) + "\ns_mov_b64 exec, s[64:65]\n";
    far += "s_waitcnt vmcnt(0)\n";
    if (w == 1)
      far += "v_and_b32 v48, 3, v36\nv_lshlrev_b32 v48, 3, v48\nv_bfe_u32 v26, v49, v48, 8\n";
    else
      far += "v_alignbyte_b32 v26, v50, v49, v36\n" +
             std::string(w == 8 ? "v_alignbyte_b32 v27, v47, v50, v36\n" : "");
    if (smode) far += lenmask;  // (exec: the far lanes inside the image and before LEN)
    far += ".Lfd" + U + ":\ns_mov_b64 exec, s[66:67]\ns_branch .Lmrg" + U + "\n";
    ool += far;
    return s;
  }

  // One copy of the program. fast: window loads from preloaded registers (ldxk_fast).
  bool copy(const Marker& m, const std::string& P, bool fast, std::string& main,
            std::string& ool) {
    wcache = 0;
    for (uint32_t i = 0; i < n; i++) {
      if (start[i] && target[i]) wcache = 0;  // (store mode's chunk cache, ldxk_lds)
      if (start[i] && far_mode && !ool.empty() &&
          (size_t)std::count(main.begin() + std::min(island_from, main.size()), main.end(), '\n') >
              kIslandLines) {
        const std::string L = ".L" + P + "isl" + std::to_string(i);
        main += "s_branch " + L + "\n" + ool + L + ":\n";
        ool.clear();
        island_from = main.size();
      }
      if (start[i]) {
        main += ".L" + P + "b" + std::to_string(i) + ":\n";
        const std::string pm = pm_reg(i);
        // (every lane parked here is in the mask; with exec empty, one instruction takes the mask
        // into exec and clears it: mask = exec = 0, exec = old mask | 0)
        if (i < cm_of.size() && cm_of[i])  // (a complement target: the region's survivors)
          main += std::string("s_mov_b64 exec, ") + kCmP + "\n";
        else if (!pm.empty())
          main += i > 0 && clears_exec(i - 1)
                      ? "s_or_saveexec_b64 " + pm + ", " + pm + "\n"
                      : "s_or_b64 exec, exec, " + pm + "\ns_mov_b64 " + pm + ", 0\n";
        else if (target[i] && !loops && i > 0 && clears_exec(i - 1))  // (exec is empty here)
          main += "s_mov_b64 exec, -1\nv_cmpx_eq_u32 vcc, " + std::to_string(i) + ", v28\n";
        else if (target[i])
          main += "s_or_saveexec_b64 s[64:65], -1\nv_cmp_eq_u32 vcc, " + std::to_string(i) +
                  ", v28\ns_or_b64 exec, s[64:65], vcc\n";
        // (far mode: a skip past many micro-ops -- a long straight-line run with no target, e.g.
        // the exact copy's one-micro-op blocks -- may pass s_cbranch's reach: a long jump)
        const uint32_t nt = next_target(i);
        const std::string skip = ".L" + P + "b" + std::to_string(nt);
        // (a mask target whose block is register ALU work and a jump runs it with an empty exec
        // instead of skipping: nothing happens, its jump's own skip follows -- one instruction
        // less per rule of a rule chain, whose masks are seldom empty)
        if (i < cm_start.size() && cm_start[i])  // (the start of a complement region)
          main += std::string("s_mov_b64 ") + kCmP + ", exec\n";
        if (!((pm_reg(i).size() || (i < cm_of.size() && cm_of[i])) && alu_block(i)))
          main += far_mode && nt - i > kFarSkipUops ? jmp("execz", skip)
                                                    : "s_cbranch_execz " + skip + "\n";
        if (loops && hoist[i] != -2) main += "v_mov_b32 v28, " + std::to_string(hoist[i]) + "\n";
        if (loops && proven && !counted_entry(m, i, P, main, ool)) return false;
        if (loops) main += ".L" + P + "body" + std::to_string(i) + ":\n";
        if (loops)  // biased counter: the add's carry-out is the budget test (budget_check)
          main += "v_add_co_u32_e32 v29, vcc, " + std::to_string(t[i].blen) + ", v29\n" +
                  budget_check(i, P);
        else
          main += "v_add_u32 v29, " + std::to_string(t[i].blen) + ", v29\n";
      }
      if (!emit_uop(m, i, P, fast, main, ool)) return false;
    }
    main += ".L" + P + "b" + std::to_string(n) + ":\n";
    if (loops) main += "v_mov_b32 v28, -1\n";  // lanes past the end are done
    return true;
  }

  // ---- counted single-block loops (the proven copy) ----
  // A loop whose block L..J runs `add rI, 1` once, leaves only through its back edge
  // `jlt rI, rN` (or `jgt rN, rI`; both signed, Q2) with rN unchanged in the block, and holds no
  // micro-op that can fault, runs max(1, rN - rI) times from its entry when rI and rN are in
  // [0, 2^24] there (the range analysis): the steps its lanes will retire are known at the entry.
  // If no lane's total passes the budget, they are added once and the block runs as a copy
  // without the per-iteration step count and budget check (out of line, prefix PU); otherwise
  // the ordinary block runs. Returns false only on a compiler error.
  bool counted_entry(const Marker& m, uint32_t L, const std::string& P, std::string& main,
                     std::string& ool) {
    if (!loops || exact || hoist[L] == -2 || ranges.empty()) return true;
    uint32_t J = L;
    while (J + 1 < n && !start[J + 1]) J++;
    const Uop& jb = uops[J];
    uint32_t rI, rN;
    if (jb.op == U_JLT && (jb.aux & F_SRC) && (uint32_t)jb.x == L) {
      rI = jb.dst, rN = jb.src;
    } else if (jb.op == U_JGT && (jb.aux & F_SRC) && (uint32_t)jb.x == L) {
      rI = jb.src, rN = jb.dst;
    } else {
      return true;
    }
    if (rI == rN || rI > 10 || rN > 10) return true;
    uint32_t incs = 0;
    for (uint32_t i = L; i < J; i++) {
      const Uop& u = uops[i];
      const bool alu = u.op <= U_ARSH32 && u.op != U_DIV64 && u.op != U_MOD64 && u.op != U_DIV32 &&
                       u.op != U_MOD32 && u.op != U_ARSH64 && u.op != U_ARSH32;
      const bool ok = alu || (u.op >= U_ZX16 && u.op <= U_BSWAP64) || u.op == U_LDIMM ||
                      (u.op == U_LDX && u.aux == 1 && inb[i]);
      if (!ok || u.dst == rN) return true;  // (not a counted loop)
      if (u.dst == rI) {
        if (u.op != U_ADD64 || (u.aux & F_SRC) || u.k != 1) return true;
        incs++;
      }
    }
    if (incs != 1) return true;
    const AbsVal &vi = ranges[L][rI], &vn = ranges[L][rN];
    if (vi.hi > kLenMax || vn.hi > kLenMax) return true;
    // the entry's step total blen * max(1, rN - rI) <= blen * 2^24 must fit the 32-bit counter
    if ((uint64_t)t[L].blen * kLenMax >= (1ull << 32)) return true;
    // an address copy `mov rA, rZ; add rA, rC` with rZ = 0 whose value only the block's one-byte
    // loads read (rA dead at both successors, rC unchanged until those loads): the loads take
    // rC as their base and the copy is not emitted
    std::vector<char> skip(n, 0);
    const std::vector<uint32_t> lv = live();
    for (uint32_t i = L; i + 1 < J; i++) {
      const Uop &a = uops[i], &b = uops[i + 1];
      if (a.op != U_MOV64 || !(a.aux & F_SRC) || ranges[i][a.src].hi != 0 || b.op != U_ADD64 ||
          !(b.aux & F_SRC) || b.dst != a.dst || b.src == a.dst)
        continue;
      const uint32_t rA = a.dst, rC = b.src;
      if ((lv[L] >> rA) & 1 || (lv[J + 1] >> rA) & 1) continue;  // (lv[n]: r0)
      bool ok = true;
      std::vector<uint32_t> loads;
      for (uint32_t k = i + 2; k <= J && ok; k++) {
        const Uop& u = uops[k];
        const bool reads_a = (u.dst == rA && u.op != U_MOV64 && u.op != U_MOV32 && u.op != U_LDIMM) ||
                             ((u.aux & F_SRC) && u.src == rA && u.op != U_LDX) || u.dst == rA;
        if (u.op == U_LDX && u.src == rA && u.dst != rA) loads.push_back(k);
        else if (reads_a) ok = false;
        if (u.dst == rC) {  // rC written (an LDX into rC included, which itself still reads the
                            // old value): later loads would see another value
          for (uint32_t q = k + 1; q <= J && ok; q++) ok = !(uops[q].op == U_LDX && uops[q].src == rA);
          break;
        }
      }
      if (!ok || loads.empty()) continue;
      skip[i] = skip[i + 1] = 1;
      for (uint32_t k : loads) addr_src[k] = (int)rC;
      i++;
    }
    const std::string PU = P + "n" + std::to_string(L) + "_", Ls = std::to_string(L);
    std::string grp;
    const int g = counted_group(m, L, J, rI, rN, skip, P, PU, grp);
    if (g < 0) return false;
    main += "; counted loop: max(1, r" + std::to_string(rN) + " - r" + std::to_string(rI) +
            ") runs of " + std::to_string(t[L].blen) + " steps" +
            (g ? ", 8 per pass from one qword while 8 are left" : "") + "\n"
            "v_sub_u32 v46, v" + std::to_string(2 * rN) + ", v" + std::to_string(2 * rI) + "\n"
            "v_max_i32 v46, 1, v46\n"
            // the trip count may be 2^24 itself (r2 = LEN = mem_size = 2^24), past the 24-bit
            // multiplier: blen * (trip - 1) + blen
            "v_add_u32 v46, -1, v46\n"
            "v_mul_u32_u24 v46, " + std::to_string(t[L].blen) + ", v46\n"
            "v_add_u32 v46, " + std::to_string(t[L].blen) + ", v46\n"
            "v_add_co_u32_e32 v46, vcc, v46, v29\n"
            "s_cbranch_vccnz .L" + P + "body" + Ls + "\n"
            "v_mov_b32 v29, v46\n"
            "s_branch .L" + PU + (g ? "gent" : "body" + Ls) + "\n";
    std::string c = ".L" + PU + "body" + Ls + ":\n";
    bool ok = true;
    for (uint32_t i = L; i <= J && ok; i++)
      if (!skip[i]) ok = emit_uop(m, i, PU, false, c, ool);
    for (uint32_t i = L; i <= J; i++) addr_src[i] = -1;
    if (!ok) return false;
    ool += c + "s_branch .L" + P + "b" + std::to_string(J + 1) + "\n" + grp;
    return true;
  }

  // Whether text names an SGPR in [lo, hi] (sN or s[a:b]).
  static bool names_sgpr(const std::string& text, uint32_t lo, uint32_t hi) {
    return names_reg(text, 's', lo, hi);
  }
  // Whether text names register kind k ('s' or 'v') in [lo, hi] (kN or k[a:b]).
  static bool names_reg(const std::string& text, char k, uint32_t lo, uint32_t hi) {
    for (size_t p = 0; p + 1 < text.size(); p++) {
      if (text[p] != k || (p && (isalnum((unsigned char)text[p - 1]) || text[p - 1] == '_' ||
                                   text[p - 1] == '.')))
        continue;
      size_t q = p + 1;
      const bool range = text[q] == '[';
      if (range) q++;
      if (q >= text.size() || !isdigit((unsigned char)text[q])) continue;
      const uint32_t a = (uint32_t)strtoul(text.c_str() + q, nullptr, 10);
      uint32_t b = a;
      if (range) {
        const size_t colon = text.find(':', q);
        if (colon == std::string::npos) continue;
        b = (uint32_t)strtoul(text.c_str() + colon + 1, nullptr, 10);
      } else {
        while (q < text.size() && isdigit((unsigned char)text[q])) q++;
        if (q < text.size() && (isalpha((unsigned char)text[q]) || text[q] == '_')) continue;
      }
      if (a <= hi && b >= lo) return true;
    }
    return false;
  }

  // ---- counted loops in passes of 8 iterations (the proven copy, zero windows + qword cache) ----
  // A counted loop (counted_entry) whose only load is the one-byte `ldxb rD, [rI + d]` (d fixed,
  // rI read as the iteration starts; the base may be an address copy's source, addr_src) reads
  // bytes a0 .. a0 + 7 in its next 8 iterations. A lane with rN - rI >= 8 left runs those 8
  // iterations without any exit test -- the back edge is the loop's only way out and is taken 7
  // times in a row -- so a pass replicates the block 8 times (the jump dropped, rI's increments
  // summed into one add when nothing else reads rI) and takes the loads from one ds_read_b64 of
  // the lane's window: byte k is merged into rD's low byte as the one-byte load merges (Q1), one
  // v_perm (or v_bfi) per byte. A pass needs a0 8-aligned and [a0, a0 + 8) inside the window (zero past len):
  // lanes outside it are refilled first in an aligned tile; misaligned lanes (or, in an unaligned
  // tile, lanes past its window) run one ordinary iteration instead and retry. Lanes with fewer
  // than 8 left run the ordinary counted copy; lanes that finished in passes skip it. The steps
  // were already added at the entry. s[41:47] (micro-op field SGPRs none of the block's code names;
  // checked) hold the byte selectors, the loop's lanes and the lanes that ran a pass. Returns 1 with the code (out of
  // line, entered at .L<PU>gent) in out, 0 when the loop does not qualify, -1 on a compiler error.
  int counted_group(const Marker& m, uint32_t L, uint32_t J, uint32_t rI, uint32_t rN,
                    const std::vector<char>& skip, const std::string& P, const std::string& PU,
                    std::string& out, bool p16 = true) {
    if (!zwin || !qcache) return 0;
    int ld = -1, inc = -1;
    bool others_read_i = false;
    for (uint32_t i = L; i < J; i++) {
      if (skip[i]) continue;
      const Uop& u = uops[i];
      if (u.op == U_LDX) {
        if (ld >= 0) return 0;
        ld = (int)i;
      } else if (u.dst == rI) {
        inc = (int)i;  // (counted_entry: the one write of rI is `add rI, 1`)
      } else if ((u.aux & F_SRC) && u.src == rI) {
        others_read_i = true;
      }
    }
    if (ld < 0 || inc < 0) return 0;
    const uint32_t base = addr_src[ld] >= 0 ? (uint32_t)addr_src[ld] : uops[ld].src;
    const int64_t d = (int64_t)t[ld].imm + (inc < ld ? 1 : 0);
    if (base != rI || uops[ld].dst == rI || d < -(1 << 20) || d > (1 << 20)) return 0;
    const std::string G = ".L" + PU + "g", vI = "v" + std::to_string(2 * rI),
                      vN = "v" + std::to_string(2 * rN), D0 = "v" + std::to_string(uops[ld].dst * 2);
    std::string A = vI, uc, uo;  // uc / uo: the micro-ops' code (checked for s[41:47])
    std::string body16;          // the 16-byte pass's micro-op code (checked for v[48:51])
    const bool fold = !others_read_i;
    // The byte-sum idiom: a block of exactly `ldxb rD, [rI + d]; add rS, rD` (+ the increment,
    // folded) adds rD = (rD & ~0xff) | b_k for each byte b_k, so a pass of nb bytes adds
    // nb * (rD & ~0xff) + the bytes' sum (v_sad_u8 against zero: four bytes per instruction;
    // exact mod 2^64) and leaves rD's low byte at the last byte -- a few VALU instead of a
    // dependent select + 64-bit add per byte.
    int sum_add = -1;
    if (fold) {
      int others = 0;
      for (uint32_t i = L; i < J; i++) {
        if (skip[i] || (int)i == inc || (int)i == ld) continue;
        const Uop& u = uops[i];
        if (u.op == U_NOP) continue;  // (promote_slots' folded slot accesses)
        others++;
        if ((int)i > ld && u.op == U_ADD64 && (u.aux & F_SRC) && u.src == uops[ld].dst &&
            u.dst != uops[ld].dst && u.dst != rI && u.dst != rN)  // (the add after the load)
          sum_add = (int)i;
      }
      if (others != 1) sum_add = -1;
    }
    const std::string D1 = "v" + std::to_string(uops[ld].dst * 2 + 1);
    // nb copies of the block, the load of copy k taking byte k & 3 of dword src[k / 4]
    auto pass = [&](uint32_t nb, const std::vector<std::string>& src, const std::string& tag,
                    std::string& c) {
      if (sum_add >= 0) {
        const std::string S = vpair(2 * uops[sum_add].dst, 0, 1);
        c += "v_sad_u8 v26, " + src[0] + ", 0, 0\n";
        for (size_t q = 1; q < src.size(); q++) c += "v_sad_u8 v26, " + src[q] + ", 0, v26\n";
        c += "v_mov_b32 v27, 0\n"
             "v_and_b32 v42, 0xffffff00, " + D0 + "\n"
             "v_mov_b32 v43, " + D1 + "\n"
             "v_lshlrev_b64 v[42:43], " + std::string(nb == 16 ? "4" : "3") + ", v[42:43]\n"
             "v_lshl_add_u64 v[42:43], v[26:27], 0, v[42:43]\n"
             "v_lshl_add_u64 " + S + ", v[42:43], 0, " + S + "\n"
             "v_perm_b32 " + D0 + ", " + D0 + ", " + src.back() + ", s43\n"
             "v_lshl_add_u64 " + vpair(2 * rI, 0, 1) + ", " + vpair(2 * rI, 0, 1) + ", 0, " +
             std::to_string(nb) + "\n"
             "s_branch " + G + "top\n";
        return true;
      }
      for (uint32_t k = 0; k < nb; k++) {
        const std::string Pk = PU + tag + std::to_string(k) + "_";
        for (uint32_t i = L; i < J; i++) {
          if (skip[i] || (fold && (int)i == inc)) continue;
          if ((int)i == ld) {
            const std::string& Q = src[k / 4];
            if ((k & 3) == 0)
              c += "v_bfi_b32 " + D0 + ", s56, " + Q + ", " + D0 + "\n";
            else  // byte k & 3 of Q into byte 0, bytes 1-3 kept (selector 0x070605XX in s41..s43)
              c += "v_perm_b32 " + D0 + ", " + D0 + ", " + Q + ", s" + std::to_string(40 + (k & 3)) +
                   "\n";
            continue;
          }
          std::string mc, mo;
          if (!emit_uop(m, i, Pk, false, mc, mo)) return false;
          uc += mc;
          uo += mo;
          if (nb == 16) body16 += mc + mo;
          c += mc;
        }
      }
      if (fold)
        c += "v_lshl_add_u64 " + vpair(2 * rI, 0, 1) + ", " + vpair(2 * rI, 0, 1) + ", 0, " +
             std::to_string(nb) + "\n";
      c += "s_branch " + G + "top\n";
      return true;
    };
    std::string coop;
    // (on the deep kernel only: compile_into_template sends a program with such a loop there)
    if (sum_add >= 0 && deep_regs) coop = coop_sum_compact(J, rI, rN, d, ld, sum_add, G, P);
    std::string c = (coop.empty() ? G + "ent:\n" : coop + G + "ent2:\n") +
                    "s_mov_b64 s[44:45], exec\ns_mov_b64 s[46:47], 0\n"
                    "s_mov_b32 s41, 0x07060501\ns_mov_b32 s42, 0x07060502\n"
                    "s_mov_b32 s43, 0x07060503\n" + G + "top:\n"
                    "s_mov_b64 exec, s[44:45]\n"
                    "v_sub_u32 v46, " + vN + ", " + vI + "\n"
                    "v_cmp_le_i32 vcc, 8, v46\n"
                    "s_and_b64 exec, exec, vcc\n"
                    "s_cbranch_execz " + G + "rem\n"
                    "s_or_b64 s[46:47], s[46:47], exec\n";
    if (d != 0) {
      c += "v_add_u32 v36, " + std::to_string(d) + ", " + vI + "\n";
      A = "v36";
    }
    c += "v_sub_u32 v42, " + A + ", v22\n";
    if (p16) {
      // passes of 16 while every lane has 16 left and a0 16-aligned inside the window (one
      // ds_read_b128; its second qword becomes the qword cache)
      c += "v_cmp_gt_i32 vcc, 16, v46\n"
           "s_cbranch_vccnz " + G + "p8\n"
           "v_and_b32 v43, 0xffffffcf, v42\n"
           "v_cmp_ne_u32 vcc, 0, v43\n"
           "s_cbranch_vccnz " + G + "c16\n" + G + "r16:\n"
           "v_xad_u32 v43, v35, v42, v34\n"
           "ds_read_b128 v[48:51], v43\n"
           "v_add_u32 v55, 8, " + A + "\n"
           "s_waitcnt lgkmcnt(0)\n"
           "v_mov_b32 v52, v50\nv_mov_b32 v53, v51\n";
      if (!pass(16, {"v48", "v49", "v50", "v51"}, "h", c)) return -1;
      c += G + "c16:\n"
           "v_and_b32 v43, 15, v42\n"
           "v_cmp_ne_u32 vcc, 0, v43\n"
           "s_cbranch_vccnz " + G + "p8\n"
           "s_cmp_eq_u32 " + m.aligned + ", 0\n"
           "s_cbranch_scc1 " + G + "p8\n"
           "v_cmp_le_u32 vcc, 64, v42\n"
           "s_mov_b64 s[68:69], vcc\n" + refill_zero(A, PU + "h") +
           "v_sub_u32 v42, " + A + ", v22\n"
           "s_branch " + G + "r16\n" + G + "p8:\n";
    }
    c += "v_and_b32 v43, 0xffffffc7, v42\n"
         "v_cmp_ne_u32 vcc, 0, v43\n"
         "s_cbranch_vccnz " + G + "chk\n" + G + "rd:\n"
         "v_xad_u32 v43, v35, v42, v34\n"
         "ds_read_b64 v[52:53], v43\n"
         "v_mov_b32 v55, " + A + "\n"
         "s_waitcnt lgkmcnt(0)\n";
    if (!pass(8, {"v52", "v53"}, "g", c)) return -1;
    // lanes failing the pass's test (vcc): misaligned ones run one ordinary iteration; aligned
    // ones past the window are refilled, or run one iteration in an unaligned tile
    c += G + "chk:\n"
         "v_and_b32 v43, 7, v42\n"
         "v_cmp_ne_u32 vcc, 0, v43\n"
         "s_cbranch_vccnz " + G + "one\n"
         "v_cmp_le_u32 vcc, 64, v42\n"
         "s_cmp_eq_u32 " + m.aligned + ", 0\n"
         "s_cbranch_scc1 " + G + "one\n"
         "s_mov_b64 s[68:69], vcc\n" + refill_zero(A, PU + "g") +
         "v_sub_u32 v42, " + A + ", v22\n"
         "s_branch " + G + "rd\n" + G + "one:\ns_mov_b64 exec, vcc\n";
    for (uint32_t i = L; i < J; i++) {
      if (skip[i]) continue;
      std::string mc;
      if (!emit_uop(m, i, PU + "g1x_", false, mc, uo)) return -1;
      uc += mc;
      c += mc;
    }
    c += "s_branch " + G + "top\n" + G + "rem:\n"
         "s_mov_b64 exec, s[44:45]\n"
         "v_cmp_ne_u32 vcc, " + vN + ", " + vI + "\n"
         "s_andn2_b64 s[46:47], s[46:47], vcc\n"
         "s_andn2_b64 exec, exec, s[46:47]\n"
         "s_cbranch_execz .L" + P + "b" + std::to_string(J + 1) + "\n"
         "s_branch .L" + PU + "body" + std::to_string(L) + "\n";
    if (names_sgpr(uc + uo, 41, 47)) return 0;
    if (p16 && names_reg(body16, 'v', 48, 51))  // the block's code uses the 16-byte pass's registers
      return counted_group(m, L, J, rI, rN, skip, P, PU, out, false);
    out = c + uo;
    return 1;
  }

  // ---- the byte-sum idiom over a whole range (counted_group's entry) ----
  // A counted byte-sum loop adds, over its n = rN - rI iterations, n * (rD & ~0xff) + the sum of
  // the bytes [a0, a0 + n) (a0 = rI + d, every one proven a packet byte: prove_loads), leaves rD's
  // low byte at the last byte and rI at rI + n. Lanes with at least kCoopMin bytes to go get that
  // result without scanning their windows: the wave sums their ranges together straight from HBM.
  static constexpr uint32_t kCoopMin = 128;

  // ---- coop_sum_compact (the deep kernel) ----
  // Only the C cooperating lanes' packets are walked: lane ranks
  // 0..C-1 (mbcnt over the cooperating mask; the other lanes take C..63, so ds_permute_b32 makes a
  // full permutation srcl[rank] = lane), and LPP lanes read one packet, 16 bytes each, with LPP
  // chosen from C so that four load instructions cover every packet: C <= 16 -> 16 lanes (256
  // bytes per packet per round), C <= 32 -> 8 lanes (one 128-byte line), else 4 lanes (64 bytes).
  // So a tile of 32 long packets among 32 short ones fills every lane of every load instead of
  // half. Three buffers (v[56:71], v[72:87], v[88:103]): the next two rounds' loads are in flight
  // while a round is summed. After the rounds, each packet's LPP partial sums are added (DPP
  // within a row) and moved to the packet's lane by ds_bpermute. Uses (deep kernel only; every
  // prefetch stage is invalidated after) v[88:96] for the per-lane ranges and ranks before the
  // rounds, v[97:100] after them, v104 for the window's part, s41 for C and s[46:47], besides
  // v[23:71] (the refill prefetch registers, drained and invalidated first; the qword cache and
  // the prefetch tags are invalidated after) and s[60:67].
  std::string coop_sum_compact(uint32_t J, uint32_t rI, uint32_t rN, int64_t d, int ld,
                               int sum_add, const std::string& G, const std::string& P) const {
    const std::string vI = "v" + std::to_string(2 * rI), vN = "v" + std::to_string(2 * rN),
                      D0 = "v" + std::to_string(uops[ld].dst * 2),
                      D1 = "v" + std::to_string(uops[ld].dst * 2 + 1),
                      S = vpair(2 * uops[sum_add].dst, 0, 1), I2 = vpair(2 * rI, 0, 1),
                      C = G + "k";
    auto v = [](uint32_t r) { return "v" + std::to_string(r); };
    auto vp = [](uint32_t r) { return "v[" + std::to_string(r) + ":" + std::to_string(r + 1) + "]"; };
    auto num = [](int64_t x) { return std::to_string(x); };
    std::string r = G + "ent:\n"
                    "; the byte sum of whole ranges, compacted (coop_sum_compact)\n"
                    "v_sub_u32 v46, " + vN + ", " + vI + "\n"
                    "v_cmp_le_i32 vcc, " + num(kCoopMin) + ", v46\n"
                    "s_and_b64 s[60:61], exec, vcc\n"
                    "s_cbranch_scc0 " + G + "ent2\n"
                    "s_mov_b64 s[62:63], exec\n"
                    "s_mov_b64 exec, -1\n"
                    "s_waitcnt vmcnt(0)\n"  // (refill prefetches may be in flight)
                    // per lane: v[88:89] = (BASE + a0) & ~15, v90 = (BASE + a0) & 15, v91 = v90 + n
                    // on the cooperating lanes (0 elsewhere: nothing is read for them)
                    "v_sub_u32 v91, " + vN + ", " + vI + "\n" +
                    (d ? "v_add_u32 v88, " + num(d) + ", " + vI + "\n" : "v_mov_b32 v88, " + vI + "\n") +
                    "v_mov_b32 v89, 0\n"
                    "v_lshl_add_u64 v[88:89], v[32:33], 0, v[88:89]\n"
                    "v_and_b32 v90, 15, v88\n"
                    "v_and_b32 v88, -16, v88\n"
                    "v_add_u32 v91, v90, v91\n"
                    "v_cndmask_b32_e64 v91, 0, v91, s[60:61]\n"
                    "v_mov_b32 v104, 0\n" +
                    coop_window_part(vI, vN, d, G) +
                    // ranks: v93 = cooperating lanes below this one; srcl (v92) by forward permute
                    "v_mbcnt_lo_u32_b32 v95, -1, 0\nv_mbcnt_hi_u32_b32 v95, -1, v95\n"
                    "v_mbcnt_lo_u32_b32 v93, s60, 0\nv_mbcnt_hi_u32_b32 v93, s61, v93\n"
                    "s_bcnt1_i32_b64 s41, s[60:61]\n"
                    "v_sub_u32 v24, v95, v93\n"
                    "v_add_u32 v24, s41, v24\n"
                    "v_cndmask_b32_e64 v24, v24, v93, s[60:61]\n"
                    "v_lshlrev_b32 v24, 2, v24\n"
                    "ds_permute_b32 v92, v24, v95\n"
                    "s_waitcnt lgkmcnt(0)\n"
                    "s_cmp_gt_u32 s41, 32\n"
                    "s_cbranch_scc1 " + C + "4\n"
                    "s_cmp_gt_u32 s41, 16\n"
                    "s_cbranch_scc1 " + C + "8\n";
    // one variant per LPP (lanes per packet): PPI = 64 / LPP packets per load instruction
    for (uint32_t lpp : {16u, 8u, 4u}) {
      const uint32_t ppi = 64 / lpp, T = 16 * lpp, lg = lpp == 16 ? 4 : lpp == 8 ? 3 : 2,
                     lgp = lpp == 16 ? 2 : lpp == 8 ? 3 : 4;
      const std::string K = C + std::to_string(lpp);
      r += K + ":\n"
           "v_lshrrev_b32 v24, " + num(lg) + ", v95\n"
           "v_lshlrev_b32 v24, 2, v24\n";
      // slot k's packet: rank k * PPI + lane / LPP
      const char* sr[4] = {"v25", "v26", "v27", "v23"};
      for (uint32_t k = 0; k < 4; k++)
        r += std::string("ds_bpermute_b32 ") + sr[k] + ", v24, v92" +
             (k ? " offset:" + num(4 * ppi * k) : std::string()) + "\n";
      r += "s_waitcnt lgkmcnt(0)\n";
      for (uint32_t k = 0; k < 4; k++) r += std::string("v_lshlrev_b32 ") + sr[k] + ", 2, " + sr[k] + "\n";
      for (uint32_t k = 0; k < 4; k++)
        r += std::string("ds_bpermute_b32 ") + v(36 + 2 * k) + ", " + sr[k] + ", v88\n" +
             "ds_bpermute_b32 " + v(37 + 2 * k) + ", " + sr[k] + ", v89\n" +
             "ds_bpermute_b32 " + v(44 + k) + ", " + sr[k] + ", v90\n" +
             "ds_bpermute_b32 " + v(48 + k) + ", " + sr[k] + ", v91\n";
      r += "v_and_b32 v96, " + num(lpp - 1) + ", v95\n"
           "v_lshlrev_b32 v96, 4, v96\n"
           "s_waitcnt lgkmcnt(0)\n";
      for (uint32_t k = 0; k < 4; k++)
        r += "v_add_co_u32 " + v(36 + 2 * k) + ", vcc, " + v(36 + 2 * k) + ", v96\n"
             "v_addc_co_u32 " + v(37 + 2 * k) + ", vcc, 0, " + v(37 + 2 * k) + ", vcc\n"
             "v_sub_u32 " + v(44 + k) + ", " + v(44 + k) + ", v96\n"
             "v_sub_u32 " + v(48 + k) + ", " + v(48 + k) + ", v96\n"
             "v_mov_b32 " + v(52 + k) + ", 0\n";
      // the loads of round s64 + m T into the buffer at `base` (m > 0: s65 = s64 + m T)
      auto loads = [&](uint32_t base, uint32_t m) {
        std::string q = m ? "s_add_u32 s65, s64, " + num(m * T) + "\n" : std::string();
        for (uint32_t k = 0; k < 4; k++)
          q += "v_cmp_lt_i32 vcc, " + std::string(m ? "s65" : "s64") + ", " + v(48 + k) + "\n"
               "s_mov_b64 exec, vcc\n"
               "global_load_dwordx4 v[" + num(base + 4 * k) + ":" + num(base + 3 + 4 * k) + "], " +
               vp(36 + 2 * k) + ", off" + (m ? " offset:" + num(m * T) : std::string()) + "\n"
               "s_mov_b64 exec, -1\n";
        return q;
      };
      auto sums = [&](uint32_t base, const std::string& tag) {
        std::string q;
        for (uint32_t k = 0; k < 4; k++) {
          const std::string Kk = K + tag + std::to_string(k), A = v(52 + k);
          q += "v_cmp_ge_i32 vcc, s64, " + v(44 + k) + "\n"
               "v_subrev_u32 v24, 16, " + v(48 + k) + "\n"
               "v_cmp_le_i32_e64 s[66:67], s64, v24\n"
               "s_and_b64 s[66:67], s[66:67], vcc\n"
               "v_cmp_lt_i32 vcc, s64, " + v(48 + k) + "\n"
               "s_andn2_b64 vcc, vcc, s[66:67]\n"
               "s_mov_b64 exec, s[66:67]\n";
          for (uint32_t dw = 0; dw < 4; dw++)
            q += "v_sad_u8 " + A + ", " + v(base + 4 * k + dw) + ", 0, " + A + "\n";
          q += "s_mov_b64 exec, vcc\n"
               "s_cbranch_execz " + Kk + "s\n"
               "v_subrev_u32 v24, s64, " + v(44 + k) + "\n"
               "v_subrev_u32 v25, s64, " + v(48 + k) + "\n";
          for (uint32_t dw = 0; dw < 4; dw++) {
            const std::string Dw = v(base + 4 * k + dw), o4 = num(4 * dw);
            q += "v_subrev_u32 v26, " + o4 + ", v24\nv_med3_i32 v26, v26, 0, 4\n"
                 "v_subrev_u32 v27, " + o4 + ", v25\nv_med3_i32 v27, v27, 0, 4\n"
                 "v_sub_u32 v27, v27, v26\nv_max_i32 v27, 0, v27\n"
                 "v_lshlrev_b32 v27, 3, v27\nv_lshlrev_b32 v26, 3, v26\n"
                 "v_bfm_b32 v23, v27, v26\n"
                 "v_cmp_eq_u32 s[66:67], 32, v27\n"
                 "v_cndmask_b32_e64 v23, v23, -1, s[66:67]\n"
                 "v_and_b32 " + Dw + ", " + Dw + ", v23\n"
                 "v_sad_u8 " + A + ", " + Dw + ", 0, " + A + "\n";
          }
          q += Kk + "s:\ns_mov_b64 exec, -1\n";
        }
        return q;
      };
      // (s[46:47] = T: VOP3 takes no literal on gfx950)
      const std::string next =
          "v_lshl_add_u64 " + vp(36) + ", " + vp(36) + ", 0, s[46:47]\n"
          "v_lshl_add_u64 " + vp(38) + ", " + vp(38) + ", 0, s[46:47]\n"
          "v_lshl_add_u64 " + vp(40) + ", " + vp(40) + ", 0, s[46:47]\n"
          "v_lshl_add_u64 " + vp(42) + ", " + vp(42) + ", 0, s[46:47]\n"
          "s_add_u32 s64, s64, " + num(T) + "\n"
          "v_max3_i32 v24, v48, v49, v50\nv_max_i32 v24, v24, v51\n"
          "v_cmp_lt_i32 vcc, s64, v24\n";
      // three rounds in flight (v[56:71], v[72:87], v[88:103]): a round is summed while the
      // next two are loading (two rounds: slower, removed in round 5)
      r += "s_mov_b32 s64, 0\ns_mov_b32 s46, " + num(T) + "\ns_mov_b32 s47, 0\n" + loads(56, 0);
      r += loads(72, 1) + K + "w:\n" + loads(88, 2) + "s_waitcnt vmcnt(8)\n" + sums(56, "a") +
           next + "s_cbranch_vccz " + K + "x\n" + loads(56, 2) + "s_waitcnt vmcnt(8)\n" +
           sums(72, "b") + next + "s_cbranch_vccz " + K + "x\n" + loads(72, 2) +
           "s_waitcnt vmcnt(8)\n" + sums(88, "c") + next + "s_cbranch_vccnz " + K + "w\n";
      r += K + "x:\ns_waitcnt vmcnt(0)\n";
      // each packet's LPP partial sums: quads, then rows (lane LPP * j + src of packet j)
      for (uint32_t k = 0; k < 4; k++) {
        const std::string A = v(52 + k);
        r += "s_nop 1\nv_add_u32_dpp " + A + ", " + A + ", " + A +
             " quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
             "s_nop 1\nv_add_u32_dpp " + A + ", " + A + ", " + A +
             " quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n";
        if (lpp >= 8)
          r += "s_nop 1\nv_add_u32_dpp " + A + ", " + A + ", " + A +
               " row_shr:4 row_mask:0xf bank_mask:0xf\n";
        if (lpp == 16)
          r += "s_nop 1\nv_add_u32_dpp " + A + ", " + A + ", " + A +
               " row_shr:8 row_mask:0xf bank_mask:0xf\n";
      }
      const uint32_t src_off = lpp == 16 ? 12 : lpp == 8 ? 4 : 0;
      // the cooperating lane of rank q: slot q / PPI, lane LPP * (q % PPI) + src_off
      r += "v_mbcnt_lo_u32_b32 v93, s60, 0\nv_mbcnt_hi_u32_b32 v93, s61, v93\n"  // (the ranks again)
           "v_and_b32 v24, " + num(ppi - 1) + ", v93\n"
           "v_lshlrev_b32 v24, " + num(lg + 2) + ", v24\n" +
           (src_off ? "v_add_u32 v24, " + num(4 * src_off) + ", v24\n" : std::string());
      for (uint32_t k = 0; k < 4; k++)
        r += "ds_bpermute_b32 " + v(97 + k) + ", v24, " + v(52 + k) + "\n";
      r += "v_lshrrev_b32 v25, " + num(lgp) + ", v93\n"
           "s_waitcnt lgkmcnt(0)\n";
      for (uint32_t k = 1; k < 4; k++)
        r += "v_cmp_eq_u32 vcc, " + num(k) + ", v25\n"
             "v_cndmask_b32 v97, v97, " + v(97 + k) + ", vcc\n";
      r += "s_branch " + C + "fin\n";
    }
    r += C + "fin:\n"
         // the cooperating lanes: v24 = the bytes' sum, v25 = n, v26 = the last byte
         "s_mov_b64 exec, s[60:61]\n"
         "v_add_u32 v24, v97, v104\n"
         "v_sub_u32 v25, " + vN + ", " + vI + "\n"
         "v_add_u32 v26, " + vI + ", v25\n" +
         (d - 1 ? "v_add_u32 v26, " + num(d - 1) + ", v26\n" : std::string()) +
         "v_mov_b32 v27, 0\n"
         "v_lshl_add_u64 v[26:27], v[32:33], 0, v[26:27]\n"
         "global_load_ubyte v26, v[26:27], off\n"
         "v_and_b32 v27, 0xffffff00, " + D0 + "\n"
         "v_mad_u64_u32 v[42:43], s[66:67], v27, v25, 0\n"
         "v_mul_lo_u32 v27, " + D1 + ", v25\n"
         "v_add_u32 v43, v43, v27\n"
         "v_add_co_u32 v42, vcc, v42, v24\nv_addc_co_u32 v43, vcc, 0, v43, vcc\n"
         "v_lshl_add_u64 " + S + ", v[42:43], 0, " + S + "\n"
         "v_mov_b32 v24, v25\nv_mov_b32 v25, 0\n"
         "v_lshl_add_u64 " + I2 + ", " + I2 + ", 0, v[24:25]\n"
         "s_waitcnt vmcnt(0)\n"
         "v_bfi_b32 " + D0 + ", s56, v26, " + D0 + "\n"
         "s_mov_b64 exec, -1\n"
         "v_mov_b32 v55, 0x80000000\n" + invalidate_prefetch() +
         "s_andn2_b64 exec, s[62:63], s[60:61]\n"
         "s_cbranch_execz .L" + P + "b" + std::to_string(J + 1) + "\n";
    coop_emitted = true;
    return r;
  }

  // coop_sum_compact's use of the lane's LDS window: a cooperating lane whose window [WB, WB + 64)
  // (v22 = WB, the packet offset the window holds; invalid tags are never within 64 of a0) covers
  // a0 sums the window's bytes [a0 - WB, 64) here -- every one in the range, since n >= 128 --
  // into v104, and its HBM range starts at WB + 64 instead (v[88:91] redone), so the bytes the
  // tile's window DMA already brought are not fetched again. Runs with exec = -1, v[88:91] set.
  std::string coop_window_part(const std::string& vI, const std::string& vN, int64_t d,
                               const std::string& G) const {
    std::string r = "; the window's part of the range\n" +
                    (d ? "v_add_u32 v24, " + std::to_string(d) + ", " + vI + "\n"
                       : "v_mov_b32 v24, " + vI + "\n") +
                    "v_sub_u32 v25, v24, v22\n"  // off = a0 - WB
                    "v_cmp_gt_u32 vcc, 64, v25\n"
                    "s_and_b64 s[66:67], vcc, s[60:61]\n"
                    "s_mov_b64 exec, s[66:67]\n"
                    "s_cbranch_execz " + G + "nowin\n"
                    "s_waitcnt lgkmcnt(0)\n";
    for (int c = 0; c < 4; c++)
      r += "v_xad_u32 v26, v35, " + std::to_string(16 * c) + ", v34\n"
           "ds_read_b128 v[" + std::to_string(56 + 4 * c) + ":" + std::to_string(59 + 4 * c) + "], v26\n";
    r += "s_waitcnt lgkmcnt(0)\n";
    for (int j = 0; j < 16; j++) {
      // dword j keeps its bytes at window offsets >= off: mask = low dword of (~0 << 8 m),
      // m = clamp(off - 4 j, 0, 4)
      const std::string Dw = "v" + std::to_string(56 + j);
      r += "v_subrev_u32 v26, " + std::to_string(4 * j) + ", v25\n"
           "v_med3_i32 v26, v26, 0, 4\n"
           "v_lshlrev_b32 v26, 3, v26\n"
           "v_lshlrev_b64 v[26:27], v26, -1\n"
           "v_and_b32 " + Dw + ", " + Dw + ", v26\n"
           "v_sad_u8 v104, " + Dw + ", 0, v104\n";
    }
    // the HBM range: [WB + 64, a0 + n)
    r += "v_sub_u32 v27, " + vN + ", " + vI + "\n"  // n
         "v_add_u32 v27, v27, v25\n"                  // n + off
         "v_subrev_u32 v27, 64, v27\n"                // a0 + n - (WB + 64)
         "v_add_u32 v88, 64, v22\n"
         "v_mov_b32 v89, 0\n"
         "v_lshl_add_u64 v[88:89], v[32:33], 0, v[88:89]\n"
         "v_and_b32 v90, 15, v88\n"
         "v_and_b32 v88, -16, v88\n"
         "v_add_u32 v91, v90, v27\n" + G + "nowin:\n"
         "s_mov_b64 exec, -1\n";
    return r;
  }

  std::string invalidate_prefetch() const {
    std::string r;
    r += "v_mov_b32 v23, 0x80000001\n";
    return r;
  }

  // The code of micro-op i (no block entry) in copy P.
  bool emit_uop(const Marker& m, uint32_t i, const std::string& P, bool fast, std::string& main,
                std::string& ool) {
    const uint32_t id = t[i].hoff / TILE_SLOT;
    if (id >= (uint32_t)T_COUNT || id == (uint32_t)T_DONE) {
      err = "bad handler id";
      return false;
    }
    // (the main.rs layout's forward code: a jump on a register the range analysis bounds below
    // 2^32 -- its high half zero -- against a constant; narrow_compares takes the marker)
    if (main_layout && !loops && !ranges.empty() && reached.size() == n && reached[i] &&
        is_jump(uops[i]) && uops[i].op != U_JA && !(uops[i].aux & F_SRC) &&
        ranges[i][uops[i].dst].hi < (1ull << 32))
      main += "; hi0 v" + std::to_string(2 * uops[i].dst + 1) + "\n";
    if (stk && stk->any_dyn) {  // store mode: the header window lives in LDS
      const Uop& o = uops[i];
      if ((o.op == U_ST || o.op == U_STX) && stk->off[i] == kNoStack) {
        if (stk->pw[i] != kNoStack) {
          main += lds_store_const(i);
          const uint32_t p = (uint32_t)stk->pw[i];  // (the cached chunks see the store too)
          uint32_t ch = 0;
          for (uint32_t b = p; b < p + o.aux; b++) ch |= 1u << (b >> 4);
          if (wcache & ch) main += store_bytes(i, p, 64);
        } else if (stk->dyn[i]) {
          main += lds_store_dyn(i, P, ool);
          wcache = 0;
        } else {
          main += "; unreachable store\n";
        }
        return true;
      }
      if (is_ldxk(id)) {
        main += ldxk_lds(i);
        return true;
      }
      // (a constant-address load past the window reads the packet: a lane that has stored into
      // its overflow image leaves for the general interpreter first)
      if (!dm.empty() && (id == T_LDXK_FAR_C || id == T_LDXK_FAR_E)) {
        // (the deopt-free proof judged constant-address loads by the range analysis: a load the
        // folder made constant where the ranges saw several values would deoptimize dirty lanes
        // the proof let through -- refuse to compile rather than run without the pass)
        if (stk->no_deopt && (i >= stk->kld.size() || !stk->kld[i])) {
          err = "store_mode_no_deopt: micro-op " + std::to_string(i) +
                " compiled as a constant-address load the proof did not classify as one";
          return false;
        }
        main += ovf_dirty_deopt(P + "u" + std::to_string(i), entry_label(P, next_start(i)), t[i].a0,
                                t[i].x - t[i].a0);
      }
    }
    if (stk && (uops[i].op == U_ST || uops[i].op == U_STX)) {
      // (a store the load-time dataflow never reached has no offset: no lane executes it)
      main += stk->pw[i] != kNoStack    ? pw_store(i)
              : stk->off[i] == kNoStack ? std::string("; unreachable store\n")
                                        : stack_store(i);
      return true;
    }
    if (stk && uops[i].op == U_ATOMIC) {
      main += stk->off[i] == kNoStack ? std::string("; unreachable atomic\n") : stack_atomic(i, P);
      return true;
    }
    if (stk && uops[i].op == U_LDX && stk->off[i] != kNoStack) {
      main += stack_load(i);
      return true;
    }
    if (fast && is_ldxk(id)) {
      main += ldxk_fast(i);
      return true;
    }
    if (const int co = ctx_load(i); co >= 0) {  // (xdp_ctx: the staged ctx's data / data_end)
      main += co && xdp_rebase ? "v_add_u32 v" + std::to_string(2 * uops[i].dst) + ", 8, v31\n"
                               : "v_mov_b32 v" + std::to_string(2 * uops[i].dst) + ", " +
                                     (co ? "v31" : "8") + "\n";
      return true;
    }
    if (!loops && (m.fixed == "1" || m.stack || m.varl) &&
        (id == T_LDX_C || id == T_LDX_E || id == T_LDX1_C || id == T_LDX1_E)) {
      std::string ot;
      main += ldx_fixed(i, id == T_LDX1_C || id == T_LDX1_E, P, ot, m.stack || m.varl);
      ool += ot;
      return true;
    }
    if (loops && stk && (id == T_LDX_C || id == T_LDX_E)) {  // (the overlay needs the value)
      std::string ot;
      main += ldx_fixed(i, false, P, ot, true, true);
      ool += ot;
      return true;
    }
    if (loops && (id == T_LDX1_C || id == T_LDX1_E)) {
      std::string ot;
      main += ldx1_loop(i, m, P, ot);
      ool += ot;
      return true;
    }
    std::set<uint32_t> sg;
    std::string mt, ot;
    if (!expand(kJitTemplates[id][0], i, m, P, sg, mt)) return false;
    if (!expand(kJitTemplates[id][1], i, m, P, sg, ot)) return false;
    const uint32_t* w = (const uint32_t*)&t[i];
    for (uint32_t d : sg)
      main += "s_mov_b32 s" + std::to_string(kFieldSgpr + d) + ", " + hex32(w[d]) + "\n";
    mt = resolve_ifs(mt);
    ot = resolve_ifs(ot);
    if (ot.empty()) mt = fold_copy(fold_copy(mt, 24), 54);  // (out-of-line code may read them)
    if (qcache && (touches(mt, 50, 55) || touches(ot, 50, 55))) cache_conflict = true;
    main += mt;
    ool += ot;
    return true;
  }

  // The step budget (s71 = max_steps) at a block entry of a loop program, as the interpreter's
  // dispatcher: the block copy restarts the tile in exact mode when some lane would pass it inside
  // the block (s70 = 1, windows re-read where refills are possible, tile_kernel's .Lbudget); the
  // exact copy (one micro-op per block) stops the lanes whose step this would be, ST_STEPS.
  // Loop programs keep the step counter biased, v29 = steps + (2^32 - 1 - max_steps) (s57 holds
  // the bias; body_loop sets and removes it), so the block entry's add carries out exactly for
  // the lanes whose steps pass max_steps (vcc).
  std::string budget_check(uint32_t i, const std::string& P) const {
    std::string s;
    if (!exact) return s + jmp("vccnz", ".L" + P + "budget");
    const std::string ok = ".L" + P + "bok" + std::to_string(i);
    return s + "s_cbranch_vccz " + ok + "\ns_mov_b64 s[64:65], exec\ns_mov_b64 exec, vcc\n"
               "v_mov_b32 v30, 5\nv_mov_b32 v28, -1\nv_subrev_u32 v29, 1, v29\n"
               "s_andn2_b64 exec, s[64:65], vcc\ns_cbranch_scc0 " +
           entry_label(P, next_start(i)) + "\n" + ok + ":\n";
  }

  // The stack window starts as the image's bytes there: zeros (fixed slots: the launch checked
  // that it lies past every packet byte); s57 = its image address S0 = r10 - k (s48 = r10).
  std::string stack_zero() const {
    std::string s = "; stack window: " + std::to_string(stk->k) + " bytes\ns_sub_u32 s57, s48, " +
                    std::to_string(stk->k) + "\n";
    for (uint32_t j = 0; j < stk->k / 4; j += 2)
      s += j + 1 < stk->k / 4 ? "v_mov_b64 v[" + std::to_string(kStackVgpr + j) + ":" +
                                    std::to_string(kStackVgpr + j + 1) + "], 0\n"
                              : "v_mov_b32 " + sv(j) + ", 0\n";
    return s;
  }

  // Other layouts: lanes whose packet reaches into the window take its bytes there, byte by
  // byte, out of line (the launch checked S0 >= 64, so they are never header-window bytes).
  std::string stack_init(const std::string& P, std::string& ool) const {
    // per window dword j (image address b = S0 + 4j, 4-aligned): the lanes whose packet holds
    // byte b load the aligned packet dwords around it -- the second only if it holds a packet
    // byte too (no access leaves the page of a packet byte, interp.hip pkt_read) -- and keep the
    // bytes below LEN; one wait per dword (the byte-by-byte form waited once per byte)
    ool += ".L" + P + "skinit:\ns_mov_b64 s[66:67], exec\ns_mov_b64 s[68:69], vcc\n";
    for (uint32_t j = 0; j < stk->k / 4; j++) {
      const std::string L = ".L" + P + "sk" + std::to_string(j);
      ool += "s_mov_b64 exec, s[68:69]\nv_add_u32_e64 v36, s57, " + std::to_string(4 * j) +
             "\nv_cmp_gt_u32 vcc, v31, v36\ns_and_b64 exec, exec, vcc\ns_cbranch_execz " + L + "\n"
             "v_mov_b32 v37, 0\nv_lshl_add_u64 v[38:39], v[32:33], 0, v[36:37]\n"
             "v_and_b32 v40, 3, v38\nv_and_b32 v38, -4, v38\n"
             "global_load_dword v41, v[38:39], off\nv_mov_b32 v42, 0\n"
             "v_sub_u32 v43, v36, v40\nv_add_u32 v43, 4, v43\nv_cmp_gt_u32 vcc, v31, v43\n"
             "s_and_saveexec_b64 s[64:65], vcc\n"
             "global_load_dword v42, v[38:39], off offset:4\n"
             "s_mov_b64 exec, s[64:65]\ns_waitcnt vmcnt(0)\n"
             "v_lshlrev_b32 v40, 3, v40\nv_alignbit_b32 v41, v42, v41, v40\n"
             "v_sub_u32 v43, v31, v36\nv_min_u32 v43, 4, v43\nv_lshlrev_b32 v43, 3, v43\n"
             "v_lshlrev_b64 v[44:45], v43, 1\nv_add_u32 v44, -1, v44\n"
             "v_and_b32 " + sv(j) + ", v44, v41\n" + L + ":\n";
    }
    ool += "s_mov_b64 exec, s[66:67]\ns_branch .L" + P + "skdone\n";
    return "v_cmp_lt_u32 vcc, s57, v31\ns_cbranch_vccnz .L" + P + "skinit\n.L" + P + "skdone:\n";
  }

  // The window shift of the xdp_md convention (see body): packet dwords 0..13 into v[66:79],
  // the ctx into v[64:65] (data = 8, data_end = LEN = 8 + len), all 16 written back in place.
  static std::string xdp_shift() {
    std::string s;
    for (uint32_t c = 0; c < 4; c++)
      s += "v_xad_u32 v" + std::to_string(36 + c) + ", v35, " + std::to_string(16 * c) + ", v34\n";
    s += "ds_read_b128 v[66:69], v36\nds_read_b128 v[70:73], v37\nds_read_b128 v[74:77], v38\n"
         "ds_read_b64 v[78:79], v39\nv_mov_b32 v64, 8\nv_mov_b32 v65, v31\ns_waitcnt lgkmcnt(0)\n";
    for (uint32_t c = 0; c < 4; c++)
      s += "ds_write_b128 v" + std::to_string(36 + c) + ", v[" + std::to_string(64 + 4 * c) + ":" +
           std::to_string(67 + 4 * c) + "]\n";
    return s;
  }

  // The program's code for the statement behind marker m. In the fixed-slot layout, a program
  // with window loads gets a second, fast copy: the window dwords it loads are read from LDS
  // once, up front (one ds_read_b128 per 16-byte chunk), and each load becomes one or two VALU
  // ops. The fast copy runs when mem_size covers every such load's end (so none can fault);
  // otherwise the handlers' copy, with its per-load bounds checks.
  bool body(const Marker& m, std::string& out) {
    if (stk && stk->any_dyn) return body_store(m, out);
    if (main_layout && !stk && ranges.empty()) prove_loads();  // (no stores: the ranges hold)
    const std::string P = "J" + m.n + "_";
    ovl_tag = m.n;
    overlay_widths = 0;
    island_from = 0;
    std::string main = "; compiled eBPF program: " + std::to_string(n) + " micro-ops\n"
                       "s_mov_b32 s52, s33\ns_mov_b32 s53, 0\n";
    pm_assign(m);
    main += pm_zero();
    if (stk) main += stack_zero();
    // xdp_md in place (fixed-slot kernel; the other kernels shift in C++, interp.hip xdp_window):
    // the lane's window holds packet bytes [0, 64), the program reads image bytes [0, 64) =
    // {u32 data = 8, u32 data_end = LEN} + packet bytes [0, 56) (xdp.rs:16-20): shifted once in
    // LDS, before any window read (LDS operations of a wave complete in order)
    bool reads_window = false;
    for (const Uop& o : uops) reads_window = reads_window || o.op == U_LDX;
    if ((m.fixed == "1" || m.varl) && reads_window && !m.xdp.empty() && !m.occ)
      main += "s_cmp_lg_u32 " + m.xdp + ", 0\ns_cbranch_scc0 .L" + P + "noxdp\n" + xdp_shift() +
              ".L" + P + "noxdp:\n";
    std::string ool;
    if (stk && m.stack) main += stack_init(P, ool);
    uint32_t chunks = 0, maxend = 0;
    if ((m.fixed == "1" && !m.occ) || m.stack || m.varl)
      for (uint32_t i = 0; i < n; i++) {
        const TUop& u = t[i];
        if (!is_ldxk(u.hoff / TILE_SLOT)) continue;
        const uint32_t a0 = u.a0, end = u.x, width = end - a0;
        const uint32_t last = width == 8 && (a0 & 3) ? (a0 >> 2) + 2 : (end - 1) >> 2;
        for (uint32_t k = a0 >> 2; k <= last && k < 16; k++) chunks |= 1u << (k >> 2);
        maxend = std::max(maxend, end);
      }
    // packet-window stores merge into the preloaded dwords; such programs have only the fast
    // copy (the launch checks mem_size >= every window load's end, host.cpp stack_launch_ok)
    const bool pw = stk && stk->any_pw && (m.fixed == "1" || m.stack);
    for (uint32_t i = 0; pw && i < n; i++)
      if (stk->pw[i] != kNoStack)
        for (uint32_t b = (uint32_t)stk->pw[i]; b < (uint32_t)stk->pw[i] + uops[i].aux; b++)
          chunks |= 1u << (b >> 4);
    if (chunks) {
      const std::string F = "J" + m.n + "f_";
      if (!pw)
        main += "s_cmp_gt_u32 " + std::to_string(maxend) + ", s33\n" + jmp("scc1", ".L" + P + "slow");
      for (uint32_t c = 0; c < 4; c++)
        if (chunks & (1u << c))
          main += "v_xad_u32 v36, v35, " + std::to_string(16 * c) + ", v34\nds_read_b128 v[" +
                  std::to_string(64 + 4 * c) + ":" + std::to_string(67 + 4 * c) + "], v36\n";
      main += "s_waitcnt lgkmcnt(0)\n";
      if (m.stack || m.varl) {  // var layouts: the preloaded bytes at or past LEN are zeros (main.rs:16),
                      // skipped when every lane's packet covers the window
        const std::string D = ".L" + F + "pmd";
        main += "v_cmp_gt_u32 vcc, 64, v31\ns_cbranch_vccz " + D + "\n";
        for (uint32_t j = 0; j < 16; j++)
          if (chunks & (1u << (j >> 2)))
            main += "v_subrev_u32 v36, " + std::to_string(4 * j) + ", v31\n"
                    "v_med3_i32 v36, v36, 0, 4\nv_lshlrev_b32 v36, 3, v36\n"
                    "v_lshlrev_b64 v[36:37], v36, 1\nv_add_u32 v36, -1, v36\n"
                    "v_and_b32 v" + std::to_string(64 + j) + ", v36, v" + std::to_string(64 + j) +
                    "\n";
        main += D + ":\n";
      }
      main += "s_mov_b64 exec, 0\n";
      if (!copy(m, F, true, main, ool)) return false;
      main += jmp("", ".L" + P + "end") + (pw ? "" : ".L" + P + "slow:\n");
    }
    if (!pw) {
      main += "s_mov_b64 exec, 0\n";
      if (!copy(m, P, false, main, ool)) return false;
    }
    main += ".L" + P + "end:\n";
    ool += overlay_routines();
    if (!ool.empty()) main += "s_branch .Ldone" + m.n + "\n" + ool;
    out = peephole(main);
    return true;
  }

  // A loop program (this compiler: the block table; xc: the exact table's) for the statement of
  // ebpf_tile_jit_loop: s70 = 0 runs the block copy, whose budget failure restarts the tile
  // (.Lreinit of the statement's prologue) with s70 = 1, which runs the exact copy.
  bool body_loop(const Marker& m, Compiler& xc, std::string& out) {
    pm_of.clear();  // (LPC parking only)
    // (compile_into_template may run this twice -- a dry run finds a cooperative sum, then the
    // real one: every piece of state a run writes is reset here, so the two agree)
    for (Compiler* k : {this, &xc}) {
      std::fill(k->addr_src.begin(), k->addr_src.end(), -1);
      k->err.clear();
      k->coop_emitted = false;
      k->proven = false;
    }
    // (A 16-byte per-lane byte cache, an opt-in A/B variant until round 5, measured 474 vs
    // 466 us on the checksum config: the extra selects and its miss path's SALU turned the LDS
    // waits into issue stalls, profiles/r02_pmc_checksum_bytecache.json.)
    // (stack-window programs: the plain refillable windows, the loads' store-forwarding overlay)
    bool only_bytes = !stk;
    for (uint32_t i = 0; i < n; i++)
      only_bytes = only_bytes && (uops[i].op != U_LDX || uops[i].aux == 1 || ctx_load(i) >= 0);
    zwin = xc.zwin = only_bytes;
    qcache = xc.qcache = zwin;
    prefetch = xc.prefetch = zwin;
    cache_conflict = xc.cache_conflict = false;
    if (!body_loop_once(m, xc, out)) return false;
    if (!cache_conflict && !xc.cache_conflict) return true;
    qcache = xc.qcache = false;  // (the qword cache's v[50:55] named by other compiled code)
    return body_loop_once(m, xc, out);
  }

  // Whether body_loop will give this program prefetching refills (zero-past-len windows: every
  // register load one byte wide).
  bool prefetches() const {
    if (stk) return false;
    for (uint32_t i = 0; i < n; i++)
      if (uops[i].op == U_LDX && uops[i].aux != 1 && ctx_load(i) < 0) return false;
    return true;
  }

  // A stack-slot promoted program (guard_k): the lanes about to run (LPC 0) whose packet reaches
  // the stack window (LEN > r10 - guard_k: a packet load could read a slot's bytes, which the
  // promoted program keeps in a register) deoptimize before their first step -- the general
  // interpreter runs their packets after the launch (host.cpp, the deopt pass).
  std::string promo_guard(const std::string& P) const {
    if (!guard_k) return "";
    const std::string G = ".L" + P + "pguard";
    // (r10 from s48, the statement's copy of LaunchArgs::r10: the promoted program may never
    // read r10, so its register can be left uninitialised by the live-in init)
    return "; stack-slot promotion guard: LEN <= r10 - " + std::to_string(guard_k) + "\n"
           "s_mov_b64 s[64:65], exec\ns_mov_b64 exec, -1\n"
           "v_mov_b32 v36, s48\nv_subrev_u32 v36, " + std::to_string(guard_k) + ", v36\n"
           "v_cmp_gt_u32 vcc, v31, v36\n"
           "v_cmp_eq_u32 s[60:61], 0, v28\n"
           "s_and_b64 vcc, vcc, s[60:61]\n"
           "s_cbranch_vccz " + G + "\n"
           "s_mov_b64 exec, vcc\n"
           "v_mov_b32 v30, 0x80\nv_mov_b32 v28, -1\n" + G + ":\n"
           "s_mov_b64 exec, s[64:65]\n";
  }

  // s70 (set by the statement's prologue, tile_jit.inc): bit 0 = exact mode (the step-budget
  // restart), bit 1 = registers not in the main.rs layout (init_regs) or requested as outputs.
  // With bit 1 clear, a program with loads proven in bounds (prove_loads) runs its proven copy.
  bool body_loop_once(const Marker& m, Compiler& xc, std::string& out) {
    const std::string P = "J" + m.n + "_", PX = "J" + m.n + "x_", PC = "J" + m.n + "c_";
    ovl_tag = m.n;
    xc.ovl_tag = m.n + "x";
    overlay_widths = xc.overlay_widths = 0;
    island_from = 0;
    std::string ool;
    // (stack-window programs keep the budget's bias in s54 -- the statement's table pointer, which
    // compiled code never reads -- s57 being the window's address)
    const std::string B = stk ? "s54" : "s57";
    std::string main = "; compiled eBPF loop program: " + std::to_string(n) + " micro-ops\n"
                       "s_mov_b32 s52, s33\ns_mov_b32 s53, 0\ns_movk_i32 s56, 0xff\n"
                       "s_not_b32 " + B + ", s71\ns_mov_b64 exec, -1\nv_add_u32 v29, " + B +
                       ", v29\n"
                       "v_mov_b32 v55, 0x80000000\n" + window_zero_prologue(m, P) +
                       prefetch_prologue(m, P) +
                       (stk ? stack_zero() + stack_init(P, ool) : std::string()) + promo_guard(P) +
                       "s_bitcmp1_b32 s70, 0\n" + jmp("scc1", ".L" + PX + "start");
    prove_loads();
    const bool any = std::find(inb.begin(), inb.end(), 1) != inb.end();
    if (any) {
      main += "; one-byte loads proven in bounds: the proven copy unless s70 bit 1\n"
              "s_bitcmp1_b32 s70, 1\n" + jmp("scc1", ".L" + PC + "go") + "s_mov_b64 exec, 0\n";
      proven = true;
      const bool ok = copy(m, P, false, main, ool);
      proven = false;
      if (!ok) return false;
      main += jmp("", ".L" + P + "end") + ".L" + PC + "go:\n";
    }
    main += "s_mov_b64 exec, 0\n";
    const std::string PB = any ? PC : P;  // the checked block copy
    if (!copy(m, PB, false, main, ool)) return false;
    main += jmp("", ".L" + P + "end") + (any ? ".L" + PC + "budget:\n" : std::string()) +
            ".L" + P + "budget:\ns_or_b32 s70, s70, 1\n"
            "s_cmp_eq_u32 " + m.aligned + ", 0\ns_cbranch_scc1 .L" + P + "bkeep\n"
            "v_mov_b32 v22, -64\n.L" + P + "bkeep:\ns_mov_b64 exec, -1\n"
            "s_branch .Lreinit" + m.n + "\n.L" + PX + "start:\ns_mov_b64 exec, 0\n";
    xc.island_from = main.size();
    if (!xc.copy(m, PX, false, main, ool)) {
      err = xc.err;
      return false;
    }
    main += ".L" + P + "end:\ns_mov_b64 exec, -1\nv_subrev_u32 v29, " + B + ", v29\n" +
            std::string(prefetch ? "s_waitcnt vmcnt(0)\n" : "");
    ool += overlay_routines() + xc.overlay_routines();
    if (!ool.empty()) main += "s_branch .Ldone" + m.n + "\n" + ool;
    out = peephole(main);
    return true;
  }

  // mov + add of the same 64-bit destination in a row (e.g. `mov r4, r1; add r4, r3`, adjacent
  // micro-ops with no block entry between them): one add from the moved source. mov + and / or /
  // xor with an operand that is not the destination (`mov r8, r5; and r8, 0xff`, a rule's mask):
  // the two halves' ops from the moved source (an and with 0 a move of 0).
  static std::string peephole(const std::string& text) {
    std::vector<std::string> ln;
    for (size_t p = 0; p < text.size();) {
      size_t e = text.find('\n', p);
      if (e == std::string::npos) e = text.size();
      ln.push_back(text.substr(p, e - p));
      p = e + 1;
    }
    std::string out;
    for (size_t i = 0; i < ln.size(); i++) {
      uint32_t d0, d1, s0, s1;
      char rest[128];
      if (i + 1 < ln.size() &&
          sscanf(ln[i].c_str(), "v_mov_b64 v[%u:%u], v[%u:%u]", &d0, &d1, &s0, &s1) == 4) {
        const std::string D = "v[" + std::to_string(d0) + ":" + std::to_string(d1) + "]";
        const std::string head = "v_lshl_add_u64 " + D + ", " + D + ", 0, ";
        if (ln[i + 1].compare(0, head.size(), head) == 0 &&
            sscanf(ln[i + 1].c_str() + head.size(), "%127s", rest) == 1 &&
            ln[i + 1].find(D, head.size()) == std::string::npos) {
          out += "v_lshl_add_u64 " + D + ", v[" + std::to_string(s0) + ":" + std::to_string(s1) +
                 "], 0, " + ln[i + 1].substr(head.size()) + "\n";
          i++;
          continue;
        }
        // (an s_mov of the op's constant may sit between: it touches no VGPR)
        const size_t k = i + 1 < ln.size() && ln[i + 1].compare(0, 10, "s_mov_b32 ") == 0 ? i + 2 : i + 1;
        auto half = [&](size_t j, uint32_t d, std::string& op, std::string& x) {
          char o[16], a[64], b[32];
          if (j >= ln.size() || sscanf(ln[j].c_str(), "%15s v%*u, %63[^,], %31s", o, a, b) != 3) return false;
          op = o, x = a;
          const std::string vd = "v" + std::to_string(d);
          return (op == "v_and_b32" || op == "v_or_b32" || op == "v_xor_b32") &&
                 ln[j] == op + " " + vd + ", " + x + ", " + vd && x.find('v') == std::string::npos;
        };
        std::string o0, x0, o1, x1;
        if (d1 == d0 + 1 && s1 == s0 + 1 && half(k, d0, o0, x0) && half(k + 1, d1, o1, x1) && o0 == o1) {
          // (the s_mov's constant straight into the low half's op -- a VOP2 literal -- when only
          // that op reads it)
          char sreg[16], kv[32];
          if (k == i + 2 && sscanf(ln[i + 1].c_str(), "s_mov_b32 %15[^,], %31s", sreg, kv) == 2 &&
              x0 == sreg && x1 != sreg)
            x0 = kv;
          else if (k == i + 2)
            out += ln[i + 1] + "\n";
          out += o0 + " v" + std::to_string(d0) + ", " + x0 + ", v" + std::to_string(s0) + "\n";
          out += o0 == "v_and_b32" && x1 == "0"
                     ? "v_mov_b32 v" + std::to_string(d1) + ", 0\n"
                     : o0 + " v" + std::to_string(d1) + ", " + x1 + ", v" + std::to_string(s1) + "\n";
          i = k + 1;
          continue;
        }
      }
      out += ln[i] + "\n";
    }
    return cmpx_pass(negate_leave(sink_high_zero(narrow_compares(out))));
  }

  // A register's high half zeroed just before a jump (`v_mov_b32 vH, 0` of a fused mov + and,
  // its compare narrowed to the low half) whose leaving lanes go where the register is dead
  // (the `; dead@leave` marker of jtail): the move goes after the jump's exec update, so only
  // the staying lanes run it -- in a rule chain, the rule's first test sends nearly every lane to
  // the next rule, which overwrites the register, and the move leaves the common path.
  // A jump whose NOT-taken lanes leave into a pending mask (jtail_code: s[64:65] = exec & ~vcc,
  // OR-ed into the mask, exec &= vcc) after a VOPC compare into vcc: the compare negated, so the
  // leaving lanes are vcc and the mask takes them directly (two SALU instead of three).
  static std::string negate_leave(const std::string& text) {
    std::vector<std::string> ln;
    for (size_t p = 0; p < text.size();) {
      size_t e = text.find('\n', p);
      if (e == std::string::npos) e = text.size();
      ln.push_back(text.substr(p, e - p));
      p = e + 1;
    }
    static const std::map<std::string, std::string> neg = {
        {"eq", "ne"}, {"ne", "eq"}, {"gt", "le"}, {"le", "gt"}, {"ge", "lt"}, {"lt", "ge"}};
    std::vector<std::string> out;
    out.reserve(ln.size());
    for (size_t i = 0; i < ln.size(); i++) {
      char op[8], ty[8], pm[32];
      if (i + 2 < ln.size() && ln[i] == "s_andn2_b64 s[64:65], exec, vcc" &&
          sscanf(ln[i + 1].c_str(), "s_or_b64 %31[^,], ", pm) == 1 &&
          ln[i + 1] == "s_or_b64 " + std::string(pm) + ", " + pm + ", s[64:65]" &&
          std::string(pm).compare(0, 3, "s[7") == 0 && ln[i + 2] == "s_and_b64 exec, exec, vcc") {
        size_t c = out.size();  // the compare: the last non-comment line before
        while (c > 0 && !out[c - 1].empty() && out[c - 1][0] == ';') c--;
        if (c > 0 && sscanf(out[c - 1].c_str(), "v_cmp_%2[a-z]_%3[a-z0-9] vcc, ", op, ty) == 2 &&
            neg.count(op) && out[c - 1].find("_e64") == std::string::npos &&
            out[c - 1].compare(0, 6 + strlen(op) + 1 + strlen(ty), std::string("v_cmp_") + op + "_" + ty) == 0) {
          out[c - 1] = "v_cmp_" + neg.at(op) + out[c - 1].substr(6 + strlen(op));
          out.push_back("s_or_b64 " + std::string(pm) + ", " + pm + ", vcc");
          out.push_back("s_andn2_b64 exec, exec, vcc");
          i += 2;
          continue;
        }
      }
      out.push_back(ln[i]);
    }
    std::string r;
    for (const std::string& l : out) r += l + "\n";
    return r;
  }

  // A compare into vcc whose only use is the exec update right after it (comments between):
  // `v_cmp_<op> vcc, ..` + `s_and_b64 exec, exec, vcc` -> `v_cmpx_<op> vcc, ..`, and with
  // `s_andn2_b64 exec, exec, vcc` the negated compare -- the tests of a complement region
  // (cm_assign), one VALU instruction each.
  static std::string cmpx_pass(const std::string& text) {
    std::vector<std::string> ln;
    for (size_t p = 0; p < text.size();) {
      size_t e = text.find('\n', p);
      if (e == std::string::npos) e = text.size();
      ln.push_back(text.substr(p, e - p));
      p = e + 1;
    }
    static const std::map<std::string, std::string> neg = {
        {"eq", "ne"}, {"ne", "eq"}, {"gt", "le"}, {"le", "gt"}, {"ge", "lt"}, {"lt", "ge"}};
    std::vector<std::string> out;
    out.reserve(ln.size());
    for (size_t i = 0; i < ln.size(); i++) {
      const bool an = ln[i] == "s_andn2_b64 exec, exec, vcc", a = ln[i] == "s_and_b64 exec, exec, vcc";
      if ((an || a) && i > 0 && ln[i - 1] == "; cmx") {  // (the marker itself is dropped below)
        size_t c = out.size();
        while (c > 0 && !out[c - 1].empty() && out[c - 1][0] == ';') c--;
        char op[8], ty[8];
        if (c > 0 && sscanf(out[c - 1].c_str(), "v_cmp_%2[a-z]_%3[a-z0-9] vcc, ", op, ty) == 2 &&
            neg.count(op) && out[c - 1].find("_e64") == std::string::npos &&
            out[c - 1].compare(0, 6 + strlen(op) + 1 + strlen(ty), std::string("v_cmp_") + op + "_" + ty) == 0) {
          out[c - 1] = "v_cmpx_" + (an ? neg.at(op) : std::string(op)) + out[c - 1].substr(6 + strlen(op));
          continue;
        }
      }
      if (ln[i] == "; cmx") continue;
      out.push_back(ln[i]);
    }
    std::string r;
    for (const std::string& l : out) r += l + "\n";
    return r;
  }

  static std::string sink_high_zero(const std::string& text) {
    std::vector<std::string> ln;
    for (size_t p = 0; p < text.size();) {
      size_t e = text.find('\n', p);
      if (e == std::string::npos) e = text.size();
      ln.push_back(text.substr(p, e - p));
      p = e + 1;
    }
    auto names = [](const std::string& l, const std::string& v) {
      for (size_t q = 0; (q = l.find(v, q)) != std::string::npos; q += v.size()) {
        const bool lo = q == 0 || !(isalnum((unsigned char)l[q - 1]) || l[q - 1] == '_');
        const size_t e = q + v.size();
        const bool hi = e >= l.size() || !isalnum((unsigned char)l[e]);
        if (lo && hi) return true;
      }
      // a register range v[a:b] holding it (a 64-bit operand)
      uint32_t r, a, b;
      if (sscanf(v.c_str(), "v%u", &r) != 1) return false;
      for (size_t q = 0; (q = l.find("v[", q)) != std::string::npos; q += 2)
        if (sscanf(l.c_str() + q, "v[%u:%u]", &a, &b) == 2 && a <= r && r <= b) return true;
      return false;
    };
    for (size_t m = 0; m < ln.size(); m++) {
      if (ln[m].compare(0, 12, "; dead@leave") != 0) continue;
      size_t x = m + 1;  // the exec update of the jump tail
      while (x < ln.size() && x <= m + 4 && ln[x].compare(0, 16, "s_and_b64 exec, ") != 0 &&
             ln[x].compare(0, 18, "s_andn2_b64 exec, ") != 0)
        x++;
      if (x >= ln.size() || x > m + 4 || (ln[x] != "s_and_b64 exec, exec, vcc" &&
                                          ln[x] != "s_andn2_b64 exec, exec, vcc"))
        continue;
      // where the sunk code goes: after the exec update -- or, when the next line starts a block
      // with no entry code (one predecessor, this fall-through) and its empty-exec skip, after
      // that skip, so that a jump that sent every lane away skips it too
      size_t ins = x + 1;
      if (x + 2 < ln.size() && ln[x + 1].size() > 3 && ln[x + 1].compare(0, 2, ".L") == 0 &&
          ln[x + 1].back() == ':' && ln[x + 2].compare(0, 16, "s_cbranch_execz ") == 0)
        ins = x + 3;
      // `v_and_b32 vL, 0xff|0xffff, vS` + `v_cmp_<op>_u32 vcc, K, vL` right before the marker, the
      // register (vL, vL+1) dead where the leaving lanes go: the compare reads vS's low byte / half
      // itself (SDWA), and the and goes after the exec update with the high half's move
      {
        uint32_t L, S, L2;
        char msk[16], op[8], kv[32];
        size_t ka = m >= 2 ? m - 2 : 0;  // the and: right before the compare, or before the high
        uint32_t hz;                      // half's move and the `; hi0` marker
        while (ka > 0 && ka + 4 >= m &&
               ((sscanf(ln[ka].c_str(), "v_mov_b32 v%u, 0", &hz) == 1 && ln[ka] == "v_mov_b32 v" + std::to_string(hz) + ", 0") ||
                ln[ka].compare(0, 6, "; hi0 ") == 0))
          ka--;
        if (m >= 2 && sscanf(ln[ka].c_str(), "v_and_b32 v%u, %15[^,], v%u", &L, msk, &S) == 3 &&
            ln[ka] == "v_and_b32 v" + std::to_string(L) + ", " + msk + ", v" + std::to_string(S) &&
            (std::string(msk) == "0xff" || std::string(msk) == "0xffff") && S != L && S != L + 1 &&
            sscanf(ln[m - 1].c_str(), "v_cmp_%2[a-z]_u32 vcc, %31[^,], v%u", op, kv, &L2) == 3 &&
            L2 == L && ln[m - 1] == std::string("v_cmp_") + op + "_u32 vcc, " + kv + ", v" + std::to_string(L) &&
            names(ln[m], "v" + std::to_string(L + 1)) && L % 2 == 0 && [&] {
              for (size_t q = m; q <= x; q++)  // (vL unread, vS unwritten up to the exec update)
                if (q != m && (names(ln[q], "v" + std::to_string(L)) || names(ln[q], "v" + std::to_string(S))))
                  return false;
              return true;
            }()) {
          // the low half: a 16-bit compare with K as its literal; the low byte: SDWA, whose
          // operands take inline constants but no literal (a larger K keeps the and)
          char* ke = nullptr;
          const unsigned long kn = strtoul(kv, &ke, 0);
          const bool kok = ke && *ke == 0 && kv[0] != '-';
          std::string cmp;
          if (kok && std::string(msk) == "0xffff" && kn <= 0xffff)
            cmp = std::string("v_cmp_") + op + "_u16 vcc, " + kv + ", v" + std::to_string(S);
          else if (kok && std::string(msk) == "0xff" && kn <= 64)
            cmp = std::string("v_cmp_") + op + "_u32_sdwa vcc, " + kv + ", v" + std::to_string(S) +
                  " src0_sel:DWORD src1_sel:BYTE_0";
          if (!cmp.empty()) {
            const std::string a = ln[ka];
            ln.erase(ln.begin() + ka);
            m--, x--, ins--;
            ln[m - 1] = cmp;
            ln.insert(ln.begin() + ins, a);
          }
        }
      }
      for (size_t k = m; k-- > 0 && k + 6 > m;) {
        uint32_t h;
        if (sscanf(ln[k].c_str(), "v_mov_b32 v%u, 0", &h) != 1 || ln[k] != "v_mov_b32 v" + std::to_string(h) + ", 0")
          continue;
        const std::string vh = "v" + std::to_string(h);
        if (!names(ln[m], vh)) continue;
        bool clear = true;  // nothing between the move and the exec update names vH or is a label
        for (size_t q = k + 1; q <= x && clear; q++)
          clear = !names(ln[q], vh) || ln[q][0] == ';';  // (markers are comments)
        for (size_t q = k + 1; q <= x && clear; q++) clear = ln[q].empty() || ln[q][0] != '.';
        if (!clear) continue;
        ln.insert(ln.begin() + ins, ln[k]);
        ln.erase(ln.begin() + k);
        m--;
        x--;
        ins--;
      }
    }
    std::string r;
    for (const std::string& l : ln) r += l + "\n";
    return r;
  }

  // A 64-bit compare of a register whose high half was just zeroed with a constant below 2^32
  // (`v_mov_b32 vH, 0` -- or the `; hi0 vH` marker of a register the range analysis bounds below
  // 2^32 -- then s[48:49] = {K, 0}, `v_cmp_<op>_[iu]64 vcc, s[48:49], v[L:H]`, in a row):
  // both sides lie in [0, 2^32), where the signed and unsigned orders agree, so the 32-bit
  // unsigned compare of the low halves gives the same vcc -- with K as the VOPC's literal (the
  // s_movs of s[48:49] go: a micro-op's code sets every field register it reads).
  static std::string narrow_compares(const std::string& text) {
    std::vector<std::string> ln;
    for (size_t p = 0; p < text.size();) {
      size_t e = text.find('\n', p);
      if (e == std::string::npos) e = text.size();
      ln.push_back(text.substr(p, e - p));
      p = e + 1;
    }
    std::vector<std::string> out;
    for (size_t i = 0; i < ln.size(); i++) {
      char op[8], sg;
      uint32_t lo, hi, h0;
      if (i >= 3 && ln[i - 1] == "s_mov_b32 s49, 0x0" && ln[i - 2].compare(0, 15, "s_mov_b32 s48, ") == 0 &&
          ((sscanf(ln[i - 3].c_str(), "v_mov_b32 v%u, 0", &h0) == 1 &&
            ln[i - 3] == "v_mov_b32 v" + std::to_string(h0) + ", 0") ||
           (sscanf(ln[i - 3].c_str(), "; hi0 v%u", &h0) == 1 &&
            ln[i - 3] == "; hi0 v" + std::to_string(h0))) &&
          sscanf(ln[i].c_str(), "v_cmp_%2[a-z]_%c64 vcc, s[48:49], v[%u:%u]", op, &sg, &lo, &hi) == 4 &&
          (sg == 'u' || sg == 'i') && hi == lo + 1 && hi == h0 &&
          ln[i] == std::string("v_cmp_") + op + "_" + sg + "64 vcc, s[48:49], v[" + std::to_string(lo) +
                       ":" + std::to_string(hi) + "]") {
        const std::string o(op), k = ln[i - 2].substr(15);
        if ((o == "eq" || o == "ne" || o == "gt" || o == "ge" || o == "lt" || o == "le") &&
            out.size() >= 2 && out.back() == ln[i - 1] && out[out.size() - 2] == ln[i - 2]) {
          out.resize(out.size() - 2);
          out.push_back("v_cmp_" + o + "_u32 vcc, " + k + ", v" + std::to_string(lo));
          continue;
        }
      }
      // `; hi0 vH` then `v_cmp_<op>_[iu]64 vcc, K, v[L:H]` with K an inline constant in [0, 64]
      uint32_t kk;
      if (i >= 1 && sscanf(ln[i - 1].c_str(), "; hi0 v%u", &h0) == 1 &&
          sscanf(ln[i].c_str(), "v_cmp_%2[a-z]_%c64 vcc, %u, v[%u:%u]", op, &sg, &kk, &lo, &hi) == 5 &&
          (sg == 'u' || sg == 'i') && hi == lo + 1 && hi == h0 && kk <= 64 &&
          ln[i] == std::string("v_cmp_") + op + "_" + sg + "64 vcc, " + std::to_string(kk) + ", v[" +
                       std::to_string(lo) + ":" + std::to_string(hi) + "]") {
        const std::string o(op);
        if (o == "eq" || o == "ne" || o == "gt" || o == "ge" || o == "lt" || o == "le") {
          out.push_back("v_cmp_" + o + "_u32 vcc, " + std::to_string(kk) + ", v" + std::to_string(lo));
          continue;
        }
      }
      out.push_back(ln[i]);
    }
    std::string r;
    for (const std::string& l : out) r += l + "\n";
    return r;
  }
};

#define COMGR_OK(x) ((x) == AMD_COMGR_STATUS_SUCCESS)

std::string comgr_log(amd_comgr_data_set_t set) {
  size_t nl = 0;
  std::string all;
  if (!COMGR_OK(amd_comgr_action_data_count(set, AMD_COMGR_DATA_KIND_LOG, &nl))) return all;
  for (size_t i = 0; i < nl; i++) {
    amd_comgr_data_t l;
    if (!COMGR_OK(amd_comgr_action_data_get_data(set, AMD_COMGR_DATA_KIND_LOG, i, &l))) continue;
    size_t sz = 0;
    amd_comgr_get_data(l, &sz, nullptr);
    std::string b(sz, '\0');
    amd_comgr_get_data(l, &sz, &b[0]);
    all += b;
    amd_comgr_release_data(l);
  }
  return all;
}

// .s -> relocatable -> executable code object, in process.
bool assemble(const std::string& src, std::vector<char>& co, std::string* err) {
  amd_comgr_data_t d{};
  amd_comgr_data_set_t in{}, rel{}, exe{};
  amd_comgr_action_info_t ai{};
  bool ok = COMGR_OK(amd_comgr_create_data(AMD_COMGR_DATA_KIND_SOURCE, &d)) &&
            COMGR_OK(amd_comgr_set_data(d, src.size(), src.data())) &&
            COMGR_OK(amd_comgr_set_data_name(d, "ebpf_jit.s")) &&
            COMGR_OK(amd_comgr_create_data_set(&in)) && COMGR_OK(amd_comgr_create_data_set(&rel)) &&
            COMGR_OK(amd_comgr_create_data_set(&exe)) && COMGR_OK(amd_comgr_data_set_add(in, d)) &&
            COMGR_OK(amd_comgr_create_action_info(&ai)) &&
            COMGR_OK(amd_comgr_action_info_set_isa_name(ai, "amdgcn-amd-amdhsa--gfx950")) &&
            COMGR_OK(amd_comgr_action_info_set_language(ai, AMD_COMGR_LANGUAGE_NONE)) &&
            COMGR_OK(amd_comgr_action_info_set_logging(ai, true));
  if (ok && !COMGR_OK(amd_comgr_do_action(AMD_COMGR_ACTION_ASSEMBLE_SOURCE_TO_RELOCATABLE, ai, in,
                                          rel))) {
    ok = false;
    if (err) *err = "assembler: " + comgr_log(rel);
  }
  if (ok && !COMGR_OK(amd_comgr_do_action(AMD_COMGR_ACTION_LINK_RELOCATABLE_TO_EXECUTABLE, ai, rel,
                                          exe))) {
    ok = false;
    if (err) *err = "linker: " + comgr_log(exe);
  }
  if (ok) {
    amd_comgr_data_t e;
    size_t sz = 0;
    ok = COMGR_OK(amd_comgr_action_data_get_data(exe, AMD_COMGR_DATA_KIND_EXECUTABLE, 0, &e));
    if (ok) {
      amd_comgr_get_data(e, &sz, nullptr);
      co.resize(sz);
      ok = COMGR_OK(amd_comgr_get_data(e, &sz, co.data()));
      amd_comgr_release_data(e);
    }
    if (!ok && err) *err = "no executable";
  }
  if (ai.handle) amd_comgr_destroy_action_info(ai);
  if (exe.handle) amd_comgr_destroy_data_set(exe);
  if (rel.handle) amd_comgr_destroy_data_set(rel);
  if (in.handle) amd_comgr_destroy_data_set(in);
  if (d.handle) amd_comgr_release_data(d);
  return ok;
}

}  // namespace

namespace {

// Far mode (compile_into_template) past this many lines of code in one body: s_branch reaches
// +-32 Ki dwords, and a line of the body is at most 12 bytes, most 4 or 8.
constexpr size_t kFarLines = 8192;

// A body moved out of line (far mode): its exits to the statement (.Ldone: the epilogue behind
// the marker, .Lreinit: a loop program's exact-mode restart) become long jumps, and so does its
// fall-through end.
std::string relocated_body(const std::string& b, const std::string& n, uint32_t& tag) {
  auto lj = [&](const std::string& l) { return long_jump(l, "r" + std::to_string(tag++)); };
  std::string out = ".Lbody" + n + ":\n";
  size_t p = 0;
  while (p < b.size()) {
    size_t e = b.find('\n', p);
    if (e == std::string::npos) e = b.size();
    const std::string ln = b.substr(p, e - p);
    p = e + 1;
    if (ln == "s_branch .Ldone" + n || ln == "s_branch .Lreinit" + n)
      out += lj(ln.substr(9));
    else
      out += ln + "\n";
  }
  return out + lj(".Ldone" + n);
}

// Insert the compiled code at every marker of the template assembly (markers of the other kind of
// kernel -- loop vs forward-only -- get an empty body: never launched for this program), then
// assemble. Far mode, when a body passes kFarLines: every body out of line, behind its kernel's
// code (entered by a long jump), so that no branch of the template or of the statement around it
// spans the program.
// ebpf_tile_jit_fixed_occ: whether a compiled body names only the VGPRs its statement owns
// (v[0:55], TILE_ASM_CLOBBER in interp.hip); the others hold the kernel's own values.
bool occ_regs_ok(const std::string& b) {
  for (size_t q = 0; (q = b.find('v', q)) != std::string::npos; q++) {
    if (q > 0 && (isalnum((unsigned char)b[q - 1]) || b[q - 1] == '_' || b[q - 1] == '.')) continue;
    uint32_t lo = 0, hi = 0;
    if (b[q + 1] == '[') {
      if (sscanf(b.c_str() + q, "v[%u:%u]", &lo, &hi) != 2) continue;
    } else if (isdigit((unsigned char)b[q + 1])) {
      if (sscanf(b.c_str() + q, "v%u", &lo) != 1) continue;
      hi = lo;
    } else {
      continue;
    }
    if (hi >= 56) return false;
  }
  return true;
}

// Programs the occupancy variant of the fixed-slot kernel takes (host.cpp routes their
// fixed-slot batches there): every forward program it can take (kOccMinUops) -- first meant for
// issue-bound rule chains, it also runs short programs faster when launches overlap (two
// streams). EBPFEMU_FIXED_OCC=0|1 (A/B) turns it off / on for every program it can take.
bool occ_wanted(uint32_t n_uops) {
  static const int force = [] {
    const char* e = getenv("EBPFEMU_FIXED_OCC");
    return e ? (e[0] == '1' ? 1 : 0) : -1;
  }();
  return force >= 0 ? force == 1 : n_uops >= kOccMinUops;
}

bool compile_into_template(Compiler& c, Compiler* xc, std::vector<char>& code_object,
                           std::string* err, std::string* asm_out, bool* deep_out = nullptr) {
  std::string tmpl(kJitTemplateAsm);
  if (c.xdp_rebase) {  // (the all-registers init: r2 = 8 + LEN, the image's length)
    const std::string from = "v_mov_b32 v4, v31\n", to = "v_add_u32 v4, 8, v31\n";
    for (size_t q = 0; (q = tmpl.find(from, q)) != std::string::npos; q += to.size())
      tmpl.replace(q, from.size(), to);
  }
  // cache policy of the window DMA (the fixed-slot kernel's whole tiles): non-temporal -- every
  // packet byte is read once (MI355X guide, nt-weights: issued -> landed ~18 % shorter). A/B, one
  // box, 1 Mi packets: 5-tuple 16.5 vs 17.3 us, drop-all 13.7 vs 14.7; 8 Mi: 94.5 vs 103.8.
  {
    const std::string key = " ; @DMAPOLICY@", val = " nt";
    size_t q;
    while ((q = tmpl.find(key)) != std::string::npos) tmpl.replace(q, key.size(), val);
  }
  // the fixed-slot statement's window DMA: only the lanes of the chunks the program reads
  {
    const uint32_t C = xc ? 4u : c.window_chunks();
    uint64_t mask = 0;  // lane l DMAs logical chunk (l & 3) ^ ((l >> 4) & 3) (gen_tile fixed_dma)
    for (uint32_t l = 0; l < 64; l++)
      if ((((l & 3) ^ ((l >> 4) & 3))) < C) mask |= 1ull << l;
    const std::string on = C >= 4 ? "" : "s_mov_b32 exec_lo, " + hex32((uint32_t)mask) +
                                             "\ns_mov_b32 exec_hi, " + hex32((uint32_t)(mask >> 32));
    const std::string off = C >= 4 ? "" : "s_mov_b64 exec, -1";
    for (const auto& kv : {std::make_pair(std::string("; @DMAXE@"), off),
                           std::make_pair(std::string("; @DMAX@"), on)}) {
      size_t q;
      while ((q = tmpl.find(kv.first)) != std::string::npos) tmpl.replace(q, kv.first.size(), kv.second);
    }
    c.dma_chunks = C;
  }
  std::vector<Marker> marks;
  if (!find_markers(tmpl, marks)) {
    if (err) *err = "template markers not found";
    return false;
  }
  std::string src;
  size_t at = 0;
  const std::string init = c.init_code();
  // A loop program with a cooperative byte sum (coop_sum_compact) goes to the deep kernel (4
  // waves per SIMD, v[72:105] free for the program): found by a dry run of the deep kernel's body.
  // (Refills prefetching two or three windows ahead, and the cooperative sum without compaction,
  // were A/B variants until round 5: neither faster.)
  bool deep = false;
  if (xc && !c.stk && c.prefetches()) {
    for (const Marker& m : marks)
      if (m.loops == "1" && m.deep && !m.stack) {
        std::string dry;
        c.coop_emitted = xc->coop_emitted = false;
        c.deep_regs = xc->deep_regs = true;
        deep = c.body_loop(m, *xc, dry) && (c.coop_emitted || xc->coop_emitted);
        break;
      }
    c.coop_emitted = xc->coop_emitted = false;
  }
  c.deep_regs = xc ? (xc->deep_regs = deep) : false;
  // (far: the relocated bodies wait for the end of their kernel's code, its .Lfunc_end label)
  std::string pending;
  uint32_t tag = 0;
  bool far = false;
  auto copy_tmpl = [&](size_t from, size_t to) {
    for (size_t q; far && !pending.empty() && (q = tmpl.find("\n.Lfunc_end", from)) < to;) {
      src += tmpl.substr(from, q + 1 - from) + pending;
      pending.clear();
      from = q + 1;
    }
    src += tmpl.substr(from, to - from);
  };
  std::vector<std::string> bodies(marks.size());
  std::vector<char> live(marks.size(), 0);
  for (int pass = 0; pass < 2; pass++) {
  if (pass == 1 && !far) break;
  c.far_mode = far;
  if (xc) xc->far_mode = far;
  for (size_t k = 0; k < marks.size(); k++) {
    const Marker& m = marks[k];
    std::string& b = bodies[k];
    const bool loop_marker = m.loops == "1";
    // (stack-window programs: the fixed-slot kernel and the var kernel's stack statement; other
    // programs: every statement but that one)
    if (loop_marker != (xc != nullptr) || (loop_marker && m.deep != deep) ||
        (c.stk ? !(m.stack || (!loop_marker && m.fixed == "1" && (!c.stk->any_dyn || m.st)))
               : m.stack) ||
        (m.occ && (c.stk || !occ_wanted(c.n) ||
                   (m.waves == std::to_string(kOccWideWaves)) != (c.n >= kOccWideUops)))) {
      b = "s_mov_b64 exec, 0  ; (not this program's kernel)\n";
      continue;
    }
    if (!(xc ? c.body_loop(m, *xc, b) : c.body(m, b))) {
      if (err) *err = c.err;
      return false;
    }
    if (m.occ) {
      c.occ_ok = occ_regs_ok(b);
      if (!c.occ_ok) {  // (code naming the kernel's own registers: never launched)
        b = "s_mov_b64 exec, 0  ; (occupancy variant: the code needs more registers)\n";
        continue;
      }
    }
    live[k] = 1;
    far = far || (size_t)std::count(b.begin(), b.end(), '\n') > kFarLines;
  }
  }
  for (size_t k = 0; k < marks.size(); k++) {
    const Marker& m = marks[k];
    const std::string& b = bodies[k];
    copy_tmpl(at, m.init_begin);
    src += init;
    copy_tmpl(m.init_end, m.begin);
    if (far && live[k]) {
      src += "; the program's code: out of line\n" +
             long_jump(".Lbody" + m.n, "e" + std::to_string(tag++));
      pending += relocated_body(b, m.n, tag);
    } else {
      src += b;
    }
    at = m.end;
  }
  copy_tmpl(at, tmpl.size());
  if (!pending.empty()) {
    if (err) *err = "far mode: no kernel end behind a marker";
    return false;
  }
  if (asm_out) *asm_out = src;
  if (deep_out) *deep_out = deep;
  return assemble(src, code_object, err);
}

}  // namespace

// Store mode on the var tile loop (ebpf_tile_jit_varl_stack): can any lane deoptimize? A forward
// dataflow of the registers' value ranges (Compiler::av_step, the main.rs layout: r1 = 0 the
// image's start, r2 = LEN; stores change no register, an atomic's fetch makes its registers
// unknown) bounds every access's address at every reachable micro-op. No lane can leave when
//   * every register-address store ends at or below byte 128 (the overflow image's end; the host
//     also needs the stack window to start at or past 128), and
//   * if any such store may end past byte 64 (a lane may be dirty: jit.cpp ovf_*), every
//     register-address load ends at or below 128 and no constant-address load ends past 64 (a
//     dirty lane would leave at either).
// Loads straddling byte 64 are served (ldx_fixed); addresses below 0 or past mem_size fault,
// which is not a deoptimization. Calls: no proof. (`why`: the first micro-op that failed.)
bool store_mode_no_deopt(const std::vector<Uop>& uops, const StackPlan& stk, uint32_t* why,
                         std::vector<char>* kld, uint64_t* st_bound, bool* len_bound) {
  using AbsVal = Compiler::AbsVal;
  using AbsRegs = Compiler::AbsRegs;
  const uint32_t n = (uint32_t)uops.size();
  if (why) *why = UINT32_MAX;
  if (!stk.any_dyn || stk.dyn.size() != n || stk.off.size() != n || stk.pw.size() != n) return false;
  for (uint32_t i = 0; i < n; i++)
    if (uops[i].op == U_CALL) {
      if (why) *why = i;
      return false;
    }
  std::vector<AbsRegs> in(n);
  std::vector<char> seen(n, 0);
  AbsRegs init;
  for (int r = 0; r < 11; r++) init[r] = Compiler::av_const(0);
  init[2] = AbsVal();
  init[2].hi = Compiler::kLenMax, init[2].slack = 0, init[2].is_len = true;  // r2 = LEN
  init[10] = AbsVal();                                                      // r10: a launch value
  std::vector<uint32_t> work{0};
  in[0] = init;
  seen[0] = 1;
  auto flow = [&](uint32_t to, const AbsRegs& st) {
    if (to >= n) return;
    if (!seen[to]) {
      in[to] = st, seen[to] = 1, work.push_back(to);
      return;
    }
    AbsRegs m;
    bool ch = false;
    for (int r = 0; r < 11; r++) {
      m[r] = Compiler::av_meet(in[to][r], st[r]);
      ch = ch || !Compiler::av_eq(m[r], in[to][r]);
    }
    if (ch) in[to] = m, work.push_back(to);
  };
  for (size_t steps = 0; !work.empty(); steps++) {
    if (steps > 100000) return false;  // (forward programs settle far sooner)
    const uint32_t i = work.back();
    work.pop_back();
    const Uop& u = uops[i];
    if ((u.op >= U_JA && u.op <= U_JLE32 && (uint32_t)u.x <= i) ) return false;  // (a back edge)
    AbsRegs nt, tk;
    Compiler::av_step(u, in[i], nt, tk, false);
    if (u.op == U_ATOMIC) {  // (fetch forms write src, CMPXCHG writes r0)
      nt[u.src] = AbsVal();
      nt[0] = AbsVal();
    }
    if (u.op == U_EXIT || u.op == U_FAULT) continue;
    if (u.op == U_JA) {
      flow((uint32_t)u.x, tk);
      continue;
    }
    if (u.op >= U_JEQ && u.op <= U_JLE32) flow((uint32_t)u.x, tk);
    flow(i + 1, nt);
  }
  // the largest end of a register-address store / load, of a constant-address load
  uint64_t st_end = 0, ld_end = 0, kld_end = 0;
  uint32_t st_at = UINT32_MAX, ld_at = UINT32_MAX, kld_at = UINT32_MAX;
  // accesses proven to end inside the packet (base slack d >= off + width: r + off + width <=
  // LEN <= mem_size) -- a write at the frame's tail, r1 + r2 - 4 -- are bounded by mem_size, not
  // by the ranges: the host then needs mem_size <= kOvfEnd and the stack window past mem_size
  bool len_st = false, len_ld = false;
  if (kld) kld->assign(n, 0);
  for (uint32_t i = 0; i < n; i++) {
    if (!seen[i]) {  // (no lane reaches it: whatever its code, it never deoptimizes)
      if (kld && uops[i].op == U_LDX) (*kld)[i] = 1;
      continue;
    }
    const Uop& u = uops[i];
    const int64_t off = (int64_t)(int32_t)u.x;
    auto end_of = [&](const AbsVal& b) -> uint64_t {  // (unbounded: UINT64_MAX)
      if (b.hi >= (1ull << 40)) return UINT64_MAX;
      const int64_t e = (int64_t)b.hi + off + (int64_t)u.aux;
      return e < 0 ? 0 : (uint64_t)e;
    };
    auto in_len = [&](const AbsVal& b) { return b.slack >= 0 && off + (int64_t)u.aux <= b.slack; };
    if (u.op == U_ST || u.op == U_STX) {
      if (stk.off[i] != kNoStack || stk.pw[i] != kNoStack || !stk.dyn[i]) continue;
      const uint64_t e = end_of(in[i][u.dst]);
      if (e > kOvfEnd && in_len(in[i][u.dst])) {
        len_st = true;
        continue;
      }
      if (e > st_end) st_end = e, st_at = i;
    } else if (u.op == U_LDX) {
      if (stk.off[i] != kNoStack) continue;  // (the stack window)
      const AbsVal& b = in[i][u.src];
      const uint64_t e = end_of(b);
      if (b.lo == b.hi) {
        if (kld) (*kld)[i] = 1;
        if (e > kld_end) kld_end = e, kld_at = i;
      } else if (e > kOvfEnd && in_len(b)) {
        len_ld = true;
      } else if (e > ld_end) {
        ld_end = e, ld_at = i;
      }
    } else if (u.op == U_ATOMIC && stk.off[i] == kNoStack) {
      if (why) *why = i;
      return false;
    }
  }
  // (the overflow image, jit.cpp ovf_fill: a store ending past kOvfEnd deoptimizes, and so may
  // a load of a dirty lane ending past it, or a constant-address load of a filled block)
  if (st_end > kOvfEnd) {
    if (why) *why = st_at;
    return false;
  }
  if ((st_end > 64 || len_st) && (ld_end > kOvfEnd || kld_end > 64)) {
    if (why) *why = ld_end > kOvfEnd ? ld_at : kld_at;
    return false;
  }
  if (st_bound) *st_bound = std::max<uint64_t>(st_end, 128);
  if (len_bound) *len_bound = len_st || len_ld;
  return true;
}

bool jit_compile(const std::vector<Uop>& uops, const std::vector<TUop>& t,
                 std::vector<char>& code_object, std::string* err, std::string* asm_out,
                 const StackPlan* stk, bool* occ, bool main_layout) {
  if (uops.empty() || uops.size() > kJitMaxUops || t.size() < uops.size() ||
      (stk && (stk->k == 0 || stk->k > kStackMax || stk->k % 4 || stk->off.size() != uops.size() ||
               stk->pw.size() != uops.size() ||
               (stk->any_dyn && stk->dyn.size() != uops.size())))) {
    if (err) *err = "not a tile program";
    return false;
  }
  Compiler c(uops, t, false, false, stk);
  c.main_layout = main_layout;
  const bool ok = compile_into_template(c, nullptr, code_object, err, asm_out);
  if (occ) *occ = ok && c.occ_ok;
  return ok;
}

bool jit_compile_loop(const std::vector<Uop>& uops, const std::vector<TUop>& t,
                      const std::vector<TUop>& tx, std::vector<char>& code_object,
                      std::string* err, std::string* asm_out, const StackPlan* stk,
                      bool* deep, uint32_t guard_k, bool xdp_ctx, bool xdp_rebase) {
  if (uops.empty() || uops.size() > kJitMaxUops || t.size() < uops.size() ||
      tx.size() < uops.size() ||
      (stk && (stk->k == 0 || stk->k > kStackMax || stk->k % 4 || stk->off.size() != uops.size() ||
               stk->any_pw || stk->any_dyn))) {
    if (err) *err = "not a tile program";
    return false;
  }
  // (xdp_rebase: the tables with every packet load's offset 8 lower, Compiler::xdp_rebase)
  std::vector<TUop> tr, txr;
  if (xdp_rebase) {
    Compiler probe(uops, t, true, false, nullptr);
    probe.xdp_ctx = true;
    if (stk || guard_k || !xdp_ctx || !probe.rebase_ok(tx)) {
      if (err) *err = "xdp_md rebase: a load not proven past the ctx";
      return false;
    }
    tr = t, txr = tx;
    for (uint32_t i = 0; i < uops.size(); i++)
      if (probe.reached[i] && uops[i].op == U_LDX && probe.ctx_load(i) < 0) tr[i].imm -= 8, txr[i].imm -= 8;
  }
  Compiler c(uops, xdp_rebase ? tr : t, true, false, stk), xc(uops, xdp_rebase ? txr : tx, true, true, stk);
  c.xdp_ctx = xc.xdp_ctx = xdp_ctx;
  c.xdp_rebase = xc.xdp_rebase = xdp_rebase;
  if (guard_k) {  // a promoted program: its packet loads cannot reach the window of any lane
    if (stk || !c.all_loads_proven()) {  // whose LEN <= r10 - guard_k
      if (err) *err = "promoted program: a load not proven inside the packet";
      return false;
    }
    c.guard_k = xc.guard_k = guard_k;
  }
  return compile_into_template(c, &xc, code_object, err, asm_out, deep);
}

bool jit_load(const std::vector<char>& co, hipModule_t* mod, JitFns* fns) {
  hipModule_t m = nullptr;
  if (hipModuleLoadData(&m, co.data()) != hipSuccess) return false;
  JitFns f;
  if (hipModuleGetFunction(&f.fixed, m, "ebpf_tile_jit_fixed") != hipSuccess ||
      hipModuleGetFunction(&f.var, m, "ebpf_tile_jit_var") != hipSuccess ||
      hipModuleGetFunction(&f.loop, m, "ebpf_tile_jit_loop") != hipSuccess ||
      hipModuleGetFunction(&f.var_stack, m, "ebpf_tile_jit_var_stack") != hipSuccess ||
      hipModuleGetFunction(&f.loop_stack, m, "ebpf_tile_jit_loop_stack") != hipSuccess ||
      hipModuleGetFunction(&f.loop_deep, m, "ebpf_tile_jit_loop_deep") != hipSuccess ||
      hipModuleGetFunction(&f.varl, m, "ebpf_tile_jit_varl") != hipSuccess ||
      hipModuleGetFunction(&f.varl_stack, m, "ebpf_tile_jit_varl_stack") != hipSuccess ||
      hipModuleGetFunction(&f.fixed_occ, m, "ebpf_tile_jit_fixed_occ") != hipSuccess ||
      hipModuleGetFunction(&f.fixed_occw, m, "ebpf_tile_jit_fixed_occw") != hipSuccess) {
    (void)hipModuleUnload(m);
    return false;
  }
  *mod = m;
  *fns = f;
  return true;
}

}  // namespace ebpfemu
