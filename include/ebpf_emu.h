/*
 * ebpf_emu.h — C ABI of libebpfemu.so, the MI355X-native batched eBPF/XDP interpreter.
 *
 * Drop-in boundary for b1tg/ebpf-emu's load-program / run(packet) -> verdict surface
 * (reference snapshot 2024-12-20). Each entry point names the reference interface it
 * replaces. Plain pointers and sizes only; no torch / C++ types. Every call returns an int:
 * 0 = OK, < 0 = EBPF_E* (no aborts). Per-packet faults go to a status array instead of the
 * reference's process-killing panics.
 *
 * Threading: a loaded program is immutable and may be shared across host threads and
 * devices. Batch launches are asynchronous and ordered on the caller's HIP stream. The library's
 * per-(device, stream) workspace (counter shards, the deopt list, the overflow images) is found
 * and grown under a lock and never freed while the library is loaded, so host threads may launch
 * concurrently; but launches on the SAME stream from two threads must be ordered by the caller
 * (as any work on one HIP stream): the workspace is reused by every launch on that stream.
 */
#ifndef EBPF_EMU_H
#define EBPF_EMU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ebpf_prog ebpf_prog;
typedef struct ihipStream_t* ebpf_stream_t; /* == hipStream_t */

/* ---- error codes (load-time rejects mirror the reference's decode panics) ---- */
#define EBPF_OK             0
#define EBPF_EINVAL        (-1)  /* bad argument */
#define EBPF_ELEN          (-2)  /* image not a whole number of 8-byte words (ins.rs:66-67) */
#define EBPF_EREG          (-3)  /* register nibble >= 12 (ins.rs:32) */
#define EBPF_EOP           (-4)  /* ALU/JMP op > 0xd (ins.rs:251,257) */
#define EBPF_EMODE         (-5)  /* LS mode 0xe0 (ins.rs:187) or invalid discriminant 0x80/0xa0 */
#define EBPF_ELDDW         (-6)  /* wide instruction missing its second word (ins.rs:112) */
#define EBPF_ELDDW_OVF     (-7)  /* imm64 fold overflow (debug-build panic, ins.rs:112) */
#define EBPF_EHEX          (-8)  /* malformed hex (ins.rs:46-74 error strings) */
#define EBPF_ENOMEM        (-9)
#define EBPF_EHIP          (-10) /* a HIP runtime call failed */
#define EBPF_ETOOBIG       (-11) /* program beyond the device limit (EBPF_MAX_INSNS) */
#define EBPF_ERCCL         (-12) /* an RCCL call failed */
#define EBPF_EPCAP         (-13) /* not a classic pcap capture, or a truncated record */
#define EBPF_EJIT          (-14) /* the program compiler failed (amd_comgr assembler/linker) */

/* ---- per-packet status (u8) ---- */
#define EBPF_ST_OK          0  /* exit with empty frame stack or pc past the end (emu.rs:49,277) */
#define EBPF_ST_MEM         1  /* memory bounds / address-overflow panic (mmu.rs:16,26; emu.rs:344) */
#define EBPF_ST_MEM_UB      2  /* first byte in bounds, tail not: UB in the reference (mmu.rs:23-30) */
#define EBPF_ST_INSN        3  /* runtime instruction panic (emu.rs:206,270,336,339,351,421,438) */
#define EBPF_ST_ARITH       4  /* debug-build overflow panic (emu.rs:162,268,393,427) */
#define EBPF_ST_STEPS       5  /* step budget exhausted (reference: no limit, hangs; emu.rs:452) */
#define EBPF_ST_CALLDEPTH   6  /* frame stack deeper than EBPF_MAX_CALL_DEPTH */
#define EBPF_ST_BADPKT      7  /* packet longer than the memory image (main.rs:20-21) */
#define EBPF_ST_JIT         8  /* a compiled kernel's load-time proof did not hold for this packet
                                 (a library bug, never expected: the packet was not run) */

/* ---- verdict byte (xdp_action, xdp.rs:3-9) ---- */
#define EBPF_XDP_ABORTED    0
#define EBPF_XDP_DROP       1
#define EBPF_XDP_PASS       2
#define EBPF_XDP_TX         3
#define EBPF_XDP_REDIRECT   4
#define EBPF_VERDICT_OTHER  0xFE /* r0 >= 5 */
#define EBPF_VERDICT_FAULT  0xFF /* status != OK */

/* ---- counters[EBPF_NCOUNTERS] (accumulated, u64) ---- */
#define EBPF_CNT_R0_0       0   /* ... EBPF_CNT_R0_0 + 4: r0 == 0..4 */
#define EBPF_CNT_OTHER      5   /* r0 >= 5 */
#define EBPF_CNT_FAULT      6   /* status != OK */
#define EBPF_CNT_RETIRED    7   /* eBPF instructions executed */
#define EBPF_NCOUNTERS      8

#define EBPF_MAX_INSNS      65536  /* decoded instructions per program */
#define EBPF_MAX_CALL_DEPTH 64
/* ebpf_batch.flags: run on the general interpreter even when the program qualifies for the
 * forward-jump fast path (differential testing; results are identical by contract). */
#define EBPF_BATCH_GENERIC 1u
/* ebpf_batch.flags: the xdp_md calling convention (xdp.rs:16-20, struct xdp_md { u32 data;
 * u32 data_end; }). Each packet's memory image becomes [xdp_md][packet][zeros]: data = 8,
 * data_end = 8 + len at image offsets 0 and 4, the packet at offset 8, so r1 (= 0) is the ctx
 * pointer, standard XDP programs run unchanged, and r2 = 8 + len (main.rs:18-29 gives r2 the
 * image length). This is exactly the image the reference executes when main.rs is handed the
 * ctx-prefixed bytes. The compiled forward kernels (and the tile interpreter on offsets / lens
 * layouts) run such a batch in place: the ctx is synthesised in each packet's LDS window and the
 * packet read 8 bytes further on, with no extra pass over the frames. Other kernels (loop
 * programs, the general interpreter) run images the library stages in the workspace first.
 * Requires mem_size <= 65528. */
#define EBPF_BATCH_XDP_MD  2u
/* ebpf_batch.flags: run a compiled program (ebpf_prog_compile) on the tile interpreter instead
 * (differential testing; results are identical by contract). */
#define EBPF_BATCH_NO_JIT  4u
#define EBPF_DEFAULT_MEM    1024   /* main.rs:16 */
#define EBPF_DEFAULT_R10    512    /* main.rs:31 */
#define EBPF_DEFAULT_STEPS  (1ull << 22)

/* Batch descriptor. All pointers are DEVICE pointers on the device the stream belongs to.
 * Memory image per packet (main.rs:14-31 layout, sizes as launch parameters): mem_size zeroed
 * bytes, packet at [0,len), r1 = 0, r2 = len, r10 = r10, other registers 0. */
typedef struct ebpf_batch {
  const uint8_t* frames;    /* packet bytes */
  const uint32_t* offsets;  /* packet i at frames + offsets[i]; NULL => frames + i*stride */
  const uint16_t* lens;     /* packet i length; NULL => stride */
  uint64_t stride;          /* bytes between packets in the stride layout, where frames must hold
                               n * stride bytes (every slot whole, as in a ring of fixed slots) */
  uint64_t n;               /* packets */
  uint32_t mem_size;        /* bytes of the per-packet memory image, 0..2^24 (any length: Mmu.memory
                               is a Vec<u8>, mmu.rs:2-4) */
  uint32_t flags;           /* 0, or EBPF_BATCH_GENERIC | EBPF_BATCH_XDP_MD | EBPF_BATCH_NO_JIT */
  uint64_t r10;             /* initial r10 (stack top) */
  uint64_t max_steps;       /* per-packet step budget, 1..; faults EBPF_ST_STEPS beyond */
  void* workspace;          /* optional device scratch of ebpf_workspace_bytes() bytes, ZEROED before its
                               first use and then reused as is (each batch leaves its counter
                               shards at zero); one workspace per stream; NULL => library-owned
                               per (device, stream) */
  uint64_t workspace_bytes;
  const uint64_t* init_regs; /* optional device u64[11]: initial r0..r10 for every packet, replacing
                                the main.rs layout (Emu.state.regs set by the caller, emu.rs:14-17) */
  const uint32_t* init_fp;  /* optional device u32[init_fp_len]: the initial frame stack of every
                               packet, bottom first (Emu.fp is pub, emu.rs:26; an EXIT pops its top,
                               emu.rs:273-279). A batch with one runs on the general interpreter */
  uint32_t init_fp_len;     /* 0..EBPF_MAX_CALL_DEPTH */
} ebpf_batch;

/* Outputs (device pointers; any may be NULL). */
typedef struct ebpf_batch_out {
  uint8_t* verdict;   /* u8[n]: r0 < 5 ? r0 : 0xFE; 0xFF on fault */
  uint64_t* r0;       /* u64[n]: raw r0 (two's complement of the reference's i64, main.rs:43);
                         for a packet with status != EBPF_ST_OK (the reference panics) r0 is the
                         register at the fault, except on a stack-slot promoted program's kernel,
                         where it is unspecified */
  uint8_t* status;    /* u8[n]: EBPF_ST_* */
  uint64_t* counters; /* u64[EBPF_NCOUNTERS], ADDED to (not overwritten) */
  uint8_t* mem;       /* u8[n][mem_size]: final memory image per packet (Emu.state.mmu.memory) */
  uint64_t* regs;     /* u64[n][11]: final r0..r10 per packet (Emu.state.regs) */
  uint32_t* fp;       /* u32[n][EBPF_MAX_CALL_DEPTH]: final frame stack per packet, bottom first
                         (Emu.fp; non-empty when a program falls off its end inside a call) */
  uint8_t* fp_len;    /* u8[n]: its depth */
} ebpf_batch_out;

/* Fill a batch descriptor with the reference harness defaults (mem 1024, r10 512). */
void ebpf_batch_init(ebpf_batch* b);

/* Load a program from its little-endian byte image.
 * Replaces ins::u64s_to_instructions (ins.rs:96-119) + Instruction::from (ins.rs:121-132) +
 * Code::from (ins.rs:148-173); a decode panic becomes an EBPF_E* return. On error,
 * *bad_word (if non-NULL) receives the index of the offending 8-byte word. */
int ebpf_prog_load(const uint8_t* code, size_t nbytes, ebpf_prog** out, size_t* bad_word);

/* Load from hex text. Replaces ins::hexs_to_instructions (ins.rs:91-94): whitespace is
 * removed, the rest parsed as 16-digit big-endian u64 words (ins.rs:60-74). */
int ebpf_prog_load_hex(const char* hex, ebpf_prog** out, size_t* bad_word);

void ebpf_prog_free(ebpf_prog* prog);

/* Number of decoded instructions (a wide lddw counts once, ins.rs:107-116). */
size_t ebpf_prog_len(const ebpf_prog* prog);

/* Copy decoded instruction i out as the reference's Instruction fields (ins.rs:37-45). */
int ebpf_prog_insn(const ebpf_prog* prog, size_t i, int32_t* imm, int64_t* imm64, int16_t* off,
                   uint8_t* src, uint8_t* dst, uint8_t* code);

/* Memory tier the device path uses for this program: 0 = read-only packet window (no stores,
 * no calls), 1 = general per-packet image in device workspace. */
int ebpf_prog_tier(const ebpf_prog* prog);

/* 1 when the program (memory tier 0, every jump forward, <= EBPF_MAX_COMPILED_UOPS micro-ops)
 * runs on the forward-jump fast path -- for batches with max_steps >= its length and without
 * EBPF_BATCH_GENERIC; past 256 micro-ops only compiled (ebpf_prog_compile), not with
 * EBPF_BATCH_NO_JIT -- else 0; -1 for NULL. */
int ebpf_prog_forward_only(const ebpf_prog* prog);

/* Memory tier 0.5: the bytes of the stack window [r10 - k, r10) of a program whose memory writes
 * are ST/STX/ATOMIC at r10 + c (c known at load time, all in the window; atomics 4-aligned), or
 * ST/STX into the packet's first 64 bytes at load-time constant addresses (then every other load
 * must be a constant-address or stack-window one); forward jumps only, no CALL, <= 62 micro-ops.
 * Such a program keeps the window (and the stored packet bytes) in registers of the compiled
 * fixed-slot kernel, for batches in the fixed-slot layout with the main.rs register layout whose
 * window lies past every packet byte and inside the image (r10 % 4 == 0); other batches run it
 * on the general interpreter. A program with packet stores only reports a 4-byte window.
 * 0 = not such a program; -1 for NULL. */
int ebpf_prog_stack_window(const ebpf_prog* prog);

/* Store mode: ST/STX through a register whose value is not known at load time (a packet pointer
 * behind a variable-length header; reference emu.rs:354-372). Such a program runs on the compiled
 * fixed-slot kernel (fixed slots) or the var kernels with its header window in LDS; a lane whose access leaves the image bytes the kernel
 * holds is re-run by the general interpreter after the launch (the deopt pass). 0 = not store
 * mode, 1 = store mode with the deopt pass, 2 = store mode proven at load time to need no pass
 * for main.rs-layout batches (no lane can leave; a lane that did would fault EBPF_ST_JIT); -1 for
 * NULL. */
int ebpf_prog_store_mode(const ebpf_prog* prog);

/* Micro-ops (after local calls are flattened into one copy per frame stack) of the longest
 * program the compiler takes; longer programs run on the general interpreter. */
#define EBPF_MAX_COMPILED_UOPS 4096

/* Compile the program to gfx950 machine code now, if it is one the tile kernels run (memory tier
 * 0): straight-line code in pc order with direct register operands, replacing the interpreter's
 * dispatch, for programs of <= EBPF_MAX_COMPILED_UOPS micro-ops. Forward-only programs get the forward kernels
 * (batches with max_steps >= the program length); every such program also gets the loop kernel
 * (back edges, or a step budget that can bind: the exact budget of the reference's step count). Needs no
 * GPU; done implicitly by the first upload. Returns 1 = compiled, 0 = not such a program,
 * EBPF_EJIT on a compiler failure (ebpf_prog_jit_error says why; EBPF_BATCH_NO_JIT runs a compiled
 * program's batch interpreted). */
int ebpf_prog_compile(ebpf_prog* prog);

/* The compiled program's gfx950 assembly (variant 0: forward-only, batches with init_regs; 1:
 * forward-only, the main.rs register layout, whose constant-address loads are resolved; 2: the
 * loop-program kernel), for inspection: copies up to cap bytes (NUL-terminated) and sets *len to
 * the full length. EBPF_EINVAL if that variant is not compiled. */
int ebpf_prog_jit_asm(ebpf_prog* prog, int variant, char* buf, size_t cap, size_t* len);

/* Why the program is not (wholly) compiled: compiles it first, then copies up to cap bytes
 * (NUL-terminated) of the reason -- the compiler's or assembler's error, or why the program is
 * not one the compiler takes -- and sets *len to its length; "" when every variant compiled.
 * (new: no reference counterpart; diagnostics for ebpf_prog_compile) */
int ebpf_prog_jit_error(ebpf_prog* prog, char* buf, size_t cap, size_t* len);

/* Device scratch a batch needs (counter shards; tier 1 adds per-wave memory images). */
uint64_t ebpf_workspace_bytes(const ebpf_prog* prog, const ebpf_batch* batch, int device);

/* Copy the device micro-op table to `device` now (otherwise done on first run there).
 * Synchronous; call it before capturing ebpf_run_batch into a HIP graph. */
int ebpf_prog_upload(ebpf_prog* prog, int device);

/* Run a batch on the device owning `stream` (NULL = the current device's null stream).
 * Replaces, per packet, Emu::default() + Mmu setup + Emu::run() + reading state.regs[0]
 * (main.rs:14-43, emu.rs:30-45,452-458). Asynchronous, stream-ordered: one interpreter
 * kernel; with out->counters, its last workgroup folds the per-shard sums into them. */
int ebpf_run_batch(ebpf_prog* prog, const ebpf_batch* batch, const ebpf_batch_out* out,
                   ebpf_stream_t stream);

/* The kernel ebpf_run_batch would run for this batch and outputs on `device` (uploads the
 * program there first, so it needs that device): one of EBPF_KERNEL_*, or < 0 = EBPF_E*. */
#define EBPF_KERNEL_GENERAL_T0 0  /* interp_kernel, memory tier 0 (read-only packet window) */
#define EBPF_KERNEL_GENERAL_T1 1  /* interp_kernel, memory tier 1 (per-packet images in scratch) */
#define EBPF_KERNEL_DAG        2  /* dag_kernel: forward-only programs of 63..256 micro-ops */
#define EBPF_KERNEL_TILE       3  /* tile interpreter, forward-only programs */
#define EBPF_KERNEL_TILE_LOOP  4  /* tile interpreter, loop mode */
#define EBPF_KERNEL_JIT_FIXED  5  /* compiled program, fixed-slot layout (ebpf_tile_jit_fixed) */
#define EBPF_KERNEL_JIT_VAR    6  /* compiled program, other layouts (ebpf_tile_jit_var) */
#define EBPF_KERNEL_JIT_LOOP   7  /* compiled loop program (ebpf_tile_jit_loop) */
#define EBPF_KERNEL_JIT_STACK  8  /* compiled stack-window program (memory tier 0.5, fixed slots;
                                    store mode included) */
#define EBPF_KERNEL_JIT_VAR_STACK 9  /* compiled stack-window program, other layouts
                                        (ebpf_tile_jit_var_stack) */
#define EBPF_KERNEL_JIT_LOOP_STACK 10 /* compiled stack-window loop program
                                         (ebpf_tile_jit_loop_stack) */
#define EBPF_KERNEL_JIT_VARL   11 /* compiled program, offsets + lens batches: the var tile loop
                                    (ebpf_tile_jit_varl; offsets and lens 4-byte aligned, no
                                    final images) */
#define EBPF_KERNEL_JIT_VARL_STACK 12 /* the var tile loop for stack-window programs
                                         (ebpf_tile_jit_varl_stack; store mode included) */
#define EBPF_KERNEL_JIT_FIXED_OCC 13 /* compiled forward program, fixed-slot layout: the kernel's
                                        occupancy variant (ebpf_tile_jit_fixed_occ; every program
                                        whose code fits it, not xdp_md, no stack window) */
int ebpf_batch_kernel(ebpf_prog* prog, const ebpf_batch* batch, const ebpf_batch_out* out,
                      int device);

/* Whether ebpf_run_batch stages this EBPF_BATCH_XDP_MD batch's images (one copy kernel writing
 * [ctx][packet] per packet into the workspace before the program's kernel, xdp.rs:16-20) on
 * `device`: 1 staged, 0 in place (or not an xdp_md batch), < 0 = EBPF_E*. */
int ebpf_batch_staged(ebpf_prog* prog, const ebpf_batch* batch, const ebpf_batch_out* out,
                      int device);

/* Multi-GPU: shard s runs on devices[s] / streams[s] (distinct devices); the shards' counters are
 * summed with one RCCL all-reduce over xGMI, and the global totals of this call are ADDED to
 * every outs[s].counters (accumulated as in ebpf_run_batch, never overwritten; the per-shard sums
 * go through 64 bytes of the shard's workspace first -- batches[s].workspace, or the
 * library-owned one of (device, stream)). Shards are independent (no data-path exchange).
 * Requires counters in every out. A failing call leaves every caller counter untouched. Returns
 * after enqueueing (asynchronous on each stream, so calls on the same streams are ordered). */
int ebpf_run_batch_multi(ebpf_prog* prog, int nshards, const int* devices,
                         const ebpf_batch* batches, const ebpf_batch_out* outs,
                         ebpf_stream_t const* streams);

/* Host ingestion (the path starts in host memory, "a pcap buffer or NIC ring").
 * Index a classic libpcap capture held in host memory (magic a1b2c3d4 / a1b23c4d, either byte
 * order): offsets[i] / lens[i] = the byte offset and captured length of record i's packet
 * within buf. A device copy of the same bytes plus these arrays is an offsets + lens batch, so
 * the capture runs unmodified (no repacking). Records are indexed in file order; at most cap of
 * them (offsets/lens may be NULL with cap 0 to count). *n receives the number of records in
 * the buffer, *linktype the capture's link type (1 = Ethernet). Returns EBPF_EPCAP for a bad
 * header or a truncated record, EBPF_ETOOBIG for a record longer than 65535 bytes or a buffer
 * past 4 GiB (u32 offsets: index such a capture in pieces), EBPF_EINVAL when more than cap
 * records exist (the first cap are indexed). The reference reads its packet from argv
 * (main.rs:14-22); this replaces that per-packet input for whole captures. */
int ebpf_pcap_index(const uint8_t* buf, size_t nbytes, uint32_t* offsets, uint16_t* lens,
                    size_t cap, size_t* n, uint32_t* linktype);

/* Human-readable message for an EBPF_E* code. */
const char* ebpf_strerror(int err);

/* Version string of the library (build configuration). */
/* Diagnostics: with EBPFEMU_TRACE=1 in the environment, the compiled fixed-slot kernel writes
 * per-wave s_memrealtime stamps (100 MHz) into a device buffer of `device`: a ring of 4 launches
 * of 65536 waves x 16 u64 (launch k in slot k % 4, zeroed once); wave w's 16 u64 at
 * w * 16 -- [0] entry, [1..10] after each tile, [12] before and [13] after the counter flush,
 * [14] XCC_ID << 32 | HW_ID, [15] tiles. NULL / 0 when off. */
int ebpf_debug_trace(int device, void** dev_ptr, size_t* bytes);

const char* ebpf_version(void);

#ifdef __cplusplus
}
#endif
#endif
