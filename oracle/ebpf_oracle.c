/*
 * ebpf_oracle.c — TEST INFRASTRUCTURE ONLY (see ebpf_oracle.h for the contract).
 *
 * A plain-C restatement of b1tg/ebpf-emu's interpreter. Every branch cites the reference
 * line it restates. It is written for clarity, not speed: it is the checker the HIP kernel
 * is compared against, and the CPU baseline bench.py times beside it ("kind": "port").
 */
#include "ebpf_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ins.rs:1-8 */
enum { CLASS_LD = 0, CLASS_LDX = 1, CLASS_ST = 2, CLASS_STX = 3, CLASS_ALU = 4, CLASS_JMP = 5,
       CLASS_JMP32 = 6, CLASS_ALU64 = 7 };
/* ins.rs:177-183 */
enum { MODE_IMM = 0x00, MODE_ABS = 0x20, MODE_IND = 0x40, MODE_MEM = 0x60, MODE_ATOMIC = 0xc0 };
/* ins.rs:213-228 */
enum { A_ADD, A_SUB, A_MUL, A_DIV, A_OR, A_AND, A_LSH, A_RSH, A_NEG, A_MOD, A_XOR, A_MOV, A_ARSH,
       A_END };
/* ins.rs:232-247 */
enum { J_JA, J_JEQ, J_JGT, J_JGE, J_JSET, J_JNE, J_JSGT, J_JSGE, J_CALL, J_EXIT, J_JLT, J_JLE,
       J_JSLT, J_JSLE };

static int is_ls(uint8_t code) { return (code & 7) <= CLASS_STX; } /* ins.rs:163 */

static uint64_t le64(const uint8_t* p) {
  uint64_t v = 0;
  for (int i = 7; i >= 0; i--) v = (v << 8) | p[i];
  return v;
}

/* Code::from (ins.rs:148-173) validity only; returns 0 or an OR_E_* code. */
static int check_code(uint8_t code) {
  uint8_t cls = code & 7;
  if (cls == CLASS_ALU || cls == CLASS_ALU64 || cls == CLASS_JMP || cls == CLASS_JMP32) {
    if ((code >> 4) > 0xd) return OR_E_OP; /* AOp/JOp::from assert ins.rs:251,257 */
    return 0;
  }
  uint8_t mode = code & 0xe0; /* ins.rs:165 */
  if (mode > 0xc0) return OR_E_MODE; /* ins.rs:187 */
  if (mode == 0x80 || mode == 0xa0) return OR_E_MODE; /* invalid discriminant (UB), ins.rs:188 */
  return 0;
}

long or_decode(const uint8_t* code, size_t nbytes, or_insn* out, size_t cap, size_t* bad_word) {
  if (bad_word) *bad_word = 0;
  if (nbytes % 8) { /* hexs_to_u64s, ins.rs:63-68 */
    if (bad_word) *bad_word = nbytes / 8;
    return OR_E_LEN;
  }
  size_t nw = nbytes / 8, i = 0, n = 0;
  while (i < nw) { /* u64s_to_instructions loop, ins.rs:100-117 */
    uint64_t w = le64(code + 8 * i); /* from_be of the BE-parsed hex word, ins.rs:97 */
    or_insn ins;
    /* Instruction::from field order, ins.rs:123-129: imm, imm64, off, src, dst, code */
    ins.imm = (int32_t)(uint32_t)(w >> 32);
    ins.imm64 = (int64_t)(w >> 32); /* zero-extended (u64 >> 32) as i64, ins.rs:125 */
    ins.off = (int16_t)(uint16_t)((w >> 16) & 0xffff);
    ins.src = (uint8_t)((w >> 12) & 0xf);
    ins.dst = (uint8_t)((w >> 8) & 0xf);
    ins.code = (uint8_t)(w & 0xff);
    if (bad_word) *bad_word = i;
    if (ins.src >= 12 || ins.dst >= 12) return OR_E_REG; /* Register::from assert, ins.rs:32 */
    int e = check_code(ins.code);
    if (e) return e;
    if (is_ls(ins.code) && (ins.code & 0xe0) == MODE_IMM) { /* ins.rs:107-114 */
      i += 1;
      if (i >= nw) return OR_E_LDDW; /* u64s[i] out of bounds */
      int64_t lo = (int64_t)(uint32_t)ins.imm, hi = (int64_t)le64(code + 8 * i);
      int64_t sum;
      if (__builtin_add_overflow(lo, hi, &sum)) return OR_E_LDDW_OVF; /* debug add panic */
      ins.imm64 = sum;
      ins.imm = 0;
    }
    if (n < cap) out[n] = ins;
    n++;
    i += 1;
  }
  return (long)n;
}

static uint64_t bswap16(uint64_t v) { return (uint16_t)((v >> 8 & 0xff) | (v & 0xff) << 8); }

typedef struct {
  uint8_t* mem;
  size_t mem_size;
} mmu_t;

/* Address for a first-byte-checked access, emu.rs:343-344 / 366-367 + mmu.rs:23-30.
 * Returns a status; *addr set on OK. w = bytes the caller then copies (Q16: only the first
 * byte is bounds-checked by the reference; the tail is UB -> OR_ST_MEM_UB). */
static int mem_addr(const mmu_t* m, int64_t base, int16_t off, int w, size_t* addr) {
  int64_t a;
  if (__builtin_add_overflow(base, (int64_t)off, &a)) return OR_ST_MEM; /* debug add panic */
  uint64_t ua = (uint64_t)a;                                               /* as usize */
  if (ua >= (uint64_t)m->mem_size) return OR_ST_MEM;                       /* memory[a..a+1] */
  if (ua + (uint64_t)w > (uint64_t)m->mem_size) return OR_ST_MEM_UB;
  *addr = (size_t)ua;
  return OR_ST_OK;
}

int or_run_fp(const or_insn* prog, size_t n, uint8_t* mem, size_t mem_size, int64_t regs[11],
              uint32_t fp[OR_MAX_CALL_DEPTH], size_t* fp_len_io, uint64_t max_steps,
              uint64_t* steps_out) {
  mmu_t m = {mem, mem_size};
  uint32_t pc = 0;                   /* emu.rs:23,33 */
  /* fp: emu.rs:26 (pub Vec<u32>, bounded here), the caller's initial frame stack */
  size_t fp_len = *fp_len_io > OR_MAX_CALL_DEPTH ? OR_MAX_CALL_DEPTH : *fp_len_io;
  uint64_t steps = 0;
  int st = OR_ST_OK;
  for (;;) {
    if ((size_t)pc >= n) break; /* instructions.get(pc) == None, emu.rs:49,448-450 */
    if (max_steps && steps >= max_steps) { st = OR_ST_STEPS; break; }
    const or_insn* ins = &prog[pc];
    pc += 1; /* emu.rs:63 */
    uint8_t code = ins->code, cls = code & 7;
    if (!is_ls(code)) {
      /* Code::AJ, emu.rs:65-309 */
      uint8_t op = code >> 4, source = (code >> 3) & 1;
      int64_t src;
      if (source == 0) {
        src = (int64_t)ins->imm; /* emu.rs:67 */
      } else {
        if (ins->src >= 11) { st = OR_ST_INSN; break; } /* regs[11] panics, emu.rs:69 */
        src = regs[ins->src];
      }
      if (cls == CLASS_ALU || cls == CLASS_ALU64) {
        if (ins->dst >= 11) { st = OR_ST_INSN; break; } /* emu.rs:75 */
        int64_t d = regs[ins->dst];
        int alu32 = (cls == CLASS_ALU);
        if (alu32 && op != A_END) { /* emu.rs:76-79 */
          d = (int64_t)(uint32_t)d;
          src = (int64_t)(uint32_t)src;
        }
        switch (op) {
          case A_ADD: d = (int64_t)((uint64_t)d + (uint64_t)src); break; /* :81-83 */
          case A_SUB: d = (int64_t)((uint64_t)d - (uint64_t)src); break; /* :84-86 */
          case A_MUL: d = (int64_t)((uint64_t)d * (uint64_t)src); break; /* :87-89 */
          case A_DIV: /* :90-100 unsigned; /0 -> 0 */
            d = src != 0 ? (int64_t)((uint64_t)d / (uint64_t)src) : 0;
            break;
          case A_OR: d |= src; break;   /* :101-103 */
          case A_AND: d &= src; break;  /* :104-106 */
          case A_LSH: /* :107-117 wrapping_shl masks the count */
            if (alu32) d = (int64_t)(uint32_t)((uint32_t)d << ((uint32_t)src & 31));
            else d = (int64_t)((uint64_t)d << ((uint32_t)src & 63));
            break;
          case A_RSH: /* :118-124 */
            if (alu32) d = (int64_t)(uint32_t)((uint32_t)d >> ((uint32_t)src & 31));
            else d = (int64_t)((uint64_t)d >> ((uint32_t)src & 63));
            break;
          case A_NEG: d = (int64_t)((uint64_t)d * (uint64_t)-1); break; /* :125 ignores src */
          case A_MOD: /* :126-135 unsigned; %0 leaves dst */
            if (src != 0) d = (int64_t)((uint64_t)d % (uint64_t)src);
            break;
          case A_XOR: d ^= src; break; /* :136-138 */
          case A_MOV: d = src; break;  /* :139-141 */
          case A_ARSH: {               /* :142-164 rotate, then multiply by the sign */
            int64_t sign = 1;
            if (alu32 && (int32_t)(uint32_t)d < 0) sign = -1;
            else if (!alu32 && d < 0) sign = -1;
            if (alu32) {
              uint32_t x = (uint32_t)d, k = (uint32_t)src & 31;
              int32_t r = (int32_t)(k ? (x >> k) | (x << (32 - k)) : x);
              d = (int64_t)r * sign; /* cannot overflow */
            } else {
              uint64_t x = (uint64_t)d;
              uint32_t k = (uint32_t)src & 63;
              int64_t r = (int64_t)(k ? (x >> k) | (x << (64 - k)) : x);
              if (__builtin_mul_overflow(r, sign, &d)) { st = OR_ST_ARITH; goto done; } /* :162 */
            }
            break;
          }
          case A_END: /* :165-209; source bit selects to_le (truncate) / to_be (swap) */
            if (ins->imm == 16) {
              d = source == 0 ? (int64_t)(uint16_t)d : (int64_t)bswap16((uint64_t)d);
            } else if (ins->imm == 32) {
              d = source == 0 ? (int64_t)(uint32_t)d
                              : (int64_t)__builtin_bswap32((uint32_t)d);
            } else if (ins->imm == 64) {
              if (source) d = (int64_t)__builtin_bswap64((uint64_t)d);
            } else {
              st = OR_ST_INSN; /* unreachable! :206 */
              goto done;
            }
            break;
          default: st = OR_ST_INSN; goto done; /* not reachable: decode bounds op <= 0xd */
        }
        if (alu32 && op != A_END) d = (int64_t)(uint32_t)d; /* :214-216 */
        regs[ins->dst] = d;
      } else {
        /* JMP / JMP32, emu.rs:218-304 */
        int32_t off = ins->off;
        if (ins->dst >= 11) { st = OR_ST_INSN; break; } /* :220 reads regs[dst] for every op */
        int64_t d = regs[ins->dst];
        if (cls == CLASS_JMP32) { /* :221-224 sign-extend the low words */
          d = (int64_t)(int32_t)(uint32_t)d;
          src = (int64_t)(int32_t)(uint32_t)src;
        }
        int take = 0;
        switch (op) {
          case J_JA: take = 1; break;
          case J_JEQ: take = d == src; break;
          case J_JGT: take = d > src; break; /* signed, :234-238 */
          case J_JGE: take = d >= src; break;
          case J_JSET: take = (d & src) != 0; break;
          case J_JNE: take = d != src; break;
          case J_JSGT: take = d > src; break;
          case J_JSGE: take = d >= src; break;
          case J_CALL: /* :265-272 */
            if (source != 0) { st = OR_ST_INSN; goto done; } /* todo!() */
            pc = pc + (uint32_t)off;
            if (pc == UINT32_MAX) { st = OR_ST_ARITH; goto done; } /* pc + 1 debug overflow */
            if (fp_len >= OR_MAX_CALL_DEPTH) { st = OR_ST_CALLDEPTH; goto done; }
            fp[fp_len++] = pc + 1;
            break;
          case J_EXIT: /* :273-279 */
            if (fp_len > 0) {
              pc = fp[--fp_len];
            } else {
              steps++;
              goto done; /* return None: normal stop */
            }
            break;
          case J_JLT: take = d < src; break;
          case J_JLE: take = d <= src; break;
          case J_JSLT: take = d < src; break;
          case J_JSLE: take = d <= src; break;
          default: st = OR_ST_INSN; goto done;
        }
        if (take) pc = pc + (uint32_t)off; /* wrapping_add_signed on u32, :227 */
      }
    } else {
      /* Code::LS, emu.rs:311-444 */
      uint8_t mode = code & 0xe0, size = code & 0x18;
      int w = size == 0x00 ? 4 : size == 0x08 ? 2 : size == 0x10 ? 1 : 8; /* :312-318 */
      int64_t imm = ins->imm64;                                          /* :319 */
      if (ins->src >= 11 || ins->dst >= 11) { st = OR_ST_INSN; break; }  /* :320,322 */
      int64_t src = regs[ins->src];
      int64_t r0 = regs[0];
      int64_t dst = regs[ins->dst];
      if (cls == CLASS_LD || cls == CLASS_LDX) {
        if (mode == MODE_IMM) {
          dst = imm; /* :332-334 */
        } else if (mode == MODE_MEM) {
          if (cls != CLASS_LDX) { st = OR_ST_INSN; break; } /* assert :339 */
          size_t a;
          st = mem_addr(&m, src, ins->off, w, &a);
          if (st) break;
          /* copy w bytes into the low bytes of dst; upper bytes preserved (:341-349) */
          uint64_t v = (uint64_t)dst;
          for (int i = 0; i < w; i++) {
            v &= ~((uint64_t)0xff << (8 * i));
            v |= (uint64_t)mem[a + i] << (8 * i);
          }
          dst = (int64_t)v;
        } else {
          st = OR_ST_INSN; /* ABS/IND :335-337, ATOMIC :351 */
          break;
        }
      } else {
        int64_t source = cls == CLASS_ST ? imm : src; /* :355-359 */
        if (mode == MODE_MEM) {                      /* :361-372 */
          size_t a;
          st = mem_addr(&m, dst, ins->off, w, &a);
          if (st) break;
          for (int i = 0; i < w; i++) mem[a + i] = (uint8_t)((uint64_t)source >> (8 * i));
        } else if (mode == MODE_ATOMIC) { /* :373-437 */
          int64_t a64;
          if (__builtin_add_overflow(dst, (int64_t)ins->off, &a64)) { st = OR_ST_MEM; break; }
          uint64_t ua = (uint64_t)a64;
          if (ua >= mem_size || ua + 8 > mem_size) { st = OR_ST_MEM; break; } /* read::<i64> */
          int64_t orig = (int64_t)le64(mem + ua);
          int with_fetch = (imm & 1) == 1;
          int64_t bak = 0;
          if (with_fetch) bak = orig;
          uint64_t high = 0;
          if (size == 0) { /* :382-389 */
            src = (int64_t)(uint32_t)src;
            high = (uint64_t)orig >> 32;
            orig = (int64_t)(uint32_t)orig;
            r0 = (int64_t)(uint32_t)r0;
            bak = (int64_t)(uint32_t)bak;
          }
          switch (imm & 0xfe) { /* MASK_ATOMIC :11,391 */
            case 0x00: /* ADD :392-394, non-wrapping += */
              if (__builtin_add_overflow(orig, src, &orig)) { st = OR_ST_ARITH; goto done; }
              break;
            case 0x40: orig |= src; break;
            case 0x50: orig &= src; break;
            case 0xa0: orig ^= src; break;
            case 0xe0: { int64_t t = orig; orig = src; bak = t; break; } /* XCHG :404-408 */
            case 0xf0: /* CMPXCHG :409-419 */
              if (orig == r0) orig = src;
              regs[0] = bak;
              break;
            default: st = OR_ST_INSN; goto done; /* unimplemented! :421 */
          }
          /* :427-428 recombine the high word (a 32-bit ADD carry leaks into it) */
          if (__builtin_add_overflow(orig, (int64_t)(high << 32), &orig)) {
            st = OR_ST_ARITH;
            goto done;
          }
          for (int i = 0; i < 8; i++) mem[ua + i] = (uint8_t)((uint64_t)orig >> (8 * i));
          if (with_fetch) { /* :433-436 */
            src = bak;
            regs[ins->src] = src;
          }
        } else {
          st = OR_ST_INSN; /* :438 */
          break;
        }
      }
      regs[ins->dst] = dst; /* :443 snapshot write-back (Q14) */
    }
    steps++; /* ins_count += 1, :446 */
  }
done:
  if (steps_out) *steps_out = steps;
  *fp_len_io = fp_len;
  return st;
}

int or_run(const or_insn* prog, size_t n, uint8_t* mem, size_t mem_size, int64_t regs[11],
           uint64_t max_steps, uint64_t* steps_out) {
  uint32_t fp[OR_MAX_CALL_DEPTH];
  size_t fp_len = 0;
  return or_run_fp(prog, n, mem, mem_size, regs, fp, &fp_len, max_steps, steps_out);
}

int or_run_packet(const or_insn* prog, size_t n, const uint8_t* pkt, size_t len, size_t mem_size,
                  uint64_t r10_init, uint64_t max_steps, uint64_t* r0, uint64_t* steps) {
  if (steps) *steps = 0;
  if (r0) *r0 = 0;
  if (len > mem_size) return OR_ST_BADPKT; /* main.rs:20-21 */
  uint8_t stackbuf[4096];
  uint8_t* mem = mem_size <= sizeof stackbuf ? stackbuf : (uint8_t*)malloc(mem_size);
  if (!mem) return OR_ST_BADPKT;
  memset(mem, 0, mem_size); /* main.rs:16 */
  if (len) memcpy(mem, pkt, len);
  int64_t regs[11] = {0};
  regs[2] = (int64_t)len;        /* main.rs:28 */
  regs[1] = 0;                   /* main.rs:30 */
  regs[10] = (int64_t)r10_init;  /* main.rs:31 */
  int st = or_run(prog, n, mem, mem_size, regs, max_steps, steps);
  if (r0) *r0 = (uint64_t)regs[0];
  if (mem != stackbuf) free(mem);
  return st;
}

typedef struct {
  const or_insn* prog;
  size_t n;
  const uint8_t* frames;
  const uint32_t* offsets;
  const uint16_t* lens;
  uint64_t stride, lo, hi;
  size_t mem_size;
  uint64_t r10, max_steps;
  uint64_t* r0_out;
  uint8_t* status_out;
  uint64_t counters[8];
  int xdp; /* the xdp_md convention: image = [u32 8][u32 8 + len][packet] (xdp.rs:16-20) */
} batch_job;

static void* batch_worker(void* arg) {
  batch_job* j = (batch_job*)arg;
  uint64_t cnt[8] = {0}; /* thread-local: the jobs share cache lines */
  uint8_t* img = j->xdp ? (uint8_t*)malloc(8 + 0xFFFF) : NULL;
  for (uint64_t i = j->lo; i < j->hi; i++) {
    const uint8_t* p = j->frames + (j->offsets ? (uint64_t)j->offsets[i] : i * j->stride);
    size_t len = j->lens ? j->lens[i] : (size_t)j->stride;
    if (img) { /* the bytes main.rs is handed for an XDP program: ctx, then the packet */
      if (len > 0xFFFF) len = 0xFFFF;
      const uint32_t data = 8, data_end = (uint32_t)(8 + len);
      memcpy(img, &data, 4);
      memcpy(img + 4, &data_end, 4);
      if (len + 8 <= j->mem_size) memcpy(img + 8, p, len); /* (else ST_BADPKT from the length) */
      p = img;
      len += 8;
    }
    uint64_t r0 = 0, steps = 0;
    int st = or_run_packet(j->prog, j->n, p, len, j->mem_size, j->r10, j->max_steps, &r0, &steps);
    if (j->r0_out) j->r0_out[i] = r0;
    if (j->status_out) j->status_out[i] = (uint8_t)st;
    if (st) cnt[6]++;
    else if (r0 < 5) cnt[r0]++;
    else cnt[5]++;
    cnt[7] += steps;
  }
  memcpy(j->counters, cnt, sizeof cnt);
  free(img);
  return NULL;
}

int or_run_batch(const or_insn* prog, size_t n, const uint8_t* frames, const uint32_t* offsets,
                 const uint16_t* lens, uint64_t stride, uint64_t npkts, size_t mem_size,
                 uint64_t r10_init, uint64_t max_steps, uint64_t* r0_out, uint8_t* status_out,
                 uint64_t counters[8], int threads) {
  return or_run_batch_xdp(prog, n, frames, offsets, lens, stride, npkts, mem_size, r10_init,
                          max_steps, r0_out, status_out, counters, threads, 0);
}

int or_run_batch_xdp(const or_insn* prog, size_t n, const uint8_t* frames,
                     const uint32_t* offsets, const uint16_t* lens, uint64_t stride, uint64_t npkts,
                     size_t mem_size, uint64_t r10_init, uint64_t max_steps, uint64_t* r0_out,
                     uint8_t* status_out, uint64_t counters[8], int threads, int xdp) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  batch_job jobs[256];
  pthread_t tids[256];
  for (int t = 0; t < threads; t++) {
    batch_job* j = &jobs[t];
    memset(j, 0, sizeof *j);
    j->prog = prog; j->n = n; j->frames = frames; j->offsets = offsets; j->lens = lens;
    j->stride = stride; j->mem_size = mem_size; j->r10 = r10_init; j->max_steps = max_steps;
    j->r0_out = r0_out; j->status_out = status_out; j->xdp = xdp;
    j->lo = npkts * (uint64_t)t / (uint64_t)threads;
    j->hi = npkts * (uint64_t)(t + 1) / (uint64_t)threads;
  }
  for (int t = 1; t < threads; t++) pthread_create(&tids[t], NULL, batch_worker, &jobs[t]);
  batch_worker(&jobs[0]);
  for (int t = 1; t < threads; t++) pthread_join(tids[t], NULL);
  if (counters) {
    for (int t = 0; t < threads; t++)
      for (int k = 0; k < 8; k++) counters[k] += jobs[t].counters[k];
  }
  return 0;
}
