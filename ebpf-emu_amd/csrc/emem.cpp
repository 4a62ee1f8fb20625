// emem.cpp — bpf_conformance plugin CLI, byte-for-byte the reference's protocol (src/main.rs):
//   emem [<memory hex>]            program hex on one stdin line
//   emem <ignored> <program hex>   when the stdin line is blank (main.rs:33-37)
// prints r0 as lowercase hex without padding (main.rs:43: "{:x}" of i64 = two's complement).
// The single execution runs on the GPU through libebpfemu.so (a batch of one packet).
// Where the reference panics (exit code 101) this CLI prints the reason to stderr and exits 101.
#include <hip/hip_runtime.h>

#include <cctype>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>
#include <vector>

#include "../../include/ebpf_emu.h"

static int panic(const std::string& msg) {
  std::fprintf(stderr, "thread 'main' panicked: %s\n", msg.c_str());
  return 101;
}

// hexs_to_u8s (ins.rs:46-59): trim, remove spaces, 2-digit chunks via from_str_radix.
static bool hexs_to_u8s(const std::string& in, std::vector<uint8_t>& out, std::string& err) {
  size_t b = 0, e = in.size();
  while (b < e && std::isspace((unsigned char)in[b])) b++;
  while (e > b && std::isspace((unsigned char)in[e - 1])) e--;
  std::string t;
  for (size_t i = b; i < e; i++)
    if (in[i] != ' ') t.push_back(in[i]);
  out.clear();
  for (size_t i = 0; i < t.size(); i += 2) {
    if (i + 2 > t.size()) { err = "invalid hex format"; return false; }
    int v = 0;
    for (size_t j = 0; j < 2; j++) {
      const char c = t[i + j];
      int d;
      if (c >= '0' && c <= '9') d = c - '0';
      else if (c >= 'a' && c <= 'f') d = c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') d = c - 'A' + 10;
      else if (c == '+' && j == 0) continue;
      else { err = "invalid digit found in string"; return false; }
      v = v * 16 + d;
    }
    out.push_back((uint8_t)v);
  }
  return true;
}

#define HIPCHECK(x)                                                  \
  do {                                                               \
    hipError_t e_ = (x);                                             \
    if (e_ != hipSuccess) return panic(hipGetErrorString(e_));       \
  } while (0)

int main(int argc, char** argv) {
  std::string line;
  std::getline(std::cin, line);  // stdin.read_line (main.rs:6-8)
  const size_t mem_cap = EBPF_DEFAULT_MEM;  // vec![0u8; 1024] (main.rs:15-17)
  std::vector<uint8_t> memory;
  uint64_t r2 = 0;
  if (argc == 2) {  // main.rs:18-29
    std::string err;
    if (!hexs_to_u8s(argv[1], memory, err)) return panic("called `Result::unwrap()` on an `Err` value: " + err);
    if (memory.size() > mem_cap) return panic("index out of bounds: the len is 1024");
    r2 = memory.size();
  }
  bool blank = true;
  for (char c : line)
    if (!std::isspace((unsigned char)c)) blank = false;
  if (blank && argc < 3) return panic("index out of bounds: the len is " + std::to_string(argc) + " but the index is 2");
  const std::string hx = blank ? std::string(argv[2]) : line;

  ebpf_prog* prog = nullptr;
  size_t bad = 0;
  int rc = ebpf_prog_load_hex(hx.c_str(), &prog, &bad);
  if (rc) return panic(std::string(ebpf_strerror(rc)) + " at word " + std::to_string(bad));

  // one packet = the memory image's first r2 bytes (zero-extended to 1024 by the kernel)
  uint8_t* d_frame = nullptr;
  uint64_t* d_out = nullptr;
  uint8_t* d_st = nullptr;
  const size_t flen = memory.empty() ? 8 : memory.size();
  HIPCHECK(hipMalloc(&d_frame, flen));
  HIPCHECK(hipMalloc(&d_out, sizeof(uint64_t)));
  HIPCHECK(hipMalloc(&d_st, 1));
  HIPCHECK(hipMemset(d_frame, 0, flen));
  if (!memory.empty()) HIPCHECK(hipMemcpy(d_frame, memory.data(), memory.size(), hipMemcpyHostToDevice));
  uint16_t len16 = (uint16_t)r2;
  uint16_t* d_len = nullptr;
  HIPCHECK(hipMalloc(&d_len, sizeof(uint16_t)));
  HIPCHECK(hipMemcpy(d_len, &len16, sizeof len16, hipMemcpyHostToDevice));

  ebpf_batch b;
  ebpf_batch_init(&b);
  b.frames = d_frame;
  b.lens = d_len;
  b.stride = flen;
  b.n = 1;
  const char* ms = std::getenv("EMEM_MAX_STEPS");
  if (ms) b.max_steps = std::strtoull(ms, nullptr, 0);
  ebpf_batch_out o{};
  o.r0 = d_out;
  o.status = d_st;
  rc = ebpf_run_batch(prog, &b, &o, nullptr);
  if (rc) return panic(ebpf_strerror(rc));
  HIPCHECK(hipDeviceSynchronize());
  uint64_t r0 = 0;
  uint8_t st = 0;
  HIPCHECK(hipMemcpy(&r0, d_out, sizeof r0, hipMemcpyDeviceToHost));
  HIPCHECK(hipMemcpy(&st, d_st, 1, hipMemcpyDeviceToHost));
  (void)hipFree(d_frame);
  (void)hipFree(d_out);
  (void)hipFree(d_st);
  (void)hipFree(d_len);
  ebpf_prog_free(prog);
  if (st != EBPF_ST_OK) {
    static const char* names[] = {"ok", "memory out of bounds", "memory access past the end (UB)",
                                  "illegal instruction", "arithmetic overflow",
                                  "step budget exhausted", "call stack overflow", "packet too large"};
    return panic(st < 8 ? names[st] : "fault");
  }
  std::printf("%llx\n", (unsigned long long)r0);
  return 0;
}
