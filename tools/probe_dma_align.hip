// Probe (diagnostic): do global_load_lds_dwordx4 (LDS-DMA) and global_load_dwordx4 move the right
// 16 bytes from a source that is not 16-byte aligned? Lane l moves the 16 bytes at src + o + step l
// (step 16, 80, 24) for every o in 0..15 (into LDS, then copied out; or straight to VGPRs); the
// host compares with the source bytes.
//   hipcc --offload-arch=gfx950 -O2 tools/probe_dma_align.hip -o build/probe_dma_align
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

__global__ void probe(const uint8_t* src, uint8_t* out, uint32_t o, uint32_t step) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[64 * 16];
  const uint32_t l = threadIdx.x;
  const uintptr_t g = (uintptr_t)(src + o + step * l);
  const uint32_t dst = (uint32_t)(uintptr_t)lds;
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0\n\ts_waitcnt vmcnt(0)"
               : "=&s"(keep) : "v"(g), "s"(dst) : "memory");
  __syncthreads();
  for (int k = 0; k < 16; k++) out[16 * l + k] = lds[16 * l + k];
}

// the same through a plain 16-byte load of an align-1 type (hipcc emits global_load_dwordx4)
typedef uint4 __attribute__((aligned(1))) uint4_any;
__global__ void probe_plain(const uint8_t* src, uint8_t* out, uint32_t o, uint32_t step) {
  const uint32_t l = threadIdx.x;
  *(uint4*)(out + 16 * l) = *(const uint4_any*)(src + o + step * l);
}

int main() {
  const size_t nb = 8192;
  std::vector<uint8_t> h(nb);
  for (size_t i = 0; i < nb; i++) h[i] = (uint8_t)(i * 37 + 11);
  uint8_t *d, *o;
  hipMalloc(&d, nb);
  hipMalloc(&o, 1024);
  hipMemcpy(d, h.data(), nb, hipMemcpyHostToDevice);
  int bad_total = 0;
  for (int plain = 0; plain < 2; plain++)
  for (uint32_t step : {16u, 80u, 24u}) {
    for (uint32_t off = 0; off < 16; off++) {
      hipMemset(o, 0, 1024);
      if (plain) hipLaunchKernelGGL(probe_plain, dim3(1), dim3(64), 0, 0, d, o, off, step);
      else hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, o, off, step);
      std::vector<uint8_t> r(1024);
      if (hipMemcpy(r.data(), o, 1024, hipMemcpyDeviceToHost) != hipSuccess) { printf("hip error\n"); return 2; }
      int bad = 0;
      for (int l = 0; l < 64; l++)
        for (int k = 0; k < 16; k++)
          if (r[16 * l + k] != h[off + step * l + k]) bad++;
      printf("%s step %u offset %2u: %s (%d bytes differ)\n", plain ? "plain" : "dma", step, off,
             bad ? "WRONG" : "ok", bad);
      bad_total += bad;
    }
  }
  printf("%s\n", bad_total ? "UNALIGNED 16-BYTE LOADS: WRONG DATA" : "UNALIGNED 16-BYTE LOADS: EXACT");
  return 0;
}
