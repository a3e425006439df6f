// Gather-rate probe (diagnostics, not part of the library): 16-B-per-lane loads
// of an NHWC bf16 tensor where a wave instruction covers either 16 pixels x 64 B
// (4 lanes per pixel: one 32-channel slice, the conv tile kernels' pattern) or
// 8 pixels x 128 B (8 lanes per pixel: a 64-channel slice, whole 128-B lines).
// Same bytes either way; prints GB/s of each pattern through registers and
// through LDS-DMA.  hipcc --offload-arch=gfx950 -O3 gather_probe.hip -o gp
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef __attribute__((address_space(3))) void lds_void_t;

template <int LPP, bool DMA>
__global__ __launch_bounds__(256) void gather(const uint4* __restrict__ src, int npix, int cstride16, int iters,
                                              uint4* __restrict__ out) {
  __shared__ uint4 buf[256 * 4];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int ppi = 64 / LPP;  // pixels per wave instruction
  uint4 acc = make_uint4(0, 0, 0, 0);
  const int m0 = (int)(uintptr_t)(lds_void_t*)buf;
  for (int it = 0; it < iters; ++it) {
    // pixels of this instruction: a pseudo-random but fixed row of the image
    const int base = ((blockIdx.x * 977 + it * 131 + wv * 37) % (npix / ppi)) * ppi;
    const int pix = base + lane / LPP, ch = lane % LPP;
    const int idx = pix * cstride16 + ch;
    if (DMA) {
      const unsigned voff = (unsigned)idx * 16u;
      const int lds = __builtin_amdgcn_readfirstlane(m0 + (it & 3) * 4096 + wv * 1024);
      const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, 0x7fffffff, 0x00020000);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(uintptr_t)lds, 16, voff, 0, 0, 0);
    } else {
      const uint4 v = src[idx];
      acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
    }
  }
  __syncthreads();
  if (DMA) acc = buf[tid];
  if (acc.x == 0x12345678u) out[blockIdx.x * 256 + tid] = acc;
}

int main() {
  const int npix = 16 * 64 * 64, C = 128, cstride16 = C * 2 / 16;  // 16 x 64 x 64 x 128 bf16 = 16.8 MB
  uint4 *src, *out;
  hipMalloc(&src, (size_t)npix * cstride16 * 16);
  hipMalloc(&out, 4096 * 256 * 16);
  hipMemset(src, 1, (size_t)npix * cstride16 * 16);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int blocks = 2048, iters = 256;
  const double bytes = (double)blocks * 256 * iters * 16;
  auto run = [&](auto kern, const char* name) {
    for (int r = 0; r < 3; ++r) kern<<<blocks, 256>>>(src, npix, cstride16, iters, out);
    hipEventRecord(e0);
    for (int r = 0; r < 10; ++r) kern<<<blocks, 256>>>(src, npix, cstride16, iters, out);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    printf("%-36s %8.1f GB/s  (%.1f B/clk/CU at 2.4 GHz)\n", name, bytes * 10 / (ms * 1e-3) / 1e9,
           bytes * 10 / (ms * 1e-3) / 256 / 2.4e9);
  };
  run(gather<4, false>, "regs: 16 px x 64 B per instr");
  run(gather<8, false>, "regs:  8 px x 128 B per instr");
  run(gather<4, true>, "lds-dma: 16 px x 64 B per instr");
  run(gather<8, true>, "lds-dma:  8 px x 128 B per instr");
  return 0;
}
