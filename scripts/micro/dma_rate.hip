// Microbenchmark: per-CU streaming rate of (a) LDS-DMA buffer_load_dwordx4 ... lds, (b) global_load_dwordx4
// to VGPRs, (c) (b) + ds_write_b128 into LDS, from an L2-resident buffer.  Each workgroup (WAVES waves)
// streams NITER x 1 KiB pieces per wave with DEPTH pieces in flight.  Prints bytes/clk/CU.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

using lds_ptr = __attribute__((address_space(3))) void*;

template <int MODE, int DEPTH>
__global__ void __launch_bounds__(256) stream_kernel(const char* src, unsigned src_bytes, int niter, float* sink) {
  __shared__ __attribute__((aligned(16))) char lds[64 * 1024];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, (int)src_bytes, 0x00020000);
  unsigned base = ((blockIdx.x * 4 + wave) * 8192u) % (src_bytes - 65536);
  float acc = 0.f;
  for (int it = 0; it < niter; it += DEPTH) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      const unsigned off = base + ((it + d) & 63) * 1024 + lane * 16;
      char* dst = lds + wave * 16384 + (d & 15) * 1024;
      if constexpr (MODE == 0) {
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr)dst, 16, off, 0, 0, 0);
      } else {
        const uint4 v = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
        if constexpr (MODE == 2) *reinterpret_cast<uint4*>(dst + lane * 16) = v;
        else acc += __uint_as_float(v.x ^ v.y ^ v.z ^ v.w);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  if (acc == 12345.f) sink[threadIdx.x] = acc + lds[threadIdx.x];
}

template <int MODE, int DEPTH>
void run(const char* name, const char* src, unsigned bytes, float* sink, int blocks) {
  const int niter = 4096;
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  stream_kernel<MODE, DEPTH><<<blocks, 256>>>(src, bytes, niter, sink);
  hipEventRecord(e0);
  for (int k = 0; k < 5; ++k) stream_kernel<MODE, DEPTH><<<blocks, 256>>>(src, bytes, niter, sink);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  const double total = 5.0 * blocks * 4 * (double)niter * 1024;
  const double tbs = total / (ms * 1e-3) / 1e12;
  printf("%-28s depth %2d  blocks %5d: %7.2f TB/s = %6.1f B/clk/CU @2.4GHz\n", name, DEPTH, blocks, tbs, tbs * 1e12 / 256 / 2.4e9);
}

int main() {
  const unsigned bytes = 2u << 20;  // 2 MiB: L2 resident
  char* src; float* sink;
  hipMalloc(&src, bytes); hipMalloc(&sink, 4096);
  hipMemset(src, 1, bytes);
  for (int blocks : {256, 512, 1024}) {
    run<0, 4>("lds-dma dwordx4", src, bytes, sink, blocks);
    run<0, 8>("lds-dma dwordx4", src, bytes, sink, blocks);
    run<0, 16>("lds-dma dwordx4", src, bytes, sink, blocks);
    run<1, 8>("global_load_dwordx4 (vgpr)", src, bytes, sink, blocks);
    run<1, 16>("global_load_dwordx4 (vgpr)", src, bytes, sink, blocks);
    run<2, 8>("global_load + ds_write_b128", src, bytes, sink, blocks);
  }
  return 0;
}
