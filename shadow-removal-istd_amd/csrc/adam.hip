// Multi-tensor Adam (torch.optim.Adam semantics, amsgrad=False, weight_decay=0) --
// the optimiser of STCGAN/stcgan.py:60-65 (lr_G 5e-5 / lr_D 2e-5, betas (0.5, 0.999)).
// One launch covers every parameter tensor of an optimiser: a device table of
// {param, grad, exp_avg, exp_avg_sq, numel, first_block} records; each block finds
// its tensor by binary search over first_block.  HBM-bound: 16 B read + 12 B written
// per element.
#include "common.hpp"

namespace stc {

constexpr int ADAM_BLOCK = 256, ADAM_ELEMS = 4;  // 4 elements per thread, 1024 per block

__global__ void __launch_bounds__(ADAM_BLOCK) adam_kernel(const long long* table, int ntensors, float lr_over_bc1,
                                                          float bc2_sqrt, float beta1, float beta2, float eps) {
  // locate tensor: largest i with first_block[i] <= blockIdx.x
  int lo = 0, hi = ntensors - 1;
  const int blk = blockIdx.x;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (table[mid * 6 + 5] <= blk) lo = mid;
    else hi = mid - 1;
  }
  const long long* rec = table + lo * 6;
  float* p = reinterpret_cast<float*>(rec[0]);
  const float* g = reinterpret_cast<const float*>(rec[1]);
  float* m = reinterpret_cast<float*>(rec[2]);
  float* v = reinterpret_cast<float*>(rec[3]);
  const long long n = rec[4];
  const long long base = (long long)(blk - rec[5]) * ADAM_BLOCK * ADAM_ELEMS;
  const float w = 1.f - beta1;
  const float omb2 = 1.f - beta2;
#pragma unroll
  for (int k = 0; k < ADAM_ELEMS; ++k) {
    const long long i = base + (long long)k * ADAM_BLOCK + threadIdx.x;
    if (i >= n) break;
    const float gi = g[i];
    float mi = m[i];
    // torch.lerp(start=m, end=g, weight=w)
    mi = fabsf(w) < 0.5f ? mi + w * (gi - mi) : gi - (gi - mi) * (1.f - w);
    float vi = v[i];
    vi = vi * beta2 + omb2 * (gi * gi);
    const float denom = sqrtf(vi) / bc2_sqrt + eps;
    p[i] = p[i] + (-lr_over_bc1) * (mi / denom);
    m[i] = mi;
    v[i] = vi;
  }
}

}  // namespace stc

using namespace stc;

extern "C" int stc_adam_step(const int64_t* table, int ntensors, int64_t total_blocks, float lr, float beta1,
                             float beta2, float eps, int step, void* stream) {
  STC_REQUIRE(ntensors > 0 && step >= 1, "stc_adam_step: bad arguments");
  const double bc1 = 1.0 - pow((double)beta1, (double)step);
  const double bc2 = 1.0 - pow((double)beta2, (double)step);
  const float step_size = (float)((double)lr / bc1);
  const float bc2_sqrt = (float)sqrt(bc2);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(adam_kernel, dim3((unsigned)total_blocks), dim3(ADAM_BLOCK), 0, st, (const long long*)table,
                     ntensors, step_size, bc2_sqrt, beta1, beta2, eps);
  STC_CHECK_LAUNCH();
  return 0;
}

extern "C" int stc_adam_elems_per_block(void) { return ADAM_BLOCK * ADAM_ELEMS; }
