// Multi-tensor Adam (torch.optim.Adam semantics, amsgrad=False, weight_decay=0) --
// the optimiser of STCGAN/stcgan.py:60-65 (lr_G 5e-5 / lr_D 2e-5, betas (0.5, 0.999)).
// One launch covers every parameter tensor of an optimiser: a device table of
// {param, grad, exp_avg, exp_avg_sq, numel, first_block} records; each block finds
// its tensor by binary search over first_block.  HBM-bound: 16 B read + 12 B written
// per element (+ 2 B per packed bf16 operand in adam_pack_kernel).
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

// ---- Adam + GEMM-operand repack in one pass (stc_adam_pack_step) ------------------------------
// A 4x4 conv / convT weight [P][Q][4][4] is updated a 16x16 (p, q) tile per block (16 contiguous
// runs of 16*16 floats, read and written with coalesced float4 accesses), with Adam exactly as
// adam_kernel, and the new values also land in an LDS tile;
// the block then writes each of the weight's packed GEMM operands (stc_pack_weights layouts: the
// bf16 / fp32 copies the convolutions read) from that tile with 16-lane-contiguous stores.  The
// separate pack pass -- re-reading every fp32 weight once per packed layout -- goes away.
// Other tensors (biases, BatchNorm affine) and weights without a packed copy: 1024 elements per
// block as adam_kernel.
constexpr int AP_W = 24;  // int64 per table record
// record: 0 param, 1 grad, 2 exp_avg, 3 exp_avg_sq, 4 numel, 5 first_block, 6 kind (0 flat, 1 4x4 weight),
// 7 P, 8 Q, 9 q-tiles, 10 packs, then per pack (11 + 5j): mode, out, N_pad, C_pad, dtype

__device__ __forceinline__ float adam_elem(float pi, float gi, float& mi, float& vi, float lr_over_bc1, float bc2_sqrt,
                                           float beta1, float beta2, float eps) {
  const float w = 1.f - beta1;
  mi = fabsf(w) < 0.5f ? mi + w * (gi - mi) : gi - (gi - mi) * (1.f - w);
  vi = vi * beta2 + (1.f - beta2) * (gi * gi);
  const float denom = sqrtf(vi) / bc2_sqrt + eps;
  return pi + (-lr_over_bc1) * (mi / denom);
}

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
template <bool NT>
__device__ __forceinline__ void st4(float* q, const float4& a) {  // NT: streaming store (not re-read this step)
  if (NT) __builtin_nontemporal_store(f32x4{a.x, a.y, a.z, a.w}, reinterpret_cast<f32x4*>(q));
  else *reinterpret_cast<float4*>(q) = a;
}
template <bool NT>
__device__ __forceinline__ float4 ld4(const float* q) {  // NT: streaming load (read once)
  if (NT) {
    const f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(q));
    return make_float4(v.x, v.y, v.z, v.w);
  }
  return *reinterpret_cast<const float4*>(q);
}

// V bit 0 (XCD): blocks b, b+8, ... (one XCD) take consecutive tiles, so the neighbouring tiles whose packed
// bf16 runs share 128-byte lines are written through one L2 close together.  Bit 1: p / m / v stored
// streaming.  Bit 2: packed operands stored streaming.  Bit 3: the 4x4 weights' p / g / m / v loaded streaming.
template <int V>
__global__ void __launch_bounds__(256) adam_pack_kernel(const long long* table, int ntensors, float lr_over_bc1,
                                                        float bc2_sqrt, float beta1, float beta2, float eps,
                                                        const float* __restrict__ coef) {
  constexpr bool XCD = V & 1, NT = V & 2, NTP = V & 4, NTL = V & 8;
  __shared__ __attribute__((aligned(16))) float tile[16][16][20];  // [p][tap][q] (rows of 20: 16-byte aligned q quads)
  if (coef != nullptr) {  // device-resident step (graph replay): the coefficients adam_coef_kernel computed
    lr_over_bc1 = coef[0];
    bc2_sqrt = coef[1];
  }
  int lo = 0, hi = ntensors - 1;
  int blk = blockIdx.x;
  if (XCD) {
    const int nwg = gridDim.x, xcd = blk & 7, q = nwg >> 3, r = nwg & 7;
    blk = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (blk >> 3);
  }
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (table[mid * AP_W + 5] <= blk) lo = mid;
    else hi = mid - 1;
  }
  const long long* rec = table + lo * AP_W;
  float* p = reinterpret_cast<float*>(rec[0]);
  const float* g = reinterpret_cast<const float*>(rec[1]);
  float* m = reinterpret_cast<float*>(rec[2]);
  float* v = reinterpret_cast<float*>(rec[3]);
  const int b = blk - (int)rec[5];
  if (rec[6] == 0) {
    const long long n = rec[4];
    const long long base = (long long)b * 1024;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const long long i = base + (long long)k * 256 + threadIdx.x;
      if (i >= n) break;
      float mi = m[i], vi = v[i];
      p[i] = adam_elem(p[i], g[i], mi, vi, lr_over_bc1, bc2_sqrt, beta1, beta2, eps);
      m[i] = mi;
      v[i] = vi;
    }
    return;
  }
  const int P = (int)rec[7], Q = (int)rec[8], qt = (int)rec[9];
  const int p0 = (b / qt) * 16, q0 = (b % qt) * 16;
  const int np = min(16, P - p0), nq = min(16, Q - q0);
  // the tile's rows p are contiguous runs of nq*16 floats: wave w updates rows w, w+4, w+8, w+12,
  // lane l the 4 floats at 4l of the run (one 1 KiB coalesced access per wave-instruction)
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int ql = lane >> 2, t0 = (lane & 3) * 4;
  // all four rows' loads are issued before any store (p / m / v may alias as far as the compiler
  // knows: stores between them would serialise the rows' memory latencies)
  float4 pp[4], gg[4], mm[4], vv[4];
  bool ok[4];
  long long e0[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int pl = wave + 4 * r;
    ok[r] = pl < np && ql < nq;
    e0[r] = ok[r] ? ((long long)(p0 + pl) * Q + q0) * 16 + 4 * lane : 0;
    if (ok[r]) {
      pp[r] = ld4<NTL>(p + e0[r]);
      gg[r] = ld4<NTL>(g + e0[r]);
      mm[r] = ld4<NTL>(m + e0[r]);
      vv[r] = ld4<NTL>(v + e0[r]);
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    if (!ok[r]) continue;
    const int pl = wave + 4 * r;
    float4 a = pp[r], mq = mm[r], vq = vv[r];
    const float4 gq = gg[r];
    a.x = adam_elem(a.x, gq.x, mq.x, vq.x, lr_over_bc1, bc2_sqrt, beta1, beta2, eps);
    a.y = adam_elem(a.y, gq.y, mq.y, vq.y, lr_over_bc1, bc2_sqrt, beta1, beta2, eps);
    a.z = adam_elem(a.z, gq.z, mq.z, vq.z, lr_over_bc1, bc2_sqrt, beta1, beta2, eps);
    a.w = adam_elem(a.w, gq.w, mq.w, vq.w, lr_over_bc1, bc2_sqrt, beta1, beta2, eps);
    st4<NT>(p + e0[r], a);
    st4<NT>(m + e0[r], mq);
    st4<NT>(v + e0[r], vq);
    tile[pl][t0][ql] = a.x; tile[pl][t0 + 1][ql] = a.y;
    tile[pl][t0 + 2][ql] = a.z; tile[pl][t0 + 3][ql] = a.w;
  }
  __syncthreads();
  const int npk = (int)rec[10];
  for (int j = 0; j < npk; ++j) {
    const long long* pk = rec + 11 + 5 * j;
    const int mode = (int)pk[0];
    char* out = reinterpret_cast<char*>(pk[1]);
    const int npad = (int)pk[2], cpad = (int)pk[3], f32 = (int)pk[4] == STC_F32;
    const bool phased = mode == STC_PACK_CONV_DGRAD || mode == STC_PACK_CONVT_FWD;
    const bool n_is_p = mode == STC_PACK_CONV_FWD || mode == STC_PACK_CONVT_DGRAD;
    const int nb = n_is_p ? p0 : q0, cb = n_is_p ? q0 : p0;
    // 4 consecutive c per thread-iteration (one 8- / 16-byte store), 4 iterations per thread
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int idx = threadIdx.x + 256 * k;
      const int c4 = (idx & 3) * 4, rest = idx >> 2, nl = rest >> 4;
      long long o;
      int tap;
      if (!phased) {
        tap = rest & 15;
        o = ((long long)(nb + nl) * 16 + tap) * cpad + cb + c4;
      } else {
        const int t = rest & 3, z = (rest >> 2) & 3, ph = z >> 1, pw = z & 1;
        tap = ((1 - ph) + 2 * (t >> 1)) * 4 + (1 - pw) + 2 * (t & 1);
        o = (((long long)z * npad + nb + nl) * 4 + t) * cpad + cb + c4;
      }
      // (p, q) of the 4 values: n_is_p -> p = nl, q = c4..c4+3; else q = nl, p = c4..c4+3
      const int lim_n = n_is_p ? np : nq, lim_c = n_is_p ? nq : np;
      if (nl >= lim_n || c4 >= lim_c) continue;
      float w[4];
      if (n_is_p) {
        const float4 q4 = *reinterpret_cast<const float4*>(&tile[nl][tap][c4]);
        w[0] = q4.x; w[1] = q4.y; w[2] = q4.z; w[3] = q4.w;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) w[e] = tile[c4 + e][tap][nl];
      }
      if (c4 + 4 <= lim_c) {
        if (f32) {
          st4<NTP>(reinterpret_cast<float*>(out) + o, make_float4(w[0], w[1], w[2], w[3]));
        } else {
          const u32x2 u{pack_bf16x2(w[0], w[1]), pack_bf16x2(w[2], w[3])};
          if (NTP) __builtin_nontemporal_store(u, reinterpret_cast<u32x2*>(reinterpret_cast<bf16*>(out) + o));
          else *reinterpret_cast<u32x2*>(reinterpret_cast<bf16*>(out) + o) = u;
        }
      } else {
        for (int e = 0; e < lim_c - c4; ++e) {
          if (f32) reinterpret_cast<float*>(out)[o + e] = w[e];
          else st1<bf16>(reinterpret_cast<bf16*>(out) + o + e, w[e]);
        }
      }
    }
  }
}

// ---- device-resident step count (a captured train step replays with the count advancing on the GPU):
// one thread advances the group's step and turns it into the two Adam coefficients exactly as the host
// path does -- lr / (1 - beta1^step) in double, rounded to float, and the float sqrt(1 - beta2^step) --
// from tables of 1 - beta1^s (double) and sqrt(1 - beta2^s) (float) the host filled with the same
// libm formulas (bit-identical to stc_adam_pack_step at every step).
__global__ void adam_coef_kernel(long long* __restrict__ step, const double* __restrict__ lr,
                                 const double* __restrict__ bc1_tab, const float* __restrict__ bc2s_tab, int tab_len,
                                 float* __restrict__ coef) {
  if (threadIdx.x != 0) return;
  const long long s = step[0] + 1;
  step[0] = s;
  const int i = (int)(s < tab_len ? s : tab_len - 1);
  coef[0] = (float)(lr[0] / bc1_tab[i]);
  coef[1] = bc2s_tab[i];
}

// ---- multi-tensor gradient accumulation: dst[e] += src[e] for up to GA_MAX tensors in one launch.
// Replaces the per-parameter ATen adds autograd issues when a network is called twice in one
// differentiated graph (the discriminators' real + fake calls, STCGAN/stcgan.py:215-227).
constexpr int GA_MAX = 16;
constexpr int GA_ELEMS = 4096;  // per block: 256 threads x 4 float4
struct GradAccArgs {
  float* dst[GA_MAX];
  const float* src[GA_MAX];
  long long n[GA_MAX];
  int first_block[GA_MAX + 1];
  int vec[GA_MAX];
  int count;
};

__global__ __launch_bounds__(256) void grad_acc_kernel(GradAccArgs a) {
  const int b = blockIdx.x;
  int e = 0;
  while (e + 1 < a.count && b >= a.first_block[e + 1]) ++e;
  const long long n = a.n[e];
  float* __restrict__ d = a.dst[e];
  const float* __restrict__ s = a.src[e];
  const long long base = (long long)(b - a.first_block[e]) * GA_ELEMS;
  if (a.vec[e]) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const long long i = base + (long long)(k * 256 + threadIdx.x) * 4;
      if (i + 3 < n) {
        float4 x = *reinterpret_cast<const float4*>(d + i);
        const float4 y = *reinterpret_cast<const float4*>(s + i);
        x.x += y.x; x.y += y.y; x.z += y.z; x.w += y.w;
        *reinterpret_cast<float4*>(d + i) = x;
      } else {
        for (long long j = i; j < n && j < i + 4; ++j) d[j] += s[j];
      }
    }
  } else {
    for (int k = threadIdx.x; k < GA_ELEMS; k += 256) {
      const long long i = base + k;
      if (i < n) d[i] += s[i];
    }
  }
}

// The update launch: adam_pack_kernel<10> -- streaming p / m / v stores and streaming loads (nothing re-reads
// them this step) took the generators' update 961 -> 730 us and the train step -0.2 ms (interleaved pairs);
// streaming the packed operands was slower (the next forward reads them from the memory-side cache) and the
// XCD grouping gained nothing (profiles/r03/diag/adam_variants.log: the other V bits, all bit-identical).
static inline auto adam_pack_fn() { return adam_pack_kernel<10>; }

}  // namespace stc

using namespace stc;

extern "C" int stc_adam_pack_step(const int64_t* table, int ntensors, int64_t total_blocks, float lr, float beta1,
                                  float beta2, float eps, int step, void* stream) {
  STC_REQUIRE(ntensors > 0 && step >= 1, "stc_adam_pack_step: bad arguments");
  const double bc1 = 1.0 - pow((double)beta1, (double)step);
  const double bc2 = 1.0 - pow((double)beta2, (double)step);
  hipLaunchKernelGGL(adam_pack_fn(), dim3((unsigned)total_blocks), dim3(256), 0, (hipStream_t)stream,
                     (const long long*)table, ntensors, (float)((double)lr / bc1), (float)sqrt(bc2), beta1, beta2, eps,
                     (const float*)nullptr);
  STC_CHECK_LAUNCH();
  return 0;
}

extern "C" int stc_adam_pack_step_dev(const int64_t* table, int ntensors, int64_t total_blocks, int64_t* step_dev,
                                      const double* lr_dev, const double* bc1_tab, const float* bc2s_tab, int tab_len,
                                      float* coef_dev, float beta1, float beta2, float eps, void* stream) {
  STC_REQUIRE(ntensors > 0 && step_dev && lr_dev && bc1_tab && bc2s_tab && coef_dev && tab_len >= 2,
              "stc_adam_pack_step_dev: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(adam_coef_kernel, dim3(1), dim3(64), 0, st, (long long*)step_dev, lr_dev, bc1_tab, bc2s_tab,
                     tab_len, coef_dev);
  STC_CHECK_LAUNCH();
  hipLaunchKernelGGL(adam_pack_fn(), dim3((unsigned)total_blocks), dim3(256), 0, st, (const long long*)table,
                     ntensors, 0.f, 1.f, beta1, beta2, eps, (const float*)coef_dev);
  STC_CHECK_LAUNCH();
  return 0;
}

// The two halves of stc_adam_pack_step_dev, for an update split into several launches (the buckets of a
// network's gradients updated as the backward completes them, optim.Adam overlap): the step count advanced
// once, then any number of table launches reading its coefficients.
extern "C" int stc_adam_coef_dev(int64_t* step_dev, const double* lr_dev, const double* bc1_tab, const float* bc2s_tab,
                                 int tab_len, float* coef_dev, void* stream) {
  STC_REQUIRE(step_dev && lr_dev && bc1_tab && bc2s_tab && coef_dev && tab_len >= 2, "stc_adam_coef_dev: bad arguments");
  hipLaunchKernelGGL(adam_coef_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, (long long*)step_dev, lr_dev, bc1_tab,
                     bc2s_tab, tab_len, coef_dev);
  STC_CHECK_LAUNCH();
  return 0;
}

// One table launch of the update with host coefficients (coef_dev == nullptr: lr / (1 - beta1^step) and
// sqrt(1 - beta2^step) computed here exactly as stc_adam_pack_step) or the device ones stc_adam_coef_dev wrote.
extern "C" int stc_adam_pack_apply(const int64_t* table, int ntensors, int64_t total_blocks, float lr, int step,
                                   const float* coef_dev, float beta1, float beta2, float eps, void* stream) {
  STC_REQUIRE(ntensors > 0 && (coef_dev != nullptr || step >= 1), "stc_adam_pack_apply: bad arguments");
  float lbc1 = 0.f, bc2s = 1.f;
  if (coef_dev == nullptr) {
    const double bc1 = 1.0 - pow((double)beta1, (double)step);
    const double bc2 = 1.0 - pow((double)beta2, (double)step);
    lbc1 = (float)((double)lr / bc1);
    bc2s = (float)sqrt(bc2);
  }
  hipLaunchKernelGGL(adam_pack_fn(), dim3((unsigned)total_blocks), dim3(256), 0, (hipStream_t)stream,
                     (const long long*)table, ntensors, lbc1, bc2s, beta1, beta2, eps, coef_dev);
  STC_CHECK_LAUNCH();
  return 0;
}

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

extern "C" int stc_grad_accumulate(int ntensors, float* const* dst, const float* const* src, const int64_t* numel,
                                   void* stream) {
  STC_REQUIRE(ntensors >= 0 && ntensors <= GA_MAX, "stc_grad_accumulate: 0..16 tensors per call");
  if (ntensors == 0) return 0;
  GradAccArgs a{};
  int blocks = 0;
  for (int e = 0; e < ntensors; ++e) {
    STC_REQUIRE(dst[e] != nullptr && src[e] != nullptr && numel[e] >= 0, "stc_grad_accumulate: bad tensor");
    a.dst[e] = dst[e];
    a.src[e] = src[e];
    a.n[e] = numel[e];
    a.vec[e] = ((((uintptr_t)dst[e]) | ((uintptr_t)src[e])) & 15) == 0;
    a.first_block[e] = blocks;
    const long long nb = (numel[e] + GA_ELEMS - 1) / GA_ELEMS;
    STC_REQUIRE(blocks + nb < (1ll << 30), "stc_grad_accumulate: too large");
    blocks += (int)nb;
  }
  a.first_block[ntensors] = blocks;
  a.count = ntensors;
  if (blocks == 0) return 0;
  hipLaunchKernelGGL(grad_acc_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, a);
  STC_CHECK_LAUNCH();
  return 0;
}
