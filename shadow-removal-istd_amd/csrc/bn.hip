// BatchNorm2d forward statistics / finalize and the fused BN + activation backward
// (STCGAN/networks.py:107,109,170,179; activations :106,108,158,171,180).
//
// Forward: the conv epilogue writes the raw (pre-BN) output; stc_chan_stats
// reduces per-channel shifted sums over pixel chunks, stc_bn_finalize merges
// the chunks in a fixed order (Chan's parallel variance, fp64) and emits the
// (scale, shift) table that the *consumer* GEMM applies as its load prologue,
// plus the running-stat update.  Nothing normalised is written to HBM.
// Backward: dn = g1*act1'(n) + g2*act2'(n) is recomputed on the fly from the raw
// input (n = x*scale + shift), reduced to sum(dn), sum(dn*xhat), then applied.
// All reductions are fixed-order => bitwise reproducible.
#include <type_traits>

#include "common.hpp"

namespace stc {

constexpr int STAT_PIX = 64;  // pixels per statistics chunk (upper bound of chunk count below)

__host__ __device__ inline int stat_chunks(long long P) {
  long long c = (P + STAT_PIX - 1) / STAT_PIX;
  if (c > 1024) c = 1024;
  if (c < 1) c = 1;
  return (int)c;
}

// ---- 16-byte vectors of T (8 bf16 / 4 fp32 channels per thread)
template <typename T> struct VW;
template <> struct VW<float> {
  static constexpr int N = 4;
  __device__ __forceinline__ static void load(const float* p, float* f) {
    const float4 v = *reinterpret_cast<const float4*>(p);
    f[0] = v.x; f[1] = v.y; f[2] = v.z; f[3] = v.w;
  }
  __device__ __forceinline__ static void store(float* p, const float* f) {
    *reinterpret_cast<float4*>(p) = make_float4(f[0], f[1], f[2], f[3]);
  }
};
template <> struct VW<bf16> {
  static constexpr int N = 8;
  __device__ __forceinline__ static void load(const bf16* p, float* f) {
    const uint4 v = *reinterpret_cast<const uint4*>(p);
    const unsigned w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) { f[2 * q] = __uint_as_float(w[q] << 16); f[2 * q + 1] = __uint_as_float(w[q] & 0xffff0000u); }
  }
  __device__ __forceinline__ static void store(bf16* p, const float* f) {
    uint4 v;
    v.x = (unsigned)f2bf(f[0]) | ((unsigned)f2bf(f[1]) << 16);
    v.y = (unsigned)f2bf(f[2]) | ((unsigned)f2bf(f[3]) << 16);
    v.z = (unsigned)f2bf(f[4]) | ((unsigned)f2bf(f[5]) << 16);
    v.w = (unsigned)f2bf(f[6]) | ((unsigned)f2bf(f[7]) << 16);
    *reinterpret_cast<uint4*>(p) = v;
  }
};

// pixel index -> (b, y, x); exact float-reciprocal division below 2^24 pixels, integer division above
struct PixDiv {
  int HW, W;
  float inv_hw, inv_w;
  bool big;
};
static inline PixDiv mkpix(int B, int H, int W) {
  PixDiv d;
  d.HW = H * W; d.W = W;
  d.inv_hw = 1.f / (float)(H * W); d.inv_w = 1.f / (float)W;
  d.big = (long long)B * H * W >= (1ll << 24);
  return d;
}
__device__ __forceinline__ int qdiv(int n, int d, float inv) {
  int q = (int)((float)n * inv);
  const int r = n - q * d;
  return q + (r >= d) - (r < 0);
}
__device__ __forceinline__ void pix_bxy(const PixDiv& d, long long pix, int& b, int& y, int& x) {
  int rem;
  if (d.big) {
    b = (int)(pix / d.HW);
    rem = (int)(pix - (long long)b * d.HW);
    y = rem / d.W;
  } else {
    const int pi = (int)pix;
    b = qdiv(pi, d.HW, d.inv_hw);
    rem = pi - b * d.HW;
    y = qdiv(rem, d.W, d.inv_w);
  }
  x = rem - y * d.W;
}

template <typename T>
__device__ __forceinline__ const T* vptr(const View& v, int b, int y, int x, int c) {
  return reinterpret_cast<const T*>(v.p) + vidx(v, b, y, x, c);
}

// Reduction layout shared by the per-channel reductions: thread = (channel group cg of N channels,
// pixel lane pl); the block owns a contiguous pixel range and the lanes stride through it.
// part[chunk][c] = {n, S1, S2, shift}
template <typename T>
__global__ void __launch_bounds__(256) chan_stats_kernel(View x, PixDiv pd, long long P, int C, float* part, int nchunks) {
  constexpr int N = VW<T>::N;
  const int CG = C / N;
  const int RL = 256 / CG;
  const int cg = threadIdx.x % CG, pl = threadIdx.x / CG;
  const long long per = (P + nchunks - 1) / nchunks;
  const long long p0 = blockIdx.x * per, p1 = min(P, p0 + per);
  __shared__ float red[256][2 * N + 1];
  float s1[N], s2[N], sh[N], cnt = 0.f;
#pragma unroll
  for (int e = 0; e < N; ++e) { s1[e] = 0.f; s2[e] = 0.f; sh[e] = 0.f; }
  if (pl < RL && p0 < p1) {
    int b, yy, xx;
    pix_bxy(pd, p0, b, yy, xx);
    VW<T>::load(vptr<T>(x, b, yy, xx, N * cg), sh);
#pragma unroll 4
    for (long long pix = p0 + pl; pix < p1; pix += RL) {
      pix_bxy(pd, pix, b, yy, xx);
      float v[N];
      VW<T>::load(vptr<T>(x, b, yy, xx, N * cg), v);
#pragma unroll
      for (int e = 0; e < N; ++e) {
        const float d = v[e] - sh[e];
        s1[e] += d;
        s2[e] += d * d;
      }
      cnt += 1.f;
    }
  }
#pragma unroll
  for (int e = 0; e < N; ++e) { red[threadIdx.x][e] = s1[e]; red[threadIdx.x][N + e] = s2[e]; }
  red[threadIdx.x][2 * N] = cnt;
  __syncthreads();
  if (pl == 0) {
    float a1[N], a2[N], n = 0.f;
#pragma unroll
    for (int e = 0; e < N; ++e) { a1[e] = 0.f; a2[e] = 0.f; }
    for (int k = 0; k < RL; ++k) {  // fixed order
      const int t = k * CG + cg;
#pragma unroll
      for (int e = 0; e < N; ++e) { a1[e] += red[t][e]; a2[e] += red[t][N + e]; }
      n += red[t][2 * N];
    }
#pragma unroll
    for (int e = 0; e < N; ++e)
      *reinterpret_cast<float4*>(part + ((long long)blockIdx.x * C + N * cg + e) * 4) = make_float4(n, a1[e], a2[e], sh[e]);
  }
}

// Merge of the per-chunk statistics {n, S1 = sum(x - shift), S2 = sum((x - shift)^2), shift}:
// chunk mean m_b = shift + S1/n, chunk M2_b = S2 - S1^2/n; then (exactly, in fp64)
//   mean = sum n_b m_b / N,   M2 = sum [M2_b + n_b (m_b - mean)^2]
// in two passes over the chunks (one block per channel, fixed-order tree -> deterministic).
// (butterfly within each wave, then the 4 wave totals in a fixed order: deterministic, 2 barriers)
__device__ __forceinline__ double block_sum256(double v, double* sh) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  const double r = (sh[0] + sh[1]) + (sh[2] + sh[3]);
  __syncthreads();
  return r;
}

__global__ void __launch_bounds__(256) bn_finalize_kernel(const float* part, int nchunks, int C,
                                                          const float* gamma, const float* beta,
                                                          float* rmean, float* rvar, long long* nbt,
                                                          float momentum, float eps,
                                                          float* mean_o, float* rstd_o, float* scale, float* shift) {
  const int c = blockIdx.x;
  __shared__ double sh[256];
  // chunk partials are read in groups of 4 per thread (the 4 loads in flight together: one
  // memory latency per group -- the first layers merge up to 4096 chunks per channel)
  auto load4 = [&](int k0, float4* pp) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int k = k0 + u * 256;
      pp[u] = k < nchunks ? *reinterpret_cast<const float4*>(part + ((long long)k * C + c) * 4)
                          : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  const BnPre pre = bn_pre(c, gamma, beta, rmean, rvar);  // (issued with the partials' loads)
  auto sum1 = [&](const float4* pp, double& n, double& sm) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (pp[u].x <= 0.f) continue;
      n += pp[u].x;
      sm += (double)pp[u].x * pp[u].w + (double)pp[u].y;  // n_b * m_b = n_b*shift + S1
    }
  };
  auto sum2 = [&](const float4* pp, double mu, double& m2) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (pp[u].x <= 0.f) continue;
      const double nb = pp[u].x, s1 = pp[u].y, r = s1 / nb;
      double q = (double)pp[u].z - s1 * r;
      if (q < 0) q = 0;
      const double d = (double)pp[u].w + r - mu;
      m2 += q + nb * d * d;
    }
  };
  // up to 4096 chunks: every thread loads its (up to) 4 groups of 4 partials at once and keeps them in registers
  // for both passes (one memory latency); the sums run in the loop's order below, so the results are the same
  auto in_regs = [&](auto Gc, double& n, double& sm, double& m2) {
    constexpr int G = decltype(Gc)::value;
    float4 pp[G][4];
#pragma unroll
    for (int g = 0; g < G; ++g) load4(threadIdx.x + 1024 * g, pp[g]);
#pragma unroll
    for (int g = 0; g < G; ++g) sum1(pp[g], n, sm);
    n = block_sum256(n, sh);
    sm = block_sum256(sm, sh);
    const double mu = n > 0 ? sm / n : 0.0;
#pragma unroll
    for (int g = 0; g < G; ++g) sum2(pp[g], mu, m2);
    sm = mu;
  };
  double n = 0, sm = 0, m2 = 0;
  if (nchunks <= 1024) {
    in_regs(std::integral_constant<int, 1>{}, n, sm, m2);
  } else if (nchunks <= 2048) {
    in_regs(std::integral_constant<int, 2>{}, n, sm, m2);
  } else if (nchunks <= 4096) {
    in_regs(std::integral_constant<int, 4>{}, n, sm, m2);
  } else {
    for (int k0 = threadIdx.x; k0 < nchunks; k0 += 1024) {
      float4 pp[4];
      load4(k0, pp);
      sum1(pp, n, sm);
    }
    n = block_sum256(n, sh);
    sm = block_sum256(sm, sh);
    const double mu = n > 0 ? sm / n : 0.0;
    for (int k0 = threadIdx.x; k0 < nchunks; k0 += 1024) {
      float4 pp[4];
      load4(k0, pp);
      sum2(pp, mu, m2);
    }
    sm = mu;
  }
  const double N = n, mu = sm;
  const double M2 = block_sum256(m2, sh);
  if (threadIdx.x == 0)
    bn_finalize_store(c, N, mu, M2, pre, rmean, rvar, nbt, momentum, eps, mean_o, rstd_o, scale, shift);
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// The same merge with one wave per channel (4 channels per block, no block barriers): the
// finalize runs once per BatchNorm per pass, so its latency, not its bytes, is what it costs.
__global__ void __launch_bounds__(256) bn_finalize_wave_kernel(const float* part, int nchunks, int C,
                                                               const float* gamma, const float* beta,
                                                               float* rmean, float* rvar, long long* nbt,
                                                               float momentum, float eps,
                                                               float* mean_o, float* rstd_o, float* scale, float* shift) {
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= C) return;
  auto load4 = [&](int k0, float4* pp) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int k = k0 + u * 64;
      pp[u] = k < nchunks ? *reinterpret_cast<const float4*>(part + ((long long)k * C + c) * 4)
                          : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  const BnPre pre = bn_pre(c, gamma, beta, rmean, rvar);  // (issued with the partials' loads)
  auto sum1 = [&](const float4* pp, double& n, double& sm) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (pp[u].x <= 0.f) continue;
      n += pp[u].x;
      sm += (double)pp[u].x * pp[u].w + (double)pp[u].y;
    }
  };
  auto sum2 = [&](const float4* pp, double mu, double& m2) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (pp[u].x <= 0.f) continue;
      const double nb = pp[u].x, s1 = pp[u].y, r = s1 / nb;
      double q = (double)pp[u].z - s1 * r;
      if (q < 0) q = 0;
      const double d = (double)pp[u].w + r - mu;
      m2 += q + nb * d * d;
    }
  };
  // up to 1024 chunks: every lane loads its (up to) 4 groups of 4 partials at once and keeps them in registers for
  // both passes (one memory latency); the sums run in the loop's order below, so the results are the same
  auto in_regs = [&](auto Gc, double& n, double& sm, double& m2) {
    constexpr int G = decltype(Gc)::value;
    float4 pp[G][4];
#pragma unroll
    for (int g = 0; g < G; ++g) load4(lane + 256 * g, pp[g]);
#pragma unroll
    for (int g = 0; g < G; ++g) sum1(pp[g], n, sm);
    n = wave_sum(n);
    sm = wave_sum(sm);
    const double mu = n > 0 ? sm / n : 0.0;
#pragma unroll
    for (int g = 0; g < G; ++g) sum2(pp[g], mu, m2);
    return mu;
  };
  double n = 0, sm = 0, m2 = 0, mu;
  if (nchunks <= 256) {
    mu = in_regs(std::integral_constant<int, 1>{}, n, sm, m2);
  } else if (nchunks <= 512) {
    mu = in_regs(std::integral_constant<int, 2>{}, n, sm, m2);
  } else if (nchunks <= 1024) {
    mu = in_regs(std::integral_constant<int, 4>{}, n, sm, m2);
  } else {
    for (int k0 = lane; k0 < nchunks; k0 += 256) {
      float4 pp[4];
      load4(k0, pp);
      sum1(pp, n, sm);
    }
    n = wave_sum(n);
    sm = wave_sum(sm);
    mu = n > 0 ? sm / n : 0.0;
    for (int k0 = lane; k0 < nchunks; k0 += 256) {
      float4 pp[4];
      load4(k0, pp);
      sum2(pp, mu, m2);
    }
  }
  const double M2 = wave_sum(m2);
  if (lane == 0) bn_finalize_store(c, n, mu, M2, pre, rmean, rvar, nbt, momentum, eps, mean_o, rstd_o, scale, shift);
}

// eval-mode table from running statistics
__global__ void bn_eval_table_kernel(int C, const float* gamma, const float* beta, const float* rmean,
                                     const float* rvar, float eps, float* scale, float* shift) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float rs = 1.f / sqrtf(rvar[c] + eps);
  const float sc = gamma[c] * rs;
  scale[c] = sc;
  shift[c] = beta[c] - rmean[c] * sc;
}

struct GradIn {
  View g1, g2;
  float s1, s2;
  int has1, has2;
};

template <typename T>
__device__ __forceinline__ void dn_of(const GradIn& gi, int b, int y, int x, int c, const float* n, float* d) {
  constexpr int N = VW<T>::N;
#pragma unroll
  for (int e = 0; e < N; ++e) d[e] = 0.f;
  if (gi.has1) {
    float g[N];
    VW<T>::load(vptr<T>(gi.g1, b, y, x, c), g);
#pragma unroll
    for (int e = 0; e < N; ++e) d[e] += g[e] * dact(n[e], gi.s1);
  }
  if (gi.has2) {
    float g[N];
    VW<T>::load(vptr<T>(gi.g2, b, y, x, c), g);
#pragma unroll
    for (int e = 0; e < N; ++e) d[e] += g[e] * dact(n[e], gi.s2);
  }
}

template <int N>
__device__ __forceinline__ void ldc(const float* p, float* f) {
#pragma unroll
  for (int e = 0; e < N; e += 4) {
    const float4 v = *reinterpret_cast<const float4*>(p + e);
    f[e] = v.x; f[e + 1] = v.y; f[e + 2] = v.z; f[e + 3] = v.w;
  }
}

// part2[chunk][c] = {sum dn, sum dn*xhat}
template <typename T>
__global__ void __launch_bounds__(256) bn_bwd_reduce_kernel(View x, PixDiv pd, long long P, int C, const float* scale,
                                                            const float* shift, const float* mean, const float* rstd,
                                                            GradIn gi, float* part, int nchunks) {
  constexpr int N = VW<T>::N;
  const int CG = C / N;
  const int RL = 256 / CG;
  const int cg = threadIdx.x % CG, pl = threadIdx.x / CG;
  const long long per = (P + nchunks - 1) / nchunks;
  const long long p0 = blockIdx.x * per, p1 = min(P, p0 + per);
  __shared__ float red[256][2 * N];
  float a[N], bs[N];
#pragma unroll
  for (int e = 0; e < N; ++e) { a[e] = 0.f; bs[e] = 0.f; }
  if (pl < RL) {
    const int c = N * cg;
    float sc[N], shf[N], mu[N], rs[N];
    ldc<N>(scale + c, sc); ldc<N>(shift + c, shf); ldc<N>(mean + c, mu); ldc<N>(rstd + c, rs);
#pragma unroll 4
    for (long long pix = p0 + pl; pix < p1; pix += RL) {
      int b, yy, xx;
      pix_bxy(pd, pix, b, yy, xx);
      float v[N], n[N], d[N];
      VW<T>::load(vptr<T>(x, b, yy, xx, c), v);
#pragma unroll
      for (int e = 0; e < N; ++e) n[e] = fmaf(v[e], sc[e], shf[e]);
      dn_of<T>(gi, b, yy, xx, c, n, d);
#pragma unroll
      for (int e = 0; e < N; ++e) {
        a[e] += d[e];
        bs[e] += d[e] * (v[e] - mu[e]) * rs[e];
      }
    }
  }
#pragma unroll
  for (int e = 0; e < N; ++e) { red[threadIdx.x][e] = a[e]; red[threadIdx.x][N + e] = bs[e]; }
  __syncthreads();
  if (pl == 0) {
    float r0[N], r1[N];
#pragma unroll
    for (int e = 0; e < N; ++e) { r0[e] = 0.f; r1[e] = 0.f; }
    for (int k = 0; k < RL; ++k) {
      const int t = k * CG + cg;
#pragma unroll
      for (int e = 0; e < N; ++e) { r0[e] += red[t][e]; r1[e] += red[t][N + e]; }
    }
#pragma unroll
    for (int e = 0; e < N; ++e)
      *reinterpret_cast<float2*>(part + ((long long)blockIdx.x * C + N * cg + e) * 2) = make_float2(r0[e], r1[e]);
  }
}

// dbeta[c] = sum dn, dgamma[c] = sum dn*xhat  (fixed order over chunks, one block per channel)
__global__ void __launch_bounds__(256) bn_bwd_finalize_kernel(const float* part, int nchunks, int C, float* dgamma,
                                                              float* dbeta) {
  const int c = blockIdx.x;
  __shared__ double sh[256];
  double a = 0, b = 0;
  for (int k0 = threadIdx.x; k0 < nchunks; k0 += 1024) {  // groups of 4 loads in flight
    float2 pp[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int k = k0 + u * 256;
      pp[u] = k < nchunks ? *reinterpret_cast<const float2*>(part + ((long long)k * C + c) * 2) : make_float2(0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      a += pp[u].x;
      b += pp[u].y;
    }
  }
  const double ta = block_sum256(a, sh);
  const double tb = block_sum256(b, sh);
  if (threadIdx.x == 0) {
    dbeta[c] = (float)ta;
    dgamma[c] = (float)tb;
  }
}

// one wave per channel (4 per block): as bn_bwd_finalize_kernel without block barriers
__global__ void __launch_bounds__(256) bn_bwd_finalize_wave_kernel(const float* part, int nchunks, int C, float* dgamma,
                                                                   float* dbeta) {
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= C) return;
  double a = 0, b = 0;
  for (int k0 = lane; k0 < nchunks; k0 += 256) {
    float2 pp[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int k = k0 + u * 64;
      pp[u] = k < nchunks ? *reinterpret_cast<const float2*>(part + ((long long)k * C + c) * 2) : make_float2(0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      a += pp[u].x;
      b += pp[u].y;
    }
  }
  a = wave_sum(a);
  b = wave_sum(b);
  if (lane == 0) {
    dbeta[c] = (float)a;
    dgamma[c] = (float)b;
  }
}

template <typename T, bool DENSE>
__global__ void __launch_bounds__(256) bn_bwd_apply_kernel(View x, PixDiv pd, long long P, int C, const float* scale,
                                                           const float* shift, const float* mean, const float* rstd,
                                                           const float* gamma, GradIn gi, const float* dgamma,
                                                           const float* dbeta, View dx) {
  constexpr int N = VW<T>::N;
  const int CG = C / N;
  const long long total = P * CG;
  const long long stride = (long long)gridDim.x * blockDim.x;
  const float invP = 1.f / (float)P;
  // per-channel coefficients of this thread's channel group, reloaded only when the group changes
  // (never, when the grid stride is a multiple of CG -- the usual power-of-two channel counts):
  // n = v*sc + sh;  dx = k1*dn - k0 - k2*v   with k1 = gamma*rstd, k2 = k1*rstd*dgamma/P,
  // k0 = k1*(dbeta/P - mean*rstd*dgamma/P)
  int cg_have = -1;
  float sc[N], sh[N], k0[N], k1[N], k2[N];
  auto table = [&](int cg) {
    if (cg == cg_have) return;
    cg_have = cg;
    const int c = N * cg;
    if (scale) { ldc<N>(scale + c, sc); ldc<N>(shift + c, sh); }
    else {
#pragma unroll
      for (int e = 0; e < N; ++e) { sc[e] = 1.f; sh[e] = 0.f; }
    }
    if (mean) {
      float mu[N], rs[N], gm[N], dg[N], db[N];
      ldc<N>(mean + c, mu); ldc<N>(rstd + c, rs); ldc<N>(gamma + c, gm); ldc<N>(dgamma + c, dg); ldc<N>(dbeta + c, db);
#pragma unroll
      for (int e = 0; e < N; ++e) {
        k1[e] = gm[e] * rs[e];
        k2[e] = k1[e] * rs[e] * dg[e] * invP;
        k0[e] = k1[e] * (db[e] * invP - mu[e] * rs[e] * dg[e] * invP);
      }
    } else {
#pragma unroll
      for (int e = 0; e < N; ++e) { k1[e] = 1.f; k2[e] = 0.f; k0[e] = 0.f; }
    }
  };
  struct Off {
    long long x, g1, g2, dx;
    int c;
  };
  auto offs = [&](long long idx) {
    Off o;
    const int cg = (int)(idx % CG);
    const long long pix = idx / CG;
    o.c = N * cg;
    if constexpr (DENSE) {
      o.x = pix * x.ps + x.co + o.c;
      o.g1 = pix * gi.g1.ps + gi.g1.co + o.c;
      o.g2 = pix * gi.g2.ps + gi.g2.co + o.c;
      o.dx = pix * dx.ps + dx.co + o.c;
    } else {
      int b, yy, xx;
      pix_bxy(pd, pix, b, yy, xx);
      o.x = vidx(x, b, yy, xx, o.c);
      o.g1 = vidx(gi.g1, b, yy, xx, o.c);
      o.g2 = vidx(gi.g2, b, yy, xx, o.c);
      o.dx = vidx(dx, b, yy, xx, o.c);
    }
    return o;
  };
  struct In {
    float v[N], g1[N], g2[N];
  };
  auto load = [&](const Off& o, In& in) {
    VW<T>::load(reinterpret_cast<const T*>(x.p) + o.x, in.v);
    if (gi.has1) VW<T>::load(reinterpret_cast<const T*>(gi.g1.p) + o.g1, in.g1);
    if (gi.has2) VW<T>::load(reinterpret_cast<const T*>(gi.g2.p) + o.g2, in.g2);
  };
  auto emit = [&](const Off& o, const In& in) {
    table(o.c / N);
    float d[N];
#pragma unroll
    for (int e = 0; e < N; ++e) {
      const float n = fmaf(in.v[e], sc[e], sh[e]);
      float dn = 0.f;
      if (gi.has1) dn += in.g1[e] * dact(n, gi.s1);
      if (gi.has2) dn += in.g2[e] * dact(n, gi.s2);
      d[e] = fmaf(k1[e], dn, -fmaf(k2[e], in.v[e], k0[e]));
    }
    VW<T>::store(reinterpret_cast<T*>(dx.p) + o.dx, d);
  };
  if constexpr (DENSE) {
    // Streaming form (host: every view pixel-dense with 32-bit element offsets, 256 % CG == 0, so
    // the grid stride is a whole number of pixels): this thread's channel group and its table are
    // fixed, the pixel advances by a constant -- no per-element index division.
    const unsigned nthr = gridDim.x * blockDim.x, t0 = blockIdx.x * blockDim.x + threadIdx.x;
    const unsigned pstep = nthr / (unsigned)CG, Pu = (unsigned)P;
    unsigned pix = t0 / (unsigned)CG;
    if (pix >= Pu) return;
    const int c = N * (int)(t0 % (unsigned)CG);
    table(c / N);
    const T* xp = reinterpret_cast<const T*>(x.p) + x.co + c;
    const T* g1p = reinterpret_cast<const T*>(gi.g1.p) + gi.g1.co + c;
    const T* g2p = reinterpret_cast<const T*>(gi.g2.p) + gi.g2.co + c;
    T* dp = reinterpret_cast<T*>(dx.p) + dx.co + c;
    const unsigned xs = x.ps, g1s = gi.g1.ps, g2s = gi.g2.ps, ds = dx.ps;
    auto ld = [&](unsigned q, In& in) {
      VW<T>::load(xp + q * xs, in.v);
      if (gi.has1) VW<T>::load(g1p + q * g1s, in.g1);
      if (gi.has2) VW<T>::load(g2p + q * g2s, in.g2);
    };
    auto put = [&](unsigned q, const In& in) {
      float d[N];
#pragma unroll
      for (int e = 0; e < N; ++e) {
        const float n = fmaf(in.v[e], sc[e], sh[e]);
        float dn = 0.f;
        if (gi.has1) dn += in.g1[e] * dact(n, gi.s1);
        if (gi.has2) dn += in.g2[e] * dact(n, gi.s2);
        d[e] = fmaf(k1[e], dn, -fmaf(k2[e], in.v[e], k0[e]));
      }
      VW<T>::store(dp + q * ds, d);
    };
    for (; pix + pstep < Pu; pix += 2 * pstep) {  // both pixels' loads in flight before either is used
      In a, b;
      ld(pix, a);
      ld(pix + pstep, b);
      put(pix, a);
      put(pix + pstep, b);
    }
    if (pix < Pu) {
      In a;
      ld(pix, a);
      put(pix, a);
    }
    return;
  }
  long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  for (; idx + stride < total; idx += 2 * stride) {  // both elements' loads in flight before either is used
    const Off oa = offs(idx), ob = offs(idx + stride);
    In a, b;
    load(oa, a);
    load(ob, b);
    emit(oa, a);
    emit(ob, b);
  }
  if (idx < total) {
    const Off oa = offs(idx);
    In a;
    load(oa, a);
    emit(oa, a);
  }
}

// Activation materialisation: n = x*scale + shift (identity without a table), then
// y1 = act(n, slope1) and optionally y2 = act(n, slope2) (slope 0 = ReLU, 0.2 = the
// LeakyReLU of the reference, 1 = identity).  Applied once per element, so the GEMMs
// that consume y1/y2 (each input element is re-read 4-16x by the im2col) stage plain
// operands with no per-load transform.
template <typename T, bool DENSE>
__global__ void __launch_bounds__(256) bn_apply_kernel(View x, PixDiv pd, long long P, int C, const float* scale,
                                                       const float* shift, View y1, float s1, View y2, float s2,
                                                       int has2) {
  constexpr int N = VW<T>::N;
  const int CG = C / N;
  const long long total = P * CG;
  const long long stride = (long long)gridDim.x * blockDim.x;
  int cg_have = -1;
  float sc[N], sh[N];
  auto table = [&](int cg) {  // this thread's channel group's table, reloaded only when it changes
    if (cg == cg_have) return;
    cg_have = cg;
    if (scale) { ldc<N>(scale + N * cg, sc); ldc<N>(shift + N * cg, sh); }
    else {
#pragma unroll
      for (int e = 0; e < N; ++e) { sc[e] = 1.f; sh[e] = 0.f; }
    }
  };
  auto offs = [&](long long idx, long long& ox, long long& o1, long long& o2, int& c) {
    const int cg = (int)(idx % CG);
    const long long pix = idx / CG;
    c = N * cg;
    if constexpr (DENSE) {  // every view dense in pixels: element (pix, c) at pix*ps + co + c
      ox = pix * x.ps + x.co + c;
      o1 = pix * y1.ps + y1.co + c;
      o2 = pix * y2.ps + y2.co + c;
    } else {
      int b, yy, xx;
      pix_bxy(pd, pix, b, yy, xx);
      ox = vidx(x, b, yy, xx, c);
      o1 = vidx(y1, b, yy, xx, c);
      o2 = vidx(y2, b, yy, xx, c);
    }
  };
  auto emit = [&](const float* v0, long long o1, long long o2) {
    float v[N], o[N];
#pragma unroll
    for (int e = 0; e < N; ++e) v[e] = fmaf(v0[e], sc[e], sh[e]);
#pragma unroll
    for (int e = 0; e < N; ++e) o[e] = act(v[e], s1);
    VW<T>::store(reinterpret_cast<T*>(y1.p) + o1, o);
    if (has2) {
#pragma unroll
      for (int e = 0; e < N; ++e) o[e] = act(v[e], s2);
      VW<T>::store(reinterpret_cast<T*>(y2.p) + o2, o);
    }
  };
  if constexpr (DENSE) {  // streaming form: as bn_bwd_apply_kernel's
    const unsigned nthr = gridDim.x * blockDim.x, t0 = blockIdx.x * blockDim.x + threadIdx.x;
    const unsigned pstep = nthr / (unsigned)CG, Pu = (unsigned)P;
    unsigned pix = t0 / (unsigned)CG;
    if (pix >= Pu) return;
    const int c = N * (int)(t0 % (unsigned)CG);
    table(c / N);
    const T* xp = reinterpret_cast<const T*>(x.p) + x.co + c;
    const unsigned xs = x.ps, s1s = y1.ps, s2s = y2.ps;
    const long long b1 = y1.co + c, b2 = y2.co + c;
    for (; pix + pstep < Pu; pix += 2 * pstep) {
      float va[N], vb[N];
      VW<T>::load(xp + pix * xs, va);
      VW<T>::load(xp + (pix + pstep) * xs, vb);
      emit(va, b1 + pix * s1s, b2 + pix * s2s);
      emit(vb, b1 + (pix + pstep) * s1s, b2 + (pix + pstep) * s2s);
    }
    if (pix < Pu) {
      float va[N];
      VW<T>::load(xp + pix * xs, va);
      emit(va, b1 + pix * s1s, b2 + pix * s2s);
    }
    return;
  }
  long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  for (; idx + stride < total; idx += 2 * stride) {  // two 16-byte loads in flight per thread
    long long ax, a1, a2, bx, b1, b2;
    int ca, cb;
    offs(idx, ax, a1, a2, ca);
    offs(idx + stride, bx, b1, b2, cb);
    float va[N], vb[N];
    VW<T>::load(reinterpret_cast<const T*>(x.p) + ax, va);
    VW<T>::load(reinterpret_cast<const T*>(x.p) + bx, vb);
    table(ca / N);
    emit(va, a1, a2);
    table(cb / N);
    emit(vb, b1, b2);
  }
  if (idx < total) {
    long long ax, a1, a2;
    int ca;
    offs(idx, ax, a1, a2, ca);
    float va[N];
    VW<T>::load(reinterpret_cast<const T*>(x.p) + ax, va);
    table(ca / N);
    emit(va, a1, a2);
  }
}

// part[chunk][c] = sum over the chunk's pixels of x (conv bias gradients)
template <typename T>
__global__ void __launch_bounds__(256) chan_sum_kernel(View x, PixDiv pd, long long P, int C, float* part, int nchunks) {
  constexpr int N = VW<T>::N;
  const int CG = C / N;
  const int RL = 256 / CG;
  const int cg = threadIdx.x % CG, pl = threadIdx.x / CG;
  const long long per = (P + nchunks - 1) / nchunks;
  const long long p0 = blockIdx.x * per, p1 = min(P, p0 + per);
  __shared__ float red[256][N];
  float a[N];
#pragma unroll
  for (int e = 0; e < N; ++e) a[e] = 0.f;
  if (pl < RL) {
    for (long long pix = p0 + pl; pix < p1; pix += RL) {
      int b, yy, xx;
      pix_bxy(pd, pix, b, yy, xx);
      float v[N];
      VW<T>::load(vptr<T>(x, b, yy, xx, N * cg), v);
#pragma unroll
      for (int e = 0; e < N; ++e) a[e] += v[e];
    }
  }
#pragma unroll
  for (int e = 0; e < N; ++e) red[threadIdx.x][e] = a[e];
  __syncthreads();
  if (pl == 0) {
    float r[N];
#pragma unroll
    for (int e = 0; e < N; ++e) r[e] = 0.f;
    for (int k = 0; k < RL; ++k)
#pragma unroll
      for (int e = 0; e < N; ++e) r[e] += red[k * CG + cg][e];
#pragma unroll
    for (int e = 0; e < N; ++e) part[(long long)blockIdx.x * C + N * cg + e] = r[e];
  }
}

__global__ void chan_sum_final_kernel(const float* part, int nchunks, int C, int Cout, float* out) {
  const int c = blockIdx.x;
  __shared__ double s[256];
  double a = 0;
  for (int k = threadIdx.x; k < nchunks; k += 256) a += part[(long long)k * C + c];
  s[threadIdx.x] = a;
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if (threadIdx.x < st) s[threadIdx.x] += s[threadIdx.x + st];
    __syncthreads();
  }
  if (threadIdx.x == 0 && c < Cout) out[c] = (float)s[0];
}

static GradIn mkgrad(stc_view g1, float s1, stc_view g2, float s2) {
  GradIn gi{};
  gi.has1 = g1.p != nullptr; gi.has2 = g2.p != nullptr;
  if (gi.has1) gi.g1 = mkview(g1);
  if (gi.has2) gi.g2 = mkview(g2);
  gi.s1 = s1; gi.s2 = s2;
  return gi;
}

static int grid_for(long long work) { return (int)std::max<long long>(1, std::min<long long>((work + 255) / 256, 8192)); }

}  // namespace stc

using namespace stc;

extern "C" int stc_chan_stats_chunks(int B, int H, int W) { return stat_chunks((long long)B * H * W); }

// pixel-dense view: rows and images follow each other without gaps, so pixel p sits at p * ps
static bool pix_dense(const stc_view& v) { return v.rs == (int64_t)v.W * v.ps && v.bs == (int64_t)v.H * v.rs; }

// the streaming (DENSE) element-wise form: pixel-dense views whose element offsets fit 32 bits, and a
// channel-group count dividing 256 (the grid stride is then a whole number of pixels)
static bool stream_ok(int B, const stc_view& v, int C, int N) {
  if (!v.p) return true;
  const long long extent = (long long)B * v.H * v.W * v.ps + v.co + C;
  return pix_dense(v) && extent < (1ll << 31) && 256 % (C / N) == 0;
}
static int grid_stream(long long work) {  // >= 4 pixel-vectors per thread, at most 8 blocks per CU
  return (int)std::max<long long>(1, std::min<long long>((work + 1023) / 1024, 2048));
}

static bool vec_ok(int dtype, int C, const stc_view& v) {
  const int N = dtype == STC_F32 ? 4 : 8;
  return C % N == 0 && C / N <= 256 && v.cs == 1 && v.co % N == 0 && v.ps % N == 0 && v.rs % N == 0 && v.bs % N == 0;
}

extern "C" int stc_chan_stats(int dtype, int B, stc_view x, int C, float* part, int nchunks, void* stream) {
  STC_REQUIRE(vec_ok(dtype, C, x), "stc_chan_stats: C=%d / view not 16-byte vectorisable (NHWC, <= 256 vectors)", C);
  hipStream_t st = (hipStream_t)stream;
  View v = mkview(x);
  const PixDiv pd = mkpix(B, x.H, x.W);
  const long long P = (long long)B * x.H * x.W;
  if (dtype == STC_F32) hipLaunchKernelGGL(chan_stats_kernel<float>, dim3(nchunks), dim3(256), 0, st, v, pd, P, C, part, nchunks);
  else hipLaunchKernelGGL(chan_stats_kernel<bf16>, dim3(nchunks), dim3(256), 0, st, v, pd, P, C, part, nchunks);
  STC_CHECK_LAUNCH();
  return 0;
}

extern "C" int stc_bn_apply(int dtype, int B, stc_view x, int C, const float* scale, const float* shift, stc_view y1,
                            float slope1, stc_view y2, float slope2, void* stream) {
  STC_REQUIRE((scale == nullptr) == (shift == nullptr), "stc_bn_apply: scale/shift must come together");
  STC_REQUIRE(y1.p && vec_ok(dtype, C, x) && vec_ok(dtype, C, y1) && (!y2.p || vec_ok(dtype, C, y2)),
              "stc_bn_apply: C=%d / views not 16-byte vectorisable NHWC", C);
  hipStream_t st = (hipStream_t)stream;
  View v = mkview(x), o1 = mkview(y1), o2 = y2.p ? mkview(y2) : mkview(y1);
  const PixDiv pd = mkpix(B, x.H, x.W);
  const long long P = (long long)B * x.H * x.W;
  const int N = dtype == STC_F32 ? 4 : 8;
  const bool dense = stream_ok(B, x, C, N) && stream_ok(B, y1, C, N) && stream_ok(B, y2, C, N);
  const int blocks = dense ? grid_stream(P * (C / N)) : grid_for(P * (C / N));
  const int h2 = y2.p != nullptr ? 1 : 0;
#define STC_BA(T_, D_) hipLaunchKernelGGL((bn_apply_kernel<T_, D_>), dim3(blocks), dim3(256), 0, st, v, pd, P, C, scale, shift, o1, slope1, o2, slope2, h2)
  if (dtype == STC_F32) { if (dense) STC_BA(float, true); else STC_BA(float, false); }
  else { if (dense) STC_BA(bf16, true); else STC_BA(bf16, false); }
#undef STC_BA
  STC_CHECK_LAUNCH();
  return 0;
}

extern "C" int stc_chan_sum(int dtype, int B, stc_view x, int C, int Cout, float* part, int nchunks, float* out,
                            void* stream) {
  STC_REQUIRE(vec_ok(dtype, C, x) && Cout <= C, "stc_chan_sum: bad C=%d / view", C);
  hipStream_t st = (hipStream_t)stream;
  View v = mkview(x);
  const PixDiv pd = mkpix(B, x.H, x.W);
  const long long P = (long long)B * x.H * x.W;
  if (dtype == STC_F32) hipLaunchKernelGGL(chan_sum_kernel<float>, dim3(nchunks), dim3(256), 0, st, v, pd, P, C, part, nchunks);
  else hipLaunchKernelGGL(chan_sum_kernel<bf16>, dim3(nchunks), dim3(256), 0, st, v, pd, P, C, part, nchunks);
  STC_CHECK_LAUNCH();
  hipLaunchKernelGGL(chan_sum_final_kernel, dim3(C), dim3(256), 0, st, (const float*)part, nchunks, C, Cout, out);
  STC_CHECK_LAUNCH();
  return 0;
}

extern "C" int stc_bn_finalize(const float* part, int nchunks, int C, const float* gamma, const float* beta,
                               float* running_mean, float* running_var, int64_t* num_batches_tracked,
                               float momentum, float eps, float* mean, float* rstd, float* scale, float* shift,
                               void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (part == nullptr) {
    STC_REQUIRE(gamma && beta && running_mean && running_var, "stc_bn_finalize(eval): missing tensors");
    hipLaunchKernelGGL(bn_eval_table_kernel, dim3((C + 255) / 256), dim3(256), 0, st, C, gamma, beta, running_mean,
                       running_var, eps, scale, shift);
  } else {
    if (nchunks <= 1024)  // up to 4 load groups per lane in registers; more chunks: a block per channel
      hipLaunchKernelGGL(bn_finalize_wave_kernel, dim3((C + 3) / 4), dim3(256), 0, st, part, nchunks, C, gamma, beta,
                         running_mean, running_var, (long long*)num_batches_tracked, momentum, eps, mean, rstd, scale,
                         shift);
    else
      hipLaunchKernelGGL(bn_finalize_kernel, dim3(C), dim3(256), 0, st, part, nchunks, C, gamma, beta, running_mean,
                         running_var, (long long*)num_batches_tracked, momentum, eps, mean, rstd, scale, shift);
  }
  STC_CHECK_LAUNCH();
  return 0;
}

extern "C" int stc_bn_bwd_reduce(int dtype, int B, stc_view x, int C, const float* scale, const float* shift,
                                 const float* mean, const float* rstd, stc_view g1, float slope1, stc_view g2,
                                 float slope2, float* part2, int nchunks, void* stream) {
  STC_REQUIRE(vec_ok(dtype, C, x) && (!g1.p || vec_ok(dtype, C, g1)) && (!g2.p || vec_ok(dtype, C, g2)),
              "stc_bn_bwd_reduce: bad C=%d / views", C);
  STC_REQUIRE(scale && shift && mean && rstd, "stc_bn_bwd_reduce: BN tables required");
  hipStream_t st = (hipStream_t)stream;
  GradIn gi = mkgrad(g1, slope1, g2, slope2);
  View v = mkview(x);
  const PixDiv pd = mkpix(B, x.H, x.W);
  const long long P = (long long)B * x.H * x.W;
  if (dtype == STC_F32)
    hipLaunchKernelGGL(bn_bwd_reduce_kernel<float>, dim3(nchunks), dim3(256), 0, st, v, pd, P, C, scale, shift, mean, rstd, gi, part2, nchunks);
  else
    hipLaunchKernelGGL(bn_bwd_reduce_kernel<bf16>, dim3(nchunks), dim3(256), 0, st, v, pd, P, C, scale, shift, mean, rstd, gi, part2, nchunks);
  STC_CHECK_LAUNCH();
  return 0;
}

extern "C" int stc_bn_bwd_apply(int dtype, int B, stc_view x, int C, const float* scale, const float* shift,
                                const float* mean, const float* rstd, const float* gamma, stc_view g1, float slope1,
                                stc_view g2, float slope2, const float* part2, int nchunks, stc_view dx,
                                float* dgamma, float* dbeta, void* stream) {
  STC_REQUIRE(vec_ok(dtype, C, x) && vec_ok(dtype, C, dx) && (!g1.p || vec_ok(dtype, C, g1)) &&
                  (!g2.p || vec_ok(dtype, C, g2)),
              "stc_bn_bwd_apply: bad C=%d / views", C);
  hipStream_t st = (hipStream_t)stream;
  GradIn gi = mkgrad(g1, slope1, g2, slope2);
  if (mean) {
    STC_REQUIRE(part2 && dgamma && dbeta && gamma && rstd && scale && shift, "stc_bn_bwd_apply: missing BN tensors");
    if (nchunks <= 256)
      hipLaunchKernelGGL(bn_bwd_finalize_wave_kernel, dim3((C + 3) / 4), dim3(256), 0, st, part2, nchunks, C, dgamma, dbeta);
    else
      hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(C), dim3(256), 0, st, part2, nchunks, C, dgamma, dbeta);
    STC_CHECK_LAUNCH();
  }
  View v = mkview(x), o = mkview(dx);
  const PixDiv pd = mkpix(B, x.H, x.W);
  const long long P = (long long)B * x.H * x.W;
  const int N = dtype == STC_F32 ? 4 : 8;
  const long long work = P * (C / N);
  const bool dense = stream_ok(B, x, C, N) && stream_ok(B, dx, C, N) && stream_ok(B, g1, C, N) && stream_ok(B, g2, C, N);
  const int blocks = dense ? grid_stream(work) : grid_for(work);
#define STC_BB(T_, D_) hipLaunchKernelGGL((bn_bwd_apply_kernel<T_, D_>), dim3(blocks), dim3(256), 0, st, v, pd, P, C, scale, shift, mean, rstd, gamma, gi, dgamma, dbeta, o)
  if (dtype == STC_F32) { if (dense) STC_BB(float, true); else STC_BB(float, false); }
  else { if (dense) STC_BB(bf16, true); else STC_BB(bf16, false); }
#undef STC_BB
  STC_CHECK_LAUNCH();
  return 0;
}
