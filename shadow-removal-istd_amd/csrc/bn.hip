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
#include "common.hpp"

namespace stc {

constexpr int STAT_PIX = 64;  // pixels per statistics chunk (upper bound of chunk count below)

__host__ __device__ inline int stat_chunks(long long P) {
  long long c = (P + STAT_PIX - 1) / STAT_PIX;
  if (c > 1024) c = 1024;
  if (c < 1) c = 1;
  return (int)c;
}

template <typename T>
__device__ __forceinline__ float4 vload(const View& v, int b, int y, int x, int c) {
  return Vec4<T>::load(reinterpret_cast<const T*>(v.p) + vidx(v, b, y, x, c));
}

// part[chunk][c] = {n, S1, S2, shift}
template <typename T>
__global__ void __launch_bounds__(256) chan_stats_kernel(View x, int B, int C, float* part, int nchunks) {
  const int cq = C >> 2;
  const int ppb = 256 / cq;  // pixels processed in parallel
  const int q = threadIdx.x % cq, pl = threadIdx.x / cq;
  const long long HW = (long long)x.H * x.W, P = HW * B;
  const long long per = (P + nchunks - 1) / nchunks;
  const long long p0 = blockIdx.x * per, p1 = min(P, p0 + per);
  __shared__ float red[3][256][4];
  float4 s1 = make_float4(0, 0, 0, 0), s2 = make_float4(0, 0, 0, 0), sh = make_float4(0, 0, 0, 0);
  float cnt = 0.f;
  if (pl < ppb && p0 < p1) {
    {
      const int b = (int)(p0 / HW), rem = (int)(p0 % HW);
      sh = vload<T>(x, b, rem / x.W, rem % x.W, 4 * q);
    }
    for (long long pix = p0 + pl; pix < p1; pix += ppb) {
      const int b = (int)(pix / HW), rem = (int)(pix % HW);
      float4 v = vload<T>(x, b, rem / x.W, rem % x.W, 4 * q);
      v.x -= sh.x; v.y -= sh.y; v.z -= sh.z; v.w -= sh.w;
      s1.x += v.x; s1.y += v.y; s1.z += v.z; s1.w += v.w;
      s2.x += v.x * v.x; s2.y += v.y * v.y; s2.z += v.z * v.z; s2.w += v.w * v.w;
      cnt += 1.f;
    }
  }
  red[0][threadIdx.x][0] = s1.x; red[0][threadIdx.x][1] = s1.y; red[0][threadIdx.x][2] = s1.z; red[0][threadIdx.x][3] = s1.w;
  red[1][threadIdx.x][0] = s2.x; red[1][threadIdx.x][1] = s2.y; red[1][threadIdx.x][2] = s2.z; red[1][threadIdx.x][3] = s2.w;
  red[2][threadIdx.x][0] = cnt;
  __syncthreads();
  if (pl == 0 && threadIdx.x < cq) {
    float a1[4] = {0, 0, 0, 0}, a2[4] = {0, 0, 0, 0}, n = 0.f;
    for (int k = 0; k < ppb; ++k) {  // fixed order
      const int t = k * cq + q;
      for (int e = 0; e < 4; ++e) { a1[e] += red[0][t][e]; a2[e] += red[1][t][e]; }
      n += red[2][t][0];
    }
    const float shv[4] = {sh.x, sh.y, sh.z, sh.w};
    for (int e = 0; e < 4; ++e) {
      float* o = part + ((long long)blockIdx.x * C + 4 * q + e) * 4;
      o[0] = n; o[1] = a1[e]; o[2] = a2[e]; o[3] = shv[e];
    }
  }
}

__global__ void __launch_bounds__(256) bn_finalize_kernel(const float* part, int nchunks, int C,
                                                          const float* gamma, const float* beta,
                                                          float* rmean, float* rvar, long long* nbt,
                                                          float momentum, float eps,
                                                          float* mean_o, float* rstd_o, float* scale, float* shift) {
  const int c = blockIdx.x;
  __shared__ double sn[256], sm[256], sq[256];
  double n = 0, mean = 0, m2 = 0;
  for (int k = threadIdx.x; k < nchunks; k += 256) {
    const float* pp = part + ((long long)k * C + c) * 4;
    const double nb = pp[0];
    if (nb <= 0) continue;
    const double s1 = pp[1], s2 = pp[2], shv = pp[3];
    const double mb = shv + s1 / nb;
    double qb = s2 - s1 * s1 / nb;
    if (qb < 0) qb = 0;
    const double nn = n + nb, d = mb - mean;
    mean += d * nb / nn;
    m2 += qb + d * d * n * nb / nn;
    n = nn;
  }
  sn[threadIdx.x] = n; sm[threadIdx.x] = mean; sq[threadIdx.x] = m2;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      const double na = sn[threadIdx.x], nb = sn[threadIdx.x + s];
      if (nb > 0) {
        const double nn = na + nb, d = sm[threadIdx.x + s] - sm[threadIdx.x];
        sm[threadIdx.x] += d * nb / nn;
        sq[threadIdx.x] += sq[threadIdx.x + s] + d * d * na * nb / nn;
        sn[threadIdx.x] = nn;
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const double N = sn[0], mu = sm[0];
    const double var = N > 0 ? sq[0] / N : 0.0;
    const float rs = (float)(1.0 / sqrt(var + (double)eps));
    const float g = gamma ? gamma[c] : 1.f, bt = beta ? beta[c] : 0.f;
    if (mean_o) mean_o[c] = (float)mu;
    if (rstd_o) rstd_o[c] = rs;
    const float sc = g * rs;
    scale[c] = sc;
    shift[c] = bt - (float)mu * sc;
    if (rmean) rmean[c] = (1.f - momentum) * rmean[c] + momentum * (float)mu;
    if (rvar) rvar[c] = (1.f - momentum) * rvar[c] + momentum * (float)(N > 1 ? sq[0] / (N - 1) : var);
    if (nbt && c == 0) nbt[0] += 1;
  }
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
__device__ __forceinline__ float4 dn_of(const GradIn& gi, int b, int y, int x, int c, float4 n) {
  float4 d = make_float4(0, 0, 0, 0);
  if (gi.has1) {
    const float4 g = vload<T>(gi.g1, b, y, x, c);
    d.x += g.x * dact(n.x, gi.s1); d.y += g.y * dact(n.y, gi.s1);
    d.z += g.z * dact(n.z, gi.s1); d.w += g.w * dact(n.w, gi.s1);
  }
  if (gi.has2) {
    const float4 g = vload<T>(gi.g2, b, y, x, c);
    d.x += g.x * dact(n.x, gi.s2); d.y += g.y * dact(n.y, gi.s2);
    d.z += g.z * dact(n.z, gi.s2); d.w += g.w * dact(n.w, gi.s2);
  }
  return d;
}

// part2[chunk][c] = {sum dn, sum dn*xhat}
template <typename T>
__global__ void __launch_bounds__(256) bn_bwd_reduce_kernel(View x, int B, int C, const float* scale, const float* shift,
                                                            const float* mean, const float* rstd, GradIn gi,
                                                            float* part, int nchunks) {
  const int cq = C >> 2;
  const int ppb = 256 / cq;
  const int q = threadIdx.x % cq, pl = threadIdx.x / cq;
  const long long HW = (long long)x.H * x.W, P = HW * B;
  const long long per = (P + nchunks - 1) / nchunks;
  const long long p0 = blockIdx.x * per, p1 = min(P, p0 + per);
  __shared__ float red[2][256][4];
  float a[4] = {0, 0, 0, 0}, bsum[4] = {0, 0, 0, 0};
  if (pl < ppb) {
    const int c = 4 * q;
    const float4 sc = *reinterpret_cast<const float4*>(scale + c);
    const float4 shf = *reinterpret_cast<const float4*>(shift + c);
    const float4 mu = *reinterpret_cast<const float4*>(mean + c);
    const float4 rs = *reinterpret_cast<const float4*>(rstd + c);
    for (long long pix = p0 + pl; pix < p1; pix += ppb) {
      const int b = (int)(pix / HW), rem = (int)(pix % HW);
      const int y = rem / x.W, xx = rem % x.W;
      const float4 v = vload<T>(x, b, y, xx, c);
      const float4 n = make_float4(fmaf(v.x, sc.x, shf.x), fmaf(v.y, sc.y, shf.y), fmaf(v.z, sc.z, shf.z),
                                   fmaf(v.w, sc.w, shf.w));
      const float4 d = dn_of<T>(gi, b, y, xx, c, n);
      a[0] += d.x; a[1] += d.y; a[2] += d.z; a[3] += d.w;
      bsum[0] += d.x * (v.x - mu.x) * rs.x; bsum[1] += d.y * (v.y - mu.y) * rs.y;
      bsum[2] += d.z * (v.z - mu.z) * rs.z; bsum[3] += d.w * (v.w - mu.w) * rs.w;
    }
  }
  for (int e = 0; e < 4; ++e) { red[0][threadIdx.x][e] = a[e]; red[1][threadIdx.x][e] = bsum[e]; }
  __syncthreads();
  if (pl == 0 && threadIdx.x < cq) {
    float r0[4] = {0, 0, 0, 0}, r1[4] = {0, 0, 0, 0};
    for (int k = 0; k < ppb; ++k) {
      const int t = k * cq + q;
      for (int e = 0; e < 4; ++e) { r0[e] += red[0][t][e]; r1[e] += red[1][t][e]; }
    }
    for (int e = 0; e < 4; ++e) {
      float* o = part + ((long long)blockIdx.x * C + 4 * q + e) * 2;
      o[0] = r0[e]; o[1] = r1[e];
    }
  }
}

// dbeta[c] = sum dn, dgamma[c] = sum dn*xhat  (fixed order over chunks)
__global__ void bn_bwd_finalize_kernel(const float* part, int nchunks, int C, float* dgamma, float* dbeta) {
  const int c = blockIdx.x;
  __shared__ double s0[256], s1[256];
  double a = 0, b = 0;
  for (int k = threadIdx.x; k < nchunks; k += 256) {
    a += part[((long long)k * C + c) * 2];
    b += part[((long long)k * C + c) * 2 + 1];
  }
  s0[threadIdx.x] = a; s1[threadIdx.x] = b;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) { s0[threadIdx.x] += s0[threadIdx.x + s]; s1[threadIdx.x] += s1[threadIdx.x + s]; }
    __syncthreads();
  }
  if (threadIdx.x == 0) { dbeta[c] = (float)s0[0]; dgamma[c] = (float)s1[0]; }
}

template <typename T>
__global__ void __launch_bounds__(256) bn_bwd_apply_kernel(View x, int B, int C, const float* scale, const float* shift,
                                                           const float* mean, const float* rstd, const float* gamma,
                                                           GradIn gi, const float* dgamma, const float* dbeta,
                                                           View dx) {
  const int cq = C >> 2;
  const long long HW = (long long)x.H * x.W, P = HW * B;
  const long long total = P * cq;
  const float invP = 1.f / (float)P;
  for (long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (long long)gridDim.x * blockDim.x) {
    const int q = (int)(idx % cq);
    const long long pix = idx / cq;
    const int b = (int)(pix / HW), rem = (int)(pix % HW);
    const int y = rem / x.W, xx = rem % x.W;
    const int c = 4 * q;
    const float4 v = vload<T>(x, b, y, xx, c);
    float4 n;
    if (scale) {
      const float4 sc = *reinterpret_cast<const float4*>(scale + c);
      const float4 shf = *reinterpret_cast<const float4*>(shift + c);
      n = make_float4(fmaf(v.x, sc.x, shf.x), fmaf(v.y, sc.y, shf.y), fmaf(v.z, sc.z, shf.z), fmaf(v.w, sc.w, shf.w));
    } else {
      n = v;
    }
    float4 d = dn_of<T>(gi, b, y, xx, c, n);
    if (mean) {
      const float vv[4] = {v.x, v.y, v.z, v.w};
      float dd[4] = {d.x, d.y, d.z, d.w};
      for (int e = 0; e < 4; ++e) {
        const int ch = c + e;
        const float rs = rstd[ch];
        const float xh = (vv[e] - mean[ch]) * rs;
        dd[e] = gamma[ch] * rs * (dd[e] - dbeta[ch] * invP - xh * dgamma[ch] * invP);
      }
      d = make_float4(dd[0], dd[1], dd[2], dd[3]);
    }
    Vec4<T>::store(reinterpret_cast<T*>(dx.p) + vidx(dx, b, y, xx, c), d);
  }
}

// Activation materialisation: n = x*scale + shift (identity without a table), then
// y1 = act(n, slope1) and optionally y2 = act(n, slope2) (slope 0 = ReLU, 0.2 = the
// LeakyReLU of the reference, 1 = identity).  Applied once per element, so the GEMMs
// that consume y1/y2 (each input element is re-read 4-16x by the im2col) stage plain
// operands with no per-load transform.
template <typename T>
__global__ void __launch_bounds__(256) bn_apply_kernel(View x, int B, int C, const float* scale, const float* shift,
                                                       View y1, float s1, View y2, float s2, int has2) {
  const int cq = C >> 2;
  const long long HW = (long long)x.H * x.W, total = HW * B * cq;
  for (long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (long long)gridDim.x * blockDim.x) {
    const int q = (int)(idx % cq);
    const long long pix = idx / cq;
    const int b = (int)(pix / HW), rem = (int)(pix % HW);
    const int yy = rem / x.W, xx = rem % x.W;
    const int c = 4 * q;
    float4 v = vload<T>(x, b, yy, xx, c);
    if (scale) {
      const float4 sc = *reinterpret_cast<const float4*>(scale + c);
      const float4 sh = *reinterpret_cast<const float4*>(shift + c);
      v = make_float4(fmaf(v.x, sc.x, sh.x), fmaf(v.y, sc.y, sh.y), fmaf(v.z, sc.z, sh.z), fmaf(v.w, sc.w, sh.w));
    }
    Vec4<T>::store(reinterpret_cast<T*>(y1.p) + vidx(y1, b, yy, xx, c),
                   make_float4(act(v.x, s1), act(v.y, s1), act(v.z, s1), act(v.w, s1)));
    if (has2)
      Vec4<T>::store(reinterpret_cast<T*>(y2.p) + vidx(y2, b, yy, xx, c),
                     make_float4(act(v.x, s2), act(v.y, s2), act(v.z, s2), act(v.w, s2)));
  }
}

// part[chunk][c] = sum over the chunk's pixels of x (conv bias gradients)
template <typename T>
__global__ void __launch_bounds__(256) chan_sum_kernel(View x, int B, int C, float* part, int nchunks) {
  const int cq = C >> 2;
  const int ppb = 256 / cq;
  const int q = threadIdx.x % cq, pl = threadIdx.x / cq;
  const long long HW = (long long)x.H * x.W, P = HW * B;
  const long long per = (P + nchunks - 1) / nchunks;
  const long long p0 = blockIdx.x * per, p1 = min(P, p0 + per);
  __shared__ float red[256][4];
  float a[4] = {0, 0, 0, 0};
  if (pl < ppb) {
    for (long long pix = p0 + pl; pix < p1; pix += ppb) {
      const int b = (int)(pix / HW), rem = (int)(pix % HW);
      const float4 v = vload<T>(x, b, rem / x.W, rem % x.W, 4 * q);
      a[0] += v.x; a[1] += v.y; a[2] += v.z; a[3] += v.w;
    }
  }
  for (int e = 0; e < 4; ++e) red[threadIdx.x][e] = a[e];
  __syncthreads();
  if (threadIdx.x < cq) {
    float r[4] = {0, 0, 0, 0};
    for (int k = 0; k < ppb; ++k)
      for (int e = 0; e < 4; ++e) r[e] += red[k * cq + q][e];
    for (int e = 0; e < 4; ++e) part[(long long)blockIdx.x * C + 4 * q + e] = r[e];
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

extern "C" int stc_chan_stats(int dtype, int B, stc_view x, int C, float* part, int nchunks, void* stream) {
  STC_REQUIRE(C % 4 == 0 && C <= 1024, "stc_chan_stats: C=%d must be a multiple of 4 and <= 1024", C);
  STC_REQUIRE(x.cs == 1 && x.co % 4 == 0 && x.ps % 4 == 0, "stc_chan_stats: NHWC view, 4-aligned");
  hipStream_t st = (hipStream_t)stream;
  View v = mkview(x);
  if (dtype == STC_F32) hipLaunchKernelGGL(chan_stats_kernel<float>, dim3(nchunks), dim3(256), 0, st, v, B, C, part, nchunks);
  else hipLaunchKernelGGL(chan_stats_kernel<bf16>, dim3(nchunks), dim3(256), 0, st, v, B, C, part, nchunks);
  STC_CHECK_LAUNCH();
  return 0;
}

extern "C" int stc_bn_apply(int dtype, int B, stc_view x, int C, const float* scale, const float* shift, stc_view y1,
                            float slope1, stc_view y2, float slope2, void* stream) {
  STC_REQUIRE(C % 4 == 0, "stc_bn_apply: C=%d must be a multiple of 4", C);
  STC_REQUIRE((scale == nullptr) == (shift == nullptr), "stc_bn_apply: scale/shift must come together");
  STC_REQUIRE(x.cs == 1 && y1.cs == 1 && y1.p, "stc_bn_apply: NHWC views required");
  hipStream_t st = (hipStream_t)stream;
  View v = mkview(x), o1 = mkview(y1), o2 = y2.p ? mkview(y2) : mkview(y1);
  const long long work = (long long)B * x.H * x.W * (C / 4);
  const int blocks = grid_for(work);
  if (dtype == STC_F32)
    hipLaunchKernelGGL(bn_apply_kernel<float>, dim3(blocks), dim3(256), 0, st, v, B, C, scale, shift, o1, slope1, o2, slope2, y2.p != nullptr ? 1 : 0);
  else
    hipLaunchKernelGGL(bn_apply_kernel<bf16>, dim3(blocks), dim3(256), 0, st, v, B, C, scale, shift, o1, slope1, o2, slope2, y2.p != nullptr ? 1 : 0);
  STC_CHECK_LAUNCH();
  return 0;
}

extern "C" int stc_chan_sum(int dtype, int B, stc_view x, int C, int Cout, float* part, int nchunks, float* out,
                            void* stream) {
  STC_REQUIRE(C % 4 == 0 && C <= 1024 && Cout <= C, "stc_chan_sum: bad C=%d", C);
  hipStream_t st = (hipStream_t)stream;
  View v = mkview(x);
  if (dtype == STC_F32) hipLaunchKernelGGL(chan_sum_kernel<float>, dim3(nchunks), dim3(256), 0, st, v, B, C, part, nchunks);
  else hipLaunchKernelGGL(chan_sum_kernel<bf16>, dim3(nchunks), dim3(256), 0, st, v, B, C, part, nchunks);
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
    hipLaunchKernelGGL(bn_finalize_kernel, dim3(C), dim3(256), 0, st, part, nchunks, C, gamma, beta, running_mean,
                       running_var, (long long*)num_batches_tracked, momentum, eps, mean, rstd, scale, shift);
  }
  STC_CHECK_LAUNCH();
  return 0;
}

extern "C" int stc_bn_bwd_reduce(int dtype, int B, stc_view x, int C, const float* scale, const float* shift,
                                 const float* mean, const float* rstd, stc_view g1, float slope1, stc_view g2,
                                 float slope2, float* part2, int nchunks, void* stream) {
  STC_REQUIRE(C % 4 == 0 && C <= 1024, "stc_bn_bwd_reduce: bad C=%d", C);
  STC_REQUIRE(scale && shift && mean && rstd, "stc_bn_bwd_reduce: BN tables required");
  hipStream_t st = (hipStream_t)stream;
  GradIn gi = mkgrad(g1, slope1, g2, slope2);
  View v = mkview(x);
  if (dtype == STC_F32)
    hipLaunchKernelGGL(bn_bwd_reduce_kernel<float>, dim3(nchunks), dim3(256), 0, st, v, B, C, scale, shift, mean, rstd, gi, part2, nchunks);
  else
    hipLaunchKernelGGL(bn_bwd_reduce_kernel<bf16>, dim3(nchunks), dim3(256), 0, st, v, B, C, scale, shift, mean, rstd, gi, part2, nchunks);
  STC_CHECK_LAUNCH();
  return 0;
}

extern "C" int stc_bn_bwd_apply(int dtype, int B, stc_view x, int C, const float* scale, const float* shift,
                                const float* mean, const float* rstd, const float* gamma, stc_view g1, float slope1,
                                stc_view g2, float slope2, const float* part2, int nchunks, stc_view dx,
                                float* dgamma, float* dbeta, void* stream) {
  STC_REQUIRE(C % 4 == 0, "stc_bn_bwd_apply: bad C=%d", C);
  hipStream_t st = (hipStream_t)stream;
  GradIn gi = mkgrad(g1, slope1, g2, slope2);
  if (mean) {
    STC_REQUIRE(part2 && dgamma && dbeta && gamma && rstd && scale && shift, "stc_bn_bwd_apply: missing BN tensors");
    hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(C), dim3(256), 0, st, part2, nchunks, C, dgamma, dbeta);
    STC_CHECK_LAUNCH();
  }
  View v = mkview(x), o = mkview(dx);
  const long long work = (long long)B * x.H * x.W * (C / 4);
  if (dtype == STC_F32)
    hipLaunchKernelGGL(bn_bwd_apply_kernel<float>, dim3(grid_for(work)), dim3(256), 0, st, v, B, C, scale, shift, mean, rstd, gamma, gi, dgamma, dbeta, o);
  else
    hipLaunchKernelGGL(bn_bwd_apply_kernel<bf16>, dim3(grid_for(work)), dim3(256), 0, st, v, B, C, scale, shift, mean, rstd, gamma, gi, dgamma, dbeta, o);
  STC_CHECK_LAUNCH();
  return 0;
}
