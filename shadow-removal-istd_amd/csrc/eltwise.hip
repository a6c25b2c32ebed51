// Layout edges, Tanh/bias backward, losses and the weight packer.
//   gather/scatter : torch.cat((x, m, ...), 1) of the D/G inputs (STCGAN/stcgan.py:219-227,
//                    269-272) fused with the NCHW->NHWC edge conversion (and its backward)
//   tanh_bias_bwd  : outermost Tanh + ConvT bias (STCGAN/networks.py:112-116) backward
//   losses         : DataLoss = F.l1_loss (STCGAN/loss.py:14-26); AdversarialLoss =
//                    F.mse_loss vs 1/0 or BCE-with-logits vs 1/-1 (STCGAN/loss.py:59-86)
//   pack_weight    : torch weight [P][Q][4][4] -> GEMM operand [phase][N][tap][C]
#include "common.hpp"

namespace stc {

// ------------------------------------------------------------------ gather / scatter
struct Src4 {
  const float* p[4];
  int c[4];
};
struct Dst4 {
  float* p[4];
  int c[4];
};

template <typename T>
__global__ void gather_kernel(int B, int H, int W, int nsrc, Src4 s, View d, int Cpad) {
  const long long HW = (long long)H * W, P = HW * B;
  for (long long pix = (long long)blockIdx.x * blockDim.x + threadIdx.x; pix < P;
       pix += (long long)gridDim.x * blockDim.x) {
    const int b = (int)(pix / HW);
    const long long hw = pix % HW;
    const int y = (int)(hw / W), x = (int)(hw % W);
    T* out = reinterpret_cast<T*>(d.p) + vidx(d, b, y, x, 0);
    int c = 0;
    for (int k = 0; k < nsrc; ++k) {
      const float* src = s.p[k] + (long long)b * s.c[k] * HW + hw;
      for (int j = 0; j < s.c[k]; ++j, ++c) st1<T>(out + (long long)c * d.cs, src[(long long)j * HW]);
    }
    for (; c < Cpad; ++c) st1<T>(out + (long long)c * d.cs, 0.f);
  }
}

// Vectorised form for NHWC destinations (cs == 1, Cpad <= 16): one pixel per thread, the
// channel -> (source, plane) map in kernel arguments, 16-byte stores.
template <typename T>
__global__ void gather_vec_kernel(int B, int H, int W, int nsrc, Src4 s, View d, int Cpad) {
  constexpr int N = 16 / sizeof(T);
  const long long HW = (long long)H * W, P = HW * B;
  for (long long pix = (long long)blockIdx.x * blockDim.x + threadIdx.x; pix < P;
       pix += (long long)gridDim.x * blockDim.x) {
    const int b = (int)(pix / HW);
    const long long hw = pix - (long long)b * HW;
    const int y = (int)(hw / W), x = (int)(hw - (long long)y * W);
    float v[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) v[c] = 0.f;
    int c0 = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {  // sources unrolled: no dynamic indexing of kernel arguments
      if (k < nsrc) {
        const float* src = s.p[k] + (long long)b * s.c[k] * HW + hw;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          if (j < s.c[k]) {
            const float t = src[(long long)j * HW];
#pragma unroll
            for (int c = 0; c < 16; ++c)
              if (c == c0 + j) v[c] = t;
          }
        }
        c0 += s.c[k];
      }
    }
    T* out = reinterpret_cast<T*>(d.p) + vidx(d, b, y, x, 0);
#pragma unroll
    for (int g = 0; g < 16; g += N) {
      if (g >= Cpad) break;
      if constexpr (sizeof(T) == 4) {
        *reinterpret_cast<float4*>(out + g) = make_float4(v[g], v[g + 1], v[g + 2], v[g + 3]);
      } else {
        uint4 o;
        o.x = (unsigned)f2bf(v[g]) | ((unsigned)f2bf(v[g + 1]) << 16);
        o.y = (unsigned)f2bf(v[g + 2]) | ((unsigned)f2bf(v[g + 3]) << 16);
        o.z = (unsigned)f2bf(v[g + 4]) | ((unsigned)f2bf(v[g + 5]) << 16);
        o.w = (unsigned)f2bf(v[g + 6]) | ((unsigned)f2bf(v[g + 7]) << 16);
        *reinterpret_cast<uint4*>(out + g) = o;
      }
    }
  }
}

// Four consecutive pixels of one image row per thread (H*W < 2^31, W % 4 == 0, 16-byte aligned planes):
// one float4 load per channel plane, a per-channel (plane pointer, image stride) table instead of the
// source walk, 32-bit index math.  Same values as gather_vec_kernel.
struct ChanTab {
  const float* p[16];  // channel c's plane of image 0
  long long bs[16];    // image stride of channel c's source
  int n;               // real channels (the rest of Cpad is zero)
};
template <typename T, typename I>  // I: the quad index type (int when B * HW / 4 < 2^31: no 64-bit division)
__global__ void __launch_bounds__(256) gather4_kernel(int B, int HW, int W, ChanTab t, View d, int Cpad) {
  constexpr int N = 16 / sizeof(T);
  const I quads = (I)B * (I)(HW >> 2);
  for (I qd = (I)blockIdx.x * blockDim.x + threadIdx.x; qd < quads; qd += (I)gridDim.x * blockDim.x) {
    const int b = (int)(qd / (I)(HW >> 2));
    const int hw = (int)(qd - (I)b * (HW >> 2)) << 2;
    float4 v[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      v[c] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (c < t.n) v[c] = *reinterpret_cast<const float4*>(t.p[c] + (long long)b * t.bs[c] + hw);
    }
    const int y = hw / W, x = hw - y * W;
    T* out = reinterpret_cast<T*>(d.p) + vidx(d, b, y, x, 0);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float f[16];
#pragma unroll
      for (int c = 0; c < 16; ++c) f[c] = q == 0 ? v[c].x : q == 1 ? v[c].y : q == 2 ? v[c].z : v[c].w;
      T* o = out + (long long)q * d.ps;
#pragma unroll
      for (int g = 0; g < 16; g += N) {
        if (g >= Cpad) break;
        if constexpr (sizeof(T) == 4) {
          *reinterpret_cast<float4*>(o + g) = make_float4(f[g], f[g + 1], f[g + 2], f[g + 3]);
        } else {
          uint4 w;
          w.x = (unsigned)f2bf(f[g]) | ((unsigned)f2bf(f[g + 1]) << 16);
          w.y = (unsigned)f2bf(f[g + 2]) | ((unsigned)f2bf(f[g + 3]) << 16);
          w.z = (unsigned)f2bf(f[g + 4]) | ((unsigned)f2bf(f[g + 5]) << 16);
          w.w = (unsigned)f2bf(f[g + 6]) | ((unsigned)f2bf(f[g + 7]) << 16);
          *reinterpret_cast<uint4*>(o + g) = w;
        }
      }
    }
  }
}

template <typename T>
__global__ void scatter_kernel(int B, int H, int W, View s, int nsrc, Dst4 d) {
  const long long HW = (long long)H * W, P = HW * B;
  for (long long pix = (long long)blockIdx.x * blockDim.x + threadIdx.x; pix < P;
       pix += (long long)gridDim.x * blockDim.x) {
    const int b = (int)(pix / HW);
    const long long hw = pix % HW;
    const int y = (int)(hw / W), x = (int)(hw % W);
    const T* in = reinterpret_cast<const T*>(s.p) + vidx(s, b, y, x, 0);
    int c = 0;
    for (int k = 0; k < nsrc; ++k) {
      float* dst = d.p[k] ? d.p[k] + (long long)b * d.c[k] * HW + hw : nullptr;
      for (int j = 0; j < d.c[k]; ++j, ++c)
        if (dst) dst[(long long)j * HW] = ld1<T>(in + (long long)c * s.cs);
    }
  }
}

// ------------------------------------------------------------------ tanh + bias backward
// dq[b,y,x,c] = gy*(1-y^2) for c < C, 0 for C <= c < Cpad (dq view has Cpad channels);
// part[chunk][c] = sum over the chunk's pixels of dq (c < C)
template <typename T>
__global__ void tanh_bwd_kernel(int B, int C, int H, int W, const float* y, const float* gy, View dq, int Cpad,
                                float* part, int nchunks) {
  const long long HW = (long long)H * W, P = HW * B;
  const long long per = (P + nchunks - 1) / nchunks;
  const long long p0 = blockIdx.x * per, p1 = min(P, p0 + per);
  float acc[4] = {0, 0, 0, 0};
  for (long long pix = p0 + threadIdx.x; pix < p1; pix += blockDim.x) {
    const int b = (int)(pix / HW);
    const long long hw = pix % HW;
    const int yy = (int)(hw / W), xx = (int)(hw % W);
    T* out = reinterpret_cast<T*>(dq.p) + vidx(dq, b, yy, xx, 0);
    for (int c = 0; c < Cpad; ++c) {
      float v = 0.f;
      if (c < C) {
        const long long i = ((long long)b * C + c) * HW + hw;
        const float t = y[i];
        v = gy[i] * (1.f - t * t);
        acc[c] += v;
      }
      st1<T>(out + (long long)c * dq.cs, v);
    }
  }
  __shared__ float red[4][256];
  for (int c = 0; c < 4; ++c) red[c][threadIdx.x] = acc[c];
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s)
      for (int c = 0; c < 4; ++c) red[c][threadIdx.x] += red[c][threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x < C) part[(long long)blockIdx.x * C + threadIdx.x] = red[threadIdx.x][0];
}

// The same with 4 consecutive pixels per thread (W % 4 == 0, 16-byte NHWC dq pixels, 32-bit indices): float4 loads of
// y / gy per channel plane and one 16-byte store per pixel instead of Cpad element stores; chunks of whole quads.
// part is summed per thread in pixel order, then over the block in a fixed tree order (deterministic).
template <typename T>
__global__ void __launch_bounds__(256) tanh_bwd4_kernel(int B, int C, int HW, int W, const float* y, const float* gy,
                                                        View dq, int per4, float* part) {
  const int P = B * HW;
  const int p0 = blockIdx.x * per4, p1 = min(P, p0 + per4);
  float acc[4] = {0, 0, 0, 0};
  for (int q = p0 + 4 * (int)threadIdx.x; q < p1; q += 4 * (int)blockDim.x) {
    const int b = q / HW, hw = q - b * HW;
    const int yy = hw / W, xx = hw - yy * W;
    float v[4][4];  // [channel][pixel]
#pragma unroll
    for (int c = 0; c < 4; ++c) {
#pragma unroll
      for (int i = 0; i < 4; ++i) v[c][i] = 0.f;
      if (c < C) {
        const int o = (b * C + c) * HW + hw;
        const float4 t = *reinterpret_cast<const float4*>(y + o);
        const float4 g = *reinterpret_cast<const float4*>(gy + o);
        v[c][0] = g.x * (1.f - t.x * t.x);
        v[c][1] = g.y * (1.f - t.y * t.y);
        v[c][2] = g.z * (1.f - t.z * t.z);
        v[c][3] = g.w * (1.f - t.w * t.w);
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[c] += v[c][i];
      }
    }
    T* out = reinterpret_cast<T*>(dq.p) + vidx(dq, b, yy, xx, 0);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if constexpr (sizeof(T) == 4) {
        *reinterpret_cast<float4*>(out + (long long)i * dq.ps) = make_float4(v[0][i], v[1][i], v[2][i], v[3][i]);
      } else {
        uint4 w;
        w.x = pack_bf16x2(v[0][i], v[1][i]);
        w.y = pack_bf16x2(v[2][i], v[3][i]);
        w.z = 0u;
        w.w = 0u;
        *reinterpret_cast<uint4*>(out + (long long)i * dq.ps) = w;
      }
    }
  }
  __shared__ float red[4][256];
  for (int c = 0; c < 4; ++c) red[c][threadIdx.x] = acc[c];
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s)
      for (int c = 0; c < 4; ++c) red[c][threadIdx.x] += red[c][threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x < C) part[(long long)blockIdx.x * C + threadIdx.x] = red[threadIdx.x][0];
}

__global__ void chunk_sum_kernel(const float* part, int nchunks, int C, float* out) {
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
  if (threadIdx.x == 0) out[c] = (float)s[0];
}

// ------------------------------------------------------------------ losses
constexpr int LOSS_BLOCK = 256, LOSS_PER_BLOCK = 256 * 16;

__device__ __forceinline__ float loss_elem(int kind, float p, float t) {
  if (kind == STC_LOSS_L1) return fabsf(p - t);
  if (kind == STC_LOSS_MSE_CONST) { const float d = p - t; return d * d; }
  // BCE with logits: max(x,0) - x*t + log1p(exp(-|x|))
  return fmaxf(p, 0.f) - p * t + log1pf(expf(-fabsf(p)));
}
__device__ __forceinline__ float loss_grad(int kind, float p, float t) {
  if (kind == STC_LOSS_L1) { const float d = p - t; return d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f); }
  if (kind == STC_LOSS_MSE_CONST) return 2.f * (p - t);
  const float s = 1.f / (1.f + expf(-p));
  return s - t;
}

__global__ void loss_partial_kernel(int kind, const float* p, const float* t, float c, long long n, float* part) {
  const long long b0 = (long long)blockIdx.x * LOSS_PER_BLOCK;
  float acc = 0.f;
  for (int k = 0; k < 16; ++k) {
    const long long i = b0 + k * LOSS_BLOCK + threadIdx.x;
    if (i < n) acc += loss_elem(kind, p[i], t ? t[i] : c);
  }
  __shared__ float red[LOSS_BLOCK];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int s = LOSS_BLOCK / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

__global__ void loss_final_kernel(const float* part, int nparts, long long n, float* out) {
  __shared__ double red[256];
  double a = 0;
  for (int k = threadIdx.x; k < nparts; k += 256) a += part[k];
  red[threadIdx.x] = a;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = (float)(red[0] / (double)n);
}

__global__ void loss_bwd_kernel(int kind, const float* p, const float* t, float c, long long n, const float* gout,
                                float* grad) {
  const float g = gout[0] / (float)n;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    grad[i] = g * loss_grad(kind, p[i], t ? t[i] : c);
}

// ------------------------------------------------------------------ weight packing
// One thread per (n, c) pair: reads the 16 contiguous taps W[p][q][0..15] (64 B) once and
// writes them to their 16 (phase, tap) slots; consecutive threads take consecutive c, so
// every output write is coalesced along the operand's contiguous K dimension.
template <typename T>
__global__ void pack_kernel(int mode, const float* W, int P, int Q, T* out, int N_pad, int C_pad, int nph, int taps) {
  const long long total = (long long)N_pad * C_pad;
  const bool n_is_p = (mode == STC_PACK_CONV_FWD || mode == STC_PACK_CONVT_DGRAD);
  for (long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(idx % C_pad);
    const int n = (int)(idx / C_pad);
    const int pi = n_is_p ? n : c, qi = n_is_p ? c : n;
    float w[16];
    if (pi < P && qi < Q) {
      const float4* src = reinterpret_cast<const float4*>(W + ((long long)pi * Q + qi) * 16);
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const float4 f = src[v];
        w[4 * v] = f.x; w[4 * v + 1] = f.y; w[4 * v + 2] = f.z; w[4 * v + 3] = f.w;
      }
    } else {
#pragma unroll
      for (int t = 0; t < 16; ++t) w[t] = 0.f;
    }
    if (taps == 16) {
#pragma unroll
      for (int t = 0; t < 16; ++t) st1<T>(out + ((long long)n * 16 + t) * C_pad + c, w[t]);
    } else {
#pragma unroll
      for (int z = 0; z < 4; ++z) {
        const int ph = z >> 1, pw = z & 1;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int kh = (1 - ph) + 2 * (t >> 1), kw = (1 - pw) + 2 * (t & 1);
          st1<T>(out + (((long long)z * N_pad + n) * 4 + t) * C_pad + c, w[kh * 4 + kw]);
        }
      }
    }
  }
}

static int grid_for(long long work) { return (int)std::max<long long>(1, std::min<long long>((work + 255) / 256, 8192)); }

}  // namespace stc

using namespace stc;

extern "C" int stc_gather_nchw(int dtype, int B, int H, int W, int nsrc, const float* const* src, const int* src_c,
                               stc_view dst, int Cpad, void* stream) {
  STC_REQUIRE(nsrc >= 1 && nsrc <= 4, "stc_gather_nchw: 1..4 sources");
  Src4 s{};
  int tot = 0;
  for (int k = 0; k < nsrc; ++k) { s.p[k] = src[k]; s.c[k] = src_c[k]; tot += src_c[k]; }
  STC_REQUIRE(tot <= Cpad, "stc_gather_nchw: %d channels > Cpad %d", tot, Cpad);
  hipStream_t st = (hipStream_t)stream;
  const long long P = (long long)B * H * W;
  View d = mkview(dst);
  const int N = dtype == STC_F32 ? 4 : 8;
  if (dst.cs == 1 && Cpad <= 16 && Cpad % N == 0 && dst.ps % N == 0 && dst.co % N == 0 && dst.rs % N == 0 &&
      dst.bs % N == 0) {
    bool al = W % 4 == 0 && (long long)H * W < (1ll << 31);
    for (int k = 0; k < nsrc; ++k) al = al && ((uintptr_t)src[k] & 15) == 0;
    if (al) {
      ChanTab t{};
      const long long HW = (long long)H * W;
      for (int k = 0, c = 0; k < nsrc; ++k)
        for (int j = 0; j < src_c[k]; ++j, ++c) { t.p[c] = src[k] + j * HW; t.bs[c] = src_c[k] * HW; }
      t.n = tot;
      const int blocks = (int)std::max<long long>(1, std::min<long long>((P / 4 + 255) / 256, 4096));
      if (P / 4 < (1ll << 31)) {
        if (dtype == STC_F32) hipLaunchKernelGGL((gather4_kernel<float, int>), dim3(blocks), dim3(256), 0, st, B, (int)HW, W, t, d, Cpad);
        else hipLaunchKernelGGL((gather4_kernel<bf16, int>), dim3(blocks), dim3(256), 0, st, B, (int)HW, W, t, d, Cpad);
      } else {
        if (dtype == STC_F32) hipLaunchKernelGGL((gather4_kernel<float, long long>), dim3(blocks), dim3(256), 0, st, B, (int)HW, W, t, d, Cpad);
        else hipLaunchKernelGGL((gather4_kernel<bf16, long long>), dim3(blocks), dim3(256), 0, st, B, (int)HW, W, t, d, Cpad);
      }
      STC_CHECK_LAUNCH();
      return 0;
    }
    if (dtype == STC_F32) hipLaunchKernelGGL(gather_vec_kernel<float>, dim3(grid_for(P)), dim3(256), 0, st, B, H, W, nsrc, s, d, Cpad);
    else hipLaunchKernelGGL(gather_vec_kernel<bf16>, dim3(grid_for(P)), dim3(256), 0, st, B, H, W, nsrc, s, d, Cpad);
    STC_CHECK_LAUNCH();
    return 0;
  }
  if (dtype == STC_F32) hipLaunchKernelGGL(gather_kernel<float>, dim3(grid_for(P)), dim3(256), 0, st, B, H, W, nsrc, s, d, Cpad);
  else hipLaunchKernelGGL(gather_kernel<bf16>, dim3(grid_for(P)), dim3(256), 0, st, B, H, W, nsrc, s, d, Cpad);
  STC_CHECK_LAUNCH();
  return 0;
}

extern "C" int stc_scatter_nchw(int dtype, int B, int H, int W, stc_view src, int nsrc, float* const* dst,
                                const int* dst_c, void* stream) {
  STC_REQUIRE(nsrc >= 1 && nsrc <= 4, "stc_scatter_nchw: 1..4 destinations");
  Dst4 d{};
  for (int k = 0; k < nsrc; ++k) { d.p[k] = dst[k]; d.c[k] = dst_c[k]; }
  hipStream_t st = (hipStream_t)stream;
  const long long P = (long long)B * H * W;
  View s = mkview(src);
  if (dtype == STC_F32) hipLaunchKernelGGL(scatter_kernel<float>, dim3(grid_for(P)), dim3(256), 0, st, B, H, W, s, nsrc, d);
  else hipLaunchKernelGGL(scatter_kernel<bf16>, dim3(grid_for(P)), dim3(256), 0, st, B, H, W, s, nsrc, d);
  STC_CHECK_LAUNCH();
  return 0;
}

extern "C" int stc_tanh_bias_bwd(int dtype, int B, int C, int H, int W, const float* y, const float* gy, stc_view dq,
                                 float* dbias, float* part, int nchunks, void* stream) {
  STC_REQUIRE(C >= 1 && C <= 4, "stc_tanh_bias_bwd: C=%d", C);
  hipStream_t st = (hipStream_t)stream;
  const int Cpad = dtype == STC_F32 ? 4 : 8;
  View d = mkview(dq);
  const long long P = (long long)B * H * W;
  const bool quad = W % 4 == 0 && P * 4 < (1ll << 31) && dq.cs == 1 && dq.co == 0 && dq.ps == Cpad &&
                    dq.rs % Cpad == 0 && dq.bs % Cpad == 0 && ((uintptr_t)dq.p & 15) == 0 &&
                    ((uintptr_t)y & 15) == 0 && ((uintptr_t)gy & 15) == 0;
  if (quad) {
    const int per4 = (int)((((P + nchunks - 1) / nchunks) + 3) & ~3ll);
    if (dtype == STC_F32)
      hipLaunchKernelGGL(tanh_bwd4_kernel<float>, dim3(nchunks), dim3(256), 0, st, B, C, H * W, W, y, gy, d, per4, part);
    else
      hipLaunchKernelGGL(tanh_bwd4_kernel<bf16>, dim3(nchunks), dim3(256), 0, st, B, C, H * W, W, y, gy, d, per4, part);
  } else if (dtype == STC_F32)
    hipLaunchKernelGGL(tanh_bwd_kernel<float>, dim3(nchunks), dim3(256), 0, st, B, C, H, W, y, gy, d, Cpad, part, nchunks);
  else
    hipLaunchKernelGGL(tanh_bwd_kernel<bf16>, dim3(nchunks), dim3(256), 0, st, B, C, H, W, y, gy, d, Cpad, part, nchunks);
  STC_CHECK_LAUNCH();
  if (dbias) {
    hipLaunchKernelGGL(chunk_sum_kernel, dim3(C), dim3(256), 0, st, (const float*)part, nchunks, C, dbias);
    STC_CHECK_LAUNCH();
  }
  return 0;
}

extern "C" int stc_loss_parts(int64_t n) { return (int)((n + LOSS_PER_BLOCK - 1) / LOSS_PER_BLOCK); }

extern "C" int stc_loss_fwd(int kind, const float* p, const float* t, float c, int64_t n, float* part, float* out,
                            void* stream) {
  STC_REQUIRE(kind >= 0 && kind <= 2, "stc_loss_fwd: bad kind");
  STC_REQUIRE(n > 0, "stc_loss_fwd: empty input");
  STC_REQUIRE(kind != STC_LOSS_L1 || t != nullptr, "stc_loss_fwd: L1 needs a target tensor");
  hipStream_t st = (hipStream_t)stream;
  const int np = stc_loss_parts(n);
  hipLaunchKernelGGL(loss_partial_kernel, dim3(np), dim3(LOSS_BLOCK), 0, st, kind, p, t, c, (long long)n, part);
  STC_CHECK_LAUNCH();
  hipLaunchKernelGGL(loss_final_kernel, dim3(1), dim3(256), 0, st, (const float*)part, np, (long long)n, out);
  STC_CHECK_LAUNCH();
  return 0;
}

extern "C" int stc_loss_bwd(int kind, const float* p, const float* t, float c, int64_t n, const float* gout,
                            float* grad, void* stream) {
  STC_REQUIRE(kind >= 0 && kind <= 2, "stc_loss_bwd: bad kind");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(loss_bwd_kernel, dim3(grid_for(n)), dim3(256), 0, st, kind, p, t, c, (long long)n, gout, grad);
  STC_CHECK_LAUNCH();
  return 0;
}

// ---- several loss terms of one objective in two launches (forward) / one launch (backward) --------
// Each term is exactly stc_loss_fwd's two-level sum (same blocks, same per-block order, the same fp64
// final reduction), so its value is bit-identical to the single-term call; the objective's combination
// of the terms (STCGAN/stcgan.py:240-251, 291-299) is then evaluated with one fp32 rounding per torch op,
// in torch's order, and the backward scales each term by the same fp32 product chain autograd forms.
struct LossTerms {
  const float* p[STC_LOSS_MAX_TERMS];
  const float* t[STC_LOSS_MAX_TERMS];
  float* g[STC_LOSS_MAX_TERMS];
  long long n[STC_LOSS_MAX_TERMS];
  float c[STC_LOSS_MAX_TERMS];
  float wa[STC_LOSS_MAX_TERMS], wb[STC_LOSS_MAX_TERMS];
  int kind[STC_LOSS_MAX_TERMS];
  int first[STC_LOSS_MAX_TERMS + 1];  // first block of each term
  int count;
};

__device__ __forceinline__ int loss_term_of(const LossTerms& a, int blk) {
  int k = 0;
  while (k + 1 < a.count && blk >= a.first[k + 1]) ++k;
  return k;
}

__global__ void loss_multi_partial_kernel(LossTerms a, float* part) {
  const int k = loss_term_of(a, blockIdx.x);
  const long long b0 = (long long)(blockIdx.x - a.first[k]) * LOSS_PER_BLOCK;
  const float* p = a.p[k];
  const float* t = a.t[k];
  const long long n = a.n[k];
  const int kind = a.kind[k];
  const float c = a.c[k];
  float acc = 0.f;
  for (int q = 0; q < 16; ++q) {
    const long long i = b0 + q * LOSS_BLOCK + threadIdx.x;
    if (i < n) acc += loss_elem(kind, p[i], t ? t[i] : c);
  }
  __shared__ float red[LOSS_BLOCK];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int s = LOSS_BLOCK / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

#pragma clang fp contract(off)
// vals[k] = term k (then D1, D2 for STC_LOSS_COMBINE_D); out[0] = the objective
__global__ void loss_multi_final_kernel(LossTerms a, const float* part, int mode, float w0, float w1, float w2,
                                        float* vals, float* out) {
  __shared__ double red[256];
  __shared__ float v[STC_LOSS_MAX_TERMS];
  for (int k = 0; k < a.count; ++k) {
    double s = 0;
    for (int q = a.first[k] + threadIdx.x; q < a.first[k + 1]; q += 256) s += part[q];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int h = 128; h > 0; h >>= 1) {
      if (threadIdx.x < h) red[threadIdx.x] += red[threadIdx.x + h];
      __syncthreads();
    }
    if (threadIdx.x == 0) v[k] = (float)(red[0] / (double)a.n[k]);
    __syncthreads();
  }
  if (threadIdx.x != 0) return;
  for (int k = 0; k < a.count; ++k) vals[k] = v[k];
  if (mode == STC_LOSS_COMBINE_D) {
    // D1 = (fake1 + real1) * 0.5, D2 = (fake2 + real2) * 0.5, D = l2 * D1 + l3 * D2
    const float d1 = (v[0] + v[1]) * 0.5f, d2 = (v[2] + v[3]) * 0.5f;
    out[0] = d1 * w0 + d2 * w1;
    vals[a.count] = d1;
    vals[a.count + 1] = d2;
  } else {
    // G = ((data1 + l1 * data2) + l2 * G1) + l3 * G2
    out[0] = ((v[0] + v[1] * w0) + v[2] * w1) + v[3] * w2;
  }
}

// grad_k = ((gout * wa_k) * wb_k) / n_k * dloss_k/dp, the chain autograd applies to a term of the objective
__global__ void loss_multi_bwd_kernel(LossTerms a, const float* gout) {
  const int k = loss_term_of(a, blockIdx.x);
  float* grad = a.g[k];
  if (!grad) return;
  const float g = ((gout[0] * a.wa[k]) * a.wb[k]) / (float)a.n[k];
  const float* p = a.p[k];
  const float* t = a.t[k];
  const long long n = a.n[k];
  const int kind = a.kind[k];
  const float c = a.c[k];
  const long long nb = a.first[k + 1] - a.first[k];
  for (long long i = (long long)(blockIdx.x - a.first[k]) * 256 + threadIdx.x; i < n; i += nb * 256)
    grad[i] = g * loss_grad(kind, p[i], t ? t[i] : c);
}
#pragma clang fp contract(on)

// Multi-tensor form: one launch packs up to STC_PACK_MAX weights; block ranges per descriptor.
struct PackSet {
  stc_pack_desc d[STC_PACK_MAX];
  int bstart[STC_PACK_MAX + 1];
  int n;
};

template <typename T>
__global__ void pack_multi_kernel(const PackSet ps) {
  int i = 0;
  while (i + 1 < ps.n && (int)blockIdx.x >= ps.bstart[i + 1]) ++i;
  const stc_pack_desc& d = ps.d[i];
  const int mode = d.mode;
  const bool phased = mode == STC_PACK_CONV_DGRAD || mode == STC_PACK_CONVT_FWD;
  const int taps = phased ? 4 : 16;
  const long long total = (long long)d.N_pad * d.C_pad;
  const bool n_is_p = (mode == STC_PACK_CONV_FWD || mode == STC_PACK_CONVT_DGRAD);
  const int nblk = ps.bstart[i + 1] - ps.bstart[i];
  T* out = reinterpret_cast<T*>(d.out);
  for (long long idx = (long long)(blockIdx.x - ps.bstart[i]) * blockDim.x + threadIdx.x; idx < total;
       idx += (long long)nblk * blockDim.x) {
    const int c = (int)(idx % d.C_pad);
    const int n = (int)(idx / d.C_pad);
    const int pi = n_is_p ? n : c, qi = n_is_p ? c : n;
    float w[16];
    if (pi < d.P && qi < d.Q) {
      const float4* src = reinterpret_cast<const float4*>(d.W + ((long long)pi * d.Q + qi) * 16);
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const float4 f = src[v];
        w[4 * v] = f.x; w[4 * v + 1] = f.y; w[4 * v + 2] = f.z; w[4 * v + 3] = f.w;
      }
    } else {
#pragma unroll
      for (int t = 0; t < 16; ++t) w[t] = 0.f;
    }
    if (taps == 16) {
#pragma unroll
      for (int t = 0; t < 16; ++t) st1<T>(out + ((long long)n * 16 + t) * d.C_pad + c, w[t]);
    } else {
#pragma unroll
      for (int z = 0; z < 4; ++z) {
        const int ph = z >> 1, pw = z & 1;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int kh = (1 - ph) + 2 * (t >> 1), kw = (1 - pw) + 2 * (t & 1);
          st1<T>(out + (((long long)z * d.N_pad + n) * 4 + t) * d.C_pad + c, w[kh * 4 + kw]);
        }
      }
    }
  }
}

extern "C" int stc_pack_weights(int dtype, int n, const stc_pack_desc* descs, void* stream) {
  STC_REQUIRE(n >= 0 && n <= STC_PACK_MAX && (n == 0 || descs), "stc_pack_weights: bad count %d", n);
  if (n == 0) return 0;
  PackSet ps{};
  ps.n = n;
  int b = 0;
  for (int i = 0; i < n; ++i) {
    STC_REQUIRE(descs[i].mode >= 0 && descs[i].mode <= 4 && descs[i].W && descs[i].out, "stc_pack_weights: bad desc %d", i);
    ps.d[i] = descs[i];
    ps.bstart[i] = b;
    const long long total = (long long)descs[i].N_pad * descs[i].C_pad;
    b += (int)std::max<long long>(1, std::min<long long>((total + 255) / 256, 1024));
  }
  ps.bstart[n] = b;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == STC_F32) hipLaunchKernelGGL(pack_multi_kernel<float>, dim3(b), dim3(256), 0, st, ps);
  else hipLaunchKernelGGL(pack_multi_kernel<bf16>, dim3(b), dim3(256), 0, st, ps);
  STC_CHECK_LAUNCH();
  return 0;
}

extern "C" int stc_pack_weight(int dtype, int mode, const float* W, int P, int Q, void* out, int N_pad, int C_pad,
                               void* stream) {
  STC_REQUIRE(mode >= 0 && mode <= 4, "stc_pack_weight: bad mode");
  const bool phased = mode == STC_PACK_CONV_DGRAD || mode == STC_PACK_CONVT_FWD;
  const int nph = phased ? 4 : 1, taps = phased ? 4 : 16;
  hipStream_t st = (hipStream_t)stream;
  const long long total = (long long)N_pad * C_pad;  // one thread per (n, c)
  if (dtype == STC_F32)
    hipLaunchKernelGGL(pack_kernel<float>, dim3(grid_for(total)), dim3(256), 0, st, mode, W, P, Q, (float*)out, N_pad, C_pad, nph, taps);
  else
    hipLaunchKernelGGL(pack_kernel<bf16>, dim3(grid_for(total)), dim3(256), 0, st, mode, W, P, Q, (bf16*)out, N_pad, C_pad, nph, taps);
  STC_CHECK_LAUNCH();
  return 0;
}

static int loss_terms(int nterm, const int32_t* kinds, const float* consts, const float* const* preds,
                      const float* const* targets, const int64_t* numels, LossTerms& a, bool bwd_blocks) {
  STC_REQUIRE(nterm >= 1 && nterm <= STC_LOSS_MAX_TERMS, "stc_loss_multi: 1..%d terms", STC_LOSS_MAX_TERMS);
  int blocks = 0;
  a.count = nterm;
  for (int k = 0; k < nterm; ++k) {
    STC_REQUIRE(kinds[k] >= 0 && kinds[k] <= 2 && numels[k] > 0 && preds[k], "stc_loss_multi: bad term %d", k);
    STC_REQUIRE(kinds[k] != STC_LOSS_L1 || targets[k], "stc_loss_multi: L1 term %d needs a target", k);
    a.p[k] = preds[k];
    a.t[k] = targets[k];
    a.n[k] = numels[k];
    a.c[k] = consts[k];
    a.kind[k] = kinds[k];
    a.first[k] = blocks;
    blocks += bwd_blocks ? (int)std::min<int64_t>((numels[k] + 255) / 256, 2048) : stc_loss_parts(numels[k]);
  }
  a.first[nterm] = blocks;
  return blocks;
}

extern "C" int stc_loss_multi_parts(int nterm, const int64_t* numels) {
  int np = 0;
  for (int k = 0; k < nterm; ++k) np += stc_loss_parts(numels[k]);
  return np;
}

extern "C" int stc_loss_multi_fwd(int nterm, const int32_t* kinds, const float* consts, const float* const* preds,
                                  const float* const* targets, const int64_t* numels, int mode, const float* w,
                                  float* part, float* vals, float* out, void* stream) {
  STC_REQUIRE(mode == STC_LOSS_COMBINE_D || mode == STC_LOSS_COMBINE_G, "stc_loss_multi_fwd: bad mode");
  STC_REQUIRE(nterm == 4, "stc_loss_multi_fwd: the combinations take 4 terms");
  LossTerms a{};
  const int blocks = loss_terms(nterm, kinds, consts, preds, targets, numels, a, false);
  if (blocks < 0) return blocks;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(loss_multi_partial_kernel, dim3(blocks), dim3(LOSS_BLOCK), 0, st, a, part);
  STC_CHECK_LAUNCH();
  hipLaunchKernelGGL(loss_multi_final_kernel, dim3(1), dim3(256), 0, st, a, (const float*)part, mode, w[0], w[1],
                     w[2], vals, out);
  STC_CHECK_LAUNCH();
  return 0;
}

extern "C" int stc_loss_multi_bwd(int nterm, const int32_t* kinds, const float* consts, const float* const* preds,
                                  const float* const* targets, const int64_t* numels, const float* wa,
                                  const float* wb, const float* gout, float* const* grads, void* stream) {
  LossTerms a{};
  const int blocks = loss_terms(nterm, kinds, consts, preds, targets, numels, a, true);
  if (blocks < 0) return blocks;
  for (int k = 0; k < nterm; ++k) {
    a.g[k] = grads[k];
    a.wa[k] = wa[k];
    a.wb[k] = wb[k];
  }
  hipLaunchKernelGGL(loss_multi_bwd_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, a, gout);
  STC_CHECK_LAUNCH();
  return 0;
}
