// Weight gradient of the 4x4 conv / convT family as an implicit GEMM over pixels.
//
//   dW[r][ci][kh][kw] = sum_{b,oy,ox} D[b,oy,ox,r] * G[b, oy*s+kh-1, ox*s+kw-1, ci]
//   Conv2d s2/s1 : D = dy (output grid), G = x       (SURVEY.md a4/a5 backward)
//   ConvT  s2    : D = x  (input grid),  G = dy, s=2 (SURVEY.md a6 backward)
//
// GEMM view: C[R][16*Cg] = sum_p A[p][R]^T * Bcol[p][16*Cg]; both operands are
// pixel-major in HBM (channels contiguous), so they are staged into LDS as
// [pixel][channel] rows with 16-byte loads/stores and read by the f32 MFMA
// (v_mfma_f32_32x32x2_f32: lane l feeds A[i=l&31][k=l>>5]) with conflict-free
// ds_read_b32 across consecutive channels.  The pixel dimension is split over
// blockIdx.z into fp32 slabs that a second kernel sums in a fixed order
// (bitwise reproducible) while writing torch layout [R][Cg][4][4].
// bf16 operands are widened to fp32 while staging (exact), so both dtypes share
// the f32 MFMA path.
#include "common.hpp"

namespace stc {

struct WgradParams {
  const char* d;
  long long d_bs, d_rs;
  int d_ps, d_co;
  const char* g;
  long long g_bs, g_rs;
  int g_ps, g_co;
  int GH, GW;  // D grid (the reduction domain) -> P = B*GH*GW
  int IH, IW;  // G logical bounds
  int stride;
  int R, Cg, Ncol;  // Ncol = 16*Cg
  int P, pchunk, nsplit;
  const float *dsc, *dsh, *gsc, *gsh;
  int dact, gact;
  float dslope, gslope;
  float* ws;  // [nsplit][R][Ncol]
  int mtiles, ntiles;
};

constexpr int WG_BM = 128, WG_BN = 128, WG_BK = 32;
constexpr int WG_LDA = WG_BM + 4;  // floats; +4 keeps rows 16-byte aligned

template <typename T>
__device__ __forceinline__ float4 load4(const char* base, long long off) {
  return Vec4<T>::load(reinterpret_cast<const T*>(base) + off);
}

__device__ __forceinline__ float4 pro4(float4 v, const float* sc, const float* sh, int c, int act_on, float slope) {
  if (sc) {
    v.x = fmaf(v.x, sc[c], sh[c]); v.y = fmaf(v.y, sc[c + 1], sh[c + 1]);
    v.z = fmaf(v.z, sc[c + 2], sh[c + 2]); v.w = fmaf(v.w, sc[c + 3], sh[c + 3]);
  }
  if (act_on) {
    v.x = act(v.x, slope); v.y = act(v.y, slope); v.z = act(v.z, slope); v.w = act(v.w, slope);
  }
  return v;
}

template <typename T>
__global__ void __launch_bounds__(256)
wgrad_kernel(const WgradParams p) {
  __shared__ __attribute__((aligned(16))) float sA[2][WG_BK][WG_LDA];
  __shared__ __attribute__((aligned(16))) float sB[2][WG_BK][WG_LDA];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int nwg = p.mtiles * p.ntiles;
  int bid = blockIdx.x;
  {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int mt = bid / p.ntiles, nt = bid % p.ntiles;
  const int r0 = mt * WG_BM, c0 = nt * WG_BN;
  const int split = blockIdx.z;
  const int pbeg = split * p.pchunk;
  const int pend = min(p.P, pbeg + p.pchunk);
  const int GHW = p.GH * p.GW;

  // staging map: row (pixel) kp = tid/32 + 8*i, chunk (4 channels) = tid%32
  const int chunk = tid & 31;
  const int rr = r0 + chunk * 4;     // D channel of this chunk
  const int col = c0 + chunk * 4;    // G column of this chunk
  const bool rval = rr < p.R;
  const bool cval = col < p.Ncol;
  const int t = col / p.Cg, ci = col - t * p.Cg;
  const int kh = t >> 2, kw = t & 3;

  float4 va[4], vb[4];
  auto load = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int pix = k0 + (tid >> 5) + 8 * i;
      va[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      vb[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (pix < pend) {
        const int b = pix / GHW, rem = pix - b * GHW;
        const int oy = rem / p.GW, ox = rem - oy * p.GW;
        if (rval) {
          float4 v = load4<T>(p.d, (long long)b * p.d_bs + (long long)oy * p.d_rs + (long long)ox * p.d_ps + p.d_co + rr);
          va[i] = pro4(v, p.dsc ? p.dsc + rr : nullptr, p.dsh ? p.dsh + rr : nullptr, 0, p.dact, p.dslope);
        }
        const int iy = oy * p.stride + kh - 1, ix = ox * p.stride + kw - 1;
        if (cval && (unsigned)iy < (unsigned)p.IH && (unsigned)ix < (unsigned)p.IW) {
          float4 v = load4<T>(p.g, (long long)b * p.g_bs + (long long)iy * p.g_rs + (long long)ix * p.g_ps + p.g_co + ci);
          vb[i] = pro4(v, p.gsc ? p.gsc + ci : nullptr, p.gsh ? p.gsh + ci : nullptr, 0, p.gact, p.gslope);
        }
      }
    }
  };
  auto store = [&](int st) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int kp = (tid >> 5) + 8 * i;
      *reinterpret_cast<float4*>(&sA[st][kp][chunk * 4]) = va[i];
      *reinterpret_cast<float4*>(&sB[st][kp][chunk * 4]) = vb[i];
    }
  };

  floatx16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int nsteps = (pend - pbeg + WG_BK - 1) / WG_BK;
  if (nsteps > 0) {
    load(pbeg);
    store(0);
  }
  __syncthreads();
  const int li = lane & 31, lh = lane >> 5;
  for (int s = 0; s < nsteps; ++s) {
    const int cur = s & 1;
    if (s + 1 < nsteps) load(pbeg + (s + 1) * WG_BK);
#pragma unroll 4
    for (int kk = 0; kk < WG_BK / 2; ++kk) {
      const int k = 2 * kk + lh;
      float a0 = sA[cur][k][wm * 64 + li];
      float a1 = sA[cur][k][wm * 64 + 32 + li];
      float b0 = sB[cur][k][wn * 64 + li];
      float b1 = sB[cur][k][wn * 64 + 32 + li];
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
    }
    if (s + 1 < nsteps) store(cur ^ 1);
    __syncthreads();
  }

  float* slab = p.ws + (long long)split * p.R * p.Ncol;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = c0 + wn * 64 + 32 * j + li;
      if (n >= p.Ncol) continue;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int m = r0 + wm * 64 + 32 * i + (e & 3) + 8 * (e >> 2) + 4 * lh;
        if (m < p.R) slab[(long long)m * p.Ncol + n] = acc[i][j][e];
      }
    }
}

// dW[r][ci][kh][kw] = sum_s ws[s][r][(kh*4+kw)*Cg + ci]
__global__ void wgrad_reduce_kernel(const float* ws, int nsplit, int R, int Cg, int Cg_out, float* dW) {
  const long long total = (long long)R * Cg_out * 16;
  const long long Ncol = 16LL * Cg;
  for (long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (long long)gridDim.x * blockDim.x) {
    const int tap = (int)(idx & 15);
    const long long rc = idx >> 4;
    const int ci = (int)(rc % Cg_out);
    const int r = (int)(rc / Cg_out);
    const float* src = ws + (long long)r * Ncol + (long long)tap * Cg + ci;
    float v = 0.f;
    for (int s = 0; s < nsplit; ++s) v += src[(long long)s * R * Ncol];
    dW[idx] = v;
  }
}

struct WgPlan {
  int mtiles, ntiles, nsplit, pchunk;
};
static WgPlan wg_plan(int P, int R, int Cg) {
  WgPlan pl{};
  pl.mtiles = cdiv(R, WG_BM);
  pl.ntiles = cdiv(16LL * Cg, WG_BN);
  const long long tiles = (long long)pl.mtiles * pl.ntiles;
  int ns = 1;
  const int steps = cdiv(P, WG_BK);
  while (tiles * ns < 768 && ns * 2 <= 256 && steps / (ns * 2) >= 8) ns *= 2;
  pl.pchunk = cdiv(steps, ns) * WG_BK;
  pl.nsplit = cdiv(P, pl.pchunk);
  return pl;
}

}  // namespace stc

using namespace stc;

extern "C" int64_t stc_conv_wgrad_workspace(int dtype, int B, int Hd, int Wd, int R, int Cg) {
  (void)dtype;
  const WgPlan pl = wg_plan(B * Hd * Wd, R, Cg);
  return (int64_t)pl.nsplit * R * 16LL * Cg * 4;
}

extern "C" int stc_conv_wgrad(int dtype, int B, int stride, stc_view D, int R,
                              const float* d_scale, const float* d_shift, int d_act, float d_slope,
                              stc_view G, int Cg, int Cg_out,
                              const float* g_scale, const float* g_shift, int g_act, float g_slope,
                              float* dW, void* workspace, int64_t workspace_bytes, void* stream) {
  STC_REQUIRE(dtype == STC_F32 || dtype == STC_BF16, "stc_conv_wgrad: bad dtype");
  STC_REQUIRE(Cg >= 4 && Cg % 4 == 0, "stc_conv_wgrad: Cg=%d must be a multiple of 4", Cg);
  STC_REQUIRE(R % 4 == 0, "stc_conv_wgrad: R=%d must be a multiple of 4", R);
  STC_REQUIRE(D.cs == 1 && G.cs == 1 && D.co % 4 == 0 && G.co % 4 == 0 && D.ps % 4 == 0 && G.ps % 4 == 0,
              "stc_conv_wgrad: views must be NHWC with 4-aligned channels");
  STC_REQUIRE(Cg_out <= Cg, "stc_conv_wgrad: Cg_out > Cg");
  WgradParams p{};
  p.d = (const char*)D.p; p.d_bs = D.bs; p.d_rs = D.rs; p.d_ps = D.ps; p.d_co = D.co;
  p.g = (const char*)G.p; p.g_bs = G.bs; p.g_rs = G.rs; p.g_ps = G.ps; p.g_co = G.co;
  p.GH = D.H; p.GW = D.W; p.IH = G.H; p.IW = G.W; p.stride = stride;
  p.R = R; p.Cg = Cg; p.Ncol = 16 * Cg;
  p.P = B * D.H * D.W;
  p.dsc = d_scale; p.dsh = d_shift; p.dact = d_act; p.dslope = d_slope;
  p.gsc = g_scale; p.gsh = g_shift; p.gact = g_act; p.gslope = g_slope;
  hipStream_t st = (hipStream_t)stream;
  if (p.P == 0) {
    (void)hipMemsetAsync(dW, 0, (size_t)R * Cg_out * 16 * 4, st);
    STC_CHECK_LAUNCH();
    return 0;
  }
  const WgPlan pl = wg_plan(p.P, R, Cg);
  p.mtiles = pl.mtiles; p.ntiles = pl.ntiles; p.nsplit = pl.nsplit; p.pchunk = pl.pchunk;
  const int64_t need = (int64_t)pl.nsplit * R * 16LL * Cg * 4;
  STC_REQUIRE(workspace && workspace_bytes >= need, "stc_conv_wgrad: workspace %lld < %lld",
              (long long)workspace_bytes, (long long)need);
  p.ws = (float*)workspace;
  dim3 grid(pl.mtiles * pl.ntiles, 1, pl.nsplit);
  if (dtype == STC_F32) hipLaunchKernelGGL(wgrad_kernel<float>, grid, dim3(256), 0, st, p);
  else hipLaunchKernelGGL(wgrad_kernel<bf16>, grid, dim3(256), 0, st, p);
  STC_CHECK_LAUNCH();
  const long long total = (long long)R * Cg_out * 16;
  const int blocks = (int)std::min<long long>((total + 255) / 256, 4096);
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(blocks), dim3(256), 0, st, (const float*)p.ws, pl.nsplit, R, Cg,
                     Cg_out, dW);
  STC_CHECK_LAUNCH();
  return 0;
}
