// Implicit-GEMM 4x4 convolution family on gfx950 MFMA.
//
// One kernel template serves every forward product on the ST-CGAN path and
// both input gradients:
//   Conv2d k4 s2/s1 p1           : M = B*Ho*Wo, N = Cout, K = 16*Cin
//   ConvTranspose2d k4 s2 p1     : 4 sub-pixel phases, each M = B*Hi*Wi, N = Cout, K = 4*Cin
//   Conv-s2 dgrad == ConvT fwd geometry, ConvT dgrad == Conv-s2 geometry, Conv-s1 dgrad (flipped taps)
// A (activations, NHWC) is gathered on the fly: row m -> (b, y, x), k -> (tap, ci);
// tap offsets are affine in the tap index, so one parameter set describes every case.
// A per-channel affine + leaky prologue applies BatchNorm-apply and LeakyReLU/ReLU of
// the *producer* while loading (zero padding stays zero), so normalised activations
// are never materialised in HBM.
//
// Tile: BM x BN x (128 bytes of K) per stage, 256 threads = 4 waves, each wave a
// (BM/WM) x (BN/WN) sub-tile of 32x32 MFMA blocks.  LDS rows are 128 B of K plus
// 16 B of pad (144 B stride): the 16-lane groups of ds_read_b128 then hit 16
// distinct 16-byte bank slots (conflict-free).  fp32 uses v_mfma_f32_32x32x2_f32
// (4 MFMAs per 16-byte fragment, exact fp32 fmaf chains), bf16 uses
// v_mfma_f32_32x32x16_bf16 (1 MFMA per fragment); both read the same LDS image.
// Register-staged double buffer: the global loads of K-step s+1 are in flight
// while step s runs on MFMA; one barrier per step.
#include "common.hpp"

namespace stc {

struct ConvParams {
  const char* a;
  long long a_bs, a_rs;
  int a_ps, a_co;
  int IH, IW;
  int cin, lg_tw, in_stride;
  int offy[4], offx[4];
  int stepy, stepx;
  const float* sc;
  const float* sh;
  int pro_act;
  float slope;
  int GH, GW, M, N, K;
  int ksplit, kchunk;
  const char* b;
  long long b_phase_stride;
  char* c;
  long long c_bs, c_rs;
  int c_ps, c_co, c_cs;
  int os;
  int oy0[4], ox0[4];
  const float* bias;
  int tanh_, out_f32;
  float* ws;
  int nphase;
  int mtiles, ntiles;
};

constexpr int LDS_ROW = 144;  // 128 B of K + 16 B pad

template <typename T>
__device__ __forceinline__ uint4 prologue16(uint4 v, const float* sc, const float* sh, int ci,
                                            int act_on, float slope) {
  constexpr int VEC = 16 / sizeof(T);
  float f[VEC];
  if constexpr (sizeof(T) == 4) {
    f[0] = __uint_as_float(v.x); f[1] = __uint_as_float(v.y);
    f[2] = __uint_as_float(v.z); f[3] = __uint_as_float(v.w);
  } else {
    unsigned w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      f[2 * q] = __uint_as_float(w[q] << 16);
      f[2 * q + 1] = __uint_as_float(w[q] & 0xffff0000u);
    }
  }
  if (sc) {
#pragma unroll
    for (int e = 0; e < VEC; ++e) f[e] = fmaf(f[e], sc[ci + e], sh[ci + e]);
  }
  if (act_on) {
#pragma unroll
    for (int e = 0; e < VEC; ++e) f[e] = f[e] > 0.f ? f[e] : f[e] * slope;
  }
  uint4 r;
  if constexpr (sizeof(T) == 4) {
    r.x = __float_as_uint(f[0]); r.y = __float_as_uint(f[1]);
    r.z = __float_as_uint(f[2]); r.w = __float_as_uint(f[3]);
  } else {
    unsigned w[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
      w[q] = (unsigned)f2bf(f[2 * q]) | ((unsigned)f2bf(f[2 * q + 1]) << 16);
    r.x = w[0]; r.y = w[1]; r.z = w[2]; r.w = w[3];
  }
  return r;
}

template <typename T, int BM, int BN, int WM, int WN, bool PRO>
__global__ void __launch_bounds__(256, 2)
igemm_kernel(const ConvParams p) {
  constexpr int VEC = 16 / sizeof(T);
  constexpr int BK = 128 / sizeof(T);
  constexpr int AIT = BM / 32;  // 16-byte chunks per thread for A (8 chunks per row)
  constexpr int BIT = BN / 32;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int FM = WTM / 32, FN = WTN / 32;
  constexpr int STAGE = (BM + BN) * LDS_ROW;
  static_assert(WM * WN == 4, "4 waves");
  static_assert(FM >= 1 && FN >= 1, "wave tile >= 32x32");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  long long* rowoff = reinterpret_cast<long long*>(smem + 2 * STAGE);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;

  // XCD-aware bijective remap of the flat tile id: consecutive tiles (sharing A rows)
  // land on the same XCD's L2.
  const int nwg = p.mtiles * p.ntiles;
  int bid = blockIdx.x;
  {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int mt = bid / p.ntiles, nt = bid % p.ntiles;
  const int m0 = mt * BM, n0 = nt * BN;
  const int z = blockIdx.z;
  const int ph = z / p.ksplit, split = z % p.ksplit;
  const int kbeg = split * p.kchunk;
  const int kend = min(p.K, kbeg + p.kchunk);
  const int nsteps = (kend - kbeg + BK - 1) / BK;  // a partial last step is zero-filled past kend
  const int GHW = p.GH * p.GW;
  const int offy = p.offy[ph], offx = p.offx[ph];
  const int tw_mask = (1 << p.lg_tw) - 1;

  // ---- per-thread A row info
  const int ca = tid & 7;
  long long abase[AIT];
  int ayy[AIT], axx[AIT];
#pragma unroll
  for (int i = 0; i < AIT; ++i) {
    const int m = m0 + (tid >> 3) + 32 * i;
    if (m < p.M) {
      const int b = m / GHW, rem = m - b * GHW;
      const int y = rem / p.GW, x = rem - y * p.GW;
      abase[i] = (long long)b * p.a_bs + p.a_co;
      ayy[i] = y * p.in_stride + offy;
      axx[i] = x * p.in_stride + offx;
    } else {
      abase[i] = 0;
      ayy[i] = -100000;  // always out of bounds
      axx[i] = -100000;
    }
  }
  // ---- per-thread B row info
  const T* bptr[BIT];
  bool bval[BIT];
#pragma unroll
  for (int j = 0; j < BIT; ++j) {
    const int n = n0 + (tid >> 3) + 32 * j;
    bval[j] = n < p.N;
    bptr[j] = reinterpret_cast<const T*>(p.b) + p.b_phase_stride * ph + (long long)(bval[j] ? n : 0) * p.K + ca * VEC;
  }
  // ---- output row offsets (direct epilogue)
  if (!p.ws) {
    for (int r = tid; r < BM; r += 256) {
      const int m = m0 + r;
      long long off = -1;
      if (m < p.M) {
        const int b = m / GHW, rem = m - b * GHW;
        const int y = rem / p.GW, x = rem - y * p.GW;
        const int oy = y * p.os + p.oy0[ph], ox = x * p.os + p.ox0[ph];
        off = (long long)b * p.c_bs + (long long)oy * p.c_rs + (long long)ox * p.c_ps;
      }
      rowoff[r] = off;
    }
  }

  // Two register staging sets (ping-pong): the global loads of K-step s+2 are issued at
  // step s and written to LDS at the end of step s+1, so two steps of MFMA work cover
  // their latency (a bf16 K-step is only 16 MFMAs per wave).
  struct Regs {
    uint4 ra[AIT], rb[BIT];
    unsigned amask;  // which A chunks were in bounds (prologue must not touch padding)
    int aci;         // channel of this thread's chunk in the staged K-step
  };
  Regs r0, r1;
  const T* abase_ptr = reinterpret_cast<const T*>(p.a);
  constexpr bool has_pro = PRO;  // the engine materialises activations: PRO=false on its hot path

  auto load_regs = [&](Regs& R, int k0) {
    const int k = k0 + ca * VEC;
    const int t = k / p.cin, ci = k - t * p.cin;
    const int dy = p.stepy * (t >> p.lg_tw), dx = p.stepx * (t & tw_mask);
    R.aci = ci;
    R.amask = 0;
    const bool kin = k < kend;
#pragma unroll
    for (int i = 0; i < AIT; ++i) {
      const int iy = ayy[i] + dy, ix = axx[i] + dx;
      if (kin && (unsigned)iy < (unsigned)p.IH && (unsigned)ix < (unsigned)p.IW) {
        const T* src = abase_ptr + abase[i] + (long long)iy * p.a_rs + (long long)ix * p.a_ps + ci;
        R.ra[i] = *reinterpret_cast<const uint4*>(src);
        R.amask |= 1u << i;
      } else {
        R.ra[i] = make_uint4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int j = 0; j < BIT; ++j) {
      R.rb[j] = (bval[j] && kin) ? *reinterpret_cast<const uint4*>(bptr[j] + k0) : make_uint4(0, 0, 0, 0);
    }
  };
  auto store_lds = [&](Regs& R, int stage) {
    char* sA = smem + stage * STAGE;
    char* sB = sA + BM * LDS_ROW;
#pragma unroll
    for (int i = 0; i < AIT; ++i) {
      uint4 v = R.ra[i];
      if (has_pro && (R.amask >> i & 1u)) v = prologue16<T>(v, p.sc, p.sh, R.aci, p.pro_act, p.slope);
      *reinterpret_cast<uint4*>(sA + ((tid >> 3) + 32 * i) * LDS_ROW + ca * 16) = v;
    }
#pragma unroll
    for (int j = 0; j < BIT; ++j)
      *reinterpret_cast<uint4*>(sB + ((tid >> 3) + 32 * j) * LDS_ROW + ca * 16) = R.rb[j];
  };

  floatx16 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int lrow = lane & 31, lhalf = lane >> 5;
  auto compute = [&](int cur) {
    const char* sA = smem + cur * STAGE;
    const char* sB = sA + BM * LDS_ROW;
#pragma unroll
    for (int kc = 0; kc < 4; ++kc) {
      const int coff = (2 * kc + lhalf) * 16;
      uint4 fa[FM], fb[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i)
        fa[i] = *reinterpret_cast<const uint4*>(sA + (wm * WTM + 32 * i + lrow) * LDS_ROW + coff);
#pragma unroll
      for (int j = 0; j < FN; ++j)
        fb[j] = *reinterpret_cast<const uint4*>(sB + (wn * WTN + 32 * j + lrow) * LDS_ROW + coff);
      if constexpr (sizeof(T) == 4) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
#pragma unroll
          for (int i = 0; i < FM; ++i) {
            const float av = __uint_as_float(e == 0 ? fa[i].x : e == 1 ? fa[i].y : e == 2 ? fa[i].z : fa[i].w);
#pragma unroll
            for (int j = 0; j < FN; ++j) {
              const float bv = __uint_as_float(e == 0 ? fb[j].x : e == 1 ? fb[j].y : e == 2 ? fb[j].z : fb[j].w);
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc[i][j], 0, 0, 0);
            }
          }
        }
      } else {
        typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const bf16x8 av = __builtin_bit_cast(bf16x8, fa[i]);
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            const bf16x8 bv = __builtin_bit_cast(bf16x8, fb[j]);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, acc[i][j], 0, 0, 0);
          }
        }
      }
    }
  };

  if (nsteps > 0) {
    load_regs(r0, kbeg);
    store_lds(r0, 0);
  }
  if (nsteps > 1) load_regs(r1, kbeg + BK);
  __syncthreads();
  // step s: set (s&1) held step s (already in LDS stage s&1); set ((s+1)&1) holds step s+1
  for (int s = 0; s < nsteps; s += 2) {
    if (s + 2 < nsteps) load_regs(r0, kbeg + (s + 2) * BK);
    compute(0);
    if (s + 1 < nsteps) store_lds(r1, 1);
    __syncthreads();
    if (s + 1 >= nsteps) break;
    if (s + 3 < nsteps) load_regs(r1, kbeg + (s + 3) * BK);
    compute(1);
    if (s + 2 < nsteps) store_lds(r0, 0);
    __syncthreads();
  }

  // ---- epilogue
  if (p.ws) {
    float* slab = p.ws + (long long)z * p.M * p.N;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = n0 + wn * WTN + 32 * j + lrow;
        if (n >= p.N) continue;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int m = m0 + wm * WTM + 32 * i + (e & 3) + 8 * (e >> 2) + 4 * lhalf;
          if (m < p.M) slab[(long long)m * p.N + n] = acc[i][j][e];
        }
      }
    return;
  }
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int n = n0 + wn * WTN + 32 * j + lrow;
    if (n >= p.N) continue;
    const float bz = p.bias ? p.bias[n] : 0.f;
    const long long coff = (long long)(p.c_co + n) * p.c_cs;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int r = wm * WTM + 32 * i + (e & 3) + 8 * (e >> 2) + 4 * lhalf;
        const long long ro = rowoff[r];
        if (ro < 0) continue;
        float v = acc[i][j][e] + bz;
        if (p.tanh_) v = tanhf(v);
        if (p.out_f32) reinterpret_cast<float*>(p.c)[ro + coff] = v;
        else st1<T>(reinterpret_cast<T*>(p.c) + ro + coff, v);
      }
    }
  }
}

// Split-K / raw-slab reduction with the epilogue: out[m, n] = epi(sum_s ws[ph][s][m][n])
template <typename T>
__global__ void splitk_reduce_kernel(const ConvParams p) {
  const long long total = (long long)p.nphase * p.M * p.N;
  for (long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (long long)gridDim.x * blockDim.x) {
    const int n = (int)(idx % p.N);
    const long long pm = idx / p.N;
    const int m = (int)(pm % p.M);
    const int ph = (int)(pm / p.M);
    const float* src = p.ws + ((long long)ph * p.ksplit * p.M + m) * p.N + n;
    float v = 0.f;
    for (int s = 0; s < p.ksplit; ++s) v += src[(long long)s * p.M * p.N];
    if (p.bias) v += p.bias[n];
    if (p.tanh_) v = tanhf(v);
    const int GHW = p.GH * p.GW;
    const int b = m / GHW, rem = m - b * GHW;
    const int y = rem / p.GW, x = rem - y * p.GW;
    const int oy = y * p.os + p.oy0[ph], ox = x * p.os + p.ox0[ph];
    const long long off = (long long)b * p.c_bs + (long long)oy * p.c_rs + (long long)ox * p.c_ps +
                          (long long)(p.c_co + n) * p.c_cs;
    if (p.out_f32) reinterpret_cast<float*>(p.c)[off] = v;
    else st1<T>(reinterpret_cast<T*>(p.c) + off, v);
  }
}

// Narrow-N layers (N <= 8: the 1/3-channel generator output, the 1-channel PatchGAN
// logits, first-layer input gradients).  An MFMA tile would waste >= 3/4 of its
// columns, and these layers are HBM-bound (K*4 B read per output pixel for <= 8
// outputs), so one wave computes one output pixel: its 64 lanes stride over the K
// chunks with coalesced 16-byte loads (1 KiB per wave instruction), the weights sit
// in LDS, and a wave shuffle reduces the N partial dots.
template <typename T>
__global__ void __launch_bounds__(256) smalln_kernel(const ConvParams p) {
  constexpr int VEC = 16 / sizeof(T);
  constexpr int NMAX = 8;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* wl = reinterpret_cast<T*>(smem);  // [N][K] of this phase
  const int ph = blockIdx.y;
  const T* wsrc = reinterpret_cast<const T*>(p.b) + p.b_phase_stride * ph;
  const int NK = p.N * p.K;
  for (int i = threadIdx.x * VEC; i < NK; i += 256 * VEC)
    *reinterpret_cast<uint4*>(wl + i) = *reinterpret_cast<const uint4*>(wsrc + i);
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nchunks = p.K / VEC;
  const int GHW = p.GH * p.GW;
  const int tw_mask = (1 << p.lg_tw) - 1;
  const int offy = p.offy[ph], offx = p.offx[ph];
  const T* A = reinterpret_cast<const T*>(p.a);
  for (int m = blockIdx.x * 4 + wave; m < p.M; m += gridDim.x * 4) {
    const int b = m / GHW, rem = m - b * GHW;
    const int y = rem / p.GW, x = rem - y * p.GW;
    const long long abase = (long long)b * p.a_bs + p.a_co;
    float acc[NMAX];
#pragma unroll
    for (int n = 0; n < NMAX; ++n) acc[n] = 0.f;
    for (int c = lane; c < nchunks; c += 64) {
      const int k = c * VEC;
      const int t = k / p.cin, ci = k - t * p.cin;
      const int iy = y * p.in_stride + offy + p.stepy * (t >> p.lg_tw);
      const int ix = x * p.in_stride + offx + p.stepx * (t & tw_mask);
      if ((unsigned)iy >= (unsigned)p.IH || (unsigned)ix >= (unsigned)p.IW) continue;
      uint4 v = *reinterpret_cast<const uint4*>(A + abase + (long long)iy * p.a_rs + (long long)ix * p.a_ps + ci);
      if (p.sc || p.pro_act) v = prologue16<T>(v, p.sc, p.sh, ci, p.pro_act, p.slope);
      float av[VEC];
      if constexpr (sizeof(T) == 4) {
        av[0] = __uint_as_float(v.x); av[1] = __uint_as_float(v.y);
        av[2] = __uint_as_float(v.z); av[3] = __uint_as_float(v.w);
      } else {
        const unsigned w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) { av[2 * q] = __uint_as_float(w[q] << 16); av[2 * q + 1] = __uint_as_float(w[q] & 0xffff0000u); }
      }
#pragma unroll
      for (int n = 0; n < NMAX; ++n) {
        if (n >= p.N) break;
        const T* wr = wl + n * p.K + k;
#pragma unroll
        for (int e = 0; e < VEC; ++e) acc[n] = fmaf(av[e], ld1<T>(wr + e), acc[n]);
      }
    }
#pragma unroll
    for (int n = 0; n < NMAX; ++n) {
      if (n >= p.N) break;
      float s = acc[n];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
      acc[n] = s;
    }
    if (lane < p.N) {
      float v = 0.f;
#pragma unroll
      for (int n = 0; n < NMAX; ++n) if (n == lane) v = acc[n];
      if (p.bias) v += p.bias[lane];
      if (p.tanh_) v = tanhf(v);
      const int oy = y * p.os + p.oy0[ph], ox = x * p.os + p.ox0[ph];
      const long long off = (long long)b * p.c_bs + (long long)oy * p.c_rs + (long long)ox * p.c_ps +
                            (long long)(p.c_co + lane) * p.c_cs;
      if (p.out_f32) reinterpret_cast<float*>(p.c)[off] = v;
      else st1<T>(reinterpret_cast<T*>(p.c) + off, v);
    }
  }
}

// Spatially tiled narrow-N kernel (the fast path for N <= 8).  One thread owns one
// GEMM-grid point (all 4 sub-pixel phases for the ConvT geometry); the block stages
// the input halo region for one 128-byte channel chunk in LDS (pixel stride 144 B:
// 16 lanes at consecutive pixels hit 16 distinct bank slots), so each input element
// is read from L2/HBM once per tile instead of once per output.  Weights are indexed
// only by loop counters (wave-uniform -> scalar / broadcast loads).
//   GEOM 0: ConvT-s2 phased geometry (taps in {0,1}^2 per phase, 3x3 neighbourhood),
//           TY x TX = 16 x 16 grid points, 256 threads.
//   GEOM 1: Conv k4 s1 (16 taps, 4x4 neighbourhood), 8 x 8 points, 64 threads.
template <typename T, int GEOM, int NMAX>
__global__ void narrow_tiled_kernel(const ConvParams p, int tiles_x, int tiles_per_img) {
  constexpr int TY = GEOM == 0 ? 16 : 8, TX = GEOM == 0 ? 16 : 8;
  constexpr int NT = TY * TX;
  constexpr int HALO = GEOM == 0 ? 2 : 3;  // region = (TY+HALO) x (TX+HALO), origin (-1,-1)
  constexpr int RY = TY + HALO, RX = TX + HALO;
  constexpr int VEC = 16 / sizeof(T);
  constexpr int CC = 128 / sizeof(T);  // channels per chunk
  constexpr int PSTR = 144;            // LDS bytes per staged pixel
  constexpr int NPH = GEOM == 0 ? 4 : 1;
  __shared__ __attribute__((aligned(16))) char tile[RY * RX * PSTR];

  const int tid = threadIdx.x;
  const int img = blockIdx.x / tiles_per_img, tix = blockIdx.x % tiles_per_img;
  const int y0 = (tix / tiles_x) * TY, x0 = (tix % tiles_x) * TX;
  const int ty = tid / TX, tx = tid % TX;
  const int gy = y0 + ty, gx = x0 + tx;
  const T* A = reinterpret_cast<const T*>(p.a) + (long long)img * p.a_bs + p.a_co;
  const T* Wt = reinterpret_cast<const T*>(p.b);
  const int taps = GEOM == 0 ? 4 : 16;

  float acc[NPH][NMAX];
#pragma unroll
  for (int q = 0; q < NPH; ++q)
#pragma unroll
    for (int n = 0; n < NMAX; ++n) acc[q][n] = 0.f;

  for (int c0 = 0; c0 < p.cin; c0 += CC) {
    // ---- stage the halo region (in-bounds pixels get the producer prologue)
    for (int i = tid; i < RY * RX * 8; i += NT) {
      const int pix = i >> 3, part = i & 7;
      const int ry = pix / RX, rx = pix - ry * RX;
      const int iy = y0 - 1 + ry, ix = x0 - 1 + rx;
      uint4 v = make_uint4(0, 0, 0, 0);
      if ((unsigned)iy < (unsigned)p.IH && (unsigned)ix < (unsigned)p.IW) {
        const int ci = c0 + part * VEC;
        v = *reinterpret_cast<const uint4*>(A + (long long)iy * p.a_rs + (long long)ix * p.a_ps + ci);
        if (p.sc || p.pro_act) v = prologue16<T>(v, p.sc, p.sh, ci, p.pro_act, p.slope);
      }
      *reinterpret_cast<uint4*>(tile + pix * PSTR + part * 16) = v;
    }
    __syncthreads();
    // ---- accumulate
#pragma unroll
    for (int part = 0; part < 8; ++part) {
      const int cbase = c0 + part * VEC;
      if constexpr (GEOM == 0) {
#pragma unroll
        for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
          for (int dx = -1; dx <= 1; ++dx) {
            const uint4 v = *reinterpret_cast<const uint4*>(tile + ((ty + 1 + dy) * RX + (tx + 1 + dx)) * PSTR + part * 16);
            float f[VEC];
            if constexpr (sizeof(T) == 4) {
              f[0] = __uint_as_float(v.x); f[1] = __uint_as_float(v.y); f[2] = __uint_as_float(v.z); f[3] = __uint_as_float(v.w);
            } else {
              const unsigned w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
              for (int q = 0; q < 4; ++q) { f[2 * q] = __uint_as_float(w[q] << 16); f[2 * q + 1] = __uint_as_float(w[q] & 0xffff0000u); }
            }
#pragma unroll
            for (int ph = 0; ph < 2; ++ph)
#pragma unroll
              for (int pw = 0; pw < 2; ++pw) {
                const int th = ph - dy, tw = pw - dx;  // out(2y+ph) += in(y + ph - th) * w[tap th]
                if (th < 0 || th > 1 || tw < 0 || tw > 1) continue;
                const int phase = ph * 2 + pw, tap = th * 2 + tw;
#pragma unroll
                for (int n = 0; n < NMAX; ++n) {
                  if (n >= p.N) break;
                  const T* wr = Wt + p.b_phase_stride * phase + ((long long)n * taps + tap) * p.cin + cbase;
                  float s = acc[phase][n];
#pragma unroll
                  for (int e = 0; e < VEC; ++e) s = fmaf(f[e], ld1<T>(wr + e), s);
                  acc[phase][n] = s;
                }
              }
          }
      } else {
#pragma unroll
        for (int kh = 0; kh < 4; ++kh)
#pragma unroll
          for (int kw = 0; kw < 4; ++kw) {
            const uint4 v = *reinterpret_cast<const uint4*>(tile + ((ty + kh) * RX + (tx + kw)) * PSTR + part * 16);
            float f[VEC];
            if constexpr (sizeof(T) == 4) {
              f[0] = __uint_as_float(v.x); f[1] = __uint_as_float(v.y); f[2] = __uint_as_float(v.z); f[3] = __uint_as_float(v.w);
            } else {
              const unsigned w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
              for (int q = 0; q < 4; ++q) { f[2 * q] = __uint_as_float(w[q] << 16); f[2 * q + 1] = __uint_as_float(w[q] & 0xffff0000u); }
            }
            const int tap = kh * 4 + kw;
#pragma unroll
            for (int n = 0; n < NMAX; ++n) {
              if (n >= p.N) break;
              const T* wr = Wt + ((long long)n * taps + tap) * p.cin + cbase;
              float s = acc[0][n];
#pragma unroll
              for (int e = 0; e < VEC; ++e) s = fmaf(f[e], ld1<T>(wr + e), s);
              acc[0][n] = s;
            }
          }
      }
    }
    __syncthreads();
  }
  if (gy >= p.GH || gx >= p.GW) return;
#pragma unroll
  for (int q = 0; q < NPH; ++q) {
    const int oy = gy * p.os + p.oy0[q], ox = gx * p.os + p.ox0[q];
    const long long base = (long long)img * p.c_bs + (long long)oy * p.c_rs + (long long)ox * p.c_ps;
#pragma unroll
    for (int n = 0; n < NMAX; ++n) {
      if (n >= p.N) break;
      float v = acc[q][n];
      if (p.bias) v += p.bias[n];
      if (p.tanh_) v = tanhf(v);
      const long long off = base + (long long)(p.c_co + n) * p.c_cs;
      if (p.out_f32) reinterpret_cast<float*>(p.c)[off] = v;
      else st1<T>(reinterpret_cast<T*>(p.c) + off, v);
    }
  }
}

template <typename T>
static bool launch_narrow_tiled(int kind, int B, ConvParams& p, hipStream_t st) {
  const int CC = 128 / sizeof(T);
  if (p.cin % CC != 0) return false;
  const int geom = kind == STC_CONVT_S2 ? 0 : (kind == STC_CONV_S1 ? 1 : -1);
  if (geom < 0) return false;
  const int TY = geom == 0 ? 16 : 8, TX = geom == 0 ? 16 : 8;
  const int tiles_x = cdiv(p.GW, TX), tiles_y = cdiv(p.GH, TY);
  const int tpi = tiles_x * tiles_y;
  dim3 grid((unsigned)(B * tpi));
  const bool n4 = p.N <= 4;
  main_timer_begin(st);
  if (geom == 0) {
    if (n4) hipLaunchKernelGGL((narrow_tiled_kernel<T, 0, 4>), grid, dim3(256), 0, st, p, tiles_x, tpi);
    else hipLaunchKernelGGL((narrow_tiled_kernel<T, 0, 8>), grid, dim3(256), 0, st, p, tiles_x, tpi);
  } else {
    if (n4) hipLaunchKernelGGL((narrow_tiled_kernel<T, 1, 4>), grid, dim3(64), 0, st, p, tiles_x, tpi);
    else hipLaunchKernelGGL((narrow_tiled_kernel<T, 1, 8>), grid, dim3(64), 0, st, p, tiles_x, tpi);
  }
  main_timer_end(st);
  return true;
}

// ------------------------------------------------------------------------- host
static int ilog2_exact(int v) {
  int l = 0;
  while ((1 << l) < v) ++l;
  return (1 << l) == v ? l : -1;
}

struct Plan {
  int BM, BN, ksplit, kchunk, mtiles, ntiles;
};

static Plan plan_for(int dtype, int M, int N, int K, int nphase) {
  const int BK = dtype == STC_F32 ? 32 : 64;
  Plan pl{};
  if (N <= 32) { pl.BM = 128; pl.BN = 32; }
  else if (N <= 64) { pl.BM = 128; pl.BN = 64; }
  else { pl.BM = 128; pl.BN = 128; }
  if (M <= 64 && N >= 128) { pl.BM = 32; pl.BN = 128; }
  else if (M <= 512 && N >= 64) { pl.BM = 64; pl.BN = 64; }
  pl.mtiles = cdiv(M, pl.BM);
  pl.ntiles = cdiv(N, pl.BN);
  const long long tiles = (long long)pl.mtiles * pl.ntiles * nphase;
  const int ksteps = cdiv(K, BK);
  int ks = 1;
  // split K until the grid covers the chip (~2 waves of 256 CUs), keeping >= 4 K-steps per split
  while (tiles * ks < 512 && ks * 2 <= 64 && ksteps / (ks * 2) >= 4) ks *= 2;
  pl.ksplit = ks;
  pl.kchunk = cdiv(ksteps, ks) * BK;
  pl.ksplit = cdiv(K, pl.kchunk);
  return pl;
}

static size_t lds_bytes(int BM, int BN) { return 2 * (size_t)(BM + BN) * LDS_ROW + BM * 8; }

template <typename T>
static int launch_igemm(const Plan& pl, ConvParams& p, hipStream_t st) {
  dim3 grid(pl.mtiles * pl.ntiles, 1, p.nphase * pl.ksplit);
  const size_t lds = lds_bytes(pl.BM, pl.BN);
  const bool pro = p.sc != nullptr || p.pro_act != 0;
  main_timer_begin(st);
#define STC_L(BM_, BN_, WM_, WN_)                                                                  \
  if (pl.BM == BM_ && pl.BN == BN_) {                                                              \
    if (pro) hipLaunchKernelGGL((igemm_kernel<T, BM_, BN_, WM_, WN_, true>), grid, dim3(256), lds, st, p); \
    else hipLaunchKernelGGL((igemm_kernel<T, BM_, BN_, WM_, WN_, false>), grid, dim3(256), lds, st, p);    \
  } else
  STC_L(128, 128, 2, 2)
  STC_L(128, 64, 2, 2)
  STC_L(128, 32, 4, 1)
  STC_L(64, 64, 2, 2)
  STC_L(32, 128, 1, 4)
  { return fail(-1, "igemm: no kernel for tile %dx%d", pl.BM, pl.BN); }
#undef STC_L
  main_timer_end(st);
  STC_CHECK_LAUNCH();
  if (p.ws) {
    const long long total = (long long)p.nphase * p.M * p.N;
    const int blocks = (int)std::min<long long>((total + 255) / 256, 4096);
    hipLaunchKernelGGL(splitk_reduce_kernel<T>, dim3(blocks), dim3(256), 0, st, p);
    STC_CHECK_LAUNCH();
  }
  return 0;
}

}  // namespace stc

using namespace stc;

static bool use_smalln(int dtype, int N, int K) {
  const int esz = dtype == STC_F32 ? 4 : 2;
  return N <= 8 && (long long)N * K * esz <= 64 * 1024;
}

namespace stc {
bool bf16_conv_eligible(int kind, int B, const stc_view& x, int Cin, int Cout);
int bf16_conv_query(int kind, int B, int Hg, int Wg, int Cin, int Cout, int out_f32, const int32_t* force,
                    int64_t* ws_bytes, int32_t* stats_chunks, int32_t* plan_out);
int bf16_conv_fwd(int kind, int B, stc_view x, int Cin, const void* w_packed, int Cout, stc_view y,
                  const float* bias, int epi_tanh, int out_f32, float* stats, int stats_chunks,
                  const int32_t* force, void* ws, int64_t ws_bytes, hipStream_t st,
                  const stc_bnb_fuse* bnb = nullptr, float* part2 = nullptr,
                  const stc_view* act2 = nullptr, int act_n = 0, float act_s1 = 0.f, float act_s2 = 0.f,
                  int bnb_act = 0);
bool bf16_conv_act_ok(int kind, int B, const stc_view& x, int Cin, int Cout, const stc_view& y1, const stc_view* y2);
bool bf16_narrow_eligible(int kind, int Cin, int Cout);
int64_t bf16_narrow_workspace(int kind, int B, int GH, int GW, int Cin, int Cout);
int bf16_narrow_fwd(int kind, int B, stc_view x, int Cin, const void* w_packed, int Cout, stc_view y,
                    const float* bias, int epi_tanh, int out_f32, void* ws, int64_t ws_bytes, hipStream_t st,
                    const int32_t* force = nullptr);
}  // namespace stc

// bf16 operands on the LDS-DMA kernel (igemm_bf16.hip) whenever the shape allows (no prologue,
// N >= 16, 16-byte channel alignment); the query mirrors that decision for an NHWC input view.
static bool bf16_path(int dtype, int kind, int Cin, int Cout) {
  if (dtype != STC_BF16) return false;
  const Geometry g = geometry(kind);
  const int taps = g.taps_lg_tw == 2 ? 16 : 4;
  return Cin % 8 == 0 && Cout >= 16 && Cout % 8 == 0 && Cout <= 2048 && !use_smalln(dtype, Cout, taps * Cin);
}

extern "C" int64_t stc_conv_fwd_workspace(int dtype, int kind, int B, int Hg, int Wg, int Cin, int Cout) {
  const Geometry g = geometry(kind);
  const int taps = g.taps_lg_tw == 2 ? 16 : 4;
  const int M = B * Hg * Wg, K = taps * Cin;
  if (use_smalln(dtype, Cout, K))
    return dtype == STC_BF16 && bf16_narrow_eligible(kind, Cin, Cout) ? bf16_narrow_workspace(kind, B, Hg, Wg, Cin, Cout) : 0;
  int64_t ws_new = 0;
  if (bf16_path(dtype, kind, Cin, Cout))  // the prologue form still runs the register-staged kernel: max of both
    bf16_conv_query(kind, B, Hg, Wg, Cin, Cout, 0, nullptr, &ws_new, nullptr, nullptr);
  const Plan pl = plan_for(dtype, M, Cout, K, g.nphase);
  const int64_t ws_old = pl.ksplit <= 1 ? 0 : (int64_t)g.nphase * pl.ksplit * (int64_t)M * Cout * 4;
  return std::max(ws_old, ws_new);
}

// out[0..3] = {BM, BN, ksplit, narrow-N path}; Hg x Wg is the GEMM grid (output grid for
// the conv kinds, input grid for STC_CONVT_S2).
extern "C" int stc_conv_fwd_plan(int dtype, int kind, int B, int Hg, int Wg, int Cin, int Cout, int32_t* out) {
  STC_REQUIRE(kind >= 0 && kind <= 3 && out, "stc_conv_fwd_plan: bad arguments");
  const Geometry g = geometry(kind);
  const int taps = g.taps_lg_tw == 2 ? 16 : 4;
  const int M = B * Hg * Wg, K = taps * Cin;
  if (use_smalln(dtype, Cout, K)) {
    out[0] = 1; out[1] = Cout; out[2] = 1; out[3] = 1;
    return 0;
  }
  if (bf16_path(dtype, kind, Cin, Cout)) {
    int32_t po[5];
    bf16_conv_query(kind, B, Hg, Wg, Cin, Cout, 0, nullptr, nullptr, nullptr, po);
    for (int i = 0; i < 4; ++i) out[i] = po[i];
    return 0;
  }
  const Plan pl = plan_for(dtype, M, Cout, K, g.nphase);
  out[0] = pl.BM; out[1] = pl.BN; out[2] = pl.ksplit; out[3] = 0;
  return 0;
}

// Forward conv with fused BatchNorm output statistics and an optional forced plan
// {tile config, ksplit} (bf16 LDS-DMA kernel only; tuning / tests).  stats_part: [chunks][Cout][4]
// in stc_chan_stats format (merged by stc_bn_finalize).  plan_out[5] = {BM, BN, ksplit, narrow, cfg}.
extern "C" int stc_conv_fwd_query(int dtype, int kind, int B, int Hg, int Wg, int Cin, int Cout, int out_f32,
                                  const int32_t* force_plan, int64_t* workspace_bytes, int32_t* stats_chunks,
                                  int32_t* plan_out) {
  STC_REQUIRE(kind >= 0 && kind <= 3, "stc_conv_fwd_query: bad kind %d", kind);
  const Geometry g = geometry(kind);
  if (bf16_path(dtype, kind, Cin, Cout))
    return bf16_conv_query(kind, B, Hg, Wg, Cin, Cout, out_f32, force_plan, workspace_bytes, stats_chunks, plan_out);
  const long long P = (long long)B * Hg * Wg * (g.nphase == 4 ? 4 : 1);
  if (workspace_bytes) *workspace_bytes = stc_conv_fwd_workspace(dtype, kind, B, Hg, Wg, Cin, Cout);
  if (stats_chunks) *stats_chunks = stc_chan_stats_chunks(1, 1, (int)std::min<long long>(P, 1 << 30));
  if (plan_out) {
    int32_t o[4];
    stc_conv_fwd_plan(dtype, kind, B, Hg, Wg, Cin, Cout, o);
    for (int i = 0; i < 4; ++i) plan_out[i] = o[i];
    plan_out[4] = -1;
  }
  return 0;
}

extern "C" int stc_conv_fwd_ex(int dtype, int kind, int B, stc_view x, int Cin, const void* w_packed, int Cout,
                               stc_view y, const float* bias, int epi_tanh, int out_f32, float* stats_part,
                               int stats_chunks, const int32_t* force_plan, void* workspace, int64_t workspace_bytes,
                               void* stream) {
  STC_REQUIRE(kind >= 0 && kind <= 3, "stc_conv_fwd_ex: bad kind %d", kind);
  hipStream_t st = (hipStream_t)stream;
  if (bf16_path(dtype, kind, Cin, Cout) && !epi_tanh && bf16_conv_eligible(kind, B, x, Cin, Cout))
    return bf16_conv_fwd(kind, B, x, Cin, w_packed, Cout, y, bias, epi_tanh, out_f32, stats_part, stats_chunks,
                         force_plan, workspace, workspace_bytes, st);
  if (force_plan && stats_part == nullptr && dtype == STC_BF16 && use_smalln(dtype, Cout, 16 * Cin) &&
      bf16_narrow_eligible(kind, Cin, Cout))  // tuning hook: force_plan = {tile rows, 16-column blocks}
    return bf16_narrow_fwd(kind, B, x, Cin, w_packed, Cout, y, bias, epi_tanh, out_f32, workspace, workspace_bytes, st,
                           force_plan);
  const int rc = stc_conv_fwd(dtype, kind, B, x, Cin, nullptr, nullptr, 0, 0.f, w_packed, Cout, y, bias, epi_tanh,
                              out_f32, workspace, workspace_bytes, stream);
  if (rc != 0 || stats_part == nullptr) return rc;
  STC_REQUIRE(!out_f32 || dtype == STC_F32, "stc_conv_fwd_ex: stats of a non-activation output");
  return stc_chan_stats(dtype, B, y, Cout, stats_part, stats_chunks, stream);
}

// conv + BatchNorm (train mode) + activation as one call: stc_conv_fwd_ex with the batch statistics, stc_bn_finalize,
// stc_bn_apply -- the three launches of a BN layer's forward, enqueued by one host call (the train step makes ~50
// of them; each separate call costs host time the GPU then waits for).  fws = [stats partials nchunks*Cout*4 |
// mean | rstd | scale | shift] (Cout each); y1.p == NULL: no apply (the caller only needs the statistics).
extern "C" int stc_conv_bn_fwd(int dtype, int kind, int B, stc_view x, int Cin, const void* w_packed, int Cout,
                               stc_view y, float* fws, int nchunks, const float* gamma, const float* beta,
                               float* running_mean, float* running_var, int64_t* num_batches_tracked, float momentum,
                               float eps, stc_view apply_x, stc_view y1, float slope1, stc_view y2, float slope2,
                               void* workspace, int64_t workspace_bytes, void* stream) {
  STC_REQUIRE(fws && nchunks > 0 && gamma && beta, "stc_conv_bn_fwd: statistics workspace and BN affine required");
  int rc = stc_conv_fwd_ex(dtype, kind, B, x, Cin, w_packed, Cout, y, nullptr, 0, 0, fws, nchunks, nullptr, workspace,
                           workspace_bytes, stream);
  if (rc) return rc;
  float* tab = fws + (int64_t)nchunks * Cout * 4;
  rc = stc_bn_finalize(fws, nchunks, Cout, gamma, beta, running_mean, running_var, num_batches_tracked, momentum, eps,
                       tab, tab + Cout, tab + 2 * Cout, tab + 3 * Cout, stream);
  if (rc || !y1.p) return rc;
  return stc_bn_apply(dtype, B, apply_x, Cout, tab + 2 * Cout, tab + 3 * Cout, y1, slope1, y2, slope2, stream);
}

extern "C" int stc_conv_fwd(int dtype, int kind, int B, stc_view x, int Cin,
                            const float* pro_scale, const float* pro_shift, int pro_act, float pro_slope,
                            const void* w_packed, int Cout, stc_view y,
                            const float* bias, int epi_tanh, int out_f32,
                            void* workspace, int64_t workspace_bytes, void* stream) {
  STC_REQUIRE(dtype == STC_F32 || dtype == STC_BF16, "stc_conv_fwd: bad dtype %d", dtype);
  STC_REQUIRE(kind >= 0 && kind <= 3, "stc_conv_fwd: bad kind %d", kind);
  const int VEC = dtype == STC_F32 ? 4 : 8;
  const int BK = dtype == STC_F32 ? 32 : 64;
  STC_REQUIRE(Cin >= VEC && Cin % VEC == 0, "stc_conv_fwd: Cin=%d must be a multiple of %d", Cin, VEC);
  STC_REQUIRE(x.co % VEC == 0 && x.ps % VEC == 0 && x.cs == 1, "stc_conv_fwd: input view must be NHWC, 16-byte aligned channels");
  const Geometry g = geometry(kind);
  const int taps = g.taps_lg_tw == 2 ? 16 : 4;
  const int K = taps * Cin;
  (void)BK;
  // GEMM grid: conv kinds -> output grid; convT -> input grid
  int GH, GW;
  if (kind == STC_CONVT_S2) { GH = x.H; GW = x.W; }
  else { GH = y.H; GW = y.W; }
  ConvParams p{};
  p.a = (const char*)x.p; p.a_bs = x.bs; p.a_rs = x.rs; p.a_ps = x.ps; p.a_co = x.co;
  p.IH = x.H; p.IW = x.W;
  p.cin = Cin; p.lg_tw = g.taps_lg_tw; p.in_stride = g.in_stride;
  for (int i = 0; i < 4; ++i) { p.offy[i] = g.offy[i]; p.offx[i] = g.offx[i]; }
  p.stepy = g.stepy; p.stepx = g.stepx;
  p.sc = pro_scale; p.sh = pro_shift; p.pro_act = pro_act; p.slope = pro_slope;
  STC_REQUIRE((pro_scale == nullptr) == (pro_shift == nullptr), "stc_conv_fwd: scale/shift must come together");
  p.GH = GH; p.GW = GW; p.M = B * GH * GW; p.N = Cout; p.K = K;
  p.b = (const char*)w_packed;
  p.b_phase_stride = (long long)Cout * K;
  p.c = (char*)y.p; p.c_bs = y.bs; p.c_rs = y.rs; p.c_ps = y.ps; p.c_co = y.co; p.c_cs = y.cs;
  p.os = g.os;
  for (int i = 0; i < 4; ++i) { p.oy0[i] = g.nphase == 4 ? (i >> 1) : 0; p.ox0[i] = g.nphase == 4 ? (i & 1) : 0; }
  p.bias = bias; p.tanh_ = epi_tanh; p.out_f32 = out_f32 || dtype == STC_F32;
  p.nphase = g.nphase;
  if (p.M == 0 || Cout == 0) return 0;
  hipStream_t st0 = (hipStream_t)stream;
  if (use_smalln(dtype, Cout, K)) {
    if (dtype == STC_BF16 && p.sc == nullptr && pro_act == 0 && bf16_narrow_eligible(kind, Cin, Cout))
      return bf16_narrow_fwd(kind, B, x, Cin, w_packed, Cout, y, bias, epi_tanh, out_f32, workspace, workspace_bytes,
                             st0);
    p.mtiles = 1; p.ntiles = 1; p.ksplit = 1; p.kchunk = K;
    const int esz = dtype == STC_F32 ? 4 : 2;
    STC_REQUIRE(K % VEC == 0, "stc_conv_fwd: K=%d", K);
    const bool tiled = dtype == STC_F32 ? launch_narrow_tiled<float>(kind, B, p, st0)
                                        : launch_narrow_tiled<bf16>(kind, B, p, st0);
    if (tiled) {
      STC_CHECK_LAUNCH();
      return 0;
    }
    dim3 grid((unsigned)std::min(cdiv(p.M, 4), 4096), g.nphase);
    const size_t lds = (size_t)Cout * K * esz;
    main_timer_begin(st0);
    if (dtype == STC_F32) hipLaunchKernelGGL(smalln_kernel<float>, grid, dim3(256), lds, st0, p);
    else hipLaunchKernelGGL(smalln_kernel<bf16>, grid, dim3(256), lds, st0, p);
    main_timer_end(st0);
    STC_CHECK_LAUNCH();
    return 0;
  }
  if (dtype == STC_BF16 && p.sc == nullptr && pro_act == 0 && !epi_tanh && bf16_conv_eligible(kind, B, x, Cin, Cout))
    return bf16_conv_fwd(kind, B, x, Cin, w_packed, Cout, y, bias, epi_tanh, out_f32, nullptr, 0, nullptr,
                         workspace, workspace_bytes, st0);
  const Plan pl = plan_for(dtype, p.M, Cout, K, g.nphase);
  p.ksplit = pl.ksplit; p.kchunk = pl.kchunk; p.mtiles = pl.mtiles; p.ntiles = pl.ntiles;
  if (pl.ksplit > 1) {
    const int64_t need = (int64_t)g.nphase * pl.ksplit * (int64_t)p.M * Cout * 4;
    STC_REQUIRE(workspace && workspace_bytes >= need, "stc_conv_fwd: workspace %lld < %lld bytes",
                (long long)workspace_bytes, (long long)need);
    p.ws = (float*)workspace;
  }
  hipStream_t st = (hipStream_t)stream;
  if (dtype == STC_F32) return launch_igemm<float>(pl, p, st);
  return launch_igemm<bf16>(pl, p, st);
}

// ---- input-gradient conv + fused BN-backward reduction
static bool bnb_fused_path(int dtype, int kind, int B, const stc_view& dy, int Cin, int Cout, const stc_view& out) {
  const bool vec = out.cs == 1 && out.co % 8 == 0 && out.ps % 8 == 0 && out.rs % 8 == 0 && out.bs % 8 == 0 &&
                   ((uintptr_t)out.p & 15) == 0;
  return bf16_path(dtype, kind, Cin, Cout) && vec && bf16_conv_eligible(kind, B, dy, Cin, Cout);
}

namespace stc {
int stem_bnb_chunks(int kind, int B, int Hg, int Wg, int Cin, int Cout);
int bf16_bnb_chunks(int kind, int B, const stc_view& x, int Cin, int Cout, const stc_view& y, bool g_other);
}

// the part2 chunk count of stc_conv_bwd_bn for these exact views (the kernel route depends on the layout)
static int bwd_bn_chunks_of(int dtype, int kind, int B, const stc_view& dy, int Cin, int Cout, const stc_view& out,
                            const stc_bnb_fuse& bnb) {
  if (bnb_fused_path(dtype, kind, B, dy, Cin, Cout, out))
    return bf16_bnb_chunks(kind, B, dy, Cin, Cout, out, bnb.g_other.p != nullptr);
  return stc_chan_stats_chunks(B, bnb.x.H, bnb.x.W);
}

extern "C" int stc_conv_bwd_bn_chunks_ex(int dtype, int kind, int B, stc_view dy, int Cin, int Cout, stc_view out,
                                         const stc_bnb_fuse* bnb) {
  if (!bnb || kind < 0 || kind > 3) return fail(-1, "stc_conv_bwd_bn_chunks_ex: bad arguments"), 0;
  return bwd_bn_chunks_of(dtype, kind, B, dy, Cin, Cout, out, *bnb);
}

// (shape-only form: assumes dense 16-byte NHWC views at channel offset 0 and no second gradient for the 31 x 31
// logits-layer input gradient -- stc_conv_bwd_bn_chunks_ex answers for the actual views)
extern "C" int stc_conv_bwd_bn_chunks(int dtype, int kind, int B, int Hg, int Wg, int Cin, int Cout, int xH, int xW) {
  if (bf16_path(dtype, kind, Cin, Cout)) {
    if (const int sn = stem_bnb_chunks(kind, B, Hg, Wg, Cin, Cout)) return sn;  // (the streaming Cin = 8 kernel)
    int32_t nch = 0;
    bf16_conv_query(kind, B, Hg, Wg, Cin, Cout, 0, nullptr, nullptr, &nch, nullptr);
    return nch;  // (NHWC 16-byte aligned views assumed: the fused path)
  }
  return stc_chan_stats_chunks(B, xH, xW);
}

extern "C" int stc_conv_bwd_bn(int dtype, int kind, int B, stc_view dy, int Cin, const void* w_packed, int Cout,
                               stc_view out, const stc_bnb_fuse* bnb, float* part2, int nchunks, void* workspace,
                               int64_t workspace_bytes, void* stream) {
  STC_REQUIRE(bnb && part2, "stc_conv_bwd_bn: bnb and part2 required");
  hipStream_t st = (hipStream_t)stream;
  if (bnb_fused_path(dtype, kind, B, dy, Cin, Cout, out)) {
    const int need = bwd_bn_chunks_of(dtype, kind, B, dy, Cin, Cout, out, *bnb);
    STC_REQUIRE(nchunks == need, "stc_conv_bwd_bn: %d chunks != %d (use stc_conv_bwd_bn_chunks_ex)", nchunks, need);
    return bf16_conv_fwd(kind, B, dy, Cin, w_packed, Cout, out, nullptr, 0, 0, nullptr, need, nullptr, workspace,
                         workspace_bytes, st, bnb, part2);
  }
  int rc = stc_conv_fwd(dtype, kind, B, dy, Cin, nullptr, nullptr, 0, 0.f, w_packed, Cout, out, nullptr, 0, 0,
                        workspace, workspace_bytes, stream);
  if (rc) return rc;
  stc_view g1 = out;  // this conv's output, at the BN channels, over the BN extent
  g1.co += bnb->ch_off;
  g1.H = bnb->x.H;
  g1.W = bnb->x.W;
  const int need = stc_chan_stats_chunks(B, bnb->x.H, bnb->x.W);
  STC_REQUIRE(nchunks == need, "stc_conv_bwd_bn: %d chunks != %d (use stc_conv_bwd_bn_chunks_ex)", nchunks, need);
  return stc_bn_bwd_reduce(dtype, B, bnb->x, bnb->C, bnb->scale, bnb->shift, bnb->mean, bnb->rstd, g1, bnb->slope_self,
                           bnb->g_other, bnb->slope_other, part2, need, stream);
}

// stc_conv_bwd_bn followed by its stc_bn_bwd_apply (the conv output at the BN channels over the BN extent as the
// first gradient): a BN layer's whole input-gradient step from one host call
extern "C" int stc_conv_bwd_bn_apply(int dtype, int kind, int B, stc_view dy, int Cin, const void* w_packed, int Cout,
                                     stc_view out, const stc_bnb_fuse* bnb, float* part2, int nchunks,
                                     const float* gamma, stc_view dx, float* dgamma, float* dbeta, void* workspace,
                                     int64_t workspace_bytes, void* stream) {
  int rc = stc_conv_bwd_bn(dtype, kind, B, dy, Cin, w_packed, Cout, out, bnb, part2, nchunks, workspace,
                           workspace_bytes, stream);
  if (rc) return rc;
  stc_view g1 = out;
  g1.co += bnb->ch_off;
  g1.H = bnb->x.H;
  g1.W = bnb->x.W;
  return stc_bn_bwd_apply(dtype, B, bnb->x, bnb->C, bnb->scale, bnb->shift, bnb->mean, bnb->rstd, gamma, g1,
                          bnb->slope_self, bnb->g_other, bnb->slope_other, part2, nchunks, dx, dgamma, dbeta, stream);
}

// ---- input-gradient conv + activation backward (layers without BatchNorm)
namespace stc {
bool bf16_conv_bwd_act_ok(int kind, int B, const stc_view& dy, int Cin, int Cout, const stc_view& out, const stc_view& x,
                          const stc_view* g_other);
}  // namespace stc
extern "C" int stc_conv_bwd_act_ok(int dtype, int kind, int B, stc_view dy, int Cin, int Cout, stc_view out, stc_view x,
                                   stc_view g_other) {
  if (kind < 0 || kind > 3 || !bf16_path(dtype, kind, Cin, Cout)) return 0;
  return bf16_conv_bwd_act_ok(kind, B, dy, Cin, Cout, out, x, &g_other) ? 1 : 0;
}

extern "C" int stc_conv_bwd_act(int dtype, int kind, int B, stc_view dy, int Cin, const void* w_packed, int Cout,
                                stc_view out, stc_view x, float slope_self, stc_view g_other, float slope_other,
                                void* stream) {
  STC_REQUIRE(stc_conv_bwd_act_ok(dtype, kind, B, dy, Cin, Cout, out, x, g_other),
              "stc_conv_bwd_act: no fused activation backward for this shape / view (check stc_conv_bwd_act_ok)");
  stc_bnb_fuse f{};
  f.x = x;
  f.g_other = g_other;
  f.slope_self = slope_self;
  f.slope_other = slope_other;
  f.C = Cout;
  f.ch_off = 0;
  return bf16_conv_fwd(kind, B, dy, Cin, w_packed, Cout, out, nullptr, 0, 0, nullptr, 0, nullptr, nullptr, 0,
                       (hipStream_t)stream, &f, nullptr, nullptr, 0, 0.f, 0.f, 1);
}

// ---- conv + activation epilogue (layers without BatchNorm)
extern "C" int stc_conv_fwd_act_ok(int dtype, int kind, int B, stc_view x, int Cin, int Cout, stc_view y1, stc_view y2) {
  if (kind < 0 || kind > 3 || !bf16_path(dtype, kind, Cin, Cout)) return 0;
  return bf16_conv_act_ok(kind, B, x, Cin, Cout, y1, y2.p ? &y2 : nullptr) ? 1 : 0;
}

extern "C" int stc_conv_fwd_act(int dtype, int kind, int B, stc_view x, int Cin, const void* w_packed, int Cout,
                                stc_view y1, float slope1, stc_view y2, float slope2, const float* bias,
                                void* workspace, int64_t workspace_bytes, void* stream) {
  STC_REQUIRE(stc_conv_fwd_act_ok(dtype, kind, B, x, Cin, Cout, y1, y2),
              "stc_conv_fwd_act: no activation epilogue for this shape (check stc_conv_fwd_act_ok)");
  return bf16_conv_fwd(kind, B, x, Cin, w_packed, Cout, y1, bias, 0, 0, nullptr, 0, nullptr, workspace, workspace_bytes,
                       (hipStream_t)stream, nullptr, nullptr, &y2, y2.p ? 2 : 1, slope1, slope2);
}
