// The U-Net's innermost levels (1x1 - 8x8 grids) as ONE launch per layer (gfx950, bf16 MFMA).
//
// At bs = 32 these layers -- STCGAN/networks.py:104-105 (down convs of the three innermost blocks) and :119-121,
// :126-128 (their up ConvTs) -- have 32 - 512 GEMM rows per phase against 8.4 - 16.8 MB of weights: the time is
// latency and weight streaming, not MFMA work.  The im2col path ran each as four launches (the GEMM, a split-K
// reduction, the BatchNorm finalize, the BatchNorm + activation pass); here one launch does all of it:
//
//   * A operand: register-staged from the RAW (pre-BatchNorm) output of the previous layer, BatchNorm affine +
//     activation applied in registers as the tile is staged (these activations are <= 1 M elements, so the
//     transform costs nothing), up to two sources (the U-Net concat [skip | up] of a ConvT's input);
//   * the BatchNorm table of each source is merged in the prologue from the producer's per-tile statistics
//     partials ({n, S1, S2, shift} chunks, the stc_bn_finalize format), in fp64 and in a fixed order, for the
//     channels the block's K range reads -- every block that reads a channel derives bit-identical values, and
//     a designated block per channel writes the mean / rstd / scale / shift tables (for the backward) and the
//     running statistics (no grid-wide hand-off: the table is a pure function of the partials);
//   * split-K without a second launch: every K-slice block stores its fp32 tile (accumulator order), takes a
//     ticket on its tile (agent-scope release / acquire, cdna_hip_programming.md Guideline 16 counter form);
//     the block drawing the last ticket sums the slices in split order (deterministic for any arrival order),
//     writes the bf16 output through LDS as 16-byte NHWC rows and the tile's BatchNorm statistics partial
//     (count, mean, M2 from the fp32 sums), and resets the ticket for the next launch;
//   * taps that read only padding for every row of the launch (1x1 grids: 4 of 16 conv taps, 1 of 4 ConvT taps
//     per phase) are dropped from K on the host (their weights are never read).
//
// v_mfma_f32_16x16x32_bf16, 4 waves (2 x 2), K-steps of 64 (one tap, 64 channels of one source), LDS double
// buffer, A and B both register-staged (one uniform vmcnt discipline; the weights are read once per block).
#include <type_traits>

#include "igemm_bf16.hpp"

namespace stc {

struct DeepSrc {
  const bf16* p;
  long long bs;
  int rs, ps, co;
  int nc;               // K channels taken from this source
  const float* part;    // statistics partials [nch][nc][4] (null: table / identity)
  int nch;
  const float* scale;   // ready table (part == null); null with part == null: identity
  const float* shift;
  const float* gamma;
  const float* beta;
  float eps, momentum, slope;
  int mode;             // 0 pass-through, 1 affine + activation
  float* mean_o; float* rstd_o; float* scale_o; float* shift_o;  // designated outputs (null: none)
  float* rmean; float* rvar; long long* nbt;
};

struct DeepParams {
  DeepSrc src[2];
  int nsrc, convt;
  int IH, IW;               // A extent (both sources)
  int GH, GW, M;            // GEMM grid (conv: output, ConvT: input), rows per phase
  int N, Cin, ntaps;        // K = ntaps * Cin
  unsigned long long tapl[4];  // per phase: packed tap index of K-tap t in bits [4t, 4t + 4)
  const bf16* w;
  int w_taps;               // taps per phase in the packed layout (16 / 4)
  long long w_phase_stride; // elements
  bf16* out;
  long long o_bs;
  int o_rs, o_ps, o_co;
  float* slab;              // [tiles][ksplit][BM * BN]
  unsigned* tickets;        // [tiles]
  float* stats;             // [nphase * mtiles][N][4] or null
  int nphase, mtiles, ntiles, ksplit, kps;  // kps: K-steps (64) per split
  float inv_ghw, inv_gw;
};

// BatchNorm merge of one channel from {n, S1, S2, shift} partials (stc_bn_finalize's two fp64 passes, serial order)
__device__ __forceinline__ void deep_merge(const DeepSrc& s, int c, double& N, double& mu, double& M2) {
  double n = 0, sm = 0;
  for (int k = 0; k < s.nch; ++k) {
    const float4 pp = *reinterpret_cast<const float4*>(s.part + ((long long)k * s.nc + c) * 4);
    if (pp.x <= 0.f) continue;
    n += pp.x;
    sm += (double)pp.x * pp.w + (double)pp.y;
  }
  mu = n > 0 ? sm / n : 0.0;
  double m2 = 0;
  for (int k = 0; k < s.nch; ++k) {
    const float4 pp = *reinterpret_cast<const float4*>(s.part + ((long long)k * s.nc + c) * 4);
    if (pp.x <= 0.f) continue;
    const double nb = pp.x, s1 = pp.y, r = s1 / nb;
    double q = (double)pp.z - s1 * r;
    if (q < 0) q = 0;
    const double d = (double)pp.w + r - mu;
    m2 += q + nb * d * d;
  }
  N = n;
  M2 = m2;
}

// (scale, shift) of channel c of source s: the same arithmetic as bn_finalize_store
__device__ __forceinline__ void deep_table(const DeepSrc& s, int c, float& sc, float& sh) {
  if (s.part) {
    double N, mu, M2;
    deep_merge(s, c, N, mu, M2);
    const double var = N > 0 ? M2 / N : 0.0;
    const float rs = (float)(1.0 / sqrt(var + (double)s.eps));
    const float g = s.gamma ? s.gamma[c] : 1.f, bt = s.beta ? s.beta[c] : 0.f;
    sc = g * rs;
    sh = bt - (float)mu * sc;
  } else if (s.scale) {
    sc = s.scale[c];
    sh = s.shift[c];
  } else {
    sc = 1.f;
    sh = 0.f;
  }
}

template <int BM, int BN>
__global__ void __launch_bounds__(256) deep_conv_kernel(const DeepParams p) {
  constexpr int WM = 2, WN = 2;
  constexpr int TM = BM / WM, TN = BN / WN, FM = TM / 16, FN = TN / 16;
  constexpr int AC = BM * 8 / 256, BC = BN * 8 / 256;  // 16-byte chunks per thread per K-step (A / B)
  constexpr int STAGE = (BM + BN) * 128;
  static_assert(FM >= 1 && FN >= 1 && AC >= 1 && BC >= 1, "tile");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // LDS: [stage 0][stage 1][table: scale[1024] shift[1024]] ; the epilogue reuses the stages
  float* tsc = reinterpret_cast<float*>(smem + 2 * STAGE);
  float* tsh = tsc + 1024;

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  // XCD-aware: a tile's K slices on one XCD (its reducer then reads same-XCD slabs), consecutive tiles together
  const int nwg = p.nphase * p.mtiles * p.ntiles * p.ksplit;
  int bid = blockIdx.x;
  {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int split = bid % p.ksplit;
  const int tile = bid / p.ksplit;
  const int nt = tile % p.ntiles;
  const int mt = (tile / p.ntiles) % p.mtiles;
  const int ph = tile / (p.ntiles * p.mtiles);
  const int py = ph >> 1, px = ph & 1;
  const int m0 = mt * BM, n0 = nt * BN;
  const int cpt = p.Cin / 64;  // K-steps per tap
  const int nks = p.ntaps * cpt;
  const int ks0 = split * p.kps, ks1 = min(nks, ks0 + p.kps);

  // ---- designated finalize outputs: block b owns channels [b * nc / nwg, (b + 1) * nc / nwg) of each source
  auto designated = [&](const DeepSrc& s) {
    if (!s.mean_o) return;
    const int c0 = (int)((long long)blockIdx.x * s.nc / nwg), c1 = (int)((long long)(blockIdx.x + 1) * s.nc / nwg);
    for (int c = c0 + tid; c < c1; c += 256) {
      double N, mu, M2;
      deep_merge(s, c, N, mu, M2);
      bn_finalize_store(c, N, mu, M2, s.gamma, s.beta, s.rmean, s.rvar, nullptr, s.momentum, s.eps, s.mean_o, s.rstd_o,
                        s.scale_o, s.shift_o);
    }
    if (blockIdx.x == 0 && tid == 0 && s.nbt) s.nbt[0] += 1;
  };
  designated(p.src[0]);
  if (p.nsrc == 2) designated(p.src[1]);

  // ---- prologue tables of the channels this block's K range reads (LDS, indexed by the K channel)
  {
    const int a0 = ks0 % cpt, len = ks1 - ks0;
    for (int kc = tid; kc < p.Cin; kc += 256) {
      // K channel kc is read when some K-step in [ks0, ks1) has channel block kc / 64
      if (((kc >> 6) - a0 + cpt) % cpt >= len) continue;
      float sc, sh;
      if (p.nsrc == 2 && kc >= p.src[0].nc) {
        if (p.src[1].mode == 0) continue;
        deep_table(p.src[1], kc - p.src[0].nc, sc, sh);
      } else {
        if (p.src[0].mode == 0) continue;
        deep_table(p.src[0], kc, sc, sh);
      }
      tsc[kc] = sc;
      tsh[kc] = sh;
    }
  }

  // ---- per-thread A rows (fixed over the K loop): GEMM row -> (image, grid y, grid x)
  int a_row[AC], a_b[AC], a_gy[AC], a_gx[AC], a_cj[AC];
  bool a_in[AC], a_pad[AC];
#pragma unroll
  for (int u = 0; u < AC; ++u) {
    const int ch = tid + u * 256;
    a_row[u] = ch >> 3;
    a_cj[u] = ch & 7;
    const int m = m0 + a_row[u];
    a_in[u] = m < p.M;
    const int mm = a_in[u] ? m : 0;
    const int GHW = p.GH * p.GW;
    a_b[u] = fast_div(mm, GHW, p.inv_ghw);
    const int rem = mm - a_b[u] * GHW;
    a_gy[u] = fast_div(rem, p.GW, p.inv_gw);
    a_gx[u] = rem - a_gy[u] * p.GW;
  }
  int b_row[BC], b_cj[BC];
#pragma unroll
  for (int u = 0; u < BC; ++u) {
    const int ch = tid + u * 256;
    b_row[u] = ch >> 3;
    b_cj[u] = ch & 7;
  }
  const bf16* wph = p.w + (long long)ph * p.w_phase_stride;

  // register ring: NS K-steps of A / B chunks in flight (one Regs per step, held by value: compile-time slots)
  constexpr int NS = (AC + BC) <= 4 ? 3 : 2;
  struct Regs {
    uint4 a[AC], b[BC];
    bool pad[AC];
  };
  const unsigned long long tapl = ph == 0 ? p.tapl[0] : (ph == 1 ? p.tapl[1] : (ph == 2 ? p.tapl[2] : p.tapl[3]));
  auto load = [&](int ks) {
    Regs r;
    const int ti = ks / cpt, cb = (ks - ti * cpt) * 64;
    const int tap = (int)((tapl >> (4 * ti)) & 15u);
    int dy, dx;
    if (p.convt) { dy = py - (tap >> 1); dx = px - (tap & 1); }
    else { dy = (tap >> 2) - 1; dx = (tap & 3) - 1; }
    // (source fields by a select, not a dynamic index into the parameter struct: no private copy of it)
    const bool s1 = p.nsrc == 2 && cb >= p.src[0].nc;
    const bf16* sp = s1 ? p.src[1].p : p.src[0].p;
    const long long sbs = s1 ? p.src[1].bs : p.src[0].bs;
    const int srs = s1 ? p.src[1].rs : p.src[0].rs, sps = s1 ? p.src[1].ps : p.src[0].ps;
    const int c = (s1 ? p.src[1].co : p.src[0].co) + cb - (s1 ? p.src[0].nc : 0);
#pragma unroll
    for (int u = 0; u < AC; ++u) {
      const int iy = p.convt ? a_gy[u] + dy : 2 * a_gy[u] + dy, ix = p.convt ? a_gx[u] + dx : 2 * a_gx[u] + dx;
      const bool ok = a_in[u] && iy >= 0 && iy < p.IH && ix >= 0 && ix < p.IW;
      const int iyc = ok ? iy : 0, ixc = ok ? ix : 0;
      // (clamped in-bounds address; the padding is zeroed when the chunk is staged -- a select on the loaded value
      // here would wait for the load)
      r.a[u] = *reinterpret_cast<const uint4*>(sp + (long long)a_b[u] * sbs + (long long)iyc * srs +
                                               (long long)ixc * sps + c + 8 * a_cj[u]);
      r.pad[u] = !ok;  // (padding: zero after the activation, not act(affine(0)))
    }
#pragma unroll
    for (int u = 0; u < BC; ++u) {
      const int n = min(n0 + b_row[u], p.N - 1);  // (rows past N: any row; their columns are not stored)
      r.b[u] = *reinterpret_cast<const uint4*>(wph + ((long long)n * p.w_taps + tap) * p.Cin + cb + 8 * b_cj[u]);
    }
    return r;
  };
  auto stage_store = [&](int ks, const Regs r, char* st) {
    const int cb = (ks % cpt) * 64;
    const bool s1 = p.nsrc == 2 && cb >= p.src[0].nc;
    const int mode = s1 ? p.src[1].mode : p.src[0].mode;
    const float slope = s1 ? p.src[1].slope : p.src[0].slope;
#pragma unroll
    for (int u = 0; u < AC; ++u) {
      uint4 v = r.pad[u] ? make_uint4(0u, 0u, 0u, 0u) : r.a[u];
      if (mode && !r.pad[u]) {
        const int kc = cb + 8 * a_cj[u];
        const unsigned w[4] = {v.x, v.y, v.z, v.w};
        unsigned o[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float lo = fmaf(__uint_as_float(w[q] << 16), tsc[kc + 2 * q], tsh[kc + 2 * q]);
          const float hi = fmaf(__uint_as_float(w[q] & 0xffff0000u), tsc[kc + 2 * q + 1], tsh[kc + 2 * q + 1]);
          o[q] = pack_bf16x2(act(lo, slope), act(hi, slope));
        }
        v = make_uint4(o[0], o[1], o[2], o[3]);
      }
      const int row = a_row[u];
      *reinterpret_cast<uint4*>(st + row * 128 + ((a_cj[u] ^ (row & 7)) * 16)) = v;
    }
#pragma unroll
    for (int u = 0; u < BC; ++u) {
      const int row = b_row[u];
      *reinterpret_cast<uint4*>(st + BM * 128 + row * 128 + ((b_cj[u] ^ (row & 7)) * 16)) = r.b[u];
    }
  };

  floatx4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int rl = lane & 15, kq = lane >> 4;
  auto compute = [&](const char* st) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8_t fa[FM], fb[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int row = wm * TM + 16 * i + rl;
        fa[i] = *reinterpret_cast<const bf16x8_t*>(st + row * 128 + (((4 * kk + kq) ^ (row & 7)) * 16));
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int row = wn * TN + 16 * j + rl;
        fb[j] = *reinterpret_cast<const bf16x8_t*>(st + BM * 128 + row * 128 + (((4 * kk + kq) ^ (row & 7)) * 16));
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
  };

  __syncthreads();  // (the prologue table)
  if (ks0 < ks1) {
    // (loads of steps past ks1 are clamped to the last step: harmless re-reads, no branch around a load)
    Regs R0 = load(ks0), R1 = load(min(ks0 + 1, ks1 - 1)), R2;
    if constexpr (NS == 3) R2 = load(min(ks0 + 2, ks1 - 1));
    stage_store(ks0, R0, smem);
    __syncthreads();
    // step ks: its registers (slot (ks - ks0) % NS) were staged into LDS buffer (ks - ks0) & 1 by the previous step;
    // refill the slot with step ks + NS, compute step ks, stage step ks + 1 into the other buffer, one barrier
    auto step = [&](int base, auto dc, Regs& mine, const Regs& next) {
      constexpr int d = decltype(dc)::value;
      const int ks = base + d;
      if (ks >= ks1) return;
      mine = load(min(ks + NS, ks1 - 1));
      compute(smem + ((ks - ks0) & 1) * STAGE);
      if (ks + 1 < ks1) stage_store(ks + 1, next, smem + (((ks - ks0) & 1) ^ 1) * STAGE);
      __syncthreads();
    };
    for (int base = ks0; base < ks1; base += NS) {
      if constexpr (NS == 3) {
        step(base, std::integral_constant<int, 0>{}, R0, R1);
        step(base, std::integral_constant<int, 1>{}, R1, R2);
        step(base, std::integral_constant<int, 2>{}, R2, R0);
      } else {
        step(base, std::integral_constant<int, 0>{}, R0, R1);
        step(base, std::integral_constant<int, 1>{}, R1, R0);
      }
    }
  }

  // ---- split-K: slab store, ticket, the last arriver reduces in split order
  unsigned* flag = reinterpret_cast<unsigned*>(tsh + 1024);  // (inside the one LDS array)
  if (p.ksplit > 1) {
    float* my = p.slab + ((long long)tile * p.ksplit + split) * (BM * BN);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        *reinterpret_cast<floatx4*>(my + ((wave * FM + i) * FN + j) * 256 + lane * 4) = acc[i][j];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned old = __hip_atomic_fetch_add(p.tickets + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *flag = old == (unsigned)(p.ksplit - 1) ? 1u : 0u;
    }
    __syncthreads();
    if (*flag == 0u) return;
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(p.tickets + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // (next launch)
    }
    __syncthreads();
    floatx4 sum[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) sum[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    const float* base = p.slab + (long long)tile * p.ksplit * (BM * BN);
    // every slab loaded (the own one too: no per-element register-or-load select), groups of RG slabs in flight,
    // summed in split order
    constexpr int RG = FM * FN <= 4 ? 4 : 2;
    const int S = p.ksplit;
    for (int s0 = 0; s0 < S; s0 += RG) {
      floatx4 v[RG][FM][FN];
#pragma unroll
      for (int g = 0; g < RG; ++g) {
        const int s = min(s0 + g, S - 1);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            v[g][i][j] = *reinterpret_cast<const floatx4*>(base + (long long)s * (BM * BN) +
                                                           ((wave * FM + i) * FN + j) * 256 + lane * 4);
      }
#pragma unroll
      for (int g = 0; g < RG; ++g) {
        if (s0 + g >= S) break;
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) sum[i][j] += v[g][i][j];
      }
    }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = sum[i][j];
  }

  // ---- epilogue: BatchNorm statistics of the tile (fp32 sums), bf16 tile through LDS -> 16-byte NHWC stores
  const int rq = 4 * (lane >> 4), cl = lane & 15;
  const int GHW = p.GH * p.GW;
  if (p.stats) {
    float* red = reinterpret_cast<float*>(smem);  // [WM][BN][4] {S1, S2, shift, rows}
    int rows_w = min(TM, max(0, p.M - (m0 + wm * TM)));
    float sh[FN], s1[FN], s2[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      sh[j] = __shfl(acc[0][j][0], cl, 64);
      s1[j] = 0.f;
      s2[j] = 0.f;
    }
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float d = 16 * i + rq + r < rows_w ? acc[i][j][r] - sh[j] : 0.f;
          s1[j] += d;
          s2[j] = fmaf(d, d, s2[j]);
        }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      s1[j] += __shfl_xor(s1[j], 16, 64);
      s1[j] += __shfl_xor(s1[j], 32, 64);
      s2[j] += __shfl_xor(s2[j], 16, 64);
      s2[j] += __shfl_xor(s2[j], 32, 64);
    }
    if (lane < 16) {
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        float* q = red + (wm * BN + wn * TN + 16 * j + lane) * 4;
        q[0] = s1[j]; q[1] = s2[j]; q[2] = sh[j]; q[3] = (float)max(rows_w, 0);
      }
    }
    __syncthreads();
    for (int c = tid; c < BN; c += 256) {
      const int n = n0 + c;
      if (n >= p.N) continue;
      float cnt = 0.f, mean = 0.f, m2 = 0.f;
#pragma unroll
      for (int w = 0; w < WM; ++w) {
        const float* q = red + (w * BN + c) * 4;
        const float nw = q[3];
        if (nw <= 0.f) continue;
        const float mw = q[2] + q[0] / nw, m2w = fmaxf(q[1] - q[0] * (q[0] / nw), 0.f);
        const float ntot = cnt + nw, dl = mw - mean;
        mean += dl * (nw / ntot);
        m2 += m2w + dl * dl * (cnt * nw / ntot);
        cnt = ntot;
      }
      *reinterpret_cast<float4*>(p.stats + (((long long)ph * p.mtiles + mt) * p.N + n) * 4) =
          make_float4(cnt, 0.f, m2, mean);
    }
    __syncthreads();
  }
  constexpr int PITCH = BN * 2 + 16;
  char* tl = smem;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wm * TM + 16 * i + rq + r, col = wn * TN + 16 * j + cl;
        *reinterpret_cast<unsigned short*>(tl + row * PITCH + col * 2) = f2bf(acc[i][j][r]);
      }
  __syncthreads();
  constexpr int CPR = BN / 8;
  for (int e = tid; e < BM * CPR; e += 256) {
    const int row = e / CPR, cc = e % CPR;
    const int m = m0 + row, n = n0 + cc * 8;
    if (m >= p.M || n >= p.N) continue;
    const int b = fast_div(m, GHW, p.inv_ghw), rem = m - b * GHW;
    const int gy = fast_div(rem, p.GW, p.inv_gw), gx = rem - gy * p.GW;
    const int oy = p.convt ? 2 * gy + py : gy, ox = p.convt ? 2 * gx + px : gx;
    *reinterpret_cast<uint4*>(p.out + (long long)b * p.o_bs + (long long)oy * p.o_rs + (long long)ox * p.o_ps + p.o_co + n) =
        *reinterpret_cast<const uint4*>(tl + row * PITCH + cc * 16);
  }
}

// ------------------------------------------------------------------------- host
struct DeepPlan {
  int BM, BN, ksplit, kps, mtiles, ntiles, ntaps;
  unsigned char taps[4][16];
};

// taps of each phase that read inside the input for at least one grid point (all others only read padding)
static int deep_taps(int convt, int IH, int IW, int GH, int GW, unsigned char (&taps)[4][16]) {
  int nt = -1;
  for (int ph = 0; ph < (convt ? 4 : 1); ++ph) {
    int n = 0;
    for (int t = 0; t < (convt ? 4 : 16); ++t) {
      int dy, dx, sy, sx;
      if (convt) { dy = (ph >> 1) - (t >> 1); dx = (ph & 1) - (t & 1); sy = 1; sx = 1; }
      else { dy = (t >> 2) - 1; dx = (t & 3) - 1; sy = 2; sx = 2; }
      bool rowok = false, colok = false;
      for (int g = 0; g < GH && !rowok; ++g) rowok = sy * g + dy >= 0 && sy * g + dy < IH;
      for (int g = 0; g < GW && !colok; ++g) colok = sx * g + dx >= 0 && sx * g + dx < IW;
      if (rowok && colok) taps[ph][n++] = (unsigned char)t;
    }
    if (nt < 0) nt = n;
    if (n != nt) return -1;  // (phases with different counts: not used by these shapes)
  }
  return nt;
}

static const int kDeepTiles[][2] = {{32, 32}, {32, 64}, {64, 64}, {64, 128}, {128, 64}, {128, 128}};

static bool deep_plan(int convt, int B, int GH, int GW, int IH, int IW, int Cin, int N, const int32_t* force, DeepPlan& pl) {
  pl.ntaps = deep_taps(convt, IH, IW, GH, GW, pl.taps);
  if (pl.ntaps <= 0) return false;
  const int nph = convt ? 4 : 1;
  const long long M = (long long)B * GH * GW;
  const int nks = pl.ntaps * (Cin / 64);
  double best = 1e30;
  int bi = -1, bs = 1;
  for (int t = 0; t < 6; ++t) {
    const int BM = kDeepTiles[t][0], BN = kDeepTiles[t][1];
    if (force && force[0] >= 0 && force[0] != t) continue;
    if (BN > N || (BM > 32 && BM / 2 >= M)) continue;
    const long long tiles = nph * ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
    for (int s = 1; s <= 64 && s <= nks; s *= 2) {
      if (force && force[1] > 0 && force[1] != s) continue;
      const long long blocks = tiles * s;
      if (!force && (blocks > 1024 || (blocks < 128 && s * 2 <= nks))) continue;
      const int kps = (nks + s - 1) / s;
      // cost model (us): waves of blocks x (operand bytes per block at ~100 GB/s per CU + MFMA time) + the
      // reducer's slab read + the launch's fixed latency
      const double per_block = (double)(BM + BN) * kps * 128 / 100e3 + (double)BM * BN * kps * 64 * 2 / 9.8e6;
      const double waves = (double)((blocks + 511) / 512);
      const double red = s > 1 ? (double)s * BM * BN * 4 / 100e3 + 2.0 : 0.0;
      const double cost = waves * per_block * (blocks > 256 ? 2.0 : 1.0) + red;
      if (cost < best) { best = cost; bi = t; bs = s; }
    }
  }
  if (bi < 0) return false;
  pl.BM = kDeepTiles[bi][0];
  pl.BN = kDeepTiles[bi][1];
  pl.mtiles = (int)((M + pl.BM - 1) / pl.BM);
  pl.ntiles = (N + pl.BN - 1) / pl.BN;
  pl.kps = (nks + bs - 1) / bs;
  pl.ksplit = (nks + pl.kps - 1) / pl.kps;
  return true;
}

// [two stages][scale / shift table of 1024 channels][flag]; the epilogue's tile and statistics area fit in the stages
static size_t deep_lds(int BM, int BN) { return 2 * (size_t)(BM + BN) * 128 + 2 * 1024 * 4 + 16; }

}  // namespace stc

using namespace stc;

static bool deep_shape_ok(int kind, int Cin, int Cout) {
  return (kind == STC_CONV_S2 || kind == STC_CONVT_S2) && Cin % 64 == 0 && Cin <= 1024 && Cout % 32 == 0 && Cout <= 2048;
}

extern "C" int stc_deep_conv_query(int kind, int B, int Hg, int Wg, int IH, int IW, int Cin, int Cout,
                                   const int32_t* force_plan, int64_t* ws_bytes, int32_t* ntickets,
                                   int32_t* stats_chunks, int32_t* plan_out) {
  STC_REQUIRE(deep_shape_ok(kind, Cin, Cout), "stc_deep_conv_query: kind %d Cin %d Cout %d not supported", kind, Cin, Cout);
  DeepPlan pl;
  STC_REQUIRE(deep_plan(kind == STC_CONVT_S2, B, Hg, Wg, IH, IW, Cin, Cout, force_plan, pl),
              "stc_deep_conv_query: no plan for this shape");
  const int nph = kind == STC_CONVT_S2 ? 4 : 1;
  const long long tiles = (long long)nph * pl.mtiles * pl.ntiles;
  if (ws_bytes) *ws_bytes = pl.ksplit > 1 ? tiles * pl.ksplit * pl.BM * pl.BN * 4 : 0;
  if (ntickets) *ntickets = (int32_t)tiles;
  if (stats_chunks) *stats_chunks = nph * pl.mtiles;
  if (plan_out) {
    plan_out[0] = pl.BM; plan_out[1] = pl.BN; plan_out[2] = pl.ksplit; plan_out[3] = pl.ntaps;
    plan_out[4] = (int32_t)(tiles * pl.ksplit);
  }
  return 0;
}

extern "C" int stc_deep_conv(int kind, int B, int nsrc, const stc_deep_src* src, const void* w_packed, int Cout,
                             stc_view y, float* stats_part, int stats_chunks, const int32_t* force_plan,
                             uint32_t* tickets, int ntickets, void* workspace, int64_t workspace_bytes, void* stream) {
  STC_REQUIRE(nsrc == 1 || nsrc == 2, "stc_deep_conv: 1 or 2 sources");
  const int IH = src[0].x.H, IW = src[0].x.W;
  int Cin = 0;
  for (int i = 0; i < nsrc; ++i) {
    const stc_view& v = src[i].x;
    STC_REQUIRE(v.p && v.H == IH && v.W == IW && v.cs == 1 && v.co % 8 == 0 && v.ps % 8 == 0 && v.rs % 8 == 0 &&
                    v.bs % 8 == 0 && ((uintptr_t)v.p & 15) == 0 && src[i].C % 64 == 0 && src[i].C > 0,
                "stc_deep_conv: source %d must be a 16-byte NHWC bf16 view of a multiple of 64 channels", i);
    Cin += src[i].C;
  }
  STC_REQUIRE(deep_shape_ok(kind, Cin, Cout), "stc_deep_conv: kind %d Cin %d Cout %d not supported", kind, Cin, Cout);
  const bool convt = kind == STC_CONVT_S2;
  const int GH = convt ? IH : y.H, GW = convt ? IW : y.W;
  if (convt) STC_REQUIRE(y.H == 2 * GH && y.W == 2 * GW, "stc_deep_conv: ConvT output %dx%d for input %dx%d", y.H, y.W, IH, IW);
  else STC_REQUIRE(IH == 2 * GH || IH == 2 * GH - 1, "stc_deep_conv: conv input %d for output %d", IH, GH);
  STC_REQUIRE(y.cs == 1 && y.co % 8 == 0 && y.ps % 8 == 0 && y.rs % 8 == 0 && y.bs % 8 == 0 && ((uintptr_t)y.p & 15) == 0,
              "stc_deep_conv: output must be a 16-byte NHWC bf16 view");
  DeepPlan pl;
  STC_REQUIRE(deep_plan(convt, B, GH, GW, IH, IW, Cin, Cout, force_plan, pl), "stc_deep_conv: no plan for this shape");
  const int nph = convt ? 4 : 1;
  const long long tiles = (long long)nph * pl.mtiles * pl.ntiles;
  STC_REQUIRE(tickets && ntickets >= tiles, "stc_deep_conv: %d tickets < %lld tiles", ntickets, tiles);
  const long long need = pl.ksplit > 1 ? tiles * pl.ksplit * pl.BM * pl.BN * 4 : 0;
  STC_REQUIRE(workspace_bytes >= need && (need == 0 || workspace), "stc_deep_conv: workspace %lld < %lld",
              (long long)workspace_bytes, need);
  if (stats_part) STC_REQUIRE(stats_chunks >= nph * pl.mtiles, "stc_deep_conv: stats chunks %d < %d", stats_chunks, nph * pl.mtiles);
  DeepParams p{};
  p.nsrc = nsrc;
  for (int i = 0; i < nsrc; ++i) {
    const stc_deep_src& s = src[i];
    DeepSrc& d = p.src[i];
    d.p = (const bf16*)s.x.p; d.bs = s.x.bs; d.rs = (int)s.x.rs; d.ps = s.x.ps; d.co = s.x.co;
    d.nc = s.C;
    d.part = s.part; d.nch = s.nchunks;
    STC_REQUIRE(!s.part || s.nchunks > 0, "stc_deep_conv: partials without chunks");
    d.scale = s.scale; d.shift = s.shift; d.gamma = s.gamma; d.beta = s.beta;
    d.eps = s.eps; d.momentum = s.momentum; d.slope = s.slope;
    d.mode = (s.part || s.scale || s.slope != 1.f) ? 1 : 0;
    d.mean_o = s.mean_out; d.rstd_o = s.rstd_out; d.scale_o = s.scale_out; d.shift_o = s.shift_out;
    d.rmean = s.running_mean; d.rvar = s.running_var; d.nbt = (long long*)s.num_batches_tracked;
    STC_REQUIRE(!d.mean_o || (s.part && d.rstd_o && d.scale_o && d.shift_o),
                "stc_deep_conv: designated outputs need partials and all four tables");
  }
  p.convt = convt ? 1 : 0;
  p.IH = IH; p.IW = IW; p.GH = GH; p.GW = GW; p.M = B * GH * GW;
  STC_REQUIRE(p.M < (1 << 24), "stc_deep_conv: M");
  p.inv_ghw = 1.0f / (float)(GH * GW);
  p.inv_gw = 1.0f / (float)GW;
  p.N = Cout; p.Cin = Cin; p.ntaps = pl.ntaps;
  for (int a = 0; a < 4; ++a) {
    p.tapl[a] = 0;
    for (int b = 0; b < pl.ntaps; ++b) p.tapl[a] |= (unsigned long long)(pl.taps[a][b] & 15) << (4 * b);
  }
  p.w = (const bf16*)w_packed;
  p.w_taps = convt ? 4 : 16;
  p.w_phase_stride = (long long)Cout * p.w_taps * Cin;
  p.out = (bf16*)y.p; p.o_bs = y.bs; p.o_rs = (int)y.rs; p.o_ps = y.ps; p.o_co = y.co;
  p.slab = (float*)workspace;
  p.tickets = tickets;
  p.stats = stats_part;
  p.nphase = nph; p.mtiles = pl.mtiles; p.ntiles = pl.ntiles; p.ksplit = pl.ksplit; p.kps = pl.kps;
  const dim3 grid((unsigned)(tiles * pl.ksplit));
  hipStream_t st = (hipStream_t)stream;
  const size_t lds = deep_lds(pl.BM, pl.BN);
  main_timer_begin(st);
#define STC_D(BM_, BN_) \
  if (pl.BM == BM_ && pl.BN == BN_) hipLaunchKernelGGL((deep_conv_kernel<BM_, BN_>), grid, dim3(256), lds, st, p); else
  STC_D(32, 32) STC_D(32, 64) STC_D(64, 64) STC_D(64, 128) STC_D(128, 64) STC_D(128, 128)
  { return fail(-1, "stc_deep_conv: no kernel for tile %dx%d", pl.BM, pl.BN); }
#undef STC_D
  main_timer_end(st);
  STC_CHECK_LAUNCH();
  return 0;
}
