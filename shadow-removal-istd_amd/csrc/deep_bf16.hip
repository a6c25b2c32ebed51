// The U-Net's innermost levels (1x1 - 8x8 grids) as ONE launch per layer (gfx950, bf16 MFMA).
//
// At bs = 32 these layers -- STCGAN/networks.py:104-105 (down convs of the three innermost blocks) and :119-121,
// :126-128 (their up ConvTs) -- have 32 - 512 GEMM rows per phase against 8.4 - 16.8 MB of weights: the time is
// latency and weight streaming, not MFMA work.  The im2col path ran each as four launches (the GEMM, a split-K
// reduction, the BatchNorm finalize, the BatchNorm + activation pass); here one launch does all of it:
//
//   * A operand: register-staged from the RAW (pre-BatchNorm) output of the previous layer, its BatchNorm affine +
//     activation applied in registers as the tile is staged (these activations are <= 1 M elements, so the
//     transform costs nothing), up to two sources (the U-Net concat [skip | up] of a ConvT's input), each with the
//     (scale, shift) table its producer wrote;
//   * split-K without a second launch: every K-slice block stores its fp32 tile (accumulator order), takes a
//     ticket on its tile (agent-scope release / acquire, cdna_hip_programming.md Guideline 16 counter form);
//     the block drawing the last ticket sums the slices in split order (deterministic for any arrival order) and
//     writes the bf16 output through LDS as 16-byte NHWC rows;
//   * the output's BatchNorm without a finalize launch: each tile's reducer stores its (count, mean, M2) per
//     channel and takes a ticket on its column of tiles; the last of a column merges that column's partials in
//     a fixed order (fp64, stc_bn_finalize's arithmetic) into the mean / rstd / scale / shift tables and the
//     running statistics of those channels -- the next layer reads the table as its source's affine;
//   * taps that read only padding for every row of the launch (1x1 grids: 4 of 16 conv taps, 1 of 4 ConvT taps
//     per phase) are dropped from K on the host (their weights are never read).
//
// v_mfma_f32_16x16x32_bf16, 4 waves (2 x 2), K-steps of 64 (one tap, 64 channels of one source), LDS double
// buffer, A and B both register-staged (one uniform vmcnt discipline; the weights are read once per block).
#include <type_traits>

#include "igemm_bf16.hpp"

namespace stc {

#ifndef DEEP_RING  // K-steps of register-staged loads in flight
#define DEEP_RING 2
#endif

struct DeepSrc {
  const bf16* p;
  unsigned bytes;       // extent of the source buffer (buffer-load range check: padding rows read zeros)
  long long bs;
  int rs, ps, co;
  int nc;               // K channels taken from this source
  const float* scale;   // (scale, shift) table of its BatchNorm (null: identity)
  const float* shift;
  float slope;          // activation after the affine
  int mode;             // 0 pass-through, 1 affine + activation
};

struct DeepBN {  // the output's BatchNorm (train mode): tables + running statistics written by the column finishers
  const float* gamma;
  const float* beta;
  float eps, momentum;
  float* mean_o; float* rstd_o; float* scale_o; float* shift_o;
  float* rmean; float* rvar; long long* nbt;
};

struct DeepParams {
  DeepSrc src[2];
  int nsrc, convt;
  int IH, IW;               // A extent (both sources)
  int GH, GW, M;            // GEMM grid (conv: output, ConvT: input), rows per phase
  int N, Cin, ntaps;        // K = ntaps * Cin
  int lg_cpt;               // log2(Cin / 64): K-steps per tap
  unsigned long long tapl[4];  // per phase: packed tap index of K-tap t in bits [4t, 4t + 4)
  const bf16* w;
  int w_taps;               // taps per phase in the packed layout (16 / 4)
  long long w_phase_stride; // elements
  bf16* out;
  long long o_bs;
  int o_rs, o_ps, o_co;
  float* slab;              // [tiles][ksplit][BM * BN]
  unsigned* tickets;        // [tiles] tile tickets, then [ntiles] column tickets
  float* stats;             // [nphase * mtiles][N][4] tile statistics partials, or null (no BatchNorm)
  DeepBN bn;
  int nphase, mtiles, ntiles, ksplit, kps;  // kps: K-steps (64) per split
  int acquire;              // hand-offs also take the agent acquire (grids of more than one block per CU)
  float inv_ghw, inv_gw;
  unsigned long long* dbg;  // diagnostics (stc_deep_debug_next): per block 8 wall-clock stamps, or null
};

// phase stamps of the diagnostic build-free timeline (scripts/deep_tune.py --phases): 0 start, 1 tables staged, 2 K
// loop done, 3 split-K hand-off passed (reducers), 4 tile output stored, 5 column hand-off passed (finishers), 6 end
#define DEEP_STAMP(i) \
  do { if (p.dbg && threadIdx.x == 0) p.dbg[(long long)blockIdx.x * 8 + (i)] = wall_clock64(); } while (0)

// the in-launch hand-offs: last_arriver / st_sc1 / ld_sc1 (igemm_bf16.hpp)
__device__ __forceinline__ bool deep_last_arriver(unsigned* counter, unsigned total, unsigned* flag, bool acquire) {
  return last_arriver(counter, total, flag, acquire);
}

// The column finisher: channel n's batch statistics from the column's tile partials {count, 0, M2, mean} (one per
// (phase, m tile), merged in chunk order, fp64, the two passes of stc_bn_finalize), then table + running statistics.
__device__ __forceinline__ void deep_finalize(const DeepParams& p, __amdgpu_buffer_rsrc_t rst, int n, bool count_batch) {
  const int nch = p.nphase * p.mtiles;
  constexpr int G = 16;  // chunk loads in flight per group
  double nt = 0, sm = 0;
  for (int k0 = 0; k0 < nch; k0 += G) {
    floatx4 v[G];
#pragma unroll
    for (int u = 0; u < G; ++u)
      v[u] = ld_sc1(rst, (unsigned)((min(k0 + u, nch - 1) * p.N + n) * 16));
#pragma unroll
    for (int u = 0; u < G; ++u) {
      if (k0 + u >= nch || v[u][0] <= 0.f) continue;
      nt += v[u][0];
      sm += (double)v[u][0] * v[u][3] + (double)v[u][1];
    }
  }
  const double mu = nt > 0 ? sm / nt : 0.0;
  double m2 = 0;
  for (int k0 = 0; k0 < nch; k0 += G) {
    floatx4 v[G];
#pragma unroll
    for (int u = 0; u < G; ++u)
      v[u] = ld_sc1(rst, (unsigned)((min(k0 + u, nch - 1) * p.N + n) * 16));
#pragma unroll
    for (int u = 0; u < G; ++u) {
      if (k0 + u >= nch || v[u][0] <= 0.f) continue;
      const double nb = v[u][0], s1 = v[u][1], r = s1 / nb;
      double q = (double)v[u][2] - s1 * r;
      if (q < 0) q = 0;
      const double d = (double)v[u][3] + r - mu;
      m2 += q + nb * d * d;
    }
  }
  bn_finalize_store(n, nt, mu, m2, p.bn.gamma, p.bn.beta, p.bn.rmean, p.bn.rvar, count_batch ? p.bn.nbt : nullptr,
                    p.bn.momentum, p.bn.eps, p.bn.mean_o, p.bn.rstd_o, p.bn.scale_o, p.bn.shift_o);
}

template <int BM, int BN>
__global__ void __launch_bounds__(256) deep_conv_kernel(const DeepParams p) {
  constexpr int WM = 2, WN = 2;
  constexpr int TM = BM / WM, TN = BN / WN, FM = TM / 16, FN = TN / 16;
  constexpr int AC = BM * 8 / 256, BC = BN * 8 / 256;  // 16-byte chunks per thread per K-step (A / B)
  constexpr int STAGE = (BM + BN) * 128;
  constexpr int NSTG = 2;                              // LDS double buffer
  constexpr int AG = BM / 32, BG = BN / 32, P = AG + BG;  // 1 KiB DMA pieces per wave per K-step
  static_assert(FM >= 1 && FN >= 1 && AC >= 1 && BC >= 1, "tile");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // LDS: [NSTG stages][table: scale[1024] shift[1024]][flag]; the epilogue reuses the stages
  float* tsc = reinterpret_cast<float*>(smem + NSTG * STAGE);
  float* tsh = tsc + 1024;

  DEEP_STAMP(0);
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  // XCD-aware: consecutive ids share an XCD (blocks b, b + 8, ... are dealt to one); the order is (phase, column of
  // output channels, row tile, K slice) -- a tile's K slices on one XCD (its reducer reads same-XCD slabs) and the
  // row tiles of one column of channels together, so each XCD streams its own slice of the weights (with the
  // columns spread over the XCDs, every XCD's L2 fetched every weight: 8x the HBM traffic of the layer's weights)
  const int nwg = p.nphase * p.mtiles * p.ntiles * p.ksplit;
  int bid = blockIdx.x;
  {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int split = bid % p.ksplit;
  const int tq = bid / p.ksplit;  // (phase, column, row tile)
  const int mt = tq % p.mtiles;
  const int nt = (tq / p.mtiles) % p.ntiles;
  const int ph = tq / (p.mtiles * p.ntiles);
  const int tile = (ph * p.mtiles + mt) * p.ntiles + nt;  // (slab / ticket index)
  const int py = ph >> 1, px = ph & 1;
  const int m0 = mt * BM, n0 = nt * BN;
  const int cpt = p.Cin / 64;  // K-steps per tap
  const int nks = p.ntaps * cpt;
  const int ks0 = split * p.kps, ks1 = min(nks, ks0 + p.kps);

  // ---- the sources' (scale, shift) tables of the channels this block's K range reads (LDS, indexed by K channel)
  auto fill_tables = [&]() {
    const int a0 = ks0 % cpt, len = ks1 - ks0;
    float vs[4], vh[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {  // (all loads in flight, then the LDS writes: Cin <= 1024)
      const int kc = tid + 256 * u;
      vs[u] = 1.f;
      vh[u] = 0.f;
      if (kc >= p.Cin || ((kc >> 6) - a0 + cpt) % cpt >= len) continue;
      const bool s1 = p.nsrc == 2 && kc >= p.src[0].nc;
      const float* sc = s1 ? p.src[1].scale : p.src[0].scale;
      const float* sh = s1 ? p.src[1].shift : p.src[0].shift;
      const int c = kc - (s1 ? p.src[0].nc : 0);
      if (sc) {
        vs[u] = sc[c];
        vh[u] = sh[c];
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int kc = tid + 256 * u;
      if (kc < p.Cin) {
        tsc[kc] = vs[u];
        tsh[kc] = vh[u];
      }
    }
  };

  // ---- staging roles: a K-step stages BM + BN rows of 128 B (64 bf16 channels) as 8-row pieces; lane -> row
  // lane >> 3 of a piece, LDS slot lane & 7 holding source chunk slot ^ (row & 7) (the swizzle the fragment reads
  // are conflict-free with).  Per staged row, computed once: the byte offset of its tap-0 source pixel in each source
  // and the taps that read padding (bit t: K-tap t; every bit for rows past M) -- a K-step then costs an add, a
  // shift and an OR per row, its scalar terms shifts and table lookups (K-steps per tap a power of two).
  const int prow = lane >> 3, pslot = lane & 7;
  const int schunk = pslot ^ prow;  // (pieces start at multiples of 8 rows: row & 7 == prow)
  const int GHW = p.GH * p.GW;
  const unsigned long long tapl = ph == 0 ? p.tapl[0] : (ph == 1 ? p.tapl[1] : (ph == 2 ? p.tapl[2] : p.tapl[3]));
  // tap -> (row, column) offset of its source pixel from the tap-0 pixel's (conv: (+ky, +kx) from (2gy - 1, 2gx - 1);
  // ConvT phase (py, px): (-ty, -tx) from (gy + py, gx + px))
  auto tap_rc = [&](int tap, int& dy, int& dx) {
    if (p.convt) { dy = -(tap >> 1); dx = -(tap & 1); }
    else { dy = tap >> 2; dx = tap & 3; }
  };
  unsigned a_off[2][AG], a_inv[AG];
#pragma unroll
  for (int g = 0; g < AG; ++g) {
    const int m = m0 + (wave * AG + g) * 8 + prow;
    const bool in = m < p.M;
    const int mm = in ? m : 0;
    const int b = fast_div(mm, GHW, p.inv_ghw), rem = mm - b * GHW;
    const int gy = fast_div(rem, p.GW, p.inv_gw), gx = rem - gy * p.GW;
    const int y0 = p.convt ? gy + py : 2 * gy - 1, x0 = p.convt ? gx + px : 2 * gx - 1;
    unsigned inv = 0;
    for (int t = 0; t < p.ntaps; ++t) {
      int dy, dx;
      tap_rc((int)((tapl >> (4 * t)) & 15u), dy, dx);
      const int iy = y0 + dy, ix = x0 + dx;
      if (!(in && iy >= 0 && iy < p.IH && ix >= 0 && ix < p.IW)) inv |= 1u << t;
    }
    a_inv[g] = inv;
#pragma unroll
    for (int si = 0; si < 2; ++si) {
      const DeepSrc& q = si ? p.src[1] : p.src[0];
      a_off[si][g] = 2u * (unsigned)(b * q.bs + (long long)y0 * q.rs + (long long)x0 * q.ps + q.co + 8 * schunk);
    }
  }
  const __amdgpu_buffer_rsrc_t ra0 =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.src[0].p, (short)0, (int)p.src[0].bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t ra1 = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.nsrc == 2 ? p.src[1].p : p.src[0].p), (short)0, (int)(p.nsrc == 2 ? p.src[1].bytes : p.src[0].bytes),
      0x00020000);
  const bf16* wph = p.w + (long long)ph * p.w_phase_stride;
  const __amdgpu_buffer_rsrc_t rw =
      __builtin_amdgcn_make_buffer_rsrc((void*)wph, (short)0, (int)(p.w_phase_stride * 2), 0x00020000);
  unsigned b_off[BG];
#pragma unroll
  for (int h = 0; h < BG; ++h) {
    const int n = n0 + (wave * BG + h) * 8 + prow;
    b_off[h] = n < p.N ? 2u * (unsigned)(n * p.w_taps * p.Cin + 8 * schunk) : OOB;
  }
  // K-step ks: K-tap index ti, its packed tap, channel block cb (of the concatenated sources), source s1
  auto step_terms = [&](int ks, int& ti, int& tap, int& cb, bool& s1) {
    ti = ks >> p.lg_cpt;
    cb = (ks & ((1 << p.lg_cpt) - 1)) << 6;
    tap = (int)((tapl >> (4 * ti)) & 15u);
    s1 = p.nsrc == 2 && cb >= p.src[0].nc;
  };

  // ---- the K loop, register-staged: the A / B chunks of K-step s + R load into VGPRs while steps s .. s + R - 1
  // compute; at step s its chunks get the source's BatchNorm affine + activation in registers and go to LDS stage
  // s & 1; one barrier per step (a stage is rewritten two steps after it was read, behind the barrier between)
  const int nsteps = ks1 - ks0;
  struct Stg {
    u32x4 a[AG], b[BG];
  };
  auto load = [&](int ks, Stg& r) {  // (a step past the block's K range loads zeros: the loop runs in groups of R)
    int ti, tap, cb;
    bool s1;
    step_terms(ks, ti, tap, cb, s1);
    const unsigned past = ks >= ks1 ? OOB : 0u;
    int dy, dx;
    tap_rc(tap, dy, dx);
    const unsigned adelta = 2u * (unsigned)((s1 ? p.src[1].rs : p.src[0].rs) * dy +
                                            (s1 ? p.src[1].ps : p.src[0].ps) * dx + cb - (s1 ? p.src[0].nc : 0));
#pragma unroll
    for (int g = 0; g < AG; ++g) {
      const unsigned off = ((s1 ? a_off[1][g] : a_off[0][g]) + adelta) | ((a_inv[g] << (31 - ti)) & OOB) | past;
      r.a[g] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(s1 ? ra1 : ra0, off, 0, 0));
    }
    const unsigned bdelta = 2u * (unsigned)(tap * p.Cin + cb);
#pragma unroll
    for (int h = 0; h < BG; ++h)
      r.b[h] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rw, (b_off[h] + bdelta) | past, 0, 0));
  };
  auto store = [&](int ks, const Stg& r, int st) {
    int ti, tap, cb;
    bool s1;
    step_terms(ks, ti, tap, cb, s1);
    char* sA = smem + st * STAGE;
    char* sB = sA + BM * 128;
    if ((s1 ? p.src[1].mode : p.src[0].mode) != 0) {
      const float slope = s1 ? p.src[1].slope : p.src[0].slope;  // (in [0, 1]: act(x) = max(x, slope x))
      const int kc = cb + 8 * schunk;
      const float4 c0 = *reinterpret_cast<const float4*>(tsc + kc), c1 = *reinterpret_cast<const float4*>(tsc + kc + 4);
      const float4 h0 = *reinterpret_cast<const float4*>(tsh + kc), h1 = *reinterpret_cast<const float4*>(tsh + kc + 4);
      const float sc[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
      const float sh[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
#pragma unroll
      for (int g = 0; g < AG; ++g) {
        // (padding stays zero: a mask, not a branch -- a branch here costs the loads' counted waits)
        const unsigned keep = ((a_inv[g] >> ti) & 1u) | (ks >= ks1 ? 1u : 0u) ? 0u : 0xffffffffu;
        u32x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float lo = fmaf(__uint_as_float(r.a[g][e] << 16), sc[2 * e], sh[2 * e]);
          const float hi = fmaf(__uint_as_float(r.a[g][e] & 0xffff0000u), sc[2 * e + 1], sh[2 * e + 1]);
          o[e] = pack_bf16x2(fmaxf(lo, slope * lo), fmaxf(hi, slope * hi)) & keep;
        }
        *reinterpret_cast<u32x4*>(sA + (wave * AG + g) * 1024 + lane * 16) = o;
      }
    } else {
#pragma unroll
      for (int g = 0; g < AG; ++g) *reinterpret_cast<u32x4*>(sA + (wave * AG + g) * 1024 + lane * 16) = r.a[g];
    }
#pragma unroll
    for (int h = 0; h < BG; ++h) *reinterpret_cast<u32x4*>(sB + (wave * BG + h) * 1024 + lane * 16) = r.b[h];
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

  constexpr int R = DEEP_RING;  // K-steps of loads in flight
  Stg r[R];
#pragma unroll
  for (int u = 0; u < R; ++u) load(ks0 + u, r[u]);
  fill_tables();
  __syncthreads();  // (the tables)
  DEEP_STAMP(1);
  for (int s = 0; s < nsteps; s += R) {  // (a count that is not a multiple of R ends with steps of zeros)
#pragma unroll
    for (int u = 0; u < R; ++u) {
      store(ks0 + s + u, r[u], u & 1);
      load(ks0 + s + u + R, r[u]);
      __syncthreads();
      compute(smem + (u & 1) * STAGE);
    }
  }
  __syncthreads();  // (the epilogue reuses the stages)

  DEEP_STAMP(2);
  // ---- split-K: slab store, ticket, the last arriver reduces in split order
  unsigned* flag = reinterpret_cast<unsigned*>(tsh + 1024);  // (inside the one LDS array)
  if (p.ksplit > 1) {
    const __amdgpu_buffer_rsrc_t rsl = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(p.slab + (long long)tile * p.ksplit * (BM * BN)), (short)0, p.ksplit * BM * BN * 4, 0x00020000);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        st_sc1(rsl, (unsigned)((split * (BM * BN) + ((wave * FM + i) * FN + j) * 256 + lane * 4) * 4), acc[i][j]);
    if (!deep_last_arriver(p.tickets + tile, (unsigned)p.ksplit, flag, p.acquire)) {
      DEEP_STAMP(6);
      return;
    }
    DEEP_STAMP(3);
    floatx4 sum[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) sum[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    // every slab loaded (the own one too: no per-element register-or-load select), groups of RG slabs in flight,
    // summed in split order
    constexpr int RG = FM * FN <= 1 ? 16 : (FM * FN <= 2 ? 8 : (FM * FN <= 4 ? 4 : 2));  // (<= 64 VGPRs in flight)
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
            v[g][i][j] = ld_sc1(rsl, (unsigned)((s * (BM * BN) + ((wave * FM + i) * FN + j) * 256 + lane * 4) * 4));
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
    const __amdgpu_buffer_rsrc_t rst = __builtin_amdgcn_make_buffer_rsrc(
        (void*)p.stats, (short)0, p.nphase * p.mtiles * p.N * 16, 0x00020000);
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
      st_sc1(rst, (unsigned)(((ph * p.mtiles + mt) * p.N + n) * 16), floatx4{cnt, 0.f, m2, mean});
    }
    // the last tile of this column of channels finalizes their BatchNorm (the next layer reads the table)
    const long long ntiles_all = (long long)p.nphase * p.mtiles * p.ntiles;
    if (deep_last_arriver(p.tickets + ntiles_all + nt, (unsigned)(p.nphase * p.mtiles), flag, p.acquire)) {
      DEEP_STAMP(5);
      for (int c = tid; c < BN; c += 256)
        if (n0 + c < p.N) deep_finalize(p, rst, n0 + c, nt == 0 && c == 0);
    }
    __syncthreads();
  }
  DEEP_STAMP(4);
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
  DEEP_STAMP(6);
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
      // cost model (us, fitted to the plan sweeps of scripts/deep_tune.py): a K-step costs a block ~0.25 us of
      // issue and waits plus ~3.5 ns per staged row (a second block per CU overlaps little: rounds of 256 blocks),
      // the reducer reads its tile's slabs (~40 GB/s per block) after a ~1.5 us hand-off; the loop runs whole
      // groups of DEEP_RING steps
      const int kpr = (kps + DEEP_RING - 1) / DEEP_RING * DEEP_RING;
      const double rounds = (double)((blocks + 255) / 256);
      const double red = s > 1 ? 1.5 + (double)s * BM * BN * 4 / 40e3 : 0.0;
      const double cost = rounds * kpr * (0.25 + 0.0035 * (BM + BN)) + red;
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
  const int cpt = Cin / 64;  // (K-steps per tap: a power of two, the kernel's step terms are shifts)
  return (kind == STC_CONV_S2 || kind == STC_CONVT_S2) && Cin % 64 == 0 && Cin <= 1024 && (cpt & (cpt - 1)) == 0 &&
         Cout % 32 == 0 && Cout <= 2048;
}

static unsigned long long* g_deep_dbg = nullptr;  // (diagnostics: the next launch's stamps; one-shot)
extern "C" int stc_deep_debug_next(void* stamps) {
  g_deep_dbg = (unsigned long long*)stamps;
  return 0;
}

extern "C" int stc_deep_conv_query(int kind, int B, int Hg, int Wg, int IH, int IW, int Cin, int Cout,
                                   const int32_t* force_plan, int64_t* ws_bytes, int32_t* ntickets, int32_t* plan_out) {
  STC_REQUIRE(deep_shape_ok(kind, Cin, Cout), "stc_deep_conv_query: kind %d Cin %d Cout %d not supported", kind, Cin, Cout);
  DeepPlan pl;
  STC_REQUIRE(deep_plan(kind == STC_CONVT_S2, B, Hg, Wg, IH, IW, Cin, Cout, force_plan, pl),
              "stc_deep_conv_query: no plan for this shape");
  const int nph = kind == STC_CONVT_S2 ? 4 : 1;
  const long long tiles = (long long)nph * pl.mtiles * pl.ntiles;
  if (ws_bytes)
    *ws_bytes = (pl.ksplit > 1 ? tiles * pl.ksplit * pl.BM * pl.BN * 4 : 0) + (long long)nph * pl.mtiles * Cout * 16;
  if (ntickets) *ntickets = (int32_t)(tiles + pl.ntiles);
  if (plan_out) {
    plan_out[0] = pl.BM; plan_out[1] = pl.BN; plan_out[2] = pl.ksplit; plan_out[3] = pl.ntaps;
    plan_out[4] = (int32_t)(tiles * pl.ksplit);
  }
  return 0;
}

extern "C" int stc_deep_conv(int kind, int B, int nsrc, const stc_deep_src* src, const void* w_packed, int Cout,
                             stc_view y, const stc_deep_bn* bn, const int32_t* force_plan, uint32_t* tickets,
                             int ntickets, void* workspace, int64_t workspace_bytes, void* stream) {
  STC_REQUIRE(nsrc == 1 || nsrc == 2, "stc_deep_conv: 1 or 2 sources");
  const int IH = src[0].x.H, IW = src[0].x.W;
  int Cin = 0;
  for (int i = 0; i < nsrc; ++i) {
    const stc_view& v = src[i].x;
    STC_REQUIRE(v.p && v.H == IH && v.W == IW && v.cs == 1 && v.co % 8 == 0 && v.ps % 8 == 0 && v.rs % 8 == 0 &&
                    v.bs % 8 == 0 && ((uintptr_t)v.p & 15) == 0 && src[i].C % 64 == 0 && src[i].C > 0,
                "stc_deep_conv: source %d must be a 16-byte NHWC bf16 view of a multiple of 64 channels", i);
    STC_REQUIRE((src[i].scale == nullptr) == (src[i].shift == nullptr), "stc_deep_conv: scale / shift come together");
    Cin += src[i].C;
  }
  STC_REQUIRE(deep_shape_ok(kind, Cin, Cout), "stc_deep_conv: kind %d Cin %d Cout %d not supported", kind, Cin, Cout);
  const bool convt = kind == STC_CONVT_S2;
  const int GH = convt ? IH : y.H, GW = convt ? IW : y.W;
  if (convt) STC_REQUIRE(y.H == 2 * GH && y.W == 2 * GW, "stc_deep_conv: ConvT output %dx%d for input %dx%d", y.H, y.W, IH, IW);
  else STC_REQUIRE((IH == 2 * GH || IH == 2 * GH - 1) && (IW == 2 * GW || IW == 2 * GW - 1),
                   "stc_deep_conv: conv input %dx%d for output %dx%d", IH, IW, GH, GW);
  STC_REQUIRE(y.cs == 1 && y.co % 8 == 0 && y.ps % 8 == 0 && y.rs % 8 == 0 && y.bs % 8 == 0 && ((uintptr_t)y.p & 15) == 0,
              "stc_deep_conv: output must be a 16-byte NHWC bf16 view");
  DeepPlan pl;
  STC_REQUIRE(deep_plan(convt, B, GH, GW, IH, IW, Cin, Cout, force_plan, pl), "stc_deep_conv: no plan for this shape");
  const int nph = convt ? 4 : 1;
  const long long tiles = (long long)nph * pl.mtiles * pl.ntiles;
  STC_REQUIRE(tickets && ntickets >= tiles + pl.ntiles, "stc_deep_conv: %d tickets < %lld", ntickets, tiles + pl.ntiles);
  const long long slab = pl.ksplit > 1 ? tiles * pl.ksplit * pl.BM * pl.BN * 4 : 0;
  const long long need = slab + (long long)nph * pl.mtiles * Cout * 16;
  STC_REQUIRE(workspace && workspace_bytes >= need, "stc_deep_conv: workspace %lld < %lld", (long long)workspace_bytes, need);
  DeepParams p{};
  p.nsrc = nsrc;
  for (int i = 0; i < nsrc; ++i) {
    const stc_deep_src& s = src[i];
    DeepSrc& d = p.src[i];
    d.p = (const bf16*)s.x.p; d.bs = s.x.bs; d.rs = (int)s.x.rs; d.ps = s.x.ps; d.co = s.x.co;
    const long long bytes = ((long long)(B - 1) * s.x.bs + (long long)(s.x.H - 1) * s.x.rs + (long long)(s.x.W - 1) * s.x.ps +
                             s.x.co + s.C) * 2;
    STC_REQUIRE(bytes < (1ll << 31), "stc_deep_conv: source %d spans >= 2 GiB", i);
    d.bytes = (unsigned)bytes;
    d.nc = s.C;
    d.scale = s.scale; d.shift = s.shift; d.slope = s.slope;
    d.mode = (s.scale || s.slope != 1.f) ? 1 : 0;
    STC_REQUIRE(!d.mode || (s.slope >= 0.f && s.slope <= 1.f), "stc_deep_conv: activation slope %g not in [0, 1]", s.slope);
  }
  if (bn) {
    STC_REQUIRE(bn->mean_out && bn->rstd_out && bn->scale_out && bn->shift_out,
                "stc_deep_conv: the output BatchNorm needs its four table outputs");
    p.bn.gamma = bn->gamma; p.bn.beta = bn->beta; p.bn.eps = bn->eps; p.bn.momentum = bn->momentum;
    p.bn.mean_o = bn->mean_out; p.bn.rstd_o = bn->rstd_out; p.bn.scale_o = bn->scale_out; p.bn.shift_o = bn->shift_out;
    p.bn.rmean = bn->running_mean; p.bn.rvar = bn->running_var; p.bn.nbt = (long long*)bn->num_batches_tracked;
    p.stats = (float*)((char*)workspace + slab);
  }
  p.convt = convt ? 1 : 0;
  p.IH = IH; p.IW = IW; p.GH = GH; p.GW = GW; p.M = B * GH * GW;
  STC_REQUIRE(p.M < (1 << 24), "stc_deep_conv: M");
  p.inv_ghw = 1.0f / (float)(GH * GW);
  p.inv_gw = 1.0f / (float)GW;
  p.N = Cout; p.Cin = Cin; p.ntaps = pl.ntaps;
  p.lg_cpt = __builtin_ctz((unsigned)(Cin / 64));
  for (int a = 0; a < 4; ++a) {
    p.tapl[a] = 0;
    for (int b = 0; b < pl.ntaps; ++b) p.tapl[a] |= (unsigned long long)(pl.taps[a][b] & 15) << (4 * b);
  }
  p.w = (const bf16*)w_packed;
  p.w_taps = convt ? 4 : 16;
  p.w_phase_stride = (long long)Cout * p.w_taps * Cin;
  STC_REQUIRE(p.w_phase_stride * 2 < (1ll << 31), "stc_deep_conv: weights");
  p.out = (bf16*)y.p; p.o_bs = y.bs; p.o_rs = (int)y.rs; p.o_ps = y.ps; p.o_co = y.co;
  p.slab = (float*)workspace;
  p.tickets = tickets;
  p.nphase = nph; p.mtiles = pl.mtiles; p.ntiles = pl.ntiles; p.ksplit = pl.ksplit; p.kps = pl.kps;
  p.dbg = g_deep_dbg;
  g_deep_dbg = nullptr;
  static int ncu = 0;  // (CUs of the device: one process drives one GPU)
  if (ncu == 0) {
    int dev = 0, n = 256;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
      ncu = n;
    else
      ncu = 256;
  }
  p.acquire = tiles * pl.ksplit > ncu ? 1 : 0;
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
