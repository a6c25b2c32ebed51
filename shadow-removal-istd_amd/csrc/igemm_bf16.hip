// bf16 implicit-GEMM 4x4 convolution on gfx950 MFMA, staged by LDS-DMA.
//
// Same problem family as igemm.hip (Conv2d k4 s2/s1, ConvTranspose2d k4 s2 as 4 phases,
// and both input gradients), bf16 operands / fp32 accumulation:
//   * operands move HBM/L2 -> LDS with buffer_load_dwordx4 ... lds (one 1 KiB wave
//     instruction = 8 rows x 128 B of K), no VGPR round trip and no ds_write pass.
//     Zero padding / K tails / rows past M come for free: their byte offset is put
//     out of the buffer range, and the range check delivers zeros.
//   * LDS image per stage: [rows][128 B] with the 16-byte chunk index XOR-swizzled by
//     (row & 7) on the *source* side (the DMA image is lane-linear), so every
//     ds_read_b128 lane group hits 16 distinct bank slots.
//   * v_mfma_f32_16x16x32_bf16, wave tile (BM/WM) x (BN/WN); 2-stage ring, BK = 64:
//     the DMA of K-step s+1 is in flight under the MFMAs of step s, one barrier per step.
//   * epilogue: either fp32 split-K slabs, or + bias -> bf16 through an LDS tile and
//     16-byte row stores (NHWC rows are contiguous channels), with the BatchNorm batch
//     statistics of the tile fused in (two-pass: tile mean, then centred sum of
//     squares, in fp32 from the accumulators) -> part[tile][n] = {count, 0, M2, mean},
//     the format stc_bn_finalize merges (Chan's parallel variance).

#include <map>
#include <mutex>
#include <tuple>
#include <unordered_map>

#include "igemm_bf16.hpp"

namespace stc {

// LD > 0: LD extra "loader" waves issue every LDS-DMA piece and the WM*WN compute waves only read
// fragments and issue MFMAs (one barrier per K-step; the loaders run NST-1 steps ahead), so the DMA
// issue never sits in a compute wave's instruction stream.
template <int BM, int BN, int WM, int WN, int NST, int BK, bool BNB, int LD>
__device__ __forceinline__ void igemm_bf16_body(const GParams& p) {
  constexpr int NW = WM * WN;
  constexpr int NL = LD > 0 ? LD : NW;   // waves that issue the DMA
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int FM = TM / 16, FN = TN / 16;
  constexpr int RB = BK * 2;             // bytes per LDS row (one GEMM row's K-step)
  constexpr int CH = BK / 8;             // 16-byte chunks per row
  constexpr int RPP = 1024 / RB;         // rows per 1 KiB DMA piece
  constexpr int AG = BM / (RPP * NL), BG = BN / (RPP * NL);  // pieces per loading wave per K-step
  constexpr int STAGE = (BM + BN) * RB;
  constexpr int KK = BK / 32;            // 16x16x32 MFMA sub-steps per K-step
  static_assert(AG * RPP * NL == BM && BG * RPP * NL == BN, "tile rows must split into whole pieces per wave");
  static_assert(FM >= 1 && FN >= 1, "wave tile >= 16x16");
  static_assert(NST >= 2 && NST <= 8, "2..8-stage ring (wait_ahead covers up to 6 steps ahead)");
  static_assert(BK == 64 || BK == 32, "BK");

  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int lw = LD > 0 ? wave - NW : wave;  // index among the loading waves

  // XCD-aware bijective remap of the linear block id (blocks b, b+8, ... share an XCD).  phase_major (the
  // 4-phase ConvT geometry without split-K): the grid is linear over (tile, phase) with the phase fastest,
  // so the 4 phase blocks of a tile -- which read the same input pixels -- run side by side on one XCD
  // and share its L2, instead of each phase sweeping the whole input a quarter of the launch apart.
  const int nwg = p.mtiles * p.ntiles * (p.phase_major ? p.nphase : 1);
  int bid = blockIdx.x;
  {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  int ph, split;
  if (p.phase_major) {
    ph = bid % p.nphase;
    bid /= p.nphase;
    split = 0;
  } else {
    ph = (int)blockIdx.z / p.ksplit;
    split = (int)blockIdx.z % p.ksplit;
  }
  const int mt = bid / p.ntiles, nt = bid % p.ntiles;
  const int m0 = mt * BM, n0 = nt * BN;
  const int z = ph * p.ksplit + split;
  const int kbeg = split * p.kchunk;
  const int kend = min(p.K, kbeg + p.kchunk);
  const int nsteps = (kend - kbeg + BK - 1) / BK;
  const int GHW = p.GH * p.GW;

  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)p.a, (short)0, (int)p.a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)p.b, (short)0, (int)p.b_bytes, 0x00020000);

  // ---- DMA lane roles: lane -> (row in its 8-row piece, source chunk) ; LDS slot = lane & 7
  // Every offset is computed unconditionally and pushed out of range by OR-ing bit 31 where the
  // element is padding (any offset >= 2^31 > num_records reads zeros): no divergent branches
  // around the DMA instructions.
  const int prow = lane / CH;                   // row within the piece
  const int schunk = (lane % CH) ^ kswz<BK>(prow);  // source chunk of this lane's LDS slot
  // Per DMA row: element offset of the tap-(0,0) source pixel, and the set of out-of-range taps
  // (bit t = ty << lg_tw | tx, the K loop's tap index; all bits for rows past M) -- the K loop then
  // needs one add and a bit extract per row instead of re-deriving and bounds-checking the im2col
  // address.  The in-range taps of one axis are an interval (closed form, tap_mask).
  const int ntap1 = 1 << p.lg_tw;
  unsigned a_off0[AG], a_inv[AG];
#pragma unroll
  for (int g = 0; g < AG; ++g) {
    const int m = m0 + (lw * AG + g) * RPP + prow;
    const int mm = m < p.M ? m : 0;
    const int b = fast_div(mm, GHW, p.inv_ghw), rem = mm - b * GHW;
    const int y = fast_div(rem, p.GW, p.inv_gw), x = rem - y * p.GW;
    const int ay = y * p.in_stride + p.offy[ph], ax = x * p.in_stride + p.offx[ph];
    a_off0[g] = (unsigned)(b * p.a_bs + p.a_co) + (unsigned)ay * (unsigned)p.a_rs + (unsigned)ax * (unsigned)p.a_ps;
    const unsigned rm = tap_mask(ay, p.IH, p.stepy, ntap1), cmk = tap_mask(ax, p.IW, p.stepx, ntap1);
    a_inv[g] = m < p.M ? ~(cmk * tap_spread(rm, p.lg_tw)) : ~0u;
  }
  unsigned b_off[BG];
#pragma unroll
  for (int g = 0; g < BG; ++g) {
    const int n = n0 + (lw * BG + g) * RPP + prow;
    b_off[g] = n < p.N ? (unsigned)(ph * p.b_phase_stride + n * p.K) : OOB;
  }
  const int tw_mask = ntap1 - 1;
  // this lane's K position: k = kbeg + BK*s + 8*schunk = t*cin + ci, advanced incrementally
  int kcur = kbeg + schunk * 8;
  int tcur = kcur / p.cin, ccur = kcur - tcur * p.cin;
  const bool cdivk = (BK % p.cin) == 0;
  const int tadv = cdivk ? BK / p.cin : 0;

  // one K-step's DMA = AG + BG pieces; the step's shared terms (the K-tail penalty and the tap
  // delta of this lane's K position) are computed once (prep), the pieces one at a time (piece),
  // so that they can be spread between the MFMAs of the previous step (compute_il)
  unsigned st_kpen = 0, st_delta = 0;
  int st_tcur = 0;
  auto prep = [&]() {
    st_kpen = kcur < kend ? 0u : OOB;
    const int ty = tcur >> p.lg_tw, tx = tcur & tw_mask;
    st_delta = (unsigned)(p.stepy * ty) * (unsigned)p.a_rs + (unsigned)(p.stepx * tx) * (unsigned)p.a_ps + (unsigned)ccur;
    st_tcur = tcur;
  };
  auto piece = [&](int stage, int g) {
    char* sA = smem + stage * STAGE;
    char* sB = sA + BM * RB;
    if (g < AG) {
      const unsigned pen = (((a_inv[g] >> (st_tcur & 31)) & 1u) << 31) | st_kpen;
      dma16(ra, sA + (lw * AG + g) * 1024, ((a_off0[g] + st_delta) * 2u) | pen);
    } else {
      const int h = g - AG;
      const unsigned off = ((b_off[h] + (unsigned)(kcur)) * 2u) | st_kpen | (b_off[h] & OOB);
      dma16(rb, sB + (lw * BG + h) * 1024, off);
    }
  };
  auto advance = [&]() {  // to the next K-step
    kcur += BK;
    if (cdivk) {
      tcur += tadv;
    } else {
      ccur += BK;
      while (ccur >= p.cin) { ccur -= p.cin; ++tcur; }
    }
  };
  auto issue = [&](int stage) {
    prep();
#pragma unroll
    for (int g = 0; g < AG + BG; ++g) piece(stage, g);
    advance();
  };

  floatx4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  // fragment read offsets: row (l & 15), chunk 4*kk + (l >> 4), slot = chunk ^ swizzle(row)
  const int frow = lane & 15;
  int rd_off[KK];
#pragma unroll
  for (int kk = 0; kk < KK; ++kk) rd_off[kk] = frow * RB + (((4 * kk + (lane >> 4)) ^ kswz<BK>(frow)) * 16);

  auto compute = [&](int stage) {
    const char* sA = smem + stage * STAGE + (wm * TM) * RB;
    const char* sB = smem + stage * STAGE + BM * RB + (wn * TN) * RB;
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      bf16x8_t fa[FM], fb[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) fa[i] = *reinterpret_cast<const bf16x8_t*>(sA + i * 16 * RB + rd_off[kk]);
#pragma unroll
      for (int j = 0; j < FN; ++j) fb[j] = *reinterpret_cast<const bf16x8_t*>(sB + j * 16 * RB + rd_off[kk]);
#if STC_SETPRIO
      __builtin_amdgcn_s_setprio(1);  // (guide T5: the MFMA cluster at raised wave priority)
#endif
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = exp_mfma(fa[i], fb[j], acc[i][j]);
#if STC_SETPRIO
      __builtin_amdgcn_s_setprio(0);
#endif
    }
  };

  // compute with the next step's DMA pieces interleaved: one piece after each MFMA row (FN MFMAs),
  // so the wave's LDS-DMA issue overlaps its own queued MFMAs instead of preceding all of them
  auto compute_il = [&](int stage, int nstage, bool dma) {
    const char* sA = smem + stage * STAGE + (wm * TM) * RB;
    const char* sB = smem + stage * STAGE + BM * RB + (wn * TN) * RB;
    if (dma) prep();
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      bf16x8_t fa[FM], fb[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) fa[i] = *reinterpret_cast<const bf16x8_t*>(sA + i * 16 * RB + rd_off[kk]);
#pragma unroll
      for (int j = 0; j < FN; ++j) fb[j] = *reinterpret_cast<const bf16x8_t*>(sB + j * 16 * RB + rd_off[kk]);
#pragma unroll
      for (int i = 0; i < FM; ++i) {
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = exp_mfma(fa[i], fb[j], acc[i][j]);
        const int slot = kk * FM + i;
        if (dma && slot < AG + BG) {
          piece(nstage, slot);
          __builtin_amdgcn_sched_group_barrier(0x008, FN, 0);  // the row's MFMAs, then the piece
          __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        }
      }
    }
    if (dma) {
#pragma unroll
      for (int g = KK * FM; g < AG + BG; ++g) piece(nstage, g);
      advance();
    }
  };

  if constexpr (LD > 0) {
    constexpr int P = AG + BG;
    if (wave >= NW) {  // loader: steps 0 .. NST-2 ahead, then one refill per K-step
#pragma unroll
      for (int i = 0; i < NST - 1; ++i)
        if (i < nsteps) issue(i);
      int nxt = NST - 1;
      for (int s = 0; s < nsteps; ++s) {
        wait_ahead<P>(min(NST - 2, nsteps - 1 - s));  // this wave's pieces of step s have landed
        __builtin_amdgcn_s_barrier();                 // ... and every loader's; step s - 1 is read
        if (s + NST - 1 < nsteps) issue(nxt);         // into the stage step s - 1 used
        nxt = nxt == NST - 1 ? 0 : nxt + 1;
      }
      return;  // (a terminated wave no longer counts at the epilogue's barriers)
    }
    int cur = 0;
    for (int s = 0; s < nsteps; ++s) {
      __builtin_amdgcn_s_barrier();
      compute(cur);
      cur = cur == NST - 1 ? 0 : cur + 1;
    }
  } else if constexpr (NST == 2 && STC_IGEMM_INTERLEAVE) {
    if (nsteps > 0) issue(0);
    for (int s = 0; s < nsteps; ++s) {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      compute_il(s & 1, (s + 1) & 1, s + 1 < nsteps);
    }
  } else if constexpr (NST == 2) {
    // DMA of step s+1 lands under the MFMAs of step s; one barrier per step.  Both buffers are free
    // at the start, so steps 0 and 1 are issued together (one memory latency, not two, before the
    // first MFMA -- the whole K loop of the K <= 128 layers) and step 0 waits with step 1 in flight.
    constexpr int P = AG + BG;
    if (nsteps > 0) issue(0);
    if (nsteps > 1) issue(1);
    for (int s = 0; s < nsteps; ++s) {
      wait_ahead<P>(s == 0 && nsteps > 1 ? 1 : 0);  // counted vmcnt + lgkmcnt(0), then a raw barrier
      __builtin_amdgcn_s_barrier();
      if (s > 0 && s + 1 < nsteps) issue((s + 1) & 1);
      compute(s & 1);
    }
  } else {
    // NST-stage ring: NST-1 K-steps in flight.  At step s wait only for step s's pieces (the
    // P*(steps issued after s) youngest stay in flight across the raw barrier), then refill the
    // stage that step s-1 read (every wave has passed the barrier, so those reads are done).
    constexpr int P = AG + BG;
#pragma unroll
    for (int i = 0; i < NST - 1; ++i)
      if (i < nsteps) issue(i);
    int cur = 0;
    for (int s = 0; s < nsteps; ++s) {
      const int ahead = min(NST - 2, nsteps - 1 - s);  // steps already issued beyond s
      wait_ahead<P>(ahead);
      __builtin_amdgcn_s_barrier();
      if (s + NST - 1 < nsteps) issue(cur == 0 ? NST - 1 : cur - 1);
      compute(cur);
      cur = cur == NST - 1 ? 0 : cur + 1;
    }
  }

#if STC_EXP_NOEPI
  {
    float s_ = 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) s_ += acc[i][j][0] + acc[i][j][3];
    if (s_ == 1.2345f) p.ws[threadIdx.x] = s_;
    return;
  }
#endif
  if (p.tickets) {  // in-launch split-K: the tile's last arriver runs the epilogue on the summed slabs
    __syncthreads();  // (every wave is done with the stage buffers: the hand-off flag lives in LDS)
    if (!splitk_combine<BM, BN, WM, WN>(p, acc, (ph * p.mtiles + mt) * p.ntiles + nt, split, smem)) return;
  }
  igemm_epilogue<BM, BN, WM, WN, BNB>(p, acc, m0, n0, ph, mt, z, smem);
}

template <int BM, int BN, int WM, int WN, int NST, int BK, bool BNB>
__global__ void __launch_bounds__(64 * WM * WN) igemm_bf16_kernel(const GParams p) {
  igemm_bf16_body<BM, BN, WM, WN, NST, BK, BNB, 0>(p);
}

// Loader-wave blocks (LD extra DMA-only waves): LD = 2 -> two 6-wave blocks per CU (3 waves per SIMD, the
// register budget capped to fit), LD = 4 -> one 8-wave block (2 waves per SIMD).
template <int BM, int BN, int WM, int WN, int NST, int BK, bool BNB, int LD>
__global__ void __launch_bounds__(64 * (WM * WN + LD), (LD == 2 ? 3 : 2)) igemm_bf16_ld_kernel(const GParams p) {
  igemm_bf16_body<BM, BN, WM, WN, NST, BK, BNB, LD>(p);
}

// Split-K reduction: out[row] = sum_s slab[s][row] (+bias, tanh) -> bf16 16-byte stores, with the
// BatchNorm partial statistics of the block's rows (shift = the block's first row, Chan-mergeable).
// Thread = 8 consecutive channels of one GEMM row; the block walks a contiguous row range.
__global__ void __launch_bounds__(256) splitk_reduce_stats_kernel(const GParams p, int rows_per_block) {
  const int CG = p.N / 8;  // channel groups (N % 8 == 0, N <= 2048)
  const int RL = 256 / CG;  // rows in parallel
  const int cg = threadIdx.x % CG, rl = threadIdx.x / CG;
  const long long R = (long long)p.nphase * p.M;  // rows = (phase, m)
  const long long r0 = (long long)blockIdx.x * rows_per_block;
  const long long r1 = min(R, r0 + rows_per_block);
  const int n = cg * 8;
  const int GHW = p.GH * p.GW;
  float sh[8], s1[8], s2[8];
  float cnt = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) { sh[e] = 0.f; s1[e] = 0.f; s2[e] = 0.f; }
  float bz[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) bz[e] = p.bias ? p.bias[n + e] : 0.f;
  const long long MN = (long long)p.M * p.N;
  auto rowval = [&](long long row, float* v) {
    const int ph = (int)(row / p.M), m = (int)(row - (long long)ph * p.M);
    const float* src = p.ws + ((long long)ph * p.ksplit * p.M + m) * p.N + n;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = bz[e];
    // slabs in groups of 4: the 8 loads of a group are in flight together (one memory latency
    // per group, not per slab -- the deep layers run 8-64 slabs over a handful of rows); the sum
    // order stays s = 0, 1, 2, ... per element
    int s = 0;
    for (; s + 4 <= p.ksplit; s += 4) {
      float4 a[4], b[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        a[u] = *reinterpret_cast<const float4*>(src + (s + u) * MN);
        b[u] = *reinterpret_cast<const float4*>(src + (s + u) * MN + 4);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        v[0] += a[u].x; v[1] += a[u].y; v[2] += a[u].z; v[3] += a[u].w;
        v[4] += b[u].x; v[5] += b[u].y; v[6] += b[u].z; v[7] += b[u].w;
      }
    }
    for (; s < p.ksplit; ++s) {
      const float4 a = *reinterpret_cast<const float4*>(src + s * MN);
      const float4 b = *reinterpret_cast<const float4*>(src + s * MN + 4);
      v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w;
      v[4] += b.x; v[5] += b.y; v[6] += b.z; v[7] += b.w;
    }
    if (p.tanh_) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = tanhf(v[e]);
    }
  };
  if (rl < RL && r0 < r1 && p.stats) {
    rowval(r0, sh);
  }
  float ba[8], bb[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { ba[e] = 0.f; bb[e] = 0.f; }
  const int bnch = n - p.bch_off;
  const bool bnb_on = p.part2 != nullptr && bnch >= 0 && bnch < p.bC;
  if (rl < RL) {
    for (long long row = r0 + rl; row < r1; row += RL) {
      float v[8];
      rowval(row, v);
      const int ph = (int)(row / p.M), m = (int)(row - (long long)ph * p.M);
      const int b = fast_div(m, GHW, p.inv_ghw), rem = m - b * GHW;
      const int y = fast_div(rem, p.GW, p.inv_gw), x = rem - y * p.GW;
      const int oy = y * p.os + p.oy0[ph], ox = x * p.os + p.ox0[ph];
      const long long off = (long long)b * p.c_bs + (long long)oy * p.c_rs + (long long)ox * p.c_ps + p.c_co + n;
      uint4 o;
      o.x = (unsigned)f2bf(v[0]) | ((unsigned)f2bf(v[1]) << 16);
      o.y = (unsigned)f2bf(v[2]) | ((unsigned)f2bf(v[3]) << 16);
      o.z = (unsigned)f2bf(v[4]) | ((unsigned)f2bf(v[5]) << 16);
      o.w = (unsigned)f2bf(v[6]) | ((unsigned)f2bf(v[7]) << 16);
      *reinterpret_cast<uint4*>(reinterpret_cast<bf16*>(p.c) + off) = o;
      if (bnb_on && oy < p.bxH && ox < p.bxW) {
        float vr[8];  // the bf16-rounded values, as a separate reduction pass would read them
        const unsigned w[4] = {o.x, o.y, o.z, o.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) { vr[2 * e] = __uint_as_float(w[e] << 16); vr[2 * e + 1] = __uint_as_float(w[e] & 0xffff0000u); }
        bnb_accum(p, b, oy, ox, bnch, vr, ba, bb);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float d = v[e] - sh[e];
        s1[e] += d;
        s2[e] += d * d;
      }
      cnt += 1.f;
    }
  }
  if (p.part2) {
    __shared__ float bred[256][16];
#pragma unroll
    for (int e = 0; e < 8; ++e) { bred[threadIdx.x][e] = ba[e]; bred[threadIdx.x][8 + e] = bb[e]; }
    __syncthreads();
    if (rl == 0 && bnb_on) {
      float ta[8], tb[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) { ta[e] = 0.f; tb[e] = 0.f; }
      for (int k = 0; k < RL; ++k) {
        const int t = k * CG + cg;
#pragma unroll
        for (int e = 0; e < 8; ++e) { ta[e] += bred[t][e]; tb[e] += bred[t][8 + e]; }
      }
#pragma unroll
      for (int e = 0; e < 8; ++e)
        *reinterpret_cast<float2*>(p.part2 + ((long long)blockIdx.x * p.bC + bnch + e) * 2) = make_float2(ta[e], tb[e]);
    }
  }
  if (!p.stats) return;
  __shared__ float red[2][256][8];
  __shared__ float rcnt[256];
#pragma unroll
  for (int e = 0; e < 8; ++e) { red[0][threadIdx.x][e] = s1[e]; red[1][threadIdx.x][e] = s2[e]; }
  rcnt[threadIdx.x] = cnt;
  __syncthreads();
  if (rl == 0) {
    float a1[8], a2[8], nn = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) { a1[e] = 0.f; a2[e] = 0.f; }
    for (int k = 0; k < RL; ++k) {
      const int t = k * CG + cg;
#pragma unroll
      for (int e = 0; e < 8; ++e) { a1[e] += red[0][t][e]; a2[e] += red[1][t][e]; }
      nn += rcnt[t];
    }
#pragma unroll
    for (int e = 0; e < 8; ++e)
      *reinterpret_cast<float4*>(p.stats + ((long long)blockIdx.x * p.N + n + e) * 4) = make_float4(nn, a1[e], a2[e], sh[e]);
  }
}

// The same reduction for few rows over many splits (the deep 1x1 - 4x4 layers): one wave per (row,
// 8-channel group), lane l summing splits l, l + 64, ... in order, then a fixed xor butterfly.  Every
// row is its own statistics chunk ({1, 0, 0, value}: Chan-mergeable) and, with the fused BN backward,
// its own {dn, dn * xhat} chunk -- so no block-level row reduction is needed.
__global__ void __launch_bounds__(256) splitk_reduce_wide_kernel(const GParams p) {
  const int CG = p.N / 8;
  const long long R = (long long)p.nphase * p.M;
  const long long unit = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (unit >= R * CG) return;
  const int lane = threadIdx.x & 63;
  const long long row = unit / CG;
  const int cg = (int)(unit - row * CG), n = cg * 8;
  const int ph = (int)(row / p.M), m = (int)(row - (long long)ph * p.M);
  const long long MN = (long long)p.M * p.N;
  const float* src = p.ws + ((long long)ph * p.ksplit * p.M + m) * p.N + n;
  float v[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = 0.f;
  for (int s = lane; s < p.ksplit; s += 64) {
    const float4 a = *reinterpret_cast<const float4*>(src + s * MN);
    const float4 b = *reinterpret_cast<const float4*>(src + s * MN + 4);
    v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w;
    v[4] += b.x; v[5] += b.y; v[6] += b.z; v[7] += b.w;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] += __shfl_xor(v[e], o, 64);
  if (lane != 0) return;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    if (p.bias) v[e] += p.bias[n + e];
    if (p.tanh_) v[e] = tanhf(v[e]);
  }
  const int GHW = p.GH * p.GW;
  const int b = fast_div(m, GHW, p.inv_ghw), rem = m - b * GHW;
  const int y = fast_div(rem, p.GW, p.inv_gw), x = rem - y * p.GW;
  const int oy = y * p.os + p.oy0[ph], ox = x * p.os + p.ox0[ph];
  const long long off = (long long)b * p.c_bs + (long long)oy * p.c_rs + (long long)ox * p.c_ps + p.c_co + n;
  uint4 o;
  o.x = pack_bf16x2(v[0], v[1]); o.y = pack_bf16x2(v[2], v[3]);
  o.z = pack_bf16x2(v[4], v[5]); o.w = pack_bf16x2(v[6], v[7]);
  *reinterpret_cast<uint4*>(reinterpret_cast<bf16*>(p.c) + off) = o;
  if (p.stats) {
#pragma unroll
    for (int e = 0; e < 8; ++e)
      *reinterpret_cast<float4*>(p.stats + (row * p.N + n + e) * 4) = make_float4(1.f, 0.f, 0.f, v[e]);
  }
  if (p.part2) {
    const int bnch = n - p.bch_off;
    if (bnch >= 0 && bnch < p.bC) {
      float ba[8], bb[8], vr[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) { ba[e] = 0.f; bb[e] = 0.f; }
      const unsigned w[4] = {o.x, o.y, o.z, o.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) { vr[2 * e] = __uint_as_float(w[e] << 16); vr[2 * e + 1] = __uint_as_float(w[e] & 0xffff0000u); }
      if (oy < p.bxH && ox < p.bxW) bnb_accum(p, b, oy, ox, bnch, vr, ba, bb);
#pragma unroll
      for (int e = 0; e < 8; ++e)
        *reinterpret_cast<float2*>(p.part2 + (row * p.bC + bnch + e) * 2) = make_float2(ba[e], bb[e]);
    }
  }
}

// ------------------------------------------------------------------------- host
struct BPlan {
  int cfg;  // index into the tile table
  int BM, BN, ksplit, kchunk, mtiles, ntiles;
};

struct TileCfg {
  int BM, BN, WM, WN, NST, BK;
};
static const TileCfg kTiles[] = {
    {128, 128, 2, 2, 2, 64},  // 0
    {256, 128, 2, 2, 2, 64},  // 1
    {128, 64, 2, 2, 2, 64},   // 2
    {256, 64, 4, 1, 2, 64},   // 3
    {64, 128, 1, 4, 2, 64},   // 4
    {64, 64, 2, 2, 2, 64},    // 5
    {256, 256, 2, 4, 2, 64},  // 6
    {128, 256, 2, 4, 2, 64},  // 7
    {128, 128, 2, 2, 3, 64},  // 8
    {128, 256, 2, 4, 3, 64},  // 9
    {64, 128, 1, 4, 3, 64},   // 10
    {128, 64, 2, 2, 3, 64},   // 11
    {64, 64, 2, 2, 3, 64},    // 12
    {256, 128, 4, 2, 3, 64},  // 13
    {256, 256, 2, 4, 4, 32},  // 14
    {256, 128, 4, 2, 4, 32},  // 15
    {128, 256, 2, 4, 4, 32},  // 16
    {128, 128, 2, 2, 4, 32},  // 17
    {128, 64, 2, 2, 4, 32},   // 18
    {64, 64, 2, 2, 4, 32},    // 19
    {128, 128, 2, 2, 3, 32},  // 20: 48 KiB -> 3 blocks/CU
    {128, 128, 2, 2, 2, 32},  // 21
    {256, 128, 4, 2, 3, 32},  // 22
    {128, 64, 2, 2, 3, 32},   // 23
    {128, 128, 2, 4, 2, 64},  // 24: 8 waves of 64x32 (4 waves per SIMD at 2 blocks per CU)
    {128, 128, 4, 2, 2, 64},  // 25: 8 waves of 32x64
    {128, 64, 4, 2, 2, 64},   // 26: 8 waves of 32x32
    {256, 128, 4, 4, 2, 64},  // 27: 16 waves of 64x32
    {128, 256, 4, 4, 2, 64},  // 28: 16 waves of 32x64
    {128, 128, 2, 2, 4, 64},  // 29: + 4 loader waves (LD), 4 stages
    {128, 128, 2, 2, 3, 64},  // 30: + 4 loader waves, 3 stages
    {256, 128, 4, 2, 3, 64},  // 31: + 4 loader waves, 3 stages (8 compute waves)
    {128, 64, 2, 2, 4, 64},   // 32: + 4 loader waves, 4 stages
    {128, 128, 2, 2, 2, 64},  // 33: + 2 loader waves, 2 stages (64 KiB: two blocks per CU, as config 0)
    {128, 64, 2, 2, 2, 64},   // 34: + 2 loader waves, 2 stages
    {128, 256, 2, 4, 2, 64},  // 35: + 2 loader waves, 2 stages
};
// loader waves of a configuration's blocks besides the WM*WN compute waves
static inline int tile_loaders(int cfg) { return cfg >= 33 ? 2 : (cfg >= 29 ? 4 : 0); }
constexpr int kNumTiles = sizeof(kTiles) / sizeof(kTiles[0]);

static size_t bf16_lds_bytes(int cfg) {
  const TileCfg& t = kTiles[cfg];
  size_t stage = (size_t)t.NST * (t.BM + t.BN) * t.BK * 2;
  // the epilogue's bf16 tile and, past it, the BatchNorm statistics' [WM][BN][4] merge area (igemm_epilogue)
  size_t epi = (size_t)t.BM * (t.BN * 2 + 16) + (size_t)t.WM * t.BN * 16;
  return std::max(stage, epi);
}

// In-launch split-K (igemm_bf16_body / splitk_combine) for the split layers that are not reduced by the wide kernel;
// false: every split layer takes the separate reduction launch (A/B)
static bool g_splitk_inlaunch = true;
extern "C" int stc_set_splitk_inlaunch(int on) {
  const int old = g_splitk_inlaunch ? 1 : 0;
  if (on >= 0) g_splitk_inlaunch = on != 0;
  return old;
}

// Tile / split-K choice (fitted to the sweep of scripts/tune_bf16.py over one train step, see
// profiles/): prefer the largest tile that still gives a full wave of workgroups (about one
// 8-wave block or two 4-wave blocks per CU), splitting K only when no tile does.
static BPlan bf16_plan(int M, int N, int K, int nphase, int force_cfg, int force_ks, bool allow_split) {
  BPlan pl{};
  auto tiles = [&](int c) { return (long long)cdiv(M, kTiles[c].BM) * cdiv(N, kTiles[c].BN) * nphase; };
  const int ksteps = cdiv(K, 64);
  int cfg = -1, ks = 1;
  if (force_cfg >= 0 && force_cfg < kNumTiles) {
    cfg = force_cfg;
    ks = force_ks > 0 ? force_ks : 1;
  } else {
    int order[5], no = 0;
    // (the loader-wave tiles 29 / 31 win these layers in isolation, profiles/r03/diag/loader_tiles_conv.log, but
    // lose 0.36 ms per train step in situ: one of their blocks fills a CU's LDS, so the side streams' kernels
    // cannot share it; they stay reachable through force_plan only)
    if (N >= 256) {
      if ((long long)M * nphase >= 8192 && K >= 8192) {
        order[0] = 6; order[1] = 7; order[2] = 0; order[3] = 4; order[4] = 5; no = 5;
      } else if ((long long)M * nphase >= 8192) { order[0] = 6; order[1] = 0; order[2] = 4; order[3] = 5; no = 4; }
      else { order[0] = 0; order[1] = 4; order[2] = 12; order[3] = 5; no = 4; }
    } else if (N >= 128) {
      order[0] = 0; order[1] = 4; order[2] = 5; no = 3;
    } else if (K <= 128) {  // first layers (Cin = 8): 3-stage BK = 32, 3-4 blocks per CU
      order[0] = 23; order[1] = 2; order[2] = 5; no = 3;
    } else if (K <= 512) {  // (Cin = 128 ConvT-geometry dgrads: the 3-stage BK = 32 128x64 tile, -9 %)
      order[0] = 23; order[1] = 2; order[2] = 5; no = 3;
    } else {  // (N = 64 ConvT d1: the 3-stage 128x64 tile, -4 % vs 64x64 in scripts/sweep_cfg.sh)
      order[0] = 11; order[1] = 5; order[2] = 2; no = 3;
    }
    for (int k = 1; k <= 8 && cfg < 0; k *= 2) {
      if (k > 1 && (ksteps / k < 8 || !allow_split)) break;
      for (int i = 0; i < no; ++i) {
        const int c = order[i];
        const long long need = (c == 6 || c == 7 || c == 9 || tile_loaders(c)) ? 240 : 400;
        if (tiles(c) * k >= need) { cfg = c; ks = k; break; }
      }
    }
    if (cfg < 0) {
      cfg = order[no - 1];
      ks = 1;
      // the 1x1 / 2x2 grids (<= 256 GEMM rows): up to 32 splits of >= 4 K-steps, reduced by
      // splitk_reduce_wide_kernel (deep-layer sweep, scripts/deep_sweep.py: 12.9 -> 9.2 us at 1x1)
      const bool tiny = (long long)M * nphase <= 256;
      const int kmax = tiny ? 32 : 8, smin = tiny ? 4 : 8;
      while (allow_split && tiles(cfg) * ks < 400 && ks < kmax && ksteps / (ks * 2) >= smin) ks *= 2;
    }
  }
  if (!allow_split) ks = 1;
  const TileCfg& t = kTiles[cfg];
  pl.cfg = cfg;
  pl.BM = t.BM;
  pl.BN = t.BN;
  pl.mtiles = cdiv(M, t.BM);
  pl.ntiles = cdiv(N, t.BN);
  pl.kchunk = cdiv(ksteps, ks) * 64;
  pl.ksplit = cdiv(K, pl.kchunk);
  return pl;
}

static int reduce_rows_per_block(long long rows, int N) {
  const int RL = 256 / (N / 8);
  long long blocks = std::min<long long>(1024, std::max<long long>(1, rows / std::max(RL, 4)));
  return (int)((rows + blocks - 1) / blocks);
}

}  // namespace stc

using namespace stc;

namespace stc {

struct Bf16Problem {
  int M, N, K, nphase;
  BPlan pl;
  bool vec_out;
  int64_t ws_bytes;
  int stats_chunks;
  int reduce_rows;
  bool wide;      // split-K reduction by splitk_reduce_wide_kernel (a chunk per row)
  bool inlaunch;  // split-K combined in the launch (GParams::slab / tickets): the tile statistics of one launch
};

// Ticket counters of the in-launch split-K.  A region belongs to one (device, stream, capture): launches on one stream
// run one after another and every launch leaves its counters zero, so eager launches on a stream share its region; a
// launch made while the stream is being captured gets a region of that capture (the graph's replays may run beside
// eager work on the same stream handle, or on another stream), kept for the process lifetime.  The pool is allocated
// and zeroed once, outside any capture, by the first split-K launch of the device (its stream waits for the zeroing:
// no device-wide synchronisation); regions need no zeroing of their own.  (A per-region hipMemsetAsync captured into
// the graph left a replay launched on another stream with stale counters on this ROCm -- no tile finished.)
constexpr int kTicketRegion = 4096, kTicketRegions = 512;  // (8 MiB per device: streams are pooled)
static unsigned* splitk_tickets(hipStream_t st, int tiles) {
  static std::mutex mu;
  static std::map<std::tuple<int, uintptr_t, unsigned long long>, int> region;  // (device, stream, capture) -> region
  static unsigned* pool[64] = {};
  static int used[64] = {};
  if (tiles > kTicketRegion) return nullptr;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  unsigned long long cap_id = 0;
  if (hipStreamGetCaptureInfo(st, &cs, &cap_id) != hipSuccess) return nullptr;
  const unsigned long long cap = cs == hipStreamCaptureStatusActive ? cap_id + 1 : 0;
  std::lock_guard<std::mutex> lk(mu);
  if (!pool[dev]) {
    if (cs != hipStreamCaptureStatusNone) return nullptr;
    void* q = nullptr;
    const size_t bytes = (size_t)kTicketRegion * kTicketRegions * sizeof(unsigned);
    if (hipMalloc(&q, bytes) != hipSuccess) return nullptr;
    if (hipMemsetAsync(q, 0, bytes, st) != hipSuccess || hipStreamSynchronize(st) != hipSuccess) return nullptr;
    pool[dev] = (unsigned*)q;
  }
  const auto key = std::make_tuple(dev, (uintptr_t)st, cap);
  auto it = region.find(key);
  if (it != region.end()) return pool[dev] + (size_t)it->second * kTicketRegion;
  if (used[dev] >= kTicketRegions) return nullptr;
  region[key] = used[dev];
  return pool[dev] + (size_t)used[dev]++ * kTicketRegion;
}

// Shared planning for query and launch.
static Bf16Problem bf16_problem(int M, int N, int K, int nphase, const int32_t* force, bool vec_out) {
  Bf16Problem pr{};
  pr.M = M; pr.N = N; pr.K = K; pr.nphase = nphase;
  pr.pl = bf16_plan(M, N, K, nphase, force ? force[0] : -1, force ? force[1] : 0, vec_out);
  pr.vec_out = vec_out;
  if (pr.pl.ksplit > 1) {
    pr.ws_bytes = (int64_t)nphase * pr.pl.ksplit * (int64_t)M * N * 4;
    const long long rows = (long long)nphase * M;
    pr.wide = pr.pl.ksplit >= 16 && rows * (N / 8) <= 16384;  // a wave per unit pays off with >= 16 splits
    pr.reduce_rows = reduce_rows_per_block(rows, N);
    pr.stats_chunks = pr.wide ? (int)rows : (int)((rows + pr.reduce_rows - 1) / pr.reduce_rows);
    const long long tiles = (long long)nphase * pr.pl.mtiles * pr.pl.ntiles;
    // (up to 4 splits: with 8 the last arrivers' slab reads outweigh the reduction launch -- the 4 x 4 / 2 x 2 deep
    // layers measured 22.0 / 16.1 us in-launch against 13.7 + 6.6 / 6.6 + 6.3 us with the reduction kernel)
    pr.inlaunch = g_splitk_inlaunch && !pr.wide && vec_out && pr.pl.ksplit <= 4 && tiles <= kTicketRegion;
    if (pr.inlaunch) {
      pr.ws_bytes = tiles * pr.pl.ksplit * (int64_t)pr.pl.BM * pr.pl.BN * 4;
      pr.stats_chunks = nphase * pr.pl.mtiles;
    }
  } else {
    pr.ws_bytes = 0;
    pr.stats_chunks = nphase * pr.pl.mtiles;
  }
  return pr;
}

bool bf16_igemm_eligible(int N, int K) { return N >= 16 && N % 8 == 0 && N <= 2048 && K % 8 == 0; }

int bf16_igemm_query(int M, int N, int K, int nphase, const int32_t* force, int64_t* ws_bytes, int32_t* stats_chunks,
                     int32_t* plan_out) {
  Bf16Problem pr = bf16_problem(M, N, K, nphase, force, true);
  if (ws_bytes) *ws_bytes = pr.ws_bytes;
  if (stats_chunks) *stats_chunks = pr.stats_chunks;
  if (plan_out) {
    plan_out[0] = pr.pl.BM; plan_out[1] = pr.pl.BN; plan_out[2] = pr.pl.ksplit; plan_out[3] = 0;
    plan_out[4] = pr.pl.cfg;
  }
  return 0;
}

// p: filled by the caller (geometry, operands, output); returns 0 or error.

int bf16_igemm_launch(GParams& p, const int32_t* force, void* ws, int64_t ws_bytes, float* stats, int stats_chunks,
                      hipStream_t st) {
  Bf16Problem pr = bf16_problem(p.M, p.N, p.K, p.nphase, force, p.vec_out != 0);
  const BPlan& pl = pr.pl;
  p.ksplit = pl.ksplit; p.kchunk = pl.kchunk; p.mtiles = pl.mtiles; p.ntiles = pl.ntiles;
  p.stats = nullptr;
  p.ws = nullptr;
  float* part2 = p.part2;
  p.slab = nullptr;
  p.tickets = nullptr;
  p.acquire = 0;
  if (pl.ksplit > 1) {
    STC_REQUIRE(ws && ws_bytes >= pr.ws_bytes, "bf16 igemm: workspace %lld < %lld bytes", (long long)ws_bytes,
                (long long)pr.ws_bytes);
    if (pr.inlaunch) {
      p.tickets = splitk_tickets(st, pl.mtiles * pl.ntiles * p.nphase);
      STC_REQUIRE(p.tickets, "bf16 igemm: no split-K ticket region for this stream (first use inside a capture?)");
      p.slab = (float*)ws;
      p.acquire = 1;
      p.stats = stats;  // (the last arriver's epilogue: tile statistics / fused BN-backward sums)
    } else {
      p.ws = (float*)ws;
      p.part2 = nullptr;  // computed by the split-K reduction
    }
  } else {
    p.stats = stats;
  }
  if (stats || part2)
    STC_REQUIRE(stats_chunks == pr.stats_chunks, "bf16 igemm: stats chunks %d != %d (query again after changing the "
                "split-K mode)", stats_chunks, pr.stats_chunks);
  p.phase_major = (p.nphase > 1 && pl.ksplit == 1) ? 1 : 0;
  dim3 grid = p.phase_major ? dim3(pl.mtiles * pl.ntiles * p.nphase, 1, 1)
                            : dim3(pl.mtiles * pl.ntiles, 1, p.nphase * pl.ksplit);
  const size_t lds = bf16_lds_bytes(pl.cfg);
#define STC_B(I, BM_, BN_, WM_, WN_, NST_, BK_)                                                             \
  case I:                                                                                                   \
    if (p.part2)                                                                                            \
      hipLaunchKernelGGL((igemm_bf16_kernel<BM_, BN_, WM_, WN_, NST_, BK_, true>), grid, dim3(64 * WM_ * WN_), lds, st, p); \
    else                                                                                                    \
      hipLaunchKernelGGL((igemm_bf16_kernel<BM_, BN_, WM_, WN_, NST_, BK_, false>), grid, dim3(64 * WM_ * WN_), lds, st, p); \
    break;
#define STC_BL(I, BM_, BN_, WM_, WN_, NST_, BK_, LD_)                                                       \
  case I:                                                                                                   \
    if (p.part2)                                                                                            \
      hipLaunchKernelGGL((igemm_bf16_ld_kernel<BM_, BN_, WM_, WN_, NST_, BK_, true, LD_>), grid, dim3(64 * (WM_ * WN_ + LD_)), lds, st, p); \
    else                                                                                                    \
      hipLaunchKernelGGL((igemm_bf16_ld_kernel<BM_, BN_, WM_, WN_, NST_, BK_, false, LD_>), grid, dim3(64 * (WM_ * WN_ + LD_)), lds, st, p); \
    break;
  main_timer_begin(st);
  switch (pl.cfg) {
    STC_B(0, 128, 128, 2, 2, 2, 64)
    STC_B(1, 256, 128, 2, 2, 2, 64)
    STC_B(2, 128, 64, 2, 2, 2, 64)
    STC_B(3, 256, 64, 4, 1, 2, 64)
    STC_B(4, 64, 128, 1, 4, 2, 64)
    STC_B(5, 64, 64, 2, 2, 2, 64)
    STC_B(6, 256, 256, 2, 4, 2, 64)
    STC_B(7, 128, 256, 2, 4, 2, 64)
    STC_B(8, 128, 128, 2, 2, 3, 64)
    STC_B(9, 128, 256, 2, 4, 3, 64)
    STC_B(10, 64, 128, 1, 4, 3, 64)
    STC_B(11, 128, 64, 2, 2, 3, 64)
    STC_B(12, 64, 64, 2, 2, 3, 64)
    STC_B(13, 256, 128, 4, 2, 3, 64)
    STC_B(14, 256, 256, 2, 4, 4, 32)
    STC_B(15, 256, 128, 4, 2, 4, 32)
    STC_B(16, 128, 256, 2, 4, 4, 32)
    STC_B(17, 128, 128, 2, 2, 4, 32)
    STC_B(18, 128, 64, 2, 2, 4, 32)
    STC_B(19, 64, 64, 2, 2, 4, 32)
    STC_B(20, 128, 128, 2, 2, 3, 32)
    STC_B(21, 128, 128, 2, 2, 2, 32)
    STC_B(22, 256, 128, 4, 2, 3, 32)
    STC_B(23, 128, 64, 2, 2, 3, 32)
    STC_B(24, 128, 128, 2, 4, 2, 64)
    STC_B(25, 128, 128, 4, 2, 2, 64)
    STC_B(26, 128, 64, 4, 2, 2, 64)
    STC_B(27, 256, 128, 4, 4, 2, 64)
    STC_B(28, 128, 256, 4, 4, 2, 64)
    STC_BL(29, 128, 128, 2, 2, 4, 64, 4)
    STC_BL(30, 128, 128, 2, 2, 3, 64, 4)
    STC_BL(31, 256, 128, 4, 2, 3, 64, 4)
    STC_BL(32, 128, 64, 2, 2, 4, 64, 4)
    STC_BL(33, 128, 128, 2, 2, 2, 64, 2)
    STC_BL(34, 128, 64, 2, 2, 2, 64, 2)
    STC_BL(35, 128, 256, 2, 4, 2, 64, 2)
    default:
      return fail(-1, "bf16 igemm: bad tile config %d", pl.cfg);
  }
#undef STC_B
#undef STC_BL
  main_timer_end(st);
  STC_CHECK_LAUNCH();
  if (pl.ksplit > 1 && !pr.inlaunch) {
    STC_REQUIRE(p.vec_out, "bf16 igemm: split-K needs a 16-byte aligned NHWC bf16 output");
    p.stats = stats;
    p.part2 = part2;
    const long long rows = (long long)p.nphase * p.M;
    if (pr.wide) {
      const long long units = rows * (p.N / 8);
      hipLaunchKernelGGL(splitk_reduce_wide_kernel, dim3((unsigned)((units + 3) / 4)), dim3(256), 0, st, p);
    } else {
      const int blocks = (int)((rows + pr.reduce_rows - 1) / pr.reduce_rows);
      hipLaunchKernelGGL(splitk_reduce_stats_kernel, dim3(blocks), dim3(256), 0, st, p, pr.reduce_rows);
    }
    STC_CHECK_LAUNCH();
  }
  return 0;
}

// ---- conv-level wrappers (geometry -> GParams), used by stc_conv_fwd_query / stc_conv_fwd_ex
static bool vec_out_ok(int B, const stc_view& y, int Cout, int out_f32) {
  const long long extent = (long long)(B - 1) * y.bs + (long long)(y.H - 1) * y.rs + (long long)(y.W - 1) * y.ps + y.co + Cout;
  return !out_f32 && y.cs == 1 && y.co % 8 == 0 && y.ps % 8 == 0 && y.rs % 8 == 0 && y.bs % 8 == 0 &&
         ((uintptr_t)y.p & 15) == 0 && extent < (1ll << 31);
}

bool bf16_conv_eligible(int kind, int B, const stc_view& x, int Cin, int Cout) {
  const Geometry g = geometry(kind);
  const int taps = g.taps_lg_tw == 2 ? 16 : 4;
  const long long a_bytes = (long long)B * x.bs * 2;
  const long long b_bytes = (long long)g.nphase * Cout * taps * Cin * 2;
  return bf16_igemm_eligible(Cout, taps * Cin) && Cin % 8 == 0 && x.cs == 1 && x.co % 8 == 0 && x.ps % 8 == 0 &&
         a_bytes < (1ll << 31) && b_bytes < (1ll << 31);
}

// The conv-s2 halo kernel (halo_bf16.hip): plan config HALO_CFG.  force_plan: NULL / {-1, .}: automatic (the
// halo kernel where eligible), {HALO_CFG, .}: the halo kernel (an error where it is not eligible), {-2, .}: the
// automatic im2col plan (A/B), {cfg >= 0, .}: that im2col tile.
constexpr int HALO_CFG = 100;
bool halo_geometry_ok(int kind, int B, int GH, int GW, int Cin, int Cout);
bool halo_auto(int kind, int B, int GH, int GW, int Cin, int Cout);
bool halo_eligible(int kind, int B, const stc_view& x, int Cin, int Cout, const stc_view& y);
int halo_chunks(int kind, int B, int GH, int GW);
int halo_launch(GParams& p, hipStream_t st, int shape);
int halo_plan_bn(int kind, int B, int GH, int GW, int Cout, int shape);
// the Cin = 8 first layers with the activation epilogue (stem_bf16.hip)
bool stem_eligible(int kind, int B, const stc_view& x, int Cin, int Cout, const stc_view& y, bool bnb);
int stem_launch(GParams& p, hipStream_t st);
bool stem_s1d_eligible(int kind, int B, const stc_view& dy, int Cin, int Cout, const stc_view& y);
int stem_s1d_launch(GParams& p, hipStream_t st);
int stem_bnb_chunks(int kind, int B, int Hg, int Wg, int Cin, int Cout);
static bool halo_plan(const int32_t* force, int kind, int B, int GH, int GW, int Cin, int Cout) {
  if (force && force[0] == HALO_CFG) return halo_geometry_ok(kind, B, GH, GW, Cin, Cout);
  return (!force || force[0] == -1) && halo_auto(kind, B, GH, GW, Cin, Cout);
}

int bf16_conv_query(int kind, int B, int Hg, int Wg, int Cin, int Cout, int out_f32, const int32_t* force,
                    int64_t* ws_bytes, int32_t* stats_chunks, int32_t* plan_out) {
  if (!out_f32 && halo_plan(force, kind, B, Hg, Wg, Cin, Cout)) {
    if (ws_bytes) *ws_bytes = 0;
    if (stats_chunks) *stats_chunks = halo_chunks(kind, B, Hg, Wg);
    if (plan_out) {
      plan_out[0] = 256; plan_out[1] = halo_plan_bn(kind, B, Hg, Wg, Cout, force && force[0] == HALO_CFG ? force[1] : 0); plan_out[2] = 1; plan_out[3] = 0;
      plan_out[4] = HALO_CFG;
    }
    return 0;
  }
  if (force && force[0] == HALO_CFG) force = nullptr;
  const Geometry g = geometry(kind);
  const int taps = g.taps_lg_tw == 2 ? 16 : 4;
  Bf16Problem pr = bf16_problem(B * Hg * Wg, Cout, taps * Cin, g.nphase, force, !out_f32);
  if (ws_bytes) *ws_bytes = pr.ws_bytes;
  if (stats_chunks) *stats_chunks = pr.stats_chunks;
  if (plan_out) {
    plan_out[0] = pr.pl.BM; plan_out[1] = pr.pl.BN; plan_out[2] = pr.pl.ksplit; plan_out[3] = 0;
    plan_out[4] = pr.pl.cfg;
  }
  return 0;
}

int bf16_conv_fwd(int kind, int B, stc_view x, int Cin, const void* w_packed, int Cout, stc_view y,
                  const float* bias, int epi_tanh, int out_f32, float* stats, int stats_chunks,
                  const int32_t* force, void* ws, int64_t ws_bytes, hipStream_t st,
                  const stc_bnb_fuse* bnb = nullptr, float* part2 = nullptr,
                  const stc_view* act2 = nullptr, int act_n = 0, float act_s1 = 0.f, float act_s2 = 0.f,
                  int bnb_act = 0) {
  const Geometry g = geometry(kind);
  const int taps = g.taps_lg_tw == 2 ? 16 : 4;
  GParams p{};
  p.a = (const char*)x.p;
  p.a_bytes = (unsigned)((long long)B * x.bs * 2);
  p.a_bs = (int)x.bs; p.a_rs = (int)x.rs; p.a_ps = x.ps; p.a_co = x.co;
  p.IH = x.H; p.IW = x.W;
  p.cin = Cin; p.lg_tw = g.taps_lg_tw; p.in_stride = g.in_stride;
  for (int i = 0; i < 4; ++i) { p.offy[i] = g.offy[i]; p.offx[i] = g.offx[i]; }
  p.stepy = g.stepy; p.stepx = g.stepx;
  if (kind == STC_CONVT_S2) { p.GH = x.H; p.GW = x.W; }
  else { p.GH = y.H; p.GW = y.W; }
  p.M = B * p.GH * p.GW; p.N = Cout; p.K = taps * Cin;
  STC_REQUIRE(p.M < (1 << 24), "bf16 conv: M = %d pixels per phase (>= 2^24)", p.M);
  p.inv_ghw = 1.0f / (float)(p.GH * p.GW);
  p.inv_gw = 1.0f / (float)p.GW;
  p.b = (const char*)w_packed;
  p.b_phase_stride = Cout * p.K;
  p.b_bytes = (unsigned)((long long)g.nphase * p.b_phase_stride * 2);
  p.c = (char*)y.p; p.c_bs = y.bs; p.c_rs = y.rs; p.c_ps = y.ps; p.c_co = y.co; p.c_cs = y.cs;
  p.os = g.os;
  for (int i = 0; i < 4; ++i) { p.oy0[i] = g.nphase == 4 ? (i >> 1) : 0; p.ox0[i] = g.nphase == 4 ? (i & 1) : 0; }
  p.bias = bias; p.tanh_ = epi_tanh; p.out_f32 = out_f32;
  p.vec_out = vec_out_ok(B, y, Cout, out_f32) && Cout % 8 == 0 ? 1 : 0;
  p.nphase = g.nphase;
  if (p.M == 0 || Cout == 0) return 0;
  STC_REQUIRE(!epi_tanh, "bf16 conv: the MFMA tile kernel has no tanh epilogue");
  if (!p.vec_out) STC_REQUIRE(!stats || out_f32 == 0, "bf16 conv: stats need a bf16 output");
  if (bnb) {
    STC_REQUIRE(p.vec_out && (part2 || bnb_act) && !stats, "bf16 conv: fused BN backward needs a 16-byte NHWC bf16 output");
    STC_REQUIRE(bnb->C % 8 == 0 && bnb->ch_off % 8 == 0 && bnb->x.cs == 1 && bnb->x.co % 8 == 0 && bnb->x.ps % 8 == 0 &&
                    (!bnb->g_other.p || (bnb->g_other.cs == 1 && bnb->g_other.co % 8 == 0 && bnb->g_other.ps % 8 == 0)) &&
                    (bnb_act || (bnb->scale && bnb->shift && bnb->mean && bnb->rstd)),
                "bf16 conv: bad fused BN-backward arguments");
    p.bnb_act = bnb_act;
    p.part2 = part2;
    p.bx = (const char*)bnb->x.p; p.bx_bs = bnb->x.bs; p.bx_rs = bnb->x.rs; p.bx_ps = bnb->x.ps; p.bx_co = bnb->x.co;
    p.bxH = bnb->x.H; p.bxW = bnb->x.W;
    p.bg = (const char*)bnb->g_other.p; p.bg_bs = bnb->g_other.bs; p.bg_rs = bnb->g_other.rs; p.bg_ps = bnb->g_other.ps;
    p.bg_co = bnb->g_other.co;
    p.bsc = bnb->scale; p.bsh = bnb->shift; p.bmu = bnb->mean; p.brs = bnb->rstd;
    p.bs_self = bnb->slope_self; p.bs_other = bnb->slope_other;
    p.bC = bnb->C; p.bch_off = bnb->ch_off;
  }
  if (act_n) {
    STC_REQUIRE(p.vec_out && !bnb && !stats && (act_n == 1 || (act2 && act2->p)),
                "bf16 conv: activation epilogue needs a 16-byte NHWC bf16 output and no statistics");
    p.act_n = act_n; p.act_s1 = act_s1; p.act_s2 = act_s2;
    if (act_n == 2) {
      p.c2 = (char*)act2->p; p.c2_bs = act2->bs; p.c2_rs = act2->rs; p.c2_ps = act2->ps; p.c2_co = act2->co;
    }
  }
  if (bnb_act) {  // (the halo kernels' epilogue only: stc_conv_bwd_act_ok)
    STC_REQUIRE(!force && !part2 && bnb->C == Cout && bnb->ch_off == 0 && halo_plan(nullptr, kind, B, p.GH, p.GW, Cin, Cout) &&
                    halo_eligible(kind, B, x, Cin, Cout, y),
                "bf16 conv: no fused activation backward for this shape / view (check stc_conv_bwd_act_ok)");
    p.ws = nullptr;
    return halo_launch(p, st, 0);
  }
  if (p.vec_out && !force && !stats && bnb && !bnb->g_other.p && stem_s1d_eligible(kind, B, x, Cin, Cout, y)) {
    p.ws = nullptr;
    return stem_s1d_launch(p, st);
  }
  if (p.vec_out && !force && !stats && (act_n || bnb) && stem_eligible(kind, B, x, Cin, Cout, y, bnb != nullptr)) {
    p.ws = nullptr;
    return stem_launch(p, st);
  }
  if (!act_n && p.vec_out && halo_plan(force, kind, B, p.GH, p.GW, Cin, Cout) && halo_eligible(kind, B, x, Cin, Cout, y)) {
    const int need = halo_chunks(kind, B, p.GH, p.GW);
    if (stats || part2) STC_REQUIRE(stats_chunks == need, "bf16 conv: stats chunks %d != %d", stats_chunks, need);
    p.stats = stats;
    p.ws = nullptr;
    return halo_launch(p, st, force && force[0] == HALO_CFG ? force[1] : 0);
  }
  STC_REQUIRE(!(force && force[0] == HALO_CFG), "bf16 conv: the halo kernel does not take this shape / view");
  return bf16_igemm_launch(p, force, ws, ws_bytes, stats, stats_chunks, st);
}

// The fused activation backward (stc_conv_bwd_act) runs in the halo kernels' BN-backward epilogue: the layer takes
// the halo route with 16-byte NHWC bf16 views of one extent.
bool bf16_conv_bwd_act_ok(int kind, int B, const stc_view& dy, int Cin, int Cout, const stc_view& out, const stc_view& x,
                          const stc_view* g_other) {
  if (!bf16_conv_eligible(kind, B, dy, Cin, Cout) || !vec_out_ok(B, out, Cout, 0) || Cout % 8 != 0) return false;
  const int Hg = kind == STC_CONVT_S2 ? dy.H : out.H, Wg = kind == STC_CONVT_S2 ? dy.W : out.W;
  if (!halo_plan(nullptr, kind, B, Hg, Wg, Cin, Cout) || !halo_eligible(kind, B, dy, Cin, Cout, out)) return false;
  auto vec = [&](const stc_view& v) {
    return v.H == out.H && v.W == out.W && v.cs == 1 && v.co % 8 == 0 && v.ps % 8 == 0 && v.rs % 8 == 0 && v.bs % 8 == 0 &&
           ((uintptr_t)v.p & 15) == 0 && (long long)B * v.bs < (1ll << 31);
  };
  return x.p && vec(x) && (!g_other || !g_other->p || vec(*g_other));
}

// Partial count of the fused BN-backward sums for these views: the route bf16_conv_fwd takes for a BN-backward
// call (no statistics, no forced plan) -- the streaming logits-gradient kernel, the streaming Cin = 8 kernel, the
// halo kernel or the im2col tile -- decides it, so views that one of the streaming / halo kernels does not take
// (not dense at channel offset 0, a second gradient for the 31 x 31 layer) get the chunk count of the kernel that
// then runs, not the shape's default.
int bf16_bnb_chunks(int kind, int B, const stc_view& x, int Cin, int Cout, const stc_view& y, bool g_other) {
  const int Hg = kind == STC_CONVT_S2 ? x.H : y.H, Wg = kind == STC_CONVT_S2 ? x.W : y.W;
  if (!g_other && stem_s1d_eligible(kind, B, x, Cin, Cout, y)) return stem_bnb_chunks(kind, B, Hg, Wg, Cin, Cout);
  if (stem_eligible(kind, B, x, Cin, Cout, y, true)) return stem_bnb_chunks(kind, B, Hg, Wg, Cin, Cout);
  if (halo_plan(nullptr, kind, B, Hg, Wg, Cin, Cout) && halo_eligible(kind, B, x, Cin, Cout, y))
    return halo_chunks(kind, B, Hg, Wg);
  const Geometry g = geometry(kind);
  const int taps = g.taps_lg_tw == 2 ? 16 : 4;
  return bf16_problem(B * Hg * Wg, Cout, taps * Cin, g.nphase, nullptr, true).stats_chunks;
}

// The activation epilogue applies when the layer runs as one LDS-DMA GEMM launch (no split-K) with 16-byte
// NHWC bf16 views for both outputs.
bool bf16_conv_act_ok(int kind, int B, const stc_view& x, int Cin, int Cout, const stc_view& y1, const stc_view* y2) {
  if (!bf16_conv_eligible(kind, B, x, Cin, Cout) || !vec_out_ok(B, y1, Cout, 0) || Cout % 8 != 0) return false;
  if (y2 && y2->p && (!vec_out_ok(B, *y2, Cout, 0) || y2->H != y1.H || y2->W != y1.W)) return false;
  const Geometry g = geometry(kind);
  const int taps = g.taps_lg_tw == 2 ? 16 : 4;
  const int Hg = kind == STC_CONVT_S2 ? x.H : y1.H, Wg = kind == STC_CONVT_S2 ? x.W : y1.W;
  const Bf16Problem pr = bf16_problem(B * Hg * Wg, Cout, taps * Cin, g.nphase, nullptr, true);
  return pr.pl.ksplit == 1;
}

}  // namespace stc
