// BatchNorm finalize inside the kernel that produces the statistics partials (no stc_bn_finalize /
// bwd-finalize launch on the chain: STCGAN/networks.py:107,109,170,179 forward, their backward).
//
// Every block of the producer writes its chunk partials for a channel range [c0, c1), then draws a
// ticket on the counter of its chunk group (GS consecutive chunks x one channel tile); the block that
// draws the group's last ticket merges the group's chunks in chunk order into a level-2 partial, and
// the block that draws the last level-2 ticket of the channel tile merges the level-2 partials in group
// order and writes the finalized tables.  Fixed merge order at both levels: deterministic.
// Hand-off (MI355X_MICROARCH.md "Workgroup dispatch ... inter-workgroup visibility", the counter
// form of cdna_hip_programming.md G16 with R1 payload stores): write-through (sc1) partial stores ->
// every wave's vmcnt(0) -> barrier -> one lane's relaxed agent fetch_add; the last arriver resets the
// counter (every arrival of this launch has happened), takes an agent acquire fence and vmcnt(0), and
// the block reads the partials after a barrier.  Counters are zero-initialised once by the caller and
// left at zero by every launch, so calls sharing a counter buffer must be stream-ordered.
#pragma once
#include "common.hpp"

namespace stc {

constexpr int BNFIN_L1 = 1024;     // level-1 counters (groups x channel tiles)
constexpr int BNFIN_L2 = 16;       // level-2 counters (channel tiles)
constexpr int BNFIN_MAXG = 64;     // chunk groups

struct BnFin {
  unsigned* counters;  // [BNFIN_L1 + BNFIN_L2], zero between launches
  float* scratch;      // [BNFIN_MAXG][C][4] level-2 partials
  int gs, ngroups;     // chunk group size, groups
  // forward (statistics {n, S1, S2, shift} -> tables); null mean_o/scale: backward sums
  const float *gamma, *beta;
  float *rmean, *rvar;
  long long* nbt;
  float momentum, eps;
  float *mean_o, *rstd_o, *scale, *shift;
  // backward ({sum dn, sum dn*xhat} -> dbeta, dgamma)
  float *dgamma, *dbeta;
};

// Write-through (sc1) stores of handed-off partials (cdna_hip_programming.md G16 R1: no release fence needed):
// 8-byte relaxed agent-scope atomic stores.
__device__ __forceinline__ void wt_store2(float* p, float a, float b) {
  const unsigned long long v = (unsigned long long)__float_as_uint(a) | ((unsigned long long)__float_as_uint(b) << 32);
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void wt_store4(float* p, float4 v) {
  wt_store2(p, v.x, v.y);
  wt_store2(p + 2, v.z, v.w);
}

// host: chunk grouping for nchunks partials
inline void bnfin_groups(int nchunks, int* gs, int* ngroups) {
  int g = nchunks <= 32 ? nchunks : 32;
  while ((nchunks + g - 1) / g > BNFIN_MAXG) g *= 2;
  *gs = g < 1 ? 1 : g;
  *ngroups = (nchunks + *gs - 1) / *gs;
}

// mean / rstd / affine table / running statistics of channel c from the merged N, mean, M2
__device__ __forceinline__ void bn_finalize_store(int c, double N, double mu, double M2, const float* gamma,
                                                  const float* beta, float* rmean, float* rvar, long long* nbt,
                                                  float momentum, float eps, float* mean_o, float* rstd_o,
                                                  float* scale, float* shift) {
  const double var = N > 0 ? M2 / N : 0.0;
  const float rs = (float)(1.0 / sqrt(var + (double)eps));
  const float g = gamma ? gamma[c] : 1.f, bt = beta ? beta[c] : 0.f;
  if (mean_o) mean_o[c] = (float)mu;
  if (rstd_o) rstd_o[c] = rs;
  const float sc = g * rs;
  scale[c] = sc;
  shift[c] = bt - (float)mu * sc;
  if (rmean) rmean[c] = (1.f - momentum) * rmean[c] + momentum * (float)mu;
  if (rvar) rvar[c] = (1.f - momentum) * rvar[c] + momentum * (float)(N > 1 ? M2 / (N - 1) : var);
  if (nbt && c == 0) nbt[0] += 1;
}

// One ticket on *ctr; true (in every thread of the block) for the block drawing ticket expected-1.
// The partials were stored write-through (wt_store*), so every wave drains its stores (vmcnt(0)) and the
// block's barrier orders them before the ticket -- no release fence (a buffer_wbl2 per block wrote back
// the whole XCD L2, output tiles included: +2.3 ms per train step).  flag: one int of LDS.
__device__ __forceinline__ bool bnfin_ticket(unsigned* ctr, unsigned expected, int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = t == expected - 1;
    if (last) {
      __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    *flag = last;
  }
  __syncthreads();
  const bool last = *flag != 0;
  __syncthreads();  // the flag word may be reused by the caller
  return last;
}

// ---- block-parallel merges.  Channels [c0, c1) are taken blockDim at a time; the T = blockDim / nc threads
// of a channel stride over the chunks (thread j: chunks k0 + j, k0 + j + T, ...), and their partial sums
// are combined through LDS in j order -- a fixed order, so the result is deterministic.  red: LDS,
// >= 2 * blockDim doubles.

// sum over the T threads of each channel (a, b) -> returned in thread j == 0 (others: undefined)
__device__ __forceinline__ void bnfin_combine(double& a, double& b, int ci, int j, int nc, int T, double* red) {
  const int NT = blockDim.x;
  red[threadIdx.x] = a;
  red[NT + threadIdx.x] = b;
  __syncthreads();
  if (j == 0) {
    double sa = 0, sb = 0;
    for (int i = 0; i < T; ++i) { sa += red[i * nc + ci]; sb += red[NT + i * nc + ci]; }
    a = sa;
    b = sb;
  }
  __syncthreads();
}

// Forward statistics {n, S1, S2, shift} of chunks [k0, k1) (chunk mean m = shift + S1/n, chunk
// M2 = S2 - S1^2/n), merged exactly in two passes (N, mean = sum n m / N; M2 = sum [M2_b + n (m - mean)^2]).
// emit(c, N, mean, M2) runs in one thread per channel.
template <typename Emit>
__device__ __forceinline__ void bnfin_merge_stats(const float* part, int C, int k0, int k1, int c0, int c1, double* red,
                                                  Emit emit) {
  const int NT = blockDim.x;
  for (int cb = c0; cb < c1; cb += NT) {
    const int nc = min(NT, c1 - cb), T = NT / nc;
    const int ci = (int)threadIdx.x % nc, j = (int)threadIdx.x / nc;
    const bool act = j < T;
    const int c = cb + ci;
    double n = 0, s = 0;
    if (act) {
      for (int kb = k0 + j; kb < k1; kb += 8 * T) {
        float4 q[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int k = kb + u * T;
          q[u] = k < k1 ? *reinterpret_cast<const float4*>(part + ((long long)k * C + c) * 4) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          if (q[u].x <= 0.f) continue;
          n += q[u].x;
          s += (double)q[u].x * q[u].w + (double)q[u].y;  // n m = n shift + S1
        }
      }
    }
    bnfin_combine(n, s, ci, j, nc, T, red);
    if (act && j == 0) red[ci] = n > 0 ? s / n : 0.0;  // the channel mean, shared through LDS
    __syncthreads();
    const double mean = act ? red[ci] : 0.0;
    __syncthreads();
    double m2 = 0, dummy = 0;
    if (act) {
      for (int kb = k0 + j; kb < k1; kb += 8 * T) {
        float4 q[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int k = kb + u * T;
          q[u] = k < k1 ? *reinterpret_cast<const float4*>(part + ((long long)k * C + c) * 4) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          if (q[u].x <= 0.f) continue;
          const double nb = q[u].x, s1 = q[u].y, r = (double)(q[u].y / q[u].x);
          double qb = (double)q[u].z - s1 * r;
          if (qb < 0) qb = 0;
          const double d = (double)q[u].w + r - mean;
          m2 += qb + nb * d * d;
        }
      }
    }
    bnfin_combine(m2, dummy, ci, j, nc, T, red);
    if (act && j == 0) emit(c, n, mean, m2);
    __syncthreads();
  }
}

// Backward sums of chunks [k0, k1): load(k, c) -> {sum dn, sum dn*xhat} of chunk k; emit(c, a, b) in one
// thread per channel.
template <typename Load, typename Emit>
__device__ __forceinline__ void bnfin_merge_sums(int k0, int k1, int c0, int c1, double* red, Load load, Emit emit) {
  const int NT = blockDim.x;
  for (int cb = c0; cb < c1; cb += NT) {
    const int nc = min(NT, c1 - cb), T = NT / nc;
    const int ci = (int)threadIdx.x % nc, j = (int)threadIdx.x / nc;
    const bool act = j < T;
    const int c = cb + ci;
    double a = 0, b = 0;
    if (act) {
      for (int kb = k0 + j; kb < k1; kb += 8 * T) {
        double2 q[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int k = kb + u * T;
          q[u] = k < k1 ? load(k, c) : make_double2(0.0, 0.0);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) { a += q[u].x; b += q[u].y; }
      }
    }
    bnfin_combine(a, b, ci, j, nc, T, red);
    if (act && j == 0) emit(c, a, b);
    __syncthreads();
  }
}

// Called by every block of the producer after it has written the partials of `chunk` for channels
// [c0, c1) (channel tile ct of nct): forward statistics (part = {n, S1, S2, shift} [nchunks][C]).
// lds: >= 2 * blockDim doubles + 1 int of LDS the block may overwrite.
__device__ __forceinline__ void bnfin_arrive_stats(const BnFin& f, const float* part, int nchunks, int C, int chunk,
                                                   int c0, int c1, int ct, int nct, void* lds) {
  double* red = reinterpret_cast<double*>(lds);
  int* flag = reinterpret_cast<int*>(red + 2 * blockDim.x);
  const int g = chunk / f.gs;
  const int k0 = g * f.gs, k1 = min(nchunks, k0 + f.gs);
  if (!bnfin_ticket(f.counters + g * nct + ct, (unsigned)(k1 - k0), flag)) return;
  auto final_store = [&](int c, double n, double mean, double m2) {
    bn_finalize_store(c, n, mean, m2, f.gamma, f.beta, f.rmean, f.rvar, f.nbt, f.momentum, f.eps, f.mean_o, f.rstd_o,
                      f.scale, f.shift);
  };
  if (f.ngroups == 1) {
    bnfin_merge_stats(part, C, k0, k1, c0, c1, red, final_store);
    return;
  }
  // level-2 partial {n, S1, S2, shift}: shift = the group mean rounded to float, S1 = the rounding residue
  // times n (the merge reads mean = shift + S1/n), S2 = M2 + S1^2/n
  bnfin_merge_stats(part, C, k0, k1, c0, c1, red, [&](int c, double n, double mean, double m2) {
    const float hi = (float)mean;
    const double s1 = (mean - (double)hi) * n;
    wt_store4(f.scratch + ((long long)g * C + c) * 4,
              make_float4((float)n, (float)s1, (float)(m2 + (n > 0 ? s1 * s1 / n : 0.0)), hi));
  });
  if (!bnfin_ticket(f.counters + BNFIN_L1 + ct, (unsigned)f.ngroups, flag)) return;
  bnfin_merge_stats(f.scratch, C, 0, f.ngroups, c0, c1, red, final_store);
}

// The same for the fused BatchNorm-backward sums (part2 = {sum dn, sum dn*xhat} [nchunks][C]):
// dbeta = sum dn, dgamma = sum dn*xhat.
__device__ __forceinline__ void bnfin_arrive_sums(const BnFin& f, const float* part2, int nchunks, int C, int chunk,
                                                  int c0, int c1, int ct, int nct, void* lds) {
  double* red = reinterpret_cast<double*>(lds);
  int* flag = reinterpret_cast<int*>(red + 2 * blockDim.x);
  const int g = chunk / f.gs;
  const int k0 = g * f.gs, k1 = min(nchunks, k0 + f.gs);
  if (!bnfin_ticket(f.counters + g * nct + ct, (unsigned)(k1 - k0), flag)) return;
  auto final_store = [&](int c, double a, double b) {
    f.dbeta[c] = (float)a;
    f.dgamma[c] = (float)b;
  };
  auto load1 = [&](int k, int c) {
    const float2 q = *reinterpret_cast<const float2*>(part2 + ((long long)k * C + c) * 2);
    return make_double2((double)q.x, (double)q.y);
  };
  if (f.ngroups == 1) {
    bnfin_merge_sums(k0, k1, c0, c1, red, load1, final_store);
    return;
  }
  // level-2 partial: each fp64 sum as a {hi, lo} float pair
  bnfin_merge_sums(k0, k1, c0, c1, red, load1, [&](int c, double a, double b) {
    const float ah = (float)a, bh = (float)b;
    wt_store4(f.scratch + ((long long)g * C + c) * 4, make_float4(ah, (float)(a - (double)ah), bh, (float)(b - (double)bh)));
  });
  if (!bnfin_ticket(f.counters + BNFIN_L1 + ct, (unsigned)f.ngroups, flag)) return;
  bnfin_merge_sums(0, f.ngroups, c0, c1, red, [&](int k, int c) {
    const float4 q = *reinterpret_cast<const float4*>(f.scratch + ((long long)k * C + c) * 4);
    return make_double2((double)q.x + (double)q.y, (double)q.z + (double)q.w);
  }, final_store);
}

}  // namespace stc
