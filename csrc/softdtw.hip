// Soft-DTW (soft_dtw_cuda.py:34-112 semantics) and hard DTW with on-device backtracking
// (dtw.py:22-75 semantics).
//
// soft-DTW forward: one workgroup per sequence pair, one lane per row i of R. Cell (i, j) is
// computed on anti-diagonal pass p = (i-1) + (j-1); the three predecessors are the lane's own
// previous value (R[i][j-1]) and the previous-row lane's values from passes p-1 (R[i-1][j]) and
// p-2 (R[i-1][j-1]), exchanged through a 3-deep LDS ring, so only the final R goes to global
// memory (it is saved for the backward). Up to 1024 lanes per pair; longer sequences put several
// rows on each lane (up to ~6.6k rows, the LDS ring's limit).
// The distance matrix of pair p is read in place from a (possibly shared) matrix:
//     D_p[i][j] = D[(p / pair_div) * s_i + (p % pair_div) * s_j + i * ld + j]
// so the b^2 all-pairs losses (loss.py:93-134) use ONE [b*n, b*m] GEMM output instead of the
// reference's [b^2, n, m, d] expand.
// soft-DTW backward: the reverse wavefront of the E recursion with the reference's boundary
// handling (R = -inf outside, R[N+1][M+1] = R[N][M], +inf cells treated as -inf).
// R and E are kept in fp64: R grows to ~sum of the path costs and the backward exponent
// (R' - R - D) / gamma is a difference of such sums, which fp32 resolves only to ~1e-3 at
// n ~ 100 (the DP is latency-bound, so fp64 costs nothing measurable).
#include "common.h"

struct PairIndex {
  int pair_div, ld;
  long long s_i, s_j;
  __device__ __forceinline__ long long base(int p) const {
    return (long long)(p / pair_div) * s_i + (long long)(p % pair_div) * s_j;
  }
};

// Distance function fused into the D reads (soft_dtw_cuda.py:325-363): the kernels read the GEMM
// output S = X Y^T in place and apply D = f(S, a_i, b_j) per cell, with a / b per-row statistics of
// X / Y (norms for the cosine forms, squared norms for the Euclidean forms). The backward writes
// dS = dL/dD * dD/dS in S's own layout and accumulates the row-statistic gradients (atomically:
// rows of the all-pairs layout are shared by b pairs) as coefficients ca / cb such that
// dX = dS Y + ca * X and dY = dS^T X + cb * Y.
enum DistKind : int { DK_RAW = 0, DK_NEG_DOT = 1, DK_COSINE = 2, DK_NEG_COSINE = 3, DK_SQEUCLID = 4, DK_EUCLID = 5 };

struct DistFn {
  int kind;
  const float* a;  // per X row (norm or squared norm), nullptr for DK_RAW / DK_NEG_DOT
  const float* b;  // per Y row
  long long a_si, a_sj, b_si, b_sj;  // row-statistic base of pair p: (p / div) * s_i + (p % div) * s_j
  float* ca;       // backward: dX row coefficients (same indexing as a), may be null
  float* cb;
  __device__ __forceinline__ long long abase(int p, int div) const { return (p / div) * a_si + (p % div) * a_sj; }
  __device__ __forceinline__ long long bbase(int p, int div) const { return (p / div) * b_si + (p % div) * b_sj; }
  __device__ __forceinline__ bool has_stats() const { return kind >= DK_COSINE; }
};

__device__ __forceinline__ float dist_val(int kind, float s, float a, float b) {
  switch (kind) {
    case DK_NEG_DOT: return -s;
    case DK_COSINE: return expf(1.f - s / fmaxf(a * b, 1e-8f));
    case DK_NEG_COSINE: return -s / fmaxf(a * b, 1e-8f);
    case DK_SQEUCLID: return fmaxf(a + b - 2.f * s, 0.f);
    case DK_EUCLID: return expf(sqrtf(fmaxf(a + b - 2.f * s, 0.f) + 1e-12f));
    default: return s;
  }
}

// dD/dS, dD/da, dD/db at one cell (a, b: the statistics as stored; the caller turns dD/da into the
// X-row coefficient: / a for norms (d||x||/dx = x / ||x||), * 2 for squared norms (d||x||^2/dx = 2x))
__device__ __forceinline__ void dist_grad(int kind, float s, float a, float b, float& ds, float& da, float& db) {
  da = db = 0.f;
  switch (kind) {
    case DK_NEG_DOT: ds = -1.f; return;
    case DK_COSINE:
    case DK_NEG_COSINE: {
      const float ab = a * b;
      const bool clamped = !(ab > 1e-8f);
      const float den = clamped ? 1e-8f : ab;
      const float c = s / den;
      const float dDdc = kind == DK_COSINE ? -expf(1.f - c) : -1.f;
      ds = dDdc / den;
      if (!clamped) { da = dDdc * (-c / a); db = dDdc * (-c / b); }
      return;
    }
    case DK_SQEUCLID:
    case DK_EUCLID: {
      const float sq = a + b - 2.f * s;
      float dDsq = sq >= 0.f ? 1.f : 0.f;
      if (kind == DK_EUCLID) {
        // d exp(r) / d sq = exp(r) / 2r is unbounded as r -> 0, and dX = ds Y + ca X would then
        // cancel two huge fp32 terms (normalize=True's self cells are exactly zero distances):
        // below the fp32 cancellation level of sq the subgradient is zero (the float64 oracle's
        // clamp gives the same at identical rows)
        const float r = sqrtf(fmaxf(sq, 0.f) + 1e-12f);
        dDsq = sq > 1e-6f * (a + b) + 1e-12f ? dDsq * expf(r) / (2.f * r) : 0.f;
      }
      ds = -2.f * dDsq;
      da = dDsq;
      db = dDsq;
      return;
    }
    default: ds = 1.f; return;
  }
}

__device__ __forceinline__ float row_coef(int kind, float dDdstat, float stat) {
  if (kind == DK_COSINE || kind == DK_NEG_COSINE) return stat > 0.f ? dDdstat / stat : 0.f;
  return 2.f * dDdstat;
}

// RPL rows per lane (row i = lane + 1 + k * blockDim.x): rows handled by one lane lie on the same
// anti-diagonal pass but are >= blockDim apart, so their predecessors always come from another
// lane through the ring; sequences up to ~6.6k (LDS ring 3 x (N+2) doubles) run on the GPU.
template <int RPL>
__global__ void softdtw_fwd_kernel(const float* __restrict__ D, PairIndex pi, DistFn df, int N, int M, float gamma_f,
                                   float bw, double* __restrict__ R, float* __restrict__ out) {
  extern __shared__ double ring[];  // [3][N+1]
  const double gamma = gamma_f;
  const int b = blockIdx.x;
  const float* Dp = D + pi.base(b);
  const float* ap = df.has_stats() ? df.a + df.abase(b, pi.pair_div) : nullptr;
  const float* bp = df.has_stats() ? df.b + df.bbase(b, pi.pair_div) : nullptr;
  double* Rp = R + (long long)b * (N + 2) * (M + 2);
  const double inv_g = 1.0 / gamma;
  // boundaries of R: R[0][0] = 0, everything else starts at +inf
  for (int k = threadIdx.x; k < (N + 2) * (M + 2); k += blockDim.x) Rp[k] = INFINITY;
  __syncthreads();
  if (threadIdx.x == 0) Rp[0] = 0.0;
  const int S = N + 1;
  // ring slot for "row 0": R[0][j] = 0 if j == 0 else inf ; row i>0 at j<=0: inf
  for (int k = threadIdx.x; k < 3 * S; k += blockDim.x) ring[k] = INFINITY;
  __syncthreads();
  double own_prev[RPL];  // R[i][j-1]
#pragma unroll
  for (int r = 0; r < RPL; ++r) own_prev[r] = INFINITY;
  const int passes = N + M - 1;
  for (int p = 0; p < passes; ++p) {
#pragma unroll
    for (int r = 0; r < RPL; ++r) {
      const int i = threadIdx.x + 1 + r * blockDim.x;  // 1-based row
      const bool row_ok = i <= N;
      const int j = p - i + 2;
      double val = INFINITY;
      if (row_ok && j >= 1 && j <= M) {
        // R[i-1][j] from pass p-1, R[i-1][j-1] from pass p-2 (row 0 handled analytically)
        double up, diag;
        if (i == 1) {
          up = INFINITY;                     // R[0][j], j >= 1
          diag = (j == 1) ? 0.0 : INFINITY;  // R[0][j-1]
        } else {
          up = ring[((p + 2) % 3) * S + (i - 1)];
          diag = ring[((p + 1) % 3) * S + (i - 1)];
          if (j == 1) diag = INFINITY;  // R[i-1][0]
        }
        const double left = own_prev[r];  // R[i][j-1] (inf at j == 1)
        if (bw > 0.f && fabsf((float)(i - j)) > bw) {
          val = INFINITY;
        } else {
          const double r0 = -diag * inv_g, r1 = -up * inv_g, r2 = -left * inv_g;
          const double rmax = fmax(fmax(r0, r1), r2);
          const double rsum = exp(r0 - rmax) + exp(r1 - rmax) + exp(r2 - rmax);
          const double softmin = -gamma * (log(rsum) + rmax);
          const float sv = Dp[(long long)(i - 1) * pi.ld + (j - 1)];
          const float dv = df.kind == DK_RAW ? sv : dist_val(df.kind, sv, ap ? ap[i - 1] : 0.f, bp ? bp[j - 1] : 0.f);
          val = (double)dv + softmin;
        }
        Rp[(long long)i * (M + 2) + j] = val;
        own_prev[r] = val;
      }
      if (row_ok) ring[(p % 3) * S + i] = val;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) out[b] = (float)Rp[(long long)N * (M + 2) + M];
}

__device__ __forceinline__ double rv(const double* Rp, int i, int j, int N, int M) {
  if (i == N + 1 && j == M + 1) {
    const double v = Rp[(long long)N * (M + 2) + M];
    return isinf(v) ? -INFINITY : v;
  }
  if (i == N + 1 || j == M + 1) return -INFINITY;
  const double v = Rp[(long long)i * (M + 2) + j];
  return isinf(v) ? -INFINITY : v;
}

// G: dL/dD per pair [P][N][M] (df.kind == DK_RAW), or dL/dS written in S's own layout (fused
// distance); the fused form also accumulates ca / cb (LDS column partials, then one atomic each).
template <int RPL>
__global__ void softdtw_bwd_kernel(const float* __restrict__ D, const double* __restrict__ R, PairIndex pi, DistFn df,
                                   int N, int M, float gamma_f, float bw, const float* __restrict__ gout,
                                   float* __restrict__ G) {
  extern __shared__ double ring[];  // [3][N+2], then (fused) float colacc[M]
  const double gamma = gamma_f;
  const int b = blockIdx.x;
  const float* Dp = D + pi.base(b);
  const double* Rp = R + (long long)b * (N + 2) * (M + 2);
  const bool fused = df.kind != DK_RAW;
  float* Gp = fused ? G + pi.base(b) : G + (long long)b * N * M;
  const long long gld = fused ? pi.ld : M;
  const float* ap = df.has_stats() ? df.a + df.abase(b, pi.pair_div) : nullptr;
  const float* bp = df.has_stats() ? df.b + df.bbase(b, pi.pair_div) : nullptr;
  auto dval = [&](int ii, int jj) {  // D at 0-based (ii, jj)
    const float sv = Dp[(long long)ii * pi.ld + jj];
    return fused ? dist_val(df.kind, sv, ap ? ap[ii] : 0.f, bp ? bp[jj] : 0.f) : sv;
  };
  const double inv_g = 1.0 / gamma;
  const double g = gout[b];
  const int S = N + 2;
  float* colacc = (float*)(ring + 3 * S);
  const bool stats = fused && df.has_stats() && df.ca != nullptr;
  for (int k = threadIdx.x; k < 3 * S; k += blockDim.x) ring[k] = 0.0;
  if (stats)
    for (int k = threadIdx.x; k < M; k += blockDim.x) colacc[k] = 0.f;
  float rowacc[RPL];
#pragma unroll
  for (int r = 0; r < RPL; ++r) rowacc[r] = 0.f;
  __syncthreads();
  double own_prev[RPL];  // E[i][j+1]
#pragma unroll
  for (int r = 0; r < RPL; ++r) own_prev[r] = 0.0;
  const int passes = N + M - 1;
  for (int q = 0; q < passes; ++q) {
    const int p = passes - 1 - q;  // anti-diagonal index, descending
#pragma unroll
    for (int r = 0; r < RPL; ++r) {
      const int i = threadIdx.x + 1 + r * blockDim.x;
      const bool row_ok = i <= N;
      const int j = p - i + 2;
      double e = 0.0;
      if (row_ok && j >= 1 && j <= M) {
        if (!(bw > 0.f && fabsf((float)(i - j)) > bw)) {
          const double rr = rv(Rp, i, j, N, M);
          const double d_down = (i + 1 <= N) ? (double)dval(i, j - 1) : 0.0;
          const double d_right = (j + 1 <= M) ? (double)dval(i - 1, j) : 0.0;
          const double d_diag = (i + 1 <= N && j + 1 <= M) ? (double)dval(i, j) : 0.0;
          const double a = exp((rv(Rp, i + 1, j, N, M) - rr - d_down) * inv_g);
          const double bb = exp((rv(Rp, i, j + 1, N, M) - rr - d_right) * inv_g);
          const double c = exp((rv(Rp, i + 1, j + 1, N, M) - rr - d_diag) * inv_g);
          // E[i+1][j] from pass p+1 (row below), E[i+1][j+1] from pass p+2; E[N+1][M+1] = 1
          double e_down, e_diag;
          if (i == N) {
            e_down = 0.0;
            e_diag = (j == M) ? 1.0 : 0.0;
          } else {
            e_down = ring[((q + 2) % 3) * S + (i + 1)];
            e_diag = (j == M) ? 0.0 : ring[((q + 1) % 3) * S + (i + 1)];
          }
          const double e_right = (j == M) ? 0.0 : own_prev[r];
          e = e_down * a + e_right * bb + e_diag * c;
        }
        const float ge = (float)(e * g);
        if (fused) {
          float ds, da, db;
          const float av = ap ? ap[i - 1] : 0.f, bv = bp ? bp[j - 1] : 0.f;
          dist_grad(df.kind, Dp[(long long)(i - 1) * pi.ld + (j - 1)], av, bv, ds, da, db);
          Gp[(long long)(i - 1) * gld + (j - 1)] = ge * ds;
          if (stats) {
            rowacc[r] += ge * da;
            atomicAdd(&colacc[j - 1], ge * db);
          }
        } else {
          Gp[(long long)(i - 1) * gld + (j - 1)] = ge;
        }
        own_prev[r] = e;
      }
      if (row_ok) ring[(q % 3) * S + i] = e;
    }
    __syncthreads();
  }
  if (stats) {
    float* cap = df.ca + df.abase(b, pi.pair_div);
    float* cbp = df.cb + df.bbase(b, pi.pair_div);
#pragma unroll
    for (int r = 0; r < RPL; ++r) {
      const int i = threadIdx.x + 1 + r * blockDim.x;
      if (i <= N) atomicAdd(&cap[i - 1], row_coef(df.kind, rowacc[r], ap[i - 1]));
    }
    for (int k = threadIdx.x; k < M; k += blockDim.x) atomicAdd(&cbp[k], row_coef(df.kind, colacc[k], bp[k]));
  }
}

static int block_for(int n) {
  int t = ((n + 63) / 64) * 64;
  t = t < 64 ? 64 : t;
  return t > 1024 ? 1024 : t;
}

static int rows_per_lane(int n) {
  const int r = (n + 1023) / 1024;
  return r <= 1 ? 1 : r <= 2 ? 2 : r <= 4 ? 4 : r <= 8 ? 8 : -1;
}

constexpr int kSdtwMaxN = 6600;  // LDS ring: 3 x (N + 2) doubles <= 160 KiB

static DistFn make_df(int kind, const float* a, const float* b, long long a_si, long long a_sj, long long b_si,
                      long long b_sj, float* ca, float* cb) {
  DistFn df;
  df.kind = kind; df.a = a; df.b = b;
  df.a_si = a_si; df.a_sj = a_sj; df.b_si = b_si; df.b_sj = b_sj;
  df.ca = ca; df.cb = cb;
  return df;
}

// D: distances (kind 0) or the GEMM output S = X Y^T read through the distance function `kind`
// (DistKind) with row statistics a / b (see DistFn).
MILNCE_API int milnce_softdtw_fwd(const float* D, int B, int N, int M, int ld, int pair_div, long long s_i,
                                  long long s_j, float gamma, float bandwidth, int kind, const float* a,
                                  const float* b, long long a_si, long long a_sj, long long b_si, long long b_sj,
                                  double* R, float* out, hipStream_t stream) {
  if (N > kSdtwMaxN || kind < 0 || kind > DK_EUCLID) return (int)hipErrorInvalidValue;
  if (kind >= DK_COSINE && (a == nullptr || b == nullptr)) return (int)hipErrorInvalidValue;
  PairIndex pi{pair_div, ld, s_i, s_j};
  const DistFn df = make_df(kind, a, b, a_si, a_sj, b_si, b_sj, nullptr, nullptr);
  const size_t lds = 3 * (N + 1) * sizeof(double);
  const int rpl = rows_per_lane(N);
  auto go = [&](auto kern) {
    if (lds > 64 * 1024) HIP_RET(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    hipLaunchKernelGGL(kern, dim3(B), dim3(block_for(N)), lds, stream, D, pi, df, N, M, gamma, bandwidth, R, out);
    return (int)hipGetLastError();
  };
  if (rpl == 1) return go(softdtw_fwd_kernel<1>);
  if (rpl == 2) return go(softdtw_fwd_kernel<2>);
  if (rpl == 4) return go(softdtw_fwd_kernel<4>);
  return go(softdtw_fwd_kernel<8>);
}

// G: kind 0 -> dL/dD as [B][N][M]; otherwise dL/dS in S's layout, and (kinds with row statistics)
// ca / cb += the X / Y row coefficients (zero them first; dX = dS Y + ca * X).
MILNCE_API int milnce_softdtw_bwd(const float* D, const double* R, int B, int N, int M, int ld, int pair_div,
                                  long long s_i, long long s_j, float gamma, float bandwidth, int kind, const float* a,
                                  const float* b, long long a_si, long long a_sj, long long b_si, long long b_sj,
                                  float* ca, float* cb, const float* gout, float* G, hipStream_t stream) {
  if (N > kSdtwMaxN || kind < 0 || kind > DK_EUCLID) return (int)hipErrorInvalidValue;
  if (kind >= DK_COSINE && (a == nullptr || b == nullptr || ca == nullptr || cb == nullptr))
    return (int)hipErrorInvalidValue;
  PairIndex pi{pair_div, ld, s_i, s_j};
  const DistFn df = make_df(kind, a, b, a_si, a_sj, b_si, b_sj, ca, cb);
  const size_t lds = 3 * (N + 2) * sizeof(double) + (kind >= DK_COSINE ? (size_t)M * sizeof(float) : 0);
  if (lds > 160 * 1024) return (int)hipErrorInvalidValue;
  const int rpl = rows_per_lane(N);
  auto go = [&](auto kern) {
    if (lds > 64 * 1024) HIP_RET(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    hipLaunchKernelGGL(kern, dim3(B), dim3(block_for(N)), lds, stream, D, R, pi, df, N, M, gamma, bandwidth, gout, G);
    return (int)hipGetLastError();
  };
  if (rpl == 1) return go(softdtw_bwd_kernel<1>);
  if (rpl == 2) return go(softdtw_bwd_kernel<2>);
  if (rpl == 4) return go(softdtw_bwd_kernel<4>);
  return go(softdtw_bwd_kernel<8>);
}

// Row statistics of X [rows][d] for the fused distances: ||x|| (squared = 0) or ||x||^2. One
// wave per row.
__global__ __launch_bounds__(256) void rowstat_kernel(const float* __restrict__ X, long long rows, int d, int squared,
                                                      float* __restrict__ out) {
  const long long r = blockIdx.x * 4LL + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= rows) return;
  float acc = 0.f;
  for (int k = lane * 4; k < d; k += 256) {
    const float4 v = *(const float4*)(X + r * d + k);
    acc += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  acc = wave_sum(acc);
  if (lane == 0) out[r] = squared ? acc : sqrtf(acc);
}

// out[r][:] += coef[r] * X[r][:] (the row-statistic term of the fused distances' dX).
__global__ __launch_bounds__(256) void rowscale_add_kernel(float* __restrict__ out, const float* __restrict__ X,
                                                           const float* __restrict__ coef, long long rows, int d) {
  const long long n4 = rows * d / 4;
  for (long long e = blockIdx.x * 256LL + threadIdx.x; e < n4; e += (long long)gridDim.x * 256) {
    const long long r = e * 4 / d;
    const float c = coef[r];
    const float4 x = ((const float4*)X)[e];
    float4 o = ((float4*)out)[e];
    o.x += c * x.x; o.y += c * x.y; o.z += c * x.z; o.w += c * x.w;
    ((float4*)out)[e] = o;
  }
}

MILNCE_API int milnce_rowstat(const float* X, long long rows, int d, int squared, float* out, hipStream_t stream) {
  if (d % 4) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(rowstat_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, stream, X, rows, d, squared, out);
  return (int)hipGetLastError();
}

MILNCE_API int milnce_rowscale_add(float* out, const float* X, const float* coef, long long rows, int d,
                                   hipStream_t stream) {
  if (d % 4) return (int)hipErrorInvalidValue;
  const long long n4 = rows * d / 4;
  const int grid = (int)((n4 + 255) / 256 < 4096 ? (n4 + 255) / 256 : 4096);
  hipLaunchKernelGGL(rowscale_add_kernel, dim3(grid > 0 ? grid : 1), dim3(256), 0, stream, out, X, coef, rows, d);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// Hard DTW (dtw.py): fp64 min-plus DP and the reference's backtracking, one lane per pair.
__global__ void dtw_path_kernel(const double* __restrict__ cost, int B, int N, int M, double* __restrict__ tc,
                                double* __restrict__ path) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const double* c = cost + (long long)b * N * M;
  double* t = tc + (long long)b * N * M;
  double* pa = path + (long long)b * N * M;
  for (int k = 0; k < N * M; ++k) pa[k] = 0.0;
  pa[(N - 1) * M + (M - 1)] = 1.0;
  t[0] = c[0];
  for (int i = 1; i < N; ++i) t[i * M] = t[(i - 1) * M] + c[i * M];
  for (int j = 1; j < M; ++j) t[j] = t[j - 1] + c[j];
  for (int i = 1; i < N; ++i)
    for (int j = 1; j < M; ++j) {
      const double v = fmin(fmin(t[(i - 1) * M + j - 1], t[(i - 1) * M + j]), t[i * M + j - 1]);
      t[i * M + j] = v + c[i * M + j];
    }
  int i = N - 1, j = M - 1;
  int guard = N + M + 2;
  while (!(i == 0 || j == 0) && guard-- > 0) {
    const double r = t[i * M + j] - c[i * M + j];
    if (r == t[(i - 1) * M + j - 1]) { pa[(i - 1) * M + j - 1] = 1.0; --i; --j; }
    else if (r == t[(i - 1) * M + j]) { pa[(i - 1) * M + j] = 1.0; --i; }
    else if (r == t[i * M + j - 1]) { pa[i * M + j - 1] = 1.0; --j; }
    else break;  // the reference prints 'error' and loops; we stop
  }
  pa[0] = 1.0;
}

MILNCE_API int milnce_dtw_path(const double* cost, int B, int N, int M, double* tc, double* path,
                               hipStream_t stream) {
  hipLaunchKernelGGL(dtw_path_kernel, dim3((B + 63) / 64), dim3(64), 0, stream, cost, B, N, M, tc, path);
  return (int)hipGetLastError();
}
