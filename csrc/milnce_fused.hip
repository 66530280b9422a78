// Fused MIL-NCE (loss.py:10-18) for large global batches: the logits x = V T^T ([Bg, Bg*K]) are
// never stored. Exact fp32 via v_mfma_f32_16x16x4_f32 (f32 in / f32 accumulate, the reference's
// fp32 logits): 64 x 64 tiles, 4 waves (16 rows x 64 columns each), D streamed through LDS.
//
//   forward : per tile, row partial (max, sum e^{x-max}) over its 64 columns and, for each of its
//             64/K text blocks, a block-column partial over its 64 rows; a finalize kernel merges
//             them into den_i = LSE(row_i U blockcol_i) and takes nom_i = LSE_k V_i . T_{iK+k}
//             (positives counted twice, as in the reference);
//   backward: G[i, j] = g/Bg (e^{x-den_i} + e^{x-den_{j/K}} - [j/K == i] e^{x-nom_i}) recomputed
//             tile by tile; dV = G T accumulated in registers by a row-tile pass, dT = G^T V by a
//             column-tile pass (no atomics, deterministic). 4 logit GEMMs per step instead of 2
//             materialised fp32 [Bg, Bg*K] tensors (1 GiB each at Bg = 8192, K = 4).
#include "common.h"

namespace {

constexpr int TM = 64, TN = 64;  // tile rows (video) x tile columns (text)
constexpr int KC = 32;           // D chunk staged per step of the logit GEMM
constexpr int SP = KC + 1;       // padded LDS row (floats)
constexpr int GP = TN + 1;       // padded S/G tile row
constexpr int DC = 64;           // D chunk of the G GEMMs
constexpr int DP = DC + 1;

__device__ __forceinline__ void lse_add(float& m, float& s, float m2, float s2) {
  if (m2 == -INFINITY) return;
  if (m == -INFINITY) { m = m2; s = s2; return; }
  if (m2 > m) { s = s * __expf(m - m2) + s2; m = m2; }
  else { s += s2 * __expf(m2 - m); }
}

// S[64 x 64] tile = V[r0 : r0+64] . T[c0 : c0+64]^T into acc (wave w: rows 16w.., all 4 column
// blocks; acc[nb][r] = S[16w + 4*(lane>>4) + r][16 nb + (lane & 15)]). Rows past the matrix read 0.
__device__ __forceinline__ void logit_tile(const float* __restrict__ V, const float* __restrict__ T, int B, int N,
                                           int D, int r0, int c0, float* Vs, float* Ts, f32x4 (&acc)[4]) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) acc[nb] = (f32x4){0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < D; k0 += KC) {
    __syncthreads();
#pragma unroll
    for (int it = 0; it < 2; ++it) {  // 64 rows x 8 float4 per matrix = 512 float4, 2 per thread
      const int e = tid + it * 256, row = e >> 3, c4 = (e & 7) * 4;
      float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
      if (r0 + row < B) a = *(const float4*)(V + (long long)(r0 + row) * D + k0 + c4);
      if (c0 + row < N) b = *(const float4*)(T + (long long)(c0 + row) * D + k0 + c4);
      float* va = Vs + row * SP + c4;
      float* tb = Ts + row * SP + c4;
      va[0] = a.x; va[1] = a.y; va[2] = a.z; va[3] = a.w;
      tb[0] = b.x; tb[1] = b.y; tb[2] = b.z; tb[3] = b.w;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < KC; kk += 4) {
      const float a = Vs[(16 * w + (lane & 15)) * SP + kk + (lane >> 4)];
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        const float b = Ts[(16 * nb + (lane & 15)) * SP + kk + (lane >> 4)];
        acc[nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[nb], 0, 0, 0);
      }
    }
  }
}

__device__ __forceinline__ void store_tile(float* Ss, const f32x4 (&acc)[4]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int nb = 0; nb < 4; ++nb)
#pragma unroll
    for (int r = 0; r < 4; ++r) Ss[(16 * w + 4 * (lane >> 4) + r) * GP + 16 * nb + (lane & 15)] = acc[nb][r];
}

}  // namespace

// rowpart: [n_ct][B] (max, sum); colpart: [n_rt][B] (max, sum) per text block.
__global__ __launch_bounds__(256) void milnce_fused_fwd_kernel(const float* __restrict__ V, const float* __restrict__ T,
                                                               int B, int K, int D, float2* __restrict__ rowpart,
                                                               float2* __restrict__ colpart) {
  __shared__ float Vs[TM * SP], Ts[TN * SP], Ss[TM * GP];
  const int N = B * K;
  const int rt = blockIdx.y, ct = blockIdx.x;
  const int r0 = rt * TM, c0 = ct * TN;
  f32x4 acc[4];
  logit_tile(V, T, B, N, D, r0, c0, Vs, Ts, acc);
  store_tile(Ss, acc);
  __syncthreads();
  const int tid = threadIdx.x;
  if (tid < TM) {  // row partial over this tile's valid columns
    const int i = r0 + tid;
    float m = -INFINITY, s = 0.f;
    for (int j = 0; j < TN && c0 + j < N; ++j) m = fmaxf(m, Ss[tid * GP + j]);
    for (int j = 0; j < TN && c0 + j < N; ++j) s += __expf(Ss[tid * GP + j] - m);
    if (i < B) rowpart[(long long)ct * B + i] = make_float2(m, s);
  }
  // block-column partials: text block b (K columns) over the tile's valid rows; 16 lanes per
  // block, 16 blocks per pass (64 / K blocks per tile)
  const int nbk = TN / K;
  const int sub = tid & 15;
  for (int b = tid >> 4; b < ((nbk + 15) / 16) * 16; b += 16) {
    float m = -INFINITY, s = 0.f;
    if (b < nbk) {
      for (int rr = sub; rr < TM; rr += 16) {
        if (r0 + rr >= B) break;
        for (int k = 0; k < K; ++k) lse_add(m, s, Ss[rr * GP + b * K + k], 1.f);
      }
    }
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
      lse_add(m, s, m2, s2);
    }
    const int blk = c0 / K + b;
    if (b < nbk && sub == 0 && blk < B) colpart[(long long)rt * B + blk] = make_float2(m, s);
  }
}

// den_i, nom_i, per-row loss; loss = mean (single block tail via a second tiny kernel).
__global__ __launch_bounds__(256) void milnce_fused_finalize_kernel(const float* __restrict__ V,
                                                                    const float* __restrict__ T, int B, int K, int D,
                                                                    const float2* __restrict__ rowpart, int n_ct,
                                                                    const float2* __restrict__ colpart, int n_rt,
                                                                    float* __restrict__ den, float* __restrict__ nom,
                                                                    float* __restrict__ li) {
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= B) return;
  float m = -INFINITY, s = 0.f;
  for (int c = lane; c < n_ct; c += 64) { const float2 p = rowpart[(long long)c * B + i]; lse_add(m, s, p.x, p.y); }
  for (int r = lane; r < n_rt; r += 64) { const float2 p = colpart[(long long)r * B + i]; lse_add(m, s, p.x, p.y); }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    lse_add(m, s, m2, s2);
  }
  // nom_i = LSE_k V_i . T_{iK+k} (exact fp32 dots)
  float mn = -INFINITY, sn = 0.f;
  for (int k = 0; k < K; ++k) {
    float d = 0.f;
    for (int e = lane; e < D; e += 64) d += V[(long long)i * D + e] * T[((long long)i * K + k) * D + e];
    d = wave_sum(d);
    lse_add(mn, sn, d, 1.f);
  }
  if (lane == 0) {
    const float dn = m + __logf(s), nm = mn + __logf(sn);
    den[i] = dn;
    nom[i] = nm;
    li[i] = dn - nm;
  }
}

__global__ __launch_bounds__(256) void milnce_fused_mean_kernel(const float* __restrict__ li, int B,
                                                                float* __restrict__ loss) {
  float s = 0.f;
  for (int i = threadIdx.x; i < B; i += 256) s += li[i];
  s = wave_sum(s);
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) loss[0] = (red[0] + red[1] + red[2] + red[3]) / (float)B;
}

namespace {

// G tile from the logit tile (into Ss, in place): rows r0.., columns c0..
__device__ __forceinline__ void grad_tile(float* Ss, int B, int K, int r0, int c0, const float* __restrict__ den,
                                          const float* __restrict__ nom, const float* __restrict__ gup) {
  const int N = B * K;
  const float gscale = gup[0] / (float)B;  // d loss / d x = (upstream grad) / Bg * (...)
  for (int e = threadIdx.x; e < TM * TN; e += 256) {
    const int rr = e / TN, cc = e - rr * TN;
    const int i = r0 + rr, j = c0 + cc;
    float g = 0.f;
    if (i < B && j < N) {
      const float x = Ss[rr * GP + cc];
      const int blk = j / K;
      g = __expf(x - den[i]) + __expf(x - den[blk]);
      if (blk == i) g -= __expf(x - nom[i]);
      g *= gscale;
    }
    Ss[rr * GP + cc] = g;
  }
}

}  // namespace

// dV[r0 : r0+64, :] = sum over column tiles of G[rows, cols] . T[cols, :]
__global__ __launch_bounds__(256) void milnce_fused_dv_kernel(const float* __restrict__ V, const float* __restrict__ T,
                                                              int B, int K, int D, const float* __restrict__ den,
                                                              const float* __restrict__ nom, const float* __restrict__ gup,
                                                              float* __restrict__ dV) {
  extern __shared__ float sm[];
  float* Vs = sm;                 // [TM][SP]
  float* Ts = Vs + TM * SP;       // [TN][SP]
  float* Ss = Ts + TN * SP;       // [TM][GP]
  float* Tc = Ss + TM * GP;       // [TN][DP]  T chunk for the G GEMM
  const int N = B * K;
  const int r0 = blockIdx.x * TM;
  const int split = blockIdx.y, splits = gridDim.y;
  dV += (long long)split * B * D;  // split > 0 (or splits > 1): partial sums, reduced afterwards
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int ndc = D / DC;
  f32x4 out[8][4];  // up to D = 512: [d chunk][16-col block] of this wave's 16 rows
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int c = 0; c < 4; ++c) out[a][c] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const int n_ct = (N + TN - 1) / TN;
  const int ct_begin = (int)((long long)split * n_ct / splits), ct_end = (int)((long long)(split + 1) * n_ct / splits);
  for (int ct = ct_begin; ct < ct_end; ++ct) {
    const int c0 = ct * TN;
    f32x4 acc[4];
    logit_tile(V, T, B, N, D, r0, c0, Vs, Ts, acc);
    store_tile(Ss, acc);
    __syncthreads();
    grad_tile(Ss, B, K, r0, c0, den, nom, gup);
#pragma unroll
    for (int dc = 0; dc < 8; ++dc) {
      if (dc < ndc) {
        __syncthreads();
        for (int e = tid; e < TN * (DC / 4); e += 256) {
          const int row = e / (DC / 4), c4 = (e % (DC / 4)) * 4;
          float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
          if (c0 + row < N) v = *(const float4*)(T + (long long)(c0 + row) * D + dc * DC + c4);
          float* d = Tc + row * DP + c4;
          d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
        }
        __syncthreads();
#pragma unroll 4
        for (int kk = 0; kk < TN; kk += 4) {
          const float a = Ss[(16 * w + (lane & 15)) * GP + kk + (lane >> 4)];
#pragma unroll
          for (int cb = 0; cb < 4; ++cb) {
            const float b = Tc[(kk + (lane >> 4)) * DP + 16 * cb + (lane & 15)];
            out[dc][cb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, out[dc][cb], 0, 0, 0);
          }
        }
      }
    }
  }
#pragma unroll
  for (int dc = 0; dc < 8; ++dc)
    if (dc < ndc)
#pragma unroll
      for (int cb = 0; cb < 4; ++cb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = r0 + 16 * w + 4 * (lane >> 4) + r;
          if (i < B) dV[(long long)i * D + dc * DC + 16 * cb + (lane & 15)] = out[dc][cb][r];
        }
}

// dT[c0 : c0+64, :] = sum over row tiles of G[rows, cols]^T . V[rows, :]
__global__ __launch_bounds__(256) void milnce_fused_dt_kernel(const float* __restrict__ V, const float* __restrict__ T,
                                                              int B, int K, int D, const float* __restrict__ den,
                                                              const float* __restrict__ nom, const float* __restrict__ gup,
                                                              float* __restrict__ dT) {
  extern __shared__ float sm[];
  float* Vs = sm;
  float* Ts = Vs + TM * SP;
  float* Ss = Ts + TN * SP;
  float* Vc = Ss + TM * GP;  // [TM][DP] V chunk
  const int N = B * K;
  const int c0 = blockIdx.x * TN;
  const int split = blockIdx.y, splits = gridDim.y;
  dT += (long long)split * N * D;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int ndc = D / DC;
  f32x4 out[8][4];  // this wave's 16 text rows (tile columns 16w..) x D
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int c = 0; c < 4; ++c) out[a][c] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const int n_rt = (B + TM - 1) / TM;
  const int rt_begin = (int)((long long)split * n_rt / splits), rt_end = (int)((long long)(split + 1) * n_rt / splits);
  for (int rt = rt_begin; rt < rt_end; ++rt) {
    const int r0 = rt * TM;
    f32x4 acc[4];
    logit_tile(V, T, B, N, D, r0, c0, Vs, Ts, acc);
    store_tile(Ss, acc);
    __syncthreads();
    grad_tile(Ss, B, K, r0, c0, den, nom, gup);
#pragma unroll
    for (int dc = 0; dc < 8; ++dc) {
      if (dc < ndc) {
        __syncthreads();
        for (int e = tid; e < TM * (DC / 4); e += 256) {
          const int row = e / (DC / 4), c4 = (e % (DC / 4)) * 4;
          float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
          if (r0 + row < B) v = *(const float4*)(V + (long long)(r0 + row) * D + dc * DC + c4);
          float* d = Vc + row * DP + c4;
          d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
        }
        __syncthreads();
#pragma unroll 4
        for (int kk = 0; kk < TM; kk += 4) {
          // A = G^T: A[i = text row 16w + (lane&15)][k = video row kk + (lane>>4)]
          const float a = Ss[(kk + (lane >> 4)) * GP + 16 * w + (lane & 15)];
#pragma unroll
          for (int cb = 0; cb < 4; ++cb) {
            const float b = Vc[(kk + (lane >> 4)) * DP + 16 * cb + (lane & 15)];
            out[dc][cb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, out[dc][cb], 0, 0, 0);
          }
        }
      }
    }
  }
#pragma unroll
  for (int dc = 0; dc < 8; ++dc)
    if (dc < ndc)
#pragma unroll
      for (int cb = 0; cb < 4; ++cb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int j = c0 + 16 * w + 4 * (lane >> 4) + r;
          if (j < N) dT[(long long)j * D + dc * DC + 16 * cb + (lane & 15)] = out[dc][cb][r];
        }
}

__global__ void milnce_split_sum_kernel(const float4* __restrict__ part, int splits, long long n4,
                                        float4* __restrict__ out) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
    float4 a = part[i];
    for (int s = 1; s < splits; ++s) {
      const float4 b = part[s * n4 + i];
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
    out[i] = a;
  }
}

// Split counts of the two backward passes: ~2 workgroups per CU over (tiles x reduction ranges).
MILNCE_API int milnce_fused_bwd_splits(int B, int K, int* s_dv, int* s_dt) {
  const int N = B * K;
  const int n_ct = (N + TN - 1) / TN, n_rt = (B + TM - 1) / TM;
  int a = (512 + n_rt - 1) / n_rt, b = (512 + n_ct - 1) / n_ct;
  *s_dv = a < n_ct ? a : n_ct;
  *s_dt = b < n_rt ? b : n_rt;
  return 0;
}

// Workspace floats needed by the fused forward (row + column partials).
MILNCE_API long long milnce_fused_ws_floats(int B, int K) {
  const long long N = (long long)B * K;
  const long long n_ct = (N + TN - 1) / TN, n_rt = (B + TM - 1) / TM;
  return 2 * (n_ct * B + n_rt * B) + B;
}

MILNCE_API int milnce_fused_fwd(const float* V, const float* T, int B, int K, int D, float* ws, float* den, float* nom,
                                float* loss, hipStream_t stream) {
  if (K < 1 || TN % K || D % DC || D > 8 * DC) return (int)hipErrorInvalidValue;
  const int N = B * K;
  const int n_ct = (N + TN - 1) / TN, n_rt = (B + TM - 1) / TM;
  float2* rowpart = (float2*)ws;
  float2* colpart = rowpart + (long long)n_ct * B;
  float* li = (float*)(colpart + (long long)n_rt * B);
  hipLaunchKernelGGL(milnce_fused_fwd_kernel, dim3(n_ct, n_rt), dim3(256), 0, stream, V, T, B, K, D, rowpart, colpart);
  HIP_RET(hipGetLastError());
  hipLaunchKernelGGL(milnce_fused_finalize_kernel, dim3((B + 3) / 4), dim3(256), 0, stream, V, T, B, K, D, rowpart,
                     n_ct, colpart, n_rt, den, nom, li);
  HIP_RET(hipGetLastError());
  hipLaunchKernelGGL(milnce_fused_mean_kernel, dim3(1), dim3(256), 0, stream, li, B, loss);
  return (int)hipGetLastError();
}

// dV / dT; with s_dv / s_dt > 1 the passes write partial sums to `part` ([s][B][D] then [s][N][D])
// which are summed into dV / dT.
MILNCE_API int milnce_fused_bwd(const float* V, const float* T, int B, int K, int D, const float* den, const float* nom,
                                const float* gup, float* dV, float* dT, int s_dv, int s_dt, float* part,
                                hipStream_t stream) {
  if (K < 1 || TN % K || D % DC || D > 8 * DC) return (int)hipErrorInvalidValue;
  const int N = B * K;
  const size_t lds = (size_t)(TM * SP + TN * SP + TM * GP + 64 * DP) * sizeof(float);
  float* pv = s_dv > 1 ? part : dV;
  hipLaunchKernelGGL(milnce_fused_dv_kernel, dim3((B + TM - 1) / TM, s_dv), dim3(256), lds, stream, V, T, B, K, D,
                     den, nom, gup, pv);
  HIP_RET(hipGetLastError());
  if (s_dv > 1) {
    const long long n4 = (long long)B * D / 4;
    hipLaunchKernelGGL(milnce_split_sum_kernel, dim3((int)((n4 + 255) / 256 < 2048 ? (n4 + 255) / 256 : 2048)),
                       dim3(256), 0, stream, (const float4*)pv, s_dv, n4, (float4*)dV);
    HIP_RET(hipGetLastError());
  }
  float* pt = s_dt > 1 ? part : dT;
  hipLaunchKernelGGL(milnce_fused_dt_kernel, dim3((N + TN - 1) / TN, s_dt), dim3(256), lds, stream, V, T, B, K, D,
                     den, nom, gup, pt);
  HIP_RET(hipGetLastError());
  if (s_dt > 1) {
    const long long n4 = (long long)N * D / 4;
    hipLaunchKernelGGL(milnce_split_sum_kernel, dim3((int)((n4 + 255) / 256 < 2048 ? (n4 + 255) / 256 : 2048)),
                       dim3(256), 0, stream, (const float4*)pt, s_dt, n4, (float4*)dT);
  }
  return (int)hipGetLastError();
}
