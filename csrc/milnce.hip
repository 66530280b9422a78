// MIL-NCE loss (loss.py:10-18) on top of the logits x = V T^T  ([Bg, Bg*K], fp32).
//
//   nom_i = logsumexp_k x[i, iK + k]
//   den_i = logsumexp( x[i, :]  U  x[:, iK : iK+K] )      (positives counted twice, as in ref)
//   loss  = mean_i (den_i - nom_i)
//   dx[i, jK+k] = (g / Bg) * ( e^{x - den_i} + e^{x - den_j} - [i == j] e^{x - nom_i} )
//
// One workgroup per i reads its row (contiguous, Bg*K) and its block-column (Bg x K, strided)
// with an online max/sum, so the [Bg, 2*Bg*K] concatenation is never materialised.
#include "common.h"

__device__ __forceinline__ void lse_merge(float& m, float& s, float m2, float s2) {
  if (m2 == -INFINITY) return;
  if (m == -INFINITY) { m = m2; s = s2; return; }
  if (m2 > m) { s = s * __expf(m - m2) + s2; m = m2; }
  else { s += s2 * __expf(m2 - m); }
}

__device__ void block_lse(float& m, float& s) {
  __shared__ float sm[32], ss[32];
  // wave-level
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    lse_merge(m, s, m2, s2);
  }
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, nw = blockDim.x >> 6;
  __syncthreads();
  if (l == 0) { sm[w] = m; ss[w] = s; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float mm = sm[0], sv = ss[0];
    for (int i = 1; i < nw; ++i) lse_merge(mm, sv, sm[i], ss[i]);
    sm[0] = mm; ss[0] = sv;
  }
  __syncthreads();
  m = sm[0]; s = ss[0];
}

__global__ __launch_bounds__(256) void milnce_fwd_kernel(const float* __restrict__ x, int B, int K,
                                                         float* __restrict__ den, float* __restrict__ nom) {
  const int i = blockIdx.x;
  const long long ld = (long long)B * K;
  float m = -INFINITY, s = 0.f;
  const float* row = x + i * ld;
  for (long long j = threadIdx.x; j < ld; j += blockDim.x) lse_merge(m, s, row[j], 1.f);
  for (long long j = threadIdx.x; j < ld; j += blockDim.x) {
    const long long r = j / K, k = j - r * K;
    lse_merge(m, s, x[r * ld + (long long)i * K + k], 1.f);
  }
  block_lse(m, s);
  float mn = -INFINITY, sn = 0.f;
  for (int k = threadIdx.x; k < K; k += blockDim.x) lse_merge(mn, sn, row[(long long)i * K + k], 1.f);
  block_lse(mn, sn);
  if (threadIdx.x == 0) {
    den[i] = m + __logf(s);
    nom[i] = mn + __logf(sn);
  }
}

__global__ void milnce_mean_kernel(const float* __restrict__ den, const float* __restrict__ nom, int B,
                                   float* __restrict__ loss) {
  float a = 0.f;
  for (int i = threadIdx.x; i < B; i += blockDim.x) a += den[i] - nom[i];
  a = wave_sum(a);
  __shared__ float sm[16];
  if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = a;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += sm[w];
    loss[0] = t / B;
  }
}

__global__ __launch_bounds__(256) void milnce_bwd_kernel(const float* __restrict__ x, const float* __restrict__ den,
                                                         const float* __restrict__ nom, const float* __restrict__ gout,
                                                         int B, int K, float* __restrict__ dx) {
  const long long ld = (long long)B * K, n = (long long)B * ld;
  const float sc = gout[0] / B;
  for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < n;
       idx += (long long)gridDim.x * blockDim.x) {
    const int i = (int)(idx / ld);
    const long long c = idx - (long long)i * ld;
    const int j = (int)(c / K);
    const float v = x[idx];
    float d = __expf(v - den[i]) + __expf(v - den[j]);
    if (i == j) d -= __expf(v - nom[i]);
    dx[idx] = sc * d;
  }
}

MILNCE_API int milnce_loss_fwd(const float* x, int B, int K, float* den, float* nom, float* loss, hipStream_t stream) {
  hipLaunchKernelGGL(milnce_fwd_kernel, dim3(B), dim3(256), 0, stream, x, B, K, den, nom);
  hipLaunchKernelGGL(milnce_mean_kernel, dim3(1), dim3(256), 0, stream, den, nom, B, loss);
  return (int)hipGetLastError();
}

MILNCE_API int milnce_loss_bwd(const float* x, const float* den, const float* nom, const float* gout, int B, int K,
                               float* dx, hipStream_t stream) {
  const long long n = (long long)B * B * K;
  long long grid = (n + 255) / 256;
  if (grid > 8192) grid = 8192;
  hipLaunchKernelGGL(milnce_bwd_kernel, dim3((int)grid), dim3(256), 0, stream, x, den, nom, gout, B, K, dx);
  return (int)hipGetLastError();
}
