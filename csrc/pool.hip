// Channels-last MaxPool3d for S3D-G:
//   * TF-'SAME' pools (s3dg.py:134-146): zero padding by the TF amounts, then ceil_mode windows
//     (cells of a window that fall past the padded extent are ignored, like PyTorch);
//   * Inception branch-3 pool (s3dg.py:20): kernel 3, stride 1, padding 1 with -inf padding.
// Each lane handles 8 channels of one output cell (16-B loads). The forward stores the winning
// tap (0..kt*kh*kw-1) as a uint8 per element; the backward is a gather: every input cell visits
// the output windows that cover it and sums the gradients whose arg-max points at it
// (deterministic, no atomics). Ties resolve to the first tap in (t, h, w) order, as in ATen.
#include "common.h"

struct PoolParams {
  int T, H, W, C, To, Ho, Wo;
  int kt, kh, kw, st, sh, sw, pt, ph, pw;  // front padding
  int Tp, Hp, Wp;                          // padded extents (input + front + back padding)
  int zero_pad;                            // 1: padded cells are zeros (candidates); 0: -inf (ignored)
};

__global__ __launch_bounds__(256) void maxpool_fwd_kernel(PoolParams p, const bf16_t* __restrict__ x,
                                                          bf16_t* __restrict__ y, uint8_t* __restrict__ arg,
                                                          long long nout_chunks) {
  const int cpr = p.C >> 3;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < nout_chunks;
       i += (long long)gridDim.x * blockDim.x) {
    long long r = i / cpr;
    const int c0 = (int)(i - r * cpr) * 8;
    const int wo = r % p.Wo; r /= p.Wo;
    const int ho = r % p.Ho; r /= p.Ho;
    const int to = r % p.To;
    const long long b = r / p.To;
    float best[8];
    uint32_t bi[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) { best[k] = -INFINITY; bi[k] = 0; }
    int tap = 0;
    for (int dt = 0; dt < p.kt; ++dt) {
      const int tp = to * p.st + dt;       // coordinate in the padded tensor
      const int ti = tp - p.pt;
      for (int dh = 0; dh < p.kh; ++dh) {
        const int hp = ho * p.sh + dh;
        const int hi = hp - p.ph;
        for (int dw = 0; dw < p.kw; ++dw, ++tap) {
          const int wp = wo * p.sw + dw;
          const int wi = wp - p.pw;
          if (tp >= p.Tp || hp >= p.Hp || wp >= p.Wp) continue;  // ceil-mode overhang
          const bool inside = (unsigned)ti < (unsigned)p.T && (unsigned)hi < (unsigned)p.H &&
                              (unsigned)wi < (unsigned)p.W;
          float f[8];
          if (inside) {
            unpack8(*(const uint4*)(x + (((b * p.T + ti) * p.H + hi) * (long long)p.W + wi) * p.C + c0), f);
          } else {
            if (!p.zero_pad) continue;
#pragma unroll
            for (int k = 0; k < 8; ++k) f[k] = 0.f;
          }
#pragma unroll
          for (int k = 0; k < 8; ++k)
            if (f[k] > best[k]) { best[k] = f[k]; bi[k] = tap; }
        }
      }
    }
    const long long o = i * 8;
    *(uint4*)(y + o) = pack8(best);
    uint2 a;
    a.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | (bi[3] << 24);
    a.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | (bi[7] << 24);
    *(uint2*)(arg + o) = a;
  }
}

__device__ __forceinline__ void win_range(int i, int pad, int k, int s, int n_out, int& lo, int& hi) {
  // output indices o with o*s - pad <= i <= o*s - pad + k - 1
  const int a = i + pad - k + 1;
  lo = a <= 0 ? 0 : (a + s - 1) / s;
  hi = (i + pad) / s;
  if (hi > n_out - 1) hi = n_out - 1;
}

// With bn_y != null the gather also emits the BN-backward partial sums of the BN layer that
// produced the pool input (dx is that layer's dz): part[blockIdx][2][C]. Requires 256 % (C/8) == 0
// so every thread keeps one channel chunk across its grid-stride loop.
__global__ __launch_bounds__(256) void maxpool_bwd_kernel(PoolParams p, const bf16_t* __restrict__ dy,
                                                          const uint8_t* __restrict__ arg,
                                                          bf16_t* __restrict__ dx, long long nin_chunks,
                                                          const bf16_t* __restrict__ bn_y,
                                                          const float* __restrict__ bn_ss, float* __restrict__ part) {
  const int cpr = p.C >> 3;
  const bool bn = bn_y != nullptr;
  const int c_fixed = (threadIdx.x % cpr) * 8;
  float mean[8], istd[8], sc[8], sh[8], a1[8], a2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    mean[k] = bn ? bn_ss[c_fixed + k] : 0.f;
    istd[k] = bn ? bn_ss[p.C + c_fixed + k] : 0.f;
    sc[k] = bn ? bn_ss[2 * p.C + c_fixed + k] : 0.f;
    sh[k] = bn ? bn_ss[3 * p.C + c_fixed + k] : 0.f;
    a1[k] = 0.f;
    a2[k] = 0.f;
  }
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < nin_chunks;
       i += (long long)gridDim.x * blockDim.x) {
    long long r = i / cpr;
    const int c0 = (int)(i - r * cpr) * 8;
    const int wi = r % p.W; r /= p.W;
    const int hi = r % p.H; r /= p.H;
    const int ti = r % p.T;
    const long long b = r / p.T;
    float acc[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = 0.f;
    int t0, t1, h0, h1, w0, w1;
    win_range(ti, p.pt, p.kt, p.st, p.To, t0, t1);
    win_range(hi, p.ph, p.kh, p.sh, p.Ho, h0, h1);
    win_range(wi, p.pw, p.kw, p.sw, p.Wo, w0, w1);
    for (int to = t0; to <= t1; ++to) {
      const int dt = ti + p.pt - to * p.st;
      for (int ho = h0; ho <= h1; ++ho) {
        const int dh = hi + p.ph - ho * p.sh;
        for (int wo = w0; wo <= w1; ++wo) {
          const int dw = wi + p.pw - wo * p.sw;
          const uint32_t tap = (dt * p.kh + dh) * p.kw + dw;
          const long long o = ((((b * p.To + to) * p.Ho + ho) * (long long)p.Wo + wo) * p.C + c0);
          const uint2 a = *(const uint2*)(arg + o);
          const uint4 g = *(const uint4*)(dy + o);
          float gf[8];
          unpack8(g, gf);
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const uint32_t ak = ((k < 4 ? a.x : a.y) >> (8 * (k & 3))) & 0xff;
            if (ak == tap) acc[k] += gf[k];
          }
        }
      }
    }
    *(uint4*)(dx + i * 8) = pack8(acc);
    if (bn) {
      float y[8];
      unpack8(*(const uint4*)(bn_y + i * 8), y);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float gm = (y[k] * sc[k] + sh[k] > 0.f) ? acc[k] : 0.f;
        a1[k] += gm;
        a2[k] += gm * (y[k] - mean[k]) * istd[k];
      }
    }
  }
  if (!bn) return;
  __shared__ float red[2][8][256];
#pragma unroll
  for (int k = 0; k < 8; ++k) { red[0][k][threadIdx.x] = a1[k]; red[1][k][threadIdx.x] = a2[k]; }
  __syncthreads();
  if ((int)threadIdx.x < cpr) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float s1 = 0.f, s2 = 0.f;
      for (int j = threadIdx.x; j < 256; j += cpr) { s1 += red[0][k][j]; s2 += red[1][k][j]; }
      part[(long long)blockIdx.x * 2 * p.C + c_fixed + k] = s1;
      part[(long long)blockIdx.x * 2 * p.C + p.C + c_fixed + k] = s2;
    }
  }
}

static PoolParams make_pool(int T, int H, int W, int C, int To, int Ho, int Wo, int kt, int kh, int kw, int st,
                            int sh, int sw, int pt0, int pt1, int ph0, int ph1, int pw0, int pw1, int zero_pad) {
  PoolParams p;
  p.T = T; p.H = H; p.W = W; p.C = C; p.To = To; p.Ho = Ho; p.Wo = Wo;
  p.kt = kt; p.kh = kh; p.kw = kw; p.st = st; p.sh = sh; p.sw = sw;
  p.pt = pt0; p.ph = ph0; p.pw = pw0;
  p.Tp = T + pt0 + pt1; p.Hp = H + ph0 + ph1; p.Wp = W + pw0 + pw1;
  p.zero_pad = zero_pad;
  return p;
}

static int grid_for(long long n) {
  long long g = (n + 255) / 256;
  return (int)(g > 16384 ? 16384 : (g < 1 ? 1 : g));
}

MILNCE_API int milnce_maxpool_fwd(const void* x, void* y, void* arg, int B, int T, int H, int W, int C, int To,
                                  int Ho, int Wo, int kt, int kh, int kw, int st, int sh, int sw, int pt0, int pt1,
                                  int ph0, int ph1, int pw0, int pw1, int zero_pad, hipStream_t stream) {
  if (C % 8) return (int)hipErrorInvalidValue;
  PoolParams p = make_pool(T, H, W, C, To, Ho, Wo, kt, kh, kw, st, sh, sw, pt0, pt1, ph0, ph1, pw0, pw1, zero_pad);
  const long long n = (long long)B * To * Ho * Wo * (C / 8);
  hipLaunchKernelGGL(maxpool_fwd_kernel, dim3(grid_for(n)), dim3(256), 0, stream, p, (const bf16_t*)x,
                     (bf16_t*)y, (uint8_t*)arg, n);
  return (int)hipGetLastError();
}

// nparts: grid size used (also the number of partial rows written when bn_y != null).
MILNCE_API int milnce_maxpool_bwd(const void* dy, const void* arg, void* dx, int B, int T, int H, int W, int C,
                                  int To, int Ho, int Wo, int kt, int kh, int kw, int st, int sh, int sw, int pt0,
                                  int pt1, int ph0, int ph1, int pw0, int pw1, int zero_pad, const void* bn_y,
                                  const float* bn_ss, float* part, int nparts, hipStream_t stream) {
  if (C % 8) return (int)hipErrorInvalidValue;
  if (bn_y != nullptr && 256 % (C / 8) != 0) return (int)hipErrorInvalidValue;
  PoolParams p = make_pool(T, H, W, C, To, Ho, Wo, kt, kh, kw, st, sh, sw, pt0, pt1, ph0, ph1, pw0, pw1, zero_pad);
  const long long n = (long long)B * T * H * W * (C / 8);
  hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(nparts), dim3(256), 0, stream, p, (const bf16_t*)dy,
                     (const uint8_t*)arg, (bf16_t*)dx, n, (const bf16_t*)bn_y, bn_ss, part);
  return (int)hipGetLastError();
}
