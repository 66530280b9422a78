// Channels-last MaxPool3d for S3D-G:
//   * TF-'SAME' pools (s3dg.py:134-146): zero padding by the TF amounts, then ceil_mode windows
//     (cells of a window that fall past the padded extent are ignored, like PyTorch);
//   * Inception branch-3 pool (s3dg.py:20): kernel 3, stride 1, padding 1 with -inf padding.
// Each lane handles 8 channels of one output cell (16-B loads). The forward stores the winning
// tap (0..kt*kh*kw-1) as a uint8 per element; the backward is a gather: every input cell visits
// the output windows that cover it and sums the gradients whose arg-max points at it
// (deterministic, no atomics). Ties resolve to the first tap in (t, h, w) order, as in ATen.
#include "common.h"
#include <algorithm>
#include <type_traits>

struct PoolParams {
  int T, H, W, C, To, Ho, Wo;
  int kt, kh, kw, st, sh, sw, pt, ph, pw;  // front padding
  int Tp, Hp, Wp;                          // padded extents (input + front + back padding)
  int zero_pad;                            // 1: padded cells are zeros (candidates); 0: -inf (ignored)
  int s1_codes;                            // stride-1 plane sweeps: 1 = workgroup-order codes (S1Geo)
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

// ---------------------------------------------------------------------------------------
// Specialised pools: window/stride are template constants (every S3D-G pool is one of four
// shapes), index math is 32-bit FastDiv, and every tap's load is issued unconditionally from a
// clamped address and masked afterwards, so the whole window's loads are in flight at once
// (the generic kernels above serialise on their per-tap branches).
struct PoolDivs {
  FastDiv fcpr, fWo, fHo, fTo, fW, fH, fT, fplane;  // fplane: T * H * W (input clip)
  FastDiv fmt, fmh, fmw;  // block counts of the stride-2 block gather (pool_bwd_block)
};

// BN: x is the raw conv output of a train-mode BN layer and z = relu(x * scale + shift) is
// pooled without being materialised (ss = [mean, invstd, scale, shift] per channel); padded
// cells stay zero candidates, as for the z the unfused pool would read.
template <int KT, int KH, int KW, int ST, int SH, int SW, bool BN = false, bool GATE = false>
__global__ __launch_bounds__(256) void maxpool_fwd_t(PoolParams p, PoolDivs d, const bf16_t* __restrict__ x,
                                                     bf16_t* __restrict__ y, uint8_t* __restrict__ arg,
                                                     uint32_t nout_chunks, const float* __restrict__ ss = nullptr,
                                                     const float* __restrict__ gate = nullptr,
                                                     bf16_t* __restrict__ yr = nullptr) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nout_chunks; i += gridDim.x * blockDim.x) {
    uint32_t r = fdiv(i, d.fcpr);
    const int c0 = (int)(i - r * d.fcpr.d) * 8;
    uint32_t q = fdiv(r, d.fWo);
    const int wo = (int)(r - q * p.Wo);
    uint32_t q2 = fdiv(q, d.fHo);
    const int ho = (int)(q - q2 * p.Ho);
    const uint32_t b = fdiv(q2, d.fTo);
    const int to = (int)(q2 - b * p.To);
    const bf16_t* xb = x + (size_t)b * p.T * p.H * p.W * p.C + c0;
    uint4 v[KT * KH * KW];
    bool in[KT * KH * KW], cand[KT * KH * KW];
#pragma unroll
    for (int dt = 0; dt < KT; ++dt)
#pragma unroll
      for (int dh = 0; dh < KH; ++dh)
#pragma unroll
        for (int dw = 0; dw < KW; ++dw) {
          const int t = (dt * KH + dh) * KW + dw;
          const int tp = to * ST + dt, hp = ho * SH + dh, wp = wo * SW + dw;
          const int ti = tp - p.pt, hi = hp - p.ph, wi = wp - p.pw;
          in[t] = ((unsigned)ti < (unsigned)p.T) & ((unsigned)hi < (unsigned)p.H) & ((unsigned)wi < (unsigned)p.W);
          // padded (non-overhang) cells are zero candidates for TF-SAME pools
          cand[t] = in[t] | (p.zero_pad & (tp < p.Tp) & (hp < p.Hp) & (wp < p.Wp));
          const size_t off = in[t] ? ((size_t)(ti * p.H + hi) * p.W + wi) * p.C : 0;
          v[t] = *(const uint4*)(xb + off);
        }
    float best[8], sc[8], sh[8], gv[8], braw[8];
    uint32_t bi[8];
    bool have_real = false;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      best[k] = -INFINITY;
      bi[k] = 0;
      braw[k] = 0.f;
      if constexpr (BN) {
        sc[k] = ss[2 * p.C + c0 + k];
        sh[k] = ss[3 * p.C + c0 + k];
        if constexpr (GATE) gv[k] = gate[(size_t)b * p.C + c0 + k];
      }
    }
#pragma unroll
    for (int t = 0; t < KT * KH * KW; ++t) {
      float f[8], raw[8];
      unpack8(v[t], f);
      if constexpr (BN) {
        // yr: the raw conv output at each arg-max (any real window cell when the maximum is a zero
        // pad candidate: every real cell's z is 0 then, so its BN mask is off like the pad's)
#pragma unroll
        for (int k = 0; k < 8; ++k) raw[k] = f[k];
      }
      if constexpr (BN) {
        // = the stored z (rounded in pairs: one v_cvt_pk_bf16_f32 per two channels, same bits)
#pragma unroll
        for (int k = 0; k < 8; k += 2) {
          const uint32_t z2 = pack2bf(fmaxf(f[k] * sc[k] + sh[k], 0.f), fmaxf(f[k + 1] * sc[k + 1] + sh[k + 1], 0.f));
          f[k] = __uint_as_float(z2 << 16);
          f[k + 1] = __uint_as_float(z2 & 0xffff0000u);
        }
        if constexpr (GATE) {  // SelfGating output z * gate[b, c], as gate_scale would store it
#pragma unroll
          for (int k = 0; k < 8; k += 2) {
            const uint32_t g2 = pack2bf(f[k] * gv[k], f[k + 1] * gv[k + 1]);
            f[k] = __uint_as_float(g2 << 16);
            f[k + 1] = __uint_as_float(g2 & 0xffff0000u);
          }
        }
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float val = in[t] ? f[k] : (cand[t] ? 0.f : -INFINITY);
        const bool gt = val > best[k];
        best[k] = gt ? val : best[k];
        bi[k] = gt ? (uint32_t)t : bi[k];
        if constexpr (BN) braw[k] = ((gt && in[t]) || (in[t] && !have_real)) ? raw[k] : braw[k];
      }
      have_real |= in[t];
    }
    const size_t o = (size_t)i * 8;
    *(uint4*)(y + o) = pack8(best);
    uint2 a;
    a.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | (bi[3] << 24);
    a.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | (bi[7] << 24);
    *(uint2*)(arg + o) = a;
    if constexpr (BN) {
      if (yr != nullptr) *(uint4*)(yr + o) = pack8(braw);  // exact: bf16 values
    }
  }
}

// Pair forward for the 1x3x3 / (1,2,2) windows without leading padding (maxpool_2a / 3a): a thread
// owns two horizontally adjacent output cells (one 8-channel chunk) and reads the 3 x 5 input patch
// under them once, each cell feeding the one or two windows that contain it: 7.5 loads and BN /
// gate transforms per output instead of 9 (the BN forward is VALU-bound on the per-tap transform).
// Cells are visited in (h, w) order, so each window still sees its taps in scan order and the first
// maximum wins. Without leading padding every window starts with a real cell and a trailing zero
// pad never beats it, so the arg-max is a real cell and yr is the raw value there. (A 2x2-quad
// version needed 4 windows of state and ran slower: occupancy and compare-mask pressure.)
template <bool BN = false, bool GATE = false>
__global__ __launch_bounds__(256) void maxpool_fwd_pair(PoolParams p, PoolDivs d, const bf16_t* __restrict__ x,
                                                        bf16_t* __restrict__ y, uint8_t* __restrict__ arg,
                                                        uint32_t npair_chunks, int Wq,
                                                        const float* __restrict__ ss = nullptr,
                                                        const float* __restrict__ gate = nullptr,
                                                        bf16_t* __restrict__ yr = nullptr) {
  constexpr bool YR = BN;  // the raw value at each arg-max (yr), when asked for
  const FastDiv fWq = d.fmw;  // Wq, set by the launcher
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < npair_chunks; i += gridDim.x * blockDim.x) {
    const uint32_t r = fdiv(i, d.fcpr);
    const int c0 = (int)(i - r * d.fcpr.d) * 8;
    const uint32_t q = fdiv(r, fWq);
    const int wq = (int)(r - q * Wq);
    const uint32_t q2 = fdiv(q, d.fHo);
    const int ho = (int)(q - q2 * p.Ho);
    const uint32_t b = fdiv(q2, d.fTo);
    const int to = (int)(q2 - b * p.To);
    const bf16_t* xb = x + ((size_t)b * p.T + to) * p.H * p.W * p.C + c0;
    const int h0 = 2 * ho, w0 = 4 * wq;
    uint4 v[3][5];
#pragma unroll
    for (int rr = 0; rr < 3; ++rr)
#pragma unroll
      for (int cc = 0; cc < 5; ++cc) {
        const bool in = (h0 + rr < p.H) & (w0 + cc < p.W);
        v[rr][cc] = *(const uint4*)(xb + (in ? ((size_t)(h0 + rr) * p.W + w0 + cc) * p.C : 0));
      }
    float sc[8], sh[8], gv[8];
    if constexpr (BN) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        sc[k] = ss[2 * p.C + c0 + k];
        sh[k] = ss[3 * p.C + c0 + k];
        if constexpr (GATE) gv[k] = gate[(size_t)b * p.C + c0 + k];
      }
    }
    float best[2][8], braw[YR ? 2 : 1][8];
    uint32_t bi[2][8];
#pragma unroll
    for (int o = 0; o < 2; ++o)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        best[o][k] = -INFINITY;
        bi[o][k] = 0u;
        if constexpr (YR) braw[o][k] = 0.f;
      }
#pragma unroll
    for (int rr = 0; rr < 3; ++rr)
#pragma unroll
      for (int cc = 0; cc < 5; ++cc) {
        const bool in = (h0 + rr < p.H) & (w0 + cc < p.W);
        const bool cand = in | (p.zero_pad & (h0 + rr < p.Hp) & (w0 + cc < p.Wp));
        float f[8], raw[8];
        unpack8(v[rr][cc], f);
        if constexpr (YR) {
#pragma unroll
          for (int k = 0; k < 8; ++k) raw[k] = f[k];
        }
        if constexpr (BN) {  // = the stored z (rounded in pairs)
#pragma unroll
          for (int k = 0; k < 8; k += 2) {
            const uint32_t z2 = pack2bf(fmaxf(f[k] * sc[k] + sh[k], 0.f), fmaxf(f[k + 1] * sc[k + 1] + sh[k + 1], 0.f));
            f[k] = __uint_as_float(z2 << 16);
            f[k + 1] = __uint_as_float(z2 & 0xffff0000u);
          }
          if constexpr (GATE) {  // SelfGating output z * gate[b, c], as gate_scale would store it
#pragma unroll
            for (int k = 0; k < 8; k += 2) {
              const uint32_t g2 = pack2bf(f[k] * gv[k], f[k + 1] * gv[k + 1]);
              f[k] = __uint_as_float(g2 << 16);
              f[k + 1] = __uint_as_float(g2 & 0xffff0000u);
            }
          }
        }
        const float pad = cand ? 0.f : -INFINITY;
#pragma unroll
        for (int o = 0; o < 2; ++o) {
          const int dw = cc - 2 * o;
          if (dw < 0 || dw > 2) continue;  // compile time after unrolling
          const uint32_t tap = (uint32_t)(rr * 3 + dw);
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const float val = in ? f[k] : pad;
            const bool gt = val > best[o][k];
            best[o][k] = gt ? val : best[o][k];
            bi[o][k] = gt ? tap : bi[o][k];
            if constexpr (YR) braw[o][k] = gt ? raw[k] : braw[o][k];
          }
        }
      }
#pragma unroll
    for (int o = 0; o < 2; ++o) {
      const int wo = 2 * wq + o;
      if (wo >= p.Wo) continue;
      const size_t oo = ((((size_t)b * p.To + to) * p.Ho + ho) * p.Wo + wo) * p.C + c0;
      *(uint4*)(y + oo) = pack8(best[o]);
      *(uint2*)(arg + oo) = make_uint2(bi[o][0] | (bi[o][1] << 8) | (bi[o][2] << 16) | (bi[o][3] << 24),
                                       bi[o][4] | (bi[o][5] << 8) | (bi[o][6] << 16) | (bi[o][7] << 24));
      if constexpr (YR) {
        if (yr != nullptr) *(uint4*)(yr + oo) = pack8(braw[o]);
      }
    }
  }
}

// BN-backward partial sums of the pool input's producer (dx is that layer's dz), accumulated
// per thread for its fixed channel chunk and reduced over the block's row groups in LDS:
// part[blockIdx][2][C] (mask = y*scale + shift > 0, xhat = (y - mean) * invstd).
struct BnAcc {
  float a1[8], a2[8];
  float mu[8], is[8], sc[8], sh[8];  // the thread's channels' [mean, invstd, scale, shift], loaded once
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int k = 0; k < 8; ++k) { a1[k] = 0.f; a2[k] = 0.f; }
  }
  __device__ __forceinline__ void load(const float* ss, int C, int c0) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      mu[k] = ss[c0 + k]; is[k] = ss[C + c0 + k]; sc[k] = ss[2 * C + c0 + k]; sh[k] = ss[3 * C + c0 + k];
    }
  }
  __device__ __forceinline__ void add(const float* d, const bf16_t* ypos) { addv(d, *(const uint4*)ypos); }
  __device__ __forceinline__ void addv(const float* d, const uint4& yraw) {
    float yv[8];
    unpack8(yraw, yv);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float gm = (yv[k] * sc[k] + sh[k] > 0.f) ? d[k] : 0.f;
      a1[k] += gm;
      a2[k] += gm * (yv[k] - mu[k]) * is[k];
    }
  }
  __device__ __forceinline__ void commit(float* red, float* part, int C, int cpr, int rpi, int cc, int rr,
                                         bool active) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int k = 0; k < 8; ++k) { red[k * 256 + tid] = a1[k]; red[(8 + k) * 256 + tid] = a2[k]; }
    __syncthreads();
    if (active && rr == 0) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float s1 = 0.f, s2 = 0.f;
        for (int j = 0; j < rpi; ++j) { s1 += red[k * 256 + j * cpr + cc]; s2 += red[(8 + k) * 256 + j * cpr + cc]; }
        part[(size_t)blockIdx.x * 2 * C + cc * 8 + k] = s1;
        part[(size_t)blockIdx.x * 2 * C + C + cc * 8 + k] = s2;
      }
    }
  }
};

// Gather backward: output windows covering input i along one dim are o = (i+pad)/S - j,
// j < ceil(K/S), valid when 0 <= o < n_out and the in-window offset i+pad-o*S < K.
template <int KT, int KH, int KW, int ST, int SH, int SW>
__device__ __forceinline__ void pool_bwd_one(const PoolParams& p, const PoolDivs& d, const bf16_t* __restrict__ dy,
                                             const uint8_t* __restrict__ arg, uint32_t pos, int c0, float* acc) {
  constexpr int NT = (KT + ST - 1) / ST, NH = (KH + SH - 1) / SH, NW = (KW + SW - 1) / SW;
  uint32_t q = fdiv(pos, d.fW);
  const int wi = (int)(pos - q * p.W);
  uint32_t q2 = fdiv(q, d.fH);
  const int hi = (int)(q - q2 * p.H);
  const uint32_t b = fdiv(q2, d.fT);
  const int ti = (int)(q2 - b * p.T);
  const size_t obase = (size_t)b * p.To * p.Ho * p.Wo * p.C + c0;
  uint4 g[NT * NH * NW];
  uint2 a[NT * NH * NW];
  uint32_t tap[NT * NH * NW];
  bool ok[NT * NH * NW];
#pragma unroll
  for (int jt = 0; jt < NT; ++jt)
#pragma unroll
    for (int jh = 0; jh < NH; ++jh)
#pragma unroll
      for (int jw = 0; jw < NW; ++jw) {
        const int u = (jt * NH + jh) * NW + jw;
        const int to = (ti + p.pt) / ST - jt, ho = (hi + p.ph) / SH - jh, wo = (wi + p.pw) / SW - jw;
        const int dt = ti + p.pt - to * ST, dh = hi + p.ph - ho * SH, dw = wi + p.pw - wo * SW;
        ok[u] = (to >= 0) & (to < p.To) & (dt < KT) & (ho >= 0) & (ho < p.Ho) & (dh < KH) & (wo >= 0) &
                (wo < p.Wo) & (dw < KW);
        tap[u] = (uint32_t)((dt * KH + dh) * KW + dw);
        const size_t o = ok[u] ? obase + ((size_t)(to * p.Ho + ho) * p.Wo + wo) * p.C : obase;
        g[u] = *(const uint4*)(dy + o);
        a[u] = *(const uint2*)(arg + o);
      }
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] = 0.f;
#pragma unroll
  for (int u = 0; u < NT * NH * NW; ++u) {
    float gf[8];
    unpack8(g[u], gf);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint32_t ak = ((k < 4 ? a[u].x : a[u].y) >> (8 * (k & 3))) & 0xff;
      acc[k] += (ok[u] & (ak == tap[u])) ? gf[k] : 0.f;
    }
  }
}

// Quad gather for the 1x3x3 stride-(1,2,2) window with no leading padding and H = 2 Ho, W = 2 Wo
// (maxpool_2a / maxpool_3a): the 2x2 input quad (2 h2 + eh, 2 w2 + ew) is covered by the outputs
// (h2 - jh, w2 - jw), jh, jw in {0, 1}, at window offsets (eh + 2 jh, ew + 2 jw) (< 3 to count).
// One thread loads those 4 output cells once for 4 inputs instead of 4 cells per input.
__device__ __forceinline__ void pool_bwd_quad(const PoolParams& p, const bf16_t* __restrict__ dy,
                                              const uint8_t* __restrict__ arg, uint32_t bt, int h2, int w2,
                                              int c0, float (*acc)[8]) {
  uint4 g[4];
  uint2 a[4];
  bool ok[4];
#pragma unroll
  for (int jh = 0; jh < 2; ++jh)
#pragma unroll
    for (int jw = 0; jw < 2; ++jw) {
      const int u = jh * 2 + jw, ho = h2 - jh, wo = w2 - jw;
      ok[u] = (ho >= 0) & (wo >= 0);
      const size_t o = ((size_t)(bt * p.Ho + (ok[u] ? ho : 0)) * p.Wo + (ok[u] ? wo : 0)) * p.C + c0;
      g[u] = *(const uint4*)(dy + o);
      a[u] = *(const uint2*)(arg + o);
    }
#pragma unroll
  for (int e = 0; e < 4; ++e)
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[e][k] = 0.f;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int jh = u >> 1, jw = u & 1;
    float gf[8];
    unpack8(g[u], gf);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int eh = e >> 1, ew = e & 1;
      const int dh = eh + 2 * jh, dw = ew + 2 * jw;
      if (dh >= 3 || dw >= 3) continue;  // compile-time after unrolling
      const uint32_t tap = (uint32_t)(dh * 3 + dw);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint32_t ak = ((k < 4 ? a[u].x : a[u].y) >> (8 * (k & 3))) & 0xff;
        acc[e][k] += (ok[u] & (ak == tap)) ? gf[k] : 0.f;
      }
    }
  }
}

// Block gather for stride-2, 3-wide windows (maxpool_2a / 3a: 1x3x3 / (1,2,2); maxpool_4a:
// 3x3x3 / 2). Along a (K=3, S=2, leading pad p in {0, 1}) dim, block index m covers the inputs
// i = 2m - p + e (e in {0, 1}), whose windows are the outputs o = m - j (j in {0, 1}) at window
// offset e + 2j (counted when < 3); with NT == 1 the T dim is (K=1, S=1): t -> t. One thread
// loads the NT*4 output cells once for its NT*4 inputs instead of NT*4 cells per input.
template <int NT>
__device__ __forceinline__ void pool_bwd_block(const PoolParams& p, const bf16_t* __restrict__ dy,
                                               const uint8_t* __restrict__ arg, uint32_t b, int mt, int mh, int mw,
                                               int c0, float (*acc)[8]) {
  constexpr int NU = NT * 4;
  uint4 g[NU];
  uint2 a[NU];
  bool ok[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int jt = u >> 2, jh = (u >> 1) & 1, jw = u & 1;
    const int to = mt - jt, ho = mh - jh, wo = mw - jw;
    ok[u] = (to >= 0) & (to < p.To) & (ho >= 0) & (ho < p.Ho) & (wo >= 0) & (wo < p.Wo);
    const size_t o = ok[u] ? ((((size_t)b * p.To + to) * p.Ho + ho) * p.Wo + wo) * p.C + c0 : (size_t)c0;
    g[u] = *(const uint4*)(dy + o);
    a[u] = *(const uint2*)(arg + o);
  }
#pragma unroll
  for (int e = 0; e < NU; ++e)
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[e][k] = 0.f;
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int jt = u >> 2, jh = (u >> 1) & 1, jw = u & 1;
    float gf[8];
    unpack8(g[u], gf);
#pragma unroll
    for (int e = 0; e < NU; ++e) {
      const int et = e >> 2, eh = (e >> 1) & 1, ew = e & 1;
      const int dt = NT == 2 ? et + 2 * jt : 0, dh = eh + 2 * jh, dw = ew + 2 * jw;
      if (dt >= 3 || dh >= 3 || dw >= 3) continue;  // compile-time after unrolling
      const uint32_t tap = (uint32_t)((dt * 3 + dh) * 3 + dw);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint32_t ak = ((k < 4 ? a[u].x : a[u].y) >> (8 * (k & 3))) & 0xff;
        acc[e][k] += (ok[u] & (ak == tap)) ? gf[k] : 0.f;
      }
    }
  }
}

// Thread = fixed 8-channel chunk cc = tid % cpr of rpi = 256/cpr input positions per step; block
// blockIdx.x walks positions [pos_begin, pos_end), two positions per thread per iteration so
// both gathers' loads are in flight together. MODE (compile time, so every variant keeps only
// the registers it needs):
//   POOL_BWD_PLAIN  dx = gathered gradient (+ BN partials of the producer, + SelfGating sums gs)
//   POOL_BWD_GATED  dx = bf16(gathered * g[b, c] + dmean[b, c] / thw): the producer gate's input
//                   gradient (its reduction already done), + BN partials; dx may be null
//   POOL_BWD_APPLY  dx = BN backward of the (optionally gated, gate_g != null) gradient with the
//                   finalised coefficients coef: the producer conv's output gradient
enum { POOL_BWD_PLAIN = 0, POOL_BWD_GATED = 1, POOL_BWD_APPLY = 2 };

template <int KT, int KH, int KW, int ST, int SH, int SW, int MODE = POOL_BWD_PLAIN, int QUAD = 0>
__global__ __launch_bounds__(256) void maxpool_bwd_t(PoolParams p, PoolDivs d, const bf16_t* __restrict__ dy,
                                                     const uint8_t* __restrict__ arg, bf16_t* __restrict__ dx,
                                                     uint32_t npos, uint32_t pos_per_block,
                                                     const bf16_t* __restrict__ bn_y, int bn_ld,
                                                     const float* __restrict__ bn_ss, float* __restrict__ part,
                                                     const bf16_t* __restrict__ gx = nullptr,
                                                     float* __restrict__ gs = nullptr,
                                                     const float* __restrict__ gate_g = nullptr,
                                                     const float* __restrict__ gate_dm = nullptr,
                                                     float inv_thw = 0.f, const float* __restrict__ coef = nullptr,
                                                     float* __restrict__ gpart = nullptr) {
  __shared__ float red[16 * 256];
  const int cpr = p.C >> 3, rpi = 256 / cpr;
  const int cc = threadIdx.x % cpr, rr = threadIdx.x / cpr;
  const bool active = rr < rpi;
  const int c0 = cc * 8;
  const bool bn = MODE != POOL_BWD_APPLY && bn_y != nullptr && part != nullptr;  // BN partial sums of dz
  const bool gated = MODE == POOL_BWD_GATED || (MODE == POOL_BWD_APPLY && gate_g != nullptr);
  BnAcc acc_bn;
  acc_bn.zero();
  if (bn && active) acc_bn.load(bn_ss, p.C, c0);
  const uint32_t pos_begin = blockIdx.x * pos_per_block;
  const uint32_t pos_end = min(npos, pos_begin + pos_per_block);
  // gate reduction of the pool input's producer (SelfGating): gs[b, c] += sum dx * gx. With gpart
  // (a block's items span at most two clips): the thread keeps its first clip's sum aside at the
  // clip change and the block writes one partial row per clip slot at the end, summed over the
  // blocks in order by pool_gs_sum_kernel (deterministic); without: one atomic per channel
  // whenever the thread's clip changes.
  float sacc[8], sprev[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) sprev[k] = 0.f;
  uint32_t cur_b = 0xffffffffu, prev_b = 0xffffffffu;
  auto gs_add = [&](uint32_t ps, const uint4& v, const uint4& xg) {
    const uint32_t bb = fdiv(ps, d.fplane);
    if (bb != cur_b) {
      if (cur_b != 0xffffffffu) {
        if (gpart != nullptr && prev_b == 0xffffffffu) {
          prev_b = cur_b;
#pragma unroll
          for (int k = 0; k < 8; ++k) sprev[k] = sacc[k];
        } else {
#pragma unroll
          for (int k = 0; k < 8; ++k) unsafeAtomicAdd(gs + (size_t)cur_b * p.C + c0 + k, sacc[k]);
        }
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) sacc[k] = 0.f;
      cur_b = bb;
    }
    float q[8], xv[8];
    unpack8(v, q);
    unpack8(xg, xv);
#pragma unroll
    for (int k = 0; k < 8; ++k) sacc[k] += q[k] * xv[k];
  };
  // SelfGating backward of the producer: dz = bf16(dx * g + dmean / thw), per-clip constants
  float gcur[8], dcur[8];
  uint32_t gb = 0xffffffffu;
  auto gate_apply = [&](uint32_t ps, uint4& v) {
    const uint32_t bb = fdiv(ps, d.fplane);
    if (bb != gb) {
      gb = bb;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        gcur[k] = gate_g[(size_t)bb * p.C + c0 + k];
        dcur[k] = gate_dm[(size_t)bb * p.C + c0 + k] * inv_thw;
      }
    }
    float q[8];
    unpack8(v, q);
#pragma unroll
    for (int k = 0; k < 8; ++k) q[k] = fmaf(q[k], gcur[k], dcur[k]);
    v = pack8(q);
  };
  // BN backward constants of this thread's channels (APPLY): dy = k0 * (dz*mask - k1 - xhat*k2)
  BnBwdC bq[8];
  if constexpr (MODE == POOL_BWD_APPLY) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int c = active ? c0 + k : 0;
      bq[k] = bn_bwd_const(bn_ss[c], bn_ss[p.C + c], bn_ss[2 * p.C + c], bn_ss[3 * p.C + c], coef[c],
                           coef[p.C + c], coef[2 * p.C + c]);
    }
  }
  auto bn_apply = [&](uint32_t ps, uint4& v, const uint4* ypre = nullptr) {
    float dz[8], yv[8], o[8];
    unpack8(v, dz);
    unpack8(ypre != nullptr ? *ypre : *(const uint4*)(bn_y + (size_t)ps * bn_ld + c0), yv);
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = bn_bwd_elem(dz[k], yv[k], bq[k]);
    v = pack8(o);
  };
  // one input position's epilogue (the quad path; the pair loop below interleaves two of them)
  // ypre / xpre: the position's bn_y / gx rows when the caller already loaded them
  auto finish = [&](uint32_t ps, const float* a, const uint4* ypre = nullptr, const uint4* xpre = nullptr) {
    uint4 v = pack8(a);
    if (gated) gate_apply(ps, v);
    if (MODE == POOL_BWD_PLAIN && gs != nullptr)
      gs_add(ps, v, xpre != nullptr ? *xpre : *(const uint4*)(gx + (size_t)ps * p.C + c0));
    if (bn) {
      float dr[8];
      unpack8(v, dr);
      if (ypre != nullptr) acc_bn.addv(dr, *ypre);
      else acc_bn.add(dr, bn_y + (size_t)ps * bn_ld + c0);
    }
    if constexpr (MODE == POOL_BWD_APPLY) bn_apply(ps, v, ypre);
    if (dx != nullptr) *(uint4*)(dx + (size_t)ps * p.C + c0) = v;
  };
  if constexpr (QUAD == 1) {  // pos indexes 2x2 input quads (b, t, h2, w2) of an even H, W plane
    for (uint32_t q = pos_begin + rr; active && q < pos_end; q += rpi) {
      const uint32_t r = fdiv(q, d.fWo);
      const int w2 = (int)(q - r * p.Wo);
      const uint32_t bt = fdiv(r, d.fHo);
      const int h2 = (int)(r - bt * p.Ho);
      float a[4][8];
      const uint32_t p00 = (bt * p.H + 2 * h2) * p.W + 2 * w2;
      // the quad's per-position side inputs (BN input rows, gate input rows) are loaded together
      // with the gather, not one after each store
      const bool need_y = MODE == POOL_BWD_APPLY || bn;
      const bool need_x = MODE == POOL_BWD_PLAIN && gs != nullptr;
      const uint32_t pq[4] = {p00, p00 + 1, p00 + p.W, p00 + p.W + 1};
      uint4 yq[4], xq[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (need_y) yq[i] = *(const uint4*)(bn_y + (size_t)pq[i] * bn_ld + c0);
        if (need_x) xq[i] = *(const uint4*)(gx + (size_t)pq[i] * p.C + c0);
      }
      pool_bwd_quad(p, dy, arg, bt, h2, w2, c0, a);
#pragma unroll
      for (int i = 0; i < 4; ++i) finish(pq[i], a[i], need_y ? &yq[i] : nullptr, need_x ? &xq[i] : nullptr);
    }
  }
  if constexpr (QUAD == 2) {  // pos indexes input blocks (b, mt, mh, mw), see pool_bwd_block
    constexpr int NT = KT == 3 ? 2 : 1, NU = NT * 4;
    for (uint32_t q = pos_begin + rr; active && q < pos_end; q += rpi) {
      const uint32_t r = fdiv(q, d.fmw);
      const int mw = (int)(q - r * d.fmw.d);
      const uint32_t r2 = fdiv(r, d.fmh);
      const int mh = (int)(r - r2 * d.fmh.d);
      const uint32_t b = fdiv(r2, d.fmt);
      const int mt = (int)(r2 - b * d.fmt.d);
      float a[NU][8];
      pool_bwd_block<NT>(p, dy, arg, b, mt, mh, mw, c0, a);
#pragma unroll
      for (int e = 0; e < NU; ++e) {
        const int it = NT == 2 ? 2 * mt - p.pt + (e >> 2) : mt;
        const int ih = 2 * mh - p.ph + ((e >> 1) & 1), iw = 2 * mw - p.pw + (e & 1);
        if (it >= 0 && it < p.T && ih >= 0 && ih < p.H && iw >= 0 && iw < p.W)
          finish(((b * p.T + it) * p.H + ih) * p.W + iw, a[e]);
      }
    }
  }
  for (uint32_t pos = pos_begin + rr; QUAD == 0 && active && pos < pos_end; pos += 2 * rpi) {
    const uint32_t pos2 = pos + rpi;
    const bool two = pos2 < pos_end;
    float a0[8], a1[8];
    // the gate operand rows are loaded up front, with the gather's loads
    uint4 xg0 = make_uint4(0, 0, 0, 0), xg1 = make_uint4(0, 0, 0, 0);
    if (MODE == POOL_BWD_PLAIN && gs != nullptr) {
      xg0 = *(const uint4*)(gx + (size_t)pos * p.C + c0);
      xg1 = *(const uint4*)(gx + (size_t)(two ? pos2 : pos) * p.C + c0);
    }
    pool_bwd_one<KT, KH, KW, ST, SH, SW>(p, d, dy, arg, pos, c0, a0);
    pool_bwd_one<KT, KH, KW, ST, SH, SW>(p, d, dy, arg, two ? pos2 : pos, c0, a1);
    uint4 v0 = pack8(a0), v1 = pack8(a1);
    if (gated) {
      gate_apply(pos, v0);
      if (two) gate_apply(pos2, v1);
    }
    if (MODE == POOL_BWD_PLAIN && gs != nullptr) {
      gs_add(pos, v0, xg0);
      if (two) gs_add(pos2, v1, xg1);
    }
    if (bn) {
      float dr[8];
      unpack8(v0, dr);
      acc_bn.add(dr, bn_y + (size_t)pos * bn_ld + c0);
      if (two) {
        unpack8(v1, dr);
        acc_bn.add(dr, bn_y + (size_t)pos2 * bn_ld + c0);
      }
    }
    if constexpr (MODE == POOL_BWD_APPLY) {
      bn_apply(pos, v0);
      if (two) bn_apply(pos2, v1);
    }
    if (dx != nullptr) {  // null: BN partial sums only (a later APPLY pass re-gathers dz)
      *(uint4*)(dx + (size_t)pos * p.C + c0) = v0;
      if (two) *(uint4*)(dx + (size_t)pos2 * p.C + c0) = v1;
    }
  }
  if (MODE == POOL_BWD_PLAIN && gs != nullptr && gpart == nullptr && cur_b != 0xffffffffu) {
#pragma unroll
    for (int k = 0; k < 8; ++k) unsafeAtomicAdd(gs + (size_t)cur_b * p.C + c0 + k, sacc[k]);
  }
  if (MODE == POOL_BWD_PLAIN && gs != nullptr && gpart != nullptr) {
    __shared__ uint32_t bfirst;
    if (threadIdx.x == 0) bfirst = 0xffffffffu;
    __syncthreads();
    const uint32_t mine = prev_b != 0xffffffffu ? prev_b : cur_b;
    if (mine != 0xffffffffu) atomicMin(&bfirst, mine);  // integer min: order-independent
    __syncthreads();
    const uint32_t b0 = bfirst;
    const bool some = b0 != 0xffffffffu;
    const bool p0 = some && prev_b == b0, p1 = some && prev_b != 0xffffffffu && prev_b == b0 + 1;
    const bool c0v = some && cur_b == b0, c1v = some && cur_b != 0xffffffffu && cur_b == b0 + 1;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      red[k * 256 + threadIdx.x] = (p0 ? sprev[k] : 0.f) + (c0v ? sacc[k] : 0.f);
      red[(8 + k) * 256 + threadIdx.x] = (p1 ? sprev[k] : 0.f) + (c1v ? sacc[k] : 0.f);
    }
    __syncthreads();
    if (active && rr == 0) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float s0 = 0.f, s1 = 0.f;
        for (int j = 0; j < rpi; ++j) { s0 += red[k * 256 + j * cpr + cc]; s1 += red[(8 + k) * 256 + j * cpr + cc]; }
        gpart[((size_t)blockIdx.x * 2) * p.C + c0 + k] = s0;
        gpart[((size_t)blockIdx.x * 2 + 1) * p.C + c0 + k] = s1;
      }
    }
    if (threadIdx.x == 0) gpart[(size_t)gridDim.x * 2 * p.C + blockIdx.x] = b0 == 0xffffffffu ? -1.f : (float)b0;
    __syncthreads();  // red is reused by the BN partial commit
  }
  if (bn) acc_bn.commit(red, part, p.C, cpr, rpi, cc, rr, active);
}

// gs[b, c] += the pool blocks' partial rows of clip b (slot b - first clip of the block), in block
// order. gpart: [nblk][2][C] rows, then nblk first-clip indices (as float, -1: empty block).
__global__ void pool_gs_sum_kernel(float* __restrict__ gs, const float* __restrict__ gpart, int nblk, int B, int C,
                                   long long ipc, long long ipb) {
  const long long n = (long long)B * C;
  const float* __restrict__ bfirst = gpart + (size_t)nblk * 2 * C;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const long long b = i / C, c = i - b * C;
    const long long lo = b * ipc / ipb, hi = min((long long)nblk - 1, ((b + 1) * ipc - 1) / ipb);
    float v = 0.f;
    for (long long blk = lo; blk <= hi; ++blk) {
      const float f = bfirst[blk];
      if (f < 0.f) continue;
      const long long slot = b - (long long)f;
      if (slot == 0 || slot == 1) v += gpart[((size_t)blk * 2 + slot) * C + c];
    }
    gs[i] += v;
  }
}

// ---------------------------------------------------------------------------------------
// Stride-1 3x3x3 pool (Inception branch 3, -inf padding 1): a thread owns one (b, t, h, chunk)
// row and slides along w, so each input column is loaded once per row (9 loads per output
// instead of 27). Forward keeps per-column maxima over the 3x3 (t, h) taps; the winning tap is
// the first maximum in (t, h, w) scan order, as in ATen.
__device__ __forceinline__ void s1_column_max(const bf16_t* __restrict__ x, const PoolParams& p, size_t clip,
                                              int t, int h, int wcol, int c0, float* v, uint32_t* tp) {
#pragma unroll
  for (int k = 0; k < 8; ++k) { v[k] = -INFINITY; tp[k] = 0; }
  const bool wv = (unsigned)wcol < (unsigned)p.W;
  uint4 r[9];
  bool ok[9];
#pragma unroll
  for (int dt = 0; dt < 3; ++dt)
#pragma unroll
    for (int dh = 0; dh < 3; ++dh) {
      const int ti = t + dt - 1, hi = h + dh - 1;
      ok[dt * 3 + dh] = wv & ((unsigned)ti < (unsigned)p.T) & ((unsigned)hi < (unsigned)p.H);
      const size_t off = ok[dt * 3 + dh] ? clip + ((size_t)(ti * p.H + hi) * p.W + wcol) * p.C + c0 : c0;
      r[dt * 3 + dh] = *(const uint4*)(x + off);
    }
#pragma unroll
  for (int u = 0; u < 9; ++u) {
    float f[8];
    unpack8(r[u], f);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const bool gt = ok[u] & (f[k] > v[k]);
      v[k] = gt ? f[k] : v[k];
      tp[k] = gt ? (uint32_t)u : tp[k];
    }
  }
}

__global__ __launch_bounds__(256) void maxpool_s1_fwd_slide(PoolParams p, PoolDivs d, const bf16_t* __restrict__ x,
                                                            bf16_t* __restrict__ y, uint8_t* __restrict__ arg,
                                                            uint32_t nrows) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nrows * (uint32_t)(p.C >> 3);
       i += gridDim.x * blockDim.x) {
    const uint32_t r = fdiv(i, d.fcpr);
    const int c0 = (int)(i - r * d.fcpr.d) * 8;
    const uint32_t q = fdiv(r, d.fH);
    const int h = (int)(r - q * p.H);
    const uint32_t b = fdiv(q, d.fT);
    const int t = (int)(q - b * p.T);
    const size_t clip = (size_t)b * p.T * p.H * p.W * p.C;
    float v0[8], v1[8], v2[8];
    uint32_t t0[8], t1[8], t2[8];
    s1_column_max(x, p, clip, t, h, -1, c0, v0, t0);
    s1_column_max(x, p, clip, t, h, 0, c0, v1, t1);
    const size_t rowbase = clip + ((size_t)(t * p.H + h) * p.W) * p.C + c0;
    for (int w = 0; w < p.W; ++w) {
      s1_column_max(x, p, clip, t, h, w + 1, c0, v2, t2);
      float best[8];
      uint32_t bt[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        // candidates in dw order; scan-order tap = (dt*3+dh)*3+dw, first maximum wins
        best[k] = v0[k];
        bt[k] = t0[k] * 3;
        const uint32_t c1 = t1[k] * 3 + 1, c2 = t2[k] * 3 + 2;
        if (v1[k] > best[k] || (v1[k] == best[k] && c1 < bt[k])) { best[k] = v1[k]; bt[k] = c1; }
        if (v2[k] > best[k] || (v2[k] == best[k] && c2 < bt[k])) { best[k] = v2[k]; bt[k] = c2; }
      }
      const size_t o = rowbase + (size_t)w * p.C;
      *(uint4*)(y + o) = pack8(best);
      uint2 a;
      a.x = bt[0] | (bt[1] << 8) | (bt[2] << 16) | (bt[3] << 24);
      a.y = bt[4] | (bt[5] << 8) | (bt[6] << 16) | (bt[7] << 24);
      *(uint2*)(arg + o) = a;
#pragma unroll
      for (int k = 0; k < 8; ++k) { v0[k] = v1[k]; t0[k] = t1[k]; v1[k] = v2[k]; t1[k] = t2[k]; }
    }
  }
}

// Backward: walking output columns wo = 0..W-1 of the 3x3 (t, h) neighbourhood, each loaded
// once; an entry whose arg-max tap has (dt, dh) equal to its position relative to this row sends
// its gradient to input column wo - 1 + dw. Input column w is final once column w + 1 is in.
__global__ __launch_bounds__(256) void maxpool_s1_bwd_slide(PoolParams p, PoolDivs d, const bf16_t* __restrict__ dy,
                                                            const uint8_t* __restrict__ arg,
                                                            bf16_t* __restrict__ dx, uint32_t nrows) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nrows * (uint32_t)(p.C >> 3);
       i += gridDim.x * blockDim.x) {
    const uint32_t r = fdiv(i, d.fcpr);
    const int c0 = (int)(i - r * d.fcpr.d) * 8;
    const uint32_t q = fdiv(r, d.fH);
    const int h = (int)(r - q * p.H);
    const uint32_t b = fdiv(q, d.fT);
    const int t = (int)(q - b * p.T);
    const size_t clip = (size_t)b * p.T * p.H * p.W * p.C;
    const size_t rowbase = clip + ((size_t)(t * p.H + h) * p.W) * p.C + c0;
    float am[8], a0[8], ap[8];  // accumulators of input columns wo-1, wo, wo+1
#pragma unroll
    for (int k = 0; k < 8; ++k) { am[k] = 0.f; a0[k] = 0.f; ap[k] = 0.f; }
    for (int wo = 0; wo < p.W; ++wo) {
      uint4 g[9];
      uint2 a[9];
      bool ok[9];
#pragma unroll
      for (int u = 0; u < 9; ++u) {
        const int dt = u / 3, dh = u % 3;  // this row is input (t, h) = (to + dt - 1, ho + dh - 1)
        const int to = t + 1 - dt, ho = h + 1 - dh;
        ok[u] = ((unsigned)to < (unsigned)p.T) & ((unsigned)ho < (unsigned)p.H);
        const size_t off = ok[u] ? clip + ((size_t)(to * p.H + ho) * p.W + wo) * p.C + c0 : c0;
        g[u] = *(const uint4*)(dy + off);
        a[u] = *(const uint2*)(arg + off);
      }
#pragma unroll
      for (int u = 0; u < 9; ++u) {
        float gf[8];
        unpack8(g[u], gf);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const uint32_t ak = ((k < 4 ? a[u].x : a[u].y) >> (8 * (k & 3))) & 0xff;
          const bool m = ok[u] & ((ak / 3) == (uint32_t)u);
          const uint32_t dw = ak % 3;  // gradient goes to input column wo - 1 + dw
          am[k] += (m & (dw == 0)) ? gf[k] : 0.f;
          a0[k] += (m & (dw == 1)) ? gf[k] : 0.f;
          ap[k] += (m & (dw == 2)) ? gf[k] : 0.f;
        }
      }
      if (wo >= 1) *(uint4*)(dx + rowbase + (size_t)(wo - 1) * p.C) = pack8(am);
#pragma unroll
      for (int k = 0; k < 8; ++k) { am[k] = a0[k]; a0[k] = ap[k]; ap[k] = 0.f; }
    }
    *(uint4*)(dx + rowbase + (size_t)(p.W - 1) * p.C) = pack8(am);
  }
}

// ---------------------------------------------------------------------------------------
// Stride-1 3x3x3 pool as three separable 1-D max stages on an LDS plane sweep.
//
//   m1 = max_dw x(w+dw-1),  m2 = max_dh m1(h+dh-1),  y = max_dt m2(t+dt-1)   (-inf padding)
//
// each stage keeping its FIRST maximum. The routing y -> m2 (dt*) -> m1 (dh*) -> x (dw*) picks the
// lexicographically first (dt, dh, dw) among the window's maxima, i.e. exactly ATen's first
// maximum in (t, h, w) scan order, and the three 2-bit stage codes of a grid position share
// one byte: code = dw* of m1 | dh* of m2 << 2 | dt* of y << 4 (all at that position).
// Forward: ~3 compares per element and stage instead of 27; backward: three 1-D 3-candidate
// gathers instead of testing 27 candidate windows per input element.
//
// Layout: one workgroup owns clip b and a chunk of G 8-channel groups over the WHOLE (t, h)
// plane (thread = (row r = t*H + h, group g)) and sweeps along w; the w stage runs in
// registers (sliding window), the h and t stages exchange one column through LDS. Every
// element is fetched from memory once, all memory ops are buffer ops on per-clip descriptors
// with out-of-range offsets for idle lanes (branch-free, so counted vmcnt waits keep the
// prefetches in flight across the LDS-only barriers), and the workgroup owns complete
// (clip, channel) planes, so plane sums need no atomics. Requires T*H*G <= 512.
//
// The arg-max codes of the sweeps are stored in workgroup order (only the sweep backward reads
// them): per clip [chunk][W][T*H][gc][8] bytes (gc = the chunk's channel groups), i.e. a column of
// a workgroup is one contiguous run in thread order and a wave's 8-B code stores / loads cover
// whole 128-B lines. In the activation layout each (row, group) is 8 B of a 128-B line that the
// clip's other workgroups fill at other times: the forward's L2 -> HBM write requests were mostly
// partial lines (tools/gpu/pool_pmc.sh). The layout depends on G, which s1_groups derives from the
// shape alone (and the workgroup-size cap, which must not change between forward and backward).
struct S1Geo {
  int rows, G, nchunk, b, chunk, r, g, t, h;
  bool active;
  uint32_t e0;  // element offset (in the clip) of this thread's column 0, or out of range
  uint32_t a0;   // byte offset (in the clip's codes) of this thread's column-0 code, or out of range
  uint32_t acs;  // code bytes per column of this chunk
};

__device__ __forceinline__ S1Geo s1_geo(const PoolParams& p, int G, int nchunk) {
  S1Geo s;
  s.rows = p.T * p.H;
  s.G = G;
  s.nchunk = nchunk;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);  // the chunks of a clip share cache lines: one L2
  s.b = bid / nchunk;
  s.chunk = bid - s.b * nchunk;
  s.r = threadIdx.x / G;
  s.g = threadIdx.x - s.r * G;
  const int cg = s.chunk * G + s.g;
  s.active = s.r < s.rows && cg < (p.C >> 3);
  s.t = s.r / p.H;
  s.h = s.r - s.t * p.H;
  s.e0 = s.active ? (uint32_t)(s.r * p.W * p.C + cg * 8) : 0x40000000u;
  const int gc = min(G, (p.C >> 3) - s.chunk * G);  // groups of this chunk (the last may be partial)
  if (p.s1_codes) {
    s.a0 = s.active ? (uint32_t)(s.chunk * G * p.W * s.rows * 8 + (s.r * gc + s.g) * 8) : 0x40000000u;
    s.acs = (uint32_t)(s.rows * gc * 8);
  } else {  // activation layout (A/B runs)
    s.a0 = s.e0;
    s.acs = (uint32_t)p.C;
  }
  return s;
}

// Buffer descriptor of a workgroup-uniform range. The operands are passed through readfirstlane:
// the compiler cannot always prove them uniform (then it wraps EVERY buffer access in a
// readfirstlane "waterfall" loop, which also defeats the counted vmcnt waits of the sweeps).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t clip_rsrc(const void* base, int nbytes) {
  const unsigned long long a = (unsigned long long)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  void* ub = (void*)(((unsigned long long)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(ub, (short)0, __builtin_amdgcn_readfirstlane(nbytes), 0x00020000);
}

__device__ __forceinline__ uint4 bld16(__amdgpu_buffer_rsrc_t rs, uint32_t byte_off) {
  return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, byte_off, 0, 0));
}
__device__ __forceinline__ uint2 bld8(__amdgpu_buffer_rsrc_t rs, uint32_t byte_off) {
  return __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rs, byte_off, 0, 0));
}
__device__ __forceinline__ void bst16(__amdgpu_buffer_rsrc_t rs, uint32_t byte_off, uint4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v), rs,
                                         byte_off, 0, 0);
}
__device__ __forceinline__ void bst8(__amdgpu_buffer_rsrc_t rs, uint32_t byte_off, uint2 v) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, v), rs,
                                        byte_off, 0, 0);
}

// first maximum over three candidates (invalid ones skipped), per channel: value and code 0..2
__device__ __forceinline__ void max3(const float* a, bool va, const float* b, bool vb, const float* c, bool vc,
                                     float* out, uint32_t* code) {
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    float m = va ? a[k] : -INFINITY;
    uint32_t cd = 0;
    if (vb && b[k] > m) { m = b[k]; cd = 1; }
    if (vc && c[k] > m) { m = c[k]; cd = 2; }
    out[k] = m;
    code[k] = cd;
  }
}

constexpr int S1_PF = 8;  // forward sweep: register ring of input columns (6 loads in flight)

// WT = W when specialised (the sweep is then fully unrolled), 0 = runtime W. (Two output columns
// per step, sharing the h / t stages' barriers, ran 5-40 % slower: tools/pool_bench.py, r4.)
template <int WT>
__global__ __launch_bounds__(512) void maxpool_s1_fwd_sep(PoolParams p, int G, int nchunk, const bf16_t* __restrict__ x,
                                                          bf16_t* __restrict__ y, uint8_t* __restrict__ arg) {
  extern __shared__ uint4 s1_lds[];  // m1 [rows+1][G], m2 [rows+1][G] (bf16 x 8); row `rows`: idle lanes
  const S1Geo s = s1_geo(p, G, nchunk);
  uint4* m1s = s1_lds;
  uint4* m2s = s1_lds + (s.rows + 1) * G;
  const size_t clip = (size_t)s.b * s.rows * p.W * p.C;
  const int nbytes = s.rows * p.W * p.C * 2;
  const auto xr = clip_rsrc(x + clip, nbytes);
  const auto yr = clip_rsrc(y + clip, nbytes);
  const auto ar = clip_rsrc(arg + clip, nbytes / 2);
  const uint32_t oob = 0x40000000u, ecol = (uint32_t)p.C;
  const int me = (s.active ? s.r : s.rows) * G + s.g;  // idle lanes own a dummy row
  // neighbour slots (clamped for idle lanes / edges; validity flags decide)
  const bool vhm = s.active && s.h > 0, vhp = s.active && s.h + 1 < p.H;
  const bool vtm = s.active && s.t > 0, vtp = s.active && s.t + 1 < p.T;
  const int ihm = vhm ? me - G : me, ihp = vhp ? me + G : me;
  const int itm = vtm ? me - p.H * G : me, itp = vtp ? me + p.H * G : me;
  auto col = [&](int w) { return (w >= 0 && w < p.W) ? (s.e0 + (uint32_t)w * ecol) : oob; };
  auto acol = [&](int w) { return (w >= 0 && w < p.W) ? (s.a0 + (uint32_t)w * s.acs) : oob; };
  // register ring of input columns, slot = column % S1_PF (column -1 reads as zeros): the loop is
  // unrolled by the ring size so a pending load is never copied between registers (a copy would
  // make the compiler wait for it), i.e. S1_PF - 2 columns stay in flight across the barriers
  uint4 ring[S1_PF];
  ring[S1_PF - 1] = make_uint4(0, 0, 0, 0);
#pragma unroll
  for (int k = 0; k < S1_PF - 1; ++k) ring[k] = bld16(xr, col(k) * 2);
  const int W = WT > 0 ? WT : p.W;
#pragma unroll
  for (int w0 = 0; w0 < W; w0 += S1_PF) {
#pragma unroll
    for (int u = 0; u < S1_PF; ++u) {
      const int w = w0 + u;
      if (w >= W) break;
      const int sp = (u + S1_PF - 1) % S1_PF, sc = u, sn = (u + 1) % S1_PF;
      float fa[8], fb[8], fc[8], m1[8], m2[8], o[8];
      uint32_t cw[8], ch[8], ct[8];
      unpack8(ring[sp], fa);
      unpack8(ring[sc], fb);
      unpack8(ring[sn], fc);
      ring[sp] = bld16(xr, col(w - 1 + S1_PF) * 2);  // column w-1's slot takes column w-1+S1_PF
      max3(fa, w > 0, fb, true, fc, w + 1 < W, m1, cw);
      m1s[me] = pack8(m1);  // exact: maxima of bf16 values
      lds_barrier();
      unpack8(m1s[ihm], fa);
      unpack8(m1s[ihp], fc);
      max3(fa, vhm, m1, true, fc, vhp, m2, ch);
      m2s[me] = pack8(m2);
      lds_barrier();
      unpack8(m2s[itm], fa);
      unpack8(m2s[itp], fc);
      max3(fa, vtm, m2, true, fc, vtp, o, ct);
      bst16(yr, col(s.active ? w : -1) * 2, pack8(o));
      uint32_t cb[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) cb[k] = cw[k] | (ch[k] << 2) | (ct[k] << 4);
      uint2 a;
      a.x = cb[0] | (cb[1] << 8) | (cb[2] << 16) | (cb[3] << 24);
      a.y = cb[4] | (cb[5] << 8) | (cb[6] << 16) | (cb[7] << 24);
      bst8(ar, acol(w), a);
    }
  }
}

// Backward of the separable sweep, output column wo per step:
//   t stage  dm2(r) = sum_dt [ct(r_o) == dt] dy(r_o),  r_o = r - (dt-1)*H   (LDS exchange of dy, codes)
//   h stage  dm1(r) = sum_dh [ch(r_o) == dh] dm2(r_o), r_o = r - (dh-1)     (LDS exchange of dm2, fp32)
//   w stage  dx(w)  = sum_dw [cw(w_o) == dw] dm1(w_o), w_o = w - dw + 1     (registers, 3 columns)
// dx column wo-1 is final at step wo. Fused epilogue (both optional, 0-record descriptors
// otherwise): acc_in  dx += acc_in (the other gradient of the pool input: the Inception 1x1
// GEMM's dX); x, gs  gs[b, c] = sum_thw dx * x (the SelfGating reduction of the block that
// produced x, from the final bf16 dx), written directly (the workgroup owns the plane).
template <int WT>
__global__ __launch_bounds__(512) void maxpool_s1_bwd_sep(PoolParams p, int G, int nchunk,
                                                          const bf16_t* __restrict__ dy,
                                                          const uint8_t* __restrict__ arg,
                                                          const bf16_t* __restrict__ acc_in,
                                                          const bf16_t* __restrict__ x, float* __restrict__ gs,
                                                          bf16_t* __restrict__ dx) {
  extern __shared__ uint4 s1_lds[];  // dy [2][rows+1][G] bf16x8 | dm2 [rows+1][G] f32x8 | codes [2][rows+1][G]
  const S1Geo s = s1_geo(p, G, nchunk);
  const int n = (s.rows + 1) * G;
  uint4* dys = s1_lds;                   // 2 * n
  // fp32 m2 as two planes of float4 (channels 0-3 | 4-7): 16-B lane stride, bank-conflict free
  // (one 32-B slot per lane halved the LDS rate: SQ_LDS_BANK_CONFLICT / IDX_ACTIVE was 0.5)
  float4* m2lo = (float4*)(s1_lds + 2 * n);  // n float4
  float4* m2hi = m2lo + n;                   // n float4
  uint2* cds = (uint2*)(s1_lds + 4 * n);    // 2 * n
  const size_t clip = (size_t)s.b * s.rows * p.W * p.C;
  const int nbytes = s.rows * p.W * p.C * 2;
  const auto dyr = clip_rsrc(dy + clip, nbytes);
  const auto agr = clip_rsrc(arg + clip, nbytes / 2);
  const auto inr = clip_rsrc(acc_in != nullptr ? acc_in + clip : dy + clip, acc_in != nullptr ? nbytes : 0);
  const auto xr = clip_rsrc(x != nullptr ? x + clip : dy + clip, gs != nullptr ? nbytes : 0);
  const auto dxr = clip_rsrc(dx + clip, nbytes);
  const uint32_t oob = 0x40000000u, ecol = (uint32_t)p.C;
  const int me = (s.active ? s.r : s.rows) * G + s.g;  // idle lanes own a dummy row
  const bool vhm = s.active && s.h > 0, vhp = s.active && s.h + 1 < p.H;
  const bool vtm = s.active && s.t > 0, vtp = s.active && s.t + 1 < p.T;
  const int ihm = vhm ? me - G : me, ihp = vhp ? me + G : me;
  const int itm = vtm ? me - p.H * G : me, itp = vtp ? me + p.H * G : me;
  auto col = [&](int w) { return (w >= 0 && w < p.W) ? (s.e0 + (uint32_t)w * ecol) : oob; };
  auto acol = [&](int w) { return (w >= 0 && w < p.W) ? (s.a0 + (uint32_t)w * s.acs) : oob; };
  auto code = [](const uint2& a, int k, int sh) {
    return ((((k < 4 ? a.x : a.y) >> (8 * (k & 3))) >> sh) & 3u);
  };
  const int W = WT > 0 ? WT : p.W;
  float sacc[8], dA[8], dB[8];  // dm1 of columns wo-2 (A), wo-1 (B)
  uint2 cA = make_uint2(0, 0), cB = make_uint2(0, 0);
#pragma unroll
  for (int k = 0; k < 8; ++k) { sacc[k] = 0.f; dA[k] = 0.f; dB[k] = 0.f; }
  uint4 gcur = bld16(dyr, col(0) * 2);
  uint2 acur = bld8(agr, acol(0));
  for (int wo = 0; wo <= W; ++wo) {
    // emit operands of column wo-1 first, then the next column's gradient and codes
    const uint32_t ep = col(wo - 1);
    const uint4 ein = bld16(inr, ep * 2), xin = bld16(xr, ep * 2);
    const uint4 gnext = bld16(dyr, col(wo + 1) * 2);
    const uint2 anext = bld8(agr, acol(wo + 1));
    float dC[8];  // dm1 of column wo
    uint2 cC = acur;
    if (wo < W) {
      const int buf = (wo & 1) * n;
      dys[buf + me] = gcur;
      cds[buf + me] = acur;
      lds_barrier();
      // t stage: candidates are the outputs at t+1 (dt=0), t (dt=1), t-1 (dt=2)
      float g0[8], g1[8], g2[8], m2[8];
      const uint2 c0 = cds[buf + itp], c2 = cds[buf + itm];
      unpack8(dys[buf + itp], g0);
      unpack8(gcur, g1);
      unpack8(dys[buf + itm], g2);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float v = code(acur, k, 4) == 1u ? g1[k] : 0.f;
        v += (vtp && code(c0, k, 4) == 0u) ? g0[k] : 0.f;
        v += (vtm && code(c2, k, 4) == 2u) ? g2[k] : 0.f;
        m2[k] = v;
      }
      m2lo[me] = make_float4(m2[0], m2[1], m2[2], m2[3]);
      m2hi[me] = make_float4(m2[4], m2[5], m2[6], m2[7]);
      lds_barrier();
      // h stage: candidates are the m2 cells at h+1 (dh=0), h (dh=1), h-1 (dh=2)
      const uint2 h0 = cds[buf + ihp], h2 = cds[buf + ihm];
      const float4 p0a = m2lo[ihp], p0b = m2hi[ihp], p2a = m2lo[ihm], p2b = m2hi[ihm];
      const float q0[8] = {p0a.x, p0a.y, p0a.z, p0a.w, p0b.x, p0b.y, p0b.z, p0b.w};
      const float q2[8] = {p2a.x, p2a.y, p2a.z, p2a.w, p2b.x, p2b.y, p2b.z, p2b.w};
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float v = code(acur, k, 2) == 1u ? m2[k] : 0.f;
        v += (vhp && code(h0, k, 2) == 0u) ? q0[k] : 0.f;
        v += (vhm && code(h2, k, 2) == 2u) ? q2[k] : 0.f;
        dC[k] = v;
      }
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) dC[k] = 0.f;
      cC = make_uint2(0, 0);
    }
    if (wo >= 1) {
      // w stage for input column wo-1: dm1 cells at wo (dw=0), wo-1 (dw=1), wo-2 (dw=2)
      float d[8], e[8], q[8], xv[8];
      unpack8(ein, e);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float v = e[k];
        v += code(cC, k, 0) == 0u ? dC[k] : 0.f;
        v += code(cB, k, 0) == 1u ? dB[k] : 0.f;
        v += code(cA, k, 0) == 2u ? dA[k] : 0.f;
        d[k] = v;
      }
      const uint4 vout = pack8(d);
      bst16(dxr, ep * 2, vout);
      unpack8(vout, q);
      unpack8(xin, xv);
#pragma unroll
      for (int k = 0; k < 8; ++k) sacc[k] += q[k] * xv[k];
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) { dA[k] = dB[k]; dB[k] = dC[k]; }
    cA = cB;
    cB = cC;
    gcur = gnext;
    acur = anext;
  }
  if (gs == nullptr) return;
  // the gate reduction over the plane's rows: a fixed-order LDS tree (LDS float atomics summed the
  // rows in arrival order, so the sums differed from run to run)
  __syncthreads();
  float* red = (float*)s1_lds;  // [rows][G][8] (fits: the sweep staged more than this per row)
  if (s.r < s.rows) {
#pragma unroll
    for (int k = 0; k < 8; ++k) red[(s.r * G + s.g) * 8 + k] = s.active ? sacc[k] : 0.f;
  }
  __syncthreads();
  int half = 1;
  while (half < s.rows) half <<= 1;
  for (half >>= 1; half >= 1; half >>= 1) {
    if (s.r < half && s.r + half < s.rows) {
#pragma unroll
      for (int k = 0; k < 8; ++k) red[(s.r * G + s.g) * 8 + k] += red[((s.r + half) * G + s.g) * 8 + k];
    }
    __syncthreads();
  }
  for (int i = threadIdx.x; i < G * 8; i += blockDim.x) {
    const int c = s.chunk * G * 8 + i;
    if (c < p.C) gs[(size_t)s.b * p.C + c] = red[i];
  }
}

// =========================================================================================
// Row sweeps (stride-1 impl 2, the default). A workgroup owns one clip and a chunk of G 8-channel
// groups over ALL T x W positions of the plane and sweeps the H rows. An item is (position, group):
// one 16-B lane access, and the G lanes of a position read G*16 contiguous bytes, so a wave-load
// covers whole 128-B lines (G = 8) where the plane sweeps above read 32-B row pieces. Every input
// element is read exactly once: the sweep carries the h neighbours, the tile holds the t / w ones.
// Separable max in the order w (LDS exchange), t (LDS exchange), h (register ring over the
// sweep); the h stage breaks value ties by the candidates' absolute frame, then by row, so the
// arg-max is the first maximum in (t, h, w) order like the reference pool (s3dg.py:20-21,
// nn.MaxPool3d). Codes per element: cw | ct << 2 | ch << 4 of the element's own cells, stored per
// (clip, chunk, row) as one contiguous run of n_it * 8 bytes (s1_rows_coff).
// =========================================================================================
struct RowItem {
  uint32_t eoff;  // byte offset of row 0 of this item in the clip (out of range when inactive)
  int i, t, w;
  bool act;
};

__device__ __forceinline__ RowItem row_item(const PoolParams& p, int G, int chunk, int i, int n_it) {
  RowItem r;
  r.i = i;
  r.act = i < n_it;
  const int pos = r.act ? i / G : 0, g = r.act ? i - pos * G : 0;
  r.t = pos / p.W;
  r.w = pos - r.t * p.W;
  r.eoff = r.act ? (uint32_t)(((r.t * p.H * p.W + r.w) * p.C + (chunk * G + g) * 8) * 2) : 0x40000000u;
  return r;
}

// code byte field `sh` (0: cw, 2: ct, 4: ch) of channel k from a lane's 8 code bytes
__device__ __forceinline__ uint32_t rcode(const uint2& a, int k, int sh) {
  return (((k < 4 ? a.x : a.y) >> (8 * (k & 3) + sh)) & 3u);
}

template <int N>
using ic = std::integral_constant<int, N>;

// max3 without control flow (bitwise boolean ops: a short-circuit && / || on per-lane values
// compiles to exec-mask branches)
__device__ __forceinline__ void max3s(const float* a, bool va, const float* b, const float* c, bool vc, float* out,
                                      uint32_t* code) {
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const bool gb = !va | (b[k] > a[k]);
    float m = gb ? b[k] : a[k];
    uint32_t cd = gb ? 1u : 0u;
    const bool gc = vc & (c[k] > m);
    out[k] = gc ? c[k] : m;
    code[k] = gc ? 2u : cd;
  }
}

// D = rows whose loads are in flight ahead of the row being processed (a register ring, the
// sweep unrolled by D so no pending load is ever copied between registers): one row in flight
// per wave measured 2.5-3.3 TB/s, latency-bound.
template <int D>
__global__ __launch_bounds__(1024) void maxpool_s1_fwd_rows(PoolParams p, int G, int nchunk,
                                                            const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                            uint8_t* __restrict__ arg) {
  extern __shared__ uint4 rows_lds[];
  const int n_it = p.T * p.W * G, WG = p.W * G;
  uint4* xs = rows_lds;              // [n_it + 1] the current input row (slot n_it: idle lanes)
  uint4* m1s = rows_lds + n_it + 1;  // [n_it + 1] its w maxima
  const int blk = xcd_remap(blockIdx.x, gridDim.x);  // a clip's chunks share lines when G*16 % 128 != 0
  const int b = blk / nchunk, chunk = blk - b * nchunk;
  const int nbytes = p.T * p.H * p.W * p.C * 2;
  const size_t clip = (size_t)b * p.T * p.H * p.W * p.C;
  const auto xr = clip_rsrc(x + clip, nbytes);
  const auto yr = clip_rsrc(y + clip, nbytes);
  const int cbytes = p.H * n_it * 8;
  const auto ar = clip_rsrc(arg + (size_t)blk * cbytes, cbytes);
  const uint32_t rowb = (uint32_t)(p.W * p.C * 2), oob = 0x40000000u;
  const RowItem it = row_item(p, G, chunk, threadIdx.x, n_it);
  const int H = p.H;
  // branch-free: idle lanes work on a dummy slot with no neighbours; their stores go out of range
  const int i = it.act ? it.i : n_it;
  const bool wm = it.act && it.w > 0, wp = it.act && it.w + 1 < p.W;
  const bool tm = it.act && it.t > 0, tp = it.act && it.t + 1 < p.T;
  const int iwm = wm ? i - G : i, iwp = wp ? i + G : i, itm = tm ? i - WG : i, itp = tp ? i + WG : i;
  const uint32_t cbase = it.act ? (uint32_t)(i * 8) : oob, crow = (uint32_t)(n_it * 8);
  auto xo = [&](int h) { return h < H ? it.eoff + (uint32_t)h * rowb : oob; };
  uint4 ring[D];
#pragma unroll
  for (int d = 0; d < D; ++d) ring[d] = bld16(xr, xo(d));
  // rows h-2 (A), h-1 (B), h (C): t-stage maxima and the cells' own codes (4 bits per channel:
  // cw | ct << 2)
  uint4 mA = make_uint4(0, 0, 0, 0), mB = mA;
  uint32_t cA = 0, cB = 0;
  auto step = [&](auto slot_c, int h) {
    constexpr int slot = decltype(slot_c)::value;
    uint4 mC = make_uint4(0, 0, 0, 0);
    uint32_t cC = 0;
    if (h < H) {  // (uniform)
      const uint4 xc = ring[slot];
      xs[i] = xc;
      ring[slot] = bld16(xr, xo(h + D));
      lds_barrier();
      uint32_t cw = 0;
      uint4 m1;
      {
        float a[8], bb[8], c[8], m[8];
        uint32_t cd[8];
        unpack8(xs[iwm], a);
        unpack8(xc, bb);
        unpack8(xs[iwp], c);
        max3s(a, wm, bb, c, wp, m, cd);
        m1 = pack8(m);  // exact: maxima of bf16 values
        m1s[i] = m1;
#pragma unroll
        for (int j = 0; j < 8; ++j) cw |= cd[j] << (4 * j);
      }
      lds_barrier();
      {
        float a[8], bb[8], c[8], m[8];
        uint32_t cd[8];
        unpack8(m1s[itm], a);
        unpack8(m1, bb);
        unpack8(m1s[itp], c);
        max3s(a, tm, bb, c, tp, m, cd);
        mC = pack8(m);
        cC = cw;
#pragma unroll
        for (int j = 0; j < 8; ++j) cC |= cd[j] << (4 * j + 2);
      }
    }
    if (h >= 1) {  // output row h-1 from rows h-2 (dh 0), h-1 (dh 1), h (dh 2)
      const bool va = h >= 2, vc = h < H;
      float fa[8], fb[8], fc[8], o[8];
      unpack8(mA, fa);
      unpack8(mB, fb);
      unpack8(mC, fc);
      uint32_t lo = 0, hi = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        // candidates in row order; a later one wins on a larger value or an earlier frame (the
        // frames compare by their t codes: the three cells share the output's t)
        const uint32_t ta = (cA >> (4 * j + 2)) & 3u, tb = (cB >> (4 * j + 2)) & 3u, tc = (cC >> (4 * j + 2)) & 3u;
        const bool pa = va & ((fa[j] > fb[j]) | ((fa[j] == fb[j]) & (ta <= tb)));
        float m = pa ? fa[j] : fb[j];
        const uint32_t tm2 = pa ? ta : tb;
        const bool pc = vc & ((fc[j] > m) | ((fc[j] == m) & (tc < tm2)));
        o[j] = pc ? fc[j] : m;
        const uint32_t ch = pc ? 2u : (pa ? 0u : 1u);
        const uint32_t byte = ((cB >> (4 * j)) & 0xFu) | (ch << 4);
        if (j < 4) lo |= byte << (8 * j);
        else hi |= byte << (8 * (j - 4));
      }
      bst16(yr, xo(h - 1), pack8(o));
      bst8(ar, cbase + (uint32_t)(h - 1) * crow, make_uint2(lo, hi));
    }
    mA = mB;
    cA = cB;
    mB = mC;
    cB = cC;
  };
  for (int h0 = 0; h0 <= H; h0 += D) {
    step(ic<0>{}, h0);
    if constexpr (D > 1) { if (h0 + 1 <= H) step(ic<1 % D>{}, h0 + 1); }
    if constexpr (D > 2) { if (h0 + 2 <= H) step(ic<2 % D>{}, h0 + 2); }
    if constexpr (D > 3) { if (h0 + 3 <= H) step(ic<3 % D>{}, h0 + 3); }
  }
}

// Backward, input row h' per step (the forward's stages in reverse):
//   h  dmt(h') = [ch(h'+1) == 0] dy(h'+1) + [ch(h') == 1] dy(h') + [ch(h'-1) == 2] dy(h'-1)   (registers)
//   t  dm1(t') = sum_dt [ct(t'-dt+1) == dt] dmt(t'-dt+1)                                     (LDS exchange)
//   w  dx(w')  = sum_dw [cw(w'-dw+1) == dw] dm1(w'-dw+1)                                     (LDS exchange)
// fp32 sums, dx rounded once. Fused epilogue as maxpool_s1_bwd_sep: dx += acc_in (the Inception
// head GEMM's dX), gs[b, c] = sum_thw dx * x in a fixed-order workgroup reduction.
// Register rings: dy / codes of rows h'-1 .. h'+1+D (U = D + 2 slots, row r in slot r % U), the
// epilogue operands of rows h' .. h'+D-1 (row r in slot r % D); the sweep is unrolled by U (a
// multiple of D for D = 1, 2).
template <int D>
__global__ __launch_bounds__(1024) void maxpool_s1_bwd_rows(PoolParams p, int G, int nchunk,
                                                            const bf16_t* __restrict__ dy,
                                                            const uint8_t* __restrict__ arg,
                                                            const bf16_t* __restrict__ acc_in,
                                                            const bf16_t* __restrict__ x, float* __restrict__ gs,
                                                            bf16_t* __restrict__ dx) {
  static_assert(D == 1 || D == 2, "unroll U = D + 2 must be a multiple of D");
  constexpr int U = D + 2;
  extern __shared__ uint4 rows_lds[];
  const int n_it = p.T * p.W * G, WG = p.W * G;
  const int na = max(n_it, (int)blockDim.x);  // exchange-area slots (>= threads: the gs reduction)
  float4* tlo = (float4*)rows_lds;  // t-exchange: dmt channels 0-3 | 4-7, the cells' codes
  float4* thi = tlo + na;
  uint2* tcd = (uint2*)(thi + na);
  float4* wlo = (float4*)(tcd + na);  // w-exchange: dm1, codes (a second area: no WAR barrier)
  float4* whi = wlo + na;
  uint2* wcd = (uint2*)(whi + na);
  const int blk = xcd_remap(blockIdx.x, gridDim.x);
  const int b = blk / nchunk, chunk = blk - b * nchunk;
  const int nbytes = p.T * p.H * p.W * p.C * 2;
  const size_t clip = (size_t)b * p.T * p.H * p.W * p.C;
  const auto dyr = clip_rsrc(dy + clip, nbytes);
  const int cbytes = p.H * n_it * 8;
  const auto agr = clip_rsrc(arg + (size_t)blk * cbytes, cbytes);
  const auto inr = clip_rsrc(acc_in != nullptr ? acc_in + clip : dy + clip, acc_in != nullptr ? nbytes : 0);
  const auto xr = clip_rsrc(x != nullptr ? x + clip : dy + clip, gs != nullptr ? nbytes : 0);
  const auto dxr = clip_rsrc(dx + clip, nbytes);
  const uint32_t rowb = (uint32_t)(p.W * p.C * 2), oob = 0x40000000u;
  const RowItem it = row_item(p, G, chunk, threadIdx.x, n_it);
  const int i = it.i, H = p.H;
  auto eo = [&](int h) { return (h >= 0 && h < H) ? it.eoff + (uint32_t)h * rowb : oob; };
  auto co = [&](int h) { return (h >= 0 && h < H && it.act) ? (uint32_t)((h * n_it + i) * 8) : oob; };
  uint4 g[U], e[D], xv[D];
  uint2 c[U];
  // row r in slot r % U; slot U-1 holds row -1 (zeros, invalid)
  g[U - 1] = make_uint4(0, 0, 0, 0);
  c[U - 1] = make_uint2(0, 0);
#pragma unroll
  for (int r = 0; r <= D; ++r) {
    g[r] = bld16(dyr, eo(r));
    c[r] = bld8(agr, co(r));
  }
#pragma unroll
  for (int r = 0; r < D; ++r) {
    e[r] = bld16(inr, eo(r));
    xv[r] = bld16(xr, eo(r));
  }
  float sacc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) sacc[j] = 0.f;
  const bool wm = it.w > 0, wp = it.w + 1 < p.W, tm = it.t > 0, tp = it.t + 1 < p.T;
  auto step = [&](auto sl_c, int h) {
    constexpr int s = decltype(sl_c)::value;                       // h % U
    constexpr int sa = (s + U - 1) % U, sc = (s + 1) % U, se = s % D;  // rows h-1, h+1; epilogue slot
    const bool va = h >= 1, vc = h + 1 < H;
    {
      float ga[8], gb[8], gc[8], d1[8];
      unpack8(g[sa], ga);
      unpack8(g[s], gb);
      unpack8(g[sc], gc);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float v = (vc && rcode(c[sc], j, 4) == 0u) ? gc[j] : 0.f;
        v += rcode(c[s], j, 4) == 1u ? gb[j] : 0.f;
        v += (va && rcode(c[sa], j, 4) == 2u) ? ga[j] : 0.f;
        d1[j] = v;
      }
      if (it.act) {
        tlo[i] = make_float4(d1[0], d1[1], d1[2], d1[3]);
        thi[i] = make_float4(d1[4], d1[5], d1[6], d1[7]);
        tcd[i] = c[s];
      }
    }
    // row h-1 is used up: its slot takes row h+D+1
    g[sa] = bld16(dyr, eo(h + D + 1));
    c[sa] = bld8(agr, co(h + D + 1));
    lds_barrier();
    if (it.act) {  // (a cell's own partial sums are re-read here, not held across the barriers)
      const int im = tm ? i - WG : i, ip = tp ? i + WG : i;
      const uint2 c0 = tcd[ip], c2 = tcd[im];
      const float4 p0a = tlo[ip], p0b = thi[ip], p2a = tlo[im], p2b = thi[im], p1a = tlo[i], p1b = thi[i];
      const float q0[8] = {p0a.x, p0a.y, p0a.z, p0a.w, p0b.x, p0b.y, p0b.z, p0b.w};
      const float q1[8] = {p1a.x, p1a.y, p1a.z, p1a.w, p1b.x, p1b.y, p1b.z, p1b.w};
      const float q2[8] = {p2a.x, p2a.y, p2a.z, p2a.w, p2b.x, p2b.y, p2b.z, p2b.w};
      float d1[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float v = (tp && rcode(c0, j, 2) == 0u) ? q0[j] : 0.f;
        v += rcode(c[s], j, 2) == 1u ? q1[j] : 0.f;
        v += (tm && rcode(c2, j, 2) == 2u) ? q2[j] : 0.f;
        d1[j] = v;
      }
      wlo[i] = make_float4(d1[0], d1[1], d1[2], d1[3]);
      whi[i] = make_float4(d1[4], d1[5], d1[6], d1[7]);
      wcd[i] = c[s];
    }
    lds_barrier();
    if (it.act) {
      const int im = wm ? i - G : i, ip = wp ? i + G : i;
      const uint2 c0 = wcd[ip], c2 = wcd[im];
      const float4 p0a = wlo[ip], p0b = whi[ip], p2a = wlo[im], p2b = whi[im], p1a = wlo[i], p1b = whi[i];
      const float q0[8] = {p0a.x, p0a.y, p0a.z, p0a.w, p0b.x, p0b.y, p0b.z, p0b.w};
      const float q1[8] = {p1a.x, p1a.y, p1a.z, p1a.w, p1b.x, p1b.y, p1b.z, p1b.w};
      const float q2[8] = {p2a.x, p2a.y, p2a.z, p2a.w, p2b.x, p2b.y, p2b.z, p2b.w};
      float ev[8], d[8], q[8], xf[8];
      unpack8(e[se], ev);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float v = ev[j];
        v += (wp && rcode(c0, j, 0) == 0u) ? q0[j] : 0.f;
        v += rcode(c[s], j, 0) == 1u ? q1[j] : 0.f;
        v += (wm && rcode(c2, j, 0) == 2u) ? q2[j] : 0.f;
        d[j] = v;
      }
      const uint4 vout = pack8(d);
      bst16(dxr, eo(h), vout);
      unpack8(vout, q);
      unpack8(xv[se], xf);
#pragma unroll
      for (int j = 0; j < 8; ++j) sacc[j] = fmaf(q[j], xf[j], sacc[j]);
    }
    e[se] = bld16(inr, eo(h + D));
    xv[se] = bld16(xr, eo(h + D));
  };
  for (int h0 = 0; h0 < H; h0 += U) {
    step(ic<0>{}, h0);
    if (h0 + 1 < H) step(ic<1>{}, h0 + 1);
    if (h0 + 2 < H) step(ic<2>{}, h0 + 2);
    if constexpr (U > 3) { if (h0 + 3 < H) step(ic<3 % U>{}, h0 + 3); }
  }
  if (gs == nullptr) return;
  // gs over the plane's positions per (group, channel): per-thread sums -> LDS, then a fixed-order
  // two-level reduction (P strided partial sums per output, summed in order). Thread r's sums
  // belong to group r % G.
  __syncthreads();
  float* red = (float*)rows_lds;  // [nthr][8] (the t-exchange area holds 40 B per slot)
#pragma unroll
  for (int j = 0; j < 8; ++j) red[threadIdx.x * 8 + j] = sacc[j];
  __syncthreads();
  const int nthr = blockDim.x, nout = G * 8, rows = (nthr + G - 1) / G;
  const int P = max(1, min(nthr / nout, rows));
  float* part = (float*)wlo;  // [P][nout] (the w-exchange area)
  const int o = threadIdx.x % nout, q = threadIdx.x / nout;
  if (q < P) {
    float s = 0.f;
    for (int r = q; r < rows; r += P) {
      const int src = r * G + o / 8;
      if (src < nthr) s += red[src * 8 + (o & 7)];
    }
    part[q * nout + o] = s;
  }
  __syncthreads();
  if (threadIdx.x < nout) {
    float s = 0.f;
    for (int r = 0; r < P; ++r) s += part[r * nout + threadIdx.x];
    gs[(size_t)b * p.C + chunk * nout + threadIdx.x] = s;
  }
}


// G (8-channel groups per workgroup) for the plane sweeps: as many as fit `maxthr` threads
// (all rows of the plane are always in one workgroup), at least 1.
static int s1_groups(int rows, int C, int maxthr = 256, long long B = 0) {
  const int cpr = C / 8;
  int G = rows >= maxthr ? 1 : maxthr / rows;
  if (G > cpr) G = cpr;
  // keep >= 4 workgroups per CU (1024) when the batch allows: small planes (the 2x7x7 blocks)
  // otherwise get too few, too long-lived workgroups
  if (B > 0) {
    const long long want_chunks = (1024 + B - 1) / B;
    const int gmax = (int)((cpr + want_chunks - 1) / want_chunks);
    if (G > gmax) G = gmax < 1 ? 1 : gmax;
  }
  // prefer a divisor of cpr (no idle lanes in the last chunk) if it keeps >= 3/4 of G
  for (int d = G; d >= 1 && 4 * d >= 3 * G; --d)
    if (cpr % d == 0) return d;
  return G;
}

// LDS bytes of the separable sweeps: fwd m1 + m2 columns (16 B per slot each); bwd dy and
// codes double-buffered plus the fp32 m2 column (2*16 + 2*8 + 32 = 80 B per slot).
static size_t s1_fwd_lds(int rows, int G) { return (size_t)(rows + 1) * G * 32; }
static size_t s1_bwd_lds(int rows, int G) { return (size_t)(rows + 1) * G * 80; }

// Stride-1 pool implementation: 1 = LDS plane sweeps (default), 0 = global-memory sliding
// kernels (A/B benchmarks only; milnce_set_pool_s1_impl). A tiled forward (band + halo rows in
// LDS, one barrier, all loads in flight) measured 1.6-2.4 TB/s against the sweep's 2.6-3.4: its
// h stage is recomputed per t and the VALU work, not memory, bound it (tools/ew_bench.py).
// 2 = row sweeps (MILNCE_S1_IMPL=2; a shape they cannot tile takes the plane sweeps). The plane
// sweeps stay the default: the row sweeps' backward is 9 % faster at the flagship shapes but their
// forward 23 % slower (tools/pool_bench.py, profiles/r6_pool_rows.md), net +0.1 ms per step.
static int g_s1_impl = -1;
static int s1_impl() {
  if (g_s1_impl < 0) {
    const char* e = getenv("MILNCE_S1_IMPL");
    g_s1_impl = e ? atoi(e) : 1;
  }
  return g_s1_impl;
}
static bool is_s1_333(const PoolParams& p);
#define HIP_RET_E(expr)                   \
  do {                                    \
    hipError_t _e = (expr);               \
    if (_e != hipSuccess) return _e;      \
  } while (0)
static int g_s1_maxthr = 512;  // workgroup size cap of the plane sweeps (G = cap / rows groups)
MILNCE_API int milnce_set_pool_s1_maxthr(int n) {
  const int old = g_s1_maxthr;
  if (n >= 64 && n <= 1024) g_s1_maxthr = n;
  return old;
}

// Row sweeps: G = the largest divisor of C/8 up to MILNCE_S1_G (default 4: the flagship 25x25
// planes then take 800-item tiles, one item per thread, two workgroups per CU) that keeps the
// tile at <= 1024 items. A divisor, so the per-(clip, chunk) code runs tile the arg buffer
// exactly. Depends on the shape only: the forward and the backward must agree. Prefetch depths
// MILNCE_S1_DF (forward rows in flight, 1-4, default 3) / MILNCE_S1_DB (backward, 1-2, default 2).
static int env_int(const char* name, int def, int lo, int hi) {
  const char* e = getenv(name);
  int v = e ? atoi(e) : def;
  return (v < lo || v > hi) ? def : v;
}
static int s1_rows_gmax() {
  static int g = -1;
  if (g < 0) g = env_int("MILNCE_S1_G", 4, 1, 8);
  return g;
}
static int s1_rows_G(const PoolParams& p) {
  const int cpr = p.C / 8;
  for (int g = std::min(s1_rows_gmax(), cpr); g >= 1; --g)
    if (cpr % g == 0 && p.T * p.W * g <= 1024) return g;
  return 0;
}
static bool s1_use_rows(const PoolParams& p) {
  return s1_impl() == 2 && is_s1_333(p) && s1_rows_G(p) > 0 && (long long)p.T * p.H * p.W * p.C * 2 < (1ll << 30);
}
static bool s1_use_lds(const PoolParams& p) {
  return (s1_impl() == 1 || (s1_impl() == 2 && !s1_use_rows(p))) && p.T * p.H <= 512;
}
// either sweep: arg-max codes in a sweep layout, read by the matching sweep backward only
static bool s1_sweep(const PoolParams& p) { return is_s1_333(p) && (s1_use_rows(p) || s1_use_lds(p)); }

template <typename K>
static hipError_t lds_attr(K kernel) {
  return hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
}

static hipError_t launch_s1_rows_fwd(const PoolParams& p, long long B, const void* x, void* y, void* arg,
                                     hipStream_t s) {
  const int G = s1_rows_G(p), nchunk = p.C / 8 / G, n_it = p.T * p.W * G;
  const int nthr = (n_it + 63) / 64 * 64;
  const size_t lds = (size_t)(n_it + 1) * 32;
  static int df = -1;
  if (df < 0) {
    HIP_RET_E(lds_attr(maxpool_s1_fwd_rows<1>));
    HIP_RET_E(lds_attr(maxpool_s1_fwd_rows<2>));
    HIP_RET_E(lds_attr(maxpool_s1_fwd_rows<3>));
    HIP_RET_E(lds_attr(maxpool_s1_fwd_rows<4>));
    df = env_int("MILNCE_S1_DF", 3, 1, 4);
  }
  const dim3 grid((unsigned)(B * nchunk)), block(nthr);
#define XF(n)                                                                                                  \
  hipLaunchKernelGGL((maxpool_s1_fwd_rows<n>), grid, block, lds, s, p, G, nchunk, (const bf16_t*)x, (bf16_t*)y, \
                     (uint8_t*)arg);
  switch (df) {
    case 1: XF(1) break;
    case 2: XF(2) break;
    case 4: XF(4) break;
    default: XF(3)
  }
#undef XF
  return hipSuccess;
}

static hipError_t launch_s1_rows_bwd(const PoolParams& p, long long B, const void* dy, const void* arg,
                                     const void* acc_in, const void* x, float* gs, void* dx, hipStream_t s) {
  const int G = s1_rows_G(p), nchunk = p.C / 8 / G, n_it = p.T * p.W * G;
  const int nthr = (n_it + 63) / 64 * 64;
  const size_t lds = (size_t)std::max(n_it, nthr) * 80;
  static int db = -1;
  if (db < 0) {
    HIP_RET_E(lds_attr(maxpool_s1_bwd_rows<1>));
    HIP_RET_E(lds_attr(maxpool_s1_bwd_rows<2>));
    db = env_int("MILNCE_S1_DB", 2, 1, 2);
  }
  const dim3 grid((unsigned)(B * nchunk)), block(nthr);
#define XR(n)                                                                                                  \
  hipLaunchKernelGGL((maxpool_s1_bwd_rows<n>), grid, block, lds, s, p, G, nchunk, (const bf16_t*)dy,         \
                     (const uint8_t*)arg, (const bf16_t*)acc_in, (const bf16_t*)x, gs, (bf16_t*)dx);
  if (db == 1) { XR(1) } else { XR(2) }
#undef XR
  return hipSuccess;
}
MILNCE_API int milnce_set_pool_s1_impl(int impl) {
  const int old = s1_impl();
  g_s1_impl = impl;
  return old;
}

// the sweeps, fully unrolled for the S3D-G widths (56 / 28 / 14 / 7 at 224 input; 25 / 13 / 7 at 200)
template <typename... A>
static void launch_s1_fwd(int W, dim3 grid, dim3 block, size_t lds, hipStream_t s, A... args) {
  switch (W) {
    case 25: hipLaunchKernelGGL((maxpool_s1_fwd_sep<25>), grid, block, lds, s, args...); break;
    case 28: hipLaunchKernelGGL((maxpool_s1_fwd_sep<28>), grid, block, lds, s, args...); break;
    case 13: hipLaunchKernelGGL((maxpool_s1_fwd_sep<13>), grid, block, lds, s, args...); break;
    case 14: hipLaunchKernelGGL((maxpool_s1_fwd_sep<14>), grid, block, lds, s, args...); break;
    case 7: hipLaunchKernelGGL((maxpool_s1_fwd_sep<7>), grid, block, lds, s, args...); break;
    default: hipLaunchKernelGGL((maxpool_s1_fwd_sep<0>), grid, block, lds, s, args...);
  }
}
// (the backward keeps its runtime-W loop: unrolled or with deeper register rings its carried
// columns exceed the VGPR budget and it ran 25 % slower; tools/ew_bench.py)
template <typename... A>
static void launch_s1_bwd(int W, dim3 grid, dim3 block, size_t lds, hipStream_t s, A... args) {
  (void)W;
  hipLaunchKernelGGL((maxpool_s1_bwd_sep<0>), grid, block, lds, s, args...);
}

static int s1_threads(int rows, int G) {
  const int n = rows * G;
  return ((n + 63) / 64) * 64;
}

static PoolDivs make_divs(const PoolParams& p) {
  PoolDivs d;
  d.fcpr = make_fastdiv(p.C / 8);
  d.fWo = make_fastdiv(p.Wo); d.fHo = make_fastdiv(p.Ho); d.fTo = make_fastdiv(p.To);
  d.fW = make_fastdiv(p.W); d.fH = make_fastdiv(p.H); d.fT = make_fastdiv(p.T);
  d.fplane = make_fastdiv(p.T * p.H * p.W);
  d.fmt = make_fastdiv(p.kt == 3 ? (p.T + p.pt + 1) / 2 : p.T);
  d.fmh = make_fastdiv((p.H + p.ph + 1) / 2);
  d.fmw = make_fastdiv((p.W + p.pw + 1) / 2);
  return d;
}

// Dispatch to a specialised kernel; returns false if the window shape has none.
#define MILNCE_POOL_SHAPES(X) X(1, 3, 3, 1, 2, 2) X(3, 3, 3, 2, 2, 2) X(2, 2, 2, 2, 2, 2) X(3, 3, 3, 1, 1, 1)

static bool is_s1_333(const PoolParams& p) {
  return p.kt == 3 && p.kh == 3 && p.kw == 3 && p.st == 1 && p.sh == 1 && p.sw == 1 && p.pt == 1 && p.ph == 1 &&
         p.pw == 1 && !p.zero_pad && p.To == p.T && p.Ho == p.H && p.Wo == p.W;
}

// milnce_pool_set_quad(0) turns the quad / block gathers off (A/B runs and the equality tests)
static bool g_pool_quad = true;

// Workgroups of the BN-apply pool backward (it writes no partial rows, so the grid is free;
// MILNCE_POOL_APPLY_GRID). 2048 blocks at 5 resident per CU leave a 60 %-full second round, but
// 1280 / 2560 measured the same end to end (same-box A/B, tools/gpu/env_ab.sh, r4)
static int pool_apply_grid() {
  static int g = -1;
  if (g < 0) {
    const char* e = getenv("MILNCE_POOL_APPLY_GRID");
    g = e ? atoi(e) : 2048;
    if (g < 1) g = 2048;
  }
  return g;
}

static bool pool_fwd_special(const PoolParams& p, const void* x, void* y, void* arg, long long n, hipStream_t s,
                             const float* bn_ss = nullptr, const float* gate = nullptr, void* yr = nullptr) {
  if (n >= (1ll << 31)) return false;
  const PoolDivs d = make_divs(p);
  // 1x3x3 / (1,2,2) windows without leading padding: the pair forward (maxpool_fwd_pair)
  if (p.kt == 1 && p.kh == 3 && p.kw == 3 && p.st == 1 && p.sh == 2 && p.sw == 2 && p.pt == 0 && p.To == p.T &&
      p.ph == 0 && p.pw == 0 && g_pool_quad) {
    const int Wq = (p.Wo + 1) / 2;
    const long long np = n / p.Wo * Wq;  // n = B*To*Ho*Wo*cpr
    PoolDivs dq = d;
    dq.fmw = make_fastdiv(Wq);
    const long long g = (np + 255) / 256;
    const int grid = (int)(g > 65536 ? 65536 : g);
#define XPF(bn_, gt_)                                                                                           \
    hipLaunchKernelGGL((maxpool_fwd_pair<bn_, gt_>), dim3(grid), dim3(256), 0, s, p, dq, (const bf16_t*)x,      \
                       (bf16_t*)y, (uint8_t*)arg, (uint32_t)np, Wq, bn_ss, gate, (bf16_t*)yr);
    if (bn_ss == nullptr) { XPF(false, false) }
    else if (gate != nullptr) { XPF(true, true) }
    else { XPF(true, false) }
#undef XPF
    return true;
  }
  if (bn_ss != nullptr) {
    if (s1_sweep(p)) return false;  // its backward reads sweep-layout codes
    long long g = (n + 255) / 256;
    const int grid = (int)(g > 65536 ? 65536 : g);
#define X(a, b, c, e, f, h)                                                                                      \
    if (p.kt == a && p.kh == b && p.kw == c && p.st == e && p.sh == f && p.sw == h) {                            \
      if (gate != nullptr)                                                                                           \
        hipLaunchKernelGGL((maxpool_fwd_t<a, b, c, e, f, h, true, true>), dim3(grid), dim3(256), 0, s, p, d,     \
                           (const bf16_t*)x, (bf16_t*)y, (uint8_t*)arg, (uint32_t)n, bn_ss, gate, (bf16_t*)yr);  \
      else                                                                                                       \
        hipLaunchKernelGGL((maxpool_fwd_t<a, b, c, e, f, h, true, false>), dim3(grid), dim3(256), 0, s, p, d,    \
                           (const bf16_t*)x, (bf16_t*)y, (uint8_t*)arg, (uint32_t)n, bn_ss, nullptr,             \
                           (bf16_t*)yr);                                                                         \
      return true;                                                                                               \
    }
    MILNCE_POOL_SHAPES(X)
#undef X
    return false;
  }
  if (s1_use_rows(p)) {
    const long long B = n / ((long long)p.T * p.H * p.W * (p.C / 8));
    (void)launch_s1_rows_fwd(p, B, x, y, arg, s);  // a failed launch shows in hipGetLastError
    return true;
  }
  if (is_s1_333(p) && s1_use_lds(p)) {
    const long long B = n / ((long long)p.T * p.H * p.W * (p.C / 8));
    const int rows = p.T * p.H, G = s1_groups(rows, p.C, g_s1_maxthr, B), nchunk = (p.C / 8 + G - 1) / G;
    launch_s1_fwd(p.W, dim3((unsigned)(B * nchunk)), dim3(s1_threads(rows, G)), s1_fwd_lds(rows, G), s, p, G,
                  nchunk, (const bf16_t*)x, (bf16_t*)y, (uint8_t*)arg);
    return true;
  }
  if (is_s1_333(p)) {
    const long long rows = n / p.W / (p.C / 8);  // n = B*T*H*W*cpr
    const long long thr = rows * (p.C / 8);
    const int grid = (int)((thr + 255) / 256 > 65536 ? 65536 : (thr + 255) / 256);
    hipLaunchKernelGGL(maxpool_s1_fwd_slide, dim3(grid), dim3(256), 0, s, p, d, (const bf16_t*)x, (bf16_t*)y,
                       (uint8_t*)arg, (uint32_t)rows);
    return true;
  }
  long long g = (n + 255) / 256;
  const int grid = (int)(g > 65536 ? 65536 : g);
#define X(a, b, c, e, f, h)                                                                                      \
  if (p.kt == a && p.kh == b && p.kw == c && p.st == e && p.sh == f && p.sw == h) {                              \
    hipLaunchKernelGGL((maxpool_fwd_t<a, b, c, e, f, h>), dim3(grid), dim3(256), 0, s, p, d, (const bf16_t*)x,   \
                       (bf16_t*)y, (uint8_t*)arg, (uint32_t)n);                                                  \
    return true;                                                                                                 \
  }
  MILNCE_POOL_SHAPES(X)
#undef X
  return false;
}

MILNCE_API int milnce_pool_set_quad(int on) {
  g_pool_quad = on != 0;
  return 0;
}

static bool pool_bwd_special(const PoolParams& p, const void* dy, const void* arg, void* dx, long long n,
                             const void* bn_y, int bn_ld, const float* bn_ss, float* part, int nparts,
                             hipStream_t s, const void* gx = nullptr, float* gs = nullptr,
                             const float* gate_g = nullptr, const float* gate_dm = nullptr, float inv_thw = 0.f,
                             const float* coef = nullptr) {
  if (n >= (1ll << 31)) return false;
  // codes in the sweep layout (the plane-sweep forward wrote them) are read by the sweep backward
  // only, which has no BN-partials / gate / apply epilogues
  if (s1_sweep(p) && (bn_y != nullptr || gate_g != nullptr || coef != nullptr)) return false;
  const PoolDivs d = make_divs(p);
  if (s1_use_rows(p) && bn_y == nullptr) {
    const long long B = n / ((long long)p.T * p.H * p.W * (p.C / 8));
    (void)launch_s1_rows_bwd(p, B, dy, arg, nullptr, nullptr, nullptr, dx, s);
    return true;
  }
  if (is_s1_333(p) && bn_y == nullptr && s1_use_lds(p)) {
    const long long B = n / ((long long)p.T * p.H * p.W * (p.C / 8));
    const int rows = p.T * p.H, G = s1_groups(rows, p.C, g_s1_maxthr, B), nchunk = (p.C / 8 + G - 1) / G;
    launch_s1_bwd(p.W, dim3((unsigned)(B * nchunk)), dim3(s1_threads(rows, G)), s1_bwd_lds(rows, G), s, p, G,
                  nchunk, (const bf16_t*)dy, (const uint8_t*)arg, (const bf16_t*)nullptr, (const bf16_t*)nullptr,
                  (float*)nullptr, (bf16_t*)dx);
    return true;
  }
  if (is_s1_333(p) && bn_y == nullptr) {
    const long long rows = n / p.W / (p.C / 8);
    const long long thr = rows * (p.C / 8);
    const int grid = (int)((thr + 255) / 256 > 65536 ? 65536 : (thr + 255) / 256);
    hipLaunchKernelGGL(maxpool_s1_bwd_slide, dim3(grid), dim3(256), 0, s, p, d, (const bf16_t*)dy,
                       (const uint8_t*)arg, (bf16_t*)dx, (uint32_t)rows);
    return true;
  }
  const int mode = coef != nullptr ? POOL_BWD_APPLY : (gate_g != nullptr ? POOL_BWD_GATED : POOL_BWD_PLAIN);
  if (mode == POOL_BWD_APPLY && part == nullptr) nparts = pool_apply_grid();  // grid only: no partial rows
  const uint32_t npos = (uint32_t)(n / (p.C / 8));
  const uint32_t ppb = (npos + nparts - 1) / nparts;
  // deterministic gate reduction (gs): per-block partial rows when a block's items span at most two
  // clips (items per block <= items per clip), summed in block order after the pass
  const long long nclip = (long long)npos / ((long long)p.T * p.H * p.W);
  float* gpart = nullptr;
  long long g_ipc = 0, g_ipb = 0;
  auto gs_prep = [&](long long items, long long ipb) {
    gpart = nullptr;
    if (gs == nullptr || mode != POOL_BWD_PLAIN || nclip < 1) return;
    const long long ipc = items / nclip;
    if (ipb > ipc) return;  // atomics
    g_ipc = ipc;
    g_ipb = ipb;
    gpart = stream_scratch((size_t)nparts * 2 * p.C + nparts, s, SCRATCH_POOL_GS);
  };
  auto gs_post = [&]() {
    if (gpart == nullptr) return;
    const long long nn = nclip * p.C;
    const long long g = (nn + 255) / 256;
    hipLaunchKernelGGL(pool_gs_sum_kernel, dim3((int)(g < 4096 ? g : 4096)), dim3(256), 0, s, gs, gpart, nparts,
                       (int)nclip, p.C, g_ipc, g_ipb);
  };
  const bool blk133 = p.kt == 1 && p.kh == 3 && p.kw == 3 && p.st == 1 && p.sh == 2 && p.sw == 2 && p.pt == 0 &&
                      p.To == p.T && p.ph <= 1 && p.pw <= 1;
  const bool blk333 = p.kt == 3 && p.kh == 3 && p.kw == 3 && p.st == 2 && p.sh == 2 && p.sw == 2 && p.pt <= 1 &&
                      p.ph <= 1 && p.pw <= 1;
  if ((blk133 || blk333) && g_pool_quad) {
    const uint32_t nb = npos / (p.T * p.H * p.W);
    const uint32_t nq = nb * d.fmt.d * d.fmh.d * d.fmw.d, qpb = (nq + nparts - 1) / nparts;
    // an even H, W plane without leading padding takes the leaner quad indexing (pool_bwd_quad)
    const bool even = blk133 && p.ph == 0 && p.pw == 0 && p.H == 2 * p.Ho && p.W == 2 * p.Wo;
    gs_prep(nq, qpb);
#define XQ(a, m)                                                                                                 \
    if (mode == m && even) {                                                                                     \
      hipLaunchKernelGGL((maxpool_bwd_t<1, 3, 3, 1, 2, 2, m, 1>), dim3(nparts), dim3(256), 0, s, p, d,           \
                         (const bf16_t*)dy, (const uint8_t*)arg, (bf16_t*)dx, nq, qpb, (const bf16_t*)bn_y,     \
                         bn_ld, bn_ss, part, (const bf16_t*)gx, gs, gate_g, gate_dm, inv_thw, coef, gpart);      \
      gs_post();                                                                                                 \
      return true;                                                                                               \
    }                                                                                                            \
    if (mode == m) {                                                                                             \
      hipLaunchKernelGGL((maxpool_bwd_t<a, 3, 3, a == 3 ? 2 : 1, 2, 2, m, 2>), dim3(nparts), dim3(256), 0, s,    \
                         p, d, (const bf16_t*)dy, (const uint8_t*)arg, (bf16_t*)dx, nq, qpb,                     \
                         (const bf16_t*)bn_y, bn_ld, bn_ss, part, (const bf16_t*)gx, gs, gate_g, gate_dm,        \
                         inv_thw, coef, gpart);                                                                  \
      gs_post();                                                                                                 \
      return true;                                                                                               \
    }
    if (blk133) {
      XQ(1, POOL_BWD_PLAIN) XQ(1, POOL_BWD_GATED) XQ(1, POOL_BWD_APPLY)
    } else {
      XQ(3, POOL_BWD_PLAIN) XQ(3, POOL_BWD_GATED) XQ(3, POOL_BWD_APPLY)
    }
#undef XQ
  }
  gs_prep(npos, ppb);
#define XM(a, b, c, e, f, h, m)                                                                                  \
  if (p.kt == a && p.kh == b && p.kw == c && p.st == e && p.sh == f && p.sw == h && mode == m) {                 \
    hipLaunchKernelGGL((maxpool_bwd_t<a, b, c, e, f, h, m>), dim3(nparts), dim3(256), 0, s, p, d, (const bf16_t*)dy, \
                       (const uint8_t*)arg, (bf16_t*)dx, npos, ppb, (const bf16_t*)bn_y, bn_ld, bn_ss, part,     \
                       (const bf16_t*)gx, gs, gate_g, gate_dm, inv_thw, coef, gpart);                            \
    gs_post();                                                                                                   \
    return true;                                                                                                 \
  }
#define X(a, b, c, e, f, h) XM(a, b, c, e, f, h, POOL_BWD_PLAIN) XM(a, b, c, e, f, h, POOL_BWD_GATED) \
  XM(a, b, c, e, f, h, POOL_BWD_APPLY)
  MILNCE_POOL_SHAPES(X)
#undef X
#undef XM
  return false;
}

static int g_s1_codes = 1;  // milnce_set_pool_s1_codes: code layout of the plane sweeps (S1Geo)
MILNCE_API int milnce_set_pool_s1_codes(int on) {
  const int old = g_s1_codes;
  g_s1_codes = on != 0;
  return old;
}
static PoolParams make_pool(int T, int H, int W, int C, int To, int Ho, int Wo, int kt, int kh, int kw, int st,
                            int sh, int sw, int pt0, int pt1, int ph0, int ph1, int pw0, int pw1, int zero_pad) {
  PoolParams p;
  p.T = T; p.H = H; p.W = W; p.C = C; p.To = To; p.Ho = Ho; p.Wo = Wo;
  p.kt = kt; p.kh = kh; p.kw = kw; p.st = st; p.sh = sh; p.sw = sw;
  p.pt = pt0; p.ph = ph0; p.pw = pw0;
  p.Tp = T + pt0 + pt1; p.Hp = H + ph0 + ph1; p.Wp = W + pw0 + pw1;
  p.zero_pad = zero_pad;
  p.s1_codes = g_s1_codes;
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
  if (pool_fwd_special(p, x, y, arg, n, stream)) return (int)hipGetLastError();
  hipLaunchKernelGGL(maxpool_fwd_kernel, dim3(grid_for(n)), dim3(256), 0, stream, p, (const bf16_t*)x,
                     (bf16_t*)y, (uint8_t*)arg, n);
  return (int)hipGetLastError();
}

// Train-mode BN + ReLU + max pool in one pass over the raw conv output (specialised window
// shapes only; returns hipErrorInvalidValue otherwise).
// yr (optional, pooled shape): the raw conv output x at each output's arg-max, so the BN-backward
// partial sums of the pool input's BN can be taken over the pooled tensors (the consumer's dgrad
// epilogue, csrc/conv.hip EPI 2) instead of a gather pass over the full-resolution x.
MILNCE_API int milnce_bn_relu_maxpool_fwd(const void* x, const float* ss, void* y, void* arg, int B, int T, int H,
                                          int W, int C, int To, int Ho, int Wo, int kt, int kh, int kw, int st,
                                          int sh, int sw, int pt0, int pt1, int ph0, int ph1, int pw0, int pw1,
                                          int zero_pad, void* yr, hipStream_t stream) {
  if (C % 8) return (int)hipErrorInvalidValue;
  PoolParams p = make_pool(T, H, W, C, To, Ho, Wo, kt, kh, kw, st, sh, sw, pt0, pt1, ph0, ph1, pw0, pw1, zero_pad);
  const long long n = (long long)B * To * Ho * Wo * (C / 8);
  if (!pool_fwd_special(p, x, y, arg, n, stream, ss, nullptr, yr)) return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

// nparts: grid size used (also the number of partial rows written when bn_y != null).
MILNCE_API int milnce_maxpool_bwd(const void* dy, const void* arg, void* dx, int B, int T, int H, int W, int C,
                                  int To, int Ho, int Wo, int kt, int kh, int kw, int st, int sh, int sw, int pt0,
                                  int pt1, int ph0, int ph1, int pw0, int pw1, int zero_pad, const void* bn_y,
                                  int bn_ld, const float* bn_ss, float* part, int nparts, hipStream_t stream) {
  if (C % 8) return (int)hipErrorInvalidValue;
  PoolParams p = make_pool(T, H, W, C, To, Ho, Wo, kt, kh, kw, st, sh, sw, pt0, pt1, ph0, ph1, pw0, pw1, zero_pad);
  const long long n = (long long)B * T * H * W * (C / 8);
  if (pool_bwd_special(p, dy, arg, dx, n, bn_y, bn_ld, bn_ss, part, nparts, stream)) return (int)hipGetLastError();
  if (dx == nullptr) return (int)hipErrorInvalidValue;  // partials-only passes: specialised shapes
  if (s1_sweep(p)) return (int)hipErrorInvalidValue;  // sweep-layout codes
  if (bn_y != nullptr && (256 % (C / 8) != 0 || bn_ld != C)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(nparts), dim3(256), 0, stream, p, (const bf16_t*)dy,
                     (const uint8_t*)arg, (bf16_t*)dx, n, (const bf16_t*)bn_y, bn_ss, part);
  return (int)hipGetLastError();
}

// Inception branch-3 pool backward with the fused epilogue of maxpool_s1_bwd_lds:
// dx = pool_bwd(dy) (+ acc_in), and (gs != null) gs[b, c] = sum_thw dx * x.
MILNCE_API int milnce_maxpool_s1_bwd_fused(const void* dy, const void* arg, const void* acc_in, const void* x,
                                           float* gs, void* dx, int B, int T, int H, int W, int C,
                                           hipStream_t stream) {
  if (C % 8) return (int)hipErrorInvalidValue;
  PoolParams p = make_pool(T, H, W, C, T, H, W, 3, 3, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0);
  const int rows = T * H;
  // the separable code layout must match the forward that produced arg (milnce_maxpool_fwd)
  if (gs != nullptr && x == nullptr) return (int)hipErrorInvalidValue;
  if (s1_use_rows(p)) {
    HIP_RET(launch_s1_rows_bwd(p, B, dy, arg, acc_in, x, gs, dx, stream));
    return (int)hipGetLastError();
  }
  if (!s1_use_lds(p)) return (int)hipErrorInvalidValue;
  const int G = s1_groups(rows, C, g_s1_maxthr, B), nchunk = (C / 8 + G - 1) / G;
  launch_s1_bwd(W, dim3((unsigned)((long long)B * nchunk)), dim3(s1_threads(rows, G)), s1_bwd_lds(rows, G), stream,
                p, G, nchunk, (const bf16_t*)dy, (const uint8_t*)arg, (const bf16_t*)acc_in, (const bf16_t*)x, gs,
                (bf16_t*)dx);
  return (int)hipGetLastError();
}

// TF-SAME pool backward whose input x is a SelfGating output: dx as milnce_maxpool_bwd (no BN
// partials) plus gs[b, c] += sum_thw dx * x (gs zeroed by the caller), which the gate backward
// uses instead of re-reading its gradient and output.
MILNCE_API int milnce_maxpool_bwd_gate(const void* dy, const void* arg, void* dx, int B, int T, int H, int W, int C,
                                       int To, int Ho, int Wo, int kt, int kh, int kw, int st, int sh, int sw,
                                       int pt0, int pt1, int ph0, int ph1, int pw0, int pw1, int zero_pad,
                                       const void* x, float* gs, int nparts, hipStream_t stream) {
  if (C % 8 || C / 8 > 256) return (int)hipErrorInvalidValue;
  PoolParams p = make_pool(T, H, W, C, To, Ho, Wo, kt, kh, kw, st, sh, sw, pt0, pt1, ph0, ph1, pw0, pw1, zero_pad);
  const long long n = (long long)B * T * H * W * (C / 8);
  if (is_s1_333(p)) return (int)hipErrorInvalidValue;
  if (pool_bwd_special(p, dy, arg, dx, n, nullptr, 0, nullptr, nullptr, nparts, stream, x, gs))
    return (int)hipGetLastError();
  return (int)hipErrorInvalidValue;
}

// SelfGating of a lazy BN-ReLU input followed by a TF-SAME max pool, in one pass over the raw conv
// output x: pools bf16(bf16(relu(x * scale + shift)) * gate[b, c]), the gate output the unfused ops
// would store (specialised window shapes only).
// yr (optional, pooled shape): the raw conv output x at each output's arg-max, so the BN-backward
// partial sums of x's BN can be taken over the pooled tensors (milnce_gated_pool_bn_partials).
MILNCE_API int milnce_bn_relu_gate_maxpool_fwd(const void* x, const float* ss, const float* gate, void* y, void* arg,
                                               int B, int T, int H, int W, int C, int To, int Ho, int Wo, int kt,
                                               int kh, int kw, int st, int sh, int sw, int pt0, int pt1, int ph0,
                                               int ph1, int pw0, int pw1, int zero_pad, void* yr, hipStream_t stream) {
  if (C % 8 || gate == nullptr) return (int)hipErrorInvalidValue;
  PoolParams p = make_pool(T, H, W, C, To, Ho, Wo, kt, kh, kw, st, sh, sw, pt0, pt1, ph0, ph1, pw0, pw1, zero_pad);
  const long long n = (long long)B * To * Ho * Wo * (C / 8);
  if (!pool_fwd_special(p, x, y, arg, n, stream, ss, gate, yr)) return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

// Its backward down to the BN layer: dz = bf16(bf16(pool_bwd(dy)) * g + dmean / thw), the SelfGating
// backward once its reduction (milnce_gate_dot on the pooled output) and fc backward are done, plus
// the BN-backward partials of dz (thw = T * H * W). dz may be null (partials only).
MILNCE_API int milnce_maxpool_bwd_gated(const void* dy, const void* arg, void* dz, int B, int T, int H, int W, int C,
                                        int To, int Ho, int Wo, int kt, int kh, int kw, int st, int sh, int sw,
                                        int pt0, int pt1, int ph0, int ph1, int pw0, int pw1, int zero_pad,
                                        const void* bn_y, int bn_ld, const float* bn_ss, float* part, int nparts,
                                        const float* g, const float* dmean, hipStream_t stream) {
  if (C % 8 || C / 8 > 256 || bn_y == nullptr || g == nullptr || dmean == nullptr) return (int)hipErrorInvalidValue;
  PoolParams p = make_pool(T, H, W, C, To, Ho, Wo, kt, kh, kw, st, sh, sw, pt0, pt1, ph0, ph1, pw0, pw1, zero_pad);
  const long long n = (long long)B * T * H * W * (C / 8);
  if (is_s1_333(p)) return (int)hipErrorInvalidValue;
  const int thw = T * H * W;
  const float inv_thw = 1.f / thw;
  if (pool_bwd_special(p, dy, arg, dz, n, bn_y, bn_ld, bn_ss, part, nparts, stream, nullptr, nullptr, g, dmean,
                       inv_thw))
    return (int)hipGetLastError();
  return (int)hipErrorInvalidValue;
}

// Pool backward with the BN backward of the pool input's producer applied on the fly (dz gated as in
// milnce_maxpool_bwd_gated when g != null): out = the producer conv's output gradient, so the
// full-resolution dz is never stored. coef = milnce_bn_bwd_finalize of the partials a first pass
// (milnce_maxpool_bwd / milnce_maxpool_bwd_gated with dz = null) produced.
MILNCE_API int milnce_maxpool_bwd_apply(const void* dy, const void* arg, void* out, int B, int T, int H, int W, int C,
                                        int To, int Ho, int Wo, int kt, int kh, int kw, int st, int sh, int sw,
                                        int pt0, int pt1, int ph0, int ph1, int pw0, int pw1, int zero_pad,
                                        const void* bn_y, int bn_ld, const float* bn_ss, const float* coef,
                                        const float* g, const float* dmean, int nparts, hipStream_t stream) {
  if (C % 8 || C / 8 > 256 || bn_y == nullptr || coef == nullptr || out == nullptr ||
      (g == nullptr) != (dmean == nullptr))
    return (int)hipErrorInvalidValue;
  PoolParams p = make_pool(T, H, W, C, To, Ho, Wo, kt, kh, kw, st, sh, sw, pt0, pt1, ph0, ph1, pw0, pw1, zero_pad);
  const long long n = (long long)B * T * H * W * (C / 8);
  if (is_s1_333(p)) return (int)hipErrorInvalidValue;
  const int thw = T * H * W;
  const float inv_thw = 1.f / thw;
  if (pool_bwd_special(p, dy, arg, out, n, bn_y, bn_ld, bn_ss, nullptr, nparts, stream, nullptr, nullptr, g, dmean,
                       inv_thw, coef))
    return (int)hipGetLastError();
  return (int)hipErrorInvalidValue;
}
