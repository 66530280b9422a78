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

// ---------------------------------------------------------------------------------------
// Specialised pools: window/stride are template constants (every S3D-G pool is one of four
// shapes), index math is 32-bit FastDiv, and every tap's load is issued unconditionally from a
// clamped address and masked afterwards, so the whole window's loads are in flight at once
// (the generic kernels above serialise on their per-tap branches).
struct PoolDivs {
  FastDiv fcpr, fWo, fHo, fTo, fW, fH, fT;
};

// BN: x is the raw conv output of a train-mode BN layer and z = relu(x * scale + shift) is
// pooled without being materialised (ss = [mean, invstd, scale, shift] per channel); padded
// cells stay zero candidates, as for the z the unfused pool would read.
template <int KT, int KH, int KW, int ST, int SH, int SW, bool BN = false>
__global__ __launch_bounds__(256) void maxpool_fwd_t(PoolParams p, PoolDivs d, const bf16_t* __restrict__ x,
                                                     bf16_t* __restrict__ y, uint8_t* __restrict__ arg,
                                                     uint32_t nout_chunks, const float* __restrict__ ss = nullptr) {
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
    float best[8], sc[8], sh[8];
    uint32_t bi[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      best[k] = -INFINITY;
      bi[k] = 0;
      if constexpr (BN) {
        sc[k] = ss[2 * p.C + c0 + k];
        sh[k] = ss[3 * p.C + c0 + k];
      }
    }
#pragma unroll
    for (int t = 0; t < KT * KH * KW; ++t) {
      float f[8];
      unpack8(v[t], f);
      if constexpr (BN) {
#pragma unroll
        for (int k = 0; k < 8; ++k) f[k] = bf2f(f2bf(fmaxf(f[k] * sc[k] + sh[k], 0.f)));  // = the stored z
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float val = in[t] ? f[k] : (cand[t] ? 0.f : -INFINITY);
        const bool gt = val > best[k];
        best[k] = gt ? val : best[k];
        bi[k] = gt ? (uint32_t)t : bi[k];
      }
    }
    const size_t o = (size_t)i * 8;
    *(uint4*)(y + o) = pack8(best);
    uint2 a;
    a.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | (bi[3] << 24);
    a.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | (bi[7] << 24);
    *(uint2*)(arg + o) = a;
  }
}

// BN-backward partial sums of the pool input's producer (dx is that layer's dz), accumulated
// per thread for its fixed channel chunk and reduced over the block's row groups in LDS:
// part[blockIdx][2][C] (mask = y*scale + shift > 0, xhat = (y - mean) * invstd).
struct BnAcc {
  float a1[8], a2[8];
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int k = 0; k < 8; ++k) { a1[k] = 0.f; a2[k] = 0.f; }
  }
  __device__ __forceinline__ void add(const float* d, const bf16_t* ypos, const float* ss, int C, int c0) {
    float yv[8];
    unpack8(*(const uint4*)ypos, yv);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int c = c0 + k;
      const float gm = (yv[k] * ss[2 * C + c] + ss[3 * C + c] > 0.f) ? d[k] : 0.f;
      a1[k] += gm;
      a2[k] += gm * (yv[k] - ss[c]) * ss[C + c];
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

// Thread = fixed 8-channel chunk cc = tid % cpr of rpi = 256/cpr input positions per step; block
// blockIdx.x walks positions [pos_begin, pos_end), two positions per thread per iteration so
// both gathers' loads are in flight together.
template <int KT, int KH, int KW, int ST, int SH, int SW>
__global__ __launch_bounds__(256) void maxpool_bwd_t(PoolParams p, PoolDivs d, const bf16_t* __restrict__ dy,
                                                     const uint8_t* __restrict__ arg, bf16_t* __restrict__ dx,
                                                     uint32_t npos, uint32_t pos_per_block,
                                                     const bf16_t* __restrict__ bn_y, int bn_ld,
                                                     const float* __restrict__ bn_ss, float* __restrict__ part) {
  __shared__ float red[16 * 256];
  const int cpr = p.C >> 3, rpi = 256 / cpr;
  const int cc = threadIdx.x % cpr, rr = threadIdx.x / cpr;
  const bool active = rr < rpi;
  const int c0 = cc * 8;
  const bool bn = bn_y != nullptr;
  BnAcc acc_bn;
  acc_bn.zero();
  const uint32_t pos_begin = blockIdx.x * pos_per_block;
  const uint32_t pos_end = min(npos, pos_begin + pos_per_block);
  for (uint32_t pos = pos_begin + rr; active && pos < pos_end; pos += 2 * rpi) {
    const uint32_t pos2 = pos + rpi;
    const bool two = pos2 < pos_end;
    float a0[8], a1[8];
    pool_bwd_one<KT, KH, KW, ST, SH, SW>(p, d, dy, arg, pos, c0, a0);
    pool_bwd_one<KT, KH, KW, ST, SH, SW>(p, d, dy, arg, two ? pos2 : pos, c0, a1);
    const uint4 v0 = pack8(a0), v1 = pack8(a1);
    *(uint4*)(dx + (size_t)pos * p.C + c0) = v0;
    if (two) *(uint4*)(dx + (size_t)pos2 * p.C + c0) = v1;
    if (bn) {
      float dr[8];
      unpack8(v0, dr);
      acc_bn.add(dr, bn_y + (size_t)pos * bn_ld + c0, bn_ss, p.C, c0);
      if (two) {
        unpack8(v1, dr);
        acc_bn.add(dr, bn_y + (size_t)pos2 * bn_ld + c0, bn_ss, p.C, c0);
      }
    }
  }
  if (bn) acc_bn.commit(red, part, p.C, cpr, rpi, cc, rr, active);
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

static PoolDivs make_divs(const PoolParams& p) {
  PoolDivs d;
  d.fcpr = make_fastdiv(p.C / 8);
  d.fWo = make_fastdiv(p.Wo); d.fHo = make_fastdiv(p.Ho); d.fTo = make_fastdiv(p.To);
  d.fW = make_fastdiv(p.W); d.fH = make_fastdiv(p.H); d.fT = make_fastdiv(p.T);
  return d;
}

// Dispatch to a specialised kernel; returns false if the window shape has none.
#define MILNCE_POOL_SHAPES(X) X(1, 3, 3, 1, 2, 2) X(3, 3, 3, 2, 2, 2) X(2, 2, 2, 2, 2, 2) X(3, 3, 3, 1, 1, 1)

static bool is_s1_333(const PoolParams& p) {
  return p.kt == 3 && p.kh == 3 && p.kw == 3 && p.st == 1 && p.sh == 1 && p.sw == 1 && p.pt == 1 && p.ph == 1 &&
         p.pw == 1 && !p.zero_pad && p.To == p.T && p.Ho == p.H && p.Wo == p.W;
}

static bool pool_fwd_special(const PoolParams& p, const void* x, void* y, void* arg, long long n, hipStream_t s,
                             const float* bn_ss = nullptr) {
  if (n >= (1ll << 31)) return false;
  const PoolDivs d = make_divs(p);
  if (bn_ss != nullptr) {
    long long g = (n + 255) / 256;
    const int grid = (int)(g > 65536 ? 65536 : g);
#define X(a, b, c, e, f, h)                                                                                      \
    if (p.kt == a && p.kh == b && p.kw == c && p.st == e && p.sh == f && p.sw == h) {                            \
      hipLaunchKernelGGL((maxpool_fwd_t<a, b, c, e, f, h, true>), dim3(grid), dim3(256), 0, s, p, d,             \
                         (const bf16_t*)x, (bf16_t*)y, (uint8_t*)arg, (uint32_t)n, bn_ss);                       \
      return true;                                                                                               \
    }
    MILNCE_POOL_SHAPES(X)
#undef X
    return false;
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

static bool pool_bwd_special(const PoolParams& p, const void* dy, const void* arg, void* dx, long long n,
                             const void* bn_y, int bn_ld, const float* bn_ss, float* part, int nparts,
                             hipStream_t s) {
  if (n >= (1ll << 31)) return false;
  const PoolDivs d = make_divs(p);
  if (is_s1_333(p) && bn_y == nullptr) {
    const long long rows = n / p.W / (p.C / 8);
    const long long thr = rows * (p.C / 8);
    const int grid = (int)((thr + 255) / 256 > 65536 ? 65536 : (thr + 255) / 256);
    hipLaunchKernelGGL(maxpool_s1_bwd_slide, dim3(grid), dim3(256), 0, s, p, d, (const bf16_t*)dy,
                       (const uint8_t*)arg, (bf16_t*)dx, (uint32_t)rows);
    return true;
  }
  const uint32_t npos = (uint32_t)(n / (p.C / 8));
  const uint32_t ppb = (npos + nparts - 1) / nparts;
#define X(a, b, c, e, f, h)                                                                                      \
  if (p.kt == a && p.kh == b && p.kw == c && p.st == e && p.sh == f && p.sw == h) {                              \
    hipLaunchKernelGGL((maxpool_bwd_t<a, b, c, e, f, h>), dim3(nparts), dim3(256), 0, s, p, d, (const bf16_t*)dy, \
                       (const uint8_t*)arg, (bf16_t*)dx, npos, ppb, (const bf16_t*)bn_y, bn_ld, bn_ss, part);    \
    return true;                                                                                                 \
  }
  MILNCE_POOL_SHAPES(X)
#undef X
  return false;
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
  if (pool_fwd_special(p, x, y, arg, n, stream)) return (int)hipGetLastError();
  hipLaunchKernelGGL(maxpool_fwd_kernel, dim3(grid_for(n)), dim3(256), 0, stream, p, (const bf16_t*)x,
                     (bf16_t*)y, (uint8_t*)arg, n);
  return (int)hipGetLastError();
}

// Train-mode BN + ReLU + max pool in one pass over the raw conv output (specialised window
// shapes only; returns hipErrorInvalidValue otherwise).
MILNCE_API int milnce_bn_relu_maxpool_fwd(const void* x, const float* ss, void* y, void* arg, int B, int T, int H,
                                          int W, int C, int To, int Ho, int Wo, int kt, int kh, int kw, int st,
                                          int sh, int sw, int pt0, int pt1, int ph0, int ph1, int pw0, int pw1,
                                          int zero_pad, hipStream_t stream) {
  if (C % 8) return (int)hipErrorInvalidValue;
  PoolParams p = make_pool(T, H, W, C, To, Ho, Wo, kt, kh, kw, st, sh, sw, pt0, pt1, ph0, ph1, pw0, pw1, zero_pad);
  const long long n = (long long)B * To * Ho * Wo * (C / 8);
  if (!pool_fwd_special(p, x, y, arg, n, stream, ss)) return (int)hipErrorInvalidValue;
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
  if (bn_y != nullptr && (256 % (C / 8) != 0 || bn_ld != C)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(nparts), dim3(256), 0, stream, p, (const bf16_t*)dy,
                     (const uint8_t*)arg, (bf16_t*)dx, n, (const bf16_t*)bn_y, bn_ss, part);
  return (int)hipGetLastError();
}
