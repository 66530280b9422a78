// Train-mode BatchNorm3d + ReLU around the implicit-GEMM conv (channels-last, bf16 data).
//
// forward : conv epilogue partial sums --(bn_finalize)--> mean/invstd/scale/shift + running
//           stats update (momentum 0.1, unbiased running_var, num_batches_tracked += 1)
//           --(bn_relu_apply)--> z = relu(y*scale + shift), optionally also accumulating the
//           per-(clip, channel) sum of z that the following SelfGating needs (its global mean),
//           so the gate never re-reads z for the mean.
// backward: bn_bwd_reduce (sum dz*mask, sum dz*mask*xhat per channel, mask = z > 0 recomputed
//           from y) -> bn_bwd_finalize (dgamma, dbeta, coefficients) -> bn_bwd_apply
//           dy = gamma*invstd*(dz*mask - dbeta/n - xhat*dgamma/n).
// All elementwise passes move 16 B per lane (8 bf16).
#include "common.h"

// ---------------------------------------------------------------------------------------
// Partial-slab reductions ([nparts][2][stride] fp32 -> per-channel fp64 sums). They are
// latency-bound (a few MB over few channels) and sit on the main chain of the backward pass,
// where the side stream's weight-gradient workgroups hold most of every CU (wave slots, VGPRs,
// LDS: two 80-KiB temporal-wgrad workgroups fill a CU's LDS). A finalize workgroup that needs
// 16 waves and 16 KiB (the round-5 shape) waited up to 0.67 ms for a CU to drain; this one is
// 4 waves with 512 B of LDS: 8 channels x 32 row groups, each thread summing its rows with four
// loads in flight, a fixed-order butterfly over the wave's row groups, then the 4 waves in order
// (deterministic).
#ifndef MILNCE_FIN_RG
#define MILNCE_FIN_RG 32
#endif
constexpr int FIN_CH = 8, FIN_RG = MILNCE_FIN_RG;
static_assert(FIN_RG % 8 == 0 && FIN_RG <= 128, "row groups: whole waves");
#ifndef MILNCE_BN_U
#define MILNCE_BN_U 4
#endif
constexpr int BN_U = MILNCE_BN_U;  // rows in flight per thread in the streaming apply kernels

__device__ __forceinline__ void fin_reduce(const float* __restrict__ part, int nparts, int stride, int c, bool ok,
                                           double& s1, double& s2) {
  constexpr int NWV = FIN_RG / 8;  // waves
  __shared__ double red[2][NWV][FIN_CH];
  const int cl = threadIdx.x % FIN_CH, rg = threadIdx.x / FIN_CH;
  double a[4] = {0.0, 0.0, 0.0, 0.0}, b[4] = {0.0, 0.0, 0.0, 0.0};
  if (ok) {
    int i = rg;
    for (; i + 3 * FIN_RG < nparts; i += 4 * FIN_RG) {
      float u[4], v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float* p0 = part + (long long)(i + k * FIN_RG) * 2 * stride + c;
        u[k] = p0[0];
        v[k] = p0[stride];
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        a[k] += (double)u[k];
        b[k] += (double)v[k];
      }
    }
    for (; i < nparts; i += FIN_RG) {
      a[0] += (double)part[(long long)i * 2 * stride + c];
      b[0] += (double)part[(long long)i * 2 * stride + stride + c];
    }
  }
  double x1 = (a[0] + a[1]) + (a[2] + a[3]), x2 = (b[0] + b[1]) + (b[2] + b[3]);
  // the wave's 8 row groups (lane bits 3..5): every lane ends with the same fixed-order sum
#pragma unroll
  for (int o = 8; o < 64; o <<= 1) {
    x1 += __shfl_xor(x1, o, 64);
    x2 += __shfl_xor(x2, o, 64);
  }
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) < FIN_CH) {
    red[0][wv][cl] = x1;
    red[1][wv][cl] = x2;
  }
  __syncthreads();
  double t1 = 0.0, t2 = 0.0;
#pragma unroll
  for (int w = 0; w < NWV; ++w) {
    t1 += red[0][w][cl];
    t2 += red[1][w][cl];
  }
  s1 = t1;
  s2 = t2;
}

__device__ __forceinline__ void bn_finalize_body(
    int blk, const float* __restrict__ part, int nparts, int Npad, int C, double count, const float* __restrict__ gamma,
    const float* __restrict__ beta, float* rmean, float* __restrict__ rvar, long long* __restrict__ nbt,
    float momentum, float eps, int training, float* __restrict__ out, float* yshift) {
  const int c = blk * FIN_CH + threadIdx.x % FIN_CH;
  if (training && blk == 0 && threadIdx.x == 0 && nbt != nullptr) nbt[0] += 1;
  double s, q;
  fin_reduce(part, training ? nparts : 0, Npad, c, training && c < C, s, q);
  if (threadIdx.x >= FIN_CH || c >= C) return;
  float mean, var;
  if (training) {
    const double m = s / count;
    double v = q / count - m * m;
    if (v < 0.0) v = 0.0;
    mean = (float)m;
    var = (float)v;
    const double unbiased = count > 1.0 ? v * count / (count - 1.0) : v;
    // yshift: the per-channel shift the conv epilogue subtracted before rounding (the statistics
    // and `mean` are those of the stored, shifted values, which is what apply / backward read);
    // the running mean gets the true mean. yshift may be rmean itself; a separate buffer (a fused
    // group's concatenated shifts) is advanced to the new running mean for the next step.
    const float sh = yshift != nullptr ? yshift[c] : 0.f;
    const float rm = (1.f - momentum) * rmean[c] + momentum * (mean + sh);
    rmean[c] = rm;
    if (yshift != nullptr && yshift != rmean) yshift[c] = rm;
    rvar[c] = (1.f - momentum) * rvar[c] + momentum * (float)unbiased;
  } else {
    mean = rmean[c];
    var = rvar[c];
  }
  const float invstd = rsqrtf(var + eps);
  const float sc = gamma[c] * invstd;
  out[c] = mean;
  out[C + c] = invstd;
  out[2 * C + c] = sc;
  out[3 * C + c] = beta[c] - mean * sc;
}

__global__ __launch_bounds__(FIN_CH * FIN_RG) void bn_finalize_kernel(
    const float* __restrict__ part, int nparts, int Npad, int C, double count, const float* __restrict__ gamma,
    const float* __restrict__ beta, float* rmean, float* __restrict__ rvar, long long* __restrict__ nbt,
    float momentum, float eps, int training, float* __restrict__ out /* [4][C]: mean, invstd, scale, shift */,
    float* yshift) {
  bn_finalize_body(blockIdx.x, part, nparts, Npad, C, count, gamma, beta, rmean, rvar, nbt, momentum, eps, training,
                   out, yshift);
}

// The BNs of a fused 1x1 group (members = channel slices [off, off + C) of one GEMM's
// statistics slab) finalized in one launch: block -> member by its first block.
struct FinMember {
  const float* gamma;
  const float* beta;
  float* rmean;
  float* rvar;
  long long* nbt;
  float* out;
  float* yshift;
  int off, C, blk0;
  float momentum, eps;
  int pad;
};
static_assert(sizeof(FinMember) == 80, "FinMember layout is mirrored by a ctypes.Structure");
constexpr int FIN_MAX_MEMBERS = 4;
struct FinGroup {
  FinMember m[FIN_MAX_MEMBERS];
  int n;
};

__global__ __launch_bounds__(FIN_CH * FIN_RG) void bn_finalize_group_kernel(FinGroup g, const float* __restrict__ part,
                                                                            int nparts, int Npad, double count,
                                                                            int training) {
  int i = 0;
  while (i + 1 < g.n && (int)blockIdx.x >= g.m[i + 1].blk0) ++i;
  const FinMember& m = g.m[i];
  bn_finalize_body(blockIdx.x - m.blk0, part + m.off, nparts, Npad, m.C, count, m.gamma, m.beta, m.rmean, m.rvar,
                   m.nbt, m.momentum, m.eps, training, m.out, training ? m.yshift : nullptr);
}

// ---------------------------------------------------------------------------------------
// z = relu(y*scale + shift). Grid (splits, B): block handles rows of one clip so the gating
// channel sums can be reduced in LDS and committed with one atomic per channel per block.
// WRITE = false (bn_relu_gsum_kernel): the SelfGating channel sums only, a read-only reduction
// (the lazy gate inputs' z is applied by the gate_scale pass / the consumer instead).
// MSTAT (bn_relu_gsum_mstat_kernel, with WRITE = false): also the per-clip mask statistics of this
// BN, mpart[split][b][2][C] = (sum mask, sum mask * y) (mask = y * scale + shift > 0, as the BN
// backward's; bn_mstat_sum_kernel turns the second into sum mask * xhat), which a gated pool's
// backward needs for its BN-backward partial sums (gated_pool_bn_partials_kernel).
template <bool WRITE, bool MSTAT = false>
__device__ __forceinline__ void bn_relu_apply_body(
    const bf16_t* __restrict__ y, int ldy, bf16_t* __restrict__ z, int ldz, const float* __restrict__ ss,
    int C, int rows_per_b, int rows_per_block, float* __restrict__ part, float* __restrict__ gsum,
    float* __restrict__ mpart = nullptr) {
  __shared__ float red[256 * 8];
  const int cpr = C >> 3;
  const int rpi = 256 / cpr;  // rows per iteration
  const int tid = threadIdx.x;
  const int cc = tid % cpr, rr = tid / cpr;
  const bool active = rr < rpi;
  const int b = blockIdx.y;
  const int r_begin = blockIdx.x * rows_per_block;
  const int r_end = min(rows_per_b, r_begin + rows_per_block);
  const int c0 = cc * 8;
  float sc[8], sh[8], acc[8];
  float m0[MSTAT ? 8 : 1], m1[MSTAT ? 8 : 1];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    sc[k] = active ? ss[2 * C + c0 + k] : 0.f;
    sh[k] = active ? ss[3 * C + c0 + k] : 0.f;
    acc[k] = 0.f;
    if constexpr (MSTAT) {
      m0[k] = 0.f;
      m1[k] = 0.f;
    }
  }
  if (active && r_begin + rr < r_end) {
    const long long base = (long long)b * rows_per_b;
    // BN_U rows in flight per thread: every load of a batch is issued before the first use (rows
    // past the end re-read the last row and are masked), so the wave is not one-load-at-a-time.
    for (int r0 = r_begin + rr; r0 < r_end; r0 += BN_U * rpi) {
      uint4 v[BN_U];
#pragma unroll
      for (int u = 0; u < BN_U; ++u)
        v[u] = *(const uint4*)(y + (base + min(r0 + u * rpi, r_end - 1)) * ldy + c0);
#pragma unroll
      for (int u = 0; u < BN_U; ++u) {
        const int r = r0 + u * rpi;
        if (r >= r_end) break;
        float f[8];
        unpack8(v[u], f);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          if constexpr (MSTAT) {  // sum mask and sum mask * y; xhat's affine map applied once at the end
            const bool m = f[k] * sc[k] + sh[k] > 0.f;
            m0[k] += m ? 1.f : 0.f;
            m1[k] += m ? f[k] : 0.f;
          }
          f[k] = fmaxf(f[k] * sc[k] + sh[k], 0.f);
          acc[k] += f[k];
        }
        if constexpr (WRITE) *(uint4*)(z + (base + r) * ldz + c0) = pack8(f);
      }
    }
  }
  if (gsum == nullptr) return;
#pragma unroll
  for (int k = 0; k < 8; ++k) red[k * 256 + tid] = acc[k];
  __syncthreads();
  // first row-group sums the others for its channel chunk; one partial row per (split, clip) in
  // part ([splits][B][C] scratch; bn_gsum_sum_kernel adds the splits in order), or -- inside a
  // HIP graph capture, part == null -- float atomics into gsum
  if (rr == 0 && active) {
    float* __restrict__ pr = part + ((long long)blockIdx.x * gridDim.y + b) * C + c0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float s = acc[k];
      for (int j = 1; j < rpi; ++j) s += red[k * 256 + j * cpr + cc];
      if (part != nullptr) pr[k] = s;
      else atomicAdd(gsum + (long long)b * C + c0 + k, s);
    }
  }
  if constexpr (MSTAT) {  // the mask sums the same way, one [2][C] row per (split, clip)
    float* __restrict__ mr = mpart + ((long long)blockIdx.x * gridDim.y + b) * 2 * C + c0;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      __syncthreads();  // red's previous readers are done
#pragma unroll
      for (int k = 0; k < 8; ++k) red[k * 256 + tid] = h == 0 ? m0[k] : m1[k];
      __syncthreads();
      if (rr == 0 && active) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          float v = h == 0 ? m0[k] : m1[k];
          for (int j = 1; j < rpi; ++j) v += red[k * 256 + j * cpr + cc];
          mr[h * C + k] = v;  // h = 1: sum mask * y (this row's part of sum mask * xhat, see below)
        }
      }
    }
  }
}

// gsum[i] (+)= sum over s < nsplit of part[s * n + i], in split order (deterministic gating sums);
// add = 0: overwrite
__global__ void bn_gsum_sum_kernel(float* __restrict__ gsum, const float* __restrict__ part, int nsplit, long long n,
                                   int add = 1) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    float v = part[i];
    for (int sp = 1; sp < nsplit; ++sp) v += part[(long long)sp * n + i];
    gsum[i] = add ? gsum[i] + v : v;
  }
}

__global__ __launch_bounds__(256) void bn_relu_apply_kernel(
    const bf16_t* __restrict__ y, int ldy, bf16_t* __restrict__ z, int ldz, const float* __restrict__ ss,
    int C, int rows_per_b, int rows_per_block, float* __restrict__ part, float* __restrict__ gsum) {
  bn_relu_apply_body<true>(y, ldy, z, ldz, ss, C, rows_per_b, rows_per_block, part, gsum);
}

__global__ __launch_bounds__(256) void bn_relu_gsum_kernel(
    const bf16_t* __restrict__ y, int ldy, const float* __restrict__ ss, int C, int rows_per_b,
    int rows_per_block, float* __restrict__ part, float* __restrict__ gsum) {
  bn_relu_apply_body<false>(y, ldy, nullptr, 0, ss, C, rows_per_b, rows_per_block, part, gsum);
}

__global__ __launch_bounds__(256) void bn_relu_gsum_mstat_kernel(
    const bf16_t* __restrict__ y, int ldy, const float* __restrict__ ss, int C, int rows_per_b,
    int rows_per_block, float* __restrict__ part, float* __restrict__ gsum, float* __restrict__ mpart) {
  bn_relu_apply_body<false, true>(y, ldy, nullptr, 0, ss, C, rows_per_b, rows_per_block, part, gsum, mpart);
}

// BN-backward partial sums of a SelfGating + TF-SAME max pool's input BN, taken over the POOLED
// tensors (hip_ops _GatedPool): the BN layer's dz = dx * g + dmean / thw, with dx the pool-routed
// gradient (nonzero only at arg-max cells), so
//   sum_cells dz mask (1, xhat) = sum_o dout_o g mask(yr_o) (1, xhat(yr_o)) + dmean / thw (S0, S1)
// where yr is the raw conv output at each output's arg-max (written by the pool forward) and S0 / S1
// the per-clip sums of mask and mask * xhat over all cells (mstat, from the forward's gating-sum
// pass) -- the full-resolution gather pass over dout, the arg-max codes and the raw conv output
// is not needed. (The per-cell dz of the old pass was rounded to bf16 before the sums; these sum
// its fp32 value.) Grid (splits, B): part[(split * B + b)][2][C]; split 0 adds the dmean term.
__global__ __launch_bounds__(256) void gated_pool_bn_partials_kernel(
    const bf16_t* __restrict__ dout, const bf16_t* __restrict__ yr, const float* __restrict__ g,
    const float* __restrict__ dmean, const float* __restrict__ ss, const float* __restrict__ mstat, int C,
    int rows_per_b, int rows_per_block, float inv_thw, float* __restrict__ part) {
  __shared__ float red[256 * 8];
  const int cpr = C >> 3, rpi = 256 / cpr;
  const int tid = threadIdx.x, cc = tid % cpr, rr = tid / cpr;
  const bool active = rr < rpi;
  const int b = blockIdx.y, c0 = cc * 8;
  const int r_begin = blockIdx.x * rows_per_block, r_end = min(rows_per_b, r_begin + rows_per_block);
  float gg[8], mu[8], is[8], sc[8], sh[8], a1[8], a2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int c = active ? c0 + k : 0;
    gg[k] = g[(long long)b * C + c];
    mu[k] = ss[c];
    is[k] = ss[C + c];
    sc[k] = ss[2 * C + c];
    sh[k] = ss[3 * C + c];
    a1[k] = 0.f;
    a2[k] = 0.f;
  }
  if (active && r_begin + rr < r_end) {
    const long long base = (long long)b * rows_per_b;
    for (int r0 = r_begin + rr; r0 < r_end; r0 += BN_U * rpi) {
      uint4 dv[BN_U], yv[BN_U];
#pragma unroll
      for (int u = 0; u < BN_U; ++u) {
        const long long row = base + min(r0 + u * rpi, r_end - 1);
        dv[u] = *(const uint4*)(dout + row * C + c0);
        yv[u] = *(const uint4*)(yr + row * C + c0);
      }
#pragma unroll
      for (int u = 0; u < BN_U; ++u) {
        if (r0 + u * rpi >= r_end) break;
        float d[8], v[8];
        unpack8(dv[u], d);
        unpack8(yv[u], v);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float gm = (v[k] * sc[k] + sh[k] > 0.f) ? d[k] * gg[k] : 0.f;
          a1[k] += gm;
          a2[k] += gm * (v[k] - mu[k]) * is[k];
        }
      }
    }
  }
  float* __restrict__ pr = part + ((long long)blockIdx.x * gridDim.y + b) * 2 * C + c0;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if (h) __syncthreads();
#pragma unroll
    for (int k = 0; k < 8; ++k) red[k * 256 + tid] = h == 0 ? a1[k] : a2[k];
    __syncthreads();
    if (rr == 0 && active) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float v = h == 0 ? a1[k] : a2[k];
        for (int j = 1; j < rpi; ++j) v += red[k * 256 + j * cpr + cc];
        if (blockIdx.x == 0) {
          const long long i = (long long)b * C + c0 + k;
          v += dmean[i] * inv_thw * mstat[((long long)b * 2 + h) * C + c0 + k];
        }
        pr[h * C + k] = v;
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// Per-channel partials of sum(dz*mask) and sum(dz*mask*xhat) -> part[blk][2][C]
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(
    const bf16_t* __restrict__ dz, int ldz, const bf16_t* __restrict__ y, int ldy,
    const float* __restrict__ ss, int C, long long M, int rows_per_block, float* __restrict__ part) {
  __shared__ float red[256 * 8];
  const int cpr = C >> 3;
  const int rpi = 256 / cpr;
  const int tid = threadIdx.x;
  const int cc = tid % cpr, rr = tid / cpr;
  const bool active = rr < rpi;
  const int c0 = cc * 8;
  const long long r_begin = (long long)blockIdx.x * rows_per_block;
  const long long r_end = min(M, r_begin + rows_per_block);
  float mean[8], istd[8], sc[8], sh[8], a1[8], a2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    mean[k] = active ? ss[c0 + k] : 0.f;
    istd[k] = active ? ss[C + c0 + k] : 0.f;
    sc[k] = active ? ss[2 * C + c0 + k] : 0.f;
    sh[k] = active ? ss[3 * C + c0 + k] : 0.f;
    a1[k] = 0.f;
    a2[k] = 0.f;
  }
  if (active) {
#pragma unroll 4
    for (long long r = r_begin + rr; r < r_end; r += rpi) {
      float g[8], v[8];
      unpack8(*(const uint4*)(dz + r * ldz + c0), g);
      unpack8(*(const uint4*)(y + r * ldy + c0), v);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float gm = (v[k] * sc[k] + sh[k] > 0.f) ? g[k] : 0.f;
        a1[k] += gm;
        a2[k] += gm * (v[k] - mean[k]) * istd[k];
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) red[k * 256 + tid] = a1[k];
  __syncthreads();
  if (rr == 0 && active) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float s = a1[k];
      for (int j = 1; j < rpi; ++j) s += red[k * 256 + j * cpr + cc];
      part[(long long)blockIdx.x * 2 * C + c0 + k] = s;
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 8; ++k) red[k * 256 + tid] = a2[k];
  __syncthreads();
  if (rr == 0 && active) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float s = a2[k];
      for (int j = 1; j < rpi; ++j) s += red[k * 256 + j * cpr + cc];
      part[(long long)blockIdx.x * 2 * C + C + c0 + k] = s;
    }
  }
}

// coef[3][C] = {k1 = gamma*invstd, dbeta/n, dgamma/n}; dgamma/dbeta written to the grads.
// part rows have stride 2*ps (ps = C for bn_bwd_reduce partials, Npad for conv-epilogue partials).
__device__ __forceinline__ void bn_bwd_finalize_body(int blk, const float* __restrict__ part, int nparts, int ps, int C,
                                                     double count, const float* __restrict__ gamma,
                                                     const float* __restrict__ ss, float* __restrict__ dgamma,
                                                     float* __restrict__ dbeta, float* __restrict__ coef,
                                                     int accumulate, int batch_stats);

__global__ __launch_bounds__(FIN_CH * FIN_RG) void bn_bwd_finalize_kernel(const float* __restrict__ part, int nparts, int ps,
                                                               int C, double count, const float* __restrict__ gamma,
                                                               const float* __restrict__ ss,
                                                               float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                               float* __restrict__ coef, int accumulate, int batch_stats) {
  bn_bwd_finalize_body(blockIdx.x, part, nparts, ps, C, count, gamma, ss, dgamma, dbeta, coef, accumulate,
                       batch_stats);
}

// The BN backwards of a fused 1x1 group's members (each with its own partial slab and
// parameters) finalized in one launch; each member's apply pass follows separately.
struct BwdFinMember {
  const float* part;
  const float* gamma;
  const float* ss;
  float* dgamma;
  float* dbeta;
  float* coef;
  int nparts, ps, C, blk0, accumulate, pad;
};
static_assert(sizeof(BwdFinMember) == 72, "BwdFinMember layout is mirrored by a ctypes.Structure");
struct BwdFinGroup {
  BwdFinMember m[FIN_MAX_MEMBERS];
  int n;
};

__global__ __launch_bounds__(FIN_CH * FIN_RG) void bn_bwd_finalize_group_kernel(BwdFinGroup g, double count,
                                                                                int batch_stats) {
  int i = 0;
  while (i + 1 < g.n && (int)blockIdx.x >= g.m[i + 1].blk0) ++i;
  const BwdFinMember& m = g.m[i];
  bn_bwd_finalize_body(blockIdx.x - m.blk0, m.part, m.nparts, m.ps, m.C, count, m.gamma, m.ss, m.dgamma, m.dbeta,
                       m.coef, m.accumulate, batch_stats);
}

__device__ __forceinline__ void bn_bwd_finalize_body(int blk, const float* __restrict__ part, int nparts, int ps, int C,
                                                     double count, const float* __restrict__ gamma,
                                                     const float* __restrict__ ss, float* __restrict__ dgamma,
                                                     float* __restrict__ dbeta, float* __restrict__ coef,
                                                     int accumulate, int batch_stats) {
  const int c = blk * FIN_CH + threadIdx.x % FIN_CH;
  double s1, s2;
  fin_reduce(part, nparts, ps, c, c < C, s1, s2);
  if (threadIdx.x >= FIN_CH || c >= C) return;
  // accumulate: dgamma/dbeta are the parameters' gradient buffers (written in place, += across
  // gradient-accumulation passes); otherwise fresh outputs
  dbeta[c] = accumulate ? dbeta[c] + (float)s1 : (float)s1;
  dgamma[c] = accumulate ? dgamma[c] + (float)s2 : (float)s2;
  coef[c] = gamma[c] * ss[C + c];
  // batch statistics (train mode): the mean/var depend on x, giving the two correction terms;
  // running statistics (eval mode): BN is a fixed affine map, dy = gamma * invstd * dz * mask
  coef[C + c] = batch_stats ? (float)(s1 / count) : 0.f;
  coef[2 * C + c] = batch_stats ? (float)(s2 / count) : 0.f;
}

// dy = coef0 * (dz*mask - coef1 - xhat*coef2). Each thread owns one 8-channel chunk (its
// per-channel constants live in registers) and walks rows [r_begin, r_end) of its block.
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(
    const bf16_t* __restrict__ dz, int ldz, const bf16_t* __restrict__ y, int ldy,
    const float* __restrict__ ss, const float* __restrict__ coef, int C, long long M, int rows_per_block,
    bf16_t* __restrict__ dy, int lddy) {
  const int cpr = C >> 3, rpi = 256 / cpr;
  const int cc = threadIdx.x % cpr, rr = threadIdx.x / cpr;
  if (rr >= rpi) return;
  const int c0 = cc * 8;
  BnBwdC q[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int c = c0 + k;
    q[k] = bn_bwd_const(ss[c], ss[C + c], ss[2 * C + c], ss[3 * C + c], coef[c], coef[C + c], coef[2 * C + c]);
  }
  const long long r_begin = (long long)blockIdx.x * rows_per_block;
  const long long r_end = min(M, r_begin + rows_per_block);
  if (r_begin + rr >= r_end) return;
  for (long long r0 = r_begin + rr; r0 < r_end; r0 += BN_U * rpi) {
    uint4 gv[BN_U], yv[BN_U];  // whole batch issued before the first use (see bn_relu_apply_kernel)
#pragma unroll
    for (int u = 0; u < BN_U; ++u) {
      const long long rc = min(r0 + u * rpi, r_end - 1);
      gv[u] = *(const uint4*)(dz + rc * ldz + c0);
      yv[u] = *(const uint4*)(y + rc * ldy + c0);
    }
#pragma unroll
    for (int u = 0; u < BN_U; ++u) {
      const long long r = r0 + u * rpi;
      if (r >= r_end) break;
      float g[8], v[8], o[8];
      unpack8(gv[u], g);
      unpack8(yv[u], v);
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = bn_bwd_elem(g[k], v[k], q[k]);
      *(uint4*)(dy + r * lddy + c0) = pack8(o);
    }
  }
}

// ---------------------------------------------------------------------------------------
MILNCE_API int milnce_bn_finalize(const float* part, int nparts, int Npad, int C, double count, const float* gamma,
                                  const float* beta, float* rmean, float* rvar, long long* nbt, float momentum,
                                  float eps, int training, float* out, float* yshift, hipStream_t stream) {
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + FIN_CH - 1) / FIN_CH), dim3(FIN_CH * FIN_RG), 0, stream, part,
                     nparts, Npad, C,
                     count, gamma, beta, rmean, rvar, nbt, momentum, eps, training, out, training ? yshift : nullptr);
  return (int)hipGetLastError();
}

// members: host array of n FinMember (off / C / gamma ... filled, blk0 computed here)
MILNCE_API int milnce_bn_finalize_group(const void* members, int n, const float* part, int nparts, int Npad,
                                        double count, int training, hipStream_t stream) {
  if (n < 1 || n > FIN_MAX_MEMBERS) return (int)hipErrorInvalidValue;
  FinGroup g;
  int blk = 0;
  for (int i = 0; i < n; ++i) {
    g.m[i] = ((const FinMember*)members)[i];
    g.m[i].blk0 = blk;
    blk += (g.m[i].C + FIN_CH - 1) / FIN_CH;
  }
  g.n = n;
  hipLaunchKernelGGL(bn_finalize_group_kernel, dim3(blk), dim3(FIN_CH * FIN_RG), 0, stream, g, part, nparts, Npad,
                     count, training);
  return (int)hipGetLastError();
}

static int pick_splits(long long rows, int target_rows) {
  long long s = (rows + target_rows - 1) / target_rows;
  return (int)(s < 1 ? 1 : s);
}

MILNCE_API int milnce_bn_relu_apply(const void* y, int ldy, void* z, int ldz, const float* ss, int C, int B,
                                    int rows_per_b, float* gsum, hipStream_t stream) {
  if (C % 8) return (int)hipErrorInvalidValue;
  // ~16 rows per thread (4 batches of BN_U): wide-C layers with few rows per clip (Mixed_4/5) get
  // enough blocks to fill 256 CUs instead of a couple of long serial blocks per CU.
  const int splits = pick_splits(rows_per_b, 4 * BN_U * (256 / (C / 8)));
  const int rpb = (rows_per_b + splits - 1) / splits;
  // gating sums: per-(split, clip) partial rows in scratch, then added to gsum in split order
  const long long n = (long long)B * C;
  float* part = nullptr;  // stays null inside a graph capture: atomics into gsum
  if (gsum != nullptr) part = stream_scratch((size_t)splits * n, stream, SCRATCH_BN_GSUM);
  if (z == nullptr) {  // gating sums only
    if (gsum == nullptr) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(bn_relu_gsum_kernel, dim3(splits, B), dim3(256), 0, stream, (const bf16_t*)y, ldy, ss, C,
                       rows_per_b, rpb, part, gsum);
  } else {
    hipLaunchKernelGGL(bn_relu_apply_kernel, dim3(splits, B), dim3(256), 0, stream, (const bf16_t*)y, ldy,
                       (bf16_t*)z, ldz, ss, C, rows_per_b, rpb, part, gsum);
  }
  if (part != nullptr) {
    const long long g = (n + 255) / 256;
    hipLaunchKernelGGL(bn_gsum_sum_kernel, dim3((int)(g < 4096 ? g : 4096)), dim3(256), 0, stream, gsum, part,
                       splits, n, 1);
  }
  return (int)hipGetLastError();
}

// mstat[b][0][c] = sum over splits of mpart's sum mask, mstat[b][1][c] = invstd * (sum mask * y -
// mean * sum mask) = sum mask * xhat (in split order)
__global__ void bn_mstat_sum_kernel(float* __restrict__ mstat, const float* __restrict__ mpart, int nsplit, int B,
                                    int C, const float* __restrict__ ss) {
  const long long n = (long long)B * C;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const long long b = i / C, c = i - b * C;
    float s0 = 0.f, s1 = 0.f;
    for (int sp = 0; sp < nsplit; ++sp) {
      const float* r = mpart + (((long long)sp * B + b) * 2) * C + c;
      s0 += r[0];
      s1 += r[C];
    }
    mstat[(b * 2) * C + c] = s0;
    mstat[(b * 2 + 1) * C + c] = ss[C + c] * (s1 - ss[c] * s0);
  }
}

// milnce_bn_relu_apply's gating-sums-only pass (z not written) that also leaves the per-clip mask
// statistics mstat [B][2][C] = (sum mask, sum mask * xhat) (overwritten); gsum [B][C] is added to.
// Not inside a HIP graph capture (the deterministic partial rows need the stream scratch).
MILNCE_API int milnce_bn_relu_gsum_mstat(const void* y, int ldy, const float* ss, int C, int B, int rows_per_b,
                                         float* gsum, float* mstat, hipStream_t stream) {
  if (C % 8 || C > 2048 || gsum == nullptr || mstat == nullptr) return (int)hipErrorInvalidValue;
  const int splits = pick_splits(rows_per_b, 4 * BN_U * (256 / (C / 8)));
  const int rpb = (rows_per_b + splits - 1) / splits;
  const long long n = (long long)B * C;
  float* part = stream_scratch((size_t)splits * n * 3, stream, SCRATCH_BN_GSUM);
  if (part == nullptr) return (int)hipErrorInvalidValue;
  float* mpart = part + (size_t)splits * n;
  hipLaunchKernelGGL(bn_relu_gsum_mstat_kernel, dim3(splits, B), dim3(256), 0, stream, (const bf16_t*)y, ldy, ss, C,
                     rows_per_b, rpb, part, gsum, mpart);
  long long g = (n + 255) / 256;
  hipLaunchKernelGGL(bn_gsum_sum_kernel, dim3((int)(g < 4096 ? g : 4096)), dim3(256), 0, stream, gsum, part, splits,
                     n, 1);
  hipLaunchKernelGGL(bn_mstat_sum_kernel, dim3((int)(g < 4096 ? g : 4096)), dim3(256), 0, stream, mstat, mpart,
                     splits, B, C, ss);
  return (int)hipGetLastError();
}

// BN-backward partials of a gated pool's input BN from the pooled side (gated_pool_bn_partials_kernel):
// dout / yr [B][rows_per_b][C] (pooled), g / dmean [B][C], ss [4][C], mstat [B][2][C], thw the
// full-resolution positions per clip; part [splits * B][2][C].
MILNCE_API int milnce_gated_pool_bn_partials(const void* dout, const void* yr, const float* g, const float* dmean,
                                             const float* ss, const float* mstat, int C, int B, int rows_per_b,
                                             int thw, int splits, float* part, hipStream_t stream) {
  if (C % 8 || C > 2048 || splits < 1 || rows_per_b < 1 || thw < 1) return (int)hipErrorInvalidValue;
  const int rpb = (rows_per_b + splits - 1) / splits;
  hipLaunchKernelGGL(gated_pool_bn_partials_kernel, dim3(splits, B), dim3(256), 0, stream, (const bf16_t*)dout,
                     (const bf16_t*)yr, g, dmean, ss, mstat, C, rows_per_b, rpb, 1.f / thw, part);
  return (int)hipGetLastError();
}

// part holds nparts rows of [2][ps] partial sums. have_part = 1: they were produced by the kernel
// that computed dz (conv dgrad epilogue, gate / pool backward), ps = that kernel's stride;
// have_part = 0: reduce them here (ps = C).
// ---------------------------------------------------------------------------------------
// Large BN-backward partial slabs (a dgrad epilogue's one row per M tile: up to ~40k rows x 64
// channels, 20 MB) are first summed over fixed row chunks by a full-chip pass; the finalize's
// C/8 workgroups alone stream such a slab latency-bound (0.7 ms on the conv_2b BN). Fixed
// chunks and a fixed-order lane sum keep the result deterministic. Out: [PRE_PARTS][2][ps].
constexpr int PRE_MIN_PARTS = 2048, PRE_PARTS = 512;

__global__ __launch_bounds__(256) void bn_part_prereduce_kernel(const float* __restrict__ part, int nparts, int ps,
                                                                int C, float* __restrict__ out) {
  __shared__ double red[256];
  const int ncol = 2 * C;
  const int width = ncol >= 256 ? 256 : ncol;
  const int lanes = 256 / width;  // rows in flight per column
  const int lane = threadIdx.x / width, tc = threadIdx.x % width;
  const int rpb = (nparts + gridDim.x - 1) / gridDim.x;
  const int r0 = blockIdx.x * rpb, r1 = min(nparts, r0 + rpb);
  for (int j0 = 0; j0 < ncol; j0 += width) {  // block-uniform
    const int j = j0 + tc;
    const int col = j < C ? j : ps + (j - C);
    double s0 = 0.0, s1 = 0.0;
    if (lane < lanes && j < ncol) {
      int r = r0 + lane;
      for (; r + lanes < r1; r += 2 * lanes) {
        s0 += (double)part[(long long)r * 2 * ps + col];
        s1 += (double)part[(long long)(r + lanes) * 2 * ps + col];
      }
      if (r < r1) s0 += (double)part[(long long)r * 2 * ps + col];
    }
    red[threadIdx.x] = s0 + s1;
    __syncthreads();
    if (lane == 0 && j < ncol) {
      double acc = 0.0;
      for (int l = 0; l < lanes; ++l) acc += red[l * width + tc];
      out[(long long)blockIdx.x * 2 * ps + col] = (float)acc;
    }
    __syncthreads();
  }
}

// Pre-reduces one slab into dst (PRE_PARTS x 2 x ps floats) when it is large; updates part /
// nparts to what the finalize should read.
static void prereduce(const float*& part, int& nparts, int ps, int C, float* dst, hipStream_t stream) {
  if (nparts < PRE_MIN_PARTS || dst == nullptr) return;
  hipLaunchKernelGGL(bn_part_prereduce_kernel, dim3(PRE_PARTS), dim3(256), 0, stream, part, nparts, ps, C, dst);
  part = dst;
  nparts = PRE_PARTS;
}

static void prereduce1(const float*& part, int& nparts, int ps, int C, hipStream_t stream) {
  if (nparts < PRE_MIN_PARTS) return;
  prereduce(part, nparts, ps, C, stream_scratch((size_t)PRE_PARTS * 2 * ps, stream, SCRATCH_BN_PRE), stream);
}

MILNCE_API int milnce_bn_bwd(const void* dz, int ldz, const void* y, int ldy, const float* ss, int C, long long M,
                             const float* gamma, float* part, int nparts, int ps, int have_part, float* dgamma,
                             float* dbeta, float* coef, void* dy, int lddy, int accumulate, int batch_stats,
                             hipStream_t stream) {
  if (C % 8) return (int)hipErrorInvalidValue;
  if (!have_part) {
    const int rows_per_block = (int)((M + nparts - 1) / nparts);
    hipLaunchKernelGGL(bn_bwd_reduce_kernel, dim3(nparts), dim3(256), 0, stream, (const bf16_t*)dz, ldz,
                       (const bf16_t*)y, ldy, ss, C, M, rows_per_block, part);
    ps = C;
  }
  const float* fpart = part;
  prereduce1(fpart, nparts, ps, C, stream);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + FIN_CH - 1) / FIN_CH), dim3(FIN_CH * FIN_RG), 0, stream,
                     fpart, nparts, ps, C,
                     (double)M, gamma, ss, dgamma, dbeta, coef, accumulate, batch_stats);
  const int rpi = 256 / (C / 8);
  long long nblk = (M + 16LL * rpi - 1) / (16LL * rpi);  // >= 16 rows per thread
  if (nblk > 8192) nblk = 8192;
  if (nblk < 1) nblk = 1;
  const int rpb = (int)((M + nblk - 1) / nblk);
  hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3((int)nblk), dim3(256), 0, stream, (const bf16_t*)dz, ldz,
                     (const bf16_t*)y, ldy, ss, coef, C, M, rpb, (bf16_t*)dy, lddy);
  return (int)hipGetLastError();
}

// BN-backward finalize only (dgamma, dbeta, coef from the partials) for consumers that apply the
// BN backward inside their own pass (pool.hip milnce_maxpool_bwd_apply).
MILNCE_API int milnce_bn_bwd_finalize(const float* part, int nparts, int ps, int C, double count,
                                      const float* gamma, const float* ss, float* dgamma, float* dbeta, float* coef,
                                      int accumulate, int batch_stats, hipStream_t stream) {
  prereduce1(part, nparts, ps, C, stream);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + FIN_CH - 1) / FIN_CH), dim3(FIN_CH * FIN_RG), 0, stream,
                     part, nparts, ps, C, count, gamma, ss, dgamma, dbeta, coef, accumulate, batch_stats);
  return (int)hipGetLastError();
}

// members: host array of n BwdFinMember (blk0 computed here); count = rows of the BN
MILNCE_API int milnce_bn_bwd_finalize_group(const void* members, int n, double count, int batch_stats,
                                            hipStream_t stream) {
  if (n < 1 || n > FIN_MAX_MEMBERS) return (int)hipErrorInvalidValue;
  BwdFinGroup g;
  int blk = 0;
  size_t need = 0;
  for (int i = 0; i < n; ++i) {
    g.m[i] = ((const BwdFinMember*)members)[i];
    g.m[i].blk0 = blk;
    blk += (g.m[i].C + FIN_CH - 1) / FIN_CH;
    if (g.m[i].nparts >= PRE_MIN_PARTS) need += (size_t)PRE_PARTS * 2 * g.m[i].ps;
  }
  g.n = n;
  if (need > 0) {  // each large member slab pre-reduced into its own region of the scratch
    float* dst = stream_scratch(need, stream, SCRATCH_BN_PRE);
    for (int i = 0; i < n && dst != nullptr; ++i) {
      if (g.m[i].nparts < PRE_MIN_PARTS) continue;
      prereduce(g.m[i].part, g.m[i].nparts, g.m[i].ps, g.m[i].C, dst, stream);
      dst += (size_t)PRE_PARTS * 2 * g.m[i].ps;
    }
  }
  hipLaunchKernelGGL(bn_bwd_finalize_group_kernel, dim3(blk), dim3(FIN_CH * FIN_RG), 0, stream, g, count,
                     batch_stats);
  return (int)hipGetLastError();
}

// milnce_bn_bwd's apply pass alone (coef already finalized, e.g. by milnce_bn_bwd_finalize_group)
MILNCE_API int milnce_bn_bwd_apply(const void* dz, int ldz, const void* y, int ldy, const float* ss, const float* coef,
                                   int C, long long M, void* dy, int lddy, hipStream_t stream) {
  if (C % 8) return (int)hipErrorInvalidValue;
  const int rpi = 256 / (C / 8);
  long long nblk = (M + 16LL * rpi - 1) / (16LL * rpi);
  if (nblk > 8192) nblk = 8192;
  if (nblk < 1) nblk = 1;
  const int rpb = (int)((M + nblk - 1) / nblk);
  hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3((int)nblk), dim3(256), 0, stream, (const bf16_t*)dz, ldz,
                     (const bf16_t*)y, ldy, ss, coef, C, M, rpb, (bf16_t*)dy, lddy);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// Lazy SelfGating gradient: the layer's dz is the gate backward's bf16(dout * g + dmean / thw)
// (gate.hip gate_bwd_apply_kernel produced the BN partials without storing dz); it is rebuilt here
// from dout. Grid (splits, B): g and dmean are per clip. dout / g / dmean point at the branch's
// first channel, with row strides ldo (dout) and ldg (g, dmean).
__global__ __launch_bounds__(256) void bn_bwd_apply_gate_kernel(
    const bf16_t* __restrict__ dout, int ldo, const float* __restrict__ g, const float* __restrict__ dmean, int ldg,
    float inv_thw, int thw, int rows_per_block, const bf16_t* __restrict__ y, int ldy,
    const float* __restrict__ ss, const float* __restrict__ coef, int C, bf16_t* __restrict__ dy, int lddy) {
  const int cpr = C >> 3, rpi = 256 / cpr;
  const int cc = threadIdx.x % cpr, rr = threadIdx.x / cpr;
  if (rr >= rpi) return;
  const int c0 = cc * 8, b = blockIdx.y;
  BnBwdC q[8];
  float gg[8], dm[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int c = c0 + k;
    q[k] = bn_bwd_const(ss[c], ss[C + c], ss[2 * C + c], ss[3 * C + c], coef[c], coef[C + c], coef[2 * C + c]);
    gg[k] = g[(size_t)b * ldg + c];
    dm[k] = dmean[(size_t)b * ldg + c] * inv_thw;
  }
  const int r_begin = blockIdx.x * rows_per_block, r_end = min(thw, r_begin + rows_per_block);
  const size_t row0 = (size_t)b * thw;
  if (r_begin + rr >= r_end) return;
  for (int r0 = r_begin + rr; r0 < r_end; r0 += BN_U * rpi) {
    uint4 dv[BN_U], yv[BN_U];  // whole batch issued before the first use (see bn_relu_apply_kernel)
#pragma unroll
    for (int u = 0; u < BN_U; ++u) {
      const size_t rc = row0 + min(r0 + u * rpi, r_end - 1);
      dv[u] = *(const uint4*)(dout + rc * ldo + c0);
      yv[u] = *(const uint4*)(y + rc * ldy + c0);
    }
#pragma unroll
    for (int u = 0; u < BN_U; ++u) {
      const int r = r0 + u * rpi;
      if (r >= r_end) break;
      const size_t row = row0 + r;
      float d[8], v[8], o[8];
      unpack8(dv[u], d);
      unpack8(yv[u], v);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float dz = bf2f(f2bf(fmaf(d[k], gg[k], dm[k])));  // the value gate_bwd_apply reduced
        o[k] = bn_bwd_elem(dz, v[k], q[k]);
      }
      *(uint4*)(dy + row * lddy + c0) = pack8(o);
    }
  }
}

// milnce_bn_bwd with a lazy SelfGating dz (see bn_bwd_apply_gate_kernel); the partials are required.
MILNCE_API int milnce_bn_bwd_gate(const void* dout, int ldo, const float* g, const float* dmean, int ldg, int B,
                                  int thw, const void* y, int ldy, const float* ss, int C, const float* gamma,
                                  float* part, int nparts, int ps, float* dgamma, float* dbeta, float* coef, void* dy,
                                  int lddy, int accumulate, int batch_stats, hipStream_t stream) {
  if (C % 8 || C > 2048) return (int)hipErrorInvalidValue;
  const float* fpart = part;
  prereduce1(fpart, nparts, ps, C, stream);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + FIN_CH - 1) / FIN_CH), dim3(FIN_CH * FIN_RG), 0, stream,
                     fpart, nparts, ps, C, (double)B * thw, gamma, ss, dgamma, dbeta, coef, accumulate, batch_stats);
  const int rpi = 256 / (C / 8);
  int splits = (thw + 16 * rpi - 1) / (16 * rpi);  // >= 16 rows per thread
  if (splits < 1) splits = 1;
  const int rpb = (thw + splits - 1) / splits;
  hipLaunchKernelGGL(bn_bwd_apply_gate_kernel, dim3(splits, B), dim3(256), 0, stream, (const bf16_t*)dout, ldo, g,
                     dmean, ldg, 1.f / thw, thw, rpb, (const bf16_t*)y, ldy, ss, coef, C, (bf16_t*)dy, lddy);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// The BN backward apply of every member of a fused 1x1 group (hip_ops _group_backward) in ONE pass
// over whole rows: y (the group GEMM's output, ctot channels) and dY (ditto) are read / written as
// contiguous rows instead of one c-channel slice per member launch (16-96 of 176-384 channels: 32-192
// B pieces of each row), and the members' dz come from their own sources -- a plain gradient tensor
// [M][c], or the SelfGating-lazy bf16(dout * g + dmean / thw) of bn_bwd_apply_gate_kernel (same
// arithmetic and roundings as the per-member kernels, so bitwise the same dY). Grid (splits, B): a
// block's rows lie in one clip (the gate constants are per clip).
struct GroupApplyMember {
  const bf16_t* dz;    // plain: [M][ldz]; lazy gate: the gate output gradient dout (+ channel offset)
  const float* g;      // lazy gate: g / dmean rows [B][ldg] (+ offset); null: plain
  const float* dmean;
  const float* ss;     // [4][c]: mean, invstd, scale, shift
  const float* coef;   // [3][c]
  int ldz, ldg, c0, c; // c0: first channel of the member in the group's rows
};
static_assert(sizeof(GroupApplyMember) == 56, "GroupApplyMember layout is mirrored by a ctypes.Structure");
struct GroupApply {
  GroupApplyMember m[FIN_MAX_MEMBERS];
  int n;
};

__global__ __launch_bounds__(256) void bn_bwd_apply_group_kernel(GroupApply ga, const bf16_t* __restrict__ y, int ctot,
                                                                 float inv_thw, int thw, int rows_per_block,
                                                                 bf16_t* __restrict__ dy) {
  const int cpr = ctot >> 3, rpi = 256 / cpr;
  const int cc = threadIdx.x % cpr, rr = threadIdx.x / cpr;
  if (rr >= rpi) return;
  const int ch0 = cc * 8, b = blockIdx.y;
  int mi = 0;
  while (mi + 1 < ga.n && ch0 >= ga.m[mi + 1].c0) ++mi;
  const GroupApplyMember& m = ga.m[mi];
  const int lc = ch0 - m.c0;  // channel within the member
  const bool lazy = m.g != nullptr;
  BnBwdC q[8];
  float gg[8], dm[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int c = lc + k;
    q[k] = bn_bwd_const(m.ss[c], m.ss[m.c + c], m.ss[2 * m.c + c], m.ss[3 * m.c + c], m.coef[c], m.coef[m.c + c],
                        m.coef[2 * m.c + c]);
    gg[k] = lazy ? m.g[(size_t)b * m.ldg + c] : 0.f;
    dm[k] = lazy ? m.dmean[(size_t)b * m.ldg + c] * inv_thw : 0.f;
  }
  const int r_begin = blockIdx.x * rows_per_block, r_end = min(thw, r_begin + rows_per_block);
  const size_t row0 = (size_t)b * thw;
  if (r_begin + rr >= r_end) return;
  for (int r0 = r_begin + rr; r0 < r_end; r0 += BN_U * rpi) {
    uint4 dv[BN_U], yv[BN_U];  // whole batch issued before the first use
#pragma unroll
    for (int u = 0; u < BN_U; ++u) {
      const size_t rc = row0 + min(r0 + u * rpi, r_end - 1);
      dv[u] = *(const uint4*)(m.dz + rc * m.ldz + lc);
      yv[u] = *(const uint4*)(y + rc * ctot + ch0);
    }
#pragma unroll
    for (int u = 0; u < BN_U; ++u) {
      const int r = r0 + u * rpi;
      if (r >= r_end) break;
      const size_t row = row0 + r;
      float d[8], v[8], o[8];
      unpack8(dv[u], d);
      unpack8(yv[u], v);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float dz = lazy ? bf2f(f2bf(fmaf(d[k], gg[k], dm[k]))) : d[k];
        o[k] = bn_bwd_elem(dz, v[k], q[k]);
      }
      *(uint4*)(dy + row * ctot + ch0) = pack8(o);
    }
  }
}

// members: host array of n GroupApplyMember (c0 ascending, covering [0, ctot) in multiples of 8)
MILNCE_API int milnce_bn_bwd_apply_group(const void* members, int n, const void* y, int ctot, int B, int thw,
                                         void* dy, hipStream_t stream) {
  if (n < 1 || n > FIN_MAX_MEMBERS || ctot % 8 || ctot > 2048) return (int)hipErrorInvalidValue;
  GroupApply ga;
  int c = 0;
  for (int i = 0; i < n; ++i) {
    ga.m[i] = ((const GroupApplyMember*)members)[i];
    if (ga.m[i].c0 != c || ga.m[i].c % 8) return (int)hipErrorInvalidValue;
    c += ga.m[i].c;
  }
  if (c != ctot) return (int)hipErrorInvalidValue;
  ga.n = n;
  const int rpi = 256 / (ctot / 8);
  int splits = (thw + 16 * rpi - 1) / (16 * rpi);  // >= 16 rows per thread
  if (splits < 1) splits = 1;
  const int rpb = (thw + splits - 1) / splits;
  hipLaunchKernelGGL(bn_bwd_apply_group_kernel, dim3(splits, B), dim3(256), 0, stream, ga, (const bf16_t*)y, ctot,
                     1.f / thw, thw, rpb, (bf16_t*)dy);
  return (int)hipGetLastError();
}

// milnce_bn_bwd_gate's apply pass alone (coef already finalized)
MILNCE_API int milnce_bn_bwd_gate_apply(const void* dout, int ldo, const float* g, const float* dmean, int ldg, int B,
                                        int thw, const void* y, int ldy, const float* ss, const float* coef, int C,
                                        void* dy, int lddy, hipStream_t stream) {
  if (C % 8 || C > 2048) return (int)hipErrorInvalidValue;
  const int rpi = 256 / (C / 8);
  int splits = (thw + 16 * rpi - 1) / (16 * rpi);
  if (splits < 1) splits = 1;
  const int rpb = (thw + splits - 1) / splits;
  hipLaunchKernelGGL(bn_bwd_apply_gate_kernel, dim3(splits, B), dim3(256), 0, stream, (const bf16_t*)dout, ldo, g,
                     dmean, ldg, 1.f / thw, thw, rpb, (const bf16_t*)y, ldy, ss, coef, C, (bf16_t*)dy, lddy);
  return (int)hipGetLastError();
}
