// SelfGating (s3dg.py:47-59) fused with the Inception channel concat (s3dg.py:45), plus the
// global average pool (s3dg.py:323).
//
// forward : the per-(clip, channel) sums of every branch come for free from the BN-apply
//           epilogue (bn.hip); gate_fc turns them into g = sigmoid(W * mean + b) (one block
//           per clip and branch), gate_scale writes z_i * g_i straight into its channel slice of
//           the concatenated block output (no separate th.cat pass).
// backward: gate_bwd_reduce  dpre[b, c] = (sum_thw dout * z) * g * (1 - g)   (all branches)
//           gate_fc_bwd      dmean = dpre W; dW += dpre^T mean; db += sum_b dpre (all branches)
//           gate_bwd_apply   dz_i = dout_i * g_i + dmean_i / THW              (all branches)
#include "common.h"

#define MAXSEG 4

struct SegTable {
  int nseg;
  int off[MAXSEG + 1];      // channel offsets in the concat row (off[nseg] = Ctot)
  const bf16_t* z[MAXSEG];  // branch activations [B*THW, C_i]
  bf16_t* dz[MAXSEG];       // branch grads (backward)
  const float* w[MAXSEG];   // fc weight [C_i, C_i]
  const float* bias[MAXSEG];
  float* dw[MAXSEG];
  float* db[MAXSEG];
  const bf16_t* bn_y[MAXSEG];   // producer BN raw output of each branch (backward partials), or null
  const float* bn_ss[MAXSEG];   // its [mean, invstd, scale, shift]
  int bn_ld[MAXSEG];            // row stride of bn_y
  int lazy[MAXSEG];             // forward: branch z not materialised, z = bf16(relu(bn_y*scale+shift))
};

__device__ __forceinline__ int seg_of(const SegTable& t, int c) {
  int s = 0;
#pragma unroll
  for (int k = 1; k < MAXSEG; ++k) s += (k < t.nseg && c >= t.off[k]) ? 1 : 0;
  return s;
}

// gsum/g/mean are [B, Ctot] fp32 (branch i at columns off[i]..off[i+1]).
// part != null: gsum[b, c] is first summed (in split order) from gate_gsum_kernel's nsplit partial
// rows [nsplit][B][Ctot] and stored.
__global__ void gate_fc_kernel(SegTable t, float* __restrict__ gsum, const float* __restrict__ part, int nsplit,
                               int B, float inv_thw, int Ctot, float* __restrict__ mean, float* __restrict__ g) {
  const int b = blockIdx.x, s = blockIdx.y;
  if (s >= t.nseg) return;
  const int c0 = t.off[s], C = t.off[s + 1] - c0;
  extern __shared__ float m[];
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const long long o = (long long)b * Ctot + c0 + c;
    float sum;
    if (part != nullptr) {
      sum = part[o];
      for (int sp = 1; sp < nsplit; ++sp) sum += part[(long long)sp * B * Ctot + o];
      gsum[o] = sum;
    } else {
      sum = gsum[o];
    }
    const float v = sum * inv_thw;
    m[c] = v;
    mean[o] = v;
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const float* wr = t.w[s] + (long long)c * C;
    float a = t.bias[s][c];
    for (int k = 0; k < C; ++k) a += wr[k] * m[k];
    g[(long long)b * Ctot + c0 + c] = 1.f / (1.f + __expf(-a));
  }
}

// out[row, c] = z_seg[row, c - off] * g[b, c]. Grid (splits, B): every thread owns one fixed
// 8-channel chunk of the concat row (its gate values are loaded once) and walks rows of clip b.
__global__ __launch_bounds__(256) void gate_scale_kernel(SegTable t, const float* __restrict__ g, int Ctot, int thw,
                                                         int rows_per_block, bf16_t* __restrict__ out) {
  const int cpr = Ctot >> 3, rpi = 256 / cpr, tid = threadIdx.x;
  const int cc = tid % cpr, rr = tid / cpr;
  if (rr >= rpi) return;
  const int c = cc * 8;
  const int s = seg_of(t, c);
  const int C = t.off[s + 1] - t.off[s], cl = c - t.off[s];
  const int b = blockIdx.y;
  float gg[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) gg[k] = g[(size_t)b * Ctot + c + k];
  const int r_begin = blockIdx.x * rows_per_block, r_end = min(thw, r_begin + rows_per_block);
  bf16_t* o = out + (size_t)b * thw * Ctot + c;
  if (t.lazy[s]) {
    // z = relu(y * scale + shift) rounded to bf16 (the value bn_relu_apply would have stored)
    float sc[8], sh[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) { sc[k] = t.bn_ss[s][2 * C + cl + k]; sh[k] = t.bn_ss[s][3 * C + cl + k]; }
    const bf16_t* ys = t.bn_y[s] + (size_t)b * thw * t.bn_ld[s] + cl;
#pragma unroll 4
    for (int r = r_begin + rr; r < r_end; r += rpi) {
      float f[8];
      unpack8(*(const uint4*)(ys + (size_t)r * t.bn_ld[s]), f);
#pragma unroll
      for (int k = 0; k < 8; ++k) f[k] = bf2f(f2bf(fmaxf(f[k] * sc[k] + sh[k], 0.f))) * gg[k];
      *(uint4*)(o + (size_t)r * Ctot) = pack8(f);
    }
    return;
  }
  const bf16_t* zs = t.z[s] + (size_t)b * thw * C + cl;
#pragma unroll 4
  for (int r = r_begin + rr; r < r_end; r += rpi) {
    float f[8];
    unpack8(*(const uint4*)(zs + (size_t)r * C), f);
#pragma unroll
    for (int k = 0; k < 8; ++k) f[k] *= gg[k];
    *(uint4*)(o + (size_t)r * Ctot) = pack8(f);
  }
}

// gsum[b, c] += sum over this block's rows of relu(y * scale + shift) for every (lazy) segment:
// the SelfGating input sums of all branches of an Inception block in one pass (bn.hip
// bn_relu_gsum_kernel per branch otherwise: four launches of a quarter of the work each, whose
// ramp / tail dominated the small Mixed_4 / Mixed_5 planes). Same per-element value as that kernel
// (fp32 relu before any bf16 rounding). Grid (splits, B); every thread owns one 8-channel chunk of
// the concat row and walks rows of clip b with BN_U loads in flight.
#ifndef MILNCE_GS_U
#define MILNCE_GS_U 4
#endif
constexpr int GS_U = MILNCE_GS_U;
__global__ __launch_bounds__(256) void gate_gsum_kernel(SegTable t, int Ctot, int thw, int rows_per_block,
                                                        float* __restrict__ part, float* __restrict__ gsum) {
  __shared__ float red[256 * 8];
  const int cpr = Ctot >> 3, rpi = 256 / cpr, tid = threadIdx.x;
  const int cc = tid % cpr, rr = tid / cpr;
  const bool active = rr < rpi;
  const int c = cc * 8;
  const int s = seg_of(t, active ? c : 0);
  const int C = t.off[s + 1] - t.off[s], cl = c - t.off[s];
  const int b = blockIdx.y;
  float sc[8], sh[8], acc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    sc[k] = active ? t.bn_ss[s][2 * C + cl + k] : 0.f;
    sh[k] = active ? t.bn_ss[s][3 * C + cl + k] : 0.f;
    acc[k] = 0.f;
  }
  const int r_begin = blockIdx.x * rows_per_block, r_end = min(thw, r_begin + rows_per_block);
  if (active && r_begin + rr < r_end) {
    const int ld = t.bn_ld[s];
    const bf16_t* ys = t.bn_y[s] + (size_t)b * thw * ld + cl;
    for (int r0 = r_begin + rr; r0 < r_end; r0 += GS_U * rpi) {
      uint4 v[GS_U];
#pragma unroll
      for (int u = 0; u < GS_U; ++u) v[u] = *(const uint4*)(ys + (size_t)min(r0 + u * rpi, r_end - 1) * ld);
#pragma unroll
      for (int u = 0; u < GS_U; ++u) {
        if (r0 + u * rpi >= r_end) break;
        float f[8];
        unpack8(v[u], f);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] += fmaxf(f[k] * sc[k] + sh[k], 0.f);
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) red[k * 256 + tid] = acc[k];
  __syncthreads();
  if (rr == 0 && active) {
    // one partial row per (split, clip): gate_fc_kernel sums the splits in a fixed order
    // (float atomics made the sums -- and the whole step -- differ run to run; they remain the
    // fallback inside a HIP graph capture, part == null)
    float* __restrict__ pr = part + ((size_t)blockIdx.x * gridDim.y + b) * Ctot + c;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float v = acc[k];
      for (int j = 1; j < rpi; ++j) v += red[k * 256 + j * cpr + cc];
      if (part != nullptr) pr[k] = v;
      else atomicAdd(gsum + (size_t)b * Ctot + c + k, v);
    }
  }
}

// part[split][b][c] = sum over this block's rows of dout[r, c] * z[r, c]   (grid: splits x B); the
// caller's next kernel sums the splits in a fixed order (deterministic, unlike float atomics)
__global__ __launch_bounds__(256) void gate_bwd_reduce_kernel(SegTable t, const bf16_t* __restrict__ dout,
                                                              int Ctot, int thw, int rows_per_block,
                                                              float* __restrict__ part, float* __restrict__ dg) {
  __shared__ float red[256 * 8];
  const int cpr = Ctot >> 3;
  const int tid = threadIdx.x;
  float acc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] = 0.f;
  const int b = blockIdx.y;
  const int r_begin = blockIdx.x * rows_per_block;
  const int r_end = min(thw, r_begin + rows_per_block);
  // threads sweep (row, chunk) pairs; each thread owns a fixed chunk when cpr divides 256,
  // otherwise chunks rotate -- accumulate per (chunk) through LDS at the end.
  const int groups = 256 / cpr;  // >= 1 since Ctot <= 2048
  const int cc = tid % cpr, rr = tid / cpr;
  const bool active = rr < groups;
  const int c = cc * 8;
  int s = 0, C = 0;
  if (active) { s = seg_of(t, c); C = t.off[s + 1] - t.off[s]; }
  if (active) {
    for (int r = r_begin + rr; r < r_end; r += groups) {
      const long long row = (long long)b * thw + r;
      float d[8], z[8];
      unpack8(*(const uint4*)(dout + row * Ctot + c), d);
      unpack8(*(const uint4*)(t.z[s] + row * C + (c - t.off[s])), z);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += d[k] * z[k];
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) red[k * 256 + tid] = acc[k];
  __syncthreads();
  if (active && rr == 0) {
    float* __restrict__ pr = part + ((long long)blockIdx.x * gridDim.y + b) * Ctot + c;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float v = acc[k];
      for (int j = 1; j < groups; ++j) v += red[k * 256 + j * cpr + cc];
      if (part != nullptr) pr[k] = v;
      else atomicAdd(dg + (long long)b * Ctot + c + k, v);  // graph-capture fallback
    }
  }
}

// dst[i] += sum over s < nsplit of part[s * n + i], in split order
__global__ void split_sum_kernel(float* __restrict__ dst, const float* __restrict__ part, int nsplit, long long n) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    float v = part[i];
    for (int sp = 1; sp < nsplit; ++sp) v += part[(long long)sp * n + i];
    dst[i] += v;
  }
}

// dpre = (dg + sum of the reduce's split rows, in split order) * g * (1 - g), in place (all segments
// at once: [B, Ctot])
__global__ void gate_dpre_kernel(float* __restrict__ dg, const float* __restrict__ part, int nsplit,
                                 const float* __restrict__ g, long long n) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    float v = 0.f;  // nsplit 0: the reduce added into dg itself
    for (int sp = 0; sp < nsplit; ++sp) v += part[(long long)sp * n + i];
    const float gg = g[i];
    dg[i] = (dg[i] + v) * gg * (1.f - gg);
  }
}

// dz_seg[r, c] = dout[r, c] * g[b, c] + dmean[b, c] * inv_thw.
// Grid (splits, B), each thread owns one fixed 8-channel chunk of the concat row, so when the
// branches carry producer-BN info the BN-backward partial sums of every branch's last BN layer
// (sum dz*mask, sum dz*mask*xhat) are produced here: part[b * splits + split][2][Ctot].
#ifndef MILNCE_GATE_U
#define MILNCE_GATE_U 4
#endif
constexpr int GATE_U = MILNCE_GATE_U;  // rows in flight per thread in gate_bwd_apply_kernel
__global__ __launch_bounds__(256) void gate_bwd_apply_kernel(SegTable t, const bf16_t* __restrict__ dout,
                                                             const float* __restrict__ g,
                                                             const float* __restrict__ dmean, int Ctot, int thw,
                                                             float inv_thw, int rows_per_block,
                                                             float* __restrict__ part) {
  __shared__ float red[256 * 8];
  const int cpr = Ctot >> 3, rpi = 256 / cpr, tid = threadIdx.x;
  const int cc = tid % cpr, rr = tid / cpr;
  const bool active = rr < rpi;
  const int c = cc * 8;
  const int s = active ? seg_of(t, c) : 0;
  const int C = t.off[s + 1] - t.off[s];
  const int cl = c - t.off[s];
  const bool bn = part != nullptr && t.bn_y[s] != nullptr;
  const int b = blockIdx.y;
  float mean[8], istd[8], sc[8], sh[8], a1[8], a2[8], gg[8], dm[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    mean[k] = bn && active ? t.bn_ss[s][cl + k] : 0.f;
    istd[k] = bn && active ? t.bn_ss[s][C + cl + k] : 0.f;
    sc[k] = bn && active ? t.bn_ss[s][2 * C + cl + k] : 0.f;
    sh[k] = bn && active ? t.bn_ss[s][3 * C + cl + k] : 0.f;
    gg[k] = active ? g[(size_t)b * Ctot + c + k] : 0.f;
    dm[k] = active ? dmean[(size_t)b * Ctot + c + k] * inv_thw : 0.f;
    a1[k] = 0.f;
    a2[k] = 0.f;
  }
  const int r_begin = blockIdx.x * rows_per_block, r_end = min(thw, r_begin + rows_per_block);
  if (active && r_begin + rr < r_end) {
    const size_t row0 = (size_t)b * thw;
    // dz == null: lazy gradient, rebuilt from dout by the BN backward (bn.hip milnce_bn_bwd_gate)
    bf16_t* const dzp = t.dz[s];
    const bf16_t* const yp = bn ? t.bn_y[s] : nullptr;
    const int yld = t.bn_ld[s];
    // GATE_U rows in flight per thread: the whole batch of loads is issued before the first use
    // (rows past the end re-read the last row and are masked).
    for (int r0 = r_begin + rr; r0 < r_end; r0 += GATE_U * rpi) {
      uint4 ov[GATE_U], yv[GATE_U];
#pragma unroll
      for (int u = 0; u < GATE_U; ++u) {
        const size_t rc = row0 + min(r0 + u * rpi, r_end - 1);
        ov[u] = *(const uint4*)(dout + rc * Ctot + c);
        if (bn) yv[u] = *(const uint4*)(yp + rc * yld + cl);
      }
#pragma unroll
      for (int u = 0; u < GATE_U; ++u) {
        const int r = r0 + u * rpi;
        if (r >= r_end) break;
        const size_t row = row0 + r;
        float d[8];
        unpack8(ov[u], d);
#pragma unroll
        for (int k = 0; k < 8; ++k) d[k] = fmaf(d[k], gg[k], dm[k]);
        const uint4 dv = pack8(d);
        if (dzp != nullptr) *(uint4*)(dzp + row * C + cl) = dv;
        if (bn) {
          float y[8], dr[8];
          unpack8(dv, dr);  // partials from the stored (bf16) gradient
          unpack8(yv[u], y);
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const float gm = (y[k] * sc[k] + sh[k] > 0.f) ? dr[k] : 0.f;
            a1[k] += gm;
            a2[k] += gm * (y[k] - mean[k]) * istd[k];
          }
        }
      }
    }
  }
  if (part == nullptr) return;
  const size_t prow = (size_t)blockIdx.y * gridDim.x + blockIdx.x;
#pragma unroll
  for (int k = 0; k < 8; ++k) red[k * 256 + tid] = a1[k];
  __syncthreads();
  if (rr == 0 && active) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float v = a1[k];
      for (int j = 1; j < rpi; ++j) v += red[k * 256 + j * cpr + cc];
      part[prow * 2 * Ctot + c + k] = v;
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 8; ++k) red[k * 256 + tid] = a2[k];
  __syncthreads();
  if (rr == 0 && active) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float v = a2[k];
      for (int j = 1; j < rpi; ++j) v += red[k * 256 + j * cpr + cc];
      part[prow * 2 * Ctot + Ctot + c + k] = v;
    }
  }
}

// ---------------------------------------------------------------------------------------
// global average pool over THW: x [B*THW, C] bf16 -> out [B, C] fp32 (atomics into zeroed out)
__global__ __launch_bounds__(256) void avgpool_kernel(const bf16_t* __restrict__ x, int C, int thw,
                                                      int rows_per_block, float inv, float* __restrict__ out) {
  __shared__ float red[256 * 8];
  const int cpr = C >> 3, groups = 256 / cpr, tid = threadIdx.x;
  const int cc = tid % cpr, rr = tid / cpr;
  const bool active = rr < groups;
  const int b = blockIdx.y;
  const int r_begin = blockIdx.x * rows_per_block, r_end = min(thw, r_begin + rows_per_block);
  float acc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] = 0.f;
  if (active) {
    for (int r = r_begin + rr; r < r_end; r += groups) {
      float f[8];
      unpack8(*(const uint4*)(x + ((long long)b * thw + r) * C + cc * 8), f);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += f[k];
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) red[k * 256 + tid] = acc[k];
  __syncthreads();
  if (active && rr == 0) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float v = acc[k];
      for (int j = 1; j < groups; ++j) v += red[k * 256 + j * cpr + cc];
      atomicAdd(out + (long long)b * C + cc * 8 + k, v * inv);
    }
  }
}

__global__ void avgpool_bwd_kernel(const float* __restrict__ dout, int C, int thw, long long rows, float inv,
                                   bf16_t* __restrict__ dx) {
  const int cpr = C >> 3;
  const long long n = rows * cpr;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / cpr;
    const int c = (int)(i - r * cpr) * 8;
    const int b = (int)(r / thw);
    float f[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) f[k] = dout[(long long)b * C + c + k] * inv;
    *(uint4*)(dx + r * C + c) = pack8(f);
  }
}


// SelfGating fc backward of every branch in one launch (replaces 3 hipBLASLt GEMMs, a reduction,
// a copy and two AccumulateGrad adds per branch). dpre[b, c] = src[b, c] * (g ? 1 - g[b, c] : 1)
// (src = g * sum_thw dout * z when g is given, else the finished dpre). Blocks [0, wend) compute
// dW[co, ci] = sum_b dpre[b, co] * mean[b, ci] and db[co] = sum_b dpre[b, co] on 16 co x 64 ci
// tiles (the tile's dpre columns staged in LDS); blocks [wend, ...) compute dmean[b, ci] =
// sum_co dpre[b, co] * W[co, ci] on 16 b x 64 ci tiles (the 16 dpre rows staged in LDS). Each
// wave owns 4 rows of its tile, so the LDS reads are wave-uniform broadcasts. Bit s of acc_mask:
// accumulate into dw[s] / db[s] (a flat data-parallel gradient buffer) instead of storing.
struct FcTiles {
  int wstart[MAXSEG + 1];
  int mstart[MAXSEG + 1];
};

__global__ __launch_bounds__(256) void gate_fc_bwd_kernel(SegTable t, FcTiles ft, const float* __restrict__ src,
                                                          const float* __restrict__ g,
                                                          const float* __restrict__ mean, int B, int Ctot,
                                                          int acc_mask, float* __restrict__ dmean) {
  extern __shared__ float sd[];
  int tile = blockIdx.x;
  const bool wpart = tile < ft.wstart[t.nseg];
  int s = 0;
  if (wpart) {
    while (tile >= ft.wstart[s + 1]) ++s;
    tile -= ft.wstart[s];
  } else {
    tile -= ft.wstart[t.nseg];
    while (tile >= ft.mstart[s + 1]) ++s;
    tile -= ft.mstart[s];
  }
  const int c0 = t.off[s], C = t.off[s + 1] - c0;
  const int nci = (C + 63) / 64;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int ci = (tile % nci) * 64 + lane;
  const bool cv = ci < C;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  if (wpart) {
    const int co0 = (tile / nci) * 16;
    for (int i = threadIdx.x; i < B * 16; i += 256) {
      const int b = i >> 4, co = co0 + (i & 15);
      float v = 0.f;
      if (co < C) {
        const long long k = (long long)b * Ctot + c0 + co;
        v = src[k];
        if (g != nullptr) v *= 1.f - g[k];
      }
      sd[i] = v;
    }
    __syncthreads();
    float dbs[4] = {0.f, 0.f, 0.f, 0.f};
    const float* mp = mean + c0 + (cv ? ci : 0);
    for (int b = 0; b < B; ++b) {
      const float m = mp[(long long)b * Ctot];
      const float4 d = *(const float4*)&sd[b * 16 + wv * 4];
      acc[0] += d.x * m;
      acc[1] += d.y * m;
      acc[2] += d.z * m;
      acc[3] += d.w * m;
      dbs[0] += d.x;
      dbs[1] += d.y;
      dbs[2] += d.z;
      dbs[3] += d.w;
    }
    const bool accum = (acc_mask >> s) & 1;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int co = co0 + wv * 4 + j;
      if (co >= C) continue;
      if (cv) {
        float* p = t.dw[s] + (long long)co * C + ci;
        *p = accum ? *p + acc[j] : acc[j];
      }
      if (tile % nci == 0 && lane == 0) {
        float* p = t.db[s] + co;
        *p = accum ? *p + dbs[j] : dbs[j];
      }
    }
  } else {
    const int b0 = (tile / nci) * 16;
    for (int i = threadIdx.x; i < 16 * C; i += 256) {
      const int j = i / C, co = i - j * C, b = b0 + j;
      float v = 0.f;
      if (b < B) {
        const long long k = (long long)b * Ctot + c0 + co;
        v = src[k];
        if (g != nullptr) v *= 1.f - g[k];
      }
      sd[i] = v;
    }
    __syncthreads();
    const float* wp = t.w[s] + (cv ? ci : 0);
    const float* r = sd + wv * 4 * C;
    for (int co = 0; co < C; ++co) {
      const float w = wp[(long long)co * C];
      acc[0] += r[co] * w;
      acc[1] += r[C + co] * w;
      acc[2] += r[2 * C + co] * w;
      acc[3] += r[3 * C + co] * w;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int b = b0 + wv * 4 + j;
      if (b < B && cv) dmean[(long long)b * Ctot + c0 + ci] = acc[j];
    }
  }
}

// ---------------------------------------------------------------------------------------
static SegTable make_table(int nseg, const int* widths, const void* const* z, void* const* dz,
                           const float* const* w, const float* const* bias, float* const* dw, float* const* db) {
  SegTable t;
  t.nseg = nseg;
  t.off[0] = 0;
  for (int i = 0; i < MAXSEG; ++i) {
    const bool v = i < nseg;
    t.off[i + 1] = t.off[i] + (v ? widths[i] : 0);
    t.z[i] = v && z ? (const bf16_t*)z[i] : nullptr;
    t.dz[i] = v && dz ? (bf16_t*)dz[i] : nullptr;
    t.w[i] = v && w ? w[i] : nullptr;
    t.bias[i] = v && bias ? bias[i] : nullptr;
    t.dw[i] = v && dw ? dw[i] : nullptr;
    t.db[i] = v && db ? db[i] : nullptr;
    t.bn_y[i] = nullptr;
    t.bn_ss[i] = nullptr;
    t.bn_ld[i] = 0;
    t.lazy[i] = 0;
  }
  return t;
}

static int grid_for(long long n) {
  long long g = (n + 255) / 256;
  return (int)(g > 8192 ? 8192 : (g < 1 ? 1 : g));
}

// lazy (may be null): per-branch flag; a lazy branch's z is read as relu(bn_y * scale + shift)
// from (bn_y[i], bn_ld[i], bn_ss[i]) instead of z[i].
// gsum_pass != 0: gsum (zeroed by the caller) is first computed by ONE gate_gsum_kernel pass over
// every branch's raw conv output (all branches must be lazy).
MILNCE_API int milnce_gate_fwd(int nseg, const int* widths, const void* const* z, const float* const* w,
                               const float* const* bias, float* gsum, int B, int thw, float* mean, float* g,
                               void* out, const int* lazy, const void* const* bn_y, const float* const* bn_ss,
                               const int* bn_ld, int gsum_pass, hipStream_t stream) {
  SegTable t = make_table(nseg, widths, z, nullptr, w, bias, nullptr, nullptr);
  for (int i = 0; i < nseg && lazy != nullptr; ++i) {
    t.lazy[i] = lazy[i];
    if (lazy[i]) {
      t.bn_y[i] = (const bf16_t*)bn_y[i];
      t.bn_ss[i] = bn_ss[i];
      t.bn_ld[i] = bn_ld[i];
    }
  }
  const int Ctot = t.off[nseg];
  float* gpart = nullptr;  // gsum_pass: the gsum kernel's partial rows
  int nsplit = 0;
  if (gsum_pass) {
    for (int i = 0; i < nseg; ++i)
      if (lazy == nullptr || !lazy[i]) return (int)hipErrorInvalidValue;
    if (Ctot % 8 || Ctot > 2048) return (int)hipErrorInvalidValue;
    // >= ~4 workgroups per CU over the batch, >= 16 row iterations per thread
    const int rpi = 256 / (Ctot / 8);
    int splits = (1024 + B - 1) / B;
    const int smax = (thw + 16 * rpi - 1) / (16 * rpi);
    if (splits > smax) splits = smax;
    if (splits < 1) splits = 1;
    const int rpb = (thw + splits - 1) / splits;
    gpart = stream_scratch((size_t)splits * B * Ctot, stream, SCRATCH_GATE_GSUM);  // null: atomics into gsum
    nsplit = gpart != nullptr ? splits : 0;
    hipLaunchKernelGGL(gate_gsum_kernel, dim3(splits, B), dim3(256), 0, stream, t, Ctot, thw, rpb, gpart, gsum);
  }
  int cmax = 0;
  for (int i = 0; i < nseg; ++i) cmax = widths[i] > cmax ? widths[i] : cmax;
  hipLaunchKernelGGL(gate_fc_kernel, dim3(B, nseg), dim3(256), cmax * sizeof(float), stream, t, gsum, gpart,
                     nsplit, B, 1.f / thw, Ctot, mean, g);
  if (out == nullptr) return (int)hipGetLastError();  // gate values only: a fused consumer applies them
  if (Ctot % 8 || Ctot > 2048) return (int)hipErrorInvalidValue;
  const int rpi = 256 / (Ctot / 8);
  const int splits = (thw + 32 * rpi - 1) / (32 * rpi);  // >= 32 row iterations per thread
  const int rpb = (thw + splits - 1) / splits;
  hipLaunchKernelGGL(gate_scale_kernel, dim3(splits, B), dim3(256), 0, stream, t, g, Ctot, thw, rpb,
                     (bf16_t*)out);
  return (int)hipGetLastError();
}

// Phase 1: dpre[B, Ctot] = (sum_thw dout * z) * g * (1 - g)   (dpre zeroed by the caller).
// The per-branch fc backward (milnce_gate_fc_bwd) runs in between.
MILNCE_API int milnce_gate_bwd_reduce(int nseg, const int* widths, const void* const* z, const void* dout,
                                      const float* g, int B, int thw, float* dpre, hipStream_t stream) {
  SegTable t = make_table(nseg, widths, z, nullptr, nullptr, nullptr, nullptr, nullptr);
  const int Ctot = t.off[nseg];
  const int splits = (thw + 511) / 512;
  const int rpb = (thw + splits - 1) / splits;
  const long long n = (long long)B * Ctot;
  float* part = stream_scratch((size_t)splits * n, stream, SCRATCH_GATE_DG);  // null: atomics into dpre
  hipLaunchKernelGGL(gate_bwd_reduce_kernel, dim3(splits, B), dim3(256), 0, stream, t, (const bf16_t*)dout, Ctot,
                     thw, rpb, part, dpre);
  hipLaunchKernelGGL(gate_dpre_kernel, dim3(grid_for(n)), dim3(256), 0, stream, dpre, part,
                     part != nullptr ? splits : 0, g, n);
  return (int)hipGetLastError();
}

// The SelfGating fc backward of all nseg branches (gate_fc_bwd_kernel): dw[i], db[i] (accumulated
// where bit i of acc_mask is set) and dmean [B, Ctot]. Returns hipErrorInvalidValue for shapes
// whose LDS staging would not fit (the caller then falls back to library GEMMs).
MILNCE_API int milnce_gate_fc_bwd(int nseg, const int* widths, const float* src, const float* g, const float* mean,
                                  const float* const* w, float* const* dw, float* const* db, int acc_mask, int B,
                                  float* dmean, hipStream_t stream) {
  SegTable t = make_table(nseg, widths, nullptr, nullptr, w, nullptr, dw, db);
  const int Ctot = t.off[nseg];
  FcTiles ft;
  ft.wstart[0] = ft.mstart[0] = 0;
  int cmax = 0;
  for (int i = 0; i < MAXSEG; ++i) {
    const int C = i < nseg ? widths[i] : 0;
    cmax = C > cmax ? C : cmax;
    const int nci = (C + 63) / 64;
    ft.wstart[i + 1] = ft.wstart[i] + nci * ((C + 15) / 16);
    ft.mstart[i + 1] = ft.mstart[i] + nci * ((B + 15) / 16);
  }
  const size_t lds = sizeof(float) * 16 * (size_t)(B > cmax ? B : cmax);
  if (nseg < 1 || nseg > MAXSEG || B < 1 || lds > 64 * 1024) return (int)hipErrorInvalidValue;
  const int grid = ft.wstart[nseg] + ft.mstart[nseg];
  hipLaunchKernelGGL(gate_fc_bwd_kernel, dim3(grid), dim3(256), lds, stream, t, ft, src, g, mean, B, Ctot, acc_mask,
                     dmean);
  return (int)hipGetLastError();
}

// Phase 2: dz_i = dout_i * g_i + dmean_i / THW, plus (part != null) the producer-BN partials of
// every branch whose bn_y[i] is given: nparts = B * splits, part must hold nparts * 2 * Ctot floats.
MILNCE_API int milnce_gate_bwd_apply(int nseg, const int* widths, void* const* dz, const void* dout, const float* g,
                                     const float* dmean, int B, int thw, const void* const* bn_y,
                                     const float* const* bn_ss, const int* bn_ld, float* part, int nparts,
                                     hipStream_t stream) {
  SegTable t = make_table(nseg, widths, nullptr, dz, nullptr, nullptr, nullptr, nullptr);
  for (int i = 0; i < nseg; ++i) {
    t.bn_y[i] = bn_y ? (const bf16_t*)bn_y[i] : nullptr;
    t.bn_ss[i] = bn_ss ? bn_ss[i] : nullptr;
    t.bn_ld[i] = bn_ld ? bn_ld[i] : widths[i];
  }
  const int Ctot = t.off[nseg];
  if (Ctot % 8 || Ctot > 2048) return (int)hipErrorInvalidValue;
  if (nparts % B) return (int)hipErrorInvalidValue;  // nparts = B * splits
  const int splits = nparts / B;
  const int rpb = (thw + splits - 1) / splits;
  hipLaunchKernelGGL(gate_bwd_apply_kernel, dim3(splits, B), dim3(256), 0, stream, t, (const bf16_t*)dout, g, dmean,
                     Ctot, thw, 1.f / thw, rpb, part);
  return (int)hipGetLastError();
}

// gs[b, c] += sum over the clip's rows of a[row, c] * v[row, c]  (a, v: [B * rows_per_b, C] bf16; gs
// zeroed by the caller): the SelfGating reduction taken on a pooled gate output (hip_ops._GatedPool).
MILNCE_API int milnce_gate_dot(const void* a, const void* v, int B, int rows_per_b, int C, float* gs,
                               hipStream_t stream) {
  if (C % 8 || C > 2048) return (int)hipErrorInvalidValue;
  const int widths[1] = {C};
  const void* zs[1] = {v};
  SegTable t = make_table(1, widths, zs, nullptr, nullptr, nullptr, nullptr, nullptr);
  const int splits = (rows_per_b + 511) / 512;
  const int rpb = (rows_per_b + splits - 1) / splits;
  const long long n = (long long)B * C;
  float* part = stream_scratch((size_t)splits * n, stream, SCRATCH_GATE_DOT);  // null: atomics into gs
  hipLaunchKernelGGL(gate_bwd_reduce_kernel, dim3(splits, B), dim3(256), 0, stream, t, (const bf16_t*)a, C,
                     rows_per_b, rpb, part, gs);
  if (part != nullptr)
    hipLaunchKernelGGL(split_sum_kernel, dim3(grid_for(n)), dim3(256), 0, stream, gs, part, splits, n);
  return (int)hipGetLastError();
}

MILNCE_API int milnce_avgpool(const void* x, int B, int thw, int C, float* out, hipStream_t stream) {
  const int splits = (thw + 255) / 256;
  const int rpb = (thw + splits - 1) / splits;
  hipLaunchKernelGGL(avgpool_kernel, dim3(splits, B), dim3(256), 0, stream, (const bf16_t*)x, C, thw, rpb,
                     1.f / thw, out);
  return (int)hipGetLastError();
}

MILNCE_API int milnce_avgpool_bwd(const float* dout, int B, int thw, int C, void* dx, hipStream_t stream) {
  const long long rows = (long long)B * thw;
  hipLaunchKernelGGL(avgpool_bwd_kernel, dim3(grid_for(rows * (C / 8))), dim3(256), 0, stream, dout, C, thw, rows,
                     1.f / thw, (bf16_t*)dx);
  return (int)hipGetLastError();
}
