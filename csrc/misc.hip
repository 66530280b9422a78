// Small fused kernels around the model:
//   * fused Adam over the flat fp32 parameter / moment buffers (one launch for all params,
//     all-reduce scale folded in), torch.optim.Adam arithmetic;
//   * on-device synthetic clip generator (uint8 NDHWC4), bit-compatible with data/synthetic.py;
//   * stem input conversion from the reference clip layout [B,3,T,H,W] (uint8 or float in
//     [0,1]) to the stem's [B,T,H,W,4] operand layout;
//   * text tower ReLU + max-over-words (s3dg.py:201-202) with arg-max for the backward.
#include "common.h"

__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v, long long n,
                                                   float lr, float b1, float b2, float eps, float wd, float bc1,
                                                   float sqrt_bc2, float gscale) {
  const long long n4 = n >> 2;
  const float step = lr / bc1;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4;
       i += (long long)gridDim.x * blockDim.x) {
    float4 pp = ((float4*)p)[i], gg = ((const float4*)g)[i], mm = ((float4*)m)[i], vv = ((float4*)v)[i];
    float* pa = (float*)&pp; float* ga = (float*)&gg; float* ma = (float*)&mm; float* va = (float*)&vv;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float gk = ga[k] * gscale;
      if (wd != 0.f) gk += wd * pa[k];
      ma[k] = b1 * ma[k] + (1.f - b1) * gk;
      va[k] = b2 * va[k] + (1.f - b2) * gk * gk;
      const float denom = sqrtf(va[k]) / sqrt_bc2 + eps;
      pa[k] -= step * ma[k] / denom;
    }
    ((float4*)p)[i] = pp; ((float4*)m)[i] = mm; ((float4*)v)[i] = vv;
  }
  // tail
  const long long t = (n4 << 2) + blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (blockIdx.x == 0 && t < n && threadIdx.x < 4) {
    float gk = g[t] * gscale;
    if (wd != 0.f) gk += wd * p[t];
    m[t] = b1 * m[t] + (1.f - b1) * gk;
    v[t] = b2 * v[t] + (1.f - b2) * gk * gk;
    p[t] -= step * m[t] / (sqrtf(v[t]) / sqrt_bc2 + eps);
  }
}

MILNCE_API int milnce_adam(float* p, const float* g, float* m, float* v, long long n, float lr, float b1, float b2,
                           float eps, float wd, float bc1, float bc2, float gscale, hipStream_t stream) {
  long long grid = ((n >> 2) + 255) / 256;
  if (grid > 4096) grid = 4096;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(adam_kernel, dim3((int)grid), dim3(256), 0, stream, p, g, m, v, n, lr, b1, b2, eps, wd, bc1,
                     sqrtf(bc2), gscale);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x = ((x >> 16) ^ x) * 0x45d9f3bu;
  x = ((x >> 16) ^ x) * 0x45d9f3bu;
  return ((x >> 16) ^ x) & 0x7fffffffu;
}

// One wave per (b, t, y) image row, 4 pixels (16 B) per lane: the label-dependent
// constants are per row, index math is 32-bit, and the three channel waves use the hardware
// sine (the torch reference in data/synthetic.py agrees to +-1 grey level).
__global__ __launch_bounds__(256) void synth_video_kernel(const int* __restrict__ labels, const int* __restrict__ ids,
                                                          int T, int S, uint32_t* __restrict__ out, long long nrows) {
  const int q = S >> 2;  // 4-pixel quads per row (S % 4 == 0)
  for (long long row = blockIdx.x; row < nrows; row += gridDim.x) {
    const int y = (int)(row % S);
    const int bt = (int)(row / S);
    const int t = bt % T, b = bt / T;
    const float lab = (float)labels[b];
    const float freq = 0.05f + 0.01f * fmodf(lab, 7.f);
    const float drift = 0.5f + 0.25f * fmodf(lab, 5.f);
    const uint32_t id = (uint32_t)ids[b] * 65537u;
    float color[3], ph[3];
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
      color[ch] = 64.f + 48.f * fmodf(lab * 3.f + ch * 5.f, 4.f);
      ph[ch] = (float)y * (1.f + 0.1f * ch);
    }
    uint32_t* orow = out + row * S;
    for (int x0 = threadIdx.x * 4; x0 < S; x0 += blockDim.x * 4) {
      uint32_t px[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int x = x0 + j;
        const uint32_t h = mix32(id + ((uint32_t)t * S + y) * S + x);
        const float noise = (float)(h % 64u) - 32.f;
        uint32_t v4 = 0;
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) {
          const float wave = __sinf(freq * ((float)x + ph[ch]) + drift * (float)t);
          float v = color[ch] + 60.f * wave + noise;
          v = fminf(fmaxf(v, 0.f), 255.f);
          v4 |= ((uint32_t)v & 0xffu) << (8 * ch);
        }
        px[j] = v4;
      }
      if ((S & 3) == 0) {
        *(uint4*)(orow + x0) = make_uint4(px[0], px[1], px[2], px[3]);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (x0 + j < S) orow[x0 + j] = px[j];
      }
    }
  }
}

// Per-sample metadata of a synthetic batch (data/synthetic.py SyntheticClips.labels / .text), one
// thread per caption word: sample id = base + b, its latent class and the K x W caption tokens
// (class-carrying leading words, hashed random words after), plus the int32 label / id rows the
// video kernel reads. Replaces ~40 small int64 elementwise launches per step.
__global__ __launch_bounds__(256) void synth_meta_kernel(long long base, int B, int K, int W, int vocab, int ncls,
                                                         int seed, int class_words, long long* __restrict__ tok,
                                                         long long* __restrict__ labels64, int* __restrict__ labels32,
                                                         int* __restrict__ ids32) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * K * W) return;
  const int w = i % W, k = (i / W) % K, b = i / (W * K);
  const long long id = base + b;
  const uint32_t lab = mix32((uint32_t)(id * 7919 + seed)) % (uint32_t)ncls;
  const uint32_t h = mix32((uint32_t)(id * 1000003 + k * 8191 + w * 131 + seed));
  const uint32_t v1 = (uint32_t)(vocab - 1);
  tok[i] = w < class_words ? 1 + (long long)((lab * (uint32_t)class_words + (uint32_t)w) % v1)
                           : 1 + (long long)(h % v1);
  if (k == 0 && w == 0) {
    labels64[b] = lab;
    labels32[b] = (int)lab;
    ids32[b] = (int)id;
  }
}

MILNCE_API int milnce_synth_meta(long long base, int B, int K, int W, int vocab, int ncls, int seed, int class_words,
                                 long long* tok, long long* labels64, int* labels32, int* ids32, hipStream_t stream) {
  const int n = B * K * W;
  if (n <= 0 || vocab < 2 || ncls < 1) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(synth_meta_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, base, B, K, W, vocab, ncls, seed,
                     class_words, tok, labels64, labels32, ids32);
  return (int)hipGetLastError();
}

MILNCE_API int milnce_synth_video(const int* labels, const int* ids, int B, int T, int S, void* out,
                                  hipStream_t stream) {
  const long long nrows = (long long)B * T * S;
  const long long grid = nrows < 65536 ? nrows : 65536;
  // one wave per image row: a 200-pixel row is 50 quads
  hipLaunchKernelGGL(synth_video_kernel, dim3((int)grid), dim3(64), 0, stream, labels, ids, T, S,
                     (uint32_t*)out, nrows);
  return (int)hipGetLastError();
}

// [B,3,T,H,W] -> [B,T,H,W,4] uint8 (src_kind 0) or bf16 (1: float32 in [0,1], 2: bf16); channel 3 is zero.
__global__ void stem_prep_kernel(const void* __restrict__ src, int kind, int T, int H, int W, void* __restrict__ dst,
                                 long long npix) {
  const long long plane = (long long)T * H * W;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < npix;
       i += (long long)gridDim.x * blockDim.x) {
    const long long b = i / plane, s = i - b * plane;
    if (kind == 0) {
      const uint8_t* u = (const uint8_t*)src;
      const uint32_t v = (uint32_t)u[(b * 3 + 0) * plane + s] | ((uint32_t)u[(b * 3 + 1) * plane + s] << 8) |
                         ((uint32_t)u[(b * 3 + 2) * plane + s] << 16);
      ((uint32_t*)dst)[i] = v;
    } else {
      float f[3];
      for (int c = 0; c < 3; ++c)
        f[c] = kind == 1 ? ((const float*)src)[(b * 3 + c) * plane + s]
                         : bf2f(((const bf16_t*)src)[(b * 3 + c) * plane + s]);
      uint2 o;
      o.x = pack2bf(f[0], f[1]);
      o.y = pack2bf(f[2], 0.f);
      ((uint2*)dst)[i] = o;
    }
  }
}

// uint8 [n] -> bf16 [n] * (1/255): the native clip [B,T,H,W,4] becomes the stem's bf16 operand,
// read by the conv as width pairs [B,T,H,W/2,8] (see hip_ops.stem_conv_bn_relu). 8 B in, 16 B out.
__global__ void u8_to_bf16_kernel(const uint2* __restrict__ src, uint4* __restrict__ dst, long long n8) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n8; i += (long long)gridDim.x * blockDim.x) {
    const uint2 v = src[i];
    const float s = 1.0f / 255.0f;
    float f[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      f[k] = (float)((v.x >> (8 * k)) & 0xff) * s;
      f[4 + k] = (float)((v.y >> (8 * k)) & 0xff) * s;
    }
    dst[i] = pack8(f);
  }
}

// ---------------------------------------------------------------------------------------
// One rank's slice of the one-shot peer all-gather (parallel/peer.py): copy into each peer's
// IPC-mapped receive buffer, issued on the local stream as plain vector loads / stores (the
// stores travel over that peer's xGMI link); one launch covers every destination.
constexpr int PEER_MAX = 8;
struct PeerDsts {
  void* dst[PEER_MAX];
};

__global__ __launch_bounds__(256) void peer_scatter_kernel(const uint4* __restrict__ src, PeerDsts d, int ndst,
                                                           long long n16) {
  const int k = blockIdx.y;  // destination
  uint4* __restrict__ dst = (uint4*)d.dst[k < ndst ? k : 0];
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n16; i += (long long)gridDim.x * 256) dst[i] = src[i];
}

MILNCE_API int milnce_peer_scatter(const void* src, void* const* dsts, int ndst, long long bytes, hipStream_t stream) {
  if (ndst < 1 || ndst > PEER_MAX || bytes % 16 || ((uintptr_t)src & 15)) return (int)hipErrorInvalidValue;
  PeerDsts d;
  for (int k = 0; k < PEER_MAX; ++k) {
    d.dst[k] = dsts[k < ndst ? k : 0];
    if (((uintptr_t)d.dst[k] & 15)) return (int)hipErrorInvalidValue;
  }
  const long long n16 = bytes / 16;
  long long bx = (n16 + 255) / 256;
  if (bx > 64) bx = 64;
  if (bx < 1) bx = 1;
  hipLaunchKernelGGL(peer_scatter_kernel, dim3((int)bx, ndst), dim3(256), 0, stream, (const uint4*)src, d, ndst, n16);
  return (int)hipGetLastError();
}

MILNCE_API int milnce_u8_to_bf16(const void* src, void* dst, long long n, hipStream_t stream) {
  if (n % 8) return (int)hipErrorInvalidValue;
  const long long n8 = n / 8;
  long long grid = (n8 + 255) / 256;
  if (grid > 65536) grid = 65536;
  hipLaunchKernelGGL(u8_to_bf16_kernel, dim3((int)grid), dim3(256), 0, stream, (const uint2*)src, (uint4*)dst, n8);
  return (int)hipGetLastError();
}

MILNCE_API int milnce_stem_prep(const void* src, int kind, int B, int T, int H, int W, void* dst, hipStream_t stream) {
  const long long npix = (long long)B * T * H * W;
  long long grid = (npix + 255) / 256;
  if (grid > 16384) grid = 16384;
  hipLaunchKernelGGL(stem_prep_kernel, dim3((int)grid), dim3(256), 0, stream, src, kind, T, H, W, dst, npix);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// h [N, Wd, F] bf16 -> out [N, F] fp32 = max_w relu(h); arg [N, F] uint8 (first max)
__global__ void text_relu_max_kernel(const bf16_t* __restrict__ h, int Wd, int F, float* __restrict__ out,
                                     uint8_t* __restrict__ arg, long long nchunks) {
  const int cpr = F >> 3;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < nchunks;
       i += (long long)gridDim.x * blockDim.x) {
    const long long n = i / cpr;
    const int f0 = (int)(i - n * cpr) * 8;
    float best[8];
    uint32_t bi[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) { best[k] = -INFINITY; bi[k] = 0; }
    for (int w = 0; w < Wd; ++w) {
      float v[8];
      unpack8(*(const uint4*)(h + ((n * Wd + w) * F + f0)), v);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float r = fmaxf(v[k], 0.f);
        if (r > best[k]) { best[k] = r; bi[k] = w; }
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      out[n * F + f0 + k] = best[k];
      arg[n * F + f0 + k] = (uint8_t)bi[k];
    }
  }
}

// dh [N, Wd, F] bf16: dout at the arg-max word where the max was positive (ReLU active), else 0
__global__ void text_relu_max_bwd_kernel(const float* __restrict__ dout, const float* __restrict__ out,
                                         const uint8_t* __restrict__ arg, int Wd, int F, bf16_t* __restrict__ dh,
                                         long long nchunks) {
  const int cpr = F >> 3;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < nchunks;
       i += (long long)gridDim.x * blockDim.x) {
    // i indexes (n, w, chunk)
    const long long nw = i / cpr;
    const int f0 = (int)(i - nw * cpr) * 8;
    const long long n = nw / Wd;
    const int w = (int)(nw - n * Wd);
    float g[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const long long o = n * F + f0 + k;
      g[k] = (arg[o] == w && out[o] > 0.f) ? dout[o] : 0.f;
    }
    *(uint4*)(dh + i * 8) = pack8(g);
  }
}

MILNCE_API int milnce_text_relu_max(const void* h, int N, int Wd, int F, float* out, void* arg, hipStream_t stream) {
  const long long n = (long long)N * (F / 8);
  long long grid = (n + 255) / 256;
  if (grid > 8192) grid = 8192;
  hipLaunchKernelGGL(text_relu_max_kernel, dim3((int)grid), dim3(256), 0, stream, (const bf16_t*)h, Wd, F, out,
                     (uint8_t*)arg, n);
  return (int)hipGetLastError();
}

// Text tower fc1 fused with its gather and the ReLU-max over words (s3dg.py:196-204):
//   out[n, f] = max_w relu(bf16(table[tok[n, w]] . w1[f] + b1[f])),  arg = first arg-max word
// Workgroup = 8 sentences x 64 features: the W1 tile [64][kp] is staged in LDS once and shared by
// the 8 waves; wave = one sentence (its <= 32 words as two 16-row MFMA fragments, rows gathered
// straight from the embedding table into the A operand, issued before the W1 staging) x the 64
// features (four 16-column fragments). K = kp (table and W1 zero-padded to a multiple of 32 bf16). The
// [N*Wd, F] fc1 output is never stored: the max runs on the accumulators (per lane over its
// words, then across the four row groups by shuffles).
constexpr int TXT_FT = 64;  // features per workgroup (41 KiB of W1 in LDS: 3 workgroups per CU)
template <int KS>  // K steps of 32 (kp / 32), compile time: every A fragment is loaded up front
__global__ __launch_bounds__(512) void text_fc1_max_kernel(const long long* __restrict__ tok, int N, int Wd,
                                                           const bf16_t* __restrict__ table,
                                                           const bf16_t* __restrict__ w1, const float* __restrict__ b1,
                                                           int F, int kp, float* __restrict__ out,
                                                           uint8_t* __restrict__ arg) {
  extern __shared__ __attribute__((aligned(16))) bf16_t ws[];  // [TXT_FT][kp + 8]
  const int ldw = kp + 8;
  const int f0 = blockIdx.y * TXT_FT;
  const int lane = threadIdx.x & 63;
  const int n = blockIdx.x * 8 + (threadIdx.x >> 6);
  const bool live = n < N;  // wave-uniform
  const int li = lane & 15, g = lane >> 4;
  // the sentence's gathered rows first (all K steps in flight), then the shared W1 tile
  bf16x8 a[KS][2];
#pragma unroll
  for (int rf = 0; rf < 2; ++rf) {
    const int w = rf * 16 + li;
    const long long t = (live && w < Wd) ? tok[(long long)n * Wd + w] : 0;  // rows past Wd: masked below
    const bf16_t* arow = table + t * kp + g * 8;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) a[ks][rf] = *(const bf16x8*)(arow + ks * 32);
  }
  const int cpr = kp / 8;
  for (int i = threadIdx.x; i < TXT_FT * cpr; i += blockDim.x) {
    const int r = i / cpr, c = i - r * cpr;
    *(uint4*)(ws + r * ldw + c * 8) = *(const uint4*)(w1 + (long long)(f0 + r) * kp + c * 8);
  }
  __syncthreads();
  if (!live) return;
  const bf16_t* bl = ws + li * ldw + g * 8;
  f32x4 acc[2][TXT_FT / 16];
#pragma unroll
  for (int rf = 0; rf < 2; ++rf)
#pragma unroll
    for (int cf = 0; cf < TXT_FT / 16; ++cf) acc[rf][cf] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
    for (int cf = 0; cf < TXT_FT / 16; ++cf) {
      const bf16x8 b = *(const bf16x8*)(bl + cf * 16 * ldw + ks * 32);
#pragma unroll
      for (int rf = 0; rf < 2; ++rf)
        acc[rf][cf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[ks][rf], b, acc[rf][cf], 0, 0, 0);
    }
  }
  // C[i = word][j = feature]: this lane holds feature li of each fragment and words rf*16 + 4g + r
#pragma unroll
  for (int cf = 0; cf < TXT_FT / 16; ++cf) {
    const int f = f0 + cf * 16 + li;
    const float bias = b1[f];
    float best = -INFINITY;
    int bi = 0;
#pragma unroll
    for (int rf = 0; rf < 2; ++rf)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int w = rf * 16 + 4 * g + r;  // ascending per lane
        const float v = fmaxf(bf2f(f2bf(acc[rf][cf][r] + bias)), 0.f);  // relu(bf16 fc1 output)
        if (w < Wd && v > best) { best = v; bi = w; }
      }
#pragma unroll
    for (int o = 16; o < 64; o <<= 1) {  // the 4 row groups: larger value, ties to the earlier word
      const float ov = __shfl_xor(best, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ov > best || (ov == best && oi < bi)) { best = ov; bi = oi; }
    }
    if (g == 0) {
      out[(long long)n * F + f] = best;
      arg[(long long)n * F + f] = (uint8_t)bi;
    }
  }
}

MILNCE_API int milnce_text_fc1_max(const long long* tok, int N, int Wd, const void* table, const void* w1,
                                   const float* b1, int F, int kp, float* out, void* arg, hipStream_t stream) {
  if (Wd > 32 || Wd < 1 || F % TXT_FT || kp != 320) return (int)hipErrorInvalidValue;  // 300-d word2vec
  const size_t lds = (size_t)TXT_FT * (kp + 8) * 2;
  if (lds > 160 * 1024) return (int)hipErrorInvalidValue;
  static bool attr = false;
  if (!attr) {
    HIP_RET(hipFuncSetAttribute((const void*)text_fc1_max_kernel<10>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                160 * 1024));
    attr = true;
  }
  hipLaunchKernelGGL(text_fc1_max_kernel<10>, dim3((N + 7) / 8, F / TXT_FT), dim3(512), lds, stream, tok, N, Wd,
                     (const bf16_t*)table, (const bf16_t*)w1, b1, F, kp, out, (uint8_t*)arg);
  return (int)hipGetLastError();
}

MILNCE_API int milnce_text_relu_max_bwd(const float* dout, const float* out, const void* arg, int N, int Wd, int F,
                                        void* dh, hipStream_t stream) {
  const long long n = (long long)N * Wd * (F / 8);
  long long grid = (n + 255) / 256;
  if (grid > 8192) grid = 8192;
  hipLaunchKernelGGL(text_relu_max_bwd_kernel, dim3((int)grid), dim3(256), 0, stream, dout, out,
                     (const uint8_t*)arg, Wd, F, (bf16_t*)dh, n);
  return (int)hipGetLastError();
}
