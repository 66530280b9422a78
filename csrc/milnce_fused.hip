// Fused MIL-NCE (loss.py:10-18) for large global batches: the logits x = V T^T ([Bg, Bg*K]) are
// never stored. The logit and gradient GEMMs run on bf16 MFMA (mfma_f32_16x16x32_bf16) with
// split-bf16 operands for fp32-level accuracy: every fp32 operand X is held as X_hi = bf16(X),
// X_lo = bf16(X - X_hi) (16 significant bits together), and A B = A_hi B_hi + A_hi B_lo + A_lo B_hi
// (the dropped A_lo B_lo term is 2^-16 relative): 3 bf16 MFMAs per product, i.e. 16/3 x the rate
// of the f32-input MFMA the first version used.
//
//   split   : V, T (fp32) -> row-major [R][D] hi/lo and transposed [D][Rp] hi/lo bf16 copies (the
//             transposed ones make the backward's reductions over the batch k-contiguous MFMA
//             operands, like the forward's);
//   forward : 64 x 64 logit tiles (8 waves x 16 rows x 32 columns), per tile a row partial (max, sum e^{x-max})
//             over its 64 columns and, for each of its 64/K text blocks, a block-column partial
//             over its 64 rows; a finalize kernel merges them into den_i = LSE(row_i U blockcol_i)
//             and takes nom_i = LSE_k V_i . T_{iK+k} (positives counted twice, as in the reference);
//   backward: G[i, j] = g/Bg (e^{x-den_i} + e^{x-den_{j/K}} - [j/K == i] e^{x-nom_i}) recomputed
//             tile by tile and split to bf16 hi/lo in LDS; dV = G T by a row-tile pass (64 rows x
//             D accumulated in registers), dT = G^T V by a column-tile pass; no atomics,
//             deterministic. Nothing of size [Bg, Bg*K] is ever stored.
//
// LDS images are [64 rows][64 bf16] with the 16-B chunk XOR swizzle of the conv kernels
// (conflict-free ds_read_b128 fragment reads); operands are register-staged one 64-wide K chunk
// ahead of the MFMAs.
#include "common.h"

namespace {

constexpr int TM = 64, TN = 64;  // tile rows (video) x tile columns (text)
constexpr int KC = 64;           // K chunk of every GEMM (bf16 elements per LDS row)
constexpr int GP = TN + 1;       // padded fp32 S tile row
constexpr int IMG = 64 * KC;     // elements of one [64][64] bf16 image

__device__ __forceinline__ void lse_add(float& m, float& s, float m2, float s2) {
  if (m2 == -INFINITY) return;
  if (m == -INFINITY) { m = m2; s = s2; return; }
  if (m2 > m) { s = s * __expf(m - m2) + s2; m = m2; }
  else { s += s2 * __expf(m2 - m); }
}

__device__ __forceinline__ int sw(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

constexpr int NT = 512;  // 8 waves per workgroup

// Register staging of 64 rows x 64 columns of a bf16 [rows][ld] matrix (rows >= nrows read 0):
// one 16-B piece per thread.
struct Stage1 {
  uint4 v;
  __device__ __forceinline__ void load(const bf16_t* __restrict__ src, long long ld, int row0, int nrows, int col0) {
    const int r = threadIdx.x >> 3, c = threadIdx.x & 7;
    v = row0 + r < nrows ? *(const uint4*)(src + (long long)(row0 + r) * ld + col0 + c * 8) : make_uint4(0u, 0u, 0u, 0u);
  }
  __device__ __forceinline__ void store(bf16_t* img) const {
    const int r = threadIdx.x >> 3, c = threadIdx.x & 7;
    *(uint4*)(img + r * KC + sw(r, c) * 8) = v;
  }
};

__device__ __forceinline__ bf16x8 frag(const bf16_t* img, int row, int s) {
  // 16x16x32 operand fragment: row (lane & 15) of the 16-row block, k = 32 s + 8 (lane >> 4) ..
  const int lane = threadIdx.x & 63;
  return *(const bf16x8*)(img + row * KC + sw(row, s * 4 + (lane >> 4)) * 8);
}

// acc += A B^T over one staged 64-wide K chunk with split operands: A rows arow (16 per wave),
// B rows 16 (cb0 + cb) + (lane & 15) for cb < NB.
template <int NB>
__device__ __forceinline__ void mfma_chunk(const bf16_t* Ah, const bf16_t* Al, const bf16_t* Bh, const bf16_t* Bl,
                                           int arow, int cb0, f32x4 (&acc)[NB]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const bf16x8 ah = frag(Ah, arow, s), al = frag(Al, arow, s);
#pragma unroll
    for (int cb = 0; cb < NB; ++cb) {
      const int br = 16 * (cb0 + cb) + (lane & 15);
      const bf16x8 bh = frag(Bh, br, s), bl = frag(Bl, br, s);
      acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, acc[cb], 0, 0, 0);
      acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, acc[cb], 0, 0, 0);
      acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, acc[cb], 0, 0, 0);
    }
  }
}

struct Split {  // split copies of one fp32 matrix X [R][D]
  const bf16_t* h;   // [R][D]
  const bf16_t* l;
  const bf16_t* th;  // [D][Rp], Rp = R rounded up to 64 (zero padding)
  const bf16_t* tl;
};

// S[64 x 64] = V[r0 : r0+64] . T[c0 : c0+64]^T, 8 waves: wave w holds rows 16 (w & 3).. and the
// two 16-column blocks 2 (w >> 2) + cb (acc[cb][r] = S[16 (w&3) + 4 (lane>>4) + r][16 (2 (w>>2) + cb) +
// (lane & 15)]). img: 4 images (Vh, Vl, Th, Tl).
__device__ __forceinline__ void logit_tile(const Split& V, const Split& T, int B, int N, int D, int r0, int c0,
                                           bf16_t* img, f32x4 (&acc)[2]) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int cb = 0; cb < 2; ++cb) acc[cb] = (f32x4){0.f, 0.f, 0.f, 0.f};
  Stage1 a, b, c, d;
  a.load(V.h, D, r0, B, 0);
  b.load(V.l, D, r0, B, 0);
  c.load(T.h, D, c0, N, 0);
  d.load(T.l, D, c0, N, 0);
  for (int k0 = 0; k0 < D; k0 += KC) {
    __syncthreads();  // previous chunk's fragments read
    a.store(img);
    b.store(img + IMG);
    c.store(img + 2 * IMG);
    d.store(img + 3 * IMG);
    __syncthreads();
    if (k0 + KC < D) {
      a.load(V.h, D, r0, B, k0 + KC);
      b.load(V.l, D, r0, B, k0 + KC);
      c.load(T.h, D, c0, N, k0 + KC);
      d.load(T.l, D, c0, N, k0 + KC);
    }
    mfma_chunk<2>(img, img + IMG, img + 2 * IMG, img + 3 * IMG, 16 * (w & 3) + (lane & 15), 2 * (w >> 2), acc);
  }
}

__device__ __forceinline__ void store_tile(float* Ss, const f32x4 (&acc)[2]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int cb = 0; cb < 2; ++cb)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      Ss[(16 * (w & 3) + 4 * (lane >> 4) + r) * GP + 16 * (2 * (w >> 2) + cb) + (lane & 15)] = acc[cb][r];
}

// G tile from the logit tile in Ss, split into bf16 hi / lo images. TRANS = false: image rows are
// the tile's rows i (dV pass: A = G); TRANS = true: rows are the tile's columns j (dT pass: A = G^T).
template <bool TRANS>
__device__ __forceinline__ void grad_tile(const float* Ss, bf16_t* Gh, bf16_t* Gl, int B, int K, int r0, int c0,
                                          const float* __restrict__ den, const float* __restrict__ nom,
                                          const float* __restrict__ gup) {
  const int N = B * K;
  const float gscale = gup[0] / (float)B;  // d loss / d x = (upstream grad) / Bg * (...)
  // each thread: one image row, 8 consecutive image columns per pass (one 16-B chunk of hi and lo)
  for (int e = threadIdx.x; e < 64 * 8; e += NT) {
    const int row = e >> 3, ch = e & 7;
    float hv[8], lv[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int rr = TRANS ? ch * 8 + q : row, cc = TRANS ? row : ch * 8 + q;
      const int i = r0 + rr, j = c0 + cc;
      float g = 0.f;
      if (i < B && j < N) {
        const float x = Ss[rr * GP + cc];
        const int blk = j / K;
        g = __expf(x - den[i]) + __expf(x - den[blk]);
        if (blk == i) g -= __expf(x - nom[i]);
        g *= gscale;
      }
      hv[q] = g;
    }
    uint4 h, l;
    h = pack8(hv);
    float hf[8];
    unpack8(h, hf);
#pragma unroll
    for (int q = 0; q < 8; ++q) lv[q] = hv[q] - hf[q];
    l = pack8(lv);
    *(uint4*)(Gh + row * KC + sw(row, ch) * 8) = h;
    *(uint4*)(Gl + row * KC + sw(row, ch) * 8) = l;
  }
}

}  // namespace

// X [R][D] fp32 -> h, l [R][D] and th, tl [D][Rp] bf16 (64 x 64 tiles through LDS for the transpose).
__global__ __launch_bounds__(256) void milnce_split_kernel(const float* __restrict__ X, int R, int D, bf16_t* __restrict__ h,
                                                           bf16_t* __restrict__ l, bf16_t* __restrict__ th,
                                                           bf16_t* __restrict__ tl) {
  __shared__ uint16_t sh[64][66], sl[64][66];
  const int r0 = blockIdx.x * 64, d0 = blockIdx.y * 64;
  for (int e = threadIdx.x; e < 64 * 16; e += 256) {
    const int r = e >> 4, c4 = (e & 15) * 4;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (r0 + r < R) v = *(const float4*)(X + (long long)(r0 + r) * D + d0 + c4);
    const float f[4] = {v.x, v.y, v.z, v.w};
    uint16_t hb[4], lb[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      hb[q] = f2bf(f[q]);
      lb[q] = f2bf(f[q] - bf2f(hb[q]));
      sh[r][c4 + q] = hb[q];
      sl[r][c4 + q] = lb[q];
    }
    if (r0 + r < R) {
      *(uint2*)(h + (long long)(r0 + r) * D + d0 + c4) =
          make_uint2(hb[0] | ((uint32_t)hb[1] << 16), hb[2] | ((uint32_t)hb[3] << 16));
      *(uint2*)(l + (long long)(r0 + r) * D + d0 + c4) =
          make_uint2(lb[0] | ((uint32_t)lb[1] << 16), lb[2] | ((uint32_t)lb[3] << 16));
    }
  }
  __syncthreads();
  // transposed copies [D][Rp], Rp = R rounded up to 64: the padding columns are written as zeros
  // (the backward's staging reads whole 64-column pieces)
  const long long Rp = (R + 63) / 64 * 64;
  for (int e = threadIdx.x; e < 64 * 16; e += 256) {
    const int dd = e >> 4, r4 = (e & 15) * 4;
    *(uint2*)(th + (long long)(d0 + dd) * Rp + r0 + r4) =
        make_uint2(sh[r4][dd] | ((uint32_t)sh[r4 + 1][dd] << 16), sh[r4 + 2][dd] | ((uint32_t)sh[r4 + 3][dd] << 16));
    *(uint2*)(tl + (long long)(d0 + dd) * Rp + r0 + r4) =
        make_uint2(sl[r4][dd] | ((uint32_t)sl[r4 + 1][dd] << 16), sl[r4 + 2][dd] | ((uint32_t)sl[r4 + 3][dd] << 16));
  }
}

// rowpart: [n_ct][B] (max, sum); colpart: [n_rt][B] (max, sum) per text block.
__global__ __launch_bounds__(512) void milnce_fused_fwd_kernel(Split V, Split T, int B, int K, int D,
                                                               float2* __restrict__ rowpart,
                                                               float2* __restrict__ colpart) {
  __shared__ __attribute__((aligned(16))) bf16_t img[4 * IMG];
  __shared__ float Ss[TM * GP];
  const int N = B * K;
  const int rt = blockIdx.y, ct = blockIdx.x;
  const int r0 = rt * TM, c0 = ct * TN;
  f32x4 acc[2];
  logit_tile(V, T, B, N, D, r0, c0, img, acc);
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
  // block, NT / 16 blocks per pass (64 / K blocks per tile)
  const int nbk = TN / K;
  const int sub = tid & 15;
  constexpr int BPP = NT / 16;
  for (int b = tid >> 4; b < ((nbk + BPP - 1) / BPP) * BPP; b += BPP) {
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

// One backward pass. DT = false: dV[r0 : r0+64, :] = sum over column tiles of G . T (rows of the
// block = video rows); DT = true: dT[c0 : c0+64, :] = sum over row tiles of G^T . V. The product's
// B operand is the transposed split copy ([D][Rp]) of T (resp. V), rows d, k over the tile.
// 8 waves: wave w accumulates output rows 16 (w & 3).. over the D half (w >> 2); each staging step
// brings one 64-wide d chunk of each half.
template <bool DT>
__global__ __launch_bounds__(512) void milnce_fused_grad_kernel(Split V, Split T, int B, int K, int D,
                                                                const float* __restrict__ den,
                                                                const float* __restrict__ nom,
                                                                const float* __restrict__ gup, float* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) bf16_t img[4 * IMG];  // logit operands, then two Xt chunks (hi / lo)
  __shared__ __attribute__((aligned(16))) bf16_t gimg[2 * IMG];  // G (or G^T) hi / lo
  __shared__ float Ss[TM * GP];
  const int N = B * K;
  const int blk = blockIdx.x;
  const int split = blockIdx.y, splits = gridDim.y;
  const int own0 = blk * 64;                       // rows of the output this block owns
  const int R = DT ? N : B;                        // output rows
  out += (long long)split * R * D;                 // split > 0 (or splits > 1): partial sums
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int rg = w & 3, dh = w >> 2;
  const int half = D / KC / 2;                     // d chunks per half (D % 128 == 0)
  f32x4 acc_out[4][4];  // this wave's 16 output rows x its D half (up to 256)
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc_out[a][c] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const int n_other = DT ? (B + TM - 1) / TM : (N + TN - 1) / TN;
  const int t_begin = (int)((long long)split * n_other / splits), t_end = (int)((long long)(split + 1) * n_other / splits);
  const Split& X = DT ? V : T;  // the operand whose rows the tiles walk (reduction index of the product)
  const long long xld = ((DT ? B : N) + 63) / 64 * 64;  // row length of its transposed copy
  for (int t = t_begin; t < t_end; ++t) {
    const int r0 = DT ? t * TM : own0, c0 = DT ? own0 : t * TN;
    f32x4 acc[2];
    logit_tile(V, T, B, N, D, r0, c0, img, acc);
    store_tile(Ss, acc);
    __syncthreads();
    grad_tile<DT>(Ss, gimg, gimg + IMG, B, K, r0, c0, den, nom, gup);
    const int x0 = DT ? r0 : c0;  // first row of X in this tile (k range of the product)
    Stage1 p0h, p0l, p1h, p1l;     // d chunk j of half 0 and of half 1
    p0h.load(X.th, xld, 0, D, x0);
    p0l.load(X.tl, xld, 0, D, x0);
    p1h.load(X.th, xld, half * KC, D, x0);
    p1l.load(X.tl, xld, half * KC, D, x0);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (j < half) {
        __syncthreads();  // G images written / previous chunk's fragments read
        p0h.store(img);
        p0l.store(img + IMG);
        p1h.store(img + 2 * IMG);
        p1l.store(img + 3 * IMG);
        __syncthreads();
        if (j + 1 < half) {
          p0h.load(X.th, xld, (j + 1) * KC, D, x0);
          p0l.load(X.tl, xld, (j + 1) * KC, D, x0);
          p1h.load(X.th, xld, (half + j + 1) * KC, D, x0);
          p1l.load(X.tl, xld, (half + j + 1) * KC, D, x0);
        }
        const bf16_t* xi = img + 2 * dh * IMG;
        mfma_chunk<4>(gimg, gimg + IMG, xi, xi + IMG, 16 * rg + (lane & 15), 0, acc_out[j]);
      }
    }
    __syncthreads();  // Xt images read before the next tile's logit staging overwrites them
  }
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (j < half)
#pragma unroll
      for (int cb = 0; cb < 4; ++cb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = own0 + 16 * rg + 4 * (lane >> 4) + r;
          if (i < R) out[(long long)i * D + (dh * half + j) * KC + 16 * cb + (lane & 15)] = acc_out[j][cb][r];
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

namespace {

// workspace layout (floats): rowpart [n_ct][B] float2, colpart [n_rt][B] float2, li [B], then the
// split copies of V and T (bf16: 4 [R][D] arrays each = 2 floats per element)
struct FusedWs {
  float2* rowpart;
  float2* colpart;
  float* li;
  Split V, T;
};

FusedWs carve(float* ws, int B, int K, int D) {
  const long long N = (long long)B * K;
  const long long n_ct = (N + TN - 1) / TN, n_rt = (B + TM - 1) / TM;
  FusedWs w;
  w.rowpart = (float2*)ws;
  w.colpart = w.rowpart + n_ct * B;
  w.li = (float*)(w.colpart + n_rt * B);
  long long off = 2 * (n_ct * B + n_rt * B) + B;
  off = (off + 63) / 64 * 64;  // 256-B alignment of the bf16 arrays
  bf16_t* p = (bf16_t*)(ws + off);
  const long long vb = (long long)B * D, vtb = (long long)D * ((B + 63) / 64 * 64);
  const long long tb = N * D, ttb = (long long)D * ((N + 63) / 64 * 64);
  w.V = {p, p + vb, p + 2 * vb, p + 2 * vb + vtb};
  p += 2 * vb + 2 * vtb;
  w.T = {p, p + tb, p + 2 * tb, p + 2 * tb + ttb};
  return w;
}

bool geometry_ok(int B, int K, int D) { return K >= 1 && TN % K == 0 && D % (2 * KC) == 0 && D <= 8 * KC && B >= 1; }

}  // namespace

// Split counts of the two backward passes: ~2 workgroups per CU over (tiles x reduction ranges).
MILNCE_API int milnce_fused_bwd_splits(int B, int K, int* s_dv, int* s_dt) {
  const int N = B * K;
  const int n_ct = (N + TN - 1) / TN, n_rt = (B + TM - 1) / TM;
  int a = (512 + n_rt - 1) / n_rt, b = (512 + n_ct - 1) / n_ct;
  *s_dv = a < n_ct ? a : n_ct;
  *s_dt = b < n_rt ? b : n_rt;
  return 0;
}

// Workspace floats of the fused loss (partials + the split operand copies the backward reuses).
MILNCE_API long long milnce_fused_ws_floats(int B, int K, int D) {
  const long long N = (long long)B * K;
  const long long n_ct = (N + TN - 1) / TN, n_rt = (B + TM - 1) / TM;
  const long long off = (2 * (n_ct * B + n_rt * B) + B + 63) / 64 * 64;
  const long long Bp = ((long long)B + 63) / 64 * 64, Np = (N + 63) / 64 * 64;
  return off + ((long long)B + Bp + N + Np) * D;  // 4 bf16 arrays per matrix = (R + Rp) D floats
}

MILNCE_API int milnce_fused_fwd(const float* V, const float* T, int B, int K, int D, float* ws, float* den, float* nom,
                                float* loss, hipStream_t stream) {
  if (!geometry_ok(B, K, D)) return (int)hipErrorInvalidValue;
  const int N = B * K;
  const int n_ct = (N + TN - 1) / TN, n_rt = (B + TM - 1) / TM;
  FusedWs w = carve(ws, B, K, D);
  hipLaunchKernelGGL(milnce_split_kernel, dim3((B + 63) / 64, D / 64), dim3(256), 0, stream, V, B, D,
                     (bf16_t*)w.V.h, (bf16_t*)w.V.l, (bf16_t*)w.V.th, (bf16_t*)w.V.tl);
  HIP_RET(hipGetLastError());
  hipLaunchKernelGGL(milnce_split_kernel, dim3((N + 63) / 64, D / 64), dim3(256), 0, stream, T, N, D,
                     (bf16_t*)w.T.h, (bf16_t*)w.T.l, (bf16_t*)w.T.th, (bf16_t*)w.T.tl);
  HIP_RET(hipGetLastError());
  hipLaunchKernelGGL(milnce_fused_fwd_kernel, dim3(n_ct, n_rt), dim3(NT), 0, stream, w.V, w.T, B, K, D, w.rowpart,
                     w.colpart);
  HIP_RET(hipGetLastError());
  hipLaunchKernelGGL(milnce_fused_finalize_kernel, dim3((B + 3) / 4), dim3(256), 0, stream, V, T, B, K, D, w.rowpart,
                     n_ct, w.colpart, n_rt, den, nom, w.li);
  HIP_RET(hipGetLastError());
  hipLaunchKernelGGL(milnce_fused_mean_kernel, dim3(1), dim3(256), 0, stream, w.li, B, loss);
  return (int)hipGetLastError();
}

// dV / dT from the forward's workspace (its split copies); with s_dv / s_dt > 1 the passes write
// partial sums to `part` ([s][B][D] then [s][N][D]) which are summed into dV / dT.
MILNCE_API int milnce_fused_bwd(const float* ws, int B, int K, int D, const float* den, const float* nom,
                                const float* gup, float* dV, float* dT, int s_dv, int s_dt, float* part,
                                hipStream_t stream) {
  if (!geometry_ok(B, K, D)) return (int)hipErrorInvalidValue;
  const int N = B * K;
  FusedWs w = carve((float*)ws, B, K, D);
  float* pv = s_dv > 1 ? part : dV;
  hipLaunchKernelGGL(milnce_fused_grad_kernel<false>, dim3((B + TM - 1) / TM, s_dv), dim3(NT), 0, stream, w.V, w.T,
                     B, K, D, den, nom, gup, pv);
  HIP_RET(hipGetLastError());
  if (s_dv > 1) {
    const long long n4 = (long long)B * D / 4;
    hipLaunchKernelGGL(milnce_split_sum_kernel, dim3((int)((n4 + 255) / 256 < 2048 ? (n4 + 255) / 256 : 2048)),
                       dim3(256), 0, stream, (const float4*)pv, s_dv, n4, (float4*)dV);
    HIP_RET(hipGetLastError());
  }
  float* pt = s_dt > 1 ? part : dT;
  hipLaunchKernelGGL(milnce_fused_grad_kernel<true>, dim3((N + TN - 1) / TN, s_dt), dim3(NT), 0, stream, w.V, w.T,
                     B, K, D, den, nom, gup, pt);
  HIP_RET(hipGetLastError());
  if (s_dt > 1) {
    const long long n4 = (long long)N * D / 4;
    hipLaunchKernelGGL(milnce_split_sum_kernel, dim3((int)((n4 + 255) / 256 < 2048 ? (n4 + 255) / 256 : 2048)),
                       dim3(256), 0, stream, (const float4*)pt, s_dt, n4, (float4*)dT);
  }
  return (int)hipGetLastError();
}
