// Implicit-GEMM 3-D convolution for S3D-G on gfx950 MFMA (channels-last / NDHWC).
//
//   forward / dgrad :  Y[m, n] = sum_k A[m, k] * W[n, k]
//      m = (b, to, ho, wo) output position, n = output channel,
//      k = (tap, c) with tap = (dt, dh, dw); A is gathered on the fly from X (zero padding,
//      optional uint8 input scaled by 1/255 for the stem). dgrad is the same kernel run on dY
//      with the flipped/transposed weight packing and padding k-1-p (all dgrad convs are stride 1).
//      Epilogue: bf16 output staged through LDS for 16-B coalesced stores, plus per-channel
//      BatchNorm partial statistics (sum, sum of squares from the fp32 accumulators) kept in
//      registers across the block's persistent M loop and written once per block.
//   wgrad           :  dW[n, k] = sum_m dY[m, n] * A[m, k]
//      split-K over m; both operands are staged row-major (m rows) in LDS and read as MFMA
//      fragments with ds_read_b64_tr_b16 (the reduction index is the LDS row), partial tiles
//      go to an fp32 slab that a second kernel reduces and unpacks to the PyTorch weight
//      layout [Cout, Cin, kt, kh, kw] (deterministic, no atomics).
//
// Tiles: 256 threads = 4 waves (2 x 2), mfma_f32_16x16x32_bf16, LDS double buffering with
// register staging (the gather needs per-element zero fill), XOR-swizzled A/B images so the
// 16-lane ds_read_b128 groups are bank-conflict free, XCD-aware block remap.
#include "common.h"

struct ConvParams {
  const void* x;       // [B, T, H, W, Cin] bf16 or uint8
  const bf16_t* w;     // packed [Npad, Kpad] bf16 (k = (tap, c), c fastest)
  bf16_t* y;           // [M, ldy] bf16
  float* stats;        // [grid_m, 2, Npad] or nullptr
  long long x_bstride; // T*H*W*Cin
  int T, H, W, Cin;
  int To, Ho, Wo, Cout;
  int KT, KH, KW, st, sh, sw, pt, ph, pw;
  int Ktot, Kpad, ldy, M;
  int num_m_tiles, num_n_tiles, grid_m;
  float in_scale;
  FastDiv fWo, fHo, fTo;
};

template <int BK>
__device__ __forceinline__ int swz(int row, int chunk) {
  // 16-B chunk swizzle of a [rows][BK] bf16 tile (BK*2-byte rows).
  if constexpr (BK == 32) return chunk ^ ((row >> 2) & 3);
  else return chunk ^ ((row >> 1) & 7);
}

template <int BM, int BN, int BK, bool U8>
__global__ __launch_bounds__(256) void conv_fwd_kernel(ConvParams p) {
  constexpr int VEC = U8 ? 4 : 8;
  constexpr int A_CPR = BK / VEC;
  constexpr int A_CH = BM * A_CPR / 256;
  constexpr int B_CPR = BK / 8;
  constexpr int B_CH = BN * B_CPR / 256;
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int KSTEPS = BK / 32;
  constexpr int EPAD = 16;  // epilogue staging row pad (elements)
  static_assert(A_CH >= 1 && B_CH >= 1, "tile too small");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* As = (bf16_t*)smem;          // [2][BM][BK]
  bf16_t* Bs = As + 2 * BM * BK;       // [2][BN][BK]
  bf16_t* Es = (bf16_t*)smem;          // epilogue [BM][BN+EPAD]

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;

  const int nblocks = p.num_n_tiles * p.grid_m;
  const int logical = xcd_remap(blockIdx.x, nblocks);
  const int n_tile = logical % p.num_n_tiles;
  const int m_slot = logical / p.num_n_tiles;
  const int n0 = n_tile * BN;
  const int nk = p.Kpad / BK;

  const int a_ccol = tid % A_CPR;
  const int b_ccol = tid % B_CPR;

  float st_s[TN], st_q[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) { st_s[j] = 0.f; st_q[j] = 0.f; }

  const uint8_t* xb = (const uint8_t*)p.x;
  const int esize = U8 ? 1 : 2;

  for (int m_tile = m_slot; m_tile < p.num_m_tiles; m_tile += p.grid_m) {
    const int m0 = m_tile * BM;
    // ---- per-row gather coordinates for this M tile ----
    const uint8_t* rbase[A_CH];
    int rt[A_CH], rh[A_CH], rw[A_CH], rowoff[A_CH];
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const int row = (tid + i * 256) / A_CPR;
      const int m = m0 + row;
      if (m < p.M) {
        uint32_t q = fdiv((uint32_t)m, p.fWo);
        const int wo = m - q * p.Wo;
        uint32_t q2 = fdiv(q, p.fHo);
        const int ho = q - q2 * p.Ho;
        uint32_t b = fdiv(q2, p.fTo);
        const int to = q2 - b * p.To;
        rbase[i] = xb + (long long)b * p.x_bstride * esize;
        rt[i] = to * p.st - p.pt;
        rh[i] = ho * p.sh - p.ph;
        rw[i] = wo * p.sw - p.pw;
        rowoff[i] = ((rt[i] * p.H + rh[i]) * p.W + rw[i]) * p.Cin;
      } else {
        rbase[i] = xb;
        rt[i] = -(1 << 28);
        rh[i] = 0;
        rw[i] = 0;
        rowoff[i] = 0;
      }
    }
    // ---- k state (tap, channel) of this thread's A chunk ----
    int kc = a_ccol * VEC;  // channel within tap
    int tap = 0, dt = 0, dh = 0, dw = 0;
    while (kc >= p.Cin) {
      kc -= p.Cin; ++tap;
      if (++dw == p.KW) { dw = 0; if (++dh == p.KH) { dh = 0; ++dt; } }
    }
    const int taps = p.KT * p.KH * p.KW;

    using AReg = typename std::conditional<U8, uint32_t, uint4>::type;
    AReg areg[A_CH];
    uint4 breg[B_CH];

    auto load_a = [&]() {
      const bool kval = tap < taps;
      const int toff = ((dt * p.H + dh) * p.W + dw) * p.Cin + kc;
#pragma unroll
      for (int i = 0; i < A_CH; ++i) {
        const int ti = rt[i] + dt, hi = rh[i] + dh, wi = rw[i] + dw;
        const bool v = kval && (unsigned)ti < (unsigned)p.T && (unsigned)hi < (unsigned)p.H &&
                       (unsigned)wi < (unsigned)p.W;
        const int off = rowoff[i] + toff;  // element offset inside the clip
        if constexpr (U8) {
          areg[i] = v ? *(const uint32_t*)(rbase[i] + off) : 0u;
        } else {
          areg[i] = v ? *(const uint4*)(rbase[i] + (long long)off * 2) : make_uint4(0, 0, 0, 0);
        }
      }
    };
    auto advance_k = [&]() {
      kc += BK;
      while (kc >= p.Cin) {
        kc -= p.Cin; ++tap;
        if (++dw == p.KW) { dw = 0; if (++dh == p.KH) { dh = 0; ++dt; } }
      }
    };
    auto load_b = [&](int kt) {
#pragma unroll
      for (int i = 0; i < B_CH; ++i) {
        const int row = (tid + i * 256) / B_CPR;
        breg[i] = *(const uint4*)(p.w + (long long)(n0 + row) * p.Kpad + kt * BK + b_ccol * 8);
      }
    };
    auto store_ab = [&](int buf) {
      bf16_t* a = As + buf * BM * BK;
#pragma unroll
      for (int i = 0; i < A_CH; ++i) {
        const int row = (tid + i * 256) / A_CPR;
        if constexpr (U8) {
          const uint32_t v = areg[i];
          const float s = p.in_scale;
          uint2 o;
          o.x = pack2bf((float)(v & 0xff) * s, (float)((v >> 8) & 0xff) * s);
          o.y = pack2bf((float)((v >> 16) & 0xff) * s, (float)(v >> 24) * s);
          const int k0 = a_ccol * 4;
          const int ch = swz<BK>(row, k0 >> 3);
          *(uint2*)(a + row * BK + ch * 8 + (k0 & 4)) = o;
        } else {
          const int ch = swz<BK>(row, a_ccol);
          *(uint4*)(a + row * BK + ch * 8) = areg[i];
        }
      }
      bf16_t* bsh = Bs + buf * BN * BK;
#pragma unroll
      for (int i = 0; i < B_CH; ++i) {
        const int row = (tid + i * 256) / B_CPR;
        const int ch = swz<BK>(row, b_ccol);
        *(uint4*)(bsh + row * BK + ch * 8) = breg[i];
      }
    };

    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

    load_a();
    load_b(0);
    store_ab(0);
    __syncthreads();

    for (int kt = 0; kt < nk; ++kt) {
      const int buf = kt & 1;
      if (kt + 1 < nk) {
        advance_k();
        load_a();
        load_b(kt + 1);
      }
      const bf16_t* a = As + buf * BM * BK;
      const bf16_t* bsh = Bs + buf * BN * BK;
#pragma unroll
      for (int s = 0; s < KSTEPS; ++s) {
        bf16x8 af[TM], bfr[TN];
        const int chunk = s * 4 + (lane >> 4);
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int row = wr * WM + i * 16 + (lane & 15);
          af[i] = *(const bf16x8*)(a + row * BK + swz<BK>(row, chunk) * 8);
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int row = wc * WN + j * 16 + (lane & 15);
          bfr[j] = *(const bf16x8*)(bsh + row * BK + swz<BK>(row, chunk) * 8);
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
      if (kt + 1 < nk) store_ab(buf ^ 1);
      __syncthreads();
    }

    // ---- epilogue: BN partial stats + bf16 tile through LDS ----
    if (p.stats != nullptr) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        float s = 0.f, q = 0.f;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int m = m0 + wr * WM + i * 16 + (lane >> 4) * 4 + r;
            const float v = (m < p.M) ? acc[i][j][r] : 0.f;
            s += v;
            q += v * v;
          }
        s += __shfl_xor(s, 16, 64);
        s += __shfl_xor(s, 32, 64);
        q += __shfl_xor(q, 16, 64);
        q += __shfl_xor(q, 32, 64);
        st_s[j] += s;
        st_q[j] += q;
      }
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = wr * WM + i * 16 + (lane >> 4) * 4 + r;
          const int col = wc * WN + j * 16 + (lane & 15);
          Es[row * (BN + EPAD) + col] = f2bf(acc[i][j][r]);
        }
    __syncthreads();
    constexpr int OCPR = BN / 8;
#pragma unroll
    for (int it = 0; it < BM * OCPR / 256; ++it) {
      const int cid = tid + it * 256;
      const int row = cid / OCPR, cc = cid % OCPR;
      const int m = m0 + row, n = n0 + cc * 8;
      if (m < p.M && n < p.Cout) {
        *(uint4*)(p.y + (long long)m * p.ldy + n) = *(const uint4*)(Es + row * (BN + EPAD) + cc * 8);
      }
    }
    __syncthreads();
  }

  if (p.stats != nullptr) {
    // combine the two M-waves (wr = 0, 1) that own the same columns, then one store per column.
    float* red = (float*)smem;  // [2 (wc)][2 (s,q)][WN]
    if (wr == 1 && lane < 16) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        red[(wc * 2 + 0) * WN + j * 16 + lane] = st_s[j];
        red[(wc * 2 + 1) * WN + j * 16 + lane] = st_q[j];
      }
    }
    __syncthreads();
    if (wr == 0 && lane < 16) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = n0 + wc * WN + j * 16 + lane;
        const float s = st_s[j] + red[(wc * 2 + 0) * WN + j * 16 + lane];
        const float q = st_q[j] + red[(wc * 2 + 1) * WN + j * 16 + lane];
        const int npad = p.num_n_tiles * BN;
        p.stats[(long long)m_slot * 2 * npad + col] = s;
        p.stats[(long long)m_slot * 2 * npad + npad + col] = q;
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// wgrad: dW[n, k] partial over an m-range -> slab[split][Npad][Kpad] (fp32)
struct WgradParams {
  const bf16_t* dy;    // [M, ldd] bf16
  const void* x;       // [B, T, H, W, Cin]
  float* slab;         // [splits][Npad][Kpad]
  long long x_bstride;
  int T, H, W, Cin;
  int To, Ho, Wo, Cout, ldd;
  int KT, KH, KW, st, sh, sw, pt, ph, pw;
  int Ktot, Kpad, Npad, M;
  int n_tiles, k_tiles, splits, rows_per_split;
  float in_scale;
  FastDiv fWo, fHo, fTo;
};

template <int TN_, int TK_, bool U8>
__global__ __launch_bounds__(256) void conv_wgrad_kernel(WgradParams p) {
  constexpr int R = 32;                     // reduction rows per step (one MFMA K)
  constexpr int VEC = U8 ? 4 : 8;
  constexpr int LDN = TN_ + 16, LDK = TK_ + 16;  // padded row lengths (elements)
  constexpr int D_CPR = TN_ / 8, X_CPR = TK_ / VEC;
  constexpr int D_CH = R * D_CPR / 256, X_CH = R * X_CPR / 256;
  constexpr int WN = TN_ / 2, WK = TK_ / 2;
  constexpr int TI = WN / 16, TJ = WK / 16;
  static_assert(D_CH >= 1 && X_CH >= 1, "tile too small");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* Ds = (bf16_t*)smem;               // [2][R][LDN]
  bf16_t* Xs = Ds + 2 * R * LDN;            // [2][R][LDK]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int nblocks = p.n_tiles * p.k_tiles * p.splits;
  const int logical = xcd_remap(blockIdx.x, nblocks);
  const int tile = logical / p.splits;
  const int split = logical % p.splits;
  const int n0 = (tile % p.n_tiles) * TN_;
  const int k0 = (tile / p.n_tiles) * TK_;
  const int m_begin = split * p.rows_per_split;
  const int m_end = min(p.M, m_begin + p.rows_per_split);

  // fixed (tap, c) of this thread's X chunk column
  const int x_ccol = tid % X_CPR;
  const int kk = k0 + x_ccol * VEC;
  int tap = kk / p.Cin;
  const int c = kk - tap * p.Cin;
  const bool kval = kk < p.Ktot;
  const int dw = tap % p.KW;
  const int dh = (tap / p.KW) % p.KH;
  const int dt = tap / (p.KW * p.KH);
  const int d_ccol = tid % D_CPR;
  const uint8_t* xb = (const uint8_t*)p.x;
  const int esize = U8 ? 1 : 2;

  using XReg = typename std::conditional<U8, uint32_t, uint4>::type;
  uint4 dreg[D_CH];
  XReg xreg[X_CH];

  auto load = [&](int mb) {
#pragma unroll
    for (int i = 0; i < D_CH; ++i) {
      const int row = (tid + i * 256) / D_CPR;
      const int m = mb + row;
      const int n = n0 + d_ccol * 8;
      dreg[i] = make_uint4(0, 0, 0, 0);
      if (m < m_end && n < p.Cout) dreg[i] = *(const uint4*)(p.dy + (long long)m * p.ldd + n);
    }
#pragma unroll
    for (int i = 0; i < X_CH; ++i) {
      const int row = (tid + i * 256) / X_CPR;
      const int m = mb + row;
      bool v = kval && m < m_end;
      long long off = 0;
      if (v) {
        uint32_t q = fdiv((uint32_t)m, p.fWo);
        const int wo = m - q * p.Wo;
        uint32_t q2 = fdiv(q, p.fHo);
        const int ho = q - q2 * p.Ho;
        uint32_t b = fdiv(q2, p.fTo);
        const int to = q2 - b * p.To;
        const int ti = to * p.st - p.pt + dt, hi = ho * p.sh - p.ph + dh, wi = wo * p.sw - p.pw + dw;
        v = (unsigned)ti < (unsigned)p.T && (unsigned)hi < (unsigned)p.H && (unsigned)wi < (unsigned)p.W;
        off = (long long)b * p.x_bstride + ((long long)(ti * p.H + hi) * p.W + wi) * p.Cin + c;
      }
      if constexpr (U8) {
        xreg[i] = v ? *(const uint32_t*)(xb + off) : 0u;
      } else {
        xreg[i] = v ? *(const uint4*)(xb + off * 2) : make_uint4(0, 0, 0, 0);
      }
    }
  };
  auto store = [&](int buf) {
    bf16_t* d = Ds + buf * R * LDN;
#pragma unroll
    for (int i = 0; i < D_CH; ++i) {
      const int row = (tid + i * 256) / D_CPR;
      *(uint4*)(d + row * LDN + d_ccol * 8) = dreg[i];
    }
    bf16_t* x = Xs + buf * R * LDK;
#pragma unroll
    for (int i = 0; i < X_CH; ++i) {
      const int row = (tid + i * 256) / X_CPR;
      if constexpr (U8) {
        const uint32_t v = xreg[i];
        const float s = p.in_scale;
        uint2 o;
        o.x = pack2bf((float)(v & 0xff) * s, (float)((v >> 8) & 0xff) * s);
        o.y = pack2bf((float)((v >> 16) & 0xff) * s, (float)(v >> 24) * s);
        *(uint2*)(x + row * LDK + x_ccol * 4) = o;
      } else {
        *(uint4*)(x + row * LDK + x_ccol * 8) = xreg[i];
      }
    }
  };

  f32x4 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // transposed-read lane geometry: group g = lane>>4 reads rows 4g+q (+16), cols 4p..4p+3
  const int g = lane >> 4, li = lane & 15, q = li >> 2, pp = li & 3;
  const int nsteps = (m_end - m_begin + R - 1) / R;
  if (nsteps > 0) {
    load(m_begin);
    store(0);
  }
  __syncthreads();
  for (int s = 0; s < nsteps; ++s) {
    const int buf = s & 1;
    if (s + 1 < nsteps) load(m_begin + (s + 1) * R);
    const bf16_t* d = Ds + buf * R * LDN;
    const bf16_t* x = Xs + buf * R * LDK;
    bf16x8 af[TI], bfr[TJ];
#pragma unroll
    for (int i = 0; i < TI; ++i) {
      const int col = wr * WN + i * 16 + pp * 4;
      const bf16_t* a0 = d + (4 * g + q) * LDN + col;
      const bf16_t* a1 = d + (16 + 4 * g + q) * LDN + col;
      s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)a0);
      s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)a1);
      s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      af[i] = __builtin_bit_cast(bf16x8, v);
    }
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int col = wc * WK + j * 16 + pp * 4;
      const bf16_t* b0 = x + (4 * g + q) * LDK + col;
      const bf16_t* b1 = x + (16 + 4 * g + q) * LDK + col;
      s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)b0);
      s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)b1);
      s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      bfr[j] = __builtin_bit_cast(bf16x8, v);
    }
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    if (s + 1 < nsteps) store(buf ^ 1);
    __syncthreads();
  }
  // C[i = n][j = k]: row (n) = 4*(lane>>4) + r, col (k) = lane & 15
  float* out = p.slab + (long long)split * p.Npad * p.Kpad;
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + wr * WN + i * 16 + (lane >> 4) * 4 + r;
        const int k = k0 + wc * WK + j * 16 + (lane & 15);
        out[(long long)n * p.Kpad + k] = acc[i][j][r];
      }
}

// Sum the split slabs and unpack [n][tap][c] -> PyTorch weight layout [n][c_param][tap].
__global__ void wgrad_reduce_kernel(const float* __restrict__ slab, float* __restrict__ dw, int splits,
                                    int Npad, int Kpad, int Cout, int Cin, int Cin_param, int taps,
                                    int accumulate) {
  const long long total = (long long)Cout * Cin_param * taps;
  for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < total;
       idx += (long long)gridDim.x * blockDim.x) {
    const int tap = idx % taps;
    const long long t2 = idx / taps;
    const int c = t2 % Cin_param;
    const int n = t2 / Cin_param;
    const long long k = (long long)tap * Cin + c;
    float s = 0.f;
    for (int sp = 0; sp < splits; ++sp) s += slab[((long long)sp * Npad + n) * Kpad + k];
    dw[idx] = accumulate ? dw[idx] + s : s;
  }
}

// ---------------------------------------------------------------------------------------
// Weight packing: fp32 [Cout][Cin_p][KT][KH][KW] -> bf16 [Npad][Kpad]
//   mode 0 (forward): row n = cout, k = (tap, c)        with c < Cin (c >= Cin_p -> 0)
//   mode 1 (dgrad)  : row n = cin,  k = (tap', cout)    with tap' = flipped tap
__global__ void pack_weight_kernel(const float* __restrict__ w, bf16_t* __restrict__ out, int Cout, int Cin,
                                   int Cin_p, int KT, int KH, int KW, int Npad, int Kpad, int mode) {
  const int taps = KT * KH * KW;
  const long long total = (long long)Npad * Kpad;
  for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < total;
       idx += (long long)gridDim.x * blockDim.x) {
    const int n = idx / Kpad;
    const int k = idx % Kpad;
    float v = 0.f;
    if (mode == 0) {
      const int tap = k / Cin, c = k % Cin;
      if (n < Cout && tap < taps && c < Cin_p) v = w[((long long)n * Cin_p + c) * taps + tap];
    } else {
      // dgrad: output channel = cin index n; reduction over (tap', cout)
      const int tap2 = k / Cout, co = k % Cout;
      if (n < Cin_p && tap2 < taps) {
        const int tap = taps - 1 - tap2;  // flip all three kernel dims at once
        v = w[((long long)co * Cin_p + n) * taps + tap];
      }
    }
    out[idx] = f2bf(v);
  }
}

// ---------------------------------------------------------------------------------------
template <int BM, int BN, int BK, bool U8>
static int launch_fwd(ConvParams& p, hipStream_t stream) {
  const size_t kloop = (size_t)2 * (BM + BN) * BK * 2;
  const size_t epi = (size_t)BM * (BN + 16) * 2;
  const size_t lds = kloop > epi ? kloop : epi;
  static bool attr_set = false;
  if (!attr_set) {
    HIP_RET(hipFuncSetAttribute((const void*)conv_fwd_kernel<BM, BN, BK, U8>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr_set = true;
  }
  const int nblocks = p.num_n_tiles * p.grid_m;
  hipLaunchKernelGGL((conv_fwd_kernel<BM, BN, BK, U8>), dim3(nblocks), dim3(256), lds, stream, p);
  return (int)hipGetLastError();
}

// x: input, w: packed weight [Npad][Kpad], y: out [M][ldy], stats: [grid_m][2][Npad] or null.
// Returns grid_m through *grid_m_out (for sizing the stats buffer, call with y == nullptr).
MILNCE_API int milnce_conv_fwd(const void* x, int x_u8, const void* w, void* y, float* stats,
                               int B, int T, int H, int W, int Cin, int Cout,
                               int KT, int KH, int KW, int st, int sh, int sw, int pt, int ph, int pw,
                               int Kpad, int Npad, int ldy, int bn, int bk, int grid_m,
                               hipStream_t stream) {
  ConvParams p;
  p.x = x; p.w = (const bf16_t*)w; p.y = (bf16_t*)y; p.stats = stats;
  p.T = T; p.H = H; p.W = W; p.Cin = Cin;
  p.To = (T + 2 * pt - KT) / st + 1;
  p.Ho = (H + 2 * ph - KH) / sh + 1;
  p.Wo = (W + 2 * pw - KW) / sw + 1;
  p.Cout = Cout;
  p.KT = KT; p.KH = KH; p.KW = KW; p.st = st; p.sh = sh; p.sw = sw; p.pt = pt; p.ph = ph; p.pw = pw;
  p.Ktot = KT * KH * KW * Cin; p.Kpad = Kpad; p.ldy = ldy;
  p.M = B * p.To * p.Ho * p.Wo;
  p.x_bstride = (long long)T * H * W * Cin;
  const int BM = 128;
  p.num_m_tiles = (p.M + BM - 1) / BM;
  p.num_n_tiles = Npad / bn;
  p.grid_m = grid_m;
  p.in_scale = x_u8 ? (1.0f / 255.0f) : 1.0f;
  p.fWo = make_fastdiv(p.Wo); p.fHo = make_fastdiv(p.Ho); p.fTo = make_fastdiv(p.To);
  if (x_u8) {
    if (bn == 64 && bk == 32) return launch_fwd<128, 64, 32, true>(p, stream);
    if (bn == 64 && bk == 64) return launch_fwd<128, 64, 64, true>(p, stream);
    if (bn == 128 && bk == 32) return launch_fwd<128, 128, 32, true>(p, stream);
    if (bn == 128 && bk == 64) return launch_fwd<128, 128, 64, true>(p, stream);
  } else {
    if (bn == 64 && bk == 32) return launch_fwd<128, 64, 32, false>(p, stream);
    if (bn == 64 && bk == 64) return launch_fwd<128, 64, 64, false>(p, stream);
    if (bn == 128 && bk == 32) return launch_fwd<128, 128, 32, false>(p, stream);
    if (bn == 128 && bk == 64) return launch_fwd<128, 128, 64, false>(p, stream);
  }
  return (int)hipErrorInvalidValue;
}

template <int TN_, int TK_, bool U8>
static int launch_wgrad(WgradParams& p, hipStream_t stream) {
  const size_t lds = (size_t)2 * 32 * ((TN_ + 16) + (TK_ + 16)) * 2;
  const int nblocks = p.n_tiles * p.k_tiles * p.splits;
  hipLaunchKernelGGL((conv_wgrad_kernel<TN_, TK_, U8>), dim3(nblocks), dim3(256), lds, stream, p);
  return (int)hipGetLastError();
}

MILNCE_API int milnce_conv_wgrad(const void* dy, int ldd, const void* x, int x_u8, float* slab, float* dw,
                                 int B, int T, int H, int W, int Cin, int Cin_param, int Cout,
                                 int KT, int KH, int KW, int st, int sh, int sw, int pt, int ph, int pw,
                                 int Kpad, int Npad, int tn, int tk, int splits, int accumulate,
                                 hipStream_t stream) {
  WgradParams p;
  p.dy = (const bf16_t*)dy; p.x = x; p.slab = slab;
  p.T = T; p.H = H; p.W = W; p.Cin = Cin;
  p.To = (T + 2 * pt - KT) / st + 1;
  p.Ho = (H + 2 * ph - KH) / sh + 1;
  p.Wo = (W + 2 * pw - KW) / sw + 1;
  p.Cout = Cout; p.ldd = ldd;
  p.KT = KT; p.KH = KH; p.KW = KW; p.st = st; p.sh = sh; p.sw = sw; p.pt = pt; p.ph = ph; p.pw = pw;
  p.Ktot = KT * KH * KW * Cin; p.Kpad = Kpad; p.Npad = Npad;
  p.M = B * p.To * p.Ho * p.Wo;
  p.x_bstride = (long long)T * H * W * Cin;
  p.n_tiles = Npad / tn;
  p.k_tiles = Kpad / tk;
  p.splits = splits;
  p.rows_per_split = ((p.M + splits - 1) / splits + 31) / 32 * 32;
  p.in_scale = x_u8 ? (1.0f / 255.0f) : 1.0f;
  p.fWo = make_fastdiv(p.Wo); p.fHo = make_fastdiv(p.Ho); p.fTo = make_fastdiv(p.To);
  int rc;
  if (x_u8) {
    if (tn == 64 && tk == 64) rc = launch_wgrad<64, 64, true>(p, stream);
    else if (tn == 64 && tk == 128) rc = launch_wgrad<64, 128, true>(p, stream);
    else rc = (int)hipErrorInvalidValue;
  } else {
    if (tn == 64 && tk == 64) rc = launch_wgrad<64, 64, false>(p, stream);
    else if (tn == 64 && tk == 128) rc = launch_wgrad<64, 128, false>(p, stream);
    else if (tn == 128 && tk == 64) rc = launch_wgrad<128, 64, false>(p, stream);
    else if (tn == 128 && tk == 128) rc = launch_wgrad<128, 128, false>(p, stream);
    else rc = (int)hipErrorInvalidValue;
  }
  if (rc) return rc;
  const int taps = KT * KH * KW;
  const long long total = (long long)Cout * Cin_param * taps;
  const int grid = (int)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(grid), dim3(256), 0, stream, slab, dw, splits, Npad, Kpad,
                     Cout, Cin, Cin_param, taps, accumulate);
  return (int)hipGetLastError();
}

MILNCE_API int milnce_pack_weight(const float* w, void* out, int Cout, int Cin, int Cin_p, int KT, int KH,
                                  int KW, int Npad, int Kpad, int mode, hipStream_t stream) {
  const long long total = (long long)Npad * Kpad;
  const int grid = (int)((total + 255) / 256 < 2048 ? (total + 255) / 256 : 2048);
  hipLaunchKernelGGL(pack_weight_kernel, dim3(grid), dim3(256), 0, stream, w, (bf16_t*)out, Cout, Cin, Cin_p,
                     KT, KH, KW, Npad, Kpad, mode);
  return (int)hipGetLastError();
}
