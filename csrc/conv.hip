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
#include "conv_common.h"

// Tap table entry: .x = element offset of the tap inside a clip ((dt*H + dh)*W + dw)*Cin,
// .y = dt | dh << 8 | dw << 16.
__device__ __forceinline__ void build_tap_table(int2* tab, int KT, int KH, int KW, int H, int W, int Cin) {
  const int taps = KT * KH * KW;
  for (int t = threadIdx.x; t < taps; t += blockDim.x) {
    const int dw = t % KW, dh = (t / KW) % KH, dt = t / (KW * KH);
    tab[t] = make_int2(((dt * H + dh) * W + dw) * Cin, dt | (dh << 8) | (dw << 16));
  }
}

template <int N, int CPR, int BK>
__device__ __forceinline__ void load_w_tile(uint4 (&r)[N], const bf16_t* __restrict__ w, int n0, int Kpad, int kt,
                                            int tid, int ccol) {
  const bf16_t* base = w + (long long)n0 * Kpad + kt * BK + ccol * 8;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const int row = (tid + i * 256) / CPR;
    r[i] = *(const uint4*)(base + (long long)row * Kpad);
  }
}

// Implicit-im2col gather of this thread's A chunks for K tile kt (buffer loads: out-of-range
// offsets return zero, so padding, tail rows and K padding are branch-free).
template <int N, int VEC, int ESZ, int BK, bool U8, typename AReg>
__device__ __forceinline__ void gather_a_tile(AReg (&areg)[N], __amdgpu_buffer_rsrc_t rsrc, const int2* tab,
                                              const ConvParams& p, const int (&rt)[N], const int (&rh)[N],
                                              const int (&rw)[N], const uint32_t (&rowoff)[N], int kt, int a_ccol,
                                              int taps) {
  const int k = kt * BK + a_ccol * VEC;
  const int tap = (int)fdiv((uint32_t)k, p.fCin);
  const int c = k - tap * p.Cin;
  const bool kval = tap < taps;
  const int2 te = tab[min(tap, taps - 1)];  // unconditional: no exec-mask branch
  const int dt = te.y & 0xff, dh = (te.y >> 8) & 0xff, dw = te.y >> 16;
  const uint32_t koff = (uint32_t)((te.x + c) * ESZ);
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const int ti = rt[i] + dt, hi = rh[i] + dh, wi = rw[i] + dw;
    const bool v = kval & ((unsigned)ti < (unsigned)p.T) & ((unsigned)hi < (unsigned)p.H) &
                   ((unsigned)wi < (unsigned)p.W);
    const uint32_t off = v ? rowoff[i] + koff : 0x80000000u;  // > num_records: reads 0
    if constexpr (U8) {
      areg[i] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rsrc, off, 0, 0);
    } else {
      auto r = __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, 0);
      areg[i] = __builtin_bit_cast(uint4, r);
    }
  }
}

template <int NA, int NB, int A_CPR, int B_CPR, int BM, int BN, int BK, bool U8, typename AReg>
__device__ __forceinline__ void store_tiles(const AReg (&areg)[NA], const uint4 (&breg)[NB], bf16_t* As, bf16_t* Bs,
                                            int buf, int tid, int a_ccol, int b_ccol, float in_scale) {
  bf16_t* a = As + buf * BM * BK;
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int row = (tid + i * 256) / A_CPR;
    if constexpr (U8) {
      const uint32_t v = areg[i];
      uint2 o;
      o.x = pack2bf((float)(v & 0xff) * in_scale, (float)((v >> 8) & 0xff) * in_scale);
      o.y = pack2bf((float)((v >> 16) & 0xff) * in_scale, (float)(v >> 24) * in_scale);
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
  for (int i = 0; i < NB; ++i) {
    const int row = (tid + i * 256) / B_CPR;
    const int ch = swz<BK>(row, b_ccol);
    *(uint4*)(bsh + row * BK + ch * 8) = breg[i];
  }
}

// A operand of the MFMA = weight tile (rows n), B operand = gathered activations (cols m), so
// each lane's accumulator holds 4 consecutive output channels of one output position: the
// epilogue packs them into 8-byte LDS writes and the per-channel BN sums accumulate per lane
// across the persistent M loop (one cross-lane reduction per kernel, not per tile).
// EPI (compile time, so the plain forward does not carry the backward epilogue's registers):
// 0 no statistics, 1 BN forward sums, 2 producer-BN backward partials (see ConvParams).
// __launch_bounds__(256, 2): 2 waves per SIMD = 2 blocks per CU (VGPR budget 256).
template <int BM, int BN, int BK, bool U8, int EPI>
__global__ __launch_bounds__(256, 2) void conv_fwd_kernel(ConvParams p) {
  constexpr int VEC = U8 ? 4 : 8;
  constexpr int ESZ = U8 ? 1 : 2;
  constexpr int A_CPR = BK / VEC;
  constexpr int A_CH = BM * A_CPR / 256;
  constexpr int B_CPR = BK / 8;
  constexpr int B_CH = BN * B_CPR / 256;
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int KSTEPS = BK / 32;
  constexpr int LDE = BN + 8;  // epilogue staging row (elements): 16-B aligned, 2-way max on b64 writes
  constexpr int KLOOP_ELEMS = 2 * (BM + BN) * BK;
  constexpr int EPI_ELEMS = BM * LDE;
  constexpr int TAB_OFF_BYTES = 2 * (KLOOP_ELEMS > EPI_ELEMS ? KLOOP_ELEMS : EPI_ELEMS);
  static_assert(A_CH >= 1 && B_CH >= 1, "tile too small");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* As = (bf16_t*)smem;          // [2][BM][BK]   activations (MFMA B operand)
  bf16_t* Bs = As + 2 * BM * BK;       // [2][BN][BK]   weights     (MFMA A operand)
  bf16_t* Es = (bf16_t*)smem;          // epilogue [BM][LDE]
  int2* tab = (int2*)(smem + TAB_OFF_BYTES);
  float* ssl = (float*)(smem + TAB_OFF_BYTES + 8 * 160);  // [4][BN] producer-BN constants (mode 2)

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
  KASSERT(nk * BK == p.Kpad && (int)blockIdx.x < p.num_n_tiles * p.grid_m);
  const int a_ccol = tid % A_CPR;
  const int b_ccol = tid % B_CPR;
  const int taps = p.KT * p.KH * p.KW;
  const uint32_t thw = (uint32_t)p.To * p.Ho * p.Wo;
  const uint32_t clip_bytes = (uint32_t)(p.x_bstride * ESZ);

  build_tap_table(tab, p.KT, p.KH, p.KW, p.H, p.W, p.Cin);
  if constexpr (EPI == 2) {
    for (int t = tid; t < 4 * BN; t += 256) {
      const int q = t / BN, c = n0 + (t - q * BN);
      ssl[t] = c < p.Cout ? p.bn_ss[q * p.Cout + c] : 0.f;
    }
  }
  float st_s[TN][4], st_q[TN][4];
  float e_s[8], e_q[8];  // EPI 2: partials of this thread's fixed 8-channel chunk (tid % (BN/8))
  // EPI 1: per-channel shift (bn_ss, when set: the BN's running mean) subtracted before the bf16
  // rounding, so the stored pre-BN values keep their precision when |mean| >> std
  float shv[TN][4];
#pragma unroll
  for (int k = 0; k < 8; ++k) { e_s[k] = 0.f; e_q[k] = 0.f; }
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      st_s[j][r] = 0.f;
      st_q[j][r] = 0.f;
      const int n = n0 + wc * WN + j * 16 + (lane >> 4) * 4 + r;
      shv[j][r] = (EPI == 1 && p.bn_ss != nullptr && n < p.Cout) ? p.bn_ss[n] : 0.f;
    }

  for (int m_tile = m_slot; m_tile < p.num_m_tiles; m_tile += p.grid_m) {
    const int m0 = m_tile * BM;
    // Buffer descriptor based at the tile's first clip: out-of-range offsets read as zero, so
    // padding / tail rows / K padding need no branches around the loads.
    const uint32_t b0 = (uint32_t)m0 / thw;
    const char* base = (const char*)p.x + (long long)b0 * p.x_bstride * ESZ;
    const long long remain = p.x_total_bytes - (long long)b0 * p.x_bstride * ESZ;
    const uint32_t nrec = remain > 0x7FFFFFF0LL ? 0x7FFFFFF0u : (uint32_t)remain;
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)nrec, 0x00020000);

    int rt[A_CH], rh[A_CH], rw[A_CH];
    uint32_t rowoff[A_CH];  // byte offset of the (unshifted) row origin relative to base
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
        rt[i] = to * p.st - p.pt;
        rh[i] = ho * p.sh - p.ph;
        rw[i] = wo * p.sw - p.pw;
        rowoff[i] = (b - b0) * clip_bytes + (uint32_t)(((rt[i] * p.H + rh[i]) * p.W + rw[i]) * p.Cin * ESZ);
      } else {
        rt[i] = -(1 << 28);
        rh[i] = 0;
        rw[i] = 0;
        rowoff[i] = 0;
      }
    }

    using AReg = typename std::conditional<U8, uint32_t, uint4>::type;
    AReg areg[A_CH];
    uint4 breg[B_CH];

    f32x4 acc[TN][TM];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int i = 0; i < TM; ++i) acc[j][i] = (f32x4){0.f, 0.f, 0.f, 0.f};

    __syncthreads();  // tap table ready / previous tile's epilogue done with LDS
    gather_a_tile<A_CH, VEC, ESZ, BK, U8>(areg, rsrc, tab, p, rt, rh, rw, rowoff, 0, a_ccol, taps);
    load_w_tile<B_CH, B_CPR, BK>(breg, p.w, n0, p.Kpad, 0, tid, b_ccol);
    store_tiles<A_CH, B_CH, A_CPR, B_CPR, BM, BN, BK, U8>(areg, breg, As, Bs, 0, tid, a_ccol, b_ccol, p.in_scale);
    __syncthreads();

    for (int kt = 0; kt < nk; ++kt) {
      const int buf = kt & 1;
      // Always prefetch (the last iteration re-loads the last tile into the free buffer):
      // keeping the staging path unconditional lets the compiler hold it in registers.
      const int kn = min(kt + 1, nk - 1);
      gather_a_tile<A_CH, VEC, ESZ, BK, U8>(areg, rsrc, tab, p, rt, rh, rw, rowoff, kn, a_ccol, taps);
      load_w_tile<B_CH, B_CPR, BK>(breg, p.w, n0, p.Kpad, kn, tid, b_ccol);
      const bf16_t* a = As + buf * BM * BK;
      const bf16_t* bsh = Bs + buf * BN * BK;
#pragma unroll
      for (int s = 0; s < KSTEPS; ++s) {
        bf16x8 xf[TM], wf[TN];
        const int chunk = s * 4 + (lane >> 4);
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int row = wr * WM + i * 16 + (lane & 15);
          xf[i] = *(const bf16x8*)(a + row * BK + swz<BK>(row, chunk) * 8);
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int row = wc * WN + j * 16 + (lane & 15);
          wf[j] = *(const bf16x8*)(bsh + row * BK + swz<BK>(row, chunk) * 8);
        }
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int i = 0; i < TM; ++i)
            acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], xf[i], acc[j][i], 0, 0, 0);
      }
      store_tiles<A_CH, B_CH, A_CPR, B_CPR, BM, BN, BK, U8>(areg, breg, As, Bs, buf ^ 1, tid, a_ccol, b_ccol,
                                                            p.in_scale);
      __syncthreads();
    }

    // ---- epilogue: lane holds channels n = 4*(lane>>4)+r of output row m = lane&15 ----
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row = wr * WM + i * 16 + (lane & 15);
      const bool rv = (m0 + row) < p.M;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        f32x4 v = acc[j][i];
        if constexpr (EPI == 1) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] -= shv[j][r];
          if (rv) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            st_s[j][r] += v[r];
            st_q[j][r] += v[r] * v[r];
          }
          }
        }
        uint2 o;
        o.x = pack2bf(v[0], v[1]);
        o.y = pack2bf(v[2], v[3]);
        const int col = wc * WN + j * 16 + (lane >> 4) * 4;
        *(uint2*)(Es + row * LDE + col) = o;
      }
    }
    __syncthreads();
    constexpr int OCPR = BN / 8;
#pragma unroll
    for (int it = 0; it < BM * OCPR / 256; ++it) {
      const int cid = tid + it * 256;
      const int row = cid / OCPR, cc = cid % OCPR;
      const int m = m0 + row, n = n0 + cc * 8;
      const uint4 dv = *(const uint4*)(Es + row * LDE + cc * 8);
      const bool ok = (m < p.M) & (n < p.Cout);
      if (ok) *(uint4*)(p.y + (long long)m * p.ldy + n) = dv;
      if constexpr (EPI == 2) {
        // BN-backward partials from the bf16 dz actually stored (same values the standalone
        // reduction would read); the chunk column cc == tid % OCPR is fixed for this thread.
        if (ok) {
          float d8[8], y8[8];
          unpack8(dv, d8);
          unpack8(*(const uint4*)(p.bn_y + (long long)m * p.bn_ld + n), y8);
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const int cl = cc * 8 + k;
            const float gm = (y8[k] * ssl[2 * BN + cl] + ssl[3 * BN + cl] > 0.f) ? d8[k] : 0.f;
            e_s[k] += gm;
            e_q[k] += gm * (y8[k] - ssl[cl]) * ssl[BN + cl];
          }
        }
      }
    }
  }

  if constexpr (EPI == 2) {
    constexpr int OCPR = BN / 8;
    __syncthreads();
    float* red = (float*)smem;  // [2][8][256]
#pragma unroll
    for (int k = 0; k < 8; ++k) { red[k * 256 + tid] = e_s[k]; red[(8 + k) * 256 + tid] = e_q[k]; }
    __syncthreads();
    if (tid < OCPR) {
      const int npad = p.num_n_tiles * BN;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float s1 = 0.f, s2 = 0.f;
        for (int j = tid; j < 256; j += OCPR) { s1 += red[k * 256 + j]; s2 += red[(8 + k) * 256 + j]; }
        const int col = n0 + tid * 8 + k;
        p.stats[(long long)m_slot * 2 * npad + col] = s1;
        p.stats[(long long)m_slot * 2 * npad + npad + col] = s2;
      }
    }
  }

  if constexpr (EPI == 1) {
    // reduce over the 16 lanes (output rows) that share a channel group, then over wr
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float s = st_s[j][r], q = st_q[j][r];
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          s += __shfl_xor(s, o, 64);
          q += __shfl_xor(q, o, 64);
        }
        st_s[j][r] = s;
        st_q[j][r] = q;
      }
    __syncthreads();
    float* red = (float*)smem;  // [2 (wc)][2 (s,q)][WN]
    if (wr == 1 && (lane & 15) == 0) {
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int c = j * 16 + (lane >> 4) * 4 + r;
          red[(wc * 2 + 0) * WN + c] = st_s[j][r];
          red[(wc * 2 + 1) * WN + c] = st_q[j][r];
        }
    }
    __syncthreads();
    if (wr == 0 && (lane & 15) == 0) {
      const int npad = p.num_n_tiles * BN;
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int c = j * 16 + (lane >> 4) * 4 + r;
          const int col = n0 + wc * WN + c;
          p.stats[(long long)m_slot * 2 * npad + col] = st_s[j][r] + red[(wc * 2 + 0) * WN + c];
          p.stats[(long long)m_slot * 2 * npad + npad + col] = st_q[j][r] + red[(wc * 2 + 1) * WN + c];
        }
    }
  }
}

// ---------------------------------------------------------------------------------------
// v3 forward / dgrad (bf16 input): both operand tiles are fetched global -> LDS directly by
// buffer_load ... lds (LDS-DMA: no staging VGPRs, no ds_write pass) into a STAGES-deep ring, with
// the tile for k-step kt + STAGES - 1 in flight while kt is computed; a counted vmcnt + raw
// s_barrier retire one stage per k-step (a __syncthreads() would drain every DMA in flight).
// The LDS image stays XOR-swizzled: a DMA writes lane-linearly, so each lane instead fetches the
// source chunk that belongs in its slot. Wave w's j-th DMA of a tile covers rows
// j*4*RPI + w*RPI + lane/CPR, so the swizzle term -- and hence the lane's k chunk and its
// (tap, channel) -- is the same for all of the lane's rows: one tap lookup per stage.
// Workgroup barrier for the LDS-DMA rings. __builtin_amdgcn_s_barrier() is not a memory barrier
// for the compiler (LDS reads could be hoisted above it, i.e. before other waves' DMA pieces
// for the stage have landed), and __syncthreads() would add a vmcnt(0) that drains the ring.
#ifndef V3_PRIO_DEFAULT
#define V3_PRIO_DEFAULT 1
#endif
constexpr bool V3_PRIO = V3_PRIO_DEFAULT;
// software-pipelined fragment reads inside a stage (BK 64: two k-steps per barrier)
#ifndef V3_PIPE_DEFAULT
#define V3_PIPE_DEFAULT 1
#endif
constexpr bool V3_PIPE = V3_PIPE_DEFAULT;
// the same for the register-staged wgrad (conv_wgrad_kernel): measured equal (same-box bench
// 4122.0 vs 4122.4 pairs/s), off
#ifndef WG_PIPE_DEFAULT
#define WG_PIPE_DEFAULT 0
#endif
constexpr bool WG_PIPE = WG_PIPE_DEFAULT;

// NWM waves along M (each wave a 64 x BN/2 sub-tile, 2 waves along N): BM = 64*NWM rows,
// 128*NWM threads. NWM = 4 (256 x BN tiles, 8 waves) re-reads each operand byte fewer times.
template <int BN, int BK, int STAGES, int EPI, int NWM>
__global__ __launch_bounds__(128 * NWM, 1) void conv_fwd_v3_kernel(ConvParams p) {
  constexpr int BM = 64 * NWM;
  constexpr int NT = 128 * NWM;            // threads
  constexpr int NWAVES = 2 * NWM;
  constexpr int CPR = BK / 8;              // 16-B chunks per tile row
  constexpr int RPI = 64 / CPR;            // rows per DMA instruction (1 KiB)
  constexpr int A_INST = BM / RPI / NWAVES;  // DMA instructions per wave per stage (A)
  constexpr int B_INST = BN / RPI / NWAVES;  // (B)
  constexpr int NDMA = A_INST + B_INST;
  constexpr int WM = BM / NWM, WN = BN / 2;  // wave tile: 64 rows x BN/2
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int KSTEPS = BK / 32;
  constexpr int LDE = BN + 8;
  constexpr int STAGE_ELEMS = (BM + BN) * BK;
  constexpr int RING_BYTES = STAGES * STAGE_ELEMS * 2;
  constexpr int EPI_BYTES = BM * LDE * 2;
  // the producer-BN constants (EPI 2) sit behind the epilogue staging, inside the drained ring
  // when it is large enough: the whole kernel then needs only the ring's LDS (two 80 KiB
  // workgroups per CU at BN 192 x BK 64 x 2 stages, i.e. two waves per SIMD)
  constexpr int SSL_BYTES = EPI == 2 ? 16 * BN : 0;
  static_assert(A_INST >= 1 && B_INST >= 1, "tile too small for the DMA mapping");
  static_assert(BM % (RPI * NWAVES) == 0 && BN % (RPI * NWAVES) == 0, "tile rows must split evenly over the DMAs");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* ring = (bf16_t*)smem;  // stage s: A [BM][BK] then B [BN][BK]
  bf16_t* Es = (bf16_t*)smem;    // epilogue staging [BM][LDE] (after the ring drained)
  float* ssl = (float*)(smem + EPI_BYTES);  // [4][BN] producer-BN constants (EPI 2), per tile
  // EPI 1 shift of the block's (fixed) N tile, behind everything else: written once, read by every
  // tile's epilogue from LDS (loaded per tile from global memory it cost a full vmcnt drain there)
  constexpr int SHL_OFF = RING_BYTES > EPI_BYTES + SSL_BYTES ? RING_BYTES : EPI_BYTES + SSL_BYTES;
  float* shl = (float*)(smem + SHL_OFF);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: LDS-DMA bases go to M0
  const int wr = wave >> 1, wc = wave & 1;  // wr in [0, NWM)
  const int nblocks = p.num_n_tiles * p.grid_m;
  const int logical = xcd_remap(blockIdx.x, nblocks);
  const int n_tile = logical % p.num_n_tiles;
  const int m_slot = logical / p.num_n_tiles;
  const int n0 = n_tile * BN;
  const int nk = p.Kpad / BK;
  KASSERT(nk * BK == p.Kpad && (int)blockIdx.x < p.num_n_tiles * p.grid_m);
  const int taps = p.KT * p.KH * p.KW;
  const uint32_t thw = (uint32_t)p.To * p.Ho * p.Wo;
  const uint32_t clip_bytes = (uint32_t)(p.x_bstride * 2);

  // this lane's DMA slot and the (row-invariant) source chunk
  const int slot = lane % CPR;
  const int lrow = wave * RPI + lane / CPR;  // row of instruction j: j * 4 * RPI + lrow
  const int src_chunk = swz<BK>(lrow, slot);

  const auto wrs = __builtin_amdgcn_make_buffer_rsrc((void*)p.w, (short)0, (int)((long long)p.num_n_tiles * BN * p.Kpad * 2),
                                                     0x00020000);
  // per-thread partial sums of its fixed output chunk column: EPI 1 (sum y, sum y^2) / EPI 2
  float e_s[8], e_q[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { e_s[k] = 0.f; e_q[k] = 0.f; }
  if constexpr (EPI == 1) {  // published by the first tile's barriers
    for (int t = tid; t < BN; t += NT) shl[t] = (p.bn_ss != nullptr && n0 + t < p.Cout) ? p.bn_ss[n0 + t] : 0.f;
  }

  for (int m_tile = m_slot; m_tile < p.num_m_tiles; m_tile += p.grid_m) {
    const int m0 = m_tile * BM;
    const uint32_t b0 = (uint32_t)m0 / thw;
    const char* base = (const char*)p.x + (long long)b0 * p.x_bstride * 2;
    const long long remain = p.x_total_bytes - (long long)b0 * p.x_bstride * 2;
    const uint32_t nrec = remain > 0x7FFFFFF0LL ? 0x7FFFFFF0u : (uint32_t)remain;
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)nrec, 0x00020000);

    int rt[A_INST], rh[A_INST], rw[A_INST];
    uint32_t rowoff[A_INST];
#pragma unroll
    for (int i = 0; i < A_INST; ++i) {
      const int m = m0 + i * NWAVES * RPI + lrow;
      if (m < p.M) {
        uint32_t q = fdiv((uint32_t)m, p.fWo);
        const int wo = m - q * p.Wo;
        uint32_t q2 = fdiv(q, p.fHo);
        const int ho = q - q2 * p.Ho;
        uint32_t b = fdiv(q2, p.fTo);
        const int to = q2 - b * p.To;
        rt[i] = to * p.st - p.pt;
        rh[i] = ho * p.sh - p.ph;
        rw[i] = wo * p.sw - p.pw;
        rowoff[i] = (b - b0) * clip_bytes + (uint32_t)(((rt[i] * p.H + rh[i]) * p.W + rw[i]) * p.Cin * 2);
      } else {
        rt[i] = -(1 << 28);
        rh[i] = 0;
        rw[i] = 0;
        rowoff[i] = 0;
      }
    }

    f32x4 acc[TN][TM];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int i = 0; i < TM; ++i) acc[j][i] = (f32x4){0.f, 0.f, 0.f, 0.f};

    // LDS-only barrier: the previous tile's output stores stay in flight (a __syncthreads() would
    // wait for them); the ring's counted vmcnt waits stay exact, older stores only add to the count
    ring_barrier();  // previous tile's epilogue done with the LDS

    // DMA source offsets of stage kt's pieces (pure ALU: computed before the wait / barrier that
    // precedes the issue, so the issue itself is just the buffer_load ... lds instructions)
    // DMA source offsets of the next stage to issue. Fixed bounds: arrays sized by A_INST / B_INST
    // here make clang's host pass silently drop the kernel's launch stub (undefined symbol)
    static_assert(A_INST <= 4 && B_INST <= 8, "offset arrays");
    uint32_t oa[4], ob[8];
    auto offsets = [&](int kt) {
      // (tap, c) of this lane's chunk by arithmetic: an LDS table read here would make the
      // compiler drain every LDS-DMA in flight (it cannot prove the read does not alias them)
      const int k = kt * BK + src_chunk * 8;
      const int tap = (int)fdiv((uint32_t)k, p.fCin);
      const int c = k - tap * p.Cin;
      const bool kval = tap < taps;
      const int tq = (int)fdiv((uint32_t)tap, p.fKW);
      const int dw = tap - tq * p.KW;
      const int dt = (int)fdiv((uint32_t)tq, p.fKH);
      const int dh = tq - dt * p.KH;
      const uint32_t koff = (uint32_t)((((dt * p.H + dh) * p.W + dw) * p.Cin + c) * 2);
#pragma unroll
      for (int i = 0; i < A_INST; ++i) {
        const int ti = rt[i] + dt, hi = rh[i] + dh, wi = rw[i] + dw;
        const bool v = kval & ((unsigned)ti < (unsigned)p.T) & ((unsigned)hi < (unsigned)p.H) &
                       ((unsigned)wi < (unsigned)p.W);
        oa[i] = v ? rowoff[i] + koff : 0x80000000u;
      }
#pragma unroll
      for (int i = 0; i < B_INST; ++i) {
        const int n = n0 + i * NWAVES * RPI + lrow;
        ob[i] = (uint32_t)(((long long)n * p.Kpad + kt * BK + src_chunk * 8) * 2);
      }
    };
    auto fire = [&](int kt) {
      bf16_t* sa = ring + (kt % STAGES) * STAGE_ELEMS;
      bf16_t* sb = sa + BM * BK;
#pragma unroll
      for (int i = 0; i < A_INST; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_ptr_t)(sa + (i * NWAVES * RPI + wave * RPI) * BK), 16,
                                                 oa[i], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < B_INST; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, (lds_ptr_t)(sb + (i * NWAVES * RPI + wave * RPI) * BK), 16,
                                                 ob[i], 0, 0, 0);
    };

#pragma unroll
    for (int s = 0; s < STAGES - 1; ++s) {
      if (s < nk) {
        offsets(s);
        fire(s);
      }
    }

    for (int kt = 0; kt < nk; ++kt) {
      const bool more = kt + STAGES - 1 < nk;
      if (more) offsets(kt + STAGES - 1);
      // stage kt must have landed: later stages (issued: min(nk-1, kt+STAGES-2) - kt of them) may stay in flight
      const int ahead = min(nk - 1, kt + STAGES - 2) - kt;
      wait_stages<NDMA, STAGES - 2>(ahead);
      ring_barrier();
      if (more) fire(kt + STAGES - 1);
      const bf16_t* a = ring + (kt % STAGES) * STAGE_ELEMS;
      const bf16_t* bsh = a + BM * BK;
      auto xfrag = [&](int s, int i) {
        const int row = wr * WM + i * 16 + (lane & 15);
        return *(const bf16x8*)(a + row * BK + swz<BK>(row, s * 4 + (lane >> 4)) * 8);
      };
      auto wfrag = [&](int s, int j) {
        const int row = wc * WN + j * 16 + (lane & 15);
        return *(const bf16x8*)(bsh + row * BK + swz<BK>(row, s * 4 + (lane >> 4)) * 8);
      };
      if constexpr (V3_PIPE && KSTEPS > 1) {
        // k-step s+1's fragments are read while k-step s's MFMAs run: its X fragments up front
        // (4 extra registers each), each W fragment into the register its step-s twin frees
        bf16x8 xf[TM], xn[TM], wf[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) xf[i] = xfrag(0, i);
#pragma unroll
        for (int j = 0; j < TN; ++j) wf[j] = wfrag(0, j);
#pragma unroll
        for (int s = 0; s < KSTEPS; ++s) {
          if (s + 1 < KSTEPS) {
#pragma unroll
            for (int i = 0; i < TM; ++i) xn[i] = xfrag(s + 1, i);
          }
          if constexpr (V3_PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
          for (int j = 0; j < TN; ++j) {
#pragma unroll
            for (int i = 0; i < TM; ++i)
              acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], xf[i], acc[j][i], 0, 0, 0);
            if (s + 1 < KSTEPS) wf[j] = wfrag(s + 1, j);
          }
          if constexpr (V3_PRIO) __builtin_amdgcn_s_setprio(0);
#pragma unroll
          for (int i = 0; i < TM; ++i) xf[i] = xn[i];
        }
      } else {
#pragma unroll
        for (int s = 0; s < KSTEPS; ++s) {
          bf16x8 xf[TM], wf[TN];
#pragma unroll
          for (int i = 0; i < TM; ++i) xf[i] = xfrag(s, i);
#pragma unroll
          for (int j = 0; j < TN; ++j) wf[j] = wfrag(s, j);
          if constexpr (V3_PRIO) __builtin_amdgcn_s_setprio(1);  // the MFMA burst outranks the other workgroup's loads
#pragma unroll
          for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int i = 0; i < TM; ++i)
              acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], xf[i], acc[j][i], 0, 0, 0);
          if constexpr (V3_PRIO) __builtin_amdgcn_s_setprio(0);
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    ring_barrier();  // every wave done reading the ring before the epilogue reuses it

    // EPI 1: per-channel shift (bn_ss, when set: the BN's running mean) subtracted before the bf16
    // rounding, so the stored pre-BN values keep their precision when |mean| >> std
    float4 shv[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j)
      shv[j] = EPI == 1 ? *(const float4*)(shl + wc * WN + j * 16 + (lane >> 4) * 4) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row = wr * WM + i * 16 + (lane & 15);
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        f32x4 v = acc[j][i];
        if constexpr (EPI == 1) {
          v[0] -= shv[j].x;
          v[1] -= shv[j].y;
          v[2] -= shv[j].z;
          v[3] -= shv[j].w;
        }
        uint2 o;
        o.x = pack2bf(v[0], v[1]);
        o.y = pack2bf(v[2], v[3]);
        const int col = wc * WN + j * 16 + (lane >> 4) * 4;
        *(uint2*)(Es + row * LDE + col) = o;
      }
    }
    if constexpr (EPI == 2) {
      for (int t = tid; t < 4 * BN; t += NT) {
        const int qq = t / BN, c = n0 + (t - qq * BN);
        ssl[t] = c < p.Cout ? p.bn_ss[qq * p.Cout + c] : 0.f;
      }
    }
    ring_barrier();
    // store: thread = fixed 16-B chunk column cc of RPP rows per pass (BN/8 need not divide the
    // block size; the EPI 2 partials then accumulate per fixed channel chunk)
    constexpr int OCPR = BN / 8;
    constexpr int RPP = NT / OCPR;  // rows per pass
    const int cc = tid % OCPR;
    // EPI 2: the producer rows of every row this thread stores, loaded before the first store
    // (unconditional, clamped addresses): one exposed latency per tile instead of a vmcnt(0)
    // drain of the preceding stores at every row (conditional loads merge into the full wait)
    constexpr int NIT = EPI == 2 ? (BM + RPP - 1) / RPP : 1;
    uint4 yv[NIT];
    if constexpr (EPI == 2) {
#pragma unroll
      for (int it = 0; it < NIT; ++it) {
        const int row = min(tid / OCPR + it * RPP, BM - 1);
        const int m = min(m0 + row, p.M - 1), n = min(n0 + cc * 8, p.Cout - 8);
        yv[it] = *(const uint4*)(p.bn_y + (long long)m * p.bn_ld + n);
      }
    }
    if (tid < RPP * OCPR && EPI == 2) {
#pragma unroll
      for (int it = 0; it < NIT; ++it) {
        const int row = tid / OCPR + it * RPP;
        const int m = m0 + row, n = n0 + cc * 8;
        if (row >= BM) break;
        const uint4 dv = *(const uint4*)(Es + row * LDE + cc * 8);
        const bool ok = (m < p.M) & (n < p.Cout);
        if (ok) *(uint4*)(p.y + (long long)m * p.ldy + n) = dv;
        if (ok) {
          float d8[8], y8[8];
          unpack8(dv, d8);
          unpack8(yv[it], y8);
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const int cl = cc * 8 + k;
            const float gm = (y8[k] * ssl[2 * BN + cl] + ssl[3 * BN + cl] > 0.f) ? d8[k] : 0.f;
            e_s[k] += gm;
            e_q[k] += gm * (y8[k] - ssl[cl]) * ssl[BN + cl];
          }
        }
      }
    }
    if (tid < RPP * OCPR && EPI != 2) {
#pragma unroll 4
      for (int row = tid / OCPR; row < BM; row += RPP) {
        const int m = m0 + row, n = n0 + cc * 8;
        const uint4 dv = *(const uint4*)(Es + row * LDE + cc * 8);
        const bool ok = (m < p.M) & (n < p.Cout);
        KASSERT(!ok || n + 8 <= p.ldy);
        if (ok) *(uint4*)(p.y + (long long)m * p.ldy + n) = dv;
        if constexpr (EPI == 1) {
          // BN statistics of the values actually stored (bf16), as a bf16 BN layer would see them
          if (ok) {
            float d8[8];
            unpack8(dv, d8);
#pragma unroll
            for (int k = 0; k < 8; ++k) {
              e_s[k] += d8[k];
              e_q[k] += d8[k] * d8[k];
            }
          }
        }
      }
    }
  }

  if constexpr (EPI != 0) {
    constexpr int OCPR = BN / 8;
    __syncthreads();
    float* red = (float*)smem;  // [2][8][NT]
#pragma unroll
    for (int k = 0; k < 8; ++k) { red[k * NT + tid] = e_s[k]; red[(8 + k) * NT + tid] = e_q[k]; }
    __syncthreads();
    if (tid < OCPR) {
      const int npad = p.num_n_tiles * BN;
      constexpr int ACT = (NT / OCPR) * OCPR;  // threads that stored (the rest hold zeros)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float s1 = 0.f, s2 = 0.f;
        for (int j = tid; j < ACT; j += OCPR) { s1 += red[k * NT + j]; s2 += red[(8 + k) * NT + j]; }
        const int col = n0 + tid * 8 + k;
        p.stats[(long long)m_slot * 2 * npad + col] = s1;
        p.stats[(long long)m_slot * 2 * npad + npad + col] = s2;
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
  long long x_total_bytes;
  long long dy_total_bytes;
  int T, H, W, Cin;
  int To, Ho, Wo, Cout, ldd;
  int KT, KH, KW, st, sh, sw, pt, ph, pw;
  int Ktot, Kpad, Npad, M;
  int n_tiles, k_tiles, splits, rows_per_split;
  float in_scale;
  FastDiv fWo, fHo, fTo, fCin;
};

constexpr int WG_R = 64;  // reduction rows (m) per LDS stage = two 32-deep MFMA k-steps
constexpr int WG_R_MAX = 64;

template <int TK>
constexpr int wg_xpad() { return TK == 192 ? 8 : 16; }

// Per-stage row table (one decomposition per row instead of one per row and chunk column):
// .x = element offset of the row's unshifted input origin relative to the split's first clip,
// .y = (rt + 64) | (rh + 64) << 10 | (rw + 64) << 20 (rows past m_end: all fields 0 -> invalid).
__device__ __forceinline__ void wgrad_row_table(int2* tab, const WgradParams& p, int mb, int m_end, uint32_t b_first,
                                                int tid) {
  if (tid < WG_R_MAX) {
    const int m = mb + tid;
    int2 e = make_int2(0, 0);
    if (m < m_end) {
      const uint32_t q = fdiv((uint32_t)m, p.fWo);
      const int wo = m - q * p.Wo;
      const uint32_t q2 = fdiv(q, p.fHo);
      const int ho = q - q2 * p.Ho;
      const uint32_t b = fdiv(q2, p.fTo);
      const int to = q2 - b * p.To;
      const int rt = to * p.st - p.pt, rh = ho * p.sh - p.ph, rw = wo * p.sw - p.pw;
      e.x = (int)((long long)(b - b_first) * p.x_bstride + ((long long)(rt * p.H + rh) * p.W + rw) * p.Cin);
      e.y = (rt + 64) | ((rh + 64) << 10) | ((rw + 64) << 20);
    }
    tab[tid] = e;
  }
}

// The im2col (tap, channel) of a thread's X chunks. A thread's chunk i sits in column
// (tid + 256 i) % XCPR: one fixed column when XCPR divides 256, else XP = XCPR / gcd(256, XCPR)
// columns used cyclically (TK = 192: 24 chunks per row, columns repeat every 3 chunks).
// Fixed-size arrays (see the note on launch stubs in conv_fwd_v3_kernel).
struct XCols {
  int tapoff[4], dt[4], dh[4], dw[4], col[4];
  bool kval[4];
};

constexpr int cgcd(int a, int b) { return b == 0 ? a : cgcd(b, a % b); }

template <int XCPR>
constexpr int x_period() { return XCPR / cgcd(256, XCPR); }

// Stage this thread's chunks of dY rows [mb, mb+R) and of the im2col X rows.
template <int DCH, int XCH, int DCPR, int XCPR, int VEC, int ESZ, bool U8, typename XReg>
__device__ __forceinline__ void wgrad_load(uint4 (&dreg)[DCH], XReg (&xreg)[XCH], __amdgpu_buffer_rsrc_t drs,
                                           __amdgpu_buffer_rsrc_t xrs, const WgradParams& p, const int2* tab,
                                           int mb, int m_end, int m_base, int tid, int n0, int d_ccol,
                                           const XCols& xc) {
  constexpr int XP = x_period<XCPR>();
#pragma unroll
  for (int i = 0; i < DCH; ++i) {
    const int row = (tid + i * 256) / DCPR;
    const int m = mb + row;
    const int n = n0 + ((tid + i * 256) % DCPR) * 8;  // == d_ccol when DCPR divides 256
    const bool v = (m < m_end) & (n < p.Cout);
    const uint32_t off = v ? (uint32_t)(((long long)(m - m_base) * p.ldd + n) * 2) : 0x80000000u;
    dreg[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(drs, off, 0, 0));
  }
#pragma unroll
  for (int i = 0; i < XCH; ++i) {
    const int row = (tid + i * 256) / XCPR;
    const int2 e = tab[row];
    const int j = i % XP;
    const int ti = (e.y & 1023) - 64 + xc.dt[j], hi = ((e.y >> 10) & 1023) - 64 + xc.dh[j],
              wi = (e.y >> 20) - 64 + xc.dw[j];
    const bool v = xc.kval[j] & ((unsigned)ti < (unsigned)p.T) & ((unsigned)hi < (unsigned)p.H) &
                   ((unsigned)wi < (unsigned)p.W);
    const uint32_t off = v ? (uint32_t)((e.x + xc.tapoff[j]) * ESZ) : 0x80000000u;
    if constexpr (U8) {
      xreg[i] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(xrs, off, 0, 0);
    } else {
      xreg[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xrs, off, 0, 0));
    }
  }
}

template <int DCH, int XCH, int DCPR, int XCPR, int LDN, int LDK, bool U8, typename XReg>
__device__ __forceinline__ void wgrad_store(const uint4 (&dreg)[DCH], const XReg (&xreg)[XCH], bf16_t* d, bf16_t* x,
                                            int tid, int d_ccol, const XCols& xc, float in_scale) {
  constexpr int XP = x_period<XCPR>();
#pragma unroll
  for (int i = 0; i < DCH; ++i) {
    const int row = (tid + i * 256) / DCPR;
    *(uint4*)(d + row * LDN + ((tid + i * 256) % DCPR) * 8) = dreg[i];
  }
#pragma unroll
  for (int i = 0; i < XCH; ++i) {
    const int row = (tid + i * 256) / XCPR;
    const int x_ccol = xc.col[i % XP];
    if constexpr (U8) {
      const uint32_t v = xreg[i];
      uint2 o;
      o.x = pack2bf((float)(v & 0xff) * in_scale, (float)((v >> 8) & 0xff) * in_scale);
      o.y = pack2bf((float)((v >> 16) & 0xff) * in_scale, (float)(v >> 24) * in_scale);
      *(uint2*)(x + row * LDK + x_ccol * 4) = o;
    } else {
      *(uint4*)(x + row * LDK + x_ccol * 8) = xreg[i];
    }
  }
}

// MFMA fragment of 8 reduction rows of column block [col, col+16) of a row-major LDS image:
// ds_read_b64_tr_b16 gives lane (16g + i) rows {4g..4g+3} then {16+4g..} of column col + i.
// The same k permutation is used for both operands, so the dot products are unchanged.
__device__ __forceinline__ bf16x8 tr_frag(const bf16_t* img, int ld, int k0, int col, int g, int q, int pp) {
  const bf16_t* a0 = img + (k0 + 4 * g + q) * ld + col + pp * 4;
  const bf16_t* a1 = img + (k0 + 16 + 4 * g + q) * ld + col + pp * 4;
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)a0);
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)a1);
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// DEEP: two register staging sets, so the loads for stage s + 2 are issued before stage s is
// computed and have ~two compute phases to land (the default has one).
template <int TN_, int TK_, bool U8, bool DEEP = false>
__global__ __launch_bounds__(256, 2) void conv_wgrad_kernel(WgradParams p) {
  constexpr int R = WG_R;
  constexpr int VEC = U8 ? 4 : 8;
  constexpr int ESZ = U8 ? 1 : 2;
  // padded rows: conflict-free transposed reads (TK 192: pad 8 keeps two workgroups per CU)
  constexpr int LDN = TN_ + 16, LDK = TK_ + wg_xpad<TK_>();
  constexpr int DCPR = TN_ / 8, XCPR = TK_ / VEC;
  constexpr int DCH = R * DCPR / 256, XCH = R * XCPR / 256;
  constexpr int WN = TN_ / 2, WK = TK_ / 2;
  constexpr int TI = WN / 16, TJ = WK / 16;
  static_assert(DCH >= 1 && XCH >= 1, "tile too small");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* Ds = (bf16_t*)smem;               // [2][R][LDN]
  bf16_t* Xs = Ds + 2 * R * LDN;            // [2][R][LDK]
  int2* rtab = (int2*)(Xs + 2 * R * LDK);   // [2 or 4][R] row tables

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;  // wr in [0, NWM)
  const int ntiles = p.n_tiles * p.k_tiles;
  const int nblocks = ntiles * p.splits;
  // split-major order: an XCD's contiguous logical range covers every tile of a few m-splits,
  // so the dY / X rows of a split are fetched once into that XCD's L2 and reused by all tiles.
  const int logical = xcd_remap(blockIdx.x, nblocks);
  const int split = logical / ntiles;
  const int tile = logical % ntiles;
  const int n0 = (tile % p.n_tiles) * TN_;
  const int k0 = (tile / p.n_tiles) * TK_;
  const int m_begin = split * p.rows_per_split;
  const int m_end = min(p.M, m_begin + p.rows_per_split);

  // fixed (tap, c) of this thread's X chunk column(s)
  constexpr int XP = x_period<XCPR>();
  static_assert(XP <= 4 && XCH % XP == 0, "X chunk column period");
  XCols xc;
#pragma unroll
  for (int j = 0; j < XP; ++j) {
    const int col = (tid + j * 256) % XCPR;
    const int kk = k0 + col * VEC;
    const int tap = (int)fdiv((uint32_t)kk, p.fCin);
    const int c = kk - tap * p.Cin;
    xc.col[j] = col;
    xc.kval[j] = kk < p.Ktot;
    xc.dw[j] = tap % p.KW;
    xc.dh[j] = (tap / p.KW) % p.KH;
    xc.dt[j] = tap / (p.KW * p.KH);
    xc.tapoff[j] = ((xc.dt[j] * p.H + xc.dh[j]) * p.W + xc.dw[j]) * p.Cin + c;
  }
  const int d_ccol = tid % DCPR;

  // Descriptors based at this split's first row / first clip: offsets stay 32-bit whatever the
  // tensor size, and rows past m_end fall outside the dY record range (read as zero).
  const int m_clamped = m_begin < m_end ? m_begin : 0;
  const long long dbase = (long long)m_clamped * p.ldd * 2;
  const long long dbytes = m_end > m_begin ? (long long)(m_end - m_begin) * p.ldd * 2 : 0;
  const uint32_t thw = (uint32_t)p.To * p.Ho * p.Wo;
  const uint32_t b_first = (uint32_t)m_clamped / thw;
  const long long xbase = (long long)b_first * p.x_bstride * ESZ;
  const long long xrem = p.x_total_bytes - xbase;
  const uint32_t xnrec = xrem > 0x7FFFFFF0LL ? 0x7FFFFFF0u : (uint32_t)xrem;
  const auto drs = __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)p.dy + dbase), (short)0,
                                                     (int)(dbytes > 0x7FFFFFF0LL ? 0x7FFFFFF0LL : dbytes), 0x00020000);
  const auto xrs = __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)p.x + xbase), (short)0, (int)xnrec,
                                                     0x00020000);

  using XReg = typename std::conditional<U8, uint32_t, uint4>::type;
  uint4 dreg[DCH];
  XReg xreg[XCH];

  f32x4 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int g = lane >> 4, li = lane & 15, q = li >> 2, pp = li & 3;
  const int nsteps = (m_end - m_begin + R - 1) / R;
  auto compute = [&](int buf) {
    const bf16_t* d = Ds + buf * R * LDN;
    const bf16_t* x = Xs + buf * R * LDK;
    if constexpr (WG_PIPE && R / 32 > 1) {
      // k-step ks+1's fragments are read under k-step ks's MFMAs: its X fragments up front, each
      // dY fragment into the register its step-ks twin frees after its row of MFMAs
      bf16x8 af[TI], bfr[TJ], bn[TJ];
#pragma unroll
      for (int i = 0; i < TI; ++i) af[i] = tr_frag(d, LDN, 0, wr * WN + i * 16, g, q, pp);
#pragma unroll
      for (int j = 0; j < TJ; ++j) bfr[j] = tr_frag(x, LDK, 0, wc * WK + j * 16, g, q, pp);
#pragma unroll
      for (int ks = 0; ks < R / 32; ++ks) {
        const bool more = ks + 1 < R / 32;
        if (more) {
#pragma unroll
          for (int j = 0; j < TJ; ++j) bn[j] = tr_frag(x, LDK, (ks + 1) * 32, wc * WK + j * 16, g, q, pp);
        }
#pragma unroll
        for (int i = 0; i < TI; ++i) {
#pragma unroll
          for (int j = 0; j < TJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
          if (more) af[i] = tr_frag(d, LDN, (ks + 1) * 32, wr * WN + i * 16, g, q, pp);
        }
#pragma unroll
        for (int j = 0; j < TJ; ++j) bfr[j] = bn[j];
      }
      return;
    }
#pragma unroll
    for (int ks = 0; ks < R / 32; ++ks) {
      bf16x8 af[TI], bfr[TJ];
#pragma unroll
      for (int i = 0; i < TI; ++i) af[i] = tr_frag(d, LDN, ks * 32, wr * WN + i * 16, g, q, pp);
#pragma unroll
      for (int j = 0; j < TJ; ++j) bfr[j] = tr_frag(x, LDK, ks * 32, wc * WK + j * 16, g, q, pp);
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };
  if constexpr (!DEEP) {
    if (nsteps > 0) {
      wgrad_row_table(rtab, p, m_begin, m_end, b_first, tid);
      wgrad_row_table(rtab + R, p, m_begin + R, m_end, b_first, tid);
      __syncthreads();
      wgrad_load<DCH, XCH, DCPR, XCPR, VEC, ESZ, U8>(dreg, xreg, drs, xrs, p, rtab, m_begin, m_end, m_clamped, tid,
                                                      n0, d_ccol, xc);
      wgrad_store<DCH, XCH, DCPR, XCPR, LDN, LDK, U8>(dreg, xreg, Ds, Xs, tid, d_ccol, xc, p.in_scale);
    }
    __syncthreads();
    for (int s = 0; s < nsteps; ++s) {
      const int buf = s & 1;
      const int sn = min(s + 1, nsteps - 1);  // unconditional prefetch (the last one is a harmless repeat)
      wgrad_load<DCH, XCH, DCPR, XCPR, VEC, ESZ, U8>(dreg, xreg, drs, xrs, p, rtab + (sn & 1) * R, m_begin + sn * R,
                                                      m_end, m_clamped, tid, n0, d_ccol, xc);
      // row table of stage s + 2 into the slot stage s used (its last reader was iteration s - 1)
      if (s + 2 < nsteps) wgrad_row_table(rtab + buf * R, p, m_begin + (s + 2) * R, m_end, b_first, tid);
      compute(buf);
      wgrad_store<DCH, XCH, DCPR, XCPR, LDN, LDK, U8>(dreg, xreg, Ds + (buf ^ 1) * R * LDN, Xs + (buf ^ 1) * R * LDK,
                                                       tid, d_ccol, xc, p.in_scale);
      __syncthreads();
    }
  } else {
    // register sets: stage x lives in set x & 1; row tables in a 4-slot ring (slot x & 3)
    uint4 dreg2[DCH];
    XReg xreg2[XCH];
    if (nsteps > 0) {
      for (int st = 0; st < 3; ++st) wgrad_row_table(rtab + (st & 3) * R, p, m_begin + st * R, m_end, b_first, tid);
      __syncthreads();
      wgrad_load<DCH, XCH, DCPR, XCPR, VEC, ESZ, U8>(dreg, xreg, drs, xrs, p, rtab, m_begin, m_end, m_clamped, tid,
                                                      n0, d_ccol, xc);
      wgrad_store<DCH, XCH, DCPR, XCPR, LDN, LDK, U8>(dreg, xreg, Ds, Xs, tid, d_ccol, xc, p.in_scale);
      wgrad_load<DCH, XCH, DCPR, XCPR, VEC, ESZ, U8>(dreg2, xreg2, drs, xrs, p, rtab + R, m_begin + R, m_end,
                                                      m_clamped, tid, n0, d_ccol, xc);
    }
    __syncthreads();
    for (int s = 0; s < nsteps; s += 2) {
      // even step s: stage s in LDS buf 0 / set 0 free; stage s+1 in flight in set 1
      {
        const int sl = min(s + 2, nsteps - 1);
        wgrad_load<DCH, XCH, DCPR, XCPR, VEC, ESZ, U8>(dreg, xreg, drs, xrs, p, rtab + (sl & 3) * R, m_begin + sl * R,
                                                        m_end, m_clamped, tid, n0, d_ccol, xc);
        if (s + 3 < nsteps)
          wgrad_row_table(rtab + ((s + 3) & 3) * R, p, m_begin + (s + 3) * R, m_end, b_first, tid);
        compute(0);
        wgrad_store<DCH, XCH, DCPR, XCPR, LDN, LDK, U8>(dreg2, xreg2, Ds + R * LDN, Xs + R * LDK, tid, d_ccol, xc,
                                                         p.in_scale);
        lds_barrier();  // LDS only: the loads of stage s + 2 stay in flight across the barrier
      }
      if (s + 1 >= nsteps) break;
      // odd step s+1: stage s+1 in LDS buf 1 / set 1 free; stage s+2 in flight in set 0
      {
        const int sl = min(s + 3, nsteps - 1);
        wgrad_load<DCH, XCH, DCPR, XCPR, VEC, ESZ, U8>(dreg2, xreg2, drs, xrs, p, rtab + (sl & 3) * R,
                                                        m_begin + sl * R, m_end, m_clamped, tid, n0, d_ccol, xc);
        if (s + 4 < nsteps)
          wgrad_row_table(rtab + ((s + 4) & 3) * R, p, m_begin + (s + 4) * R, m_end, b_first, tid);
        compute(1);
        wgrad_store<DCH, XCH, DCPR, XCPR, LDN, LDK, U8>(dreg, xreg, Ds, Xs, tid, d_ccol, xc, p.in_scale);
        lds_barrier();
      }
    }
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

// ---------------------------------------------------------------------------------------
// v3 wgrad: dY and im2col(X) tiles [R rows][TN|TK] arrive by LDS-DMA into a STAGES-deep ring
// (no staging VGPRs, no ds_write pass). The images are unpadded with a 16-B chunk XOR of
// 2*(row & 7), which keeps the ds_read_b64_tr_b16 fragment reads conflict-free (the eight rows a
// 32-lane group touches land on distinct chunk pairs); each lane DMAs the source chunk that
// belongs in its lane-linear slot.
__device__ __forceinline__ int wg_swz(int row, int chunk, int cpr) {
  return chunk ^ ((2 * (row & 7)) & (cpr - 1));
}

__device__ __forceinline__ bf16x8 tr_frag_sw(const bf16_t* img, int cols, int cpr, int k0, int col, int g, int q,
                                             int pp) {
  const int r0 = k0 + 4 * g + q, r1 = r0 + 16;
  const int c = col / 8 + (pp >> 1), h = (pp & 1) * 4;
  const bf16_t* a0 = img + r0 * cols + wg_swz(r0, c, cpr) * 8 + h;
  const bf16_t* a1 = img + r1 * cols + wg_swz(r1, c, cpr) * 8 + h;
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)a0);
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)a1);
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

template <int TN_, int TK_, int STAGES>
__global__ __launch_bounds__(256, 1) void conv_wgrad_v3_kernel(WgradParams p) {
  constexpr int R = WG_R;
  constexpr int DCPR = TN_ / 8, XCPR = TK_ / 8;
  constexpr int DRPI = 64 / DCPR, XRPI = 64 / XCPR;  // rows per DMA instruction
  constexpr int D_INST = R / DRPI / 4, X_INST = R / XRPI / 4;
  constexpr int NDMA = D_INST + X_INST;
  constexpr int WN = TN_ / 2, WK = TK_ / 2;
  constexpr int TI = WN / 16, TJ = WK / 16;
  constexpr int STAGE_ELEMS = R * (TN_ + TK_);
  static_assert(D_INST >= 1 && X_INST >= 1, "tile too small for the DMA mapping");

  // one static array per ring stage (stage: dY [R][TN] then X [R][TK]): a step's fragment reads
  // then provably miss the LDS-DMA filling the other stages, so the compiler does not drain that
  // DMA (s_waitcnt vmcnt(0)) in front of them -- with one dynamic buffer it did at every step
  __shared__ __attribute__((aligned(16))) bf16_t rd0[R * TN_];
  __shared__ __attribute__((aligned(16))) bf16_t rx0[R * TK_];
  __shared__ __attribute__((aligned(16))) bf16_t rd1[R * TN_];
  __shared__ __attribute__((aligned(16))) bf16_t rx1[R * TK_];
  __shared__ __attribute__((aligned(16))) bf16_t rd2[STAGES > 2 ? R * TN_ : 8];
  __shared__ __attribute__((aligned(16))) bf16_t rx2[STAGES > 2 ? R * TK_ : 8];
  auto stage_d = [&](auto SL) -> bf16_t* {
    constexpr int sl = decltype(SL)::value;
    return sl == 0 ? rd0 : (sl == 1 ? rd1 : rd2);
  };
  auto stage_x = [&](auto SL) -> bf16_t* {
    constexpr int sl = decltype(SL)::value;
    return sl == 0 ? rx0 : (sl == 1 ? rx1 : rx2);
  };

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  const int ntiles = p.n_tiles * p.k_tiles;
  const int nblocks = ntiles * p.splits;
  const int logical = xcd_remap(blockIdx.x, nblocks);
  const int split = logical / ntiles;
  const int tile = logical % ntiles;
  const int n0 = (tile % p.n_tiles) * TN_;
  const int k0 = (tile / p.n_tiles) * TK_;
  const int m_begin = split * p.rows_per_split;
  const int m_end = min(p.M, m_begin + p.rows_per_split);

  // dY DMA lane mapping (row-invariant source chunk)
  const int d_slot = lane % DCPR, d_lrow = wave * DRPI + lane / DCPR;
  const int d_chunk = wg_swz(d_lrow, d_slot, DCPR);
  const int n_lane = n0 + d_chunk * 8;
  const bool n_ok = n_lane < p.Cout;
  // X DMA lane mapping: fixed (tap, c) for the whole kernel
  const int x_slot = lane % XCPR, x_lrow = wave * XRPI + lane / XCPR;
  const int x_chunk = wg_swz(x_lrow, x_slot, XCPR);
  const int kk = k0 + x_chunk * 8;
  const int tap = (int)fdiv((uint32_t)kk, p.fCin);
  const int c = kk - tap * p.Cin;
  const bool kval = kk < p.Ktot;
  const int dw = tap % p.KW, dh = (tap / p.KW) % p.KH, dt = tap / (p.KW * p.KH);
  const int tapoff = ((dt * p.H + dh) * p.W + dw) * p.Cin + c;

  const int m_clamped = m_begin < m_end ? m_begin : 0;
  const long long dbase = (long long)m_clamped * p.ldd * 2;
  const long long dbytes = m_end > m_begin ? (long long)(m_end - m_begin) * p.ldd * 2 : 0;
  const uint32_t thw = (uint32_t)p.To * p.Ho * p.Wo;
  const uint32_t b_first = (uint32_t)m_clamped / thw;
  const long long xbase = (long long)b_first * p.x_bstride * 2;
  const long long xrem = p.x_total_bytes - xbase;
  const uint32_t xnrec = xrem > 0x7FFFFFF0LL ? 0x7FFFFFF0u : (uint32_t)xrem;
  const auto drs = __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)p.dy + dbase), (short)0,
                                                     (int)(dbytes > 0x7FFFFFF0LL ? 0x7FFFFFF0LL : dbytes), 0x00020000);
  const auto xrs = __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)p.x + xbase), (short)0, (int)xnrec,
                                                     0x00020000);

  f32x4 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nsteps = (m_end - m_begin + R - 1) / R;
  const int g = lane >> 4, li = lane & 15, q = li >> 2, pp = li & 3;

  auto issue = [&](int st, auto SL) {
    bf16_t* sd = stage_d(SL);
    bf16_t* sx = stage_x(SL);
    const int mb = m_begin + st * R;
#pragma unroll
    for (int i = 0; i < D_INST; ++i) {
      const int row = i * 4 * DRPI + d_lrow;
      const int m = mb + row;
      const bool v = (m < m_end) & n_ok;
      const uint32_t off = v ? (uint32_t)(m - m_clamped) * (uint32_t)p.ldd * 2u + (uint32_t)n_lane * 2u : 0x80000000u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(drs, (lds_ptr_t)(sd + (i * 4 * DRPI + wave * DRPI) * TN_), 16, off,
                                               0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < X_INST; ++i) {
      // row decomposition by arithmetic (no LDS reads while LDS-DMA is in flight, see fwd v3)
      const int m = mb + i * 4 * XRPI + x_lrow;
      const uint32_t q0 = fdiv((uint32_t)m, p.fWo);
      const int wo = m - q0 * p.Wo;
      const uint32_t q1 = fdiv(q0, p.fHo);
      const int ho = q0 - q1 * p.Ho;
      const uint32_t bb = fdiv(q1, p.fTo);
      const int to = q1 - bb * p.To;
      const int ti = to * p.st - p.pt + dt, hi = ho * p.sh - p.ph + dh, wi = wo * p.sw - p.pw + dw;
      const bool v = kval & (m < m_end) & ((unsigned)ti < (unsigned)p.T) & ((unsigned)hi < (unsigned)p.H) &
                     ((unsigned)wi < (unsigned)p.W);
      const uint32_t off = v ? (uint32_t)(((long long)(bb - b_first) * p.x_bstride +
                                           ((long long)(ti * p.H + hi) * p.W + wi) * p.Cin + c) * 2)
                             : 0x80000000u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (lds_ptr_t)(sx + (i * 4 * XRPI + wave * XRPI) * TK_), 16, off,
                                               0, 0, 0);
    }
  };

  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  if (nsteps > 0) issue(0, S0{});
  if (STAGES > 2 && nsteps > 1) issue(1, S1{});
  // steps in groups of STAGES (step s uses stage s % STAGES, a compile-time index per body)
  auto body = [&](int s, auto SL) {
    constexpr int sl = decltype(SL)::value;
    const int ahead = min(nsteps - 1, s + STAGES - 2) - s;
    // (the builtin, not inline asm: the compiler's wait tracking sees it)
    if (ahead <= 0) __builtin_amdgcn_s_waitcnt(vmcnt_imm(0));
    else if (ahead == 1 || STAGES < 3) __builtin_amdgcn_s_waitcnt(vmcnt_imm(NDMA));
    else __builtin_amdgcn_s_waitcnt(vmcnt_imm(STAGES > 2 ? 2 * NDMA : 0));
    ring_barrier();
    if (s + STAGES - 1 < nsteps) issue(s + STAGES - 1, std::integral_constant<int, (sl + STAGES - 1) % STAGES>{});
    const bf16_t* d = stage_d(SL);
    const bf16_t* x = stage_x(SL);
#pragma unroll
    for (int ks = 0; ks < R / 32; ++ks) {
      bf16x8 af[TI], bfr[TJ];
#pragma unroll
      for (int i = 0; i < TI; ++i) af[i] = tr_frag_sw(d, TN_, DCPR, ks * 32, wr * WN + i * 16, g, q, pp);
#pragma unroll
      for (int j = 0; j < TJ; ++j) bfr[j] = tr_frag_sw(x, TK_, XCPR, ks * 32, wc * WK + j * 16, g, q, pp);
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };
  for (int s = 0; s < nsteps; s += STAGES) {
    body(s, S0{});
    if (s + 1 < nsteps) body(s + 1, S1{});
    if (STAGES > 2 && s + 2 < nsteps) body(s + 2, std::integral_constant<int, 2>{});
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
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

// Sum the split slabs (coalesced along k) and scatter to the PyTorch weight layout
// [n][c_param][tap].
// Block = 64 output elements x WR_GROUPS split groups: group g sums splits g, g + 4, ... with four
// independent accumulators (16 slab loads in flight per element instead of 4 serial ones per
// thread), then the groups combine in LDS in a fixed order: deterministic, and the few-thousand-
// split slabs of the wide-occupancy wgrad tilings no longer run one latency-bound chain per thread.
constexpr int WR_GROUPS = 4;

__device__ __forceinline__ void wgrad_reduce_body(int blk, int nblk, const float* __restrict__ slab,
                                                  float* __restrict__ dw, int splits, int Npad, int Kpad, int Cout,
                                                  int Cin, int Cin_param, int taps, int accumulate) {
  __shared__ float part[WR_GROUPS][64];
  const int Ktot = taps * Cin;
  const long long total = (long long)Cout * Ktot;
  const long long plane = (long long)Npad * Kpad;
  const int e = threadIdx.x & 63, grp = threadIdx.x >> 6;
  for (long long base = blk * 64LL; base < total; base += nblk * 64LL) {  // block-uniform
    const long long idx = base + e;
    const int n = (int)(idx / Ktot);
    const int k = (int)(idx - (long long)n * Ktot);
    const int tap = k / Cin, c = k - tap * Cin;
    const bool live = idx < total && c < Cin_param;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    if (live) {
      const float* sp = slab + (long long)n * Kpad + k;
      int i = grp;
      for (; i + 3 * WR_GROUPS < splits; i += 4 * WR_GROUPS) {
        s0 += sp[i * plane];
        s1 += sp[(i + WR_GROUPS) * plane];
        s2 += sp[(i + 2 * WR_GROUPS) * plane];
        s3 += sp[(i + 3 * WR_GROUPS) * plane];
      }
      for (; i < splits; i += WR_GROUPS) s0 += sp[i * plane];
    }
    part[grp][e] = (s0 + s1) + (s2 + s3);
    __syncthreads();
    if (grp == 0 && live) {
      float s = part[0][e];
#pragma unroll
      for (int g = 1; g < WR_GROUPS; ++g) s += part[g][e];
      const long long o = ((long long)n * Cin_param + c) * taps + tap;
      dw[o] = accumulate ? dw[o] + s : s;
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(64 * WR_GROUPS) void wgrad_reduce_kernel(const float* __restrict__ slab,
                                                                     float* __restrict__ dw, int splits, int Npad,
                                                                     int Kpad, int Cout, int Cin, int Cin_param,
                                                                     int taps, int accumulate) {
  wgrad_reduce_body(blockIdx.x, gridDim.x, slab, dw, splits, Npad, Kpad, Cout, Cin, Cin_param, taps, accumulate);
}

// Several pending slab reductions (the side stream's wgrads of consecutive layers, hip_ops
// _ReduceBatcher) in one launch: block -> reduction by its first block. Same per-element order
// as wgrad_reduce_kernel (bitwise equal results).
struct ReduceDesc {
  const float* slab;
  float* dw;
  int splits, Npad, Kpad, Cout, Cin, Cin_param, taps, accumulate, blk0, nblk;
};
static_assert(sizeof(ReduceDesc) == 56, "ReduceDesc layout is mirrored by a ctypes.Structure");
constexpr int REDUCE_BATCH_MAX = 32;
struct ReduceBatch {
  ReduceDesc d[REDUCE_BATCH_MAX];
  int n;
};

__global__ __launch_bounds__(64 * WR_GROUPS) void wgrad_reduce_batch_kernel(ReduceBatch b) {
  int lo = 0, hi = b.n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (b.d[mid].blk0 <= (int)blockIdx.x) lo = mid; else hi = mid - 1;
  }
  const ReduceDesc& d = b.d[lo];
  wgrad_reduce_body(blockIdx.x - d.blk0, d.nblk, d.slab, d.dw, d.splits, d.Npad, d.Kpad, d.Cout, d.Cin, d.Cin_param,
                    d.taps, d.accumulate);
}

// ---------------------------------------------------------------------------------------
// Stem wgrad (paired-width stem: x2 [B, T, H, W2, 8] bf16, Cout 64, kernel (3, 7, 4), stride
// (2, 2, 1), padding (1, 3, 2), Wo = W2) as a halo-tiled direct convolution gradient.
//
// The generic wgrad gathers the im2col rows of X from L2 for every tap (84 taps x 16 B per
// output position) and re-reads dY once per K tile. Here a work item is HR = 2 output rows of
// one (clip, to): its input halo (3 t x (2*HR+5) h x (W2+4) w-pairs, 45 KB at 200x200) and its
// dY rows (HR*Wo x 64, 25.6 KB) are staged through registers into an LDS double buffer while the
// previous item is computed, so every input byte is fetched ~3x instead of ~84x. The B operand of tap row
// (dt, dh) is an overlapping-row image of the halo (row = output position, stride one w-pair,
// 32 columns = 4 w-pairs x 8 channels) read with ds_read_b64_tr_b16; each wave owns 11 of the
// 42 16-column K fragments for all 64 output channels (176 accumulators) and keeps them across
// all of its items; one partial [64][672] per workgroup goes to the slab for wgrad_reduce.
constexpr int STW_HR = 2;
constexpr int STW_KF = 42;           // 672 / 16

// 8 uint8 pixel channels (a width pair of RGB0 pixels) -> the same 8 integers as bf16 (exact:
// 0..255 need 8 significant bits, so the fp32 value's upper half IS the bf16). The stems convert
// the native clip this way while staging their halo instead of in a separate pass over the clip;
// the 1/255 scale moves to the other operand / the result (stem_fwd: the LDS weight copy,
// stem_wgrad: the fp32 partial dW), where it is applied once per workgroup, not per pixel.
__device__ __forceinline__ uint32_t u8x2_hi_bf16(float a, float b) {
  return __builtin_amdgcn_perm(__float_as_uint(b), __float_as_uint(a), 0x07060302u);
}
__device__ __forceinline__ uint4 u8x8_to_bf16x8(uint2 v) {
  uint4 o;
  o.x = u8x2_hi_bf16((float)(v.x & 0xff), (float)((v.x >> 8) & 0xff));
  o.y = u8x2_hi_bf16((float)((v.x >> 16) & 0xff), (float)(v.x >> 24));
  o.z = u8x2_hi_bf16((float)(v.y & 0xff), (float)((v.y >> 8) & 0xff));
  o.w = u8x2_hi_bf16((float)((v.y >> 16) & 0xff), (float)(v.y >> 24));
  return o;
}

// one staged halo pixel (8 channels): 16 B of bf16, or 8 B of uint8 converted on the LDS store
template <bool U8>
__device__ __forceinline__ auto stem_px_load(__amdgpu_buffer_rsrc_t rs, bool valid, int px) {
  if constexpr (U8) {
    const uint32_t off = valid ? (uint32_t)px * 8u : 0x80000000u;  // > num_records: reads 0
    return __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, 0));
  } else {
    const uint32_t off = valid ? (uint32_t)px * 16u : 0x80000000u;
    return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
  }
}

struct StemWgradParams {
  const bf16_t* dy;  // [M, 64]
  const bf16_t* x;   // [B, T, H, W2, 8] bf16 (or uint8 with the U8 kernel)
  float* slab;       // [gridDim][64][672]
  int B, T, H, W2, To, Ho, Wo;
  int nitems;        // B * To * (Ho / HR)
  int halo_px;       // 3 * (2*HR+5) * (W2+4)
  int dy_rows;       // HR * Wo rounded up to 32 (MFMA reduction chunks; tail rows are zero)
  long long x_bytes, dy_bytes;
  // POOL kernels: dY is not read but rebuilt per item from the maxpool_2a backward and the stem's
  // BN backward (csrc/pool.hip POOL_BWD_APPLY, same arithmetic and roundings): pdy / parg = the
  // pooled gradient and uint8 arg-max [B, To, Ho/2, Wo/2, 64], ybn = the raw stem output [M, 64],
  // ss = [mean, invstd, scale, shift], coef = [k0, k1, k2] (64 each)
  const bf16_t* pdy;
  const uint8_t* parg;
  const bf16_t* ybn;
  const float* ss;
  const float* coef;
};

__device__ __forceinline__ bf16x8 tr_pair(const bf16_t* a0, const bf16_t* a1) {
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)a0);
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)a1);
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

constexpr int STW_HREG = 13;  // halo pixels per thread (<= 3 * 9 * 116 at 224x224)
constexpr int STW_DREG = 7;   // dY chunks per thread (<= 224 rows x 8 chunks)

// NKQ waves, one per K range: a wave owns the 64 x (K range x 16) accumulator tile of its range.
// NKQ 4 (the round-1 kernel) holds 4 x 11 tiles per wave at one wave per SIMD; NKQ 8 holds 4 x 6
// at two waves per SIMD, so one wave's fragment reads overlap the other's MFMAs (2.73 -> 2.19 ms
// same-box; splitting the 64 channels over two 8-wave groups instead measured no gain: twice the
// dY fragment reads per MFMA).
// POOL: the item's two dY rows are one row of 2x2 quads of the 1x3x3 / (1,2,2) TF-SAME pool
// (maxpool_2a): each thread gathers a quad's 4 pooled cells + arg-max bytes one item ahead (the
// raw stem rows arrive in the D image by LDS-DMA), and the LDS store computes dz (pool_bwd_quad
// order) and the BN backward dy = k0 (dz mask - k1 - xhat k2) in place: the full-resolution dy is
// never written or read. Opt-in (hip_ops MILNCE_STEM_POOL_WGRAD=1): 3.68 ms against 2.19 + 1.09
// for the BN-apply pass and the plain wgrad (same box): the gather registers push the kernel into
// ~15 VGPR spills at two waves per SIMD and the per-item apply sits between compute and barrier.
template <bool U8, int NKQ, bool POOL = false>
__global__ __launch_bounds__(64 * NKQ, 1) void stem_wgrad_kernel(StemWgradParams p) {
  constexpr int NT = 64 * NKQ;
  constexpr int QREG = POOL ? (112 / 2 * 8 + NT - 1) / NT : 1;  // quad chunks per thread (Wo <= 112)
  constexpr int NAF = 4;                                   // dY (A) fragments per wave
  constexpr int KFW = (STW_KF + NKQ - 1) / NKQ;            // K fragments per wave (at most)
  constexpr int HREG = (STW_HREG * 256 + NT - 1) / NT;     // halo pixels per thread
  constexpr int DREG = (STW_DREG * 256 + NT - 1) / NT;     // dY chunks per thread
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wq = wave;  // K range
  const int hrows = 2 * STW_HR + 5, wpx = p.W2 + 4;
  const int buf_elems = (p.halo_px + p.dy_rows * 8) * 8;  // halo pixels, then dY rows (8 chunks each)
  bf16_t* const buf0 = (bf16_t*)smem;
  bf16_t* const buf1 = buf0 + buf_elems;
  const auto xrs = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, (int)p.x_bytes, 0x00020000);
  const int hg_per = p.Ho / STW_HR;
  const int real_rows = STW_HR * p.Wo;

  // register staging (T14): the next item's halo and dY are loaded into VGPRs while the current
  // item is computed from LDS, then written to the other buffer
  using HReg = typename std::conditional<U8, uint2, uint4>::type;
  HReg hreg[HREG];
  uint4 dreg[POOL ? 1 : DREG];
  uint4 qg[QREG][4];
  uint2 qa[QREG][4];
  const int nquad = (p.Wo / 2) * 8;  // quad chunks per item: (w2, 8-channel chunk)
  float* bnc = (float*)(smem + 2 * (size_t)buf_elems * 2);  // POOL: [7][64] ss and coef
  // dst: the LDS buffer the item will be staged in (POOL: its raw stem rows go there by LDS-DMA)
  auto load = [&](int it, bf16_t* dst) {
    const int hg = it % hg_per, q = it / hg_per;
    const int to = q % p.To, b = q / p.To;
    const int t0 = 2 * to - 1, h0 = 2 * hg * STW_HR - 3;
#pragma unroll
    for (int i = 0; i < HREG; ++i) {
      const int f = tid + NT * i;
      const int tt = f / (hrows * wpx), rem = f - tt * (hrows * wpx);
      const int hh = rem / wpx, wp = rem - hh * wpx;
      const int ti = t0 + tt, hi = h0 + hh, wi = wp - 2;
      const bool v = f < p.halo_px && tt < 3 && (unsigned)ti < (unsigned)p.T && (unsigned)hi < (unsigned)p.H &&
                     (unsigned)wi < (unsigned)p.W2;
      hreg[i] = stem_px_load<U8>(xrs, v, ((b * p.T + ti) * p.H + hi) * p.W2 + wi);
    }
    const long long m0 = ((long long)(b * p.To + to) * p.Ho + hg * STW_HR) * p.Wo;
    if constexpr (POOL) {
      static_assert(STW_HR == 2, "one quad row per item");
      const int Hp = p.Ho / 2, Wp = p.Wo / 2;
      const long long pbase = (long long)(b * p.To + to) * Hp;  // pooled row index of (b, to, 0)
      const auto prs = __builtin_amdgcn_make_buffer_rsrc((void*)(p.pdy + pbase * Wp * 64), (short)0,
                                                         Hp * Wp * 128, 0x00020000);
      const auto ars = __builtin_amdgcn_make_buffer_rsrc((void*)(p.parg + pbase * Wp * 64), (short)0,
                                                         Hp * Wp * 64, 0x00020000);
      const auto yrs = __builtin_amdgcn_make_buffer_rsrc((void*)(p.ybn + m0 * 64), (short)0, real_rows * 128,
                                                         0x00020000);
      // raw stem rows -> the D image by LDS-DMA: 1-KiB piece j holds chunks 64 j .. 64 j + 63 in
      // lane order, the lane loading the source chunk its swizzled slot holds
      char* dimg = (char*)(dst + p.halo_px * 8);
      for (int j = wave; j * 64 < real_rows * 8; j += NKQ) {
        const int ch = j * 64 + lane, row = ch >> 3;
        const uint32_t off = ch < real_rows * 8 ? (uint32_t)(row * 128 + wg_swz(row, ch & 7, 8) * 16) : 0x80000000u;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(yrs, (lds_ptr_t)(dimg + j * 1024), 16, off, 0, 0, 0);
      }
#pragma unroll
      for (int i = 0; i < QREG; ++i) {
        const int qc = tid + NT * i;
        const bool act = qc < nquad;
        const int w2 = qc >> 3, c8 = (qc & 7) * 8;
#pragma unroll
        for (int u = 0; u < 4; ++u) {  // pooled cells (hg - jh, w2 - jw), u = 2 jh + jw
          const int ho = hg - (u >> 1), wo = w2 - (u & 1);
          const bool ok = act & (ho >= 0) & (wo >= 0);
          const uint32_t cell = (uint32_t)(ho * Wp + wo);
          qg[i][u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                                    prs, ok ? cell * 128 + c8 * 2 : 0x80000000u, 0, 0));
          qa[i][u] = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(
                                                    ars, ok ? cell * 64 + c8 : 0x80000000u, 0, 0));
        }
      }
    } else {
      const auto drs = __builtin_amdgcn_make_buffer_rsrc((void*)(p.dy + m0 * 64), (short)0, real_rows * 128,
                                                         0x00020000);
#pragma unroll
      for (int i = 0; i < DREG; ++i) {
        const int ch = tid + NT * i;  // chunk = row * 8 + logical column chunk
        const uint32_t off = ch < real_rows * 8 ? (uint32_t)(ch * 16) : 0x80000000u;
        dreg[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(drs, off, 0, 0));
      }
    }
  };
  auto store = [&](bf16_t* base) {
#pragma unroll
    for (int i = 0; i < HREG; ++i) {
      const int f = tid + NT * i;
      if constexpr (U8) {  // integer-valued bf16; the 1/255 is applied to the partial dW
        if (f < p.halo_px) *(uint4*)(base + f * 8) = u8x8_to_bf16x8(hreg[i]);
      } else {
        if (f < p.halo_px) *(uint4*)(base + f * 8) = hreg[i];
      }
    }
    bf16_t* D = base + p.halo_px * 8;
    if constexpr (POOL) {
#pragma unroll
      for (int i = 0; i < QREG; ++i) {
        const int qc = tid + NT * i;
        if (qc >= nquad) continue;
        const int w2 = qc >> 3, c = qc & 7;
        // pool_bwd_quad: input (eh, ew) of the quad takes pooled cell u = (jh, jw) when its
        // arg-max tap is (eh + 2 jh) * 3 + (ew + 2 jw); summed over u in the same order
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float dz[8], yv[8], o[8];
#pragma unroll
          for (int k = 0; k < 8; ++k) dz[k] = 0.f;
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int dh = (e >> 1) + 2 * (u >> 1), dw = (e & 1) + 2 * (u & 1);
            if (dh >= 3 || dw >= 3) continue;  // compile-time after unrolling
            const uint32_t tap = (uint32_t)(dh * 3 + dw);
            float gf[8];
            unpack8(qg[i][u], gf);
#pragma unroll
            for (int k = 0; k < 8; ++k) {
              const uint32_t ak = ((k < 4 ? qa[i][u].x : qa[i][u].y) >> (8 * (k & 3))) & 0xff;
              dz[k] += (ak == tap) ? gf[k] : 0.f;  // out-of-range cells loaded as zero gradient
            }
          }
          // BN backward as csrc/pool.hip bn_apply, on the bf16-rounded dz
          const int row = (e >> 1) * p.Wo + 2 * w2 + (e & 1);
          uint4* slot = (uint4*)(D + row * 64 + wg_swz(row, c, 8) * 8);  // raw y in, dy out
          unpack8(pack8(dz), dz);
          unpack8(*slot, yv);
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const int ch = c * 8 + k;
            const BnBwdC q = bn_bwd_const(bnc[ch], bnc[64 + ch], bnc[128 + ch], bnc[192 + ch], bnc[256 + ch],
                                          bnc[320 + ch], bnc[384 + ch]);
            o[k] = bn_bwd_elem(dz[k], yv[k], q);
          }
          *slot = pack8(o);
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < DREG; ++i) {
        const int ch = tid + NT * i;
        const int row = ch >> 3, c = ch & 7;
        if (row < p.dy_rows) *(uint4*)(D + row * 64 + wg_swz(row, c, 8) * 8) = dreg[i];  // tail rows: zeros
      }
    }
  };

  f32x4 acc[NAF][KFW];
#pragma unroll
  for (int i = 0; i < NAF; ++i)
#pragma unroll
    for (int j = 0; j < KFW; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int g = lane >> 4, li = lane & 15, qq = li >> 2, pp = li & 3;
  const int kf0 = wq * STW_KF / NKQ, kf_end = (wq + 1) * STW_KF / NKQ;  // balanced K ranges
  const int nchunks = p.dy_rows / 32;
  // fragments of one 32-position chunk: 4 dY (A) fragments and this wave's 11 X (B) fragments;
  // chunk c + 1's are read while chunk c's 44 MFMAs run (two register sets)
  struct Frags {
    bf16x8 a[NAF], b[KFW];
  };
  auto read_frags = [&](const bf16_t* X, int c, Frags& f) {
    const bf16_t* D = X + p.halo_px * 8;
    const int p0 = c * 32;
#pragma unroll
    for (int nf = 0; nf < NAF; ++nf) f.a[nf] = tr_frag_sw(D, 64, 8, p0, nf * 16, g, qq, pp);
    int pb[2];  // this lane's two positions (rows of the transposed reads): halo pixel bases
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      int pos = p0 + 4 * g + qq + 16 * h;
      pos = pos < real_rows ? pos : real_rows - 1;  // tail rows: dY is zero, read any finite pixel
      const int hr = pos / p.Wo, wo = pos - hr * p.Wo;
      pb[h] = (2 * hr) * wpx + wo;
    }
#pragma unroll
    for (int j = 0; j < KFW; ++j) {
      const int kf = min(kf0 + j, STW_KF - 1);
      const int tr = kf >> 1;  // (dt, dh) tap row
      const int dt = tr / 7, dh = tr - 7 * (tr / 7);
      const int poff = (dt * hrows + dh) * wpx + 2 * (kf & 1);
      f.b[j] = tr_pair(X + (pb[0] + poff) * 8 + pp * 4, X + (pb[1] + poff) * 8 + pp * 4);
    }
  };
  auto mfmas = [&](const Frags& f) {
#pragma unroll
    for (int j = 0; j < KFW; ++j) {
      if (kf0 + j < kf_end) {
#pragma unroll
        for (int nf = 0; nf < NAF; ++nf)
          acc[nf][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.a[nf], f.b[j], acc[nf][j], 0, 0, 0);
      }
    }
  };
  auto compute = [&](const bf16_t* X) {
    Frags f0, f1;
    if constexpr (NT > 256) {  // one fragment set: the SIMD's other wave covers the read latency
      for (int c = 0; c < nchunks; ++c) {
        read_frags(X, c, f0);
        mfmas(f0);
      }
      return;
    }
    read_frags(X, 0, f0);
    int c = 0;
    for (; c + 2 <= nchunks; c += 2) {
      read_frags(X, c + 1, f1);
      mfmas(f0);
      if (c + 2 < nchunks) read_frags(X, c + 2, f0);
      mfmas(f1);
    }
    if (c < nchunks) mfmas(f0);
  };

  if constexpr (POOL) {
    // BN constants, and the tail rows past the item's positions (never written by the quads: zero)
    for (int t = tid; t < 7 * 64; t += NT) bnc[t] = t < 256 ? p.ss[t] : p.coef[t - 256];
    for (int t = tid; t < (p.dy_rows - real_rows) * 8 * 2; t += NT) {
      bf16_t* D = (t < (p.dy_rows - real_rows) * 8 ? buf0 : buf1) + p.halo_px * 8;
      const int ch = t % ((p.dy_rows - real_rows) * 8);
      const int row = real_rows + (ch >> 3), c = ch & 7;
      *(uint4*)(D + row * 64 + wg_swz(row, c, 8) * 8) = make_uint4(0, 0, 0, 0);
    }
    __syncthreads();
  }
  int it = blockIdx.x;
  if (it < p.nitems) {
    load(it, buf0);
    if constexpr (POOL) __syncthreads();  // the LDS-DMA'd stem rows landed (vmcnt(0) + barrier)
    store(buf0);
  }
  __syncthreads();
  for (int k = 0; it < p.nitems; it += gridDim.x, ++k) {
    const bool more = it + (int)gridDim.x < p.nitems;  // workgroup-uniform
    bf16_t* next = (k & 1) ? buf0 : buf1;
    if (more) load(it + gridDim.x, next);
    compute((k & 1) ? buf1 : buf0);
    if (more) {
      if constexpr (POOL) __syncthreads();
      store(next);
    }
    __syncthreads();
  }
  // partial dW[n][k] of this workgroup: C[i = n][j = k], row n = 4*(lane>>4) + r, col k = lane & 15
  float* out = p.slab + (long long)blockIdx.x * 64 * 672;
#pragma unroll
  for (int nf = 0; nf < NAF; ++nf)
#pragma unroll
    for (int j = 0; j < KFW; ++j) {
      const int kf = kf0 + j;
      if (kf < kf_end) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          out[(long long)(nf * 16 + (lane >> 4) * 4 + r) * 672 + kf * 16 + (lane & 15)] =
              U8 ? acc[nf][j][r] * (1.0f / 255.0f) : acc[nf][j][r];
      }
    }
}

// ---------------------------------------------------------------------------------------
// Stem forward (same paired-width geometry) as a halo-tiled direct convolution with the whole
// packed weight [64][672] resident in LDS (loaded once per workgroup, rows padded to 1376 B so
// every ds_read_b128 lane group of the A-fragment reads hits 16 distinct 16-B bank windows). Work item = HR output rows of one (clip, to); its
// halo is staged through registers (loaded one item ahead) into a single LDS buffer. Every
// operand address is a per-lane constant plus a compile-time immediate (W2 is a template
// parameter), so the 21-step K loop is ds_reads + MFMAs only. Waves split the 64 output
// channels in halves and the item's positions in halves (2 x 7 tiles of 16x16). Epilogue:
// bf16 stores of 4 channels per lane and BN partial statistics of the stored values, kept in
// registers across items and reduced once: stats[block][2][64].
constexpr int STF_LDW = 688;  // padded LDS row of the weight: 86 16-B chunks, conflict-free b128 groups
// Diagnostic ablations (A/B libraries only: python csrc/build.py --define STEM_ABLATE=N; results
// are garbage): bit 0 no output stores, bit 1 no halo loads, bit 2 no MFMAs
#ifndef STEM_ABLATE
#define STEM_ABLATE 0
#endif

struct StemFwdParams {
  const bf16_t* x;   // [B, T, H, W2, 8]
  const bf16_t* w;   // packed [64][Kpad] bf16
  bf16_t* y;         // [M, 64]
  float* stats;      // [gridDim][2][64]
  const float* shift;  // [64] subtracted before the bf16 rounding (the BN's running mean) or null
  int B, T, H, To, Ho, Kpad;
  int nitems;
  long long x_bytes;
};

// HR output rows per item, NPG position groups: 2 * NPG waves (two channel halves per group).
// NPG 4 = two waves per SIMD, so one wave's fragment reads overlap the other's MFMAs.
template <int W2, bool U8, int HR, int NPG, int CW = 2>
__global__ __launch_bounds__(64 * (4 / CW) * NPG, 1) void stem_fwd_kernel(StemFwdParams p) {
  // CW: 16-channel fragments per wave (2: the two channel halves on wave pairs; 4: every wave all
  // 64 channels, NPG position groups -- fewer fragment reads per MFMA, the B fragments are read once)
  static_assert(CW == 2 || CW == 4, "channel fragments per wave");
  constexpr int NSPL = 4 / CW;                     // waves per position group
  constexpr int NT = 64 * NSPL * NPG;
  constexpr int WO = W2, WPX = W2 + 4, HROWS = 2 * HR + 5;
  constexpr int HALO = 3 * HROWS * WPX;
  constexpr int ROWS = HR * WO;                    // positions per item
  constexpr int PF = (ROWS + 15) / 16;             // 16-position fragments
  constexpr int PFW = (PF + NPG - 1) / NPG;        // per wave (at most)
  constexpr int HREG = (HALO + NT - 1) / NT;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* Ws = (bf16_t*)smem;                      // [64][STF_LDW]
  bf16_t* X = Ws + 64 * STF_LDW;                   // [HALO][8]
  float* red = (float*)X;  // [NPG][128] stats, one row per position group: reuses the halo after the last item

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nh = NSPL == 2 ? (wave & 1) : 0, ph = NSPL == 2 ? (wave >> 1) : wave;
  const int cbase = nh * 16 * CW;                  // this wave's first output channel
  const int l16 = lane & 15, lg = lane >> 4;
  const auto xrs = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, (int)p.x_bytes, 0x00020000);
  const int hg_per = p.Ho / HR;

  // weight -> LDS (once); for the uint8 clip (integer-valued bf16 halo) scaled by 1/255 here
  for (int c = tid; c < 64 * 84; c += NT) {
    const int n = c / 84, k8 = c - n * 84;
    uint4 wv = *(const uint4*)(p.w + (long long)n * p.Kpad + k8 * 8);
    if constexpr (U8) {
      float f[8];
      unpack8(wv, f);
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] *= 1.0f / 255.0f;
      wv = pack8(f);
    }
    *(uint4*)(Ws + n * STF_LDW + k8 * 8) = wv;
  }
  using HReg = typename std::conditional<U8, uint2, uint4>::type;
  HReg hreg[HREG];
  // uint8 clip: converted (integer-valued bf16) part-way through the current item's K loop, where
  // the VALU work issues between MFMAs and the prefetch has had time to land; store() copies
  uint4 hcv[U8 ? HREG : 1];
  auto convert = [&]() {
    if constexpr (U8) {
#pragma unroll
      for (int i = 0; i < HREG; ++i) hcv[i] = u8x8_to_bf16x8(hreg[i]);
    }
  };
  // item-invariant part of this thread's halo pixels: (tt, hh, wp) packed, -1 past the halo
  int hgeo[HREG];
#pragma unroll
  for (int i = 0; i < HREG; ++i) {
    const int f = tid + NT * i;
    const int tt = f / (HROWS * WPX), rem = f - tt * (HROWS * WPX);
    const int hh = rem / WPX, wp = rem - hh * WPX;
    hgeo[i] = f < HALO ? (tt | (hh << 2) | (wp << 8)) : -1;
  }
  auto load = [&](int it) {
    if constexpr ((STEM_ABLATE & 2) != 0) return;
    const int hg = it % hg_per, q = it / hg_per;
    const int to = q % p.To, b = q / p.To;
    const int t0 = 2 * to - 1, h0 = 2 * hg * HR - 3;
    const int base = ((b * p.T + t0) * p.H + h0) * W2 - 2;  // pixel index of (tt, hh, wp) = (0, 0, 0)
#pragma unroll
    for (int i = 0; i < HREG; ++i) {
      const int gq = hgeo[i];
      const int tt = gq & 3, hh = (gq >> 2) & 63, wp = gq >> 8;
      const bool v = gq >= 0 && (unsigned)(t0 + tt) < (unsigned)p.T && (unsigned)(h0 + hh) < (unsigned)p.H &&
                     (unsigned)(wp - 2) < (unsigned)W2;
      hreg[i] = stem_px_load<U8>(xrs, v, base + (tt * p.H + hh) * W2 + wp);
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int i = 0; i < HREG; ++i) {
      const int f = tid + NT * i;
      if constexpr (U8) {
        if (f < HALO) *(uint4*)(X + f * 8) = hcv[i];
      } else {
        if (f < HALO) *(uint4*)(X + f * 8) = hreg[i];
      }
    }
  };

  // per-lane constant operand addresses (bytes): A rows of the two channel fragments, B pixels
  // of this wave's position fragments (tail positions clamped to a real one; never stored)
  uint32_t abase[CW], bbase[PFW];
#pragma unroll
  for (int nf = 0; nf < CW; ++nf)
    abase[nf] = (uint32_t)(((cbase + nf * 16 + l16) * STF_LDW + lg * 8) * 2);
  const int pf0 = ph * PF / NPG;  // balanced split of the PF fragments over the groups
  const int npf = (ph + 1) * PF / NPG - pf0;
#pragma unroll
  for (int j = 0; j < PFW; ++j) {
    int pos = (pf0 + j) * 16 + l16;
    pos = pos < ROWS ? pos : ROWS - 1;
    const int hr = pos / WO, wo = pos - hr * WO;
    // absolute LDS byte address (X follows the weight), so only the per-step tap offset
    // (<= 40 KB) is left for the ds_read immediate
    bbase[j] = (uint32_t)(64 * STF_LDW * 2 + (((2 * hr) * WPX + wo + lg) * 8) * 2);
  }
  const char* Wb = (const char*)Ws;
  const char* Xb = (const char*)smem;

  float s1[CW][4], s2[CW][4], shv[CW][4];
#pragma unroll
  for (int nf = 0; nf < CW; ++nf)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      s1[nf][r] = 0.f;
      s2[nf][r] = 0.f;
      shv[nf][r] = p.shift != nullptr ? p.shift[cbase + nf * 16 + lg * 4 + r] : 0.f;
    }
  // the shift loads are conditional: left pending into the item loop, the compiler's waits merge
  // them with the loop's paths and drained every epilogue's output stores (vmcnt(0) per fragment)
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)

  int it = blockIdx.x;
  if (it < p.nitems) {
    load(it);
    convert();
    store();
  }
  if (it + (int)gridDim.x < p.nitems) load(it + gridDim.x);
  __syncthreads();
  for (; it < p.nitems; it += gridDim.x) {
    f32x4 acc[CW][PFW];
#pragma unroll
    for (int nf = 0; nf < CW; ++nf)
#pragma unroll
      for (int j = 0; j < PFW; ++j) acc[nf][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 21; ++ks) {
      if (U8 && ks == 12 && it + (int)gridDim.x < p.nitems) convert();
      const int dt = ks / 7, dh = ks % 7;
      const uint32_t boff = (uint32_t)(((dt * HROWS + dh) * WPX) * 16);
      bf16x8 af[CW], bf[PFW];
#pragma unroll
      for (int nf = 0; nf < CW; ++nf) af[nf] = *(const bf16x8*)(Wb + abase[nf] + ks * 64);
#pragma unroll
      for (int j = 0; j < PFW; ++j) bf[j] = *(const bf16x8*)(Xb + bbase[j] + boff);
#pragma unroll
      for (int j = 0; j < PFW; ++j)
        if (j < npf && !(STEM_ABLATE & 4))
#pragma unroll
          for (int nf = 0; nf < CW; ++nf)
            acc[nf][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[nf], bf[j], acc[nf][j], 0, 0, 0);
    }
    // epilogue: C[i = n][j = p]: lane holds channels 4*lg + r of position l16
    const int hg = it % hg_per, q = it / hg_per;
    const long long m0 = ((long long)q * p.Ho + hg * HR) * WO;
#pragma unroll
    for (int j = 0; j < PFW; ++j) {
      const int pos = (pf0 + j) * 16 + l16;
      if (j < npf && pos < ROWS) {  // (uniform over the lane pairs lg, lg ^ 1: same position)
        uint2 o[CW];
#pragma unroll
        for (int nf = 0; nf < CW; ++nf) {
          const f32x4 v = acc[nf][j];
          o[nf].x = pack2bf(v[0] - shv[nf][0], v[1] - shv[nf][1]);
          o[nf].y = pack2bf(v[2] - shv[nf][2], v[3] - shv[nf][3]);
          const float q0 = __uint_as_float(o[nf].x << 16), q1 = __uint_as_float(o[nf].x & 0xffff0000u);
          const float q2 = __uint_as_float(o[nf].y << 16), q3 = __uint_as_float(o[nf].y & 0xffff0000u);
          s1[nf][0] += q0; s1[nf][1] += q1; s1[nf][2] += q2; s1[nf][3] += q3;
          s2[nf][0] += q0 * q0; s2[nf][1] += q1 * q1; s2[nf][2] += q2 * q2; s2[nf][3] += q3 * q3;
        }
        // 16-B stores: lanes lg = 2a, 2a + 1 swap halves, so lane 2a holds channels 8a .. 8a + 7 of
        // fragment 0 and lane 2a + 1 channels 16 + 8a .. of fragment 1; a wave's stores then cover
        // 64 contiguous bytes per position (8-B stores left 32-B pieces of the 128-B rows)
        const bool odd = lg & 1;
#pragma unroll
        for (int k = 0; k < CW / 2; ++k) {  // fragment pairs (2k, 2k + 1): 32 channels each
          const uint2 snd = odd ? o[2 * k] : o[2 * k + 1];
          uint2 rcv;
          rcv.x = (uint32_t)__shfl_xor((int)snd.x, 16, 64);
          rcv.y = (uint32_t)__shfl_xor((int)snd.y, 16, 64);
          const uint4 st = odd ? make_uint4(rcv.x, rcv.y, o[2 * k + 1].x, o[2 * k + 1].y)
                               : make_uint4(o[2 * k].x, o[2 * k].y, rcv.x, rcv.y);
          const int ch = cbase + k * 32 + (odd ? 16 + (lg - 1) * 4 : lg * 4);
          if (!(STEM_ABLATE & 1)) *(uint4*)(p.y + (m0 + pos) * 64 + ch) = st;
        }
      }
    }
    lds_barrier();  // every wave done reading this item's halo (output stores stay in flight)
    const bool more = it + (int)gridDim.x < p.nitems;
    if (more) store();
    if (it + 2 * (int)gridDim.x < p.nitems) load(it + 2 * gridDim.x);
    lds_barrier();  // LDS only: the register prefetch of item it + 2 * grid stays in flight
  }
  // statistics: reduce over the 16 lanes of a channel group, then over the position groups in a
  // fixed order (each group's partials in its own LDS row: deterministic, no LDS atomics)
  __syncthreads();  // every wave is done reading the halo the rows overwrite
#pragma unroll
  for (int nf = 0; nf < CW; ++nf)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float a = s1[nf][r], b2 = s2[nf][r];
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) { a += __shfl_xor(a, o, 64); b2 += __shfl_xor(b2, o, 64); }
      if (l16 == 0) {
        const int c = cbase + nf * 16 + lg * 4 + r;
        red[ph * 128 + c] = a;
        red[ph * 128 + 64 + c] = b2;
      }
    }
  __syncthreads();
  if (tid < 128) {
    float v = red[tid];
#pragma unroll
    for (int g = 1; g < NPG; ++g) v += red[g * 128 + tid];
    p.stats[(long long)blockIdx.x * 128 + tid] = v;
  }
}

template <int W2, bool U8, int HR, int NPG, int CW = 2>
static int launch_stem_fwd_t(StemFwdParams& p, int grid, hipStream_t stream) {
  constexpr int HALO = 3 * (2 * HR + 5) * (W2 + 4);
  constexpr size_t lds = (size_t)64 * STF_LDW * 2 + (size_t)HALO * 16;
  static_assert((size_t)HALO * 16 >= (size_t)NPG * 128 * 4, "statistics rows reuse the halo");
  static_assert(lds <= 160 * 1024, "stem forward LDS");
  static bool attr_set = false;
  if (!attr_set) {
    HIP_RET(hipFuncSetAttribute((const void*)stem_fwd_kernel<W2, U8, HR, NPG, CW>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr_set = true;
  }
  hipLaunchKernelGGL((stem_fwd_kernel<W2, U8, HR, NPG, CW>), dim3(grid), dim3(64 * (4 / CW) * NPG), lds, stream, p);
  return (int)hipGetLastError();
}

// Stem forward variant (MILNCE_STEM_FWD_V, read once): 1 = 4 output rows per item on 8 waves, two
// channel halves per position group (default), 2 = the same with every wave on all 64 channels
// and 8 position groups (22 % fewer fragment reads per MFMA; measured equal: 1.960 vs 1.963 ms,
// so the K loop is not LDS-read bound), 0 = 2 rows per item on 4 waves (the round-1 kernel).
static int stem_fwd_variant() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("MILNCE_STEM_FWD_V");
    v = e ? atoi(e) : 1;
  }
  return v;
}

static int stem_fwd_hr() { return stem_fwd_variant() == 0 ? 2 : 4; }

template <int W2, bool U8>
static int launch_stem_fwd(StemFwdParams& p, int grid, hipStream_t stream) {
  if (stem_fwd_variant() == 0) return launch_stem_fwd_t<W2, U8, 2, 2>(p, grid, stream);
  if (stem_fwd_variant() == 2) return launch_stem_fwd_t<W2, U8, 4, 8, 4>(p, grid, stream);
  return launch_stem_fwd_t<W2, U8, 4, 4>(p, grid, stream);
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

// Every registered weight of the step packed in ONE launch (ops/hip_ops.py _WeightPacker): a
// descriptor per (weight, mode), blocks assigned by prefix (blk0); element mapping identical to
// pack_weight_kernel. Replaces ~100 tiny per-conv pack launches per training step.
struct PackDesc {
  const float* w;
  bf16_t* out;
  // ldo: row stride of out (0: Kpad). A concatenated 1x1 group weight packs as one descriptor
  // per member weight writing its row (mode 0) or column (mode 1) slice of the shared buffer.
  int Cout, Cin, Cin_p, KT, KH, KW, Npad, Kpad, mode, blk0, ldo, pad1;
};
static_assert(sizeof(PackDesc) == 64, "PackDesc layout is mirrored by a ctypes.Structure");
constexpr int PACK_ITEMS = 8;  // elements per thread per block

__global__ __launch_bounds__(256) void pack_weight_multi_kernel(const PackDesc* __restrict__ descs, int n) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (descs[mid].blk0 <= (int)blockIdx.x) lo = mid; else hi = mid - 1;
  }
  const PackDesc d = descs[lo];
  const int taps = d.KT * d.KH * d.KW;
  const long long total = (long long)d.Npad * d.Kpad;
  const long long base = (long long)(blockIdx.x - d.blk0) * 256 * PACK_ITEMS + threadIdx.x;
#pragma unroll
  for (int i = 0; i < PACK_ITEMS; ++i) {
    const long long idx = base + (long long)i * 256;
    if (idx >= total) break;
    const int nn = idx / d.Kpad;
    const int k = idx % d.Kpad;
    float v = 0.f;
    if (d.mode == 0) {
      const int tap = k / d.Cin, c = k % d.Cin;
      if (nn < d.Cout && tap < taps && c < d.Cin_p) v = d.w[((long long)nn * d.Cin_p + c) * taps + tap];
    } else {
      const int tap2 = k / d.Cout, co = k % d.Cout;
      if (nn < d.Cin_p && tap2 < taps) v = d.w[((long long)co * d.Cin_p + nn) * taps + (taps - 1 - tap2)];
    }
    d.out[d.ldo ? (long long)nn * d.ldo + k : idx] = f2bf(v);
  }
}

int g_milnce_lds_floor = 0;
MILNCE_API int milnce_set_lds_floor(int bytes) {
  const int old = g_milnce_lds_floor;
  g_milnce_lds_floor = bytes < 0 ? 0 : bytes;
  return old;
}

MILNCE_API int milnce_pack_weights_multi(const void* descs, int n, int total_blocks, hipStream_t stream) {
  if (n <= 0 || total_blocks <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(pack_weight_multi_kernel, dim3(total_blocks), dim3(256), 0, stream, (const PackDesc*)descs, n);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------
template <int BM, int BN, int BK, bool U8, int EPI>
static int launch_fwd_epi(ConvParams& p, hipStream_t stream) {
  const size_t kloop = (size_t)2 * (BM + BN) * BK * 2;
  const size_t epi = (size_t)BM * (BN + 8) * 2;
  const size_t lds = (kloop > epi ? kloop : epi) + 8 * 160 + 16 * BN;  // + tap table + producer-BN consts
  static bool attr_set = false;
  if (!attr_set) {
    HIP_RET(hipFuncSetAttribute((const void*)conv_fwd_kernel<BM, BN, BK, U8, EPI>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr_set = true;
  }
  const int nblocks = p.num_n_tiles * p.grid_m;
  hipLaunchKernelGGL((conv_fwd_kernel<BM, BN, BK, U8, EPI>), dim3(nblocks), dim3(256), lds, stream, p);
  return (int)hipGetLastError();
}

template <int BN, int BK, int STAGES, int EPI, int NWM = 2>
static int launch_fwd_v3(ConvParams& p, hipStream_t stream) {
  constexpr int BM = 64 * NWM;
  constexpr size_t ring = (size_t)STAGES * (BM + BN) * BK * 2;
  constexpr size_t epi = (size_t)BM * (BN + 8) * 2 + (EPI == 2 ? 16 * BN : 0);
  const size_t lds_v3 = (ring > epi ? ring : epi) + (EPI == 1 ? 4 * BN : 0);  // + the EPI 1 shift (shl)
  static bool attr_set = false;
  if (!attr_set) {
    HIP_RET(hipFuncSetAttribute((const void*)conv_fwd_v3_kernel<BN, BK, STAGES, EPI, NWM>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr_set = true;
  }
  ConvParams q = p;
  q.num_m_tiles = (p.M + BM - 1) / BM;
  const int nblocks = q.num_n_tiles * q.grid_m;
  hipLaunchKernelGGL((conv_fwd_v3_kernel<BN, BK, STAGES, EPI, NWM>), dim3(nblocks), dim3(128 * NWM), lds_v3, stream, q);
  return (int)hipGetLastError();
}

// Kernel variants (the host autotunes per conv shape, ops/hip_ops.py):
//   2: register-staged double buffer; 3: LDS-DMA ring, BK as planned, 3 stages;
//   4: LDS-DMA ring, 2 stages (2 blocks/CU at BN 128); 5: LDS-DMA ring, BK 32, 4 stages.
template <int BN, int BK, int S, int NWM = 2>
static int launch_v3_epi(ConvParams& p, hipStream_t stream) {
  if (p.bn_mode == 0) return launch_fwd_v3<BN, BK, S, 0, NWM>(p, stream);
  if (p.bn_mode == 1) return launch_fwd_v3<BN, BK, S, 1, NWM>(p, stream);
  return launch_fwd_v3<BN, BK, S, 2, NWM>(p, stream);
}

//   6: 256-row tiles (8 waves), BK as planned, 3 stages; 7: same, 2 stages.
// A variant exists for an N tile only if its B rows split evenly into the 1-KiB DMA pieces of
// all waves (rows per piece 512 / BK, times the wave count); other requests run variant 3.
template <int BN, int BK, int NWAVES>
constexpr bool v3_fits() { return BN % ((512 / BK) * NWAVES) == 0; }

template <int BN, int BK>
static int launch_v3_impl(ConvParams& p, int impl, hipStream_t stream) {
  if constexpr (v3_fits<BN, BK, 8>()) {
    if (impl == 7) return launch_v3_epi<BN, BK, 2, 4>(p, stream);
    if constexpr (3 * (256 + BN) * BK * 2 <= 160 * 1024) {  // 3-stage ring within the LDS
      if (impl == 6) return launch_v3_epi<BN, BK, 3, 4>(p, stream);
    }
  }
  if constexpr (v3_fits<BN, 32, 4>()) {
    if (impl == 5) return launch_v3_epi<BN, 32, 4>(p, stream);
  }
  if (impl == 4) return launch_v3_epi<BN, BK, 2>(p, stream);
  return launch_v3_epi<BN, BK, 3>(p, stream);
}

template <int BM, int BN, int BK, bool U8>
static int launch_fwd(ConvParams& p, int impl, hipStream_t stream) {
  if constexpr (!U8) {
    if (impl >= 3) return launch_v3_impl<BN, BK>(p, impl, stream);
  }
  if constexpr (U8) {
    if (p.bn_mode == 0) return launch_fwd_epi<BM, BN, BK, true, 0>(p, stream);
    return p.bn_mode == 1 ? launch_fwd_epi<BM, BN, BK, true, 1>(p, stream) : (int)hipErrorInvalidValue;
  } else {
    if (p.bn_mode == 0) return launch_fwd_epi<BM, BN, BK, false, 0>(p, stream);
    if (p.bn_mode == 1) return launch_fwd_epi<BM, BN, BK, false, 1>(p, stream);
    return launch_fwd_epi<BM, BN, BK, false, 2>(p, stream);
  }
}

// x: input, w: packed weight [Npad][Kpad], y: out [M][ldy], stats: [grid_m][2][Npad] or null.
// Returns grid_m through *grid_m_out (for sizing the stats buffer, call with y == nullptr).
static int conv_fwd_impl(const void* x, int x_u8, const void* w, void* y, float* stats, const void* bn_y,
                         const float* bn_ss, int bn_ld,
                         int B, int T, int H, int W, int Cin, int Cout,
                         int KT, int KH, int KW, int st, int sh, int sw, int pt, int ph, int pw,
                         int Kpad, int Npad, int ldy, int bn, int bk, int grid_m, int wo_override,
                         int impl, const BoxPro& pro, hipStream_t stream) {
  ConvParams p;
  p.x = x; p.w = (const bf16_t*)w; p.y = (bf16_t*)y; p.stats = stats;
  p.bn_y = (const bf16_t*)bn_y; p.bn_ss = bn_ss; p.bn_ld = bn_ld;
  if (KT * KH * KW > 160) return (int)hipErrorInvalidValue;  // tap table capacity
  p.bn_mode = stats == nullptr ? 0 : (bn_y == nullptr ? 1 : 2);
  if (p.bn_mode == 2 && (Cout % 8 || ldy != Cout)) return (int)hipErrorInvalidValue;
  p.T = T; p.H = H; p.W = W; p.Cin = Cin;
  p.To = (T + 2 * pt - KT) / st + 1;
  p.Ho = (H + 2 * ph - KH) / sh + 1;
  p.Wo = wo_override > 0 ? wo_override : (W + 2 * pw - KW) / sw + 1;  // override: asymmetric w padding
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
  p.fCin = make_fastdiv(Cin);
  p.fKW = make_fastdiv(KW); p.fKH = make_fastdiv(KH);
  p.x_total_bytes = (long long)B * p.x_bstride * (x_u8 ? 1 : 2);
  if (impl >= 14 && impl <= 17)  // conv_box.hip
    return x_u8 ? V4_UNSUPPORTED : launch_fwd_box(p, bn, impl, pro, stream);
  if (impl >= 8) return x_u8 ? V4_UNSUPPORTED : launch_fwd_v4(p, bn, impl, stream);  // conv_v4.hip
  if (!x_u8 && (bn == 96 || bn == 160 || bn == 192)) {
    // wide / odd N tiles: LDS-DMA ring variants only, BK 64
    if (bk != 64) return (int)hipErrorInvalidValue;
    const int im = impl >= 3 ? impl : 4;
    if (bn == 96) return launch_v3_impl<96, 64>(p, im, stream);
    if (bn == 160) return launch_v3_impl<160, 64>(p, im, stream);
    return launch_v3_impl<192, 64>(p, im, stream);
  }
  if (x_u8) {
    if (bn == 64 && bk == 32) return launch_fwd<128, 64, 32, true>(p, impl, stream);
    if (bn == 64 && bk == 64) return launch_fwd<128, 64, 64, true>(p, impl, stream);
    if (bn == 128 && bk == 32) return launch_fwd<128, 128, 32, true>(p, impl, stream);
    if (bn == 128 && bk == 64) return launch_fwd<128, 128, 64, true>(p, impl, stream);
  } else {
    if (bn == 64 && bk == 32) return launch_fwd<128, 64, 32, false>(p, impl, stream);
    if (bn == 64 && bk == 64) return launch_fwd<128, 64, 64, false>(p, impl, stream);
    if (bn == 128 && bk == 32) return launch_fwd<128, 128, 32, false>(p, impl, stream);
    if (bn == 128 && bk == 64) return launch_fwd<128, 128, 64, false>(p, impl, stream);
  }
  return (int)hipErrorInvalidValue;
}

// stats set, bn_y null (BN forward statistics, epilogue mode 1): bn_ss, when set, is a per-channel
// shift [Cout] (the BN's running mean) subtracted from the outputs before their bf16 rounding; the
// statistics are those of the shifted values and milnce_bn_finalize adds the shift back.
// bn_y set: mode 2 (dgrad with the producer BN's backward partials), bn_ss = its [4][C] constants.
MILNCE_API int milnce_conv_fwd(const void* x, int x_u8, const void* w, void* y, float* stats, const void* bn_y,
                               const float* bn_ss, int bn_ld,
                               int B, int T, int H, int W, int Cin, int Cout,
                               int KT, int KH, int KW, int st, int sh, int sw, int pt, int ph, int pw,
                               int Kpad, int Npad, int ldy, int bn, int bk, int grid_m, int wo_override,
                               int impl, hipStream_t stream) {
  return conv_fwd_impl(x, x_u8, w, y, stats, bn_y, bn_ss, bn_ld, B, T, H, W, Cin, Cout, KT, KH, KW, st, sh, sw, pt,
                       ph, pw, Kpad, Npad, ldy, bn, bk, grid_m, wo_override, impl, BoxPro(), stream);
}

// Forward whose input x is the raw conv output of a BN layer: z = relu(x * scale + shift) (pro_ss
// = that layer's [4][Cin] mean / invstd / scale / shift) is applied while the box-tiled kernel
// stages its input, and written to pro_z (dense; the consumer's wgrad operand; null: not needed).
// x_ld: x's row stride in elements (x may be a channel slice of a concatenated conv output).
// Box-tiled variants only (impl 14-17); anything else returns V4_UNSUPPORTED.
MILNCE_API int milnce_conv_fwd_pro(const void* x, int x_ld, const void* w, void* y, float* stats,
                                   const float* y_shift, const float* pro_ss, void* pro_z, int B, int T, int H,
                                   int W, int Cin, int Cout,
                                   int KT, int KH, int KW, int pt, int ph, int pw, int Kpad, int Npad, int ldy,
                                   int bn, int grid_m, int impl, hipStream_t stream) {
  if (impl < 14 || impl > 17) return V4_UNSUPPORTED;
  BoxPro pro;
  pro.ss = pro_ss;
  pro.z = pro_z;
  pro.xld = x_ld;
  return conv_fwd_impl(x, 0, w, y, stats, nullptr, y_shift, 0, B, T, H, W, Cin, Cout, KT, KH, KW, 1, 1, 1, pt, ph,
                       pw, Kpad, Npad, ldy, bn, 64, grid_m, 0, impl, pro, stream);
}

// dgrad of a conv whose output went through BN -> ReLU, from dz (the gradient of the ReLU output)
// instead of dy: the box-tiled kernel stages dy = k0 * (dz * mask - k1 - xhat * k2) (y, ss: that
// BN's raw conv output and [4][C] constants; coef: [3][C] from milnce_bn_bwd_finalize) and writes
// dy to dy_out (the wgrad operand). part / bn_y / bn_ss / bn_ld: the producer-BN partials of dX as
// in milnce_conv_fwd. Box-tiled variants with N tiles <= 128 only (else V4_UNSUPPORTED).
MILNCE_API int milnce_conv_dgrad_bnbwd(const void* dz, const void* wd, void* dx, float* part, const void* bn_y,
                                       const float* bn_ss, int bn_ld, const void* y, const float* ss,
                                       const float* coef, void* dy_out, int B, int T, int H, int W, int C,
                                       int Cx, int KT, int KH, int KW, int pt, int ph, int pw, int Kpad, int Npad,
                                       int bn, int grid_m, int impl, hipStream_t stream) {
  if (impl < 14 || impl > 17) return V4_UNSUPPORTED;
  BoxPro pro;
  pro.ss = ss;
  pro.z = dy_out;
  pro.y = y;
  pro.coef = coef;
  return conv_fwd_impl(dz, 0, wd, dx, part, bn_y, bn_ss, bn_ld, B, T, H, W, C, Cx, KT, KH, KW, 1, 1, 1, pt, ph, pw,
                       Kpad, Npad, Cx, bn, 64, grid_m, 0, impl, pro, stream);
}

template <int TN_, int TK_, bool U8, bool DEEP = false>
static int launch_wgrad(WgradParams& p, hipStream_t stream) {
  const size_t lds = (size_t)2 * WG_R * ((TN_ + 16) + (TK_ + wg_xpad<TK_>())) * 2 + 4 * WG_R * sizeof(int2);
  static bool attr_set = false;
  if (!attr_set) {
    HIP_RET(hipFuncSetAttribute((const void*)conv_wgrad_kernel<TN_, TK_, U8, DEEP>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr_set = true;
  }
  const int nblocks = p.n_tiles * p.k_tiles * p.splits;
  hipLaunchKernelGGL((conv_wgrad_kernel<TN_, TK_, U8, DEEP>), dim3(nblocks), dim3(256),
                     lds_floor(conv_wgrad_kernel<TN_, TK_, U8, DEEP>, lds), stream, p);
  return (int)hipGetLastError();
}

template <int TN_, int TK_, int STAGES>
static int launch_wgrad_v3(WgradParams& p, hipStream_t stream) {
  static_assert((size_t)STAGES * WG_R * (TN_ + TK_) * 2 <= 160 * 1024, "static LDS ring");
  const int nblocks = p.n_tiles * p.k_tiles * p.splits;
  hipLaunchKernelGGL((conv_wgrad_v3_kernel<TN_, TK_, STAGES>), dim3(nblocks), dim3(256),
                     lds_floor(conv_wgrad_v3_kernel<TN_, TK_, STAGES>, 0), stream, p);
  return (int)hipGetLastError();
}

template <int TN_, int TK_>
static int launch_wgrad_impl(WgradParams& p, int impl, hipStream_t stream) {
  if constexpr (TK_ == 192) {
    // 192-wide K tiles (Ktot = 576, 1152, ...: a third of the dY re-reads of 64-wide tiles)
    // exist only register-staged (the LDS-DMA mapping needs TK / 8 to divide 64); the 2-deep
    // variant fits the 256 VGPRs of two waves per SIMD only at TN 64
    if constexpr (TN_ == 64) {
      if (impl == 5) return launch_wgrad<TN_, TK_, false, true>(p, stream);
    }
    if (impl == 2) return launch_wgrad<TN_, TK_, false>(p, stream);
    return (int)hipErrorInvalidValue;
  } else if constexpr (TN_ % 64 != 0) {
    // wide N tiles (96 / 192: Cout = 96, 192, 288, 384, ... without padding) exist only as the
    // register-staged kernels (the LDS-DMA mapping needs TN / 8 to divide 64); the 2-deep
    // variant of 192 x 128 would spill
    if constexpr (!(TN_ == 192 && TK_ == 128)) {
      if (impl == 5) return launch_wgrad<TN_, TK_, false, true>(p, stream);
    }
    if (impl == 2) return launch_wgrad<TN_, TK_, false>(p, stream);
    return (int)hipErrorInvalidValue;
  } else {
    if (impl == 5) return launch_wgrad<TN_, TK_, false, true>(p, stream);
    if (impl == 4) return launch_wgrad_v3<TN_, TK_, 2>(p, stream);
    if (impl == 3) return launch_wgrad_v3<TN_, TK_, 3>(p, stream);
    return launch_wgrad<TN_, TK_, false>(p, stream);
  }
}

int launch_wgrad_reduce(const float* slab, float* dw, int splits, int Npad, int Kpad, int Cout, int Cin,
                        int Cin_param, int taps, int accumulate, hipStream_t stream);

MILNCE_API int milnce_conv_wgrad(const void* dy, int ldd, const void* x, int x_u8, float* slab, float* dw,
                                 int B, int T, int H, int W, int Cin, int Cin_param, int Cout,
                                 int KT, int KH, int KW, int st, int sh, int sw, int pt, int ph, int pw,
                                 int Kpad, int Npad, int tn, int tk, int splits, int accumulate, int wo_override,
                                 int impl, hipStream_t stream) {
  WgradParams p;
  p.dy = (const bf16_t*)dy; p.x = x; p.slab = slab;
  p.T = T; p.H = H; p.W = W; p.Cin = Cin;
  p.To = (T + 2 * pt - KT) / st + 1;
  p.Ho = (H + 2 * ph - KH) / sh + 1;
  p.Wo = wo_override > 0 ? wo_override : (W + 2 * pw - KW) / sw + 1;
  p.Cout = Cout; p.ldd = ldd;
  p.KT = KT; p.KH = KH; p.KW = KW; p.st = st; p.sh = sh; p.sw = sw; p.pt = pt; p.ph = ph; p.pw = pw;
  p.Ktot = KT * KH * KW * Cin; p.Kpad = Kpad; p.Npad = Npad;
  p.M = B * p.To * p.Ho * p.Wo;
  p.x_bstride = (long long)T * H * W * Cin;
  p.n_tiles = Npad / tn;
  p.k_tiles = Kpad / tk;
  p.splits = splits;
  p.rows_per_split = ((p.M + splits - 1) / splits + WG_R - 1) / WG_R * WG_R;
  p.in_scale = x_u8 ? (1.0f / 255.0f) : 1.0f;
  p.fWo = make_fastdiv(p.Wo); p.fHo = make_fastdiv(p.Ho); p.fTo = make_fastdiv(p.To);
  p.fCin = make_fastdiv(Cin);
  p.x_total_bytes = (long long)B * p.x_bstride * (x_u8 ? 1 : 2);
  p.dy_total_bytes = (long long)p.M * ldd * 2;
  // per-split descriptor bases keep offsets 32-bit; one split's rows must fit in 2 GB
  if ((long long)p.rows_per_split * ldd * 2 > 0x7FFFFFF0LL) return (int)hipErrorInvalidValue;
  int rc;
  if (x_u8) {
    if (tn == 64 && tk == 64) rc = launch_wgrad<64, 64, true>(p, stream);
    else if (tn == 64 && tk == 128) rc = launch_wgrad<64, 128, true>(p, stream);
    else rc = (int)hipErrorInvalidValue;
  } else {
    if (tn == 64 && tk == 64) rc = launch_wgrad_impl<64, 64>(p, impl, stream);
    else if (tn == 64 && tk == 128) rc = launch_wgrad_impl<64, 128>(p, impl, stream);
    else if (tn == 128 && tk == 64) rc = launch_wgrad_impl<128, 64>(p, impl, stream);
    else if (tn == 128 && tk == 128) rc = launch_wgrad_impl<128, 128>(p, impl, stream);
    else if (tn == 96 && tk == 64) rc = launch_wgrad_impl<96, 64>(p, impl, stream);
    else if (tn == 96 && tk == 128) rc = launch_wgrad_impl<96, 128>(p, impl, stream);
    else if (tn == 192 && tk == 64) rc = launch_wgrad_impl<192, 64>(p, impl, stream);
    else if (tn == 192 && tk == 128) rc = launch_wgrad_impl<192, 128>(p, impl, stream);
    else if (tn == 96 && tk == 192) rc = launch_wgrad_impl<96, 192>(p, impl, stream);
    else if (tn == 128 && tk == 192) rc = launch_wgrad_impl<128, 192>(p, impl, stream);
    else if (tn == 64 && tk == 192) rc = launch_wgrad_impl<64, 192>(p, impl, stream);
    else rc = (int)hipErrorInvalidValue;
  }
  if (rc) return rc;
  if (dw == nullptr) return 0;  // the caller reduces the slab itself (milnce_wgrad_reduce, e.g. on a side stream)
  return launch_wgrad_reduce(slab, dw, splits, Npad, Kpad, Cout, Cin, Cin_param, KT * KH * KW, accumulate, stream);
}

// host launcher of the slab reduction, shared with csrc/conv_halo.hip
int launch_wgrad_reduce(const float* slab, float* dw, int splits, int Npad, int Kpad, int Cout, int Cin,
                        int Cin_param, int taps, int accumulate, hipStream_t stream) {
  const long long total = (long long)Cout * taps * Cin;
  const int grid = (int)((total + 63) / 64 < 16384 ? (total + 63) / 64 : 16384);
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(grid), dim3(64 * WR_GROUPS), 0, stream, slab, dw, splits, Npad, Kpad,
                     Cout, Cin, Cin_param, taps, accumulate);
  return (int)hipGetLastError();
}

// descs: host array of n ReduceDesc (blk0 / nblk filled here)
MILNCE_API int milnce_wgrad_reduce_batch(const void* descs, int n, hipStream_t stream) {
  if (n < 1 || n > REDUCE_BATCH_MAX) return (int)hipErrorInvalidValue;
  ReduceBatch b;
  int blk = 0;
  for (int i = 0; i < n; ++i) {
    b.d[i] = ((const ReduceDesc*)descs)[i];
    const long long total = (long long)b.d[i].Cout * b.d[i].taps * b.d[i].Cin;
    const long long want = (total + 63) / 64;
    b.d[i].nblk = (int)(want < 2048 ? (want < 1 ? 1 : want) : 2048);
    b.d[i].blk0 = blk;
    blk += b.d[i].nblk;
  }
  b.n = n;
  hipLaunchKernelGGL(wgrad_reduce_batch_kernel, dim3(blk), dim3(64 * WR_GROUPS), 0, stream, b);
  return (int)hipGetLastError();
}

// dW (+)= sum over the split slabs [splits][Npad][Kpad] of a wgrad (milnce_conv_wgrad /
// milnce_halo_wgrad called with dw == nullptr), into the parameter layout [Cout][Cin_param][taps].
MILNCE_API int milnce_wgrad_reduce(const float* slab, float* dw, int splits, int Npad, int Kpad, int Cout, int Cin,
                                   int Cin_param, int taps, int accumulate, hipStream_t stream) {
  return launch_wgrad_reduce(slab, dw, splits, Npad, Kpad, Cout, Cin, Cin_param, taps, accumulate, stream);
}

MILNCE_API int milnce_pack_weight(const float* w, void* out, int Cout, int Cin, int Cin_p, int KT, int KH,
                                  int KW, int Npad, int Kpad, int mode, hipStream_t stream) {
  const long long total = (long long)Npad * Kpad;
  const int grid = (int)((total + 255) / 256 < 2048 ? (total + 255) / 256 : 2048);
  hipLaunchKernelGGL(pack_weight_kernel, dim3(grid), dim3(256), 0, stream, w, (bf16_t*)out, Cout, Cin, Cin_p,
                     KT, KH, KW, Npad, Kpad, mode);
  return (int)hipGetLastError();
}

// Stem wgrad (see stem_wgrad_kernel): dW2 [64][8][3][7][4] (accumulated if `accumulate`).
// x2 is the bf16 clip as width pairs [B,T,H,W2,8], or (x_u8) the native uint8 clip read the same way.
// Returns hipErrorInvalidValue for geometries it does not cover (caller falls back).
template <bool U8, int NKQ, bool POOL>
static int stem_wgrad_launch(const StemWgradParams& p, int grid, size_t lds, hipStream_t stream) {
  static bool attr_set = false;
  if (!attr_set) {
    HIP_RET(hipFuncSetAttribute((const void*)stem_wgrad_kernel<U8, NKQ, POOL>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr_set = true;
  }
  hipLaunchKernelGGL((stem_wgrad_kernel<U8, NKQ, POOL>), dim3(grid), dim3(64 * NKQ), lds, stream, p);
  return (int)hipGetLastError();
}

// Geometry not covered by the stem kernels: the caller falls back to the generic implicit GEMM.
// Every other non-zero return is a HIP error and must be raised, not fallen back from.
constexpr int STEM_UNSUPPORTED = -1;

// pdy != nullptr: the POOL kernel (dY rebuilt from the maxpool_2a backward + BN backward, see
// stem_wgrad_kernel); dy is then unused.
static int stem_wgrad_impl(StemWgradParams& p, int x_u8, long long slab_floats, float* dw, int accumulate,
                           hipStream_t stream) {
  const int B = p.B, T = p.T, H = p.H, W2 = p.W2;
  p.To = (T + 2 - 3) / 2 + 1;
  p.Ho = (H + 6 - 7) / 2 + 1;
  p.Wo = W2;
  if (p.Ho % STW_HR) return STEM_UNSUPPORTED;
  p.nitems = B * p.To * (p.Ho / STW_HR);
  p.halo_px = 3 * (2 * STW_HR + 5) * (W2 + 4);
  if (p.halo_px > 256 * STW_HREG || STW_HR * p.Wo > 32 * STW_DREG) return STEM_UNSUPPORTED;
  const bool pool = p.pdy != nullptr;
  if (pool && (p.Wo % 2 || p.Wo > 112 || p.Ho % 2)) return STEM_UNSUPPORTED;
  p.dy_rows = (STW_HR * p.Wo + 31) / 32 * 32;
  p.x_bytes = (long long)B * T * H * W2 * (x_u8 ? 8 : 16);
  p.dy_bytes = (long long)B * p.To * p.Ho * p.Wo * 128;
  if (p.x_bytes > 0x7FFFFFF0LL) return STEM_UNSUPPORTED;
  const size_t lds = (size_t)2 * (p.halo_px + p.dy_rows * 8) * 16 + (pool ? 7 * 64 * 4 : 0);
  if (lds > 160 * 1024) return STEM_UNSUPPORTED;
  int grid = 256;
  if (grid > p.nitems) grid = p.nitems;
  if ((long long)grid * 64 * 672 > slab_floats) return STEM_UNSUPPORTED;
  // MILNCE_STEM_WGRAD_V (read once): 2 = 8 waves over K eighths (default), 0 = 4 waves
  static int variant = -1;
  if (variant < 0) {
    const char* e = getenv("MILNCE_STEM_WGRAD_V");
    variant = e ? atoi(e) : 2;
  }
  int rc;
  if (pool) rc = x_u8 ? stem_wgrad_launch<true, 8, true>(p, grid, lds, stream)
                      : stem_wgrad_launch<false, 8, true>(p, grid, lds, stream);
  else if (variant == 0) rc = x_u8 ? stem_wgrad_launch<true, 4, false>(p, grid, lds, stream)
                                   : stem_wgrad_launch<false, 4, false>(p, grid, lds, stream);
  else rc = x_u8 ? stem_wgrad_launch<true, 8, false>(p, grid, lds, stream)
                 : stem_wgrad_launch<false, 8, false>(p, grid, lds, stream);
  if (rc) return rc;
  return launch_wgrad_reduce(p.slab, dw, grid, 64, 672, 64, 8, 8, 84, accumulate, stream);
}

MILNCE_API int milnce_stem_wgrad(const void* dy, const void* x2, int x_u8, float* slab, long long slab_floats,
                                 float* dw, int B, int T, int H, int W2, int accumulate, hipStream_t stream) {
  StemWgradParams p = {};
  p.dy = (const bf16_t*)dy; p.x = (const bf16_t*)x2; p.slab = slab;
  p.B = B; p.T = T; p.H = H; p.W2 = W2;
  return stem_wgrad_impl(p, x_u8, slab_floats, dw, accumulate, stream);
}

// Stem wgrad straight from the maxpool_2a backward: pdy / parg = the pooled gradient and arg-max
// [B, To, Ho/2, Wo/2, 64], y = the raw stem output [M, 64], ss / coef = the stem BN's
// [mean, invstd, scale, shift] and finalised backward coefficients [k0, k1, k2] (milnce_bn_bwd_finalize).
// Same dW as milnce_maxpool_bwd_apply into dy followed by milnce_stem_wgrad, without the dy tensor.
MILNCE_API int milnce_stem_wgrad_pool(const void* pdy, const void* parg, const void* y, const float* ss,
                                      const float* coef, const void* x2, int x_u8, float* slab,
                                      long long slab_floats, float* dw, int B, int T, int H, int W2, int accumulate,
                                      hipStream_t stream) {
  StemWgradParams p = {};
  p.x = (const bf16_t*)x2; p.slab = slab;
  p.B = B; p.T = T; p.H = H; p.W2 = W2;
  p.pdy = (const bf16_t*)pdy; p.parg = (const uint8_t*)parg; p.ybn = (const bf16_t*)y;
  p.ss = ss; p.coef = coef;
  if (!pdy || !parg || !y || !ss || !coef) return (int)hipErrorInvalidValue;
  return stem_wgrad_impl(p, x_u8, slab_floats, dw, accumulate, stream);
}

// Stem forward (see stem_fwd_kernel): y [M, 64] bf16 and BN partials stats[nparts][2][64];
// x2 as for milnce_stem_wgrad (bf16, or uint8 scaled by 1/255 while staged);
// returns the number of partial rows written (> 0), STEM_UNSUPPORTED (-1) for geometries it does
// not cover (the caller falls back to the generic implicit GEMM), or -1000 - hipError on a launch error.
MILNCE_API int milnce_stem_fwd(const void* x2, int x_u8, const void* wpacked, int Kpad, void* y, float* stats,
                               long long stats_floats, const float* shift, int B, int T, int H, int W2,
                               hipStream_t stream) {
  StemFwdParams p;
  p.x = (const bf16_t*)x2; p.w = (const bf16_t*)wpacked; p.y = (bf16_t*)y; p.stats = stats; p.shift = shift;
  p.B = B; p.T = T; p.H = H; p.Kpad = Kpad;
  p.To = (T + 2 - 3) / 2 + 1;
  p.Ho = (H + 6 - 7) / 2 + 1;
  const int hr = stem_fwd_hr();
  if (p.Ho % hr || Kpad < 672) return -1;
  p.nitems = B * p.To * (p.Ho / hr);
  p.x_bytes = (long long)B * T * H * W2 * (x_u8 ? 8 : 16);
  if (p.x_bytes > 0x7FFFFFF0LL) return -1;
  int grid = 256;
  if (grid > p.nitems) grid = p.nitems;
  if ((long long)grid * 128 > stats_floats) return -1;
  int rc;
  if (W2 == 100) rc = x_u8 ? launch_stem_fwd<100, true>(p, grid, stream) : launch_stem_fwd<100, false>(p, grid, stream);
  else if (W2 == 112) rc = x_u8 ? launch_stem_fwd<112, true>(p, grid, stream) : launch_stem_fwd<112, false>(p, grid, stream);
  else if (W2 == 32) rc = x_u8 ? launch_stem_fwd<32, true>(p, grid, stream) : launch_stem_fwd<32, false>(p, grid, stream);
  else return -1;
  return rc ? -rc - 1000 : grid;
}
