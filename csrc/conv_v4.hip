// v4 implicit-GEMM forward / dgrad for S3D-G's stride-1 convs on gfx950: the v3 LDS-DMA ring
// (conv.hip conv_fwd_v3_kernel) with the per-stage address work moved to the scalar unit.
//
//   Y[m, n] = sum_k X[m + off(tap), c] * W[n, (tap, c)],  k = (tap, c), c fastest
//
// Requirement (host-checked, fwd_v4_supported): Cin % 64 == 0 and K = taps * Cin unpadded, so
// every 64-wide K stage lies inside ONE tap. The stage's tap and channel block are then
// wave-uniform (scalar registers): the weight stage offset becomes the buffer loads' SGPR
// soffset, the tap's input offset one scalar operand, and each A row keeps a per-tile bitmask of
// the taps that land inside the clip (conv padding): the per-stage vector work is one mask test,
// one add and one select per A row, instead
// of v3's three FastDiv decodes, six bound compares per row and per-row adds (~4 VALU per MFMA
// in v3's main loop, profiles/r2_session3.md). Out-of-clip rows get an offset past the buffer's
// num_records, which the LDS-DMA reads as zero.
//
// MF = 16: mfma_f32_16x16x32_bf16 fragments (as v3); MF = 32: mfma_f32_32x32x16_bf16 with the
// same 64 x BN/2 wave tile: half the MFMA instructions (each 32 cycles), so 24 of every 32
// issue cycles stay free for the partner wave's VALU / LDS-DMA issue instead of 8 of 16.
// Accumulator layout (32x32x16, A = weights rows n, B = activations cols m): lane l holds
// column m = l & 31 and rows n = 8 * (r >> 2) + 4 * (l >> 5) + (r & 3), r = 0..15 -- four runs
// of 4 consecutive channels, written to the epilogue tile as 8-byte rows.
#include "conv_common.h"

template <int MF> struct AccT { typedef f32x4 type; };
template <> struct AccT<32> { typedef f32x16 type; };

static constexpr int V4_BK = 64;

// Diagnostic ablations (separate debug libraries only, tools/gpu/v4_ablate.sh; results are
// garbage): bit 0 skips the activation LDS-DMA, bit 1 the weight LDS-DMA, bit 2 the epilogue's
// global stores and statistics. Timing them bounds what the ring traffic / epilogue cost.
#ifndef V4_ABLATE
#define V4_ABLATE 0
#endif
static constexpr int V4_BM = 128;

// per-row tap validity: bit t of the mask is set when tap t = (dt*KH + dh)*KW + dw of output row
// (rt, rh, rw) (input origin) reads inside the clip. KS: compile-time kernel shape 111 / 133 / 311,
// or 0 for runtime extents.
template <int KS>
__device__ __forceinline__ uint32_t tap_mask(int rt, int rh, int rw, const ConvParams& p) {
  const int KT = KS == 111 ? 1 : KS == 133 ? 1 : KS == 311 ? 3 : p.KT;
  const int KH = KS == 111 ? 1 : KS == 133 ? 3 : KS == 311 ? 1 : p.KH;
  const int KW = KS == 111 ? 1 : KS == 133 ? 3 : KS == 311 ? 1 : p.KW;
  uint32_t mw = 0;
#pragma unroll
  for (int dw = 0; dw < (KS ? (KS % 10) : 8); ++dw)
    if (KS || dw < KW) mw |= (uint32_t)((unsigned)(rw + dw) < (unsigned)p.W) << dw;
  uint32_t m = 0;
#pragma unroll
  for (int dt = 0; dt < (KS ? (KS / 100) : 4); ++dt) {
    if (!KS && dt >= KT) break;
    const bool tv = (unsigned)(rt + dt) < (unsigned)p.T;
#pragma unroll
    for (int dh = 0; dh < (KS ? ((KS / 10) % 10) : 8); ++dh) {
      if (!KS && dh >= KH) break;
      const bool v = tv & ((unsigned)(rh + dh) < (unsigned)p.H);
      m |= v ? mw << ((dt * KH + dh) * KW) : 0u;
    }
  }
  return m;
}

// NWM waves along M (each wave a 64 x BN/2 tile, 2 along N): BM = 64 NWM rows, 128 NWM threads.
// NWM = 4 (256-row tiles, 8 waves) halves the weight-tile re-reads per output row: at N = 192 the
// weight stream (re-read per M tile) is the larger part of the ring's L2 traffic.
template <int BN, int STAGES, int EPI, int MF, int KS, int NWM>
__global__ __launch_bounds__(128 * NWM, 1) void conv_fwd_v4_kernel(ConvParams p) {
  constexpr int BK = V4_BK, BM = 64 * NWM;
  constexpr int NT = 128 * NWM, NWAVES = 2 * NWM;
  constexpr int CPR = BK / 8;                 // 16-B chunks per tile row
  constexpr int RPI = 64 / CPR;               // rows per DMA instruction (1 KiB)
  constexpr int A_INST = BM / RPI / NWAVES;   // 4
  constexpr int B_INST = BN / RPI / NWAVES;
  constexpr int NDMA = A_INST + B_INST;
  constexpr int WM = 64, WN = BN / 2;        // wave tile 64 x BN/2 (NWM x 2 waves)
  constexpr int TM = WM / MF, TN = WN / MF;
  constexpr int KSTEPS = BK / (MF == 16 ? 32 : 16);
  constexpr int LDE = BN + 8;
  constexpr int STAGE_ELEMS = (BM + BN) * BK;
  static_assert(B_INST * RPI * NWAVES == BN && A_INST * RPI * NWAVES == BM, "DMA mapping");
  static_assert(WN % MF == 0, "wave tile must be a multiple of the MFMA tile");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* ring = (bf16_t*)smem;  // stage s: A [BM][BK] then B [BN][BK]
  bf16_t* Es = (bf16_t*)smem;    // epilogue staging [BM][LDE] (after the ring drained)
  float* ssl = (float*)(smem + BM * LDE * 2);  // [4][BN] producer-BN constants (EPI 2)
  // EPI 1 shift of the block's (fixed) N tile behind the whole layout (launch_v4_t): written once,
  // read from LDS by every tile's epilogue (per-tile global loads there cost vmcnt drains)
  constexpr int V4_RING = STAGES * STAGE_ELEMS * 2, V4_EPI = BM * LDE * 2 + (EPI == 2 ? 16 * BN : 0);
  constexpr int V4_RED = 16 * 128 * NWM * 4;
  constexpr int SHL_OFF = V4_RING > V4_EPI ? (V4_RING > V4_RED ? V4_RING : V4_RED) : (V4_EPI > V4_RED ? V4_EPI : V4_RED);
  float* shl = (float*)(smem + SHL_OFF);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;  // wr in [0, NWM)
  const int nblocks = p.num_n_tiles * p.grid_m;
  const int logical = xcd_remap(blockIdx.x, nblocks);
  const int n_tile = logical % p.num_n_tiles;
  const int m_slot = logical / p.num_n_tiles;
  const int n0 = n_tile * BN;
  const int nk = p.Kpad / BK;
  const int cps = p.Cin / BK;  // K stages per tap
  KASSERT(nk * BK == p.Kpad && p.Kpad == p.KT * p.KH * p.KW * p.Cin && cps * BK == p.Cin);
  const uint32_t thw = (uint32_t)p.To * p.Ho * p.Wo;
  const uint32_t clip_bytes = (uint32_t)(p.x_bstride * 2);

  const int slot = lane % CPR;
  const int lrow = wave * RPI + lane / CPR;
  const int src_chunk = swz<BK>(lrow, slot);

  const auto wrs = __builtin_amdgcn_make_buffer_rsrc((void*)p.w, (short)0,
                                                     (int)((long long)p.num_n_tiles * BN * p.Kpad * 2), 0x00020000);
  // weight rows: fixed voffset per DMA instruction, the stage's K offset goes in soffset
  // fixed array bounds: bounds that are template constants make clang's host pass drop the
  // kernel's launch stub when the arrays are captured by the lambdas below (as in conv.hip v3)
  static_assert(A_INST <= 4 && B_INST <= 8, "offset arrays");
  uint32_t ob[8];
#pragma unroll
  for (int i = 0; i < B_INST; ++i)
    ob[i] = (uint32_t)(((long long)(n0 + i * NWAVES * RPI + lrow) * p.Kpad + src_chunk * 8) * 2);
  // byte distance between consecutive taps' input offsets, per tap coordinate
  const int tstride_w = p.Cin * 2, tstride_h = p.W * p.Cin * 2, tstride_t = p.H * p.W * p.Cin * 2;

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

    uint32_t rowoff[4], tmask[4];
#pragma unroll
    for (int i = 0; i < A_INST; ++i) {
      const int m = m0 + i * NWAVES * RPI + lrow;
      if (m < p.M) {
        const uint32_t q = fdiv((uint32_t)m, p.fWo);
        const int wo = m - q * p.Wo;
        const uint32_t q2 = fdiv(q, p.fHo);
        const int ho = q - q2 * p.Ho;
        const uint32_t b = fdiv(q2, p.fTo);
        const int to = q2 - b * p.To;
        const int rt = to * p.st - p.pt, rh = ho * p.sh - p.ph, rw = wo * p.sw - p.pw;
        rowoff[i] = (b - b0) * clip_bytes + (uint32_t)(((rt * p.H + rh) * p.W + rw) * p.Cin * 2 + src_chunk * 16);
        tmask[i] = tap_mask<KS>(rt, rh, rw, p);
      } else {
        rowoff[i] = 0;
        tmask[i] = 0;
      }
    }

    using acc_t = typename AccT<MF>::type;
    acc_t acc[TN][TM];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int i = 0; i < TM; ++i) acc[j][i] = acc_t{};

    ring_barrier();  // previous tile's epilogue done with the LDS

    // issue state of the next stage to fire (wave-uniform, SALU): tap coordinates, channel block.
    // The A offset of a row is rowoff + koff(tap, block) in the VGPR offset (not the SGPR soffset:
    // rowoff alone is negative for rows at the top / left padding, and the buffer range check
    // sees the VGPR offset), or past num_records when the tap falls outside the clip.
    int is_cb = 0, is_dt = 0, is_dh = 0, is_dw = 0, is_tap = 0;
    uint32_t oa[4];
    auto offsets = [&]() {
      const uint32_t bit = 1u << is_tap;
      const uint32_t koff = (uint32_t)__builtin_amdgcn_readfirstlane(
          is_dt * tstride_t + is_dh * tstride_h + is_dw * tstride_w + is_cb * BK * 2);
#pragma unroll
      for (int i = 0; i < A_INST; ++i) oa[i] = (tmask[i] & bit) ? rowoff[i] + koff : 0x80000000u;
    };
    auto fire = [&](int kt) {
      bf16_t* sa = ring + (kt % STAGES) * STAGE_ELEMS;
      bf16_t* sb = sa + BM * BK;
      const int woff = __builtin_amdgcn_readfirstlane(kt * BK * 2);
#pragma unroll
      for (int i = 0; i < A_INST; ++i)
        if (!(V4_ABLATE & 1))
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_ptr_t)(sa + (i * NWAVES * RPI + wave * RPI) * BK), 16,
                                                   oa[i], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < B_INST; ++i)
        if (!(V4_ABLATE & 2))
          __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, (lds_ptr_t)(sb + (i * NWAVES * RPI + wave * RPI) * BK), 16,
                                                   ob[i], woff, 0, 0);
      // advance the issue state by one 64-wide K stage
      if (++is_cb == cps) {
        is_cb = 0;
        ++is_tap;
        if (++is_dw == p.KW) {
          is_dw = 0;
          if (++is_dh == p.KH) { is_dh = 0; ++is_dt; }
        }
      }
    };

#pragma unroll
    for (int s = 0; s < STAGES - 1; ++s) {
      if (s < nk) {
        offsets();
        fire(s);
      }
    }

    for (int kt = 0; kt < nk; ++kt) {
      const bool more = kt + STAGES - 1 < nk;
      if (more) offsets();
      const int ahead = min(nk - 1, kt + STAGES - 2) - kt;
      wait_stages<NDMA, STAGES - 2>(ahead);
      ring_barrier();
      if (more) fire(kt + STAGES - 1);
      const bf16_t* a = ring + (kt % STAGES) * STAGE_ELEMS;
      const bf16_t* bsh = a + BM * BK;
      if constexpr (MF == 16) {
        auto xfrag = [&](int s, int i) {
          const int row = wr * WM + i * 16 + (lane & 15);
          return *(const bf16x8*)(a + row * BK + swz<BK>(row, s * 4 + (lane >> 4)) * 8);
        };
        auto wfrag = [&](int s, int j) {
          const int row = wc * WN + j * 16 + (lane & 15);
          return *(const bf16x8*)(bsh + row * BK + swz<BK>(row, s * 4 + (lane >> 4)) * 8);
        };
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
          __builtin_amdgcn_s_setprio(1);
#pragma unroll
          for (int j = 0; j < TN; ++j) {
#pragma unroll
            for (int i = 0; i < TM; ++i)
              acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], xf[i], acc[j][i], 0, 0, 0);
            if (s + 1 < KSTEPS) wf[j] = wfrag(s + 1, j);
          }
          __builtin_amdgcn_s_setprio(0);
#pragma unroll
          for (int i = 0; i < TM; ++i) xf[i] = xn[i];
        }
      } else {
        // 32x32x16: lane l reads row (l & 31) of its 32-row fragment, 8 k at chunk 2s + (l >> 5)
        auto xfrag = [&](int s, int i) {
          const int row = wr * WM + i * 32 + (lane & 31);
          return *(const bf16x8*)(a + row * BK + swz<BK>(row, s * 2 + (lane >> 5)) * 8);
        };
        auto wfrag = [&](int s, int j) {
          const int row = wc * WN + j * 32 + (lane & 31);
          return *(const bf16x8*)(bsh + row * BK + swz<BK>(row, s * 2 + (lane >> 5)) * 8);
        };
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
          __builtin_amdgcn_s_setprio(1);
#pragma unroll
          for (int j = 0; j < TN; ++j) {
#pragma unroll
            for (int i = 0; i < TM; ++i)
              acc[j][i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[j], xf[i], acc[j][i], 0, 0, 0);
            if (s + 1 < KSTEPS) wf[j] = wfrag(s + 1, j);
          }
          __builtin_amdgcn_s_setprio(0);
#pragma unroll
          for (int i = 0; i < TM; ++i) xf[i] = xn[i];
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    ring_barrier();  // every wave done reading the ring before the epilogue reuses it

    // EPI 1: per-channel shift (bn_ss, when set: the BN's running mean) subtracted before the bf16
    // rounding, so the stored pre-BN values keep their precision when |mean| >> std
    auto shift4 = [&](int col, float (&sh)[4]) {
      const float4 v = EPI == 1 ? *(const float4*)(shl + col) : make_float4(0.f, 0.f, 0.f, 0.f);
      sh[0] = v.x;
      sh[1] = v.y;
      sh[2] = v.z;
      sh[3] = v.w;
    };
    if constexpr (MF == 16) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = wc * WN + j * 16 + (lane >> 4) * 4;
        float sh[4];
        shift4(col, sh);
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int row = wr * WM + i * 16 + (lane & 15);
          const f32x4 v = acc[j][i];
          uint2 o;
          o.x = pack2bf(v[0] - sh[0], v[1] - sh[1]);
          o.y = pack2bf(v[2] - sh[2], v[3] - sh[3]);
          *(uint2*)(Es + row * LDE + col) = o;
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int col = wc * WN + j * 32 + g * 8 + (lane >> 5) * 4;
          float sh[4];
          shift4(col, sh);
#pragma unroll
          for (int i = 0; i < TM; ++i) {
            const int row = wr * WM + i * 32 + (lane & 31);
            uint2 o;
            o.x = pack2bf(acc[j][i][4 * g + 0] - sh[0], acc[j][i][4 * g + 1] - sh[1]);
            o.y = pack2bf(acc[j][i][4 * g + 2] - sh[2], acc[j][i][4 * g + 3] - sh[3]);
            *(uint2*)(Es + row * LDE + col) = o;
          }
        }
      }
    }
    if constexpr (EPI == 2) {
      for (int t = tid; t < 4 * BN; t += NT) {
        const int qq = t / BN, c = n0 + (t - qq * BN);
        ssl[t] = c < p.Cout ? p.bn_ss[qq * p.Cout + c] : 0.f;
      }
    }
    ring_barrier();
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
        const bool ok = (m < p.M) & (n < p.Cout) & !(V4_ABLATE & 4);
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
        const bool ok = (m < p.M) & (n < p.Cout) & !(V4_ABLATE & 4);
        KASSERT(!ok || n + 8 <= p.ldy);
        if (ok) *(uint4*)(p.y + (long long)m * p.ldy + n) = dv;
        if constexpr (EPI == 1) {
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
      constexpr int ACT = (NT / OCPR) * OCPR;
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

template <int BN, int STAGES, int EPI, int MF, int KS, int NWM>
static int launch_v4_t(ConvParams& p, hipStream_t stream) {
  constexpr int BM = 64 * NWM;
  constexpr size_t ring = (size_t)STAGES * (BM + BN) * V4_BK * 2;
  constexpr size_t epi = (size_t)BM * (BN + 8) * 2 + (EPI == 2 ? 16 * BN : 0);
  constexpr size_t red = (size_t)16 * 128 * NWM * 4;
  constexpr size_t lds = (ring > epi ? (ring > red ? ring : red) : (epi > red ? epi : red)) + (EPI == 1 ? 4 * BN : 0);
  static_assert(lds <= 160 * 1024, "LDS");
  static bool attr_set = false;
  if (!attr_set) {
    HIP_RET(hipFuncSetAttribute((const void*)conv_fwd_v4_kernel<BN, STAGES, EPI, MF, KS, NWM>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr_set = true;
  }
  ConvParams q = p;
  q.num_m_tiles = (p.M + BM - 1) / BM;
  const int nblocks = q.num_n_tiles * q.grid_m;
  hipLaunchKernelGGL((conv_fwd_v4_kernel<BN, STAGES, EPI, MF, KS, NWM>), dim3(nblocks), dim3(128 * NWM), lds, stream,
                     q);
  return (int)hipGetLastError();
}

template <int BN, int STAGES, int MF, int KS, int NWM>
static int launch_v4_epi(ConvParams& p, hipStream_t stream) {
  if (p.bn_mode == 0) return launch_v4_t<BN, STAGES, 0, MF, KS, NWM>(p, stream);
  if (p.bn_mode == 1) return launch_v4_t<BN, STAGES, 1, MF, KS, NWM>(p, stream);
  return launch_v4_t<BN, STAGES, 2, MF, KS, NWM>(p, stream);
}

template <int BN, int STAGES, int MF, int NWM = 2>
static int launch_v4_ks(ConvParams& p, hipStream_t stream) {
  const int ks = p.KT * 100 + p.KH * 10 + p.KW;
  if (ks == 111) return launch_v4_epi<BN, STAGES, MF, 111, NWM>(p, stream);
  if (ks == 133) return launch_v4_epi<BN, STAGES, MF, 133, NWM>(p, stream);
  if (ks == 311) return launch_v4_epi<BN, STAGES, MF, 311, NWM>(p, stream);
  return launch_v4_epi<BN, STAGES, MF, 0, NWM>(p, stream);
}

template <int BN>
static int launch_v4_bn(ConvParams& p, int impl, hipStream_t stream) {
  constexpr bool mf32 = (BN / 2) % 32 == 0;
  constexpr bool three = 3 * (V4_BM + BN) * V4_BK * 2 <= 160 * 1024;
  constexpr bool wide_m = BN % 64 == 0;  // 8 waves: B rows split into 1-KiB pieces of 8 waves
  if (impl == 8) return launch_v4_ks<BN, 2, 16>(p, stream);
  if constexpr (mf32) {
    if (impl == 9) return launch_v4_ks<BN, 2, 32>(p, stream);
  }
  if constexpr (three) {
    if (impl == 10) return launch_v4_ks<BN, 3, 16>(p, stream);
    if constexpr (mf32) {
      if (impl == 11) return launch_v4_ks<BN, 3, 32>(p, stream);
    }
  }
  if constexpr (wide_m) {
    if (impl == 12) return launch_v4_ks<BN, 2, 16, 4>(p, stream);
    if (impl == 13) return launch_v4_ks<BN, 2, 32, 4>(p, stream);
  }
  return V4_UNSUPPORTED;
}

bool fwd_v4_supported(const ConvParams& p, int bn, int impl) {
  const int taps = p.KT * p.KH * p.KW;
  if (impl < 8 || impl > 13) return false;
  if (p.Cin % V4_BK || p.Kpad != taps * p.Cin || taps > 32) return false;
  if (p.KT > 4 || p.KH > 8 || p.KW > 8) return false;  // tap_mask<0> loop bounds
  if (bn != 64 && bn != 96 && bn != 128 && bn != 160 && bn != 192) return false;
  if ((impl == 9 || impl == 11) && (bn / 2) % 32) return false;
  if ((impl == 10 || impl == 11) && 3 * (V4_BM + bn) * V4_BK * 2 > 160 * 1024) return false;
  if (impl >= 12 && bn % 64) return false;
  return true;
}

int launch_fwd_v4(ConvParams& p, int bn, int impl, hipStream_t stream) {
  if (!fwd_v4_supported(p, bn, impl)) return V4_UNSUPPORTED;
  switch (bn) {
    case 64: return launch_v4_bn<64>(p, impl, stream);
    case 96: return launch_v4_bn<96>(p, impl, stream);
    case 128: return launch_v4_bn<128>(p, impl, stream);
    case 160: return launch_v4_bn<160>(p, impl, stream);
    case 192: return launch_v4_bn<192>(p, impl, stream);
  }
  return V4_UNSUPPORTED;
}
