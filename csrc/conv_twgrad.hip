// Box-tiled weight gradient of the temporal (3,1,1) convs of S3D-G (stride 1, padding (1,0,0)),
// with wide output-channel tiles and a counted LDS-DMA ring (gfx950).
//
//   dW[n, dt, c] = sum_{b,t,s} dY[b, t, s, n] * X[b, t + dt - 1, s, c]       (s = h * W + w)
//
// The im2col wgrad (csrc/conv.hip) stages every input row once per tap; the halo wgrad
// (conv_halo.hip) stages it once per box but with 64-wide output tiles (every input row again
// per 64 output channels) and a 2-stage ring that waits for each box with vmcnt(0). Here:
//
//   * a box is bt frames x bs consecutive flattened spatial positions of one clip (bt * bs = 64
//     positions, bs a multiple of 8); its input halo is the (bt + 2) x bs rows of the frames
//     t0 - 1 .. t0 + bt, and tap dt reads the halo at a constant shift of dt * bs rows (a
//     multiple of 8 rows, so the 16-B chunk swizzle of the halo image is shift-invariant);
//   * a workgroup owns BN = 64 / 128 / 192 output channels x 64 input channels x 3 taps: the
//     [BN][192] fp32 tile lives in registers (8 waves: 2 along n x 4 channel blocks of 16, all
//     three taps per wave, so each B fragment's tap shift is an immediate offset);
//   * dY [64][BN] (as BN/64 sub-images of 128-B rows) and the halo [128][64] of a box arrive by
//     LDS-DMA into a 3-stage ring; every wave issues the same number of DMA instructions per box
//     (rows past the halo / box read as zero), so the wait for box i is one compile-time vmcnt
//     that leaves boxes i+1, i+2 in flight -- no vmcnt(0) drain per box;
//   * MFMA 16x16x32 bf16: A = dY^T (rows n), B = X shifted (cols c), both read from the
//     position-major images with ds_read_b64_tr_b16 (as conv_halo.hip);
//   * persistent workgroups over a contiguous range of boxes (a split); split-major block order
//     (xcd_remap) keeps all tiles of a split on one XCD, so a box's dY / X rows come from HBM once
//     and from that XCD's L2 for the other tiles; fp32 partial tiles go to a slab that
//     wgrad_reduce_kernel sums in a fixed order (deterministic, no atomics).
//
// Reference semantics: the weight gradient of nn.Conv3d(k=(3,1,1), p=(1,0,0), bias=False)
// (/root/reference/s3dg.py:95-98).
#include "common.h"

constexpr int TW_NT = 512, TW_NW = 8;
constexpr int TW_P = 64;       // positions per box (two 32-position k-steps)
constexpr int TW_CC = 64;      // input channels per tile
constexpr int TW_XROWS = 128;  // halo rows per stage (>= (bt + 2) * bs)
constexpr int TW_NSTG = 3;

template <int BN>
struct TwGeom {
  static constexpr int NSUB = BN / 64;                   // dY sub-images of 64 channels
  static constexpr int SUB_BYTES = TW_P * 128;           // [64 positions][64 ch] bf16
  static constexpr int D_BYTES = NSUB * SUB_BYTES;
  static constexpr int X_BYTES = TW_XROWS * 128;
  static constexpr int STAGE_BYTES = D_BYTES + X_BYTES;
  static constexpr int D_INST = NSUB * (TW_P / 8) / TW_NW;  // 1-KiB DMA instructions per wave
  static constexpr int X_INST = (TW_XROWS / 8) / TW_NW;
  static constexpr int PER_BOX = D_INST + X_INST;
  static constexpr int LDS = TW_NSTG * STAGE_BYTES;
  static_assert(D_INST * TW_NW * 8 == NSUB * TW_P && X_INST * TW_NW * 8 == TW_XROWS, "DMA mapping");
};

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(3))) char lds_char;

// 128-B rows: 16-B chunk c of row r stored at chunk c ^ 2 * ((r >> 1) & 3) (conv_halo.hip Swz<8>)
__device__ __forceinline__ int tw_chunk(int row, int c) { return c ^ (2 * ((row >> 1) & 3)); }
__device__ __forceinline__ uint32_t tw_x(int row) { return (uint32_t)((row >> 1) & 3) << 5; }

__device__ __forceinline__ bf16x8 tw_join(s16x4 lo, s16x4 hi) {
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}
__device__ __forceinline__ s16x4 tw_tr(const lds_char* a) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)a);
}

template <int N>
__device__ __forceinline__ void tw_wait() {
  static_assert(N >= 0 && N <= 63, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

struct TwParams {
  const bf16_t* dy;  // [B, T, HW, ldd]
  const bf16_t* x;   // [B, T, HW, Cin]
  float* slab;       // [splits][Npad][3 * Cin]
  int B, T, HW, Cin, Cout, ldd;
  int bt, bs, lbs;   // box: bt frames x bs positions (bs = 1 << lbs)
  int ntb, nbs, nboxes;
  int n_slices, c_chunks, splits;
  int Npad, Kdim;
  FastDiv fnbs, fntb;
  // REG only, optional: x is the raw conv output of a BN layer and the operand is
  // z = relu(x * scale + shift) (xss = that BN's [mean, invstd, scale, shift][Cin]), applied to the
  // staged halo chunks as the forward's box prologue does (same roundings; padding rows stay zero),
  // so the forward need not write z for this wgrad
  const float* xss;
};

// MODE 0: LDS-DMA ring of TW_NSTG stages (two boxes in flight). MODE 1 (REG): register-staged
// boxes (NSUB + 2 16-B chunks per thread and box) in a 3-box register ring written into 2 LDS
// slots: three boxes (~100 KiB per CU) in flight instead of two, for ~1.5x the latency cover at
// the same LDS footprint of the DMA ring's two stages. MODE 2: the register ring with 3 LDS slots,
// software-pipelined across boxes: the next box's first k-step fragments are read from LDS under
// the current box's second k-step MFMAs (its slot was written a step earlier), so a step starts
// its MFMAs right after the barrier instead of waiting for the fragment reads of all 8 waves
// (counter passes, profiles/r6_twgrad_pmc.txt: 18 % of wave time waiting on LDS in MODE 1).
template <int BN, int MODE>
__global__ __launch_bounds__(TW_NT, 1) void twgrad_kernel(TwParams p) {
  constexpr bool REG = MODE >= 1;
  using G = TwGeom<BN>;
  constexpr int NBLK = BN / 16, CBLK = TW_CC / 16;  // 16-row n blocks, 16-channel c blocks
  constexpr int WK = CBLK, WN = TW_NW / WK;         // waves: 4 channel blocks x 2 n halves
  constexpr int NBW = NBLK / WN;                    // n blocks per wave
  constexpr int KBW = 3;                            // one channel block x 3 taps per wave
  static_assert(NBLK % WN == 0, "wave tiling");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  lds_char* lds = (lds_char*)smem;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wave % WN, wk = wave / WN;
  const int ntiles = p.n_slices * p.c_chunks;
  const int nblocks = ntiles * p.splits;
  const int logical = xcd_remap(blockIdx.x, nblocks);
  const int split = logical / ntiles;
  const int tile = logical - split * ntiles;
  const int n0 = (tile % p.n_slices) * BN;
  const int c0 = (tile / p.n_slices) * TW_CC;
  const int box_begin = (int)((long long)split * p.nboxes / p.splits);
  const int box_end = (int)((long long)(split + 1) * p.nboxes / p.splits);

  // DMA lane mapping: 8 lanes per 128-B row, lane-linear slot -> swizzled source chunk
  const int slot = lane & 7, lrow = lane >> 3;
  const long long clip_x = (long long)p.T * p.HW * p.Cin, clip_d = (long long)p.T * p.HW * p.ldd;
  const uint32_t xlim = (uint32_t)min(clip_x * 2, 0x7FFFFFF0LL), dlim = (uint32_t)min(clip_d * 2, 0x7FFFFFF0LL);

  // Stage of box `box` into ring slot `stage`; box >= box_end issues the same instructions with
  // every offset out of range (zero fills), so every wave's vmcnt per box is PER_BOX.
  auto issue = [&](int box, int stage) {
    lds_char* sd = lds + stage * G::STAGE_BYTES;
    lds_char* sx = sd + G::D_BYTES;
    const bool live = box < box_end;
    const int bx = live ? box : box_begin;
    const uint32_t q = fdiv((uint32_t)bx, p.fnbs);
    const int sb = bx - (int)q * p.nbs;
    const uint32_t b = fdiv(q, p.fntb);
    const int tb = (int)(q - b * p.ntb);
    const int t0 = tb * p.bt, s0 = sb << p.lbs;
    const auto drs = __builtin_amdgcn_make_buffer_rsrc((void*)(p.dy + (long long)b * clip_d), (short)0,
                                                       (int)(live ? dlim : 0u), 0x00020000);
    const auto xrs = __builtin_amdgcn_make_buffer_rsrc((void*)(p.x + (long long)b * clip_x), (short)0,
                                                       (int)(live ? xlim : 0u), 0x00020000);
#pragma unroll
    for (int i = 0; i < G::D_INST; ++i) {
      const int g = i * TW_NW + wave;          // 8-row group over the NSUB sub-images
      const int sub = g / (TW_P / 8), r0 = (g % (TW_P / 8)) * 8;
      const int r = r0 + lrow;                  // box position
      const int t = t0 + (r >> p.lbs), s = s0 + (r & ((1 << p.lbs) - 1));
      const int n = n0 + sub * 64 + tw_chunk(r, slot) * 8;
      const bool v = (t < p.T) & (s < p.HW) & (n < p.Cout);
      const uint32_t off = v ? (uint32_t)((((long long)t * p.HW + s) * p.ldd + n) * 2) : 0x80000000u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(drs, (lds_ptr_t)(sd + sub * G::SUB_BYTES + r0 * 128), 16, off, 0, 0,
                                               0);
    }
#pragma unroll
    for (int i = 0; i < G::X_INST; ++i) {
      const int r0 = (i * TW_NW + wave) * 8;
      const int r = r0 + lrow;                  // halo row: frame t0 - 1 + (r >> lbs)
      const int t = t0 - 1 + (r >> p.lbs), s = s0 + (r & ((1 << p.lbs) - 1));
      const int c = c0 + tw_chunk(r, slot) * 8;
      const bool v = (r < (p.bt + 2) << p.lbs) & ((unsigned)t < (unsigned)p.T) & (s < p.HW) & (c < p.Cin);
      const uint32_t off = v ? (uint32_t)((((long long)t * p.HW + s) * p.Cin + c) * 2) : 0x80000000u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (lds_ptr_t)(sx + r0 * 128), 16, off, 0, 0, 0);
    }
  };

  f32x4 acc[NBW][KBW];
#pragma unroll
  for (int i = 0; i < NBW; ++i)
#pragma unroll
    for (int j = 0; j < KBW; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // fragment lane constants (conv_halo.hip): positions lp and lp + 16 of a k-step, 4-channel
  // piece pp of the 16-row block
  const int g4 = lane >> 4, li = lane & 15, qq = li >> 2, pp = li & 3;
  const int lp = 4 * g4 + qq;
  uint32_t lane_a[NBW];
#pragma unroll
  for (int i = 0; i < NBW; ++i) {
    const int nb = wn * NBW + i;  // n block within the tile: sub-image nb / 4, chunk pair nb % 4
    lane_a[i] = (uint32_t)((nb >> 2) * G::SUB_BYTES + lp * 128) +
                (((uint32_t)(((nb & 3) * 2 + (pp >> 1)) << 4) | ((pp & 1) << 3)) ^ tw_x(lp));
  }
  const uint32_t lane_b = ((uint32_t)((wk * 2 + (pp >> 1)) << 4) | ((pp & 1) << 3));
  const uint32_t xa0 = ((uint32_t)(lp * 128) ^ tw_x(lp)) ^ lane_b;         // halo row lp
  const uint32_t xb0 = ((uint32_t)((lp + 16) * 128) ^ tw_x(lp + 16)) ^ lane_b;
  const uint32_t tap_step = (uint32_t)(128 << p.lbs);  // dt * bs rows (swizzle-invariant)

  auto load = [&](const lds_char* dimg, const lds_char* ximg, int ks, bf16x8 (&af)[NBW], bf16x8 (&bfr)[KBW]) {
    const lds_char* dks = dimg + ks * 32 * 128;
#pragma unroll
    for (int i = 0; i < NBW; ++i) af[i] = tw_join(tw_tr(dks + lane_a[i]), tw_tr(dks + lane_a[i] + 16 * 128));
    const lds_char* xks = ximg + ks * 32 * 128;
#pragma unroll
    for (int dt = 0; dt < KBW; ++dt)
      bfr[dt] = tw_join(tw_tr(xks + xa0 + dt * tap_step), tw_tr(xks + xb0 + dt * tap_step));
  };
  auto mma = [&](const bf16x8 (&af)[NBW], const bf16x8 (&bfr)[KBW]) {
#pragma unroll
    for (int j = 0; j < KBW; ++j)
#pragma unroll
      for (int i = 0; i < NBW; ++i)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
  };

  auto compute = [&](int slot_i) {
    const lds_char* dimg = lds + slot_i * G::STAGE_BYTES;
    const lds_char* ximg = dimg + G::D_BYTES;
    bf16x8 af0[NBW], bf0[KBW], af1[NBW], bf1[KBW];
    load(dimg, ximg, 0, af0, bf0);
    load(dimg, ximg, 1, af1, bf1);
    __builtin_amdgcn_s_setprio(1);
    mma(af0, bf0);
    mma(af1, bf1);
    __builtin_amdgcn_s_setprio(0);
  };
  auto dimg_of = [&](int slot_i) -> const lds_char* { return lds + slot_i * G::STAGE_BYTES; };

  if constexpr (REG) {
    constexpr int NR = G::NSUB + 3;  // NSUB dY chunks, 2 halo chunks, the halo chunks' validity (.x)
    const int rrow = tid >> 3, rch = tid & 7;
    // this thread's 8 input channels (the chunk rch of the tile's channel block): BN-ReLU constants
    float xsc[8], xsh[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int c = min(c0 + rch * 8 + k, p.Cin - 1);
      xsc[k] = p.xss != nullptr ? p.xss[2 * p.Cin + c] : 0.f;
      xsh[k] = p.xss != nullptr ? p.xss[3 * p.Cin + c] : 0.f;
    }
    // box -> this thread's NSUB dY chunks (row rrow of each sub-image) and 2 halo chunks (rows rrow,
    // rrow + 64); every box issues all NR loads (past box_end / the halo: out of range, zeros), so
    // the vmcnt wait before a box's LDS write is the same count on every path
    auto rload = [&](int box, uint4 (&R)[NR]) {
      const bool live = box < box_end;
      const int bx = live ? box : box_begin;
      const uint32_t q = fdiv((uint32_t)bx, p.fnbs);
      const int sb = bx - (int)q * p.nbs;
      const uint32_t b = fdiv(q, p.fntb);
      const int tb = (int)(q - b * p.ntb);
      const int t0 = tb * p.bt, s0 = sb << p.lbs;
      const auto drs = __builtin_amdgcn_make_buffer_rsrc((void*)(p.dy + (long long)b * clip_d), (short)0,
                                                         (int)(live ? dlim : 0u), 0x00020000);
      const auto xrs = __builtin_amdgcn_make_buffer_rsrc((void*)(p.x + (long long)b * clip_x), (short)0,
                                                         (int)(live ? xlim : 0u), 0x00020000);
      {
        const int t = t0 + (rrow >> p.lbs), s = s0 + (rrow & ((1 << p.lbs) - 1));
        const bool vr = (t < p.T) & (s < p.HW);
#pragma unroll
        for (int k = 0; k < G::NSUB; ++k) {
          const int n = n0 + k * 64 + rch * 8;
          const uint32_t off = (vr & (n < p.Cout)) ? (uint32_t)((((long long)t * p.HW + s) * p.ldd + n) * 2)
                                                   : 0x80000000u;
          R[k] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(drs, off, 0, 0));
        }
      }
      uint32_t valid = 0;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int r = rrow + 64 * j;
        const int t = t0 - 1 + (r >> p.lbs), s = s0 + (r & ((1 << p.lbs) - 1));
        const int c = c0 + rch * 8;
        const bool v = (r < (p.bt + 2) << p.lbs) & ((unsigned)t < (unsigned)p.T) & (s < p.HW) & (c < p.Cin);
        const uint32_t off = v ? (uint32_t)((((long long)t * p.HW + s) * p.Cin + c) * 2) : 0x80000000u;
        R[G::NSUB + j] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xrs, off, 0, 0));
        valid |= (uint32_t)v << j;
      }
      R[G::NSUB + 2] = make_uint4(valid, 0u, 0u, 0u);
    };
    auto rstore = [&](const uint4 (&R)[NR], int slot_i) {
      char* sd = smem + slot_i * G::STAGE_BYTES;
      char* sx = sd + G::D_BYTES;
#pragma unroll
      for (int k = 0; k < G::NSUB; ++k)
        *(uint4*)(sd + k * G::SUB_BYTES + rrow * 128 + tw_chunk(rrow, rch) * 16) = R[k];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int r = rrow + 64 * j;
        uint4 xv = R[G::NSUB + j];
        if (p.xss != nullptr) {  // z = relu(x * scale + shift) of the real rows; padding stays zero
          float f[8];
          unpack8(xv, f);
#pragma unroll
          for (int k = 0; k < 8; ++k) f[k] = fmaxf(f[k] * xsc[k] + xsh[k], 0.f);
          xv = ((R[G::NSUB + 2].x >> j) & 1u) ? pack8(f) : make_uint4(0u, 0u, 0u, 0u);
        }
        *(uint4*)(sx + r * 128 + tw_chunk(r, rch) * 16) = xv;
      }
    };
    if constexpr (MODE == 1) {
      uint4 R0[NR], R1[NR], R2[NR];
      rload(box_begin, R0);
      rload(box_begin + 1, R1);
      rload(box_begin + 2, R2);
      rstore(R0, 0);
      rload(box_begin + 3, R0);
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      // box j lives in register set j % 3 and LDS slot (j - box_begin) % 2. Every step issues its NR
      // loads, also past box_end (out of range: no traffic): the compiler's vmcnt before a set's LDS
      // write counts the loads issued after that set on every path into it, and a path that skipped
      // the later steps' loads made it wait for the set loaded one step earlier instead of three
      auto step = [&](int box, uint4 (&Rn)[NR]) {
        const int i = box - box_begin;
        if (box < box_end) {
          compute(i & 1);
          if (box + 1 < box_end) rstore(Rn, (i + 1) & 1);  // slot of box - 1: every wave finished it
        }
        rload(box + 4, Rn);
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      };
      for (int box = box_begin; box < box_end; box += 3) {
        step(box, R1);
        step(box + 1, R2);
        step(box + 2, R0);
      }
    } else {
      // MODE 2: box j in LDS slot (j - box_begin) % 3, stored two steps before its compute, and in
      // register set (j - box_begin) % 2 (loaded two steps before its store): two register sets
      // instead of three, the third set's registers hold the next box's fragments.
      uint4 RA[NR], RB[NR];
      rload(box_begin, RA);
      rload(box_begin + 1, RB);
      rstore(RA, 0);
      rload(box_begin + 2, RA);
      rstore(RB, 1);
      rload(box_begin + 3, RB);
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      bf16x8 af0[NBW], bf0[KBW], af1[NBW], bf1[KBW];
      load(dimg_of(0), dimg_of(0) + G::D_BYTES, 0, af0, bf0);
      // step(box): k-step 1 of box from its slot si, the k-step-0 MFMAs, k-step 0 of box + 1 (its
      // slot was written a step ago) read under the k-step-1 MFMAs, then box + 2 (in Rs) into the
      // slot box - 1 used (every wave finished it before the last barrier) and box + 4 into Rs
      // (issued on every path: uniform vmcnt counts, as in MODE 1)
      auto pstep = [&](int box, int si, uint4(&Rs)[NR]) {
        const int s1 = si == 2 ? 0 : si + 1, s2 = si == 0 ? 2 : si - 1;
        if (box < box_end) {
          load(dimg_of(si), dimg_of(si) + G::D_BYTES, 1, af1, bf1);
          __builtin_amdgcn_s_setprio(1);
          mma(af0, bf0);
          __builtin_amdgcn_s_setprio(0);
          if (box + 1 < box_end) load(dimg_of(s1), dimg_of(s1) + G::D_BYTES, 0, af0, bf0);
          __builtin_amdgcn_s_setprio(1);
          mma(af1, bf1);
          __builtin_amdgcn_s_setprio(0);
          if (box + 2 < box_end) rstore(Rs, s2);
        }
        rload(box + 4, Rs);
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      };
      for (int box = box_begin; box < box_end; box += 6) {
        pstep(box, 0, RA);
        pstep(box + 1, 1, RB);
        pstep(box + 2, 2, RA);
        pstep(box + 3, 0, RB);
        pstep(box + 4, 1, RA);
        pstep(box + 5, 2, RB);
      }
    }
  } else {
  // prologue: boxes 0 .. NSTG-2 in flight
#pragma unroll
  for (int s = 0; s < TW_NSTG - 1; ++s) issue(box_begin + s, s);
  for (int box = box_begin; box < box_end; ++box) {
    const int i = box - box_begin;
    const int stage = i % TW_NSTG;
    tw_wait<(TW_NSTG - 2) * G::PER_BOX>();  // this box landed (this wave's pieces); two behind it in flight
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // every wave's pieces; slot i-1 free
    issue(box + TW_NSTG - 1, (i + TW_NSTG - 1) % TW_NSTG);
    compute(stage);
  }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing (dummy) stages / loads

  // C[n][k]: row n = 4 * (lane >> 4) + r of the n block, col = lane & 15 of the c block
  float* out = p.slab + (long long)split * p.Npad * p.Kdim;
  const int c = c0 + wk * 16 + (lane & 15);
  if (c < p.Cin) {
#pragma unroll
    for (int i = 0; i < NBW; ++i)
#pragma unroll
      for (int dt = 0; dt < KBW; ++dt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = n0 + (wn * NBW + i) * 16 + (lane >> 4) * 4 + r;
          out[(long long)n * p.Kdim + dt * p.Cin + c] = acc[i][dt][r];
        }
  }
}

namespace {

// box shape: bt frames x bs positions, bt * bs = 64, bs a multiple of 8 with (bt + 2) * bs <=
// TW_XROWS: least padded positions (frames past T, positions past HW), then the smaller halo
bool tw_box(int T, int HW, int& bt, int& lbs) {
  double best = 1e30;
  bool ok = false;
  for (int l = 3; l <= 5; ++l) {
    const int bs = 1 << l, b_t = TW_P / bs;
    if ((b_t + 2) * bs > TW_XROWS) continue;
    const long long boxes = (long long)((T + b_t - 1) / b_t) * ((HW + bs - 1) / bs);
    const double cost = (double)boxes * (TW_P + 0.15 * (b_t + 2) * bs);
    if (cost < best) {
      best = cost;
      bt = b_t;
      lbs = l;
      ok = true;
    }
  }
  return ok;
}

template <int BN, int MODE>
int launch_tw(TwParams& p, hipStream_t stream) {
  using G = TwGeom<BN>;
  const int lds = MODE == 1 ? 2 * G::STAGE_BYTES : MODE == 2 ? 3 * G::STAGE_BYTES : G::LDS;
  static bool attr_set = false;
  if (!attr_set) {
    HIP_RET(hipFuncSetAttribute((const void*)twgrad_kernel<BN, MODE>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                lds));
    attr_set = true;
  }
  hipLaunchKernelGGL((twgrad_kernel<BN, MODE>), dim3(p.n_slices * p.c_chunks * p.splits), dim3(TW_NT),
                     lds_floor(twgrad_kernel<BN, MODE>, lds), stream,
                     p);
  return (int)hipGetLastError();
}

}  // namespace

int launch_wgrad_reduce(const float* slab, float* dw, int splits, int Npad, int Kpad, int Cout, int Cin,
                        int Cin_param, int taps, int accumulate, hipStream_t stream);

// Query: slab floats (and the split count) of the temporal box wgrad of this shape with output
// tile bn (64 / 128 / 192) and about blocks_target workgroups; an error if not supported.
MILNCE_API int milnce_twgrad_plan(int B, int T, int H, int W, int Cin, int Cout, int bn, int blocks_target,
                                  long long* slab_floats, int* splits_out) {
  if (!(bn == 64 || bn == 128 || bn == 192) || Cin % 8 || T < 1) return (int)hipErrorInvalidValue;
  int bt = 0, lbs = 0;
  if (!tw_box(T, H * W, bt, lbs)) return (int)hipErrorInvalidValue;
  const long long nboxes = (long long)B * ((T + bt - 1) / bt) * ((H * W + (1 << lbs) - 1) >> lbs);
  const int ntiles = ((Cout + bn - 1) / bn) * ((Cin + TW_CC - 1) / TW_CC);
  long long splits = fill_splits(blocks_target > 0 ? blocks_target : 256, ntiles);
  if (splits > nboxes) splits = nboxes;
  if (splits < 1) splits = 1;
  *splits_out = (int)splits;
  *slab_floats = splits * ((Cout + bn - 1) / bn) * bn * (3LL * Cin);
  return 0;
}

// dW of a (3,1,1) / stride 1 / padding (1,0,0) conv: the split slab is written to `slab`; with dw
// != null it is also reduced (accumulated when accumulate != 0) into dw [Cout][Cin_param][3][1][1].
// reg: 0 the LDS-DMA ring, 1 the register-staged boxes, 2 the same software-pipelined (MODE).
// xss (register-staged kernel only, else null): x is a BN layer's raw conv output and the operand
// its relu(x * scale + shift), xss = [mean, invstd, scale, shift][Cin] (see TwParams::xss)
MILNCE_API int milnce_twgrad(const void* dy, int ldd, const void* x, float* slab, float* dw, int accumulate, int B,
                             int T, int H, int W, int Cin, int Cin_param, int Cout, int bn, int splits, int reg,
                             const float* xss, hipStream_t stream) {
  if (!(bn == 64 || bn == 128 || bn == 192) || (xss != nullptr && !reg) || reg < 0 || reg > 2)
    return (int)hipErrorInvalidValue;
  TwParams p;
  p.dy = (const bf16_t*)dy;
  p.x = (const bf16_t*)x;
  p.xss = xss;
  p.slab = slab;
  p.B = B; p.T = T; p.HW = H * W; p.Cin = Cin; p.Cout = Cout; p.ldd = ldd;
  if (Cin % 8 || ldd % 8 || splits < 1) return (int)hipErrorInvalidValue;
  if (!tw_box(T, p.HW, p.bt, p.lbs)) return (int)hipErrorInvalidValue;
  p.bs = 1 << p.lbs;
  p.ntb = (T + p.bt - 1) / p.bt;
  p.nbs = (p.HW + p.bs - 1) / p.bs;
  const long long nboxes = (long long)B * p.ntb * p.nbs;
  if (nboxes >= (1LL << 31)) return (int)hipErrorInvalidValue;
  p.nboxes = (int)nboxes;
  p.fnbs = make_fastdiv(p.nbs);
  p.fntb = make_fastdiv(p.ntb);
  p.n_slices = (Cout + bn - 1) / bn;
  p.c_chunks = (Cin + TW_CC - 1) / TW_CC;
  p.splits = splits;
  p.Npad = p.n_slices * bn;
  p.Kdim = 3 * Cin;
  // per-clip byte offsets are 32-bit buffer offsets
  if ((long long)T * p.HW * (ldd > Cin ? ldd : Cin) * 2 > 0x7FFFFFF0LL) return (int)hipErrorInvalidValue;
  int rc;
  if (reg == 2) {
    if (bn == 64) rc = launch_tw<64, 2>(p, stream);
    else if (bn == 128) rc = launch_tw<128, 2>(p, stream);
    else rc = launch_tw<192, 2>(p, stream);
  } else if (reg) {
    if (bn == 64) rc = launch_tw<64, 1>(p, stream);
    else if (bn == 128) rc = launch_tw<128, 1>(p, stream);
    else rc = launch_tw<192, 1>(p, stream);
  } else {
    if (bn == 64) rc = launch_tw<64, 0>(p, stream);
    else if (bn == 128) rc = launch_tw<128, 0>(p, stream);
    else rc = launch_tw<192, 0>(p, stream);
  }
  if (rc) return rc;
  if (dw == nullptr) return 0;
  return launch_wgrad_reduce(slab, dw, splits, p.Npad, p.Kdim, Cout, Cin, Cin_param, 3, accumulate, stream);
}
