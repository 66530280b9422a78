// Box-tiled ("halo") weight gradient for the stride-1, same-padded separable convs of S3D-G
// ((1,3,3) spatial and (3,1,1) temporal), gfx950.
//
//   dW[n, tap, c] = sum_m dY[m, n] * X[m + off(tap), c]
//
// The im2col wgrad (csrc/conv.hip conv_wgrad_kernel) re-fetches the same input row once per tap
// and re-reads dY once per K tile: ~55 FLOP per staged byte at its 96x128 tile. Here a work item
// is a BOX of output positions of one clip (e.g. 1 x 5 x 50 at 50^2): its dY rows [P][BN] and
// its input HALO [(BT+KT-1) x (BH+KH-1) x (BW+KW-1)][CC] arrive by LDS-DMA (buffer_load ... lds,
// out-of-range halo positions read as zero, i.e. the conv padding) into a 2-stage ring, and the
// block accumulates the whole [BN] x [taps x CC] gradient tile in registers: every tap reads the
// SAME halo image at a shifted row. ~240 FLOP per staged byte at BN = CC = 64, 9 taps.
//
// MFMA (16x16x32 bf16) over the box positions: A = dY^T (rows n), B = X_shift (cols c); both
// fragments come from position-major LDS images with ds_read_b64_tr_b16, whose per-lane row
// address lets the B operand follow the halo mapping position -> halo row + tap offset (rows need
// not be contiguous). The images are unpadded with a 16-B chunk XOR of 2*(row & 7) (conflict-free
// transposed reads); each lane DMAs the source chunk that belongs in its lane-linear slot.
//
// Blocks are persistent over a contiguous range of boxes (a split) for one (n-slice, c-chunk)
// tile; each writes one fp32 partial [Npad][taps*Cin] to a slab reduced by wgrad_reduce_kernel
// (deterministic, no atomics). Split-major block order keeps the tiles of a split on one XCD so
// its dY rows / halo are fetched into that XCD's L2 once.
#include "common.h"

#include <type_traits>

struct HaloWgParams {
  const bf16_t* dy;  // [B, T, H, W, ldd]
  const bf16_t* x;   // [B, T, H, W, Cin]
  float* slab;       // [splits][Npad][Kdim]
  int B, T, H, W, Cin, Cout, ldd;
  int pt, ph, pw;
  int BT, BH, BW;    // output box
  int HH, HWd;       // halo rows per t-plane / halo row length (HT implicit)
  int P, HP;         // positions per box, halo positions per box
  int nbt, nbh, nbw, nboxes;
  int n_slices, c_chunks, splits;
  int Npad, Kdim;
  FastDiv fBW, fBH, fHWd, fHH, fnbw, fnbh, fnbt, fBHBW, fHHHW;
};

typedef __attribute__((address_space(3))) void* lds_ptr_t;

__device__ __forceinline__ void halo_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Image swizzle: 16-B chunk c of row r is stored at chunk c ^ 2*((r >> L) & M), i.e. the 32-B
// chunk PAIR index is XORed with bits of r (cpr chunks per row: M = cpr/2 - 1, L = log2(16/cpr)).
// A transposed fragment read touches one 32-B pair in each of 8 CONSECUTIVE rows: their
// (row bank half, pair) combinations are then 8 distinct 32-B bank groups for ANY starting row,
// which is what the shifted halo rows (arbitrary start) need.
template <int CPR>
struct Swz {
  static constexpr int M = CPR / 2 - 1;
  static constexpr int L = CPR == 16 ? 0 : (CPR == 8 ? 1 : 2);
  static_assert(CPR == 4 || CPR == 8 || CPR == 16, "rows of 64, 128 or 256 bytes");
  __device__ static __forceinline__ int chunk(int row, int c) { return c ^ (2 * ((row >> L) & M)); }
  // byte-address XOR term of row r (applies to the chunk-pair bits 5.. of an in-row address)
  __device__ static __forceinline__ uint32_t x(int row) { return (uint32_t)((row >> L) & M) << 5; }
};

__device__ __forceinline__ s16x4 tr_read(uint32_t byte_addr) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(uintptr_t)byte_addr);
}

__device__ __forceinline__ bf16x8 join(s16x4 lo, s16x4 hi) {
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

template <int BN, int CC>
struct HaloWgGeom {
  static constexpr int NT = 512, NW = 8;
  static constexpr int PMAX = 256;
  static constexpr int DCPR = BN / 8, XCPR = CC / 8;      // 16-B chunks per image row
  static constexpr int DRPI = 64 / DCPR, XRPI = 64 / XCPR;  // rows per 1-KiB DMA instruction
  static constexpr int D_BYTES = PMAX * BN * 2;
  static constexpr int TAB_BYTES = PMAX * 16;  // per box position: halo addresses of its dw shifts
  // halo rows: two stages of (dY image + halo image) + the table in 160 KiB
  static constexpr int HPMAX = (((163840 - TAB_BYTES) / 2 - D_BYTES) / (CC * 2)) / (XRPI * NW) * (XRPI * NW);
  static constexpr int X_BYTES = HPMAX * CC * 2;
  static constexpr int STAGE_BYTES = D_BYTES + X_BYTES;
  static constexpr int D_INST = PMAX / DRPI / NW;          // dY DMA instructions per wave
  static constexpr int X_INST = HPMAX / XRPI / NW;         // halo DMA instructions per wave (max)
};

// HWD: halo row pitch in positions (compile time, a multiple of 8 >= BW + KW - 1), so every tap
// shift is an immediate offset of the LDS read. Temporal kernels use boxes one row high (HH = 1).
template <int KT, int KH, int KW, int BN, int CC, int HWD>
__global__ __launch_bounds__(512, 1) void halo_wgrad_kernel(HaloWgParams p) {
  using G = HaloWgGeom<BN, CC>;
  constexpr int TAPS = KT * KH * KW;
  constexpr int NBLK = BN / 16, CBLK = CC / 16;
  // waves along k: wave wk owns channel blocks cb = wk, wk + WK, ... for EVERY tap, so a
  // k-block's tap (and its halo shift) is a compile-time function of the register index
  constexpr int WK = CBLK < 4 ? CBLK : 4;
  constexpr int WN = G::NW / WK;          // waves along n
  constexpr int NBW = NBLK / WN;          // n-blocks per wave
  constexpr int KBW = TAPS * (CBLK / WK);  // k-blocks per wave: j -> (tap j % TAPS, cb wk + WK * (j / TAPS))
  static_assert(NBLK % WN == 0 && CBLK % WK == 0, "wave tiling");

  // two stages and the position table as SEPARATE static arrays: a fragment read of one stage then
  // provably does not alias the LDS-DMA filling the other, so the compiler does not drain that DMA
  // (s_waitcnt vmcnt(0)) in front of the read -- with one dynamic buffer it did, at every box, and
  // the next box's load never overlapped this box's MFMAs
  __shared__ __attribute__((aligned(16))) char st0[G::STAGE_BYTES];
  __shared__ __attribute__((aligned(16))) char st1[G::STAGE_BYTES];
  __shared__ __attribute__((aligned(16))) char tabmem[G::TAB_BYTES];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wave % WN, wk = wave / WN;
  const int ntiles = p.n_slices * p.c_chunks;
  const int nblocks = ntiles * p.splits;
  const int logical = xcd_remap(blockIdx.x, nblocks);
  const int split = logical / ntiles;
  const int tile = logical - split * ntiles;
  const int n0 = (tile % p.n_slices) * BN;
  const int c0 = (tile / p.n_slices) * CC;
  const int box_begin = (int)((long long)split * p.nboxes / p.splits);
  const int box_end = (int)((long long)(split + 1) * p.nboxes / p.splits);

  // DMA lane mapping (row-invariant slot / source chunk within each instruction)
  const int d_slot = lane % G::DCPR, d_lr = lane / G::DCPR;
  const int x_slot = lane % G::XCPR, x_lr = lane / G::XCPR;
  const long long clip_elems_x = (long long)p.T * p.H * p.W * p.Cin;
  const long long clip_elems_d = (long long)p.T * p.H * p.W * p.ldd;

  f32x4 acc[NBW][KBW];
#pragma unroll
  for (int i = 0; i < NBW; ++i)
#pragma unroll
    for (int j = 0; j < KBW; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  auto issue = [&](int box, auto SC) {
    char* sd = decltype(SC)::value ? st1 : st0;
    char* sx = sd + G::D_BYTES;
    uint32_t q0 = fdiv((uint32_t)box, p.fnbw);
    const int bw = box - q0 * p.nbw;
    const uint32_t q1 = fdiv(q0, p.fnbh);
    const int bh = q0 - q1 * p.nbh;
    const uint32_t b = fdiv(q1, p.fnbt);
    const int bt = q1 - b * p.nbt;
    const int t0 = bt * p.BT, h0 = bh * p.BH, w0 = bw * p.BW;
    const auto drs = __builtin_amdgcn_make_buffer_rsrc((void*)(p.dy + (long long)b * clip_elems_d), (short)0,
                                                       (int)(clip_elems_d * 2 > 0x7FFFFFF0LL ? 0x7FFFFFF0LL : clip_elems_d * 2),
                                                       0x00020000);
    const auto xrs = __builtin_amdgcn_make_buffer_rsrc((void*)(p.x + (long long)b * clip_elems_x), (short)0,
                                                       (int)(clip_elems_x * 2 > 0x7FFFFFF0LL ? 0x7FFFFFF0LL : clip_elems_x * 2),
                                                       0x00020000);
#pragma unroll
    for (int i = 0; i < G::D_INST; ++i) {
      const int r0 = (i * G::NW + wave) * G::DRPI;
      const int r = r0 + d_lr;
      const uint32_t pq = fdiv((uint32_t)r, p.fBHBW);
      const int rem = r - pq * (p.BH * p.BW);
      const uint32_t ph_ = fdiv((uint32_t)rem, p.fBW);
      const int pw_ = rem - ph_ * p.BW;
      const int t = t0 + (int)pq, h = h0 + (int)ph_, w = w0 + pw_;
      const int chunk = Swz<G::DCPR>::chunk(r, d_slot);
      const int n = n0 + chunk * 8;
      const bool v = (r < p.P) & (t < p.T) & (h < p.H) & (w < p.W) & (n < p.Cout);
      const uint32_t off = v ? (uint32_t)((((t * p.H + h) * p.W + w) * p.ldd + n) * 2) : 0x80000000u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(drs, (lds_ptr_t)(sd + r0 * BN * 2), 16, off, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < G::X_INST; ++i) {
      const int r0 = (i * G::NW + wave) * G::XRPI;
      if (r0 < p.HP) {  // wave-uniform: rows past the box's halo are never read
        const int r = r0 + x_lr;
        const uint32_t tq = fdiv((uint32_t)r, p.fHHHW);
        const int rem = r - tq * (p.HH * p.HWd);
        const uint32_t hq = fdiv((uint32_t)rem, p.fHWd);
        const int wq = rem - hq * p.HWd;
        const int t = t0 - p.pt + (int)tq, h = h0 - p.ph + (int)hq, w = w0 - p.pw + wq;
        const int chunk = Swz<G::XCPR>::chunk(r, x_slot);
        const int c = c0 + chunk * 8;
        const bool v = (r < p.HP) & ((unsigned)t < (unsigned)p.T) & ((unsigned)h < (unsigned)p.H) &
                       ((unsigned)w < (unsigned)p.W) & (c < p.Cin);
        const uint32_t off = v ? (uint32_t)((((t * p.H + h) * p.W + w) * p.Cin + c) * 2) : 0x80000000u;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (lds_ptr_t)(sx + r0 * CC * 2), 16, off, 0, 0, 0);
      }
    }
  };

  const int g = lane >> 4, li = lane & 15, q = li >> 2, pp = li & 3;
  const int nks = (p.P + 31) / 32;
  constexpr int XROWB = CC * 2, DROWB = BN * 2;
  static_assert(HWD % 8 == 0, "row pitch");
  static_assert(KT == 1 || (KH == 1 && KW == 1), "one tap axis");
  // per box position (the box shape is the same for every box): byte address in the halo image
  // of its row shifted by dw, with the swizzle's chunk-pair XOR pre-applied (bits 5.. of the
  // row-relative address are zero, so a lane XORs its own chunk/half bits on top)
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  __attribute__((address_space(3))) u32x4* tab =
      (__attribute__((address_space(3))) u32x4*)((__attribute__((address_space(3))) char*)tabmem);
  if (tid < G::PMAX) {
    const int pos = tid;
    const uint32_t tq = fdiv((uint32_t)pos, p.fBHBW);
    const int rem = pos - tq * (p.BH * p.BW);
    const uint32_t yq = fdiv((uint32_t)rem, p.fBW);
    const int h = pos < p.P ? ((int)tq * p.HH + (int)yq) * HWD + (rem - (int)yq * p.BW) : 0;
    uint32_t u[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) u[d] = (uint32_t)((h + d) * XROWB) ^ Swz<G::XCPR>::x(h + d);
    tab[pos] = (u32x4){u[0], u[1], u[2], u[3]};
  }
  // lane constants: chunk/half bits of its fragment column, per n-block (A) and channel block (B)
  constexpr int CBW = CBLK / WK;  // channel blocks per wave
  uint32_t lane_b[CBW];
#pragma unroll
  for (int c = 0; c < CBW; ++c) lane_b[c] = (uint32_t)((((wk + WK * c) * 2 + (pp >> 1)) << 4) | ((pp & 1) << 3));
  const int lp = 4 * g + q;  // this lane's first position inside a k-step (second: lp + 16)
  uint32_t lane_a[NBW];
#pragma unroll
  for (int i = 0; i < NBW; ++i)
    lane_a[i] = (uint32_t)(lp * DROWB) +
                ((uint32_t)((((wn * NBW + i) * 2 + (pp >> 1)) << 4) | ((pp & 1) << 3)) ^ Swz<G::DCPR>::x(lp));
  typedef __attribute__((address_space(3))) char lds_char;
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  if (box_begin < box_end) issue(box_begin, S0{});
  // boxes in pairs, stage 0 then stage 1 (compile-time stages: see st0 / st1)
  auto body = [&](int box, auto SC) {
    constexpr int stage = decltype(SC)::value;
    // (the builtin, not inline asm: the compiler's wait tracking sees it, so the stage DMAs before
    // it count as complete and only the one issued below stays pending)
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    halo_barrier();  // this box's images landed (every wave waited) and the other stage is free
    if (box + 1 < box_end) issue(box + 1, std::integral_constant<int, stage ^ 1>{});
    lds_char* dimg = (lds_char*)(stage ? st1 : st0);
    lds_char* ximg = dimg + G::D_BYTES;
    auto load = [&](int ks, bf16x8 (&af)[NBW], bf16x8 (&bfr)[KBW]) {
      lds_char* dks = dimg + ks * 32 * DROWB;
#pragma unroll
      for (int i = 0; i < NBW; ++i) {
        lds_char* a = dks + lane_a[i];
        af[i] = join(__builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)a),
                     __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                         (__attribute__((address_space(3))) s16x4*)(a + 16 * DROWB)));
      }
      const u32x4 ta = tab[ks * 32 + lp], tb = tab[ks * 32 + lp + 16];
      const uint32_t ua[4] = {ta[0], ta[1], ta[2], ta[3]}, ub[4] = {tb[0], tb[1], tb[2], tb[3]};
#pragma unroll
      for (int j = 0; j < KBW; ++j) {
        const int tap = j % TAPS, c = j / TAPS;
        const int dt = tap / (KH * KW), dh = (tap / KW) % KH, dw = tap % KW;
        const int imm = (dt + dh) * HWD * XROWB;  // one tap axis per kernel: dt or dh, never both
        lds_char* xa = ximg + (ua[dw] ^ lane_b[c]) + imm;
        lds_char* xb = ximg + (ub[dw] ^ lane_b[c]) + imm;
        bfr[j] = join(__builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)xa),
                      __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)xb));
      }
    };
    auto mma = [&](const bf16x8 (&af)[NBW], const bf16x8 (&bfr)[KBW]) {
#pragma unroll
      for (int j = 0; j < KBW; ++j)
#pragma unroll
        for (int i = 0; i < NBW; ++i)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    };
    // register double buffer: the reads of k-step ks+1 are in flight during the MFMAs of ks
    bf16x8 af0[NBW], bf0[KBW], af1[NBW], bf1[KBW];
    load(0, af0, bf0);
    for (int ks = 0; ks < nks; ks += 2) {
      if (ks + 1 < nks) load(ks + 1, af1, bf1);
      mma(af0, bf0);
      if (ks + 1 >= nks) break;
      if (ks + 2 < nks) load(ks + 2, af0, bf0);
      mma(af1, bf1);
    }
  };
  for (int box = box_begin; box < box_end; box += 2) {
    body(box, S0{});
    if (box + 1 < box_end) body(box + 1, S1{});
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // C[n][k]: row (n) = 4*(lane>>4) + r, col (k) = lane & 15
  float* out = p.slab + (long long)split * p.Npad * p.Kdim;
#pragma unroll
  for (int i = 0; i < NBW; ++i)
#pragma unroll
    for (int j = 0; j < KBW; ++j) {
      const int tap = j % TAPS, cb = wk + WK * (j / TAPS);
      const int c = c0 + cb * 16 + (lane & 15);
      if (c < p.Cin) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = n0 + (wn * NBW + i) * 16 + (lane >> 4) * 4 + r;
          out[(long long)n * p.Kdim + tap * p.Cin + c] = acc[i][j][r];
        }
      }
    }
}

// csrc/conv.hip: sum the split slabs and scatter to the PyTorch weight layout
int launch_wgrad_reduce(const float* slab, float* dw, int splits, int Npad, int Kpad, int Cout, int Cin,
                        int Cin_param, int taps, int accumulate, hipStream_t stream);

namespace {

int halo_hpmax(int cc) { return cc == 64 ? HaloWgGeom<64, 64>::HPMAX : HaloWgGeom<64, 128>::HPMAX; }

struct Box {
  int bt, bh, bw, P, HP, hwd;
  double cost;
};

constexpr int kHwd[3] = {16, 32, 56};  // compile-time halo row pitches (positions)

// Output box for a (KT, KH, KW) conv over (T, H, W): minimise padded MFMA work plus a small
// weight on halo loading, with P <= 256 positions, a halo row pitch from kHwd and a halo that
// fits the stage. Temporal kernels take boxes one row high (their tap shift is the t-plane).
Box choose_box(int T, int H, int W, int KT, int KH, int KW, int hpmax) {
  Box best{1, 1, 1, 1, 1, 16, 1e30};
  for (int bt = 1; bt <= T; ++bt)
    for (int bh = 1; bh <= (KT > 1 ? 1 : H); ++bh)
      for (int bw = 1; bw <= W; ++bw) {
        const int P = bt * bh * bw;
        if (P > 256) break;
        int hwd = 0;
        for (int c : kHwd)
          if (hwd == 0 && c >= bw + KW - 1) hwd = c;
        if (hwd == 0) break;
        const int HP = (bt + KT - 1) * (bh + KH - 1) * hwd;
        if (HP > hpmax) break;
        const long long nb = (long long)((T + bt - 1) / bt) * ((H + bh - 1) / bh) * ((W + bw - 1) / bw);
        const double cost = (double)nb * (((P + 31) / 32) * 32 + 0.15 * HP + 24.0);  // + per-box overhead
        if (cost < best.cost) best = Box{bt, bh, bw, P, HP, hwd, cost};
      }
  return best;
}

template <int KT, int KH, int KW, int BN, int CC, int HWD>
int launch_halo_wgrad_t(HaloWgParams& p, hipStream_t stream) {
  using G = HaloWgGeom<BN, CC>;
  static_assert(2 * G::STAGE_BYTES + G::TAB_BYTES <= 160 * 1024, "static LDS");
  const int nblocks = p.n_slices * p.c_chunks * p.splits;
  hipLaunchKernelGGL((halo_wgrad_kernel<KT, KH, KW, BN, CC, HWD>), dim3(nblocks), dim3(G::NT), 0, stream, p);
  return (int)hipGetLastError();
}

template <int KT, int KH, int KW, int BN, int CC>
int launch_halo_wgrad(HaloWgParams& p, hipStream_t stream) {
  if (p.HWd == 16) return launch_halo_wgrad_t<KT, KH, KW, BN, CC, 16>(p, stream);
  if (p.HWd == 32) return launch_halo_wgrad_t<KT, KH, KW, BN, CC, 32>(p, stream);
  if (p.HWd == 56) return launch_halo_wgrad_t<KT, KH, KW, BN, CC, 56>(p, stream);
  return (int)hipErrorInvalidValue;
}

}  // namespace

// Query: slab floats needed (returned through *slab_floats) for the halo wgrad of this shape, or
// an error if the shape is not supported. blocks_target: workgroups to aim for (0: 2 per CU).
MILNCE_API int milnce_halo_wgrad_plan(int B, int T, int H, int W, int Cin, int Cout, int KT, int KH, int KW, int bn,
                                      int cc, int blocks_target, long long* slab_floats, int* splits_out) {
  if (!((KT == 1 && KH == 3 && KW == 3) || (KT == 3 && KH == 1 && KW == 1))) return (int)hipErrorInvalidValue;
  if (bn != 64 || !(cc == 64 || (cc == 128 && KT == 3))) return (int)hipErrorInvalidValue;
  const int hpmax = halo_hpmax(cc);
  const Box bx = choose_box(T, H, W, KT, KH, KW, hpmax);
  if (bx.cost >= 1e29) return (int)hipErrorInvalidValue;
  const int nboxes = B * ((T + bx.bt - 1) / bx.bt) * ((H + bx.bh - 1) / bx.bh) * ((W + bx.bw - 1) / bx.bw);
  const int ntiles = ((Cout + bn - 1) / bn) * ((Cin + cc - 1) / cc);
  const int target = blocks_target > 0 ? blocks_target : 512;
  int splits = (int)fill_splits(target, ntiles);
  if (splits > nboxes) splits = nboxes;
  if (splits < 1) splits = 1;
  *splits_out = splits;
  *slab_floats = (long long)splits * ((Cout + bn - 1) / bn) * bn * (KT * KH * KW * Cin);
  return 0;
}

MILNCE_API int milnce_halo_wgrad(const void* dy, int ldd, const void* x, float* slab, float* dw, int accumulate,
                                 int B, int T, int H, int W, int Cin, int Cin_param, int Cout, int KT, int KH, int KW,
                                 int bn, int cc, int splits, hipStream_t stream) {
  HaloWgParams p;
  p.dy = (const bf16_t*)dy; p.x = (const bf16_t*)x; p.slab = slab;
  p.B = B; p.T = T; p.H = H; p.W = W; p.Cin = Cin; p.Cout = Cout; p.ldd = ldd;
  p.pt = KT / 2; p.ph = KH / 2; p.pw = KW / 2;
  const Box bx = choose_box(T, H, W, KT, KH, KW, halo_hpmax(cc));
  p.BT = bx.bt; p.BH = bx.bh; p.BW = bx.bw; p.P = bx.P; p.HP = bx.HP;
  p.HH = bx.bh + KH - 1; p.HWd = bx.hwd;  // multiple of 8: see Swz
  p.nbt = (T + bx.bt - 1) / bx.bt; p.nbh = (H + bx.bh - 1) / bx.bh; p.nbw = (W + bx.bw - 1) / bx.bw;
  p.nboxes = B * p.nbt * p.nbh * p.nbw;
  p.n_slices = (Cout + bn - 1) / bn; p.c_chunks = (Cin + cc - 1) / cc; p.splits = splits;
  p.Npad = p.n_slices * bn; p.Kdim = KT * KH * KW * Cin;
  p.fBW = make_fastdiv(p.BW); p.fBH = make_fastdiv(p.BH); p.fHWd = make_fastdiv(p.HWd); p.fHH = make_fastdiv(p.HH);
  p.fnbw = make_fastdiv(p.nbw); p.fnbh = make_fastdiv(p.nbh); p.fnbt = make_fastdiv(p.nbt);
  p.fBHBW = make_fastdiv(p.BH * p.BW); p.fHHHW = make_fastdiv(p.HH * p.HWd);
  if ((long long)T * H * W * (ldd > Cin ? ldd : Cin) * 2 > 0x7FFFFFF0LL) return (int)hipErrorInvalidValue;
  int rc;
  if (KT == 1) {
    if (cc == 64) rc = launch_halo_wgrad<1, 3, 3, 64, 64>(p, stream);
    else return (int)hipErrorInvalidValue;
  } else {
    if (cc == 64) rc = launch_halo_wgrad<3, 1, 1, 64, 64>(p, stream);
    else if (cc == 128) rc = launch_halo_wgrad<3, 1, 1, 64, 128>(p, stream);
    else return (int)hipErrorInvalidValue;
  }
  if (rc) return rc;
  if (dw == nullptr) return 0;  // the caller reduces the slab (milnce_wgrad_reduce; Npad = ceil(Cout / bn) * bn, Kpad = taps * Cin)
  return launch_wgrad_reduce(slab, dw, splits, p.Npad, p.Kdim, Cout, Cin, Cin_param, KT * KH * KW, accumulate, stream);
}
