// Shared by the implicit-GEMM conv kernels (conv.hip: v2 / v3 / wgrad / stem; conv_v4.hip: the
// scalar-offset LDS-DMA ring): the launch parameters, the LDS tile swizzle and the ring
// synchronisation helpers.
#pragma once
#include "common.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));

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
  long long x_total_bytes;
  FastDiv fWo, fHo, fTo, fCin, fKW, fKH;
  // epilogue statistics: 0 none; 1 BN forward sums of this conv's output (stats);
  // 2 BN backward partials of the PRODUCER of this dgrad's output: the output is that
  //   layer's dz, bn_y/bn_ss its raw conv output and [mean, invstd, scale, shift];
  //   stats += (dz*mask, dz*mask*xhat) with mask = y*scale + shift > 0.
  int bn_mode;
  const bf16_t* bn_y;
  const float* bn_ss;
  int bn_ld;  // row stride of bn_y (elements)
};

template <int BK>
__device__ __forceinline__ int swz(int row, int chunk) {
  // 16-B chunk swizzle of a [rows][BK] bf16 tile (BK*2-byte rows).
  if constexpr (BK == 32) return chunk ^ ((row >> 2) & 3);
  else return chunk ^ ((row >> 1) & 7);
}

// One asm statement with a memory clobber orders both: this wave's LDS reads of the previous
// stage are complete (lgkmcnt(0)) and no LDS access moves across the barrier.
__device__ __forceinline__ void ring_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Wait until at most N vector-memory operations (here: LDS-DMA pieces) of this wave are
// outstanding. N must be exact (rounding up would let a piece of the stage about to be read
// still be in flight), so it is a template constant; wait_stages picks N = ahead * NDMA.
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N <= 63, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// s_waitcnt immediate for vmcnt(n) alone (gfx9 encoding: vmcnt bits [3:0] and [15:14], expcnt
// [6:4] and lgkmcnt [11:8] at their maxima), for __builtin_amdgcn_s_waitcnt: unlike an inline-asm
// wait, the compiler's own wait tracking sees it
constexpr unsigned vmcnt_imm(int n) { return 0x0F70u | ((unsigned)n & 15u) | (((unsigned)n >> 4) << 14); }

template <int NDMA, int MAXAHEAD>
__device__ __forceinline__ void wait_stages(int ahead) {
  static_assert(MAXAHEAD <= 2, "ring depth");
  if (ahead <= 0) wait_vmcnt<0>();
  else if (ahead == 1 || MAXAHEAD < 2) wait_vmcnt<NDMA>();
  else wait_vmcnt<(MAXAHEAD >= 2 ? 2 * NDMA : 0)>();
}

typedef __attribute__((address_space(3))) void* lds_ptr_t;


// v4 forward / dgrad (conv_v4.hip): uniform-tap LDS-DMA ring with scalar stage offsets.
// impl 8 / 9: 16x16x32 / 32x32x16 MFMA, 2-stage ring; 10 / 11: the same, 3 stages;
// 12 / 13: 256-row tiles (8 waves), 2 stages.
// Returns V4_UNSUPPORTED for shapes it does not cover (Cin % 64, K padding, tap count, N tile).
constexpr int V4_UNSUPPORTED = -1;
int launch_fwd_v4(ConvParams& p, int bn, int impl, hipStream_t stream);
bool fwd_v4_supported(const ConvParams& p, int bn, int impl);

// box-tiled forward / dgrad (conv_box.hip, impl 14 / 15): stride-1 same-padded (1,3,3) / (3,1,1),
// Cin % 8 == 0 (a partial last 64-channel block), N tiles 64 / 128 / 192. pro_ss: [4][Cin] BN constants of the input's producer
// (z = relu(x * scale + shift) applied while staging) or null; pro_z: where z is also written
// (the consumer's wgrad operand) or null. With pro.y / pro.coef (dgrad): x is dz of that BN and the
// staged operand is its BN backward dy (written to pro.z).
struct BoxPro {
  const float* ss = nullptr;    // [4][Cin] mean / invstd / scale / shift of the input's BN
  void* z = nullptr;            // transformed input written here (null: not needed)
  const void* y = nullptr;      // dgrad BN-backward prologue: the BN's raw conv output
  const float* coef = nullptr;  //   and its backward coefficients [3][Cin]
  int xld = 0;                  // row stride of x in elements (0: Cin)
};
int launch_fwd_box(ConvParams& p, int bn, int impl, const BoxPro& pro, hipStream_t stream);
bool fwd_box_supported(const ConvParams& p, int bn, int impl);
