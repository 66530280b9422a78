// Box-tiled implicit-GEMM forward / dgrad for S3D-G's stride-1 same-padded (1,3,3) and (3,1,1)
// convs on gfx950 (impl 14 in the autotuner, next to v3 / v4).
//
// Why: the v4 ring gathers a fresh [256 x 64] activation tile per (tap, channel block) stage, so
// every input element is staged through LDS once per tap (9x for (1,3,3), 3x for (3,1,1)). The
// v4 ablation (tools/gpu/v4_ablate.sh, profiles/r3_box_conv.md) measured that gather at ~1/3 of
// the conv_2c kernel time and the LDS-staged epilogue at another ~1/5, against a bare
// LDS-read + MFMA loop at 1.8 PF/s. Here:
//
//   * the activation operand of a tile is staged ONCE per 64-channel block as a "box": every
//     input row any tap of the tile reads, in a padded layout where each tap is a constant row
//     shift, register-staged (buffer loads -> ds_write_b128) into rows of 80 bf16 (160 B pitch:
//     conflict-free ds_read_b128 fragments at ANY row shift, see below);
//       (1,3,3): rows in the "extended" plane order e = q*(H+1)(W+1) + (h+1)(W+1) + (w+1) (q =
//                clip-frame plane; the pad row / column is shared by neighbouring planes / rows),
//                tap (dh,dw) of output m reads box row e(m) - e(m0) + dh*(W+1) + dw;
//       (3,1,1): a tile is P = 256/T positions x all T frames of one clip (rows t*P + j), the box
//                (T+2) x P rows, tap dt reads box row (t+dt)*P + j;
//   * the weight stages [(channel block, tap)] stream through a 3-deep LDS-DMA ring (the v4 swizzle)
//     that runs continuously across tiles: a tile's last iterations already fire the next tile's
//     first stages, so their latency hides under the epilogue;
//   * the next box (next channel block, or the next tile's first) is loaded into registers at the
//     first tap of a block and written to LDS after its last tap; the exact per-wave vmcnt waits
//     account for the box loads and the epilogue stores in flight (all counts compile-time);
//   * the epilogue stages the tile's bf16 rows in the box region (two 128-row halves); every thread
//     then owns an 8-channel column chunk: 16-B row stores (buffer stores: out-of-range rows go
//     past num_records, so every wave issues the same count) and BN statistics / producer-BN
//     partials accumulated in registers across the thread's tiles (as in v4), reduced once.
//
// LDS fragment reads: lane l of a 16x16x32 fragment reads row r0 + (l & 15) at chunk c0 + (l >> 4).
// With a 160-B pitch (10 chunks) the 16 lanes of each ds_read_b128 bank group hit 4-bank slots
// (10 r + c) mod 16 that are all distinct for any r0 (the rows of a group split into even / odd
// slot sets), so shifted taps stay conflict-free (the w-wrap inside a fragment can cost one).
#include "conv_common.h"

#include <algorithm>
#include <type_traits>
#include <utility>

// Two workgroup shapes (template NW): 8 waves, one workgroup per CU (impls 14 / 15): 256-row tiles
// (4 waves along M x 2 along N), a 448-row box; 4 waves, TWO workgroups per CU (impls 16 / 17,
// <= 80 KiB of LDS each): 128-row tiles (2 x 2 waves), a 288-row (1,3,3) / 192-row (3,1,1) box,
// so one workgroup's barrier waits, box / weight-stage waits and epilogue stores run while the
// other one issues MFMAs on the same SIMDs (one wave of each per SIMD).
template <int NW> struct BoxShape {
  static constexpr int BM = NW * 32;  // output rows per tile: NW / 2 waves along M x 64 rows
};
static constexpr int BX_BM = 256;        // 8-wave tile rows
static constexpr int BX_BK = 64;         // channels per box / K stage
// bf16 per box row: 16x16x32 fragments (lane rows l & 15, chunks c + (l >> 4)) are conflict-free
// at a 10-chunk pitch, 32x32x16 fragments (rows l & 31, one chunk per half-wave) at 9 chunks
template <int MF> struct BoxPitch { static constexpr int v = 80; };
template <> struct BoxPitch<32> { static constexpr int v = 72; };
static constexpr int BX_ROWS = 448;      // box capacity (rows), 8 waves
// box capacity by workgroup shape and conv: 4 waves, (1,3,3): 128 output rows span <= 288 box rows
// up to W = 50 (conv_2c at 200^2); (3,1,1): (T + 2) * P <= 192 rows (T = 8: P = 16)
__host__ __device__ constexpr int box_rows(int ks, int nw) { return nw == 8 ? BX_ROWS : ks == 133 ? 288 : 192; }
__host__ __device__ constexpr int box_lds_limit(int nw) { return nw == 8 ? 160 * 1024 : 80 * 1024; }

// Diagnostic ablations (debug libraries only, tools/gpu/box_ablate.sh; results are garbage):
// bit 0 box loads read one fixed chunk (L1-hot), bit 1 no weight DMA, bit 2 no epilogue stores /
// statistics, bit 3 no epilogue at all (no staging either), bit 4 epilogue stores issued out of
// range (no memory traffic), bit 5 no forward statistics (stores kept).
#ifndef BOX_ABLATE
#define BOX_ABLATE 0
#endif
// Phase-timestamp diagnostics (libmilnce_hip_trace.so, tools/box_trace.py): every wave of the first
// 64 workgroups records s_memtime at fixed points of its first tiles (lane e of two VGPRs holds
// event e, so recording costs a compare and a select and no memory traffic until the kernel end).
#ifndef BOX_TRACE
#define BOX_TRACE 0
#endif
// Fragment double-buffering across the K steps of a tap (see the tap loop); 0 for A/B libraries
#ifndef BOX_PIPE
#define BOX_PIPE 1
#endif
// EPI 2 epilogue rows prefetched into L2 during the last block (y_prefetch). Off: the A/B
// (gpurun_out r4ypf) measured 4351 / 4355 pairs/s without it against 4323 / 4335 with it (the
// EPI 2 variants spill more and the (1,3,3) dgrad of conv_2c went 2.24 -> 2.55 ms)
#ifndef BOX_YPF
#define BOX_YPF 0
#endif

struct BoxGeo {
  int KS;          // 133 or 311
  int W1, PL;      // 133: W + 1, (H + 1) * (W + 1)
  int P, tpc;      // 311: positions per tile (256 / T), tiles per clip
  int HW;
  FastDiv fHW, fW, fPL, fW1, ftpc, fP;
  const float* pro_ss;  // [4][Cin] of the input's BN (mean, invstd, scale, shift) or null
  bf16_t* pro_z;        // PRO 2 / 3: the transformed input, written once (the wgrad operand)
  // PRO 3 (dgrad whose input x is dz of a BN layer): that layer's raw conv output y and its
  // backward coefficients [3][Cin] (k0 = gamma * invstd, k1 = mean(dz * mask), k2 = mean(dz * mask
  // * xhat)): the staged operand is dy = k0 * (dz * mask - k1 - xhat * k2)
  const bf16_t* pro_y;
  const float* pro_coef;
  int xld;              // row stride of x in elements (Cin, or the channel count of a concatenated
                        // tensor x is a channel slice of); pro_z / pro_y are dense (stride Cin)
  long long zbytes;     // bytes of the dense pro_z / pro_y tensors
  uint32_t* trace;      // BOX_TRACE builds: per-wave phase timestamps (tools/box_trace.py), else null
};

// vmcnt wait with a runtime choice among compile-time counts (the counts must be exact)
template <int N>
__device__ __forceinline__ void bx_wait() {
  static_assert(N >= 0 && N <= 63, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// vmcnt wait for a count that folds to a constant once the tap loop is unrolled (the search
// disappears; a count left at run time would cost a branch chain per tap)
template <int LO, int HI>
__device__ __forceinline__ void bx_wait_bs(uint32_t n) {
  if constexpr (LO == HI) {
    bx_wait<LO>();
  } else {
    constexpr int MID = (LO + HI) / 2;
    if (n <= (uint32_t)MID) bx_wait_bs<LO, MID>(n);
    else bx_wait_bs<MID + 1, HI>(n);
  }
}
__device__ __forceinline__ void bx_wait_c(int n) { bx_wait_bs<0, 63>((uint32_t)n); }

// Epilogue staging LDS accesses as inline asm: the compiler treats every LDS access it can see
// after an LDS-DMA as possibly aliasing it and puts a vmcnt(0) in front (no alias scopes on the
// one dynamic LDS buffer), which would drain the next tile's weight stages, box loads and y
// prefetches at every staging write and read. The staging rows live in the box region, which no
// DMA targets, so the only ordering they need is lgkmcnt (waited explicitly) and the barriers.
typedef unsigned int bx_u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int bx_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint32_t bx_lds_addr(const void* p) {
  return (uint32_t)(size_t)(const __attribute__((address_space(3))) void*)p;
}
// (the byte offset is an immediate: unrolled accesses share one address VGPR, as compiled LDS
// accesses do -- per-access addresses would be hoisted out of the tile loop as live registers)
template <int OFF>
__device__ __forceinline__ void bx_ds_write64(uint32_t a, uint2 v) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset");
  const bx_u32x2 w = {v.x, v.y};
  asm volatile("ds_write_b64 %0, %1 offset:%2" ::"v"(a), "v"(w), "n"(OFF));
}
__device__ __forceinline__ void bx_ds_write128(uint32_t a, uint4 v) {
  const bx_u32x4 w = {v.x, v.y, v.z, v.w};
  asm volatile("ds_write_b128 %0, %1" ::"v"(a), "v"(w));
}
template <int OFF>
__device__ __forceinline__ bx_u32x4 bx_ds_read128(uint32_t a) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset");
  bx_u32x4 r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(a), "n"(OFF));
  return r;
}
// compile-time loop: f(std::integral_constant<int, i>) for i in [0, N)
template <typename F, int... I>
__device__ __forceinline__ void bx_sfor_(F& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void bx_sfor(F&& f) {
  bx_sfor_(f, std::make_integer_sequence<int, N>{});
}
__device__ __forceinline__ void bx_lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// N (1 or 4) float4 reads at byte offsets OFF + 32 k and the wait for them, as ONE asm statement:
// the values exist only after its lgkmcnt(0), so nothing that uses them can be scheduled before
// the wait (a compiled LDS read here would be preceded by a vmcnt(0) drain, see above; a separate
// read and wait could have their uses hoisted between the two). Early-clobber outputs: a result
// landing early must not overwrite the address of a later read.
template <int OFF, int N>
__device__ __forceinline__ void bx_ds_read_f4_sync(uint32_t a, float4 (&out)[4]) {
  static_assert((N == 1 || N == 4) && OFF >= 0 && OFF + 96 < 65536, "reads");
  bx_u32x4 r0, r1, r2, r3;
  if constexpr (N == 1) {
    asm volatile("ds_read_b128 %0, %1 offset:%2\n\ts_waitcnt lgkmcnt(0)" : "=&v"(r0) : "v"(a), "n"(OFF));
    r1 = r2 = r3 = r0;
  } else {
    asm volatile(
        "ds_read_b128 %0, %4 offset:%5\n\tds_read_b128 %1, %4 offset:%6\n\t"
        "ds_read_b128 %2, %4 offset:%7\n\tds_read_b128 %3, %4 offset:%8\n\ts_waitcnt lgkmcnt(0)"
        : "=&v"(r0), "=&v"(r1), "=&v"(r2), "=&v"(r3)
        : "v"(a), "n"(OFF), "n"(OFF + 32), "n"(OFF + 64), "n"(OFF + 96));
  }
  const bx_u32x4 rr[4] = {r0, r1, r2, r3};
#pragma unroll
  for (int k = 0; k < 4; ++k)
    out[k] = make_float4(__uint_as_float(rr[k].x), __uint_as_float(rr[k].y), __uint_as_float(rr[k].z),
                         __uint_as_float(rr[k].w));
}

// N (1-4) 16-B reads at byte offsets OFF + k * STRIDE and their lgkmcnt(0), as ONE asm statement
// (same reason as above: a use of a result can only follow the wait)
template <int OFF, int STRIDE, int N>
__device__ __forceinline__ void bx_ds_read128_sync(uint32_t a, bx_u32x4 (&out)[N]) {
  static_assert(N >= 1 && N <= 4 && OFF >= 0 && OFF + (N - 1) * STRIDE < 65536, "reads");
  if constexpr (N == 1) {
    asm volatile("ds_read_b128 %0, %1 offset:%2\n\ts_waitcnt lgkmcnt(0)" : "=&v"(out[0]) : "v"(a), "n"(OFF));
  } else if constexpr (N == 2) {
    asm volatile("ds_read_b128 %0, %2 offset:%3\n\tds_read_b128 %1, %2 offset:%4\n\ts_waitcnt lgkmcnt(0)"
                 : "=&v"(out[0]), "=&v"(out[1])
                 : "v"(a), "n"(OFF), "n"(OFF + STRIDE));
  } else if constexpr (N == 3) {
    asm volatile(
        "ds_read_b128 %0, %3 offset:%4\n\tds_read_b128 %1, %3 offset:%5\n\tds_read_b128 %2, %3 offset:%6\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(out[0]), "=&v"(out[1]), "=&v"(out[2])
        : "v"(a), "n"(OFF), "n"(OFF + STRIDE), "n"(OFF + 2 * STRIDE));
  } else {
    asm volatile(
        "ds_read_b128 %0, %4 offset:%5\n\tds_read_b128 %1, %4 offset:%6\n\t"
        "ds_read_b128 %2, %4 offset:%7\n\tds_read_b128 %3, %4 offset:%8\n\ts_waitcnt lgkmcnt(0)"
        : "=&v"(out[0]), "=&v"(out[1]), "=&v"(out[2]), "=&v"(out[3])
        : "v"(a), "n"(OFF), "n"(OFF + STRIDE), "n"(OFF + 2 * STRIDE), "n"(OFF + 3 * STRIDE));
  }
}

// Exact vmcnt counts of the box kernel's weight-stage waits. At tap t of a channel block the wave
// waits for stage t of the block; every vector-memory op it issued after that stage's DMA may still
// be outstanding (vmcnt retires in issue order). Issue order per tap: wait, barrier, DMA of stage
// t + STG - 1 (none at tap 0 of a later tile's first block: fired ahead in the epilogue), box
// loads P(t). Block ends: the box's z stores (ZC); tile ends: the epilogue (EPI 2 y loads, the
// prefire after the first half's barrier, the stores), then the z stores. Cases: 0 = first block
// of the first tile (STG - 1 stages fired in the prologue), 1 = a later block of the same tile,
// 2 = the first block of a later tile.
struct BoxWaits {
  int y[3][2][9];  // [case][last block of the tile][tap]
};
// TPF / PFI: the last block of a tile issues PFI y-prefetch DMAs (EPI 2) at tap TPF, after that
// tap's weight DMA and box loads; a wait whose target was issued before them and that comes after
// them counts them too.
// NH: epilogue passes per tile (each: EPI_IT y loads (EPI 2, NPRE of them before the pass's barrier)
// and EPI_IT stores; the first pass fires the next tile's stage after its barrier)
__host__ __device__ constexpr BoxWaits make_box_waits(int TAPS, int STG, int NDMA, int P0, int PT, int NPT,
                                                      int EPI_IT, int NPRE, bool EPI2, int ZC, int NH, int TPF = 0,
                                                      int PFI = 0) {
  // P(u): box loads at tap u = P0 at tap 0, PT at taps 1 .. NPT-1 (P0 = PT when spread)
  BoxWaits w{};
  for (int c = 0; c < 3; ++c) {
    for (int last = 0; last < 2; ++last) {
      for (int t = 0; t < TAPS; ++t) {
        auto P = [&](int u) { return u == 0 ? P0 : (u < NPT ? PT : 0); };
        const int g = t - (STG - 1);  // tap of this block that fired stage t (< 0: earlier)
        const int epi_after_pre = (EPI2 ? NH * EPI_IT - NPRE : 0) + NH * EPI_IT;
        const int epi_all = (EPI2 ? NH * EPI_IT : 0) + NDMA + NH * EPI_IT;
        const bool pf_here = last && TPF < t;  // this block's prefetch lies before the wait
        int y = 0;
        if (c == 2 && t == STG - 1) {  // prefired in the previous tile's epilogue
          y = epi_after_pre + ZC + P(0);
          for (int h = 1; h < t; ++h) y += NDMA + P(h);
          if (pf_here) y += PFI;
        } else if (g >= 0) {
          y = P(g);
          for (int h = g + 1; h < t; ++h) y += NDMA + P(h);
          if (pf_here && g <= TPF) y += PFI;
        } else if (c == 0) {  // fired in the prologue
          y = (STG - 2 - t) * NDMA;
          for (int h = 0; h < t; ++h) y += NDMA + P(h);
          if (pf_here) y += PFI;
        } else {  // fired at tap TAPS + g of the previous block
          const int gp = TAPS + g;
          y = P(gp);
          for (int h = gp + 1; h < TAPS; ++h) y += NDMA + P(h);
          y += (c == 2 ? epi_all : 0) + ZC;
          for (int h = 0; h < t; ++h) y += (c == 2 && h == 0 ? 0 : NDMA) + P(h);
          if (c == 2 && gp <= TPF) y += PFI;  // the previous tile's last block prefetched after it
          if (pf_here) y += PFI;
        }
        w.y[c][last][t] = y;
      }
    }
  }
  return w;
}

// weight ring depth by N tile (stage rows rounded up to 64): as deep as the LDS next to the box
// allows. A box load issued at tap t is waited for by tap t + stages at the latest.
// (3,1,1) blocks have 3 taps: at most 4 stages, so a stage's DMA is always issued within the
// previous block (the wait tables above assume it)
__host__ __device__ constexpr int box_stages(int bn, int ks, int nw = 8) {
  if (nw == 4)  // within 80 KiB next to the 288 / 192-row box (stage rows rounded to 32)
    return ks == 133 ? (bn <= 64 ? 3 : 2) : (bn <= 64 ? 4 : bn <= 128 ? 3 : 2);
  return bn <= 64 ? (ks == 133 ? 8 : 4) : bn <= 128 ? 4 : 3;
}
__host__ __device__ constexpr int box_waits_max(const BoxWaits& w, int taps) {
  int m = 0;
  for (int c = 0; c < 3; ++c)
    for (int l = 0; l < 2; ++l)
      for (int t = 0; t < taps; ++t) m = w.y[c][l][t] > m ? w.y[c][l][t] : m;
  return m;
}

template <int BN, int KS, int EPI, int PRO, int MF, int NW>
__global__ __launch_bounds__(NW * 64, NW == 4 ? 2 : 1) void conv_box_kernel(ConvParams p, BoxGeo g) {
  constexpr int BM = BoxShape<NW>::BM, BK = BX_BK, PITCH = BoxPitch<MF>::v;
  constexpr int NT = NW * 64, NWAVES = NW;
  constexpr int BXR = box_rows(KS, NW);        // box rows
  constexpr int RPB = NT / 8;                  // box rows per staging pass (8 chunks per row)
  constexpr int WM = 64, WN = BN / 2;
  constexpr int TM = WM / MF, TN = WN / MF;
  constexpr int KSTEPS = BK / (MF == 16 ? 32 : 16);
  constexpr int TAPS = KS == 133 ? 9 : 3;
  constexpr int CPR = BK / 8, RPI = 64 / CPR;  // B ring: 8 rows (1 KiB) per DMA instruction
  // weight stage rows: BN rounded up to the rows one DMA round of all waves covers (8 waves: N tiles
  // of 96 / 160 load 128 / 192 rows; the extra rows are never read)
  constexpr int BNR = (BN + RPI * NWAVES - 1) / (RPI * NWAVES) * (RPI * NWAVES);
  constexpr int B_INST = BNR / RPI / NWAVES;   // DMA pieces per wave per stage
  constexpr int NDMA = B_INST;
  constexpr int NBX = BXR * 8 / NT;            // box chunks (16 B) per thread (7 / 9 / 6)
  static_assert(NBX * NT == BXR * 8, "box staging");
  // epilogue: column-owner passes over EH-row pieces staged in the box region (128 rows, or 64
  // where a 128-row piece of a wide tile does not fit the 4-wave box)
  constexpr int LDE = BN + 8;                  // staged row (elements)
  constexpr int EH = 128 * LDE <= BXR * 80 ? 128 : 64;
  constexpr int NH = BM / EH;                  // epilogue passes per tile
  constexpr int OCPR = BN / 8;                 // 16-B chunks per output row
  constexpr int RPP = NT / OCPR;               // rows per pass
  constexpr int EPI_IT = (EH + RPP - 1) / RPP;
  constexpr int EPI_G = EPI == 2 ? 2 : 4;      // staged chunks read per LDS wait
  constexpr int ZC = PRO >= 2 ? NBX : 0;       // z stores per wave per written box
  static_assert(EH * LDE <= BXR * 80 && EH % WM == 0 && BM % EH == 0, "epilogue piece fits the box region");
  static_assert(WN % MF == 0, "wave tile");
  constexpr int STAGE_ELEMS = BNR * BK;
  constexpr int STG = box_stages(BN, KS, NW);  // weight ring stages
  // (rows past the piece are read but not stored: they stay inside the LDS allocation)
  static_assert((NT / OCPR + (EPI_IT - 1) * RPP + 1) * LDE <= BXR * 80 + STG * STAGE_ELEMS, "epilogue reads in LDS");
  static_assert(B_INST * RPI * NWAVES == BNR, "DMA mapping");
  // box loads of one block: spread over the first taps of a (1,3,3) block (one x / y row chunk
  // per tap, so each has the ring's depth in taps to land and the loads do not arrive as one
  // burst), all at tap 0 of a (3,1,1) block (3 taps)
  constexpr int LPP = PRO == 3 ? 2 : 1;        // loads per box piece (PRO 3: dz and y)
  constexpr int NPRE = EPI_IT < 4 ? EPI_IT : 4;  // EPI 2: y rows loaded before a half's barrier
  static_assert(STG - 1 <= TAPS && (KS != 133 || NBX <= TAPS), "wait tables");
  // EPI 2: y-row prefetch of the tile's epilogue rows at tap TPF of its last block (y_prefetch)
  constexpr int TPF = TAPS >= 4 ? TAPS - 4 : 0;
  constexpr int PFI = (EPI == 2 && BOX_YPF) ? ((BM * ((BN * 2 + 127) / 128) / NWAVES) + 63) / 64 : 0;
  constexpr BoxWaits kWaits = KS == 133 ? make_box_waits(TAPS, STG, NDMA, LPP, LPP, NBX, EPI_IT, NPRE, EPI == 2, ZC,
                                                         NH, TPF, PFI)
                                        : make_box_waits(TAPS, STG, NDMA, NBX * LPP, 0, 1, EPI_IT, NPRE, EPI == 2, ZC,
                                                         NH, TPF, PFI);
  static_assert(box_waits_max(kWaits, TAPS) <= 63, "vmcnt range");
  static_assert(PRO != 3 || BN <= 128, "PRO 3 registers");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* box = (bf16_t*)smem;                                   // [BXR][PITCH]
  bf16_t* ring = box + BXR * 80;                                 // [STG][BNR][BK]
  float* ss_lds = (float*)(ring + STG * STAGE_ELEMS);            // EPI 2: [4][BN]; EPI 1: shift [BN]
  float* pro_lds = ss_lds + (EPI == 2 ? 4 * BN : EPI == 1 ? BN : 0);  // PRO 1/2: [2][Cin]; PRO 3: [7][Cin]
  // EPI 2: 256 B that the epilogue's y-row L2 prefetch (LDS-DMA, one dword per lane) writes and
  // nobody reads
  char* pf_lds = (char*)(pro_lds + (PRO == 3 ? 7 * p.Cin : (PRO ? 2 * p.Cin : 0)));

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  const int nblocks = p.num_n_tiles * p.grid_m;
  uint32_t tr_v0 = 0, tr_v1 = 0;
  int tr_n = 0;
  const unsigned long long tr_base = BOX_TRACE ? __builtin_amdgcn_s_memtime() : 0ull;
  auto tev = [&]() {
    if constexpr (BOX_TRACE != 0) {
      if (tr_n < 128) {
        const uint32_t t = (uint32_t)(__builtin_amdgcn_s_memtime() - tr_base);
        if (lane == (tr_n & 63)) {
          if (tr_n < 64) tr_v0 = t;
          else tr_v1 = t;
        }
      }
      ++tr_n;
    }
  };
  const int logical = xcd_remap(blockIdx.x, nblocks);
  const int n_tile = logical % p.num_n_tiles;
  const int m_slot = logical / p.num_n_tiles;
  const int n0 = n_tile * BN;
  const int ncb = (p.Cin + BK - 1) / BK;  // the last block may be partial (its missing chunks read zero)
  const int nst_tile = ncb * TAPS;  // stages per tile
  const int Cin = p.Cin;

  // ---- one-time LDS setup: statistics accumulators, BN constants ----
  float e_s[8], e_q[8];  // epilogue statistics of this thread's column chunk, over all its tiles
#pragma unroll
  for (int k = 0; k < 8; ++k) { e_s[k] = 0.f; e_q[k] = 0.f; }
  if constexpr (EPI == 2) {
    for (int t = tid; t < 4 * BN; t += NT) {
      const int q = t / BN, c = n0 + (t - q * BN);
      ss_lds[t] = c < p.Cout ? p.bn_ss[q * p.Cout + c] : 0.f;
    }
  }
  if constexpr (EPI == 1) {
    // per-channel shift (bn_ss, when set: the BN's running mean) subtracted before the bf16
    // rounding of the staged rows, so the stored pre-BN values keep their precision when
    // |mean| >> std
    for (int t = tid; t < BN; t += NT) ss_lds[t] = (p.bn_ss != nullptr && n0 + t < p.Cout) ? p.bn_ss[n0 + t] : 0.f;
  }
  if constexpr (PRO == 1 || PRO == 2) {
    for (int t = tid; t < 2 * Cin; t += NT) pro_lds[t] = g.pro_ss[2 * Cin + t];  // scale [Cin], shift [Cin]
  }
  if constexpr (PRO == 3) {  // mean, invstd, scale, shift, k0, k1, k2
    for (int t = tid; t < 4 * Cin; t += NT) pro_lds[t] = g.pro_ss[t];
    for (int t = tid; t < 3 * Cin; t += NT) pro_lds[4 * Cin + t] = g.pro_coef[t];
  }

  // ---- weight ring (v4 layout: swizzled chunks, soffset = stage K offset) ----
  const int slot = lane % CPR;
  const int lrow = wave * RPI + lane / CPR;
  const int src_chunk = swz<BK>(lrow, slot);
  const auto wrs = __builtin_amdgcn_make_buffer_rsrc((void*)p.w, (short)0,
                                                     (int)((long long)p.num_n_tiles * BN * p.Kpad * 2), 0x00020000);
  // fixed array bounds: template-constant bounds captured by the lambdas make clang's host pass
  // drop the kernel's launch stub (as in conv_v4.hip)
  static_assert(B_INST <= 8 && TM <= 4, "offset arrays");
  uint32_t ob[8];
#pragma unroll
  for (int i = 0; i < B_INST; ++i)
    ob[i] = (uint32_t)(((long long)(n0 + i * NWAVES * RPI + lrow) * p.Kpad + src_chunk * 8) * 2);
  // stage s of a tile = (cb, tap) = (s / TAPS, s % TAPS): weight columns tap * Cin + cb * 64
  // The counted vmcnt waits (BoxWaits) assume the vector-memory ops of a tap issue in program
  // order: the stage's DMA pieces, then the box loads, then the y prefetch. The scheduler may
  // otherwise interleave independent loads with the DMA pieces (it put box loads between them),
  // and a wait that leaves the "box load" outstanding then leaves a DMA piece in flight (a race
  // that shows with cold caches on 2-stage rings): every such group is fenced by sched_barriers.
  auto fire = [&](int gslot, int s_in_tile) {
    const int cb = s_in_tile / TAPS, tap = s_in_tile - cb * TAPS;
    bf16_t* sb = ring + gslot * STAGE_ELEMS;
    const int woff = __builtin_amdgcn_readfirstlane((tap * Cin + cb * BK) * 2);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < B_INST; ++i)
      if (!(BOX_ABLATE & 2)) __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, (lds_ptr_t)(sb + (i * NWAVES * RPI + wave * RPI) * BK), 16, ob[i],
                                               woff, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  };

  // ---- tile geometry ----
  const int xch = tid & 7, xrow0 = tid >> 3;  // box staging: chunk, first row (rows xrow0 + RPB k)
  struct TileInfo {
    long long xbase;     // byte offset of the tile's input base (rows of xld elements)
    long long zbase;     // byte offset of the same rows in the dense pro_z / pro_y
    long long ybase;     // element offset of the tile's output base row
    uint32_t xnrec, znrec;
    int e0, elast, m0;   // 133: extended index of the first / last output row, first row
    int b, p0;           // 311
  };
  auto tile_info = [&](int m_tile) {
    TileInfo ti;
    if constexpr (KS == 133) {
      const int m0 = m_tile * BM;
      const int ml = min(p.M, m0 + BM) - 1;
      auto ext = [&](int m) {
        const uint32_t q = fdiv((uint32_t)m, g.fHW);
        const int r = m - (int)q * g.HW;
        const uint32_t h = fdiv((uint32_t)r, g.fW);
        const int w = r - (int)h * p.W;
        return (int)q * g.PL + ((int)h + 1) * g.W1 + w + 1;
      };
      ti.m0 = m0;
      ti.e0 = ext(m0);
      ti.elast = ext(ml);
      const int qlo = (int)fdiv((uint32_t)max(0, ti.e0 - g.W1 - 1), g.fPL);
      ti.xbase = (long long)qlo * g.HW * g.xld * 2;
      ti.zbase = (long long)qlo * g.HW * Cin * 2;
      ti.ybase = (long long)m0 * p.ldy;
      ti.b = qlo;
      ti.p0 = 0;
    } else {
      const uint32_t b = fdiv((uint32_t)m_tile, g.ftpc);
      const int pb = m_tile - (int)b * g.tpc;
      ti.b = (int)b;
      ti.p0 = pb * g.P;
      ti.xbase = (long long)b * p.T * g.HW * g.xld * 2;
      ti.zbase = (long long)b * p.T * g.HW * Cin * 2;
      ti.ybase = (long long)b * p.T * g.HW * p.ldy;
      ti.m0 = ti.e0 = ti.elast = 0;
    }
    const long long remain = p.x_total_bytes - ti.xbase;
    ti.xnrec = remain > 0x7FFFFFF0LL ? 0x7FFFFFF0u : (uint32_t)(remain > 0 ? remain : 0);
    const long long zrem = g.zbytes - ti.zbase;
    ti.znrec = zrem > 0x7FFFFFF0LL ? 0x7FFFFFF0u : (uint32_t)(zrem > 0 ? zrem : 0);
    return ti;
  };
  // input row index of box row j relative to the tile's first row (xbase / zbase), or 0x80000000
  // (reads zero) for padding / out-of-range rows
  auto box_off = [&](const TileInfo& ti, int j) -> uint32_t {
    if constexpr (KS == 133) {
      const int e = ti.e0 - g.W1 - 1 + j;
      if (e < 0 || e > ti.elast + g.W1 + 1) return 0x80000000u;
      const uint32_t q = fdiv((uint32_t)e, g.fPL);
      const int r = e - (int)q * g.PL;
      const uint32_t hh = fdiv((uint32_t)r, g.fW1);
      const int ww = r - (int)hh * g.W1;
      if (hh == 0 || ww == 0 || (int)q >= p.M / g.HW) return 0x80000000u;
      const int qrel = (int)q - ti.b;
      return (uint32_t)(((long long)qrel * p.H + (int)hh - 1) * p.W + ww - 1);
    } else {
      const int tp = (int)fdiv((uint32_t)j, g.fP), jj = j - tp * g.P;
      const int t_in = tp - 1, pos = ti.p0 + jj;
      if (t_in < 0 || t_in >= p.T || pos >= g.HW || j >= (p.T + 2) * g.P) return 0x80000000u;
      return (uint32_t)((long long)t_in * g.HW + pos);
    }
  };

  // ---- box staging registers ----
  uint4 xr[NBX], yr[PRO == 3 ? NBX : 1];
  uint32_t xo[NBX];
  __amdgpu_buffer_rsrc_t yrs_box;  // PRO 3: the producer's y over the same box (same layout as x)
  // this thread's chunk of channel block cb exists (Cin not a multiple of 64: the last block is
  // partial; its missing chunks are zero in the box and never transformed or written back)
  auto chv = [&](int cb) { return cb * BK + xch * 8 < Cin; };
  // byte offsets of a box row (row index, or the out-of-range marker) in x and in the dense tensors
  const uint32_t xrow_bytes = (uint32_t)g.xld * 2, zrow_bytes = (uint32_t)Cin * 2;
  auto xoff = [&](uint32_t r) { return r == 0x80000000u ? r : r * xrow_bytes + (uint32_t)xch * 16; };
  auto zoff = [&](uint32_t r) { return r == 0x80000000u ? r : r * zrow_bytes + (uint32_t)xch * 16; };
  // box pieces k0 .. k1-1 of channel block cb (PRO 3: each an x (dz) and a y chunk)
  auto box_load = [&](__amdgpu_buffer_rsrc_t rs, int cb, int k0, int k1) {
    const int coff = __builtin_amdgcn_readfirstlane(cb * BK * 2);
    const bool cv = chv(cb);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int k = 0; k < NBX; ++k) {  // (constant bounds: xr stays in registers; k0 / k1 fold per tap)
      if (k < k0 || k >= k1) continue;
      xr[k] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                            rs, (BOX_ABLATE & 1) ? 0u : (cv ? xoff(xo[k]) : 0x80000000u), coff, 0));
      if constexpr (PRO == 3)
        yr[k] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(yrs_box, cv ? zoff(xo[k]) : 0x80000000u,
                                                                                coff, 0));
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  auto yrsrc = [&](const TileInfo& bt, bool valid) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)g.pro_y + bt.zbase), (short)0,
                                             (int)(valid ? bt.znrec : 0u), 0x00020000);
  };
  // PRO 2: the tile's own rows of the transformed input go to pro_z (same layout as x, so the
  // same offsets) from the workgroups of N tile 0; every wave issues NBX stores (out-of-range
  // offsets for the others) so the vmcnt accounting stays exact
  // The prologue transform of the staged chunks, in registers. The per-channel constants of this
  // thread's 8 channels are read into registers once per call: with the LDS box stores in between,
  // the compiler could not reuse LDS reads across rows. (1,3,3): applied after tap 3's MFMAs of the
  // block (the loads have landed there: tap 3's stage was fired after them), so the VALU work
  // interleaves with the MFMA phases; (3,1,1): right before the store.
  auto box_xform = [&](int cb, int pk0, int pk1) {
    const int c0 = min(cb * BK + xch * 8, Cin - 8);  // (clamped: a missing chunk is not transformed)
    const bool cv = chv(cb);
    if constexpr (PRO == 1 || PRO == 2) {
      float sc[8], sh[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) { sc[u] = pro_lds[c0 + u]; sh[u] = pro_lds[Cin + c0 + u]; }
#pragma unroll
      for (int k = 0; k < NBX; ++k) {
        if (k < pk0 || k >= pk1) continue;
        if (cv && xo[k] != 0x80000000u) {
          float f[8];
          unpack8(xr[k], f);
#pragma unroll
          for (int u = 0; u < 8; ++u) f[u] = fmaxf(f[u] * sc[u] + sh[u], 0.f);
          xr[k] = pack8(f);
        }
      }
    }
    if constexpr (PRO == 3) {
      BnBwdC q[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int c = c0 + u;
        q[u] = bn_bwd_const(pro_lds[c], pro_lds[Cin + c], pro_lds[2 * Cin + c], pro_lds[3 * Cin + c],
                            pro_lds[4 * Cin + c], pro_lds[5 * Cin + c], pro_lds[6 * Cin + c]);
      }
#pragma unroll
      for (int k = 0; k < NBX; ++k) {
        if (k < pk0 || k >= pk1) continue;
        if (cv && xo[k] != 0x80000000u) {  // padding rows stay zero (dy is zero-padded)
          float d[8], yy[8];
          unpack8(xr[k], d);
          unpack8(yr[k], yy);
#pragma unroll
          for (int u = 0; u < 8; ++u) d[u] = bn_bwd_elem(d[u], yy[u], q[u]);
          xr[k] = pack8(d);
        }
      }
    }
  };
  // (1,3,3): the pieces are transformed after the block's last tap (XF_LAG = TAPS), when the loads
  // of every piece have long landed: same-box A/Bs against transforming piece k after tap k + 2 / 3
  // (interleaved with the MFMA phases): 128-wide dgrad 0.437 -> 0.403 ms, conv_2c spatial dgrad
  // 2.98 (lag 3) -> 2.5 ms -- a transform waits for its piece's load, i.e. drains the vmcnt queue
  constexpr int XF_LAG = KS == 133 ? TAPS : -1;  // -1: at the store
  // PRO 2 / 3: the tile's own rows of the transformed input go to pro_z (same layout as x, so the
  // same offsets) from the workgroups of N tile 0; every wave issues NBX stores (out-of-range
  // offsets for the others) so the vmcnt accounting stays exact
  auto box_store = [&](int cb, const TileInfo& bt, __amdgpu_buffer_rsrc_t zs) {
    if constexpr (XF_LAG < 0) box_xform(cb, 0, NBX);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int k = 0; k < NBX; ++k) {
      const uint4 v = xr[k];
      bx_ds_write128(bx_lds_addr(box + (xrow0 + RPB * k) * PITCH + xch * 8), v);
      if constexpr (PRO >= 2) {
        bool own = n_tile == 0 && xo[k] != 0x80000000u && chv(cb);
        if constexpr (KS == 133) {
          const int j = xrow0 + RPB * k;
          own = own && j >= g.W1 + 1 && j <= bt.elast - bt.e0 + g.W1 + 1;
        }
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int, v),
                                               zs, own ? zoff(xo[k]) : 0x80000000u,
                                               __builtin_amdgcn_readfirstlane(cb * BK * 2), 0);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  auto zrsrc = [&](const TileInfo& bt, bool valid) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)((char*)g.pro_z + bt.zbase), (short)0,
                                             (int)(valid ? bt.znrec : 0u), 0x00020000);
  };

  // ---- per-lane fragment rows of a tile ----
  auto frag_rows = [&](const TileInfo& ti, int (&rb)[4], uint32_t (&yo)[4]) {  // box row, output byte offset
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int lr = wr * WM + i * MF + (lane & (MF - 1));
      if constexpr (KS == 133) {
        const int m = ti.m0 + lr;
        if (m < p.M) {
          const uint32_t q = fdiv((uint32_t)m, g.fHW);
          const int r = m - (int)q * g.HW;
          const uint32_t h = fdiv((uint32_t)r, g.fW);
          const int w = r - (int)h * p.W;
          rb[i] = (int)q * g.PL + ((int)h + 1) * g.W1 + w + 1 - ti.e0;
          yo[i] = (uint32_t)(lr * p.ldy * 2);
        } else {
          rb[i] = 0;
          yo[i] = 0x80000000u;
        }
      } else {
        const int t = (int)fdiv((uint32_t)lr, g.fP), j = lr - t * g.P;
        const bool v = t < p.T && ti.p0 + j < g.HW;  // rows past T * P idle
        rb[i] = t < p.T ? lr : 0;
        yo[i] = v ? (uint32_t)(((long long)t * g.HW + ti.p0 + j) * p.ldy * 2) : 0x80000000u;
      }
    }
  };

  // EPI 2: pull the tile's producer rows bn_y[row][n0 .. n0 + BN) into L2 during the last block's
  // taps, so the epilogue's y loads (one chain per thread) hit L2 instead of paying HBM latency
  // twice per tile (tools/box_trace.py: ~1/3 of the (3,1,1) dgrad's tile time). One dword per lane
  // and 128-B line, written to pf_lds and never read; issued after the tap's weight DMA, so only
  // stages fired >= 2 taps later can wait for them.
  auto y_prefetch = [&](const TileInfo& tt) {
    if constexpr (EPI == 2) {
      constexpr int LPR = (BN * 2 + 127) / 128;          // 128-B lines per row
      constexpr int LPW = BM * LPR / NWAVES;             // lines per wave
      constexpr int PF_INST = (LPW + 63) / 64;
      static_assert(!BOX_YPF || PF_INST == PFI, "prefetch count in the wait tables");
      // rows relative to the tile's first output row (133: rows m0 + lr; 311: (t * HW + p0 + j))
      const long long row0 = KS == 133 ? (long long)tt.m0 : (long long)tt.b * p.T * g.HW + tt.p0;
      const auto prs = __builtin_amdgcn_make_buffer_rsrc((void*)(p.bn_y + row0 * p.bn_ld), (short)0, 0x7FFFFFF0,
                                                         0x00020000);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int k = 0; k < PF_INST; ++k) {
        const int L = wave * LPW + min(k * 64 + lane, LPW - 1);
        const int lr = L / LPR, piece = L - lr * LPR;
        int rel;  // row relative to row0 (out-of-tile rows clamp to the tile's last valid row)
        if constexpr (KS == 133) {
          rel = min(lr, p.M - 1 - tt.m0);
        } else {
          const int t0 = (int)fdiv((uint32_t)lr, g.fP), t = min(t0, p.T - 1);
          rel = t * g.HW + min(lr - t0 * g.P, g.HW - 1 - tt.p0);
        }
        const uint32_t off = (uint32_t)((rel * p.bn_ld + min(n0 + piece * 64, p.Cout - 8)) * 2);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(prs, (lds_ptr_t)pf_lds, 4, off, 0, 0, 0);
      }
    }
  };

  const int ntiles = p.num_m_tiles;
  int m_tile = m_slot;
  if (m_tile >= ntiles) {  // no tile for this slot: its statistics row is zero
    if constexpr (EPI != 0) {
      const int npad = p.num_n_tiles * BN;
      for (int t = tid; t < BN; t += NT) {
        p.stats[(long long)m_slot * 2 * npad + n0 + t] = 0.f;
        p.stats[(long long)m_slot * 2 * npad + npad + n0 + t] = 0.f;
      }
    }
    return;
  }

  __syncthreads();  // setup writes visible
  tev();

  // ---- prologue: first tile's box (cb 0), synchronously; first two weight stages ----
  TileInfo ti = tile_info(m_tile);
  auto xrs = __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)p.x + ti.xbase), (short)0, (int)ti.xnrec,
                                               0x00020000);
#pragma unroll
  for (int k = 0; k < NBX; ++k) xo[k] = box_off(ti, xrow0 + RPB * k);
  auto zrs = zrsrc(ti, PRO >= 2);
  if constexpr (PRO == 3) yrs_box = yrsrc(ti, true);
  box_load(xrs, 0, 0, NBX);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr (XF_LAG >= 0) box_xform(0, 0, NBX);
  box_store(0, ti, zrs);
  int gs = 0;  // global stage counter (ring slot = gs % STG)
#pragma unroll
  for (int i = 0; i < STG - 1; ++i) fire(i, i % nst_tile);
  bool first_tile = true;

  typedef typename std::conditional<MF == 16, f32x4, f32x16>::type acc_t;
  while (true) {
    int rb[4];
    {
      uint32_t yo_unused[4];
      frag_rows(ti, rb, yo_unused);
    }
    const int next_tile = m_tile + p.grid_m;
    const bool has_next = next_tile < ntiles;
    TileInfo tn = has_next ? tile_info(next_tile) : ti;
    acc_t acc[TN][TM];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int i = 0; i < TM; ++i) acc[j][i] = acc_t{};

    for (int cb = 0; cb < ncb; ++cb) {
      const bool last_cb = cb == ncb - 1;
#pragma unroll
      for (int t = 0; t < TAPS; ++t) {
        const int s = cb * TAPS + t;  // stage within the tile
        // wait for stage s (the oldest in flight; exact counts, see BoxWaits): the ops issued
        // after its DMA -- later stages, box loads, the previous tile's epilogue stores and z
        // stores -- drain only when a stage fired after them is waited for
        const bool carried = cb == 0 && !first_tile;
        // (the last-block tables differ only after the y prefetch: t > TPF, EPI 2)
        if (PFI > 0 && t > TPF && last_cb) {
          if (cb > 0) bx_wait_c(kWaits.y[1][1][t]);
          else if (first_tile) bx_wait_c(kWaits.y[0][1][t]);
          else bx_wait_c(kWaits.y[2][1][t]);
        } else {
          if (cb > 0) bx_wait_c(kWaits.y[1][0][t]);
          else if (first_tile) bx_wait_c(kWaits.y[0][0][t]);
          else bx_wait_c(kWaits.y[2][0][t]);
        }
        tev();  // W: weight stage landed (this wave's share)
        ring_barrier();
        tev();  // B: every wave at the ring barrier
        // fire stage s + STG - 1 into the slot read at the previous tap (continuing into the next
        // tile: the weights do not depend on the tile); a carried tile's first one is in flight
        if (!(t == 0 && carried)) fire((gs + STG - 1) % STG, (s + STG - 1) % nst_tile);
        if (t == 0 && last_cb) {
          // the next box is the next tile's block 0
          auto nrs = __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)p.x + tn.xbase), (short)0,
                                                       (int)(has_next ? tn.xnrec : 0u), 0x00020000);
#pragma unroll
          for (int k = 0; k < NBX; ++k) xo[k] = box_off(tn, xrow0 + RPB * k);
          if constexpr (PRO == 3) yrs_box = yrsrc(tn, has_next);
          xrs = nrs;
          zrs = zrsrc(tn, PRO >= 2 && has_next);
        }
        // prefetch pieces of the next box (next channel block of this tile, or the next tile's
        // block 0)
        if constexpr (KS == 133) {
          if (t < NBX) box_load(xrs, last_cb ? 0 : cb + 1, t, t + 1);
        } else {
          if (t == 0) box_load(xrs, last_cb ? 0 : cb + 1, 0, NBX);
        }
        if constexpr (PFI > 0) {
          if (last_cb && t == TPF) y_prefetch(ti);
        }
        // ---- MFMAs of stage s: A = weights (ring), B = box rows shifted by the tap ----
        const bf16_t* bsh = ring + (gs % STG) * STAGE_ELEMS;
        int shift;
        if constexpr (KS == 133) shift = (t / 3) * g.W1 + (t % 3);
        else shift = t * g.P;
        const int sh = __builtin_amdgcn_readfirstlane(shift * PITCH);
        auto xfrag = [&](int ks, int i) {
          const int ch = MF == 16 ? ks * 4 + (lane >> 4) : ks * 2 + (lane >> 5);
          return *(const bf16x8*)(box + rb[i] * PITCH + sh + ch * 8);
        };
        auto wfrag = [&](int ks, int j) {
          const int row = wc * WN + j * MF + (lane & (MF - 1));
          const int ch = MF == 16 ? ks * 4 + (lane >> 4) : ks * 2 + (lane >> 5);
          return *(const bf16x8*)(bsh + row * BK + swz<BK>(row, ch) * 8);
        };
        // fragments double-buffered across the K steps (BOX_PIPE): step ks + 1's LDS reads are in
        // flight while step ks's MFMAs issue, instead of every step waiting out the LDS latency
        // before its MFMAs (the register sets alternate, so the reads need not wait for the MFMAs
        // that still read the previous set)
        // (only where a second fragment set fits the VGPR budget: 32x32 tiles, narrow 16x16 ones;
        // not the 192-wide (3,1,1) variants, which then spill ~25 VGPRs)
        constexpr bool PIPE = BOX_PIPE && (TM + TN) * 4 <= 24 && !(KS == 311 && BN == 192);
        bf16x8 xf[PIPE ? 2 : 1][TM], wf[PIPE ? 2 : 1][TN];
        auto frags = [&](int ks, int b) {
#pragma unroll
          for (int i = 0; i < TM; ++i) xf[b][i] = xfrag(ks, i);
#pragma unroll
          for (int j = 0; j < TN; ++j) wf[b][j] = wfrag(ks, j);
        };
        if constexpr (PIPE) frags(0, 0);
#pragma unroll
        for (int ks = 0; ks < KSTEPS; ++ks) {
          const int b = PIPE ? (ks & 1) : 0;
          if constexpr (PIPE) {
            if (ks + 1 < KSTEPS) frags(ks + 1, b ^ 1);
          } else {
            frags(ks, 0);
          }
          __builtin_amdgcn_s_setprio(1);
#pragma unroll
          for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int i = 0; i < TM; ++i)
              if constexpr (MF == 16)
                acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[b][j], xf[b][i], acc[j][i], 0, 0, 0);
              else
                acc[j][i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[b][j], xf[b][i], acc[j][i], 0, 0, 0);
          __builtin_amdgcn_s_setprio(0);
        }
        ++gs;
        tev();  // M: the tap's fragment reads and MFMAs issued
        if constexpr (XF_LAG >= 0 && PRO != 0) {
          // pieces whose transform falls on this tap (the block's last tap takes the rest)
          const int ka = max(t - XF_LAG, 0), kb = t == TAPS - 1 ? NBX : t - XF_LAG + 1;
          if (kb > ka) box_xform(last_cb ? 0 : cb + 1, ka, kb);
        }
      }
      // every wave is done with this box: write the prefetched one (the next iteration's ring
      // barrier publishes it)
      lds_barrier();
      tev();  // X: block end, every wave done with the box
      if (!last_cb) {
        box_store(cb + 1, ti, zrs);
        tev();  // S: next block's box written
      }
    }

    // ---- epilogue, two 128-row halves staged in the box region: waves wr 2h, 2h+1 write their
    // bf16 rows, then every thread owns one 8-channel column chunk and walks rows (16-B coalesced
    // stores, statistics carried in registers across tiles as in v4) ----
#pragma unroll
    for (int half = 0; half < ((BOX_ABLATE & 8) ? 0 : NH); ++half) {
      // EPI 2: the producer's raw outputs of this thread's rows, loaded before the staging writes
      // and the barrier so their latency overlaps them (one load chain, not one per row)
      // (at most 4 rows ahead: the other half's waves still hold their accumulators here)
      uint4 ypre[EPI_IT];
      auto yload = [&](int it) {
        const int cc = tid % OCPR;
        const int lr = half * EH + min(tid / OCPR + it * RPP, EH - 1);
        long long grow;
        if constexpr (KS == 133) {
          grow = min(ti.m0 + lr, p.M - 1);
        } else {
          const int t0 = (int)fdiv((uint32_t)lr, g.fP), t = min(t0, p.T - 1);
          const int j = min(lr - t0 * g.P, g.HW - 1 - ti.p0);
          grow = (long long)(ti.b * p.T + t) * g.HW + ti.p0 + j;
        }
        const int n = min(n0 + cc * 8, p.Cout - 8);
        return *(const uint4*)(p.bn_y + grow * p.bn_ld + n);
      };
      if constexpr (EPI == 2) {
#pragma unroll
        for (int it = 0; it < NPRE; ++it) ypre[it] = yload(it);
      }
      if ((wr * WM) / EH == half) {
        // row (wr * WM) % EH + i * MF + (lane & (MF - 1)) of the piece, column wc * WN + j * MF + the
        // lane's 4-column group (+ gq * 8 for 32x32 fragments)
        const uint32_t sbase = bx_lds_addr(box + ((wr * WM) % EH + (lane & (MF - 1))) * LDE + wc * WN +
                                           (MF == 16 ? (lane >> 4) * 4 : (lane >> 5) * 4));
        // EPI 1 shift of the lane's 4-column groups of fragment column j (+ gq * 8 for 32x32), read by
        // asm: a compiled LDS read here drained the next tile's weight DMA and box loads (vmcnt(0))
        const uint32_t shbase = bx_lds_addr(ss_lds + wc * WN + (MF == 16 ? (lane >> 4) * 4 : (lane >> 5) * 4));
        bx_sfor<TN>([&](auto J) {
          constexpr int jj = decltype(J)::value;
          float4 sh4[4] = {};
          if constexpr (EPI == 1) bx_ds_read_f4_sync<jj * MF * 4, MF == 16 ? 1 : 4>(shbase, sh4);
          bx_sfor<(MF == 16 ? 1 : 4)>([&](auto Q) {
            constexpr int j = decltype(J)::value, gq = decltype(Q)::value;
            const float4 sh = sh4[gq];
            bx_sfor<TM>([&](auto I) {
              constexpr int i = decltype(I)::value;
              uint2 o;
              o.x = pack2bf(acc[j][i][gq * 4 + 0] - sh.x, acc[j][i][gq * 4 + 1] - sh.y);
              o.y = pack2bf(acc[j][i][gq * 4 + 2] - sh.z, acc[j][i][gq * 4 + 3] - sh.w);
              bx_ds_write64<(i * MF * LDE + j * MF + gq * 8) * 2>(sbase, o);
            });
          });
        });
      }
      lds_barrier();
      tev();  // H1: the half's rows staged
      // every wave is past the tile's last MFMAs: the last stage's ring slot is free for the next
      // tile's stage STG - 1, fired ahead of the stores (so the stores drain behind it)
      if (half == 0) fire((gs + STG - 1) % STG, (STG - 1) % nst_tile);
      {
        const auto yrs = __builtin_amdgcn_make_buffer_rsrc((void*)(p.y + ti.ybase), (short)0, 0x7FFFFFF0, 0x00020000);
        const int cc = tid % OCPR;
        if constexpr (EPI == 2) {
#pragma unroll
          for (int it = NPRE; it < EPI_IT; ++it) ypre[it] = yload(it);
        }
        // the thread's staged chunks read EPI_G at a time, one wait per group (the other half's
        // waves still hold their accumulators here, so not all EPI_IT at once)
        // (rows past the half -- it * RPP + tid / OCPR >= 128 -- are read but not stored; they stay
        // inside the box region)
        bx_u32x4 dvs[EPI_IT];
        const uint32_t rbase = bx_lds_addr(box + (tid / OCPR) * LDE + cc * 8);
#pragma unroll
        for (int it = 0; it < EPI_IT; ++it) {
          if (it % EPI_G == 0) {
            // the group's reads and their wait in one asm statement (with a separate
            // wait, uses of the results could be scheduled between the reads and the wait)
            bx_sfor<(EPI_IT + EPI_G - 1) / EPI_G>([&](auto G) {
              constexpr int u0 = decltype(G)::value * EPI_G;
              constexpr int n = EPI_IT - u0 < EPI_G ? EPI_IT - u0 : EPI_G;
              if (u0 == it) {
                bx_u32x4 grp[n];
                bx_ds_read128_sync<u0 * RPP * LDE * 2, RPP * LDE * 2, n>(rbase, grp);
#pragma unroll
                for (int v = 0; v < n; ++v) dvs[u0 + v] = grp[v];
              }
            });
          }
          const int row = tid / OCPR + it * RPP;  // row within the half
          const int lr = half * EH + row;
          const bool act = (tid < RPP * OCPR) & (row < EH);
          const bx_u32x4 dw = dvs[it];
          const uint4 dv = {dw.x, dw.y, dw.z, dw.w};
          uint32_t yo;
          long long grow;  // global output row
          if constexpr (KS == 133) {
            grow = ti.m0 + lr;
            yo = (act && grow < p.M) ? (uint32_t)(lr * p.ldy * 2) : 0x80000000u;
          } else {
            const int t = (int)fdiv((uint32_t)lr, g.fP), j = lr - t * g.P;
            grow = (long long)(ti.b * p.T + t) * g.HW + ti.p0 + j;
            yo = (act && t < p.T && ti.p0 + j < g.HW) ? (uint32_t)(((long long)t * g.HW + ti.p0 + j) * p.ldy * 2)
                                          : 0x80000000u;
          }
          const int n = n0 + cc * 8;
          const bool ok = (yo != 0x80000000u) & (n < p.Cout) & !(BOX_ABLATE & 4);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int, dv),
                                                 yrs, (ok && !(BOX_ABLATE & 16)) ? yo + (uint32_t)n * 2 : 0x80000000u,
                                                 0, 0);
          if constexpr (EPI == 1) {
            if (ok && !(BOX_ABLATE & 32)) {
              float d8[8];
              unpack8(dv, d8);
#pragma unroll
              for (int k = 0; k < 8; ++k) { e_s[k] += d8[k]; e_q[k] += d8[k] * d8[k]; }
            }
          }
          if constexpr (EPI == 2) {
            if (ok) {
              float d8[8], y8[8];
              unpack8(dv, d8);
              unpack8(ypre[it], y8);
#pragma unroll
              for (int k = 0; k < 8; ++k) {
                const int cl = cc * 8 + k;
                const float gm = (y8[k] * ss_lds[2 * BN + cl] + ss_lds[3 * BN + cl] > 0.f) ? d8[k] : 0.f;
                e_s[k] += gm;
                e_q[k] += gm * (y8[k] - ss_lds[cl]) * ss_lds[BN + cl];
              }
            }
          }
        }
      }
      tev();  // H2: the half's stores issued
      lds_barrier();  // the half's rows are consumed before the region is rewritten
      tev();  // H3
    }
    if constexpr ((BOX_ABLATE & 8) != 0) {
      lds_barrier();
      fire((gs + STG - 1) % STG, (STG - 1) % nst_tile);
    }
    // the next tile's first box (its loads were issued at the last block's first tap)
    if (has_next) box_store(0, tn, zrs);
    tev();  // N: next tile's box written

    if (!has_next) break;
    m_tile = next_tile;
    ti = tn;
    first_tile = false;
  }
  // drain: the trailing fires of the last tile and the epilogue stores
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr (BOX_TRACE != 0) {
    tev();  // end
    if (g.trace != nullptr && blockIdx.x < 64) {
      uint32_t* tb = g.trace + ((size_t)blockIdx.x * NWAVES + wave) * 130;
      tb[lane] = tr_v0;
      tb[64 + lane] = tr_v1;
      if (lane == 0) { tb[128] = (uint32_t)tr_n; tb[129] = (uint32_t)ncb; }
    }
  }
  if constexpr (EPI != 0) {
    // per-thread column sums -> per column chunk over the row groups (fixed order)
    __syncthreads();
    float* red = (float*)smem;  // [2][8][NT] over the box region
#pragma unroll
    for (int k = 0; k < 8; ++k) { red[k * NT + tid] = e_s[k]; red[(8 + k) * NT + tid] = e_q[k]; }
    __syncthreads();
    if (tid < OCPR) {
      const int npad = p.num_n_tiles * BN;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float s1 = 0.f, s2 = 0.f;
        for (int j = tid; j < RPP * OCPR; j += OCPR) { s1 += red[k * NT + j]; s2 += red[(8 + k) * NT + j]; }
        const int col = n0 + tid * 8 + k;
        p.stats[(long long)m_slot * 2 * npad + col] = s1;
        p.stats[(long long)m_slot * 2 * npad + npad + col] = s2;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
static int box_geo(const ConvParams& p, BoxGeo& g, int& ntiles, int nw) {
  const int BM = nw * 32, BXR = box_rows(p.KT * 100 + p.KH * 10 + p.KW, nw);
  const int ks = p.KT * 100 + p.KH * 10 + p.KW;
  if (p.st != 1 || p.sh != 1 || p.sw != 1) return V4_UNSUPPORTED;
  if (p.To != p.T || p.Ho != p.H || p.Wo != p.W) return V4_UNSUPPORTED;
  // a partial last channel block reads weight columns past its tap's (times zero activations):
  // the last tap's must stay inside the packed row (the SGPR stage offset is not range-checked)
  const int ncb = (p.Cin + BX_BK - 1) / BX_BK;
  if (p.Cin % 8 || p.Kpad < (p.KT * p.KH * p.KW - 1) * p.Cin + ncb * BX_BK) return V4_UNSUPPORTED;
  g.KS = ks;
  g.HW = p.H * p.W;
  g.fHW = make_fastdiv(g.HW);
  g.fW = make_fastdiv(p.W);
  if (ks == 133) {
    if (p.pt != 0 || p.ph != 1 || p.pw != 1) return V4_UNSUPPORTED;
    g.W1 = p.W + 1;
    g.PL = (p.H + 1) * g.W1;
    g.fPL = make_fastdiv(g.PL);
    g.fW1 = make_fastdiv(g.W1);
    g.P = g.tpc = 1;
    g.ftpc = g.fP = make_fastdiv(1);
    // box rows of the widest tile: extended span of BM output rows + one pad row and column on
    // each side (bounded by the worst alignment: a tile starting at a plane's last column)
    // e(m + BM - 1) - e(m) = BM - 1 + (row wraps) + (W + 2) (plane wraps): a row wrap skips the
    // shared pad column, a plane wrap also the shared pad row
    const long long span =
        (BM - 1) + ((BM - 1) / p.W + 1) + ((BM - 1) / g.HW + 1) * (long long)(p.W + 2) + 2 * g.W1 + 3;
    if (span > BXR) return V4_UNSUPPORTED;
    ntiles = (p.M + BM - 1) / BM;
  } else if (ks == 311) {
    if (p.pt != 1 || p.ph != 0 || p.pw != 0) return V4_UNSUPPORTED;
    // P positions of every frame per tile, T * P <= BM output rows (8 waves, T = 2: P = 112, the
    // last 32 rows of the tile idle) and (T + 2) * P box rows
    if (p.T < 1) return V4_UNSUPPORTED;
    g.P = std::min(BM / p.T, BXR / (p.T + 2));
    if (g.P < 1) return V4_UNSUPPORTED;
    g.fP = make_fastdiv(g.P);
    g.tpc = (g.HW + g.P - 1) / g.P;
    g.ftpc = make_fastdiv(g.tpc);
    g.W1 = g.PL = 1;
    g.fPL = g.fW1 = make_fastdiv(1);
    ntiles = (p.M / (p.T * g.HW)) * g.tpc;
  } else {
    return V4_UNSUPPORTED;
  }
  return 0;
}

// N tile a box variant runs for the plan's N tile bn (0: none). 4-wave 16x16x32 (impl 16) runs a
// 192-wide plan as two 96-wide N tiles (its 192-row weight stages do not fit 80 KiB next to a box).
static int box_bn(int bn, int impl) {
  switch (impl) {
    case 14: return (bn == 64 || bn == 96 || bn == 128 || bn == 160) ? bn : 0;
    case 15: return (bn == 64 || bn == 128 || bn == 192) ? bn : 0;
    case 16: return (bn == 64 || bn == 96 || bn == 128 || bn == 160) ? bn : bn == 192 ? 96 : 0;
    case 17: return (bn == 64 || bn == 128 || bn == 192) ? bn : 0;
  }
  return 0;
}
static int box_nw(int impl) { return impl >= 16 ? 4 : 8; }

bool fwd_box_supported(const ConvParams& p, int bn, int impl) {
  BoxGeo g;
  int nt;
  if (box_bn(bn, impl) == 0) return false;
  return box_geo(p, g, nt, box_nw(impl)) == 0;
}

template <int BN, int KS, int EPI, int PRO, int MF, int NW>
static int launch_box_t(ConvParams& p, const BoxGeo& g, hipStream_t stream) {
  constexpr int BNR = (BN + 8 * NW - 1) / (8 * NW) * (8 * NW);
  constexpr size_t base = (size_t)box_rows(KS, NW) * 80 * 2 + (size_t)box_stages(BN, KS, NW) * BNR * BX_BK * 2 +
                          (EPI == 2 ? 16 * BN + 256 : EPI == 1 ? 4 * BN : 0);
  if constexpr (base > (size_t)box_lds_limit(NW)) {  // (no kernel instance for a shape that never fits)
    return V4_UNSUPPORTED;
  } else {
    const size_t lds = base + (PRO == 3 ? 28 * (size_t)p.Cin : PRO ? 8 * (size_t)p.Cin : 0);
    if (lds > (size_t)box_lds_limit(NW)) return V4_UNSUPPORTED;
    static bool attr_set = false;
    if (!attr_set) {
      HIP_RET(hipFuncSetAttribute((const void*)conv_box_kernel<BN, KS, EPI, PRO, MF, NW>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, box_lds_limit(NW)));
      attr_set = true;
    }
    const int nblocks = p.num_n_tiles * p.grid_m;
    hipLaunchKernelGGL((conv_box_kernel<BN, KS, EPI, PRO, MF, NW>), dim3(nblocks), dim3(NW * 64), lds, stream, p, g);
    return (int)hipGetLastError();
  }
}

template <int BN, int KS, int MF, int NW>
static int launch_box_epi(ConvParams& p, const BoxGeo& g, hipStream_t stream) {
  if (g.pro_y != nullptr) {  // BN-backward prologue (dgrad), dy written as the by-product
    if constexpr (BN <= 128) {
      if (g.pro_ss == nullptr || g.pro_coef == nullptr || g.pro_z == nullptr) return V4_UNSUPPORTED;
      if (p.bn_mode == 0) return launch_box_t<BN, KS, 0, 3, MF, NW>(p, g, stream);
      if (p.bn_mode == 2) return launch_box_t<BN, KS, 2, 3, MF, NW>(p, g, stream);
    }
    return V4_UNSUPPORTED;
  }
  if (g.pro_ss != nullptr && g.pro_z != nullptr) {
    if (p.bn_mode == 0) return launch_box_t<BN, KS, 0, 2, MF, NW>(p, g, stream);
    if (p.bn_mode == 1) return launch_box_t<BN, KS, 1, 2, MF, NW>(p, g, stream);
    return V4_UNSUPPORTED;
  }
  if (g.pro_ss != nullptr) {
    if (p.bn_mode == 0) return launch_box_t<BN, KS, 0, 1, MF, NW>(p, g, stream);
    if (p.bn_mode == 1) return launch_box_t<BN, KS, 1, 1, MF, NW>(p, g, stream);
    return V4_UNSUPPORTED;
  }
  if (p.bn_mode == 0) return launch_box_t<BN, KS, 0, 0, MF, NW>(p, g, stream);
  if (p.bn_mode == 1) return launch_box_t<BN, KS, 1, 0, MF, NW>(p, g, stream);
  return launch_box_t<BN, KS, 2, 0, MF, NW>(p, g, stream);
}

template <int BN, int MF, int NW = 8>
static int launch_box_bn(ConvParams& p, const BoxGeo& g, hipStream_t stream) {
  if (g.KS == 133) return launch_box_epi<BN, 133, MF, NW>(p, g, stream);
  return launch_box_epi<BN, 311, MF, NW>(p, g, stream);
}

// impl 14: 16x16x32 MFMA (N tiles 64 / 96 / 128 / 160), 15: 32x32x16 (N tiles 64 / 128 / 192);
// 16 / 17: the same on 4-wave workgroups, two per CU (16: N tiles 64 / 96 / 128 / 160, a 192-wide
// plan as two 96 tiles; 17: 64 / 128 / 192), each within the 80 KiB LDS budget or unsupported
static uint32_t* g_box_trace = nullptr;
// BOX_TRACE builds: the buffer ([64 workgroups][8 waves][130] uint32) the next box launches record to
MILNCE_API int milnce_box_set_trace(void* buf) {
  g_box_trace = (uint32_t*)buf;
  return BOX_TRACE ? 0 : (int)hipErrorNotSupported;
}

int launch_fwd_box(ConvParams& p, int bn, int impl, const BoxPro& pro, hipStream_t stream) {
  BoxGeo g;
  g.trace = g_box_trace;
  int ntiles = 0;
  const int nw = box_nw(impl);
  const int bnx = box_bn(bn, impl);
  if (bnx == 0 || box_geo(p, g, ntiles, nw) != 0) return V4_UNSUPPORTED;
  if (bnx != bn) {  // sub-tiles of the plan's N tile (the packed weight's Npad is a multiple of both)
    const int npad = p.num_n_tiles * bn;
    if (npad % bnx) return V4_UNSUPPORTED;
    p.num_n_tiles = npad / bnx;
  }
  g.pro_ss = pro.ss;
  g.pro_z = (bf16_t*)pro.z;
  g.pro_y = (const bf16_t*)pro.y;
  g.pro_coef = pro.coef;
  g.xld = pro.xld > 0 ? pro.xld : p.Cin;

  g.zbytes = (long long)(p.M / (p.To * p.Ho * p.Wo)) * p.T * p.H * p.W * p.Cin * 2;
  if (g.xld != p.Cin) {
    if (g.xld < p.Cin || g.xld % 8) return V4_UNSUPPORTED;
    // x is a channel slice of a wider tensor: its last row ends Cin (not xld) elements in
    const long long rows = (long long)(p.M / (p.To * p.Ho * p.Wo)) * p.T * p.H * p.W;
    p.x_total_bytes = ((rows - 1) * g.xld + p.Cin) * 2;
  }
  p.num_m_tiles = ntiles;
  if (impl == 14) {
    if (bn == 64) return launch_box_bn<64, 16>(p, g, stream);
    if (bn == 96) return launch_box_bn<96, 16>(p, g, stream);
    if (bn == 128) return launch_box_bn<128, 16>(p, g, stream);
    if (bn == 160) return launch_box_bn<160, 16>(p, g, stream);
  } else if (impl == 15) {
    if (bn == 64) return launch_box_bn<64, 32>(p, g, stream);
    if (bn == 128) return launch_box_bn<128, 32>(p, g, stream);
    if (bn == 192) return launch_box_bn<192, 32>(p, g, stream);
  } else if (impl == 16) {
    if (bnx == 64) return launch_box_bn<64, 16, 4>(p, g, stream);
    if (bnx == 96) return launch_box_bn<96, 16, 4>(p, g, stream);
    if (bnx == 128) return launch_box_bn<128, 16, 4>(p, g, stream);
    if (bnx == 160) return launch_box_bn<160, 16, 4>(p, g, stream);
  } else if (impl == 17) {
    if (bnx == 64) return launch_box_bn<64, 32, 4>(p, g, stream);
    if (bnx == 128) return launch_box_bn<128, 32, 4>(p, g, stream);
    if (bnx == 192) return launch_box_bn<192, 32, 4>(p, g, stream);
  }
  return V4_UNSUPPORTED;
}
