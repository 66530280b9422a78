// Shared helpers for the MI355X (gfx950 / CDNA4) kernels of libmilnce_hip.so.
// All kernels are written for wave64 and the gfx950 MFMA / LDS model; nothing here is
// portable to other targets on purpose.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#define MILNCE_API extern "C" __attribute__((visibility("default")))

typedef uint16_t bf16_t;  // raw bf16 storage
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));

#define LDS_PTR(p) ((__attribute__((address_space(3))) void*)(p))

// Kernel invariant checks, compiled in only by the checking build (python csrc/build.py --check,
// -DMILNCE_KCHECK, loaded with MILNCE_LIB_PATH=.../libmilnce_hip_check.so): a failed check prints
// the condition and traps the wave, so an out-of-range tile / index shows up at its source
// instead of as a silently dropped (out-of-range buffer) access or a later fault.
#ifdef MILNCE_KCHECK
#define KASSERT(cond)                                                                              \
  do {                                                                                             \
    if (!(cond)) {                                                                                 \
      printf("KASSERT failed %s:%d block %d thread %d: %s\n", __FILE__, __LINE__, (int)blockIdx.x, \
             (int)threadIdx.x, #cond);                                                             \
      __builtin_trap();                                                                            \
    }                                                                                              \
  } while (0)
#else
#define KASSERT(cond) \
  do {                \
  } while (0)
#endif

__device__ __forceinline__ float bf2f(uint16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

__device__ __forceinline__ uint16_t f2bf(float f) {
  __bf16 h = (__bf16)f;  // lowers to v_cvt_pk_bf16_f32 (RNE, NaN-preserving) on gfx950
  return __builtin_bit_cast(uint16_t, h);
}

// Two floats -> a packed bf16 pair in ONE v_cvt_pk_bf16_f32 (RNE, same bits as two f2bf): the
// scalar form compiles to two converts plus a shift and an OR, i.e. 4 VALU per pair in every
// epilogue and streaming kernel.
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack2bf(float a, float b) {
  const f32x2_t f = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f, bf16x2_t));
}

// Unpack 8 bf16 held in a uint4 to floats.
__device__ __forceinline__ void unpack8(const uint4& v, float* f) {
  f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
  f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
  f[4] = __uint_as_float(v.z << 16); f[5] = __uint_as_float(v.z & 0xffff0000u);
  f[6] = __uint_as_float(v.w << 16); f[7] = __uint_as_float(v.w & 0xffff0000u);
}

__device__ __forceinline__ uint4 pack8(const float* f) {
  uint4 v;
  v.x = pack2bf(f[0], f[1]); v.y = pack2bf(f[2], f[3]);
  v.z = pack2bf(f[4], f[5]); v.w = pack2bf(f[6], f[7]);
  return v;
}

// Train-mode BN backward of one element: dy = k0 (dz mask - k1 - xhat k2), xhat = (y - mean) istd,
// mask = (y scale + shift > 0), folded per channel to  dy = mask ? k0 dz + c : c,  c = c1 y + c0,
// c1 = -k0 istd k2, c0 = k0 (mean istd k2 - k1): 5 VALU ops instead of 8, explicit fmas so every
// site (fused prologues, streaming passes, pool gathers) rounds identically.
struct BnBwdC {
  float s, h, c1, c0, k0;
};
__device__ __forceinline__ BnBwdC bn_bwd_const(float mean, float istd, float scale, float shift, float k0, float k1,
                                               float k2) {
  BnBwdC q;
  const float a = istd * k2;
  q.s = scale;
  q.h = shift;
  q.k0 = k0;
  q.c1 = -k0 * a;
  q.c0 = k0 * fmaf(mean, a, -k1);
  return q;
}
__device__ __forceinline__ float bn_bwd_elem(float dz, float y, const BnBwdC& q) {
  const float c = fmaf(y, q.c1, q.c0);
  return fmaf(y, q.s, q.h) > 0.f ? fmaf(dz, q.k0, c) : c;
}

// Fast unsigned division by a runtime-invariant divisor (dividend < 2^31).
struct FastDiv {
  uint32_t d, mul, shr;
};

static inline FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d;
  if (d == 1) { f.mul = 0; f.shr = 0; return f; }
  uint32_t l = 0;
  while ((1u << l) < d) ++l;  // ceil(log2 d)
  uint32_t p = 31 + l;
  uint64_t m = ((1ull << p) + d - 1) / d;
  f.mul = (uint32_t)m;
  f.shr = p - 32;
  return f;
}

__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
  return f.d == 1 ? n : (__umulhi(n, f.mul) >> f.shr);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// XCD-aware bijective remap of a 1-D block id (cdna_hip_programming.md §5, T1): blocks that
// the dispatcher deals to the same XCD (id % 8 equal) get a contiguous range of logical ids.
__device__ __forceinline__ int xcd_remap(int id, int nblocks) {
  const int q = nblocks / 8, r = nblocks % 8;
  const int xcd = id % 8, slot = id / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
}

// Workgroup barrier that orders LDS only: waits for this wave's LDS ops (lgkmcnt(0)) and
// s_barrier, with a compiler memory clobber. Unlike __syncthreads() it does not drain
// outstanding global loads (vmcnt), so register prefetches stay in flight across it.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Host: split count of a persistent kernel whose ntiles x splits workgroups share a box range
// equally: at most `target` workgroups (floor), so no last round of a few workgroups that each run a
// full share while the rest of the chip idles (the ceil overshoot by up to ntiles - 1 workgroups
// doubled or added a third round to the temporal / halo wgrads at their one-workgroup-per-CU
// residency). MILNCE_SPLIT_CEIL=1 restores the rounded-up count (A/B).
static inline long long fill_splits(long long target, long long ntiles) {
  static int ceil_mode = -1;
  if (ceil_mode < 0) {
    const char* e = getenv("MILNCE_SPLIT_CEIL");
    ceil_mode = (e != nullptr && e[0] == '1') ? 1 : 0;
  }
  const long long s = ceil_mode ? (target + ntiles - 1) / ntiles : target / ntiles;
  return s < 1 ? 1 : s;
}

// Host: device scratch (floats) for kernels that stage partial results between launches of ONE
// API call -- one growing buffer per (purpose slot, stream, device), so reuse is ordered by the
// stream. Growth synchronises that stream before freeing the old buffer. Per translation unit.
// Returns null while the stream is being captured into a HIP graph (callers then fall back).
enum ScratchSlot { SCRATCH_BN_PRE = 0, SCRATCH_BN_GSUM = 1, SCRATCH_GATE_GSUM = 2, SCRATCH_GATE_DG = 3,
                   SCRATCH_GATE_DOT = 4, SCRATCH_POOL_GS = 5, SCRATCH_SLOTS = 6 };
static inline float* stream_scratch(size_t floats, hipStream_t stream, int slot) {
  struct Buf {
    hipStream_t stream;
    int device, slot;
    float* buf;
    size_t cap;
  };
  static Buf bufs[64];
  static int nbuf = 0;
  // never inside a HIP graph capture: no allocation is allowed there, and a later growth would
  // free memory a captured graph still references -- the callers fall back to atomics
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(stream, &cap) != hipSuccess || cap != hipStreamCaptureStatusNone) return nullptr;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  Buf* e = nullptr;
  for (int i = 0; i < nbuf; ++i)
    if (bufs[i].stream == stream && bufs[i].device == dev && bufs[i].slot == slot) e = &bufs[i];
  if (e == nullptr) {
    if (nbuf == 64) return nullptr;
    e = &bufs[nbuf++];
    *e = Buf{stream, dev, slot, nullptr, 0};
  }
  if (e->cap < floats) {
    if (e->buf != nullptr && (hipStreamSynchronize(stream) != hipSuccess || hipFree(e->buf) != hipSuccess))
      return nullptr;
    e->buf = nullptr;
    e->cap = 0;
    if (hipMalloc(&e->buf, floats * sizeof(float)) != hipSuccess) return nullptr;
    e->cap = floats;
  }
  return e->buf;
}

// Minimum LDS bytes per workgroup of the weight-gradient launches (milnce_set_lds_floor; 0 = off):
// the side-stream wgrads are launched with extra dynamic LDS so that fewer of their workgroups share
// a CU, leaving LDS for the main chain's kernels (a CU whose LDS the wgrads filled cannot start any
// workgroup that needs LDS, e.g. a BN finalize or a pool backward: it waits for a wgrad workgroup
// to retire). Defined in conv.hip.
extern int g_milnce_lds_floor;
template <typename K>
static inline size_t lds_floor(K kernel, size_t dyn) {
  if (g_milnce_lds_floor <= 0) return dyn;
  hipFuncAttributes a;
  if (hipFuncGetAttributes(&a, (const void*)kernel) != hipSuccess) return dyn;
  const size_t total = a.sharedSizeBytes + dyn, floor = (size_t)g_milnce_lds_floor;
  if (total >= floor || floor > 160 * 1024) return dyn;
  const size_t want = dyn + (floor - total);
  if (want > 64 * 1024 &&
      hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)(160 * 1024 - a.sharedSizeBytes)) != hipSuccess)
    return dyn;
  return want;
}

#define HIP_RET(expr)                           \
  do {                                          \
    hipError_t _e = (expr);                     \
    if (_e != hipSuccess) return (int)_e;       \
  } while (0)
