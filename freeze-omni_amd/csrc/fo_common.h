// Shared helpers for the Freeze-Omni MI355X (gfx950) kernels.
// Everything here is CDNA4-only: 64-lane waves, bf16 MFMA, no portability layer.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fo_hip.h"

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef uint16_t bf16_t;  // raw bf16 storage

#define FO_WAVE 64

// ---------------------------------------------------------------- cross-workgroup hand-off
// Cross-workgroup hand-off without fences (MI355X_MICROARCH.md's sc1 hand-off table, first row): the producer stores
// write-through (st_wt: a relaxed agent-scope atomic store, `global_store ... sc1`, so the line leaves this XCD's L2
// without a release fence), drains its stores, and one lane takes an agent-scope ticket behind a workgroup barrier;
// the workgroup whose add came last reads the bytes back with sc1 buffer loads (ld_sc1: past its L1, from L2 or
// memory) after a workgroup barrier -- no buffer_wbl2 / buffer_inv.  Used with one workgroup per CU.
typedef __attribute__((address_space(1))) float g_f32;
__device__ __forceinline__ void st_wt(float* p, float v) {
  __hip_atomic_store((g_f32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void* base) {
  const unsigned long long b = (unsigned long long)base;
  return __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<void*>(((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(b >> 32)) << 32) |
                              (unsigned)__builtin_amdgcn_readfirstlane((unsigned)b)),
      (short)0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ float ld_sc1(__amdgpu_buffer_rsrc_t r, size_t off_floats) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (unsigned)(off_floats * 4), 0, 16));
}

// ---------------------------------------------------------------- error plumbing
// Every C-ABI entry returns 0 on success or a negative code; the message is kept
// per thread and read back with fo_last_error().
namespace fo {
void set_error(const char* fmt, ...);
int check_launch(const char* what);
// host-side launch counters per kernel family (include/fo_hip.h FoLaunchKind; fo_launch_counts): tests assert
// which kernel family a shape was routed to.  Counted when the launch is issued (a captured graph counts once,
// at capture).
void count_launch(int kind);
}  // namespace fo

#define FO_REQUIRE(cond, ...)            \
  do {                                   \
    if (!(cond)) {                       \
      fo::set_error(__VA_ARGS__);        \
      return -2;                         \
    }                                    \
  } while (0)

#define FO_HIP(call)                                                          \
  do {                                                                        \
    hipError_t e_ = (call);                                                   \
    if (e_ != hipSuccess) {                                                   \
      fo::set_error("%s failed: %s", #call, hipGetErrorString(e_));          \
      return -1;                                                              \
    }                                                                         \
  } while (0)

// ---------------------------------------------------------------- numeric helpers
__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}
// Packed fp32 activations for the <= 64-row GEMMs: element (m < 16 rbs, n) of an fp32 matrix as bf16 hi + lo (the
// split a GEMM would do on load: hi = bf16(v), lo = bf16(v - hi)) at its MFMA A-fragment position: k-step n / 32,
// row block m / 16, lane 16 (n % 32 / 8) + m % 16, element n % 8 of the lane's 8.
// With rbs = ceil(M / 16) row blocks (1..4) the k-step holds rbs fragments: [K/32][rbs][64][8] bf16 per half.
__device__ __forceinline__ void xpack_store(uint16_t* hp, uint16_t* lp, int m, int n, float v, int rbs = 1) {
  const int c = n & 31;
  const size_t o = ((size_t)(((n >> 5) * rbs + (m >> 4)) * 64 + ((c >> 3) << 4) + (m & 15))) * 8 + (c & 7);
  const __bf16 h = (__bf16)v;
  hp[o] = __builtin_bit_cast(uint16_t, h);
  lp[o] = __builtin_bit_cast(uint16_t, (__bf16)(v - (float)h));
}
// The same fragment order for an fp32 copy (a LayerNorm-on-load consumer needs the exact fp32 values): lane l of
// k-step ks, row block b holds its 8 floats contiguously at ((ks * rbs + b) * 64 + l) * 8.
__device__ __forceinline__ void xpack32_store(float* p, int m, int n, float v, int rbs) {
  const int c = n & 31;
  p[((size_t)(((n >> 5) * rbs + (m >> 4)) * 64 + ((c >> 3) << 4) + (m & 15))) * 8 + (c & 7)] = v;
}
// round-to-nearest-even f32 -> bf16 (NaN kept NaN)
__device__ __forceinline__ bf16_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x7fffffu)) return (bf16_t)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (bf16_t)(u >> 16);
}
__host__ __device__ __forceinline__ float round_f16(float f) {
  return (float)(_Float16)f;
}
// the value lane (lane ^ O) holds, O a power of two below 64, without an LDS round trip (ds_bpermute): the gfx950
// half-wave / row swaps for 32 and 16, DPP within the 16-lane row below (row_ror:8; row_shl:4 into banks 0 and 2 and
// row_shr:4 into banks 1 and 3; quad_perm for 2 and 1).  The whole wave must be active, as for __shfl_xor.
template <int CTRL, int BANK = 0xF>
__device__ __forceinline__ float dpp_mov(float old, float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, old), __builtin_bit_cast(int, v),
                                                               CTRL, 0xF, BANK, false));
}
template <int O>
__device__ __forceinline__ float lane_xor(float v) {
  static_assert(O == 1 || O == 2 || O == 4 || O == 8 || O == 16 || O == 32, "lane_xor: offset");
  if constexpr (O == 32 || O == 16) {
    const unsigned u = __builtin_bit_cast(unsigned, v);
    // {vdst, vsrc} after the swap: a lane of the lower half (row pair) finds its partner in vsrc, of the upper in vdst
    const auto r = O == 32 ? __builtin_amdgcn_permlane32_swap(u, u, false, false)
                           : __builtin_amdgcn_permlane16_swap(u, u, false, false);
    return __builtin_bit_cast(float, (threadIdx.x & O) ? r[0] : r[1]);
  } else if constexpr (O == 8) {
    return dpp_mov<0x128>(v, v);
  } else if constexpr (O == 4) {
    return dpp_mov<0x114, 0xA>(dpp_mov<0x104, 0x5>(v, v), v);
  } else if constexpr (O == 2) {
    return dpp_mov<0x4E>(v, v);
  } else {
    return dpp_mov<0xB1>(v, v);
  }
}
// butterflies over the wave in the order 32, 16, ..., 1 (the same operands in the same order as the __shfl_xor form)
__device__ __forceinline__ float wave_sum(float v) {
  v += lane_xor<32>(v);
  v += lane_xor<16>(v);
  v += lane_xor<8>(v);
  v += lane_xor<4>(v);
  v += lane_xor<2>(v);
  return v + lane_xor<1>(v);
}
__device__ __forceinline__ float wave_max(float v) {
  v = fmaxf(v, lane_xor<32>(v));
  v = fmaxf(v, lane_xor<16>(v));
  v = fmaxf(v, lane_xor<8>(v));
  v = fmaxf(v, lane_xor<4>(v));
  v = fmaxf(v, lane_xor<2>(v));
  return fmaxf(v, lane_xor<1>(v));
}
// block-wide sum for blockDim.x == 64*NW; lds must hold NW floats
template <int NW>
__device__ __forceinline__ float block_sum(float v, float* lds) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) lds[w] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NW; ++i) t += lds[i];
  return t;
}

enum FoAct { FO_ACT_NONE = 0, FO_ACT_RELU = 1, FO_ACT_SILU = 2, FO_ACT_GELU = 3, FO_ACT_SWIGLU = 4 };

__device__ __forceinline__ float apply_act(float v, int act) {
  switch (act) {
    case FO_ACT_RELU: return v > 0.f ? v : 0.f;
    case FO_ACT_SILU: return v / (1.f + expf(-v));
    case FO_ACT_GELU: return 0.5f * v * (1.f + erff(v * 0.70710678118654752f));
    default: return v;
  }
}

// ---------------------------------------------------------------- LDS-DMA by asm (k_gemm_rows, k_conv_cl)
// One 16-B-per-lane global -> LDS load the compiler does not see: its own wait placement treats an LDS-DMA as
// aliasing every later LDS read and drains all of them before each one, so these kernels count their DMA with
// explicit s_waitcnt instead (the guide's recipe: M0 saved, set, s_nop, load, restored in one statement).
template <bool NT = false>   // NT: the streaming (non-temporal) policy -- weights that must not evict X from L2
__device__ __forceinline__ void dma16(const void* gsrc, unsigned lds_byte) {
  unsigned keep;
  if constexpr (NT)
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(gsrc), "s"(lds_byte)
                 : "memory");
  else
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(gsrc), "s"(lds_byte)
                 : "memory");
}
template <typename T>
__device__ __forceinline__ unsigned lds_addr(T* p) {
  return (unsigned)(size_t)((__attribute__((address_space(3))) char*)(p));
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}
