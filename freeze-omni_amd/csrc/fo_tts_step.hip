// One AR speech-decoder step as ONE persistent kernel (fo_tts_step).
//
// Reference: LLM2TTSCodecAR.infer's loop body (models/decoder/decoder.py:341-367): embed(id) -> Llama layers
// (LlamaRMSNorm, q|k|v, RoPE, eager attention over the cache, o, RMSNorm, SwiGLU MLP) -> norm -> out_fnn ->
// [repetition penalty, :348-351] -> top-k multinomial draw.  The multi-kernel step (fo/stack.py +
// fo_sample_embed) spends ~27 launches of ~5-7 us each on ~130 MB of Infinity-Cache-resident weights at
// 8 rows; here every launch boundary becomes a device-wide barrier, and each workgroup issues the weight
// loads of its NEXT phase before it waits there, so the weight latency hides behind the barrier.
//
// Layout: G workgroups (one per CU) x 256 threads.  Activations are [16][D] fp32 rows (B <= 16 sessions;
// rows >= B are zero in the MFMA operands) and stay in L2; every phase that needs a normalised row
// recomputes the row sum of squares itself from the residual + the previous phase's partial sums, so no
// statistics plumbing crosses phases:
//   QKV(l):  R0 = xa (l = 0) | xb + sum_s dpart[s] (written back to xa); h = RMSNorm(R0) * ln1;
//            tile pair u = g of q|k|v (rope-paired packing), K = D; RoPE + paged KV append in the epilogue.
//   ATTN(l): item (b, h, s) = g: keys [s L/S, (s+1) L/S) of session b, head h -> (max, sum, sum p v).
//   O(l):    tile t = g, whole K: the attention rows are combined from the split partials as they are
//            staged; xb[:, tile] = R1 = xa + o (the residual added in the epilogue).
//   GU(l):   RMSNorm(xb) * ln2; gate/up tile pairs g, g + G; m = silu(gate) * up.
//   DOWN(l): job (tile t, K part p) = g: m[:, part p] -> dpart[p].
//   OUT:     R = xb + sum dpart; final norm; out_fnn tile g (+ bias) -> logits.
//   DRAW:    row g < B: penalty ring, top-k draw (fo_sample's small-k path, same RNG stream), history,
//            xa[g] = emb[id] (the next step's input).
// MFMA: mfma_f32_16x16x32_bf16 with the fp32 activations split into bf16 hi + lo (two MFMAs per weight
// fragment), as everywhere in the library.
#include <algorithm>

#include "fo_common.h"
#include "fo_hip.h"

namespace {

constexpr int TS_T = 256, TS_W = 4;  // threads, waves per workgroup
constexpr int TS_KW = 10;            // max k-steps per wave of one tile job (prefetch registers)
constexpr int TS_XKS = 40;           // max k-steps of X staged in LDS
constexpr int TS_KEYS = 1024;        // max keys per attention split
constexpr int TS_SD = 2;             // down-projection K parts (o takes the whole K and adds the residual)
constexpr int TS_KMAX = 64;          // largest top-k of the draw

struct SmemGemm {
  bf16x8 xh[TS_XKS][64];
  bf16x8 xl[TS_XKS][64];
  float red[TS_W][2][16][17];
  float misc[64];
};
struct SmemAttn {
  float q[64];
  float s[TS_KEYS];
  float acc[TS_W][64];
  float red[TS_W];
};
struct SmemDraw {
  float bv[TS_T];
  int bi[TS_T];
  int taken[TS_KMAX];
  float tv[TS_KMAX];
  int si[2];
};
union TsSmem {
  SmemGemm g;
  SmemAttn at;
  SmemDraw dr;
};

__device__ __forceinline__ uint64_t ts_smix(uint64_t x) {  // fo_sample.hip's stream mixer
  x += 0x9E3779B97F4A7C15ull;
  uint64_t z = x;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

typedef __attribute__((address_space(1))) unsigned ts_gu32;
typedef __attribute__((address_space(1))) float ts_gf32;
// Every value another workgroup reads after a barrier is stored write-through (sc1: a relaxed agent-scope
// atomic store), so the barrier needs no L2 write-back (release fence): each storing wave only drains its
// stores before the workgroup's ticket.  Readers acquire once per barrier (L1 invalidate) and load plainly.
__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store((ts_gf32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// ...and every load of such a value is an sc1 buffer load (past this CU's L1), so the barrier needs no
// acquire either.  One buffer descriptor per array (wave-uniform base), per-lane byte offsets.
typedef __amdgpu_buffer_rsrc_t TsRs;
__device__ __forceinline__ TsRs rs_of(const void* base) {
  const unsigned long long b = (unsigned long long)base;
  return __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<void*>(((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(b >> 32)) << 32) |
                              (unsigned)__builtin_amdgcn_readfirstlane((unsigned)b)),
      (short)0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ float4 ld4(TsRs r, size_t off_floats) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, (unsigned)(off_floats * 4), 0, 16));
}
__device__ __forceinline__ float ld1(TsRs r, size_t off_floats) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (unsigned)(off_floats * 4), 0, 16));
}

// Device-wide barrier, monotonic within a launch: workgroup g arrives on the counter of its dispatch
// group x = g % 8 (one cache line each), the last arrival of a group on the top counter, the last group
// raises the epoch word; lane 0 of wave 0 polls it with a bounded, sleeping spin.  Every wave drains its
// own (write-through) stores (s_waitcnt vmcnt(0)) before the workgroup barrier, lane 0 takes the ticket;
// every handed-off value is read back with sc1 loads, so no acquire fence (the sc1 form of the in-launch
// hand-off).  Waves 1-3 then issue their next-phase weight loads (pf), which stay in flight across the wait.
struct TsBar {
  unsigned* w;  // [0]: top counter, [16 * (1 + x)]: group counters, [16 * 9]: epoch word, [16 * 10]: exit
  unsigned epoch;
  int G;
  int* err;
  unsigned long long* trace;  // [G][64] or null: wall clock at start (0), arrival (1 + 2 e) and exit (2 + 2 e) of
                              // barrier e, end (63)
};
template <typename PF>
__device__ __forceinline__ void ts_barrier(TsBar& b, PF&& pf) {
  if (b.trace && threadIdx.x == 0 && b.epoch < 30) b.trace[blockIdx.x * 64 + 1 + 2 * b.epoch] = wall_clock64();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): LDS reads of this phase are done before reuse
  __builtin_amdgcn_s_barrier();
  b.epoch += 1;
  const int wave = threadIdx.x >> 6;
  if (wave != 0) pf();
  if (threadIdx.x == 0) {
    const int x = blockIdx.x & 7;
    const unsigned nx = (unsigned)((b.G - x + 7) / 8);
    const unsigned ngroups = (unsigned)(b.G < 8 ? b.G : 8);
    const unsigned t = __hip_atomic_fetch_add((ts_gu32*)(b.w + 16 * (1 + x)), 1u, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
    if (t + 1 == nx * b.epoch) {
      const unsigned t2 = __hip_atomic_fetch_add((ts_gu32*)b.w, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (t2 + 1 == ngroups * b.epoch)
        __hip_atomic_store((ts_gu32*)(b.w + 16 * 9), b.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (threadIdx.x == 0) {
    unsigned spins = 0;
    while (__hip_atomic_load((ts_gu32*)(b.w + 16 * 9), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < b.epoch) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1u << 24)) {  // ~seconds: a workgroup never arrived; give up, flag it, never hang
        __hip_atomic_store((ts_gu32*)b.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the loads below the poll
    if (b.trace && b.epoch <= 30) b.trace[blockIdx.x * 64 + 2 * b.epoch] = wall_clock64();
  }
  if (wave == 0) pf();  // after the poll: its loads would sit ahead of every poll in the in-order vmcnt
  // raw barrier: the waves wait for lane 0's acquire, not for wave 0's prefetch to land
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
// The last workgroup to leave re-arms the barrier words for the next launch (nobody reads them after
// its own exit ticket).
__device__ __forceinline__ void ts_exit(TsBar& b) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add((ts_gu32*)(b.w + 16 * 10), 1u, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
    if (t + 1 == (unsigned)b.G) {
      for (int i = 0; i <= 10; ++i)
        __hip_atomic_store((ts_gu32*)(b.w + 16 * i), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ---------------------------------------------------------------- tile jobs
// A job = up to two 16-column tiles x nk k-steps starting at kb of a packed weight [tiles][KS][64][8];
// wave w owns k-steps w, w + 4, ...  Loads are unconditional (indices clamped into the job) so the
// compiler's in-order vmcnt accounting stays exact; the MFMAs skip the clamped steps.
struct TsJob {
  const bf16_t* W;
  int KS, t0, nt, kb, nk;
};
__device__ __forceinline__ void job_load(bf16x8 (&w)[2][TS_KW], const TsJob& j) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (!j.W) return;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int tile = j.t0 + (t < j.nt ? t : j.nt - 1);
#pragma unroll
    for (int i = 0; i < TS_KW; ++i) {
      const int ks = min(wave + TS_W * i, j.nk - 1);
      w[t][i] = *reinterpret_cast<const bf16x8*>(j.W + (((size_t)tile * j.KS + j.kb + ks) * 64 + lane) * 8);
    }
  }
}
// acc[t] += X (staged hi/lo, k-step ks of the job at LDS step xo + ks) . W tile t
__device__ __forceinline__ void job_mma(const bf16x8 (&w)[2][TS_KW], const TsJob& j, const SmemGemm& sg, int xo,
                                        f32x4 (&acc)[2]) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int i = 0; i < TS_KW; ++i) {
    const int ks = wave + TS_W * i;
    if (ks >= j.nk) break;
    const bf16x8 hi = sg.xh[xo + ks][lane], lo = sg.xl[xo + ks][lane];
    acc[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(hi, w[0][i], acc[0], 0, 0, 0);
    acc[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(lo, w[0][i], acc[0], 0, 0, 0);
    if (j.nt > 1) {
      acc[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(hi, w[1][i], acc[1], 0, 0, 0);
      acc[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(lo, w[1][i], acc[1], 0, 0, 0);
    }
  }
}
// wave partials -> red[0][t][row][col] summed over the waves (D layout: row 4*(lane>>4)+i, col lane&15)
__device__ __forceinline__ void job_reduce(SmemGemm& sg, const f32x4 (&acc)[2]) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) sg.red[wave][t][4 * (lane >> 4) + i][lane & 15] = acc[t][i];
  __syncthreads();
  const int r = threadIdx.x >> 4, c = threadIdx.x & 15;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < TS_W; ++w) v += sg.red[w][t][r][c];
    sg.red[0][t][r][c] = v;  // each (t, r, c) is read and written by one thread only
  }
  __syncthreads();
}

__device__ __forceinline__ void split_store(SmemGemm& sg, int ks, int lane, const float (&f)[8]) {
  bf16x8 hi, lo;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const __bf16 h = (__bf16)f[e];
    hi[e] = h;
    lo[e] = (__bf16)(f[e] - (float)h);
  }
  sg.xh[ks][lane] = hi;
  sg.xl[ks][lane] = lo;
}

// Stage R * gamma, R = base + sum_{s < NP} parts[s] ([16][D] rows, part stride pst floats), as MFMA A
// fragments of all D / 32 k-steps, and rstd(row) = rsqrt(mean(R^2) + eps) into misc[16]: the RMSNorm is
// applied after the GEMM (acc * rstd, linear).  TPR = 16 threads per row when B > 8, else 32 (all threads
// busy); thread: row t / TPR, fragment slots q = t % TPR + TPR i (k-step q / 4, columns 8 (q % 4) ..).
// Four slots' loads are issued together (one memory round trip per pass, not per slot).  Slots with
// (row * D/8 + q) % G == g are written back (write-through) to wb when non-null.
template <int NP>
__device__ void stage_norm(SmemGemm& sg, const float* base, const float* parts, size_t pst, const float* gamma,
                           int B, int D, float eps, float* wb, int g, int G) {
  const int tpr = B > 8 ? 16 : 32;
  const int r = threadIdx.x / tpr, sub = threadIdx.x % tpr;
  const int nq = D / 8;  // slots per row
  const TsRs rb = rs_of(base), rp = rs_of(parts ? parts : base);
  float ss = 0.f;
  for (int q0 = 0; q0 < nq; q0 += 4 * tpr) {
    float4 x[4][NP + 1][2];
    float4 gm[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = q0 + sub + tpr * i;
      if (q < nq && r < B) {
        const size_t o = (size_t)r * D + 8 * q;
        x[i][0][0] = ld4(rb, o);
        x[i][0][1] = ld4(rb, o + 4);
#pragma unroll
        for (int s = 0; s < NP; ++s) {
          x[i][s + 1][0] = ld4(rp, s * pst + o);
          x[i][s + 1][1] = ld4(rp, s * pst + o + 4);
        }
        gm[i][0] = *reinterpret_cast<const float4*>(gamma + 8 * q);
        gm[i][1] = *reinterpret_cast<const float4*>(gamma + 8 * q + 4);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = q0 + sub + tpr * i;
      if (q >= nq) continue;
      float f[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (r < B) {
        float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s <= NP; ++s) {
          v[0] += x[i][s][0].x; v[1] += x[i][s][0].y; v[2] += x[i][s][0].z; v[3] += x[i][s][0].w;
          v[4] += x[i][s][1].x; v[5] += x[i][s][1].y; v[6] += x[i][s][1].z; v[7] += x[i][s][1].w;
        }
        if (wb && (r * nq + q) % G == g) {
          const size_t o = (size_t)r * D + 8 * q;
#pragma unroll
          for (int e = 0; e < 8; ++e) st_sc1(wb + o + e, v[e]);
        }
        const float gv[8] = {gm[i][0].x, gm[i][0].y, gm[i][0].z, gm[i][0].w,
                             gm[i][1].x, gm[i][1].y, gm[i][1].z, gm[i][1].w};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          ss += v[e] * v[e];
          f[e] = v[e] * gv[e];
        }
      }
      if (r < 16) split_store(sg, q >> 2, r + 16 * (q & 3), f);
    }
  }
  for (int o = tpr >> 1; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);  // the row's tpr threads
  if (sub == 0 && r < 16) sg.misc[r] = r < B ? rsqrtf(ss / (float)D + eps) : 0.f;
  if (B <= 8) {  // rows 8..15 are nobody's at 32 threads per row: zero their fragments
    const float z[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (threadIdx.x < 8) sg.misc[8 + threadIdx.x] = 0.f;
    for (int e = threadIdx.x; e < 8 * nq; e += TS_T) split_store(sg, (e % nq) >> 2, 8 + e / nq + 16 * ((e % nq) & 3), z);
  }
}

// Stage plain fp32 rows src[r][col0 + ...] (row stride ld) over nks k-steps (no norm); four items' loads
// issued together
__device__ void stage_plain(SmemGemm& sg, const float* src, int ld, int col0, int nks, int B) {
  const TsRs rs = rs_of(src);
  const int n = 16 * nks * 4;
  for (int e0 = 0; e0 < n; e0 += 4 * TS_T) {
    float4 x[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = e0 + threadIdx.x + TS_T * i;
      const int r = e / (nks * 4), q = e % (nks * 4);
      if (e < n && r < B) {
        const size_t o = (size_t)r * ld + col0 + 8 * q;
        x[i][0] = ld4(rs, o);
        x[i][1] = ld4(rs, o + 4);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = e0 + threadIdx.x + TS_T * i;
      if (e >= n) continue;
      const int r = e / (nks * 4), q = e % (nks * 4);
      float f[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (r < B) {
        f[0] = x[i][0].x; f[1] = x[i][0].y; f[2] = x[i][0].z; f[3] = x[i][0].w;
        f[4] = x[i][1].x; f[5] = x[i][1].y; f[6] = x[i][1].z; f[7] = x[i][1].w;
      }
      split_store(sg, q >> 2, r + 16 * (q & 3), f);
    }
  }
}

// Stage the attention output columns [col0, col0 + 32 nks) of every row, combining the S <= TS_SMAX key-split
// partials (max, sum, sum p v) of the heads they belong to: o = sum_s e^(m_s - M) o_s / sum_s e^(m_s - M) l_s.
// Two items' partial loads are issued together.
constexpr int TS_SMAX = 4;
__device__ void stage_att(SmemGemm& sg, const float* apart, int col0, int nks, int B, int H, int hd, int S) {
  const TsRs ra = rs_of(apart);
  const int n = 16 * nks * 4;
  for (int e0 = 0; e0 < n; e0 += 2 * TS_T) {
    float ml[2][TS_SMAX][2];
    float4 ov[2][TS_SMAX][2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int e = e0 + threadIdx.x + TS_T * i;
      const int r = e / (nks * 4), q = e % (nks * 4);
      if (e < n && r < B) {
        const int col = col0 + 8 * q, h = col / hd, d = col - h * hd;
        const size_t p = (size_t)(r * H + h) * S * (hd + 4);
#pragma unroll
        for (int s = 0; s < TS_SMAX; ++s) {
          if (s < S) {
            const size_t ps = p + s * (hd + 4);
            ml[i][s][0] = ld1(ra, ps);
            ml[i][s][1] = ld1(ra, ps + 1);
            ov[i][s][0] = ld4(ra, ps + 4 + d);
            ov[i][s][1] = ld4(ra, ps + 8 + d);
          }
        }
      }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int e = e0 + threadIdx.x + TS_T * i;
      if (e >= n) continue;
      const int r = e / (nks * 4), q = e % (nks * 4);
      float f[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (r < B) {
        float M = -INFINITY;
#pragma unroll
        for (int s = 0; s < TS_SMAX; ++s)
          if (s < S) M = fmaxf(M, ml[i][s][0]);
        float l = 0.f;
#pragma unroll
        for (int s = 0; s < TS_SMAX; ++s) {
          if (s < S) {
            const float wgt = ml[i][s][0] == -INFINITY ? 0.f : expf(ml[i][s][0] - M);
            l += wgt * ml[i][s][1];
            f[0] += wgt * ov[i][s][0].x; f[1] += wgt * ov[i][s][0].y; f[2] += wgt * ov[i][s][0].z;
            f[3] += wgt * ov[i][s][0].w; f[4] += wgt * ov[i][s][1].x; f[5] += wgt * ov[i][s][1].y;
            f[6] += wgt * ov[i][s][1].z; f[7] += wgt * ov[i][s][1].w;
          }
        }
        const float il = 1.f / l;
#pragma unroll
        for (int k = 0; k < 8; ++k) f[k] *= il;
      }
      split_store(sg, q >> 2, r + 16 * (q & 3), f);
    }
  }
}

// ---------------------------------------------------------------- the step
struct TsPtrs {  // scratch carve of a.ws
  float *xb, *q, *apart, *m, *dpart;
};

__global__ __launch_bounds__(TS_T) void k_tts_step(FoTtsStep a) {
  __shared__ TsSmem sm;
  const int g = blockIdx.x, G = gridDim.x;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int B = a.B, D = a.D, H = a.H, hd = a.hd, F = a.F;
  const int KSd = D / 32, KSf = F / 32;
  const size_t RD = (size_t)16 * D;
  TsPtrs P;
  P.xb = a.ws;
  P.q = P.xb + RD;
  P.apart = P.q + RD;
  P.m = P.apart + (size_t)16 * H * a.S * (hd + 4);
  P.dpart = P.m + (size_t)16 * F;
  TsBar bar{a.bar, 0u, G, a.err, a.trace};
  if (a.trace && tid == 0) a.trace[g * 64] = wall_clock64();
  float* xa = a.x;

  const int nqkv = 3 * D / 32;             // rope tile pairs of q|k|v
  const int nattn = B * H * a.S;
  const int nt_d = D / 16;                 // o / down output tiles
  const int nk_d = KSf / TS_SD;
  const int ngu = F / 16;                  // gate/up tile pairs
  const int nout = (a.V + 15) / 16;

  auto qkv_job = [&](int l) {
    return g < nqkv ? TsJob{(const bf16_t*)a.wqkv[l], KSd, 2 * g, 2, 0, KSd} : TsJob{nullptr, 0, 0, 0, 0, 0};
  };
  auto o_job = [&](int l) {
    return g < nt_d ? TsJob{(const bf16_t*)a.wo[l], KSd, g, 1, 0, KSd} : TsJob{nullptr, 0, 0, 0, 0, 0};
  };
  auto gu_job = [&](int l, int u) {
    return u < ngu ? TsJob{(const bf16_t*)a.wgu[l], KSd, 2 * u, 2, 0, KSd} : TsJob{nullptr, 0, 0, 0, 0, 0};
  };
  constexpr int DCH = 38;                  // down K part processed in chunks of <= DCH k-steps
  auto down_job = [&](int l) {             // (the first chunk: what the barrier prefetches)
    return g < nt_d * TS_SD ? TsJob{(const bf16_t*)a.wdown[l], KSf, g / TS_SD, 1, (g % TS_SD) * nk_d, min(DCH, nk_d)}
                            : TsJob{nullptr, 0, 0, 0, 0, 0};
  };
  auto out_job = [&]() {
    return g < nout ? TsJob{(const bf16_t*)a.wout, KSd, g, 1, 0, KSd} : TsJob{nullptr, 0, 0, 0, 0, 0};
  };

  bf16x8 w[2][TS_KW];
  {
    const TsJob j = qkv_job(0);
    job_load(w, j);
  }
  for (int l = 0; l < a.nl; ++l) {
    // ---------------- QKV: h = RMSNorm(R0) * ln1; q|k|v tile pair g; RoPE; q -> P.q, k/v -> cache
    {
      const TsJob j = qkv_job(l);
      if (j.W) {
        const bool tr = a.trace && l == 1 && tid == 0;  // sub-phase clocks of layer 1's q|k|v (profiling)
        if (l == 0) stage_norm<0>(sm.g, xa, nullptr, 0, a.ln1[l], B, D, a.eps, nullptr, g, nqkv);
        else stage_norm<TS_SD>(sm.g, P.xb, P.dpart, RD, a.ln1[l], B, D, a.eps, xa, g, nqkv);  // -> xa
        __syncthreads();
        if (tr) a.trace[g * 64 + 50] = wall_clock64();
        f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
        job_mma(w, j, sm.g, 0, acc);
        if (tr) a.trace[g * 64 + 51] = wall_clock64();
        job_reduce(sm.g, acc);
        if (tr) a.trace[g * 64 + 52] = wall_clock64();
        const int r = tid >> 4, c = tid & 15;
        if (r < B) {
          const int half = hd >> 1, per = hd >> 5;
          const int n = (g / per) * hd + (g % per) * 16 + c;  // rope_col: columns (n, n + hd/2) of head n / hd
          const int h = n / hd, i = n - h * hd;
          const float x1 = sm.g.red[0][0][r][c] * sm.g.misc[r], x2 = sm.g.red[0][1][r][c] * sm.g.misc[r];
          const int sl = a.tok_slot[r], page = sl / a.PS, off = sl - page * a.PS;
          if (h < 2 * H) {
            const int p = a.tok_pos[r];
            const float cs = a.cos_t[(size_t)p * half + i], sn = a.sin_t[(size_t)p * half + i];
            const float o1 = x1 * cs - x2 * sn, o2 = x2 * cs + x1 * sn;
            float* d = h < H ? P.q + (size_t)r * D + (size_t)h * hd
                             : a.kc[l] + (((size_t)page * H + (h - H)) * a.PS + off) * hd;
            st_sc1(d + i, o1);
            st_sc1(d + i + half, o2);
          } else {
            float* d = a.vc[l] + (((size_t)page * H + (h - 2 * H)) * a.PS + off) * hd;
            st_sc1(d + i, x1);
            st_sc1(d + i + half, x2);
          }
        }
        if (tr) a.trace[g * 64 + 53] = wall_clock64();
      }
      ts_barrier(bar, [] {});
    }
    // ---------------- ATTN: item (b, h, s) = g -> apart[(b H + h) S + s] = (max, sum, sum p v[hd])
    {
      if (g < nattn) {
        const int s = g % a.S, bh = g / a.S, b = bh / H, h = bh % H;
        const int L = a.tok_nvis[b];
        const int kps = (L + a.S - 1) / a.S;
        const int k0 = s * kps, k1 = min(L, k0 + kps);
        float* out = P.apart + (size_t)g * (hd + 4);  // (max, sum, -, -, sum p v[hd]): 16-B aligned rows
        if (kps > TS_KEYS) {  // host contract broken: poison rather than read past LDS
          if (tid < hd + 4) st_sc1(out + tid, NAN);
        } else if (k0 >= k1) {
          if (tid < hd + 4) st_sc1(out + tid, tid == 0 ? -INFINITY : 0.f);
        } else {
          const int* bt = a.block_table + (size_t)b * a.maxb;
          const size_t page_sz = (size_t)H * a.PS * hd, head_off = (size_t)h * a.PS * hd;
          const TsRs rk = rs_of(a.kc[l]), rv = rs_of(a.vc[l]), rq = rs_of(P.q);  // sc1: the new key is this launch's
          if (tid < hd) sm.at.q[tid] = ld1(rq, (size_t)b * D + (size_t)h * hd + tid) * a.scale;
          __syncthreads();
          float mx = -INFINITY;
          for (int j = k0 + tid; j < k1; j += TS_T) {
            const size_t kr = (size_t)bt[j / a.PS] * page_sz + head_off + (size_t)(j % a.PS) * hd;
            float sc = 0.f;
            for (int d = 0; d < hd; d += 4) {
              const float4 k4 = ld4(rk, kr + d);
              sc += sm.at.q[d] * k4.x + sm.at.q[d + 1] * k4.y + sm.at.q[d + 2] * k4.z + sm.at.q[d + 3] * k4.w;
            }
            sm.at.s[j - k0] = sc;
            mx = fmaxf(mx, sc);
          }
          mx = wave_max(mx);
          if (lane == 0) sm.at.red[wave] = mx;
          __syncthreads();
          mx = fmaxf(fmaxf(sm.at.red[0], sm.at.red[1]), fmaxf(sm.at.red[2], sm.at.red[3]));
          float sum = 0.f;
          for (int j = tid; j < k1 - k0; j += TS_T) {
            const float p = expf(sm.at.s[j] - mx);
            sm.at.s[j] = p;
            sum += p;
          }
          sum = block_sum<TS_W>(sum, sm.at.red);  // its barriers also publish s[]
          // P.V: hd/4 lanes per key (a float4 of the row each), 64/(hd/4) keys per wave, waves interleaved
          const int lpk = hd >> 2, kpw = 64 / lpk;
          const int sub = lane / lpk, l4 = lane % lpk;
          float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
          for (int j = k0 + wave * kpw + sub; j < k1; j += kpw * TS_W) {
            const float p = sm.at.s[j - k0];
            const float4 v = ld4(rv, (size_t)bt[j / a.PS] * page_sz + head_off + (size_t)(j % a.PS) * hd + 4 * l4);
            acc.x += p * v.x;
            acc.y += p * v.y;
            acc.z += p * v.z;
            acc.w += p * v.w;
          }
          for (int o = lpk; o < 64; o <<= 1) {
            acc.x += __shfl_xor(acc.x, o, 64);
            acc.y += __shfl_xor(acc.y, o, 64);
            acc.z += __shfl_xor(acc.z, o, 64);
            acc.w += __shfl_xor(acc.w, o, 64);
          }
          if (sub == 0) *reinterpret_cast<float4*>(&sm.at.acc[wave][4 * l4]) = acc;
          __syncthreads();
          if (tid < hd) {
            float o = 0.f;
#pragma unroll
            for (int w2 = 0; w2 < TS_W; ++w2) o += sm.at.acc[w2][tid];
            st_sc1(out + 4 + tid, o);
          }
          if (tid == 0) {
            st_sc1(out, mx);
            st_sc1(out + 1, sum);
          }
        }
      }
      const TsJob jn = o_job(l);
      ts_barrier(bar, [&] { job_load(w, jn); });
    }
    // ---------------- O: tile g, whole K: xb[:, tile] = xa[:, tile] + attention rows . Wo^T
    {
      const TsJob j = o_job(l);
      if (j.W) {
        const int r = tid >> 4, c = tid & 15;
        const float res = r < B ? ld1(rs_of(xa), (size_t)r * D + j.t0 * 16 + c) : 0.f;
        stage_att(sm.g, P.apart, 0, j.nk, B, H, hd, a.S);
        __syncthreads();
        f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
        job_mma(w, j, sm.g, 0, acc);
        job_reduce(sm.g, acc);
        if (r < B) st_sc1(P.xb + (size_t)r * D + j.t0 * 16 + c, res + sm.g.red[0][0][r][c]);
      }
      const TsJob jn = gu_job(l, g);
      ts_barrier(bar, [&] { job_load(w, jn); });
    }
    // ---------------- GU: RMSNorm(xb) * ln2 (post-scaled); pairs g, g + G -> m
    {
      if (g < ngu) {
        const bool tr = a.trace && l == 1 && tid == 0;
        stage_norm<0>(sm.g, P.xb, nullptr, 0, a.ln2[l], B, D, a.eps, nullptr, g, min(G, ngu));
        __syncthreads();
        if (tr) a.trace[g * 64 + 54] = wall_clock64();
        for (int u = g; u < ngu; u += G) {
          const TsJob j = gu_job(l, u);
          if (u != g) job_load(w, j);
          f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
          job_mma(w, j, sm.g, 0, acc);
          job_reduce(sm.g, acc);
          const int r = tid >> 4, c = tid & 15;
          const float gt = sm.g.red[0][0][r][c] * sm.g.misc[r], up = sm.g.red[0][1][r][c] * sm.g.misc[r];
          st_sc1(P.m + (size_t)r * F + u * 16 + c, r < B ? gt / (1.f + expf(-gt)) * up : 0.f);
          __syncthreads();  // red[] is rewritten by the next pair
          if (tr && u == g) a.trace[g * 64 + 55] = wall_clock64();
        }
        if (tr) a.trace[g * 64 + 56] = wall_clock64();
      }
      const TsJob jn = down_job(l);
      ts_barrier(bar, [&] { job_load(w, jn); });
    }
    // ---------------- DOWN: job (tile, K part) = g -> dpart[part][row][tile cols], in chunks of DCH k-steps
    {
      const TsJob j = down_job(l);
      if (j.W) {
        f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
        for (int c0 = 0; c0 < nk_d; c0 += DCH) {
          const TsJob jc{j.W, KSf, j.t0, 1, j.kb + c0, min(DCH, nk_d - c0)};
          if (c0 > 0) {
            job_load(w, jc);
            __syncthreads();  // the previous chunk's fragments are read
          }
          stage_plain(sm.g, P.m, F, jc.kb * 32, jc.nk, B);
          __syncthreads();
          job_mma(w, jc, sm.g, 0, acc);
        }
        job_reduce(sm.g, acc);
        const int r = tid >> 4, c = tid & 15;
        st_sc1(P.dpart + (g % TS_SD) * RD + (size_t)r * D + j.t0 * 16 + c, r < B ? sm.g.red[0][0][r][c] : 0.f);
      }
      const TsJob jn = l + 1 < a.nl ? qkv_job(l + 1) : out_job();
      ts_barrier(bar, [&] { job_load(w, jn); });
    }
  }
  // ---------------- OUT: R = xb + sum dpart; final norm; out_fnn tile g + bias -> logits
  {
    const TsJob j = out_job();
    if (j.W) {
      stage_norm<TS_SD>(sm.g, P.xb, P.dpart, RD, a.norm, B, D, a.eps, nullptr, g, nout);
      __syncthreads();
      f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
      job_mma(w, j, sm.g, 0, acc);
      job_reduce(sm.g, acc);
      const int r = tid >> 4, c = tid & 15, n = g * 16 + c;
      if (r < B && n < a.V)
        st_sc1(a.logits + (size_t)r * a.V + n, sm.g.red[0][0][r][c] * sm.g.misc[r] + (a.bout ? a.bout[n] : 0.f));
    }
    ts_barrier(bar, [] {});
  }
  // ---------------- DRAW: row g: penalty, top-k draw, history, next input xa[g] = emb[id]
  if (g < B) {
    const int row = g;
    float* lg = a.logits + (size_t)row * a.V;
    const int st = a.step[row];
    if (a.W > 0 && a.win) {  // k_penalty: ring entry of this step's input, then /= penalty per entry
      if (tid == 0) {
        int* wr = a.win + (size_t)row * a.W;
        wr[st % a.W] = a.ids[row];
        const int n = st + 1 < a.W ? st + 1 : a.W;
        for (int j = 0; j < n; ++j) {
          const int t = wr[j];
          if (t >= 0 && t < a.V) st_sc1(lg + t, ld1(rs_of(lg), t) / a.penalty);
        }
      }
      __syncthreads();
    }
    const int k = max(1, min(a.top_k[row], TS_KMAX));  // the host routes other k to fo_sample
    const uint64_t key = (uint64_t)a.key[row];
    const float u01 =
        (float)(uint32_t)(ts_smix(a.seed ^ (0x9E37ull * (key + 1)) + (uint64_t)st) >> 40) * (1.0f / 16777216.0f);
    SmemDraw& d = sm.dr;
    const TsRs rlg = rs_of(lg);  // the logits rows came from other workgroups (sc1)
    for (int q = 0; q < k; ++q) {  // k block arg-max passes (ties -> smallest index), as fo_sample
      float best = -INFINITY;
      int besti = 0x7fffffff;
      for (int i = tid; i < a.V_sample; i += TS_T) {
        const float x = ld1(rlg, i);
        bool skip = false;
        for (int t = 0; t < q; ++t) skip |= d.taken[t] == i;
        if (!skip && (x > best || (x == best && i < besti))) {
          best = x;
          besti = i;
        }
      }
      d.bv[tid] = best;
      d.bi[tid] = besti;
      __syncthreads();
      for (int o = TS_T / 2; o > 0; o >>= 1) {
        if (tid < o) {
          const float v2 = d.bv[tid + o];
          const int i2 = d.bi[tid + o];
          if (v2 > d.bv[tid] || (v2 == d.bv[tid] && i2 < d.bi[tid])) {
            d.bv[tid] = v2;
            d.bi[tid] = i2;
          }
        }
        __syncthreads();
      }
      if (tid == 0) {
        d.taken[q] = d.bi[0];
        d.tv[q] = d.bv[0];
      }
      __syncthreads();
    }
    if (tid == 0) {
      int pick = d.taken[0];
      if (k > 1) {  // temperature 1, no top-p: softmax over the sorted top-k, inverse-CDF draw
        float p[TS_KMAX];
        float z = 0.f;
        for (int q = 0; q < k; ++q) {
          p[q] = expf(d.tv[q] - d.tv[0]);
          z += p[q];
        }
        const float u = u01 * z;
        float c = 0.f;
        pick = d.taken[k - 1];
        for (int q = 0; q < k; ++q) {
          c += p[q];
          if (u < c) {
            pick = d.taken[q];
            break;
          }
        }
      }
      d.si[0] = pick;
      a.ids[row] = pick;
      if (a.hist) a.hist[(size_t)a.hist_row[0] * a.hist_ld + row] = pick;
    }
    __syncthreads();
    const bf16_t* er = (const bf16_t*)a.emb + (size_t)d.si[0] * a.emb_ld;
    for (int i = tid; i < D; i += TS_T) xa[(size_t)row * D + i] = bf2f(er[i]);
  }
  if (a.trace && tid == 0) a.trace[g * 64 + 63] = wall_clock64();
  ts_exit(bar);
}

}  // namespace

extern "C" {

long long fo_tts_step_ws_floats(int D, int H, int hd, int F, int S) {
  const long long RD = 16ll * D;
  return RD * 2 + 16ll * H * S * (hd + 4) + 16ll * F + TS_SD * RD;
}

int fo_tts_step(const FoTtsStep* p, hipStream_t s) {
  FO_REQUIRE(p, "fo_tts_step: null arguments");
  const FoTtsStep& a = *p;
  FO_REQUIRE(a.B >= 1 && a.B <= 16, "fo_tts_step: B=%d (1..16 sessions)", a.B);
  FO_REQUIRE((a.hd == 64 || a.hd == 32) && a.H * a.hd == a.D && a.D % 128 == 0 && a.D <= 1024,
             "fo_tts_step: D=%d H=%d hd=%d (hd 32 or 64, D = H hd, D %% 128 == 0, D <= 1024)", a.D, a.H, a.hd);
  FO_REQUIRE(a.nl >= 1 && a.nl <= FO_TTS_MAXL, "fo_tts_step: %d layers", a.nl);
  FO_REQUIRE(a.D / 32 <= TS_XKS && a.D / 32 <= TS_W * TS_KW,
             "fo_tts_step: D=%d outside the staged / prefetched k-steps", a.D);
  FO_REQUIRE(a.F % 32 == 0 && (a.F / 32) % TS_SD == 0 && a.F % 16 == 0,
             "fo_tts_step: F=%d outside the staged / prefetched k-steps", a.F);
  FO_REQUIRE(a.V >= 1 && a.V_sample >= 1 && a.V_sample <= a.V && a.S >= 1 && a.PS >= 1 && a.maxb >= 1,
             "fo_tts_step: V=%d V_sample=%d S=%d", a.V, a.V_sample, a.S);
  FO_REQUIRE(a.ws && a.bar && a.err && a.x && a.ids && a.logits && a.top_k && a.tok_pos && a.tok_slot &&
                 a.tok_nvis && a.step && a.key && a.block_table && a.emb && a.cos_t && a.sin_t && a.norm && a.wout,
             "fo_tts_step: missing buffers");
  FO_REQUIRE(!a.hist || a.hist_row, "fo_tts_step: history without its row");
  FO_REQUIRE(a.W == 0 || (a.win && a.penalty > 0.f), "fo_tts_step: penalty window without ring / penalty");
  int dev = 0, ncu = 0;
  FO_HIP(hipGetDevice(&dev));
  FO_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  // every phase's jobs must fit the grid: one workgroup per CU, all resident (barriers)
  const int need = std::max({3 * a.D / 32, a.B * a.H * a.S, a.D / 16, (a.D / 16) * TS_SD,
                             (a.V + 15) / 16, a.B});
  FO_REQUIRE(need <= ncu, "fo_tts_step: %d jobs in a phase > %d CUs", need, ncu);
  hipLaunchKernelGGL(k_tts_step, dim3(ncu), dim3(TS_T), 0, s, a);
  return fo::check_launch("fo_tts_step");
}

}  // extern "C"
