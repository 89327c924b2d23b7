// Weight-streaming GEMM for every linear layer on the Freeze-Omni hot path.
//
//   Y[M, N] = epilogue( X[M, K] (bf16) . W[N, K]^T (bf16, pre-packed) )
//
// The reference reaches these through torch.nn.Linear under bf16 autocast
// (models/audioLLM.py:482 -> Qwen2 q/k/v/o/gate/up/down, models/encoder/attention.py:411-413,
// models/adapter.py:679, models/decoder/decoder.py:346).  On the path M is tiny (one row per
// user token: 1..~64) while W is 3..150 MB, so the kernel is an HBM weight stream:
//  * W is packed once at load into MFMA fragment order [N/16][K/32][64 lanes][8 bf16] so every
//    wave-instruction of the stream is one contiguous 1 KiB read.
//  * one workgroup = 16 output columns (2x16 for the SwiGLU pair) x up to 64 rows; its 4/8/16 waves
//    split the K range (16 when the grid is about one workgroup per CU, fewer as it grows), keep 4
//    k-steps of weights in flight each, and reduce through LDS.
//  * only when the grid is tiny (< 48 tiles) is K also split across workgroups: each split writes a
//    partial slab and a second launch (k_gemm_reduce) sums the slabs in split order and applies the
//    epilogue, so results are deterministic and no cross-workgroup fence sits inside the GEMM.
//  * mfma_f32_16x16x32_bf16 accumulates in fp32; bias/activation/residual/SwiGLU are fused
//    into the epilogue.
#include <type_traits>

#include "fo_common.h"

namespace {

struct GemmArgs {
  const void* X;
  const bf16_t* Wp;
  const float* bias;
  const float* scale;  // optional per-column affine after bias (folded eval BatchNorm)
  const float* shift;
  void* Y;
  float* ws;
  int* counters;
  int ldx, ldy;
  int M, K, N;     // N: logical output columns (after SwiGLU pairing)
  int ntiles;      // packed 16-column tiles in Wp
  int S;           // K split across workgroups
  int act, out_bf16, residual;
  // fused RMSNorm, split across two GEMMs (Qwen2RMSNorm / LlamaRMSNorm between residual updates):
  //  producer: besides Y (the residual stream) writes yg = Y * gamma_next and per-row partial sums
  //            of Y^2 per workgroup column group (sout);
  //  consumer: takes yg as X and scales its accumulators by rstd(row) = rsqrt(sum / K + eps) before
  //            bias / activation -- W (x*g*rstd) = rstd * (W (x*g)), so no separate norm kernel.
  float* sout;        // producer: [M][groups] partial sums of squares
  const float* gnext; // producer: gamma of the next norm [N]
  float* yg;          // producer: Y * gamma_next, row stride ldy
  const float* rstats;  // consumer: producer's partials
  int rgroups;          // consumer: partials per row
  float reps;           // consumer: eps
  // fused RoPE + paged-KV append (the fused q|k|v projection of a Qwen2 / Llama layer): the weight
  // is packed so each 16-column tile pair holds columns (i, i + hd/2) of one head; the epilogue
  // rotates q and k heads by the token's position and writes q to rq [M][rH*rhd], k and v rows to
  // the paged cache at the token's slot ([page][kv head][PS][hd]); Y is not written.
  const int* rpos;
  const int* rslot;
  const float* rcos;  // [pos][hd/2]
  const float* rsin;
  float* rq;
  float* rk;
  float* rv;
  int rH, rKVH, rhd, rPS;
  int rkvb;   // K / V rounded to bf16 as they are appended (fo_set_kv_bf16: the reference's autocast k_proj / v_proj A/B)
  // LayerNorm on load (the pre-norm of a speech-encoder block, models/encoder/transformer.py:103-130):
  // X rows are normalised ((x - mean) * rstd * lnw + lnb) as they are loaded, before the bf16 hi/lo
  // split; mean and variance come from the producer GEMM's per-row partial sums of Y and Y^2
  // (rstats1 / rstats), so the LayerNorm launch disappears.
  const float* lnw;
  const float* lnb;
  float lneps;
  float* sout1;          // producer: [M][groups] partial sums of Y (with sout: LayerNorm statistics)
  const float* rstats1;  // LayerNorm consumer: the producer's partial sums (rstats: sums of squares)
  unsigned long long* trc;  // probes only (fo_gemm_set_trace): per-workgroup wall clocks, 24 slots
  // fp32 X of <= 16 rows already split into bf16 hi / lo in MFMA A-fragment order ([K/32][64 lanes][8], lane l =
  // row l & 15, columns 8 (l >> 4) .. + 8 of the k-step): a wave's X fragment is one contiguous 1 KiB read per half
  // instead of 16 row segments per float4 (one-row-tile grid kernels only; nullptr: plain fp32 X)
  const bf16x8* xph;
  const bf16x8* xpl;
  // producer: yg (a next-norm input) or, without yg, Y also written packed the same way (fo_gemm_set_ypack)
  bf16_t* ypkh;
  bf16_t* ypkl;
  int prb;   // packed row blocks of xph / ypkh: ceil(M / 16) (1..4)
  // the fp32 form of the same order for a LayerNorm-on-load consumer (the encoder's residual stream):
  // producer yp32 (fo_gemm_set_ypack32, its output Y), consumer xp32 (fo_gemm_set_xpack32, k_gemm_ln only)
  float* yp32;
  const float* xp32;
};

// XF32: X is fp32 and is split per element into bf16 hi + bf16 lo (two MFMAs against the same
// bf16 weight fragment), so activations keep ~16 mantissa bits at unchanged weight traffic.
template <typename XT, bool XF32>
__device__ __forceinline__ void load_x(const XT* p, bf16x8& hi, bf16x8& lo) {
  if constexpr (XF32) {
    const float4 a = reinterpret_cast<const float4*>(p)[0];
    const float4 b = reinterpret_cast<const float4*>(p)[1];
    const float f[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const __bf16 h = (__bf16)f[j];
      hi[j] = h;
      lo[j] = (__bf16)(f[j] - (float)h);
    }
  } else {
    hi = *reinterpret_cast<const bf16x8*>(p);
  }
}

// In-launch split-K merge (gemm_body, a.counters set by fo_gemm): each split's partial tile is stored write-through
// (st_wt, fo_common.h), the split drains its stores and takes the tile's ticket; the last split to arrive reads the
// others back with ld_sc1 -- no second launch, no fences.

// Output element (m, n): bias, folded-BN affine, activation or SwiGLU, residual, store.
__device__ __forceinline__ float epilogue_store(const GemmArgs& a, bool sw, int m, int n, float v, float u) {
  if (sw) {
    v = v / (1.f + expf(-v)) * u;
  } else {
    if (a.bias) v += a.bias[n];
    if (a.scale) v = v * a.scale[n] + a.shift[n];
    v = apply_act(v, a.act);
  }
  const size_t o = (size_t)m * a.ldy + n;
  if (a.out_bf16) {
    bf16_t* y = reinterpret_cast<bf16_t*>(a.Y);
    if (a.residual) v += bf2f(y[o]);
    y[o] = f2bf(v);
  } else {
    float* y = reinterpret_cast<float*>(a.Y);
    if (a.residual) v += y[o];
    y[o] = v;
  }
  return v;
}

// Columns (n, n + hd/2) of one head, n < hd/2 within the head (transformers rotate_half RoPE, the
// reference's Qwen2 / Llama attention reached from models/audioLLM.py:482, models/decoder/decoder.py:299-311).
__device__ __forceinline__ void rope_store(const GemmArgs& a, int m, int n, float x1, float x2) {
  const int hd = a.rhd, half = hd >> 1;
  const int h = n / hd, i = n - h * hd;
  if (a.bias) {
    x1 += a.bias[n];
    x2 += a.bias[n + half];
  }
  const int sl = a.rslot[m];
  const int page = sl / a.rPS, off = sl - page * a.rPS;
  if (h < a.rH + a.rKVH) {
    const int p = a.rpos[m];
    const float c = a.rcos[(size_t)p * half + i], sn = a.rsin[(size_t)p * half + i];
    float o1 = x1 * c - x2 * sn, o2 = x2 * c + x1 * sn;
    if (a.rkvb && h >= a.rH) {
      o1 = bf2f(f2bf(o1));
      o2 = bf2f(f2bf(o2));
    }
    float* d = h < a.rH ? a.rq + (size_t)m * a.rH * hd + (size_t)h * hd
                        : a.rk + (((size_t)page * a.rKVH + (h - a.rH)) * a.rPS + off) * hd;
    d[i] = o1;
    d[i + half] = o2;
  } else {
    float* d = a.rv + (((size_t)page * a.rKVH + (h - a.rH - a.rKVH)) * a.rPS + off) * hd;
    d[i] = a.rkvb ? bf2f(f2bf(x1)) : x1;
    d[i + half] = a.rkvb ? bf2f(f2bf(x2)) : x2;
  }
}
// rope_store with the bias already added and the slot / cos / sin loaded ahead (gemm_body EPRE)
__device__ __forceinline__ void rope_store_pre(const GemmArgs& a, int m, int n, float x1, float x2, int sl, float c,
                                               float sn) {
  const int hd = a.rhd, half = hd >> 1;
  const int h = n / hd, i = n - h * hd;
  const int page = sl / a.rPS, off = sl - page * a.rPS;
  float* d;
  if (h < a.rH + a.rKVH) {
    const float o1 = x1 * c - x2 * sn, o2 = x2 * c + x1 * sn;
    x1 = o1;
    x2 = o2;
    d = h < a.rH ? a.rq + (size_t)m * a.rH * hd + (size_t)h * hd
                 : a.rk + (((size_t)page * a.rKVH + (h - a.rH)) * a.rPS + off) * hd;
  } else {
    d = a.rv + (((size_t)page * a.rKVH + (h - a.rH - a.rKVH)) * a.rPS + off) * hd;
  }
  if (a.rkvb && h >= a.rH) {
    x1 = bf2f(f2bf(x1));
    x2 = bf2f(f2bf(x2));
  }
  d[i] = x1;
  d[i + half] = x2;
}
// logical first column of rope tile pair P, column c
__device__ __forceinline__ int rope_col(const GemmArgs& a, int P, int c) {
  const int per = a.rhd >> 5;  // tile pairs per head
  return (P / per) * a.rhd + (P % per) * 16 + c;
}

// NT packed 16-column tiles per workgroup (SW: NT/2 interleaved gate/up pairs -> NT/2 output tiles)
// zero words a lane loads instead of an operand that does not exist (branch-free prologues)
__device__ float g_zeros[4];

// The per-workgroup clock hook of the grid kernels (fo_gemm_set_trace) exists only in the probe library (make probe
// -> fo/libfo_hip_probe.so, loaded through FO_LIB_PATH by scripts/gemm_trace.py): compiled into the product, even
// never armed, it cost the AR decode step 178 -> 172.5 us and the encoder stage 1239 -> 1227 us (r05zj).
#ifndef FO_GEMM_TRACE
#define FO_GEMM_TRACE 0
#endif

template <int NT, int RB, bool XF32, int NW, int U, bool SW, bool LN = false, bool PIPE = false, bool XPK = false>
__device__ __forceinline__ void gemm_body(const GemmArgs& a) {
  using XT = typename std::conditional<XF32, float, bf16_t>::type;
  static_assert(!LN || XF32, "LayerNorm on load needs fp32 X");
  // NW waves split K inside the workgroup; each keeps U k-steps of weights in flight
  constexpr int NTH = NW * 64;
  constexpr int ROWS = RB * 16;
  __shared__ float red[NW][NT][ROWS][17];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int tg = blockIdx.x, mt = blockIdx.y, sp = blockIdx.z;
  const int KS = a.K >> 5;
  const int kb = (int)((long)KS * sp / a.S), ke = (int)((long)KS * (sp + 1) / a.S);
  const int len = ke - kb;
  const int m0 = mt * ROWS;
  int rbeff = (a.M - m0 + 15) >> 4;
  if (rbeff > RB) rbeff = RB;
  unsigned long long* const trc = (FO_GEMM_TRACE && a.trc)
      ? a.trc + (size_t)(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z)) * 24 : nullptr;
  if (trc && threadIdx.x == 0) trc[0] = wall_clock64();

  // Epilogue operands prefetched when every output element of the workgroup has its own thread (the small-M,
  // latency-bound shapes): the residual, bias and next-norm gamma (plain path) or the token's slot / position,
  // its cos / sin and the q|k|v bias (RoPE path) arrive while the weights stream, instead of costing one or two
  // dependent memory round trips after the K reduction.  Ordering matters because a wave's vector-memory
  // counter retires in issue order: the independent operands (level 1) and the RMSNorm partial sums are
  // issued first, then the wave's first group of weights and X, and only then the loads whose ADDRESS needs a
  // level-1 value (cos / sin at the token's position, level 2) -- so no wait in the prologue ever waits for
  // the weight stream, and the weight stream never waits for a prologue round trip.
  constexpr int LT = SW ? NT / 2 : NT;  // logical output tiles
  constexpr bool EPRE = !SW && !LN && NT <= 2 && LT * ROWS * 16 <= NTH;
  const int ee = threadIdx.x;
  const int e_lt = ee / (ROWS * 16), e_rr = (ee >> 4) % ROWS, e_c = ee & 15;
  float p_res = 0.f, p_bias = 0.f, p_b2 = 0.f, p_cos = 1.f, p_sin = 0.f, p_gn = 0.f;
  bf16_t p_resh = f2bf(0.f);   // bf16 residual: raw bits, converted in the epilogue (no wait in the prologue)
  int p_slot = 0, p_pos = 0;
  const bool e_rope = (NT == 2 && !SW) && a.rq != nullptr;
  // split over K with the in-launch merge (fo_gemm passes counters only for plain tiles): any split may be
  // the last to arrive, so every split prefetches the epilogue operands
  const bool merge = !SW && !LN && a.S > 1 && a.counters != nullptr;
  // level 1 is branch-free: a lane whose operand does not exist loads a zero word instead (g_zeros), so no
  // divergent branch leaves a register with a pending load that a later write would have to wait for
  bool p_rot = false;   // this lane's output column is a rotated q / k column (level 2 loads its cos / sin)
  if constexpr (EPRE) {   // straight-line code: every operand load is issued, from g_zeros when it does not apply
    const bool on = (a.S == 1 || merge) && ee < LT * ROWS * 16;
    const int m = m0 + e_rr;
    const float* z = g_zeros;
    const int rhd = e_rope ? a.rhd : 32;   // (no division by a zero head size on the plain path)
    const int half = rhd >> 1;
    const int nrope = (tg / (rhd >> 5)) * rhd + (tg % (rhd >> 5)) * 16 + e_c;   // rope_col
    const int nplain = (tg * LT + e_lt) * 16 + e_c;
    const bool okr = e_rope && on && ee < ROWS * 16 && m < a.M;
    const bool okp = !e_rope && on && m < a.M && nplain < a.N;
    p_rot = okr && nrope / rhd < a.rH + a.rKVH;
    const size_t o = (size_t)m * a.ldy + nplain;
    p_slot = *(okr ? a.rslot + m : reinterpret_cast<const int*>(z));
    p_pos = *(p_rot ? a.rpos + m : reinterpret_cast<const int*>(z));
    p_bias = *(a.bias && (okr || okp) ? a.bias + (e_rope ? nrope : nplain) : z);
    p_b2 = *(a.bias && okr ? a.bias + nrope + half : z);
    p_resh = *(okp && a.residual && a.out_bf16 ? reinterpret_cast<const bf16_t*>(a.Y) + o
                                                : reinterpret_cast<const bf16_t*>(z));
    p_res = *(okp && a.residual && !a.out_bf16 ? reinterpret_cast<const float*>(a.Y) + o : z);
    const int n0 = tg * LT * 16;
    p_gn = *(!e_rope && a.yg && (a.S == 1 || merge) && lane < min(LT * 16, a.N - n0) ? a.gnext + n0 + lane : z);
  }

  // post-scaled RMSNorm: the producer's partial sums of this workgroup's rows (the first 64 per row, one
  // load per lane) are loaded now and reduced after the main loop (their latency hides behind the weight stream)
  constexpr int RPWV = (ROWS + NW - 1) / NW;  // rows per wave
  // wide variants are at the VGPR edge of their occupancy step: they load the partials after the loop
  constexpr bool RPRE = NT * U <= 8;
  float rpart[RPWV];
  auto load_rpart = [&](int j0) {   // partial sums j0, j0 + 64, ... added to rpart
#pragma unroll
    for (int i = 0; i < RPWV; ++i) {
      const int rr = wave + i * NW;
      const int m = min(m0 + rr, a.M - 1);
      float v = 0.f;
      if (rr < ROWS)
        for (int j = j0 + lane; j < a.rgroups; j += 64) v += a.rstats[(size_t)m * a.rgroups + j];
      rpart[i] += v;
    }
  };
#pragma unroll
  for (int i = 0; i < RPWV; ++i) rpart[i] = 0.f;
  if (RPRE && a.rstats && !LN) {
#pragma unroll
    for (int i = 0; i < RPWV; ++i) {
      const int rr = wave + i * NW;
      const int m = min(m0 + rr, a.M - 1);
      rpart[i] = *(rr < ROWS && lane < a.rgroups ? a.rstats + (size_t)m * a.rgroups + lane : g_zeros);
    }
  }

  f32x4 acc[NT][RB];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < RB; ++r) acc[t][r] = f32x4{0.f, 0.f, 0.f, 0.f};

  const bf16x8* bp[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t)
    bp[t] = reinterpret_cast<const bf16x8*>(a.Wp) + (size_t)(tg * NT + t) * KS * 64 + lane;
  const XT* xr[RB];
#pragma unroll
  for (int r = 0; r < RB; ++r) {
    int row = m0 + r * 16 + (lane & 15);
    if (row > a.M - 1) row = a.M - 1;  // clamp: rows >= M are computed but never stored
    xr[r] = reinterpret_cast<const XT*>(a.X) + (size_t)row * a.ldx + 8 * (lane >> 4);
  }
  // X given packed (GemmArgs::xph / xpl): only the k_gemm_xp instantiations read it (the others compile as before)
  static_assert(!XPK || (RB <= 4 && XF32 && !LN && !SW && !PIPE), "packed X: <= 4-row-block plain / RoPE kernels");
  const bool xpk = XPK && a.xph != nullptr;
  float ln_mu[RB], ln_rs[RB];
  // Whole groups of U k-steps are dealt to waves (all U weight loads of a group in flight
  // together); the < U leftover steps go one per wave, so no wave runs a serial tail.
  const int G = len / U, rem = len - G * U;
  const int gb = G * wave / NW, ge = G * (wave + 1) / NW;
  // LayerNorm on load: the producer's partial row sums are loaded first, then the wave's first group of weight
  // fragments and raw X rows, and only then does the wave wait for the sums (vmcnt retires in issue order, so
  // loads issued after the sums do not delay them): the statistics round trip and barrier overlap the weight
  // stream's first round trip instead of running before it
  bf16x8 lnbv[LN ? U : 1][NT];
  float4 lnxv[LN ? U : 1][RB][2];
  auto ln_issue = [&](int ks) {
    if constexpr (LN) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k = min(ks + u, KS - 1);   // in bounds for a wave without a group (its loads go unused)
#pragma unroll
        for (int t = 0; t < NT; ++t) lnbv[u][t] = __builtin_nontemporal_load(bp[t] + (size_t)k * 64);
#pragma unroll
        for (int r = 0; r < RB; ++r) {
          const float4* q = a.xp32 ? reinterpret_cast<const float4*>(a.xp32 + (((size_t)k * a.prb + min((m0 >> 4) + r, a.prb - 1)) * 64 + lane) * 8)
                                   : reinterpret_cast<const float4*>(xr[r] + (size_t)k * 32);
          lnxv[u][r][0] = q[0];
          lnxv[u][r][1] = q[1];
        }
      }
    }
  };
  if constexpr (LN) {
    // per-row mean / rstd of this workgroup's rows from the producer's partial sums
    constexpr int LRPW = (ROWS + NW - 1) / NW;
    __shared__ float ln_s[2][ROWS];
    float st1[LRPW], st2[LRPW];
#pragma unroll
    for (int i = 0; i < LRPW; ++i) {
      const int rr = wave + i * NW;
      const int m = min(m0 + rr, a.M - 1);
      const bool on = rr < ROWS && lane < a.rgroups;
      st1[i] = on ? a.rstats1[(size_t)m * a.rgroups + lane] : 0.f;
      st2[i] = on ? a.rstats[(size_t)m * a.rgroups + lane] : 0.f;
    }
    ln_issue(kb + min(gb, max(G - 1, 0)) * U);
#pragma unroll
    for (int i = 0; i < LRPW; ++i) {
      const int rr = wave + i * NW;
      if (rr >= ROWS) break;
      const float mean = wave_sum(st1[i]) / (float)a.K;   // (fo_gemm_ln: at most 64 producer groups)
      const float var = fmaxf(wave_sum(st2[i]) / (float)a.K - mean * mean, 0.f);
      if (lane == 0) {
        ln_s[0][rr] = mean;
        ln_s[1][rr] = 1.0f / sqrtf(var + a.lneps);
      }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      ln_mu[r] = ln_s[0][r * 16 + (lane & 15)];
      ln_rs[r] = ln_s[1][r * 16 + (lane & 15)];
    }
  }
  // X fragment of row block r at k-step ks (LayerNorm applied on load when LN)
  auto ldx = [&](int r, int ks, bf16x8& hi, bf16x8& lo) {
    if constexpr (LN) {
      const float* p = a.xp32 ? a.xp32 + (((size_t)ks * a.prb + min((m0 >> 4) + r, a.prb - 1)) * 64 + lane) * 8
                              : reinterpret_cast<const float*>(xr[r] + (size_t)ks * 32);
      const int k0 = ks * 32 + 8 * (lane >> 4);
      const float4 a0 = reinterpret_cast<const float4*>(p)[0], a1 = reinterpret_cast<const float4*>(p)[1];
      const float4 w0 = *reinterpret_cast<const float4*>(a.lnw + k0), w1 = *reinterpret_cast<const float4*>(a.lnw + k0 + 4);
      const float4 b0 = *reinterpret_cast<const float4*>(a.lnb + k0), b1 = *reinterpret_cast<const float4*>(a.lnb + k0 + 4);
      const float f[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
      const float w[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
      const float b[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float v = (f[j] - ln_mu[r]) * ln_rs[r] * w[j] + b[j];
        const __bf16 h = (__bf16)v;
        hi[j] = h;
        lo[j] = (__bf16)(v - (float)h);
      }
    } else {
      if (XF32 && xpk) {
        hi = a.xph[((size_t)ks * a.prb + min((m0 >> 4) + r, a.prb - 1)) * 64 + lane];
        lo = a.xpl[((size_t)ks * a.prb + min((m0 >> 4) + r, a.prb - 1)) * 64 + lane];
      } else {
        load_x<XT, XF32>(xr[r] + (size_t)ks * 32, hi, lo);
      }
    }
  };

  // level-2 epilogue operands (see EPRE above): cos / sin at the token's position (p_rot: a rotated q / k
  // column), issued once the wave's first group of weights is in flight
  auto level2 = [&]() {
    if constexpr (EPRE) {
      if (e_rope) {
        const int n = rope_col(a, tg, e_c), half = a.rhd >> 1;
        const int i = n - (n / a.rhd) * a.rhd;
        int pp = p_pos;
        asm volatile("" : "+v"(pp));   // (keeps the position's use -- and its wait -- behind the weight issue)
        const size_t o = (size_t)pp * half + i;
        const float c = *(p_rot ? a.rcos + o : g_zeros), sn = *(p_rot ? a.rsin + o : g_zeros);
        p_cos = p_rot ? c : 1.f;
        p_sin = p_rot ? sn : 0.f;
      }
    }
  };
  if constexpr (LN) {
    for (int g = gb; g < ge; ++g) {
      const int ks = kb + g * U;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k0 = (ks + u) * 32 + 8 * (lane >> 4);
        const float4 w0 = *reinterpret_cast<const float4*>(a.lnw + k0), w1 = *reinterpret_cast<const float4*>(a.lnw + k0 + 4);
        const float4 b0 = *reinterpret_cast<const float4*>(a.lnb + k0), b1 = *reinterpret_cast<const float4*>(a.lnb + k0 + 4);
        const float w[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
        const float b[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
        for (int r = 0; r < RB; ++r)
          if (r < rbeff) {
            const float f[8] = {lnxv[u][r][0].x, lnxv[u][r][0].y, lnxv[u][r][0].z, lnxv[u][r][0].w,
                                lnxv[u][r][1].x, lnxv[u][r][1].y, lnxv[u][r][1].z, lnxv[u][r][1].w};
            bf16x8 hi, lo;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const float v = (f[j] - ln_mu[r]) * ln_rs[r] * w[j] + b[j];
              const __bf16 h = (__bf16)v;
              hi[j] = h;
              lo[j] = (__bf16)(v - (float)h);
            }
#pragma unroll
            for (int t = 0; t < NT; ++t) {
              acc[t][r] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(hi, lnbv[u][t], acc[t][r], 0, 0, 0);
              acc[t][r] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(lo, lnbv[u][t], acc[t][r], 0, 0, 0);
            }
          }
      }
      if (g + 1 < ge) ln_issue(ks + U);
    }
  } else
  if constexpr (PIPE && XF32 && !LN) {
    // Software-pipelined weight stream: group g + 1's weight fragments AND raw X rows are issued
    // before group g's MFMAs, so a wave always has one group of loads in flight while it computes
    // (the loads of g are older than those of g + 1, so the in-order vmcnt wait for g leaves g + 1
    // in flight).  Two register buffers, ping-ponged by unrolling the loop by two groups.
    bf16x8 w0[U][NT], w1[U][NT];
    float4 x0[U][RB][2], x1[U][RB][2];
    auto issue = [&](bf16x8 (&wv)[U][NT], float4 (&xv)[U][RB][2], int ks) {
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int t = 0; t < NT; ++t) wv[u][t] = __builtin_nontemporal_load(bp[t] + (size_t)(ks + u) * 64);
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int r = 0; r < RB; ++r) {
          const float4* q = reinterpret_cast<const float4*>(xr[r] + (size_t)(ks + u) * 32);
          xv[u][r][0] = q[0];
          xv[u][r][1] = q[1];
        }
    };
    auto compute = [&](bf16x8 (&wv)[U][NT], float4 (&xv)[U][RB][2]) {
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int r = 0; r < RB; ++r) {
          if (r >= rbeff) continue;
          const float f[8] = {xv[u][r][0].x, xv[u][r][0].y, xv[u][r][0].z, xv[u][r][0].w,
                              xv[u][r][1].x, xv[u][r][1].y, xv[u][r][1].z, xv[u][r][1].w};
          bf16x8 hi, lo;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const __bf16 h = (__bf16)f[j];
            hi[j] = h;
            lo[j] = (__bf16)(f[j] - (float)h);
          }
#pragma unroll
          for (int t = 0; t < NT; ++t) {
            acc[t][r] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(hi, wv[u][t], acc[t][r], 0, 0, 0);
            acc[t][r] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(lo, wv[u][t], acc[t][r], 0, 0, 0);
          }
        }
    };
    int g = gb;
    if (g < ge) issue(w0, x0, kb + g * U);
    level2();
    for (; g + 1 < ge; g += 2) {
      issue(w1, x1, kb + (g + 1) * U);
      compute(w0, x0);
      if (g + 2 < ge) issue(w0, x0, kb + (g + 2) * U);
      compute(w1, x1);
    }
    if (g < ge) compute(w0, x0);
  } else {
    // the wave's FIRST group of weights and X goes into its own registers and is issued before the level-2
    // epilogue loads (cos / sin, below), unconditionally -- a wave without a group loads another wave's first
    // group again (same lines: L2 hits, no extra HBM bytes), so no wave-divergent branch or loop-carried
    // register makes the compiler's vmcnt accounting wait for the weights in the prologue; the wave's further
    // groups load at the top of their iteration
    bf16x8 bv0[U][NT];
    float4 xf0[XF32 ? U : 1][RB][2];
    bf16x8 xb0[XF32 ? 1 : U][RB];
    {
      const int ks = kb + min(gb, max(G - 1, 0)) * U;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k = min(ks + u, KS - 1);
#pragma unroll
        for (int t = 0; t < NT; ++t) bv0[u][t] = __builtin_nontemporal_load(bp[t] + (size_t)k * 64);
#pragma unroll
        for (int r = 0; r < RB; ++r) {
          if constexpr (XF32) {
            if (xpk) {
              xf0[u][r][0] = __builtin_bit_cast(float4, a.xph[((size_t)k * a.prb + min((m0 >> 4) + r, a.prb - 1)) * 64 + lane]);
              xf0[u][r][1] = __builtin_bit_cast(float4, a.xpl[((size_t)k * a.prb + min((m0 >> 4) + r, a.prb - 1)) * 64 + lane]);
            } else {
              const float4* q = reinterpret_cast<const float4*>(xr[r] + (size_t)k * 32);
              xf0[u][r][0] = q[0];
              xf0[u][r][1] = q[1];
            }
          } else {
            xb0[u][r] = *reinterpret_cast<const bf16x8*>(xr[r] + (size_t)k * 32);
          }
        }
      }
    }
    level2();
    if (gb < ge) {
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int r = 0; r < RB; ++r)
          if (r < rbeff) {
            bf16x8 hi, lo;
            if constexpr (XF32) {
              if (xpk) {
                hi = __builtin_bit_cast(bf16x8, xf0[u][r][0]);
                lo = __builtin_bit_cast(bf16x8, xf0[u][r][1]);
              } else {
                const float f[8] = {xf0[u][r][0].x, xf0[u][r][0].y, xf0[u][r][0].z, xf0[u][r][0].w,
                                    xf0[u][r][1].x, xf0[u][r][1].y, xf0[u][r][1].z, xf0[u][r][1].w};
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                  const __bf16 h = (__bf16)f[j];
                  hi[j] = h;
                  lo[j] = (__bf16)(f[j] - (float)h);
                }
              }
            } else {
              hi = xb0[u][r];
            }
#pragma unroll
            for (int t = 0; t < NT; ++t) {
              acc[t][r] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(hi, bv0[u][t], acc[t][r], 0, 0, 0);
              if constexpr (XF32) acc[t][r] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(lo, bv0[u][t], acc[t][r], 0, 0, 0);
            }
          }
    }
    for (int g = gb + 1; g < ge; ++g) {
      const int ks = kb + g * U;
      bf16x8 bv[U][NT];
      bf16x8 ah[U][RB], al[U][RB];
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int t = 0; t < NT; ++t) bv[u][t] = __builtin_nontemporal_load(bp[t] + (size_t)(ks + u) * 64);
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int r = 0; r < RB; ++r)
          if (r < rbeff) ldx(r, ks + u, ah[u][r], al[u][r]);
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int r = 0; r < RB; ++r)
            if (r < rbeff) {
              acc[t][r] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[u][r], bv[u][t], acc[t][r], 0, 0, 0);
              if constexpr (XF32)
                acc[t][r] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[u][r], bv[u][t], acc[t][r], 0, 0, 0);
            }
    }
  }
  for (int ks = kb + G * U + wave; ks < ke; ks += NW) {
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const bf16x8 b = __builtin_nontemporal_load(bp[t] + (size_t)ks * 64);
#pragma unroll
      for (int r = 0; r < RB; ++r)
        if (r < rbeff) {
          bf16x8 h, l;
          ldx(r, ks, h, l);
          acc[t][r] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(h, b, acc[t][r], 0, 0, 0);
          if constexpr (XF32) acc[t][r] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(l, b, acc[t][r], 0, 0, 0);
        }
    }
  }

  if (trc && lane == 0) trc[1 + wave] = wall_clock64();
  // D layout (16x16x32): col = lane & 15, row = 4*(lane>>4) + i
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < RB; ++r)
#pragma unroll
      for (int i = 0; i < 4; ++i) red[wave][t][r * 16 + 4 * (lane >> 4) + i][lane & 15] = acc[t][r][i];
  __syncthreads();
  if (trc && threadIdx.x == 0) trc[17] = wall_clock64();

  constexpr int NE = NT * ROWS * 16;
  for (int e = threadIdx.x; e < NE; e += NTH) {
    const int t = e / (ROWS * 16), rr = (e / 16) % ROWS, c = e & 15;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) v += red[w][t][rr][c];
    red[0][t][rr][c] = v;
  }
  if (a.S > 1) {
    // K split across workgroups: write this split's partial slab; without the merge k_gemm_reduce (the
    // next launch on the stream) sums the slabs in split order and applies the epilogue
    const int Mrows = gridDim.y * ROWS;
    const int Ncols = a.ntiles * 16;
    float* slab = a.ws + (size_t)sp * Mrows * Ncols;
    if (!merge) {
      __syncthreads();
      for (int e = threadIdx.x; e < NE; e += NTH) {
        const int t = e / (ROWS * 16), rr = (e / 16) % ROWS, c = e & 15;
        slab[(size_t)(m0 + rr) * Ncols + (tg * NT + t) * 16 + c] = red[0][t][rr][c];
      }
      if (trc && threadIdx.x == 0) trc[18] = wall_clock64();
      return;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < NE; e += NTH) {
      const int t = e / (ROWS * 16), rr = (e / 16) % ROWS, c = e & 15;
      st_wt(slab + (size_t)(m0 + rr) * Ncols + (tg * NT + t) * 16 + c, red[0][t][rr][c]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __shared__ int last_s;
    __syncthreads();
    if (threadIdx.x == 0) {
      int* tk = a.counters + (blockIdx.x + gridDim.x * blockIdx.y);
      const int old = __hip_atomic_fetch_add(tk, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last_s = old == a.S - 1;
      if (old == a.S - 1) __hip_atomic_store(tk, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!last_s) return;
    // the last split: every split's partial, summed in split order (k_gemm_reduce's order, bit for bit)
    const __amdgpu_buffer_rsrc_t rws = rsrc_of(a.ws);
    const size_t sl = (size_t)Mrows * Ncols;
    for (int e = threadIdx.x; e < NE; e += NTH) {
      const int t = e / (ROWS * 16), rr = (e / 16) % ROWS, c = e & 15;
      const size_t o = (size_t)(m0 + rr) * Ncols + (tg * NT + t) * 16 + c;
      const float own = red[0][t][rr][c];
      float v = 0.f;
      for (int q0 = 0; q0 < a.S; q0 += 4) {
        float tv[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
          tv[j] = (q0 + j < a.S && q0 + j != sp) ? ld_sc1(rws, (q0 + j) * sl + o) : own;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (q0 + j < a.S) v += tv[j];
      }
      red[0][t][rr][c] = v;
    }
    __syncthreads();
  }
  if (a.rstats && !LN && (a.S == 1 || merge)) {  // (split without the merge: k_gemm_reduce scales the sums)
    if (!RPRE) load_rpart(0);
    else if (a.rgroups > 64) load_rpart(64);
    __shared__ float rstd_s[ROWS];
#pragma unroll
    for (int i = 0; i < RPWV; ++i) {
      const int rr = wave + i * NW;
      const float ss = wave_sum(rpart[i]);
      if (rr < ROWS && lane == 0) rstd_s[rr] = rsqrtf(ss / (float)a.K + a.reps);
    }
    __syncthreads();
    for (int e = threadIdx.x; e < NE; e += NTH) {
      const int t = e / (ROWS * 16), rr = (e / 16) % ROWS, c = e & 15;
      red[0][t][rr][c] *= rstd_s[rr];
    }
  }
  __syncthreads();
  if constexpr (NT == 2 && !SW) {
    if (a.rq) {
      if constexpr (EPRE) {
        if (ee < ROWS * 16 && m0 + e_rr < a.M)
          rope_store_pre(a, m0 + e_rr, rope_col(a, tg, e_c), red[0][0][e_rr][e_c] + p_bias,
                         red[0][1][e_rr][e_c] + p_b2, p_slot, p_cos, p_sin);
        if (trc && threadIdx.x == 0) trc[18] = wall_clock64();
        return;
      }
      for (int e = threadIdx.x; e < ROWS * 16; e += NTH) {
        const int rr = e >> 4, c = e & 15, m = m0 + rr;
        if (m < a.M) rope_store(a, m, rope_col(a, tg, c), red[0][0][rr][c], red[0][1][rr][c]);
      }
      if (trc && threadIdx.x == 0) trc[18] = wall_clock64();
      return;
    }
  }
  if constexpr (EPRE) {
    if (ee < LT * ROWS * 16) {
      const int m = m0 + e_rr, n = (tg * LT + e_lt) * 16 + e_c;
      if (m < a.M && n < a.N) {
        float v = red[0][e_lt][e_rr][e_c] + p_bias;
        if (a.scale) v = v * a.scale[n] + a.shift[n];
        float pr = p_res;
        if (a.out_bf16) {   // (the barrier keeps the conversion, and its wait for the load, here)
          unsigned rb = p_resh;
          asm volatile("" : "+v"(rb));
          pr = bf2f((bf16_t)rb);
        }
        v = apply_act(v, a.act) + pr;
        const size_t o = (size_t)m * a.ldy + n;
        if (a.out_bf16) reinterpret_cast<bf16_t*>(a.Y)[o] = f2bf(v);
        else reinterpret_cast<float*>(a.Y)[o] = v;
        red[0][e_lt][e_rr][e_c] = v;
        if (a.ypkh && !a.yg) xpack_store(a.ypkh, a.ypkl, m, n, v, a.prb);   // Y is the next GEMM's packed input
        if (a.yp32) xpack32_store(a.yp32, m, n, v, a.prb);
      }
    }
  } else
  for (int e = threadIdx.x; e < LT * ROWS * 16; e += NTH) {
    const int lt = e / (ROWS * 16), rr = (e >> 4) % ROWS, c = e & 15;
    const int m = m0 + rr;
    const int n = (tg * LT + lt) * 16 + c;
    if (m >= a.M || n >= a.N) continue;
    float y;
    if (SW) y = epilogue_store(a, true, m, n, red[0][2 * lt][rr][c], red[0][2 * lt + 1][rr][c]);
    else y = epilogue_store(a, false, m, n, red[0][lt][rr][c], 0.f);
    if (!SW) red[0][lt][rr][c] = y;
    if (a.ypkh && !a.yg) xpack_store(a.ypkh, a.ypkl, m, n, y, a.prb);   // Y is the next GEMM's packed input
    if (a.yp32) xpack32_store(a.yp32, m, n, y, a.prb);
  }
  if (!SW && a.sout) {
    // row partial sums of squares of this workgroup's LT*16 output columns, for the next norm
    __syncthreads();
    const int n0 = tg * LT * 16;
    const int cnt = min(LT * 16, a.N - n0);
    for (int rr = wave; rr < ROWS; rr += NW) {
      const int m = m0 + rr;
      if (m >= a.M) break;
      // the workgroup's LT * 16 columns in 64-lane passes (one pass up to 4 tiles; 8-tile groups take two)
      float sq = 0.f, sm = 0.f;
#pragma unroll
      for (int c0 = 0; c0 < LT * 16; c0 += 64) {
        const int c = c0 + lane;
        const float v = c < cnt ? red[0][c >> 4][rr][c & 15] : 0.f;
        sq += v * v;
        sm += v;
        if (a.yg && c < cnt) {
          const float vg = v * (EPRE ? p_gn : a.gnext[n0 + c]);
          a.yg[(size_t)m * a.ldy + n0 + c] = vg;
          if (a.ypkh) xpack_store(a.ypkh, a.ypkl, m, n0 + c, vg, a.prb);
        }
      }
      const float ss = wave_sum(sq);
      if (lane == 0) a.sout[(size_t)m * gridDim.x + tg] = ss;
      if (a.sout1) {
        const float s1 = wave_sum(sm);
        if (lane == 0) a.sout1[(size_t)m * gridDim.x + tg] = s1;
      }
    }
  }
  if (trc && threadIdx.x == 0) trc[18] = wall_clock64();
}

// Sum of the S partial slabs + epilogue for the split-K path.  Grid (ceil(N/256), M): one row
// chunk of 256 columns per block, which is also the statistics group for a fused normalisation.
template <int SQ>   // slabs whose loads are issued up front (8; 16 for the 16-slab k_gemm_rows down / o)
__global__ __launch_bounds__(256) void k_gemm_reduce_t(GemmArgs a, int sw, int Mrows) {
  __shared__ float red_s[4];
  const int Ncols = a.ntiles * 16;
  const size_t slab = (size_t)Mrows * Ncols;
  const int m = blockIdx.y, n = blockIdx.x * 256 + threadIdx.x;
  // Every load of the launch is issued up front -- up to SQ slabs' partials, the epilogue operands and the
  // producer's RMSNorm partial sums -- so the kernel pays ONE dependent memory round trip before its sum
  // (the slabs are still summed in slab order: the same result bit for bit).  The epilogue operand loads are
  // branch-free (g_zeros when an operand does not apply), so no divergent branch makes the compiler's vmcnt
  // accounting wait early.
  const bool rope = a.rq != nullptr;
  const int ncol = rope ? a.N / 2 : a.N;
  const bool live = n < ncol;
  const int col = rope ? (n >> 4) * 32 + (n & 15) : (sw ? (n >> 4) * 32 + (n & 15) : n);
  const bool pair = rope || sw;   // two partial columns per thread (the tile pair / gate-up pair, 16 apart)
  const float* p = a.ws + (size_t)m * Ncols + (live ? col : 0);
  float tv[SQ], tu[SQ];
#pragma unroll
  for (int j = 0; j < SQ; ++j) {
    tv[j] = 0.f;
    tu[j] = 0.f;
    if (j < a.S) {
      tv[j] = p[j * slab];
      if (pair) tu[j] = p[j * slab + 16];
    }
  }
  const float* z = g_zeros;
  const bool plain = !rope && !sw && live;
  const size_t o = (size_t)m * a.ldy + n;
  bf16_t p_resh = *(plain && a.residual && a.out_bf16 ? reinterpret_cast<const bf16_t*>(a.Y) + o
                                                      : reinterpret_cast<const bf16_t*>(z));
  const float p_res = *(plain && a.residual && !a.out_bf16 ? reinterpret_cast<const float*>(a.Y) + o : z);
  const float p_bias = *(plain && a.bias ? a.bias + n : z);
  const float p_gn = *(plain && a.yg ? a.gnext + n : z);
  const bool rms = a.rstats && !a.lnw;   // RMSNorm consumer split over K: the row's rstd scales the summed partials
  const float st = *(rms && threadIdx.x < 64 && threadIdx.x < a.rgroups ? a.rstats + (size_t)m * a.rgroups + threadIdx.x : z);
  float rs = 1.f;
  if (rms) {
    if (threadIdx.x < 64) {  // lane-strided + wave_sum: the order gemm_body's unsplit path uses
      float ss = st;
      for (int j = threadIdx.x + 64; j < a.rgroups; j += 64) ss += a.rstats[(size_t)m * a.rgroups + j];
      ss = wave_sum(ss);
      if (threadIdx.x == 0) red_s[0] = rsqrtf(ss / (float)a.K + a.reps);
    }
    __syncthreads();
    rs = red_s[0];
    __syncthreads();
  }
  float v = 0.f, u = 0.f;
#pragma unroll
  for (int j = 0; j < SQ; ++j)
    if (j < a.S) {
      v += tv[j];
      u += tu[j];
    }
  for (int q = SQ; q < a.S; ++q) {   // more than SQ slabs (not used by the policies in fo_gemm)
    v += p[q * slab];
    if (pair) u += p[q * slab + 16];
  }
  if (rope) {  // one thread per column pair, packed tiles (2P, 2P + 1)
    if (live) rope_store(a, m, rope_col(a, n >> 4, n & 15), v * rs, u * rs);
    return;
  }
  float y = 0.f;
  if (live) {
    if (sw) {
      y = epilogue_store(a, true, m, n, v * rs, u * rs);
    } else {
      y = v * rs + p_bias;
      if (a.scale) y = y * a.scale[n] + a.shift[n];
      float pr = p_res;
      if (a.out_bf16) {   // (the barrier keeps the conversion, and its wait for the load, here)
        unsigned rb = p_resh;
        asm volatile("" : "+v"(rb));
        pr = bf2f((bf16_t)rb);
      }
      y = apply_act(y, a.act) + pr;
      if (a.out_bf16) reinterpret_cast<bf16_t*>(a.Y)[o] = f2bf(y);
      else reinterpret_cast<float*>(a.Y)[o] = y;
      if (a.ypkh && !a.yg) xpack_store(a.ypkh, a.ypkl, m, n, y, a.prb);   // Y is the next GEMM's packed input
      if (a.yp32) xpack32_store(a.yp32, m, n, y, a.prb);
    }
  }
  if (a.sout && !sw) {
    const float ss = block_sum<4>(live ? y * y : 0.f, red_s);
    if (threadIdx.x == 0) a.sout[(size_t)m * gridDim.x + blockIdx.x] = ss;
    if (a.sout1) {
      const float s1 = block_sum<4>(live ? y : 0.f, red_s);
      if (threadIdx.x == 0) a.sout1[(size_t)m * gridDim.x + blockIdx.x] = s1;
    }
    if (a.yg && live) {
      const float vg = y * p_gn;
      a.yg[o] = vg;
      if (a.ypkh) xpack_store(a.ypkh, a.ypkl, m, n, vg, a.prb);
    }
  }
}

// (the partials of more than 8 slabs prefetched only when there are: the 16 registers cost the paired (SwiGLU / RoPE)
// 3-slab gate/up reduce 15.5 -> 17.4 us, r06t)
inline void launch_reduce(const GemmArgs& a, int sw, int Mrows, int N, int M, hipStream_t stream) {
  if (a.S > 8) hipLaunchKernelGGL(k_gemm_reduce_t<16>, dim3((N + 255) / 256, M), dim3(256), 0, stream, a, sw, Mrows);
  else hipLaunchKernelGGL(k_gemm_reduce_t<8>, dim3((N + 255) / 256, M), dim3(256), 0, stream, a, sw, Mrows);
}

template <int NT, int RB, bool XF32, int NW, int U, bool SW>
__global__ __launch_bounds__(NW * 64) void k_gemm(GemmArgs a) {
  gemm_body<NT, RB, XF32, NW, U, SW>(a);
}
template <int NT, int RB, bool XF32, int NW, int U, bool SW>
__global__ __launch_bounds__(NW * 64) void k_gemm_wstream(GemmArgs a) {
  gemm_body<NT, RB, XF32, NW, U, SW>(a);
}
template <int NT, int RB, int NW, int U, bool SW>
__global__ __launch_bounds__(NW * 64) void k_gemm_wpipe(GemmArgs a) {
  gemm_body<NT, RB, true, NW, U, SW, false, true>(a);
}
// one-row-tile fp32-X GEMM reading X packed by its producer (GemmArgs::xph / xpl, ops.XPack)
template <int NT, int RB, int NW, int U>
__global__ __launch_bounds__(NW * 64) void k_gemm_xp(GemmArgs a) {
  gemm_body<NT, RB, true, NW, U, false, false, false, true>(a);
}

// Software-pipelined one-row-tile fp32-X weight stream (k_gemm_wpipe).  Mode: 0 = plain loops
// everywhere; 1 / 2 = every such GEMM pipelined with U / 2 k-steps per group (sweeps); 3 = the
// measured policy in fo_gemm (default).  -1 = not set yet: FO_GEMM_PIPE (0-3) decides at first use.
int g_pipe = -1;
inline int pipe_mode() {
  if (g_pipe < 0) {
    const char* e = getenv("FO_GEMM_PIPE");
    g_pipe = (e && e[0] >= '0' && e[0] <= '3') ? e[0] - '0' : 3;
  }
  return g_pipe;
}
// the pipelining fo_gemm chose for the launch it is issuing (0 none, 1 U-step, 2 two-step groups)
thread_local int g_launch_pipe = 0;
template <int NT, int RB, int NW, int U = 4>
__global__ __launch_bounds__(NW * 64) void k_gemm_ln(GemmArgs a) {
  gemm_body<NT, RB, true, NW, U, false, true>(a);
}

template <int NT, int RB, int NW, int U, bool SW>
void launch_gemm(bool wstream, bool x_f32, dim3 grid, const GemmArgs& a, hipStream_t s) {
  const size_t shm = 0;
  if constexpr (RB <= 4 && !SW) {
    if (x_f32 && a.xph && !(RB == 1 && g_launch_pipe)) {   // X packed by its producer
      hipLaunchKernelGGL((k_gemm_xp<NT, RB, NW, U>), grid, dim3(NW * 64), shm, s, a);
      return;
    }
  }
  if constexpr (RB == 1) {
    if (x_f32 && g_launch_pipe) {
      if (g_launch_pipe == 2) hipLaunchKernelGGL((k_gemm_wpipe<NT, RB, NW, 2, SW>), grid, dim3(NW * 64), shm, s, a);
      else hipLaunchKernelGGL((k_gemm_wpipe<NT, RB, NW, U, SW>), grid, dim3(NW * 64), shm, s, a);
      return;
    }
  }
  if (wstream) {
    if (x_f32) hipLaunchKernelGGL((k_gemm_wstream<NT, RB, true, NW, U, SW>), grid, dim3(NW * 64), shm, s, a);
    else hipLaunchKernelGGL((k_gemm_wstream<NT, RB, false, NW, U, SW>), grid, dim3(NW * 64), shm, s, a);
  } else {
    if (x_f32) hipLaunchKernelGGL((k_gemm<NT, RB, true, NW, U, SW>), grid, dim3(NW * 64), shm, s, a);
    else hipLaunchKernelGGL((k_gemm<NT, RB, false, NW, U, SW>), grid, dim3(NW * 64), shm, s, a);
  }
}

// 17..64-row fp32-X grid kernels (gemm_impl's mid path): X packed by its producer takes k_gemm_xp
template <int NT, int RB, int NW, bool SW>
void launch_mid(dim3 grid, const GemmArgs& a, hipStream_t s) {
  if constexpr (!SW) {
    if (a.xph) {
      hipLaunchKernelGGL((k_gemm_xp<NT, RB, NW, 2>), grid, dim3(NW * 64), 0, s, a);
      return;
    }
  }
  hipLaunchKernelGGL((k_gemm_wstream<NT, RB, true, NW, 2, SW>), grid, dim3(NW * 64), 0, s, a);
}

thread_local unsigned long long* g_trc = nullptr;  // fo_gemm_set_trace (probes)
int g_xs_var = -1;   // fo_gemm_set_xs_variant (probes); -1: FO_XS_VARIANT (0-4) decides at first use, default 0
inline int xs_variant() {
  if (g_xs_var < 0) {
    const char* e = getenv("FO_XS_VARIANT");
    g_xs_var = (e && e[0] >= '0' && e[0] <= '4') ? e[0] - '0' : 0;
  }
  return g_xs_var;
}
// packed activations armed for the calling thread's next launch, with their extent (cols, allocated row blocks)
struct PackArm {
  const void* p0 = nullptr;
  const void* p1 = nullptr;
  int cols = 0, cap_rb = 0;
};
thread_local PackArm g_xpk;    // fo_gemm_set_xpack: the next launch's packed X (hi, lo)
thread_local PackArm g_ypk;    // fo_gemm_set_ypack: the next launch's packed yg / Y output (hi, lo)
thread_local PackArm g_yp32k;  // fo_gemm_set_ypack32 / _xpack32: fp32 fragment-order copies
thread_local PackArm g_xp32k;
inline int arm_pack(PackArm& g, const void* p0, const void* p1, bool two, int cols, int cap_rb, const char* what) {
  g = PackArm{};
  FO_REQUIRE(!two || (p0 == nullptr) == (p1 == nullptr), "%s: both halves or neither", what);
  if (!p0) return 0;
  FO_REQUIRE(cols > 0 && (cols & 31) == 0 && cap_rb >= 1 && cap_rb <= 4,
             "%s: cols %d (a multiple of 32) and 1..4 row blocks (%d) required", what, cols, cap_rb);
  g = PackArm{p0, p1, cols, cap_rb};
  return 0;
}
// the launch's check of an armed pack against what it reads (cols = its K) or writes (cols = its N) at M rows
#define FO_PACK_FITS(pk, want_cols, M, what)                                                                         \
  FO_REQUIRE(!(pk).p0 || ((pk).cols == (want_cols) && (pk).cap_rb * 16 >= (M)),                                 \
             "%s: packed buffer of %d columns x %d row blocks armed for a launch of %d columns x %d rows", what, \
             (pk).cols, (pk).cap_rb, (want_cols), (M))

// forced (waves, tiles per workgroup) of the M <= 16 kernels; 0 = automatic (sweeps only)
thread_local int g_force_nw = 0, g_force_nt = 0;
// k-steps in flight per wave of the one-row-tile fp32-X grid kernel: 4 (default), 7 on 16 waves or 8 on 8
// waves (every k-step of a wave's K range in one round when waves x U covers K: the Qwen2 o / q|k|v
// projections, K = 3584 = 16 x 7 x 32); 0 = the policy in gemm_impl
thread_local int g_force_u = 0;
thread_local int g_launch_u = 4;

template <int NT, int RB, bool SW>
void launch_nw(int nw, bool wstream, bool x_f32, dim3 grid, const GemmArgs& a, hipStream_t s) {
  if constexpr (RB == 1 && NT <= 2) {
    if (g_launch_u != 4 && x_f32 && !g_launch_pipe) {
      if constexpr (NT == 1) {  // (2 tiles x 7 k-steps on 16 waves spill past the 128-VGPR budget: 8 x 8 instead)
        if (g_launch_u == 7) {
          hipLaunchKernelGGL((k_gemm<1, 1, true, 16, 7, SW>), grid, dim3(1024), 0, s, a);
          return;
        }
      }
      hipLaunchKernelGGL((k_gemm<NT, 1, true, 8, 8, SW>), grid, dim3(512), 0, s, a);
      return;
    }
  }
  if constexpr (NT >= 7) {  // 7-8 tiles x 16 waves exceed the 128-VGPR budget of a 1024-thread group
    if (nw == 16) nw = 8;
  } else if (nw == 16) {
    launch_gemm<NT, RB, 16, 4, SW>(wstream, x_f32, grid, a, s);
    return;
  }
  if (nw == 8) launch_gemm<NT, RB, 8, 4, SW>(wstream, x_f32, grid, a, s);
  else launch_gemm<NT, RB, 4, 4, SW>(wstream, x_f32, grid, a, s);
}

// X-stationary weight stream for M <= 16 fp32 rows and K = NW * KPW * 32 (Qwen2: K = 3584 = 16 x 7 x 32).
// One workgroup per CU (the LDS footprint admits one), persistent over a contiguous, balanced range of
// column units (2 packed tiles: a gate/up pair; the plain and RoPE unit forms measured slower than the grid
// kernels on the 26-33 MB projections and are not built).
//  * prologue: wave w loads ITS K slice of X once, split into bf16 hi (kept in VGPRs) and lo (kept in
//    the wave's private LDS region) -- X never goes through the vector-memory path again, so the weight
//    stream is the only VMEM traffic (the fo_gemm grid re-reads X from L2 once per column group);
//  * steady state: per unit, two tiles' weight fragments (KPW x 1 KiB per wave each) are double
//    buffered -- the next unit's loads are issued right after the MFMAs that free a buffer;
//  * per unit the NW partial tiles are reduced through LDS (two barriers), then the epilogue of the
//    row-major output (the post-scaled RMSNorm and SwiGLU) as in gemm_body.
// 16 waves x 7 k-steps (round 5, scripts/xs_variant_probe.py: 47.0-47.3 us per 271.6 MB launch against 48.6-49.5 us
// for round 4's 8 x 14, graph-replayed over cold weight copies); FO_XS_VARIANT=3 runs the 8 x 14 shape
constexpr int XS_NW = 16, XS_KPW = 7;
// VAR (probes, fo_gemm_set_xs_variant): bit 0 = no cross-wave reduction (wave 0's partial is stored: WRONG
// results, the barrier-free bound), bit 1 = default cache policy on the weight loads instead of nt, bit 2 = the
// cross-wave reduction without workgroup barriers: per-unit partial slots double-buffered by unit parity, an LDS
// arrival counter per slot; the wave that arrives last sums the NW partials in wave order (the same order, so the
// same bits as the barrier form) and runs the unit's epilogue while the other waves stream on; a wave reuses a slot
// only once the reduction two units back has been consumed (LDS generation word)
template <int NW, int KPW, int VAR = 0>  // the SwiGLU pair (gate, up) of one 16-column output tile per unit
__global__ __launch_bounds__(NW * 64) void k_gemm_xs(GemmArgs a, int units) {
  constexpr bool BF = (VAR & 4) != 0;
  __shared__ bf16x8 xlo[NW][KPW][64];
  __shared__ float part[BF ? 2 : 1][NW][2][16][17];
  __shared__ float rstd_s[16];
  __shared__ int arr_s[2], gen_s[2];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  constexpr int KS = NW * KPW;
  const int ub = (int)((long)units * blockIdx.x / gridDim.x);
  const int ue = (int)((long)units * (blockIdx.x + 1) / gridDim.x);
  // weights of this wave's K slice, tile t, k-step j: byte (t * KS + j) * 1024 (SGPR offset) + this lane's
  // (wave * KPW * 64 + lane) * 16 (one VGPR) through a buffer descriptor (no 64-bit address per load)
  const unsigned long long wbase = (unsigned long long)a.Wp;
  const __amdgpu_buffer_rsrc_t srd = __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<void*>(((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(wbase >> 32)) << 32) |
                              (unsigned)__builtin_amdgcn_readfirstlane((unsigned)wbase)),
      (short)0, __builtin_amdgcn_readfirstlane(a.ntiles * KS * 1024), 0x00020000);
  const int voff = (wave * KPW * 64 + lane) * 16;
  bf16x8 w0[KPW], w1[KPW];
  auto issue = [&](bf16x8 (&w)[KPW], int tile) {
#pragma unroll
    for (int j = 0; j < KPW; ++j)
      w[j] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(srd, voff, (tile * KS + j) * 1024,
                                                                               (VAR & 2) ? 0 : 2));
  };
  issue(w0, ub < ue ? 2 * ub : a.ntiles);
  issue(w1, ub < ue ? 2 * ub + 1 : a.ntiles);
  // X slice (hi in registers, lo in LDS); rows >= M clamp to the last row (computed, never stored)
  bf16x8 xh[KPW];
  if (a.xph) {   // X packed by its producer (GemmArgs::xph / xpl): the fragments as they are
#pragma unroll
    for (int j = 0; j < KPW; ++j) {
      xh[j] = a.xph[(size_t)(wave * KPW + j) * 64 + lane];
      xlo[wave][j][lane] = a.xpl[(size_t)(wave * KPW + j) * 64 + lane];
    }
  } else {
    const int row = min(lane & 15, a.M - 1);
    const float* xp = reinterpret_cast<const float*>(a.X) + (size_t)row * a.ldx + 8 * (lane >> 4) +
                      (size_t)wave * KPW * 32;
    // the k-steps' loads in groups of XG issued before any is used (one load behind the previous one's LDS store
    // each was KPW round trips before the first unit, r05zv); XG bounded by the 128-VGPR budget of 16 waves
    constexpr int XG = KPW > 4 ? (KPW + 1) / 2 : KPW;
#pragma unroll
    for (int j0 = 0; j0 < KPW; j0 += XG) {
      float4 p[XG][2];
#pragma unroll
      for (int g = 0; g < XG; ++g)
        if (j0 + g < KPW) {
          p[g][0] = reinterpret_cast<const float4*>(xp + (j0 + g) * 32)[0];
          p[g][1] = reinterpret_cast<const float4*>(xp + (j0 + g) * 32)[1];
        }
#pragma unroll
      for (int g = 0; g < XG; ++g)
        if (j0 + g < KPW) {
          const int j = j0 + g;
          const float f[8] = {p[g][0].x, p[g][0].y, p[g][0].z, p[g][0].w, p[g][1].x, p[g][1].y, p[g][1].z, p[g][1].w};
          bf16x8 lo;
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const __bf16 h = (__bf16)f[i];
            xh[j][i] = h;
            lo[i] = (__bf16)(f[i] - (float)h);
          }
          xlo[wave][j][lane] = lo;
        }
    }
  }
  if (a.rstats) {  // RMSNorm consumer: rstd of each row from the producer's partial sums
    for (int rr = wave; rr < 16; rr += NW) {
      const int m = min(rr, a.M - 1);
      float v = 0.f;
      for (int j = lane; j < a.rgroups; j += 64) v += a.rstats[(size_t)m * a.rgroups + j];
      v = wave_sum(v);
      if (lane == 0) rstd_s[rr] = rsqrtf(v / (float)a.K + a.reps);
    }
  }
  if constexpr (BF) {
    if (threadIdx.x < 2) {
      arr_s[threadIdx.x] = 0;
      gen_s[threadIdx.x] = 0;
    }
    __syncthreads();   // rstd_s and the counters, once (the only workgroup barrier of this form)
  }
  auto compute = [&](bf16x8 (&w)[KPW]) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < KPW; ++j) {
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xh[j], w[j], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xlo[wave][j][lane], w[j], acc, 0, 0, 0);
    }
    return acc;
  };
  for (int u = ub; u < ue; ++u) {
    // the next unit's loads are issued unconditionally (the compiler's in-order vmcnt accounting then
    // waits only for the buffer it consumes); past the last unit they address tile `ntiles`, beyond the
    // descriptor's range, which the hardware drops without touching memory
    const int nxt = u + 1 < ue ? 2 * (u + 1) : a.ntiles;
    const f32x4 c0 = compute(w0);
    issue(w0, nxt);
    const f32x4 c1 = compute(w1);
    issue(w1, nxt + (u + 1 < ue ? 1 : 0));
    if constexpr ((VAR & 1) != 0) {   // probe: no cross-wave reduction (the barrier-free bound; wrong results)
      if (wave == 0 && lane < 16)
        for (int i = 0; i < 4; ++i)
          if (4 * 0 + i < a.M) epilogue_store(a, true, i, u * 16 + lane, c0[i], c1[i]);
      continue;
    }
    if constexpr (BF) {
      const int k = u - ub, sl = k & 1;
      // the slot's previous unit (k - 2) must have been reduced: its reducer bumps gen_s[sl] once done reading
      if (k >= 2) {
        while (__hip_atomic_load(&gen_s[sl], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < (k >> 1))
          __builtin_amdgcn_s_sleep(1);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        part[sl][wave][0][4 * (lane >> 4) + i][lane & 15] = c0[i];
        part[sl][wave][1][4 * (lane >> 4) + i][lane & 15] = c1[i];
      }
      // LDS only: a wave's ds operations execute in order, so its partial writes land before its counter add; the
      // asm orders the compiler and waits for them (no vmcnt wait: the weight loads stay in flight)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      int old = 0;
      if (lane == 0) old = __hip_atomic_fetch_add(&arr_s[sl], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      old = __builtin_amdgcn_readfirstlane(old);
      if (old != NW - 1) continue;   // another wave reduces this unit
      asm volatile("" ::: "memory");
      if (lane == 0) __hip_atomic_store(&arr_s[sl], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      // this wave: the unit's 16 x 16 outputs, 4 per lane (rows 4 (lane >> 4) .. + 3, column lane & 15)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int rr = 4 * (lane >> 4) + i, c = lane & 15;
        float x1 = 0.f, x2 = 0.f;
#pragma unroll
        for (int w = 0; w < NW; ++w) {
          x1 += part[sl][w][0][rr][c];
          x2 += part[sl][w][1][rr][c];
        }
        if (a.rstats) {
          x1 *= rstd_s[rr];
          x2 *= rstd_s[rr];
        }
        const int n = u * 16 + c;
        if (rr < a.M && n < a.N) epilogue_store(a, true, rr, n, x1, x2);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the partial reads are done: the slot is free
      if (lane == 0) __hip_atomic_fetch_add(&gen_s[sl], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      continue;
    } else {
    __syncthreads();  // the previous unit's epilogue has read part[]
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      part[0][wave][0][4 * (lane >> 4) + i][lane & 15] = c0[i];
      part[0][wave][1][4 * (lane >> 4) + i][lane & 15] = c1[i];
    }
    __syncthreads();
    }
    const int e = threadIdx.x;
    if (e < 256) {
      const int rr = e >> 4, c = e & 15;
      float x1 = 0.f, x2 = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) {
        x1 += part[0][w][0][rr][c];
        x2 += part[0][w][1][rr][c];
      }
      if (a.rstats) {
        x1 *= rstd_s[rr];
        x2 *= rstd_s[rr];
      }
      const int n = u * 16 + c;
      if (rr < a.M && n < a.N) epilogue_store(a, true, rr, n, x1, x2);
    }
  }
}

// ---- probe (verdict r04 item 4: where a persistent layer would win or lose): the o -> gate/up seam of a Qwen2 layer
// at <= 16 rows as ONE launch.  Workgroups [0, n_o) are the o projection (one tile pair each, 8 waves x 14 k-steps
// over K = 3584, + residual, writing Y, yg = Y * gamma_next and the row's sum of squares per pair), then publish
// (release fence + relaxed add on `ready`); workgroups [n_o, n_o + G) are k_gemm_xs's gate/up stream: they issue
// their first two tiles' weights, then wave 0 polls `ready` (acquire; a bounded poll: past ~0.1 s the launch
// proceeds and flags *ready_timeout, so a broken producer cannot hang the GPU), then the X slice (yg) and the rstd
// from the o workgroups' partials, and the unit loop.  The dispatcher places workgroups in id order, so every o
// workgroup is resident before any gate/up workgroup waits, and none of them waits on anything: the poll always ends.
// Per-workgroup wall clocks (trc[4 w + 0..3]: start, weights of the first units issued / o reduced, ready seen /
// o stored, end).  Same math as the two launches (o reduced in a different K order: ~1 ulp differences).
__global__ __launch_bounds__(512) void k_seam_o_gu(GemmArgs ao, GemmArgs ag, int n_o, int units, int G, int* ready,
                                                   int* ready_timeout, unsigned long long* trc) {
  constexpr int NW = 8, KPW = 14, KS = NW * KPW;
  __shared__ bf16x8 xlo[NW][KPW][64];
  __shared__ float part[NW][2][16][17];
  __shared__ float rstd_s[16];
  __shared__ float rs_s[16][2];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wg = blockIdx.x;
  unsigned long long* tr = trc ? trc + (size_t)wg * 4 : nullptr;
  if (tr && threadIdx.x == 0) tr[0] = wall_clock64();
  const bool is_o = wg < n_o;
  const GemmArgs& a = is_o ? ao : ag;
  const unsigned long long wbase = (unsigned long long)a.Wp;
  const __amdgpu_buffer_rsrc_t srd = __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<void*>(((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(wbase >> 32)) << 32) |
                              (unsigned)__builtin_amdgcn_readfirstlane((unsigned)wbase)),
      (short)0, __builtin_amdgcn_readfirstlane(a.ntiles * KS * 1024), 0x00020000);
  const int voff = (wave * KPW * 64 + lane) * 16;
  bf16x8 w0[KPW], w1[KPW];
  auto issue = [&](bf16x8 (&w)[KPW], int tile) {
#pragma unroll
    for (int j = 0; j < KPW; ++j)
      w[j] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(srd, voff, (tile * KS + j) * 1024, 2));
  };
  const int gj = wg - n_o;
  const int ub = is_o ? wg : (int)((long)units * gj / G);
  const int ue = is_o ? wg + 1 : (int)((long)units * (gj + 1) / G);
  issue(w0, ub < ue ? 2 * ub : a.ntiles);
  issue(w1, ub < ue ? 2 * ub + 1 : a.ntiles);
  if (!is_o) {   // wait for every o workgroup's stores (bounded)
    if (threadIdx.x == 0) {
      long spins = 0;
      while (__hip_atomic_load(ready, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < n_o) {
        __builtin_amdgcn_s_sleep(2);
        if (++spins > (1l << 22)) {
          *ready_timeout = 1;
          break;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      if (tr) tr[2] = wall_clock64();
    }
    __syncthreads();
  }
  // X slice of this wave's k-steps (o: the attention output; gate/up: yg), hi in VGPRs, lo in LDS
  bf16x8 xh[KPW];
  {
    const int row = min(lane & 15, a.M - 1);
    const float* xp = reinterpret_cast<const float*>(a.X) + (size_t)row * a.ldx + 8 * (lane >> 4) + (size_t)wave * KPW * 32;
#pragma unroll
    for (int j = 0; j < KPW; ++j) {
      const float4 p0 = reinterpret_cast<const float4*>(xp + j * 32)[0];
      const float4 p1 = reinterpret_cast<const float4*>(xp + j * 32)[1];
      const float f[8] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w};
      bf16x8 lo;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const __bf16 h = (__bf16)f[i];
        xh[j][i] = h;
        lo[i] = (__bf16)(f[i] - (float)h);
      }
      xlo[wave][j][lane] = lo;
    }
  }
  if (!is_o) {   // rstd of each row from the o workgroups' partial sums of squares
    for (int rr = wave; rr < 16; rr += NW) {
      const int m = min(rr, a.M - 1);
      float v = 0.f;
      for (int j = lane; j < a.rgroups; j += 64) v += a.rstats[(size_t)m * a.rgroups + j];
      v = wave_sum(v);
      if (lane == 0) rstd_s[rr] = rsqrtf(v / (float)a.K + a.reps);
    }
  }
  auto compute = [&](bf16x8 (&w)[KPW]) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < KPW; ++j) {
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xh[j], w[j], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xlo[wave][j][lane], w[j], acc, 0, 0, 0);
    }
    return acc;
  };
  for (int u = ub; u < ue; ++u) {
    const int nxt = u + 1 < ue ? 2 * (u + 1) : a.ntiles;
    const f32x4 c0 = compute(w0);
    issue(w0, nxt);
    const f32x4 c1 = compute(w1);
    issue(w1, nxt + (u + 1 < ue ? 1 : 0));
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      part[wave][0][4 * (lane >> 4) + i][lane & 15] = c0[i];
      part[wave][1][4 * (lane >> 4) + i][lane & 15] = c1[i];
    }
    __syncthreads();
    if (is_o && tr && threadIdx.x == 0) tr[1] = wall_clock64();
    const int e = threadIdx.x;
    if (e < 512) {
      const int t = e >> 8, rr = (e >> 4) & 15, c = e & 15;   // o: both tiles of the pair; gate/up: the SwiGLU pair
      float x1 = 0.f, x2 = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) {
        x1 += part[w][is_o ? t : 0][rr][c];
        x2 += part[w][1][rr][c];
      }
      if (is_o) {
        const int n = (2 * u + t) * 16 + c;
        float y = 0.f;
        if (rr < a.M && n < a.N) {
          const size_t o = (size_t)rr * a.ldy + n;
          y = x1 + (a.bias ? a.bias[n] : 0.f) + reinterpret_cast<float*>(a.Y)[o];
          reinterpret_cast<float*>(a.Y)[o] = y;
          a.yg[o] = y * a.gnext[n];
        }
        // the row's sum of squares over this pair's 32 columns: 16 lanes of each tile's row, then the two tiles
        float q = y * y;
#pragma unroll
        for (int off = 8; off > 0; off >>= 1) q += __shfl_xor(q, off, 16);
        if (c == 0) rs_s[rr][t] = q;
      } else if (e < 256) {
        if (a.rstats) {
          x1 *= rstd_s[rr];
          x2 *= rstd_s[rr];
        }
        const int n = u * 16 + c;
        if (rr < a.M && n < a.N) epilogue_store(a, true, rr, n, x1, x2);
      }
    }
    if (is_o) {
      __syncthreads();
      if (threadIdx.x < 16 && (int)threadIdx.x < a.M)
        a.sout[(size_t)threadIdx.x * n_o + wg] = rs_s[threadIdx.x][0] + rs_s[threadIdx.x][1];
    }
  }
  if (is_o) {   // publish
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      if (tr) tr[2] = wall_clock64();
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_fetch_add(ready, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (tr && threadIdx.x == 0) tr[3] = wall_clock64();
}

// X-stationary weight stream for 17..64 fp32 rows (RB = 2..4 row blocks): k_gemm_xs's design with the K range
// split over workgroups, because RB row blocks of X split into bf16 hi + lo no longer fit one CU for the whole K
// (16 rows x 3584 x 4 B = 229 KB per row block).  Split s owns k-steps [s * NW * KPW, (s + 1) * NW * KPW); wave w
// of it KPW of them, whose X fragments of all RB row blocks it loads once (hi in VGPRs, lo in its LDS region).
// Units are packed tile pairs (a gate/up pair, or two adjacent plain / RoPE tiles), double buffered as in
// k_gemm_xs; per unit the NW partial tiles are reduced through LDS and stored as split s's partial slab, and
// k_gemm_reduce (the next launch) sums the slabs in split order and runs the epilogue (SwiGLU, RMSNorm rstd,
// RoPE + paged-KV append, residual, row statistics).  k-steps past K (the last split of a long-K layer) load
// nothing and multiply zero X.
template <int NW, int KPW, int RB, int UA>   // UA units (2 UA tile buffers) of weights in flight per wave
__global__ __launch_bounds__(NW * 64) void k_gemm_xsk(GemmArgs a, int units, int G) {
  // the per-unit cross-wave reduction holds both tiles when the LDS allows, else one tile at a time
  constexpr int PT = (NW * RB * KPW * 1024 + NW * 2 * RB * 16 * 17 * 4 <= 160 * 1024) ? 2 : 1;
  __shared__ bf16x8 xlo[NW][RB][KPW][64];
  __shared__ float part[NW][PT][RB * 16][17];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  constexpr int KW = NW * KPW;
  constexpr int ROWS = RB * 16;
  constexpr int NB = 2 * UA;
  const int KS = a.K >> 5;
  // XCD-aware placement: the S x G (split, column group) workgroups are dealt to the 8 XCDs (workgroup id % 8) in
  // contiguous runs of the split-major order, so a split's column groups share one XCD (at most two): its X slice
  // comes from HBM once and from that XCD's L2 after, instead of once per XCD (r04zs FETCH: the 40-row down read
  // X ~8x, 160.2 MB per launch against 138.8 MB)
  const int total = a.S * G, per_x = (total + 7) >> 3;
  const int w = (int)(blockIdx.x & 7) * per_x + (int)(blockIdx.x >> 3);
  if (w >= total) return;   // (the grid is 8 per_x: the padding workgroups leave before any barrier)
  const int sp = w / G, gx = w - sp * G;
  const int ub = (int)((long)units * gx / G);
  const int ue = (int)((long)units * (gx + 1) / G);
  // probe library only (FO_GEMM_TRACE): {wall start, wall X staged, wall end, compute cycles, reduce cycles, units}
  unsigned long long* const tr = (FO_GEMM_TRACE && a.trc) ? a.trc + 8 * (size_t)blockIdx.x : nullptr;
  unsigned long long t_comp = 0, t_red = 0;
  if (tr && threadIdx.x == 0) tr[0] = wall_clock64();
  const int ks0 = sp * KW + wave * KPW;                 // this wave's first k-step
  const int nj = max(0, min(KPW, KS - ks0));            // its k-steps inside K (wave-uniform)
  const unsigned long long wbase = (unsigned long long)a.Wp;
  const __amdgpu_buffer_rsrc_t srd = __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<void*>(((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(wbase >> 32)) << 32) |
                              (unsigned)__builtin_amdgcn_readfirstlane((unsigned)wbase)),
      (short)0, __builtin_amdgcn_readfirstlane(a.ntiles * KS * 1024), 0x00020000);
  const int voff = (ks0 * 64 + lane) * 16;
  // the weight stream's depth sets its rate (a CU's share of HBM ~ its bytes in flight): k_gemm_xs keeps 2 x 14 KiB
  // per wave in flight; with KPW = 7 k-steps per wave this kernel keeps 2 UA tiles' fragments in flight instead
  bf16x8 wb[NB][KPW];
  auto issue = [&](bf16x8 (&w)[KPW], int tile) {   // tile >= 2 ue: past the workgroup's range -> no load issued
    if (tile < 2 * ue) {
#pragma unroll
      for (int j = 0; j < KPW; ++j)
        if (j < nj)
          w[j] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(srd, voff, (tile * KS + j) * 1024, 2));
    }
  };
  bf16x8 zero;
#pragma unroll
  for (int i = 0; i < 8; ++i) zero[i] = (__bf16)0.f;
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int j = 0; j < KPW; ++j)
      if (j >= nj) wb[b][j] = zero;   // k-steps past K: no weights loaded, zero fragments
#pragma unroll
  for (int b = 0; b < NB; ++b) issue(wb[b], 2 * ub + b);
  bf16x8 xh[RB][KPW];
#pragma unroll
  for (int r = 0; r < RB; ++r) {
    const int row = min(r * 16 + (lane & 15), a.M - 1);   // rows >= M: computed, never stored by the reduce
    const float* xp = reinterpret_cast<const float*>(a.X) + (size_t)row * a.ldx + 8 * (lane >> 4) + (size_t)ks0 * 32;
#pragma unroll
    for (int j = 0; j < KPW; ++j) {
      bf16x8 hi = zero, lo = zero;
      if (j < nj) {
        const float4 p0 = reinterpret_cast<const float4*>(xp + j * 32)[0];
        const float4 p1 = reinterpret_cast<const float4*>(xp + j * 32)[1];
        const float f[8] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w};
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const __bf16 h = (__bf16)f[i];
          hi[i] = h;
          lo[i] = (__bf16)(f[i] - (float)h);
        }
      }
      xh[r][j] = hi;
      xlo[wave][r][j][lane] = lo;
    }
  }
  auto compute = [&](bf16x8 (&w)[KPW], f32x4 (&acc)[RB]) {
#pragma unroll
    for (int r = 0; r < RB; ++r) acc[r] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < KPW; ++j)
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        acc[r] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xh[r][j], w[j], acc[r], 0, 0, 0);
        acc[r] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xlo[wave][r][j][lane], w[j], acc[r], 0, 0, 0);
      }
  };
  const int Ncols = a.ntiles * 16;
  float* slab = a.ws + (size_t)sp * ROWS * Ncols;
  if (tr && threadIdx.x == 0) tr[1] = wall_clock64();
  for (int u0 = ub; u0 < ue; u0 += UA) {
#pragma unroll
    for (int q = 0; q < UA; ++q) {
      const int u = u0 + q;
      if (u < ue) {   // workgroup-uniform: the barriers below are reached by every wave
        const unsigned long long c0 = tr ? clock64() : 0;
        f32x4 c[2][RB];
        compute(wb[2 * q], c[0]);
        issue(wb[2 * q], 2 * (u + UA));
        compute(wb[2 * q + 1], c[1]);
        issue(wb[2 * q + 1], 2 * (u + UA) + 1);
        const unsigned long long c1 = tr ? clock64() : 0;
#pragma unroll
        for (int t0 = 0; t0 < 2; t0 += PT) {
          __syncthreads();  // the previous reduction has read part[]
#pragma unroll
          for (int p = 0; p < PT; ++p)
#pragma unroll
            for (int r = 0; r < RB; ++r)
#pragma unroll
              for (int i = 0; i < 4; ++i) part[wave][p][r * 16 + 4 * (lane >> 4) + i][lane & 15] = c[t0 + p][r][i];
          __syncthreads();
          for (int e = threadIdx.x; e < PT * ROWS * 16; e += NW * 64) {
            const int p = e / (ROWS * 16), rr = (e >> 4) % ROWS, cc = e & 15;
            float v = 0.f;
#pragma unroll
            for (int w = 0; w < NW; ++w) v += part[w][p][rr][cc];
            slab[(size_t)rr * Ncols + (2 * u + t0 + p) * 16 + cc] = v;
          }
        }
        if (tr) {
          t_comp += c1 - c0;
          t_red += clock64() - c1;
        }
      }
    }
  }
  if (tr && threadIdx.x == 0) {
    tr[2] = wall_clock64();
    tr[3] = t_comp;
    tr[4] = t_red;
    tr[5] = (unsigned long long)(ue - ub);
  }
}

// ---- 65..128-row weight streams (k_gemm_rows): the weights once, every row block on the matrix cores.
// A listen group of C chunks x 8 users x 2 tokens puts 128 rows through every Qwen2 GEMM (fo.engine.ListenGroupGraph,
// C = 8); the X-stationary kernels hold X per K-slice wave and ran 65..128 rows as two 64-row launches (the weights
// twice, k_gemm_xsk's per-unit cross-wave reduction each time).  Here the NWV waves of a workgroup split the ROWS
// (wave w: row blocks RPW w .. RPW w + RPW - 1; shipped: 8 waves x 1 row block) and share each k-step's weight
// fragments through LDS, so there is no cross-wave reduction and each weight byte is read from HBM once:
//  * one LDS-DMA loader ring per workgroup (global_load_lds_dwordx4, issued by every wave for its share): DW k-steps
//    of the workgroup's NTC weight tiles ahead, DX k-steps of its fp32 X rows ahead (X comes from L2; XL = 1: each X
//    load fetches 8 whole rows, laid out so the consumers' reads stay conflict-free);
//  * per k-step: one s_waitcnt on this wave's own DMA (the count of the DX - 1 younger k-steps' loads, fixed by
//    padding every k-step to the same number of loads), one workgroup barrier (every wave's loads landed, and every
//    wave is past the slot the next loads overwrite), then the wave's X fragment split into bf16 hi / lo and
//    2 RPW MFMAs per tile;
//  * workgroups = S K-splits x G tile groups (XCD-aware as k_gemm_xsk); each writes its fp32 partial tiles to split
//    sp's slab and k_gemm_reduce (the next launch) sums the slabs in split order and runs every epilogue (SwiGLU, the
//    RMSNorm rstd, residual, row statistics).  A workgroup's X over its K range passes through the CU beside its
//    weights, so the host splits K until the two are comparable (gemm_impl: gate/up thirds, down 16 slices).
// The loads are asm (the compiler's own wait placement treats an LDS-DMA as aliasing every later LDS read and drains
// the whole ring before each one); nothing else in the loop touches vector memory, so the manual counts are exact.
// (dma16 / lds_addr / wait_vm: fo_common.h)
// this wave's DMA down to N outstanding and its LDS reads done, then the workgroup barrier -- one opaque statement, so
// the compiler moves no LDS access across it (a bare s_barrier builtin orders no memory)
template <int N>
__device__ __forceinline__ void wait_vm_barrier() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"i"(N) : "memory");
}

// PROBE (fo_gemm_set_rows 4 / 5, WRONG results, timing bounds): 1 = no X loads (the weight stream alone), 2 = no loads
// XL: the X DMA's lane -> (row, 16-B chunk) map.  0: lane l fetches row l & 15, chunks 2 (l >> 4) + h of the k-step
// (each load touches 16 rows x half a line); 1: load h fetches rows 8 h .. 8 h + 7 whole (8 full 128-B lines), lane
// f = 8 c + (r & 7) + 8 h (mod 64) holding chunk c of row r, which keeps the consumer's two ds_read_b128 free of
// bank conflicts (its 16-lane groups read 16 consecutive 16-B slots)
// CM: the consumer map.  0: wave w computes row block w (RPW of them) for every tile; 1 (8 waves, RPW 1): wave w
// computes row blocks 2 (w & 3) and 2 (w & 3) + 1 for half the tiles (w >> 2) -- each weight fragment is read from LDS
// by 4 waves instead of 8 (the loads are distributed as for CM 0)
template <int NWV, int RPW, int NTC, int DW, int DX, bool WNT = false, int PROBE = 0, int XL = 0, int CM = 0>
__global__ __launch_bounds__(NWV * 64) void k_gemm_rows(GemmArgs a, int G, int tiles_per) {
  constexpr int RB = NWV * RPW;
  constexpr int LPW = (NTC + NWV - 1) / NWV;   // weight loads per wave per k-step (tile t: wave t % NWV)
  constexpr int PW = DW + 1, PX = DX + 1;
  constexpr int OPS = LPW + 2 * RPW;           // DMA loads per wave per k-step
  __shared__ bf16x8 wr[PW][NTC][64];         // weight ring: one 1 KiB fragment per (k-step slot, tile)
  __shared__ float4 xr[PX][RB][2][64];       // X ring: fp32 rows of each row block, two 16-B halves per lane
  __shared__ float4 dummy[64];               // the padding loads land here
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int KS = a.K >> 5;
  const int total = a.S * G, per_x = (total + 7) >> 3;
  const int wgi = (int)(blockIdx.x & 7) * per_x + (int)(blockIdx.x >> 3);
  if (wgi >= total) return;
  const int sp = wgi / G, gx = wgi - sp * G;
  const int tb = gx * tiles_per, te = min(a.ntiles, tb + tiles_per);
  const int nt = te - tb;   // <= NTC (host)
  const int kb = (int)((long)KS * sp / a.S), ke = (int)((long)KS * (sp + 1) / a.S);
  const int nk = ke - kb;
  const char* wbase = reinterpret_cast<const char*>(a.Wp);
  const float* xbase = reinterpret_cast<const float*>(a.X);
  // this lane's X row of each of the wave's row blocks (rows >= M clamp to M - 1: computed, never stored)
  const float* xrow[RPW][2];
#pragma unroll
  for (int r = 0; r < RPW; ++r)
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      if constexpr (XL == 0) {
        const int row = min((wave * RPW + r) * 16 + (lane & 15), a.M - 1);
        xrow[r][hf] = xbase + (size_t)row * a.ldx + 8 * (lane >> 4) + 4 * hf;
      } else {
        const int row = min((wave * RPW + r) * 16 + 8 * hf + (lane & 7), a.M - 1);
        const int c = ((lane >> 3) - hf) & 7;
        xrow[r][hf] = xbase + (size_t)row * a.ldx + 4 * c;
      }
    }
  // the consumer's two LDS slots (16-B lanes of the two loads' images)
  int xs0, xs1, xh0;
  if constexpr (XL == 0) {
    xh0 = 0;
    xs0 = xs1 = lane;
  } else {
    const int r = lane & 15, q = lane >> 4, h = r >> 3;
    xh0 = h;
    xs0 = (16 * q + (r & 7) + 8 * h) & 63;
    xs1 = (xs0 + 8) & 63;
  }
  const unsigned dummy_l = __builtin_amdgcn_readfirstlane(lds_addr(&dummy[0]));
  const void* dummy_g = wbase + (size_t)lane * 16;
  // weights of k-step i (relative to kb) into ring slot i % PW: this wave's tiles wave, wave + NWV, ...
  auto issue_w = [&](int i) {
    if constexpr (PROBE == 2) return;
#pragma unroll
    for (int q = 0; q < LPW; ++q) {
      const int t = q * NWV + wave;
      if (i < nk && t < nt && t < NTC) {
        const void* src = wbase + ((size_t)(tb + t) * KS + (kb + i)) * 1024 + (size_t)lane * 16;
        dma16<WNT>(src, __builtin_amdgcn_readfirstlane(lds_addr(&wr[i % PW][t][0])));
      } else {
        dma16(dummy_g, dummy_l);
      }
    }
  };
  auto issue_x = [&](int i) {
    if constexpr (PROBE != 0) return;
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
      const int rb = wave * RPW + r;
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        if (i < nk) {
          const void* src = xrow[r][hf] + (size_t)(kb + i) * 32;
          dma16(src, __builtin_amdgcn_readfirstlane(lds_addr(&xr[i % PX][rb][hf][0])));
        } else {
          dma16(dummy_g, dummy_l);
        }
      }
    }
  };
  static_assert(CM == 0 || (NWV == 8 && RPW == 1), "k_gemm_rows: the split consumer map is for 8 waves x 1 block");
  constexpr int RBW = CM ? 2 : RPW;                 // row blocks a wave computes
  constexpr int NTW = CM ? (NTC + 1) / 2 : NTC;     // tiles a wave computes
  const int rbw0 = CM ? 2 * (wave & 3) : wave * RPW;
  const int tw0 = CM ? (wave >> 2) * NTW : 0;
  f32x4 acc[NTW][RBW];
#pragma unroll
  for (int t = 0; t < NTW; ++t)
#pragma unroll
    for (int r = 0; r < RBW; ++r) acc[t][r] = f32x4{0.f, 0.f, 0.f, 0.f};
  // prologue in the loop's issue order (k-step j - DW's weights, then k-step j - DX's X, for j = 0 .. DW - 1) so every
  // k-step's wait below sees the same number of younger loads; X of negative k-steps: padding loads
  for (int j = 0; j < DW; ++j) {
    issue_w(j);
    if (j - (DW - DX) >= 0) issue_x(j - (DW - DX));
    else {
#pragma unroll
      for (int q = 0; q < 2 * RPW; ++q)
        if constexpr (PROBE == 0) dma16(dummy_g, dummy_l);
    }
  }
  for (int i = 0; i < nk; ++i) {
    // this wave's loads of k-step i (weights and X) have landed; after the barrier every wave's have, and every wave
    // is done reading k-step i - 1's slots, which the loads below overwrite
    wait_vm_barrier<PROBE == 0 ? (DX - 1) * OPS : (PROBE == 1 ? (DW - 1) * LPW : 0)>();
    issue_w(i + DW);
    issue_x(i + DX);
    // every read of the k-step issued before the first MFMA (one latency per k-step); tiles past the workgroup's nt
    // and row blocks past M are computed on whatever the slots hold and never stored (no branch in the loop)
    float4 xp[RBW][2];
#pragma unroll
    for (int r = 0; r < RBW; ++r) {
      if constexpr (XL == 0) {
        xp[r][0] = xr[i % PX][rbw0 + r][0][lane];
        xp[r][1] = xr[i % PX][rbw0 + r][1][lane];
      } else {
        xp[r][0] = xr[i % PX][rbw0 + r][xh0][xs0];
        xp[r][1] = xr[i % PX][rbw0 + r][xh0][xs1];
      }
    }
    bf16x8 xh[RBW], xl[RBW];
#pragma unroll
    for (int r = 0; r < RBW; ++r) {
      const float f[8] = {xp[r][0].x, xp[r][0].y, xp[r][0].z, xp[r][0].w,
                          xp[r][1].x, xp[r][1].y, xp[r][1].z, xp[r][1].w};
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const __bf16 h = (__bf16)f[e];
        xh[r][e] = h;
        xl[r][e] = (__bf16)(f[e] - (float)h);
      }
    }
    // the weight fragments in groups of TG (all of them up to 20 tiles: VGPRs), each group's hi products of every
    // (tile, row block) and then the lo ones: no accumulator is read right after it is written
    constexpr int TG = NTW * RBW <= 20 ? NTW : (NTW + 1) / 2;
#pragma unroll
    for (int t0 = 0; t0 < NTW; t0 += TG) {
      bf16x8 wf[TG];
#pragma unroll
      for (int t = 0; t < TG; ++t)
        if (t0 + t < NTW) wf[t] = wr[i % PW][min(tw0 + t0 + t, NTC - 1)][lane];
#pragma unroll
      for (int t = 0; t < TG; ++t)
        if (t0 + t < NTW)
#pragma unroll
          for (int r = 0; r < RBW; ++r)
            acc[t0 + t][r] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xh[r], wf[t], acc[t0 + t][r], 0, 0, 0);
#pragma unroll
      for (int t = 0; t < TG; ++t)
        if (t0 + t < NTW)
#pragma unroll
          for (int r = 0; r < RBW; ++r)
            acc[t0 + t][r] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xl[r], wf[t], acc[t0 + t][r], 0, 0, 0);
    }
  }
  wait_vm<0>();   // (the padding loads past the last k-step) nothing of this workgroup's DMA outlives it
  const int Ncols = a.ntiles * 16;
  const int ROWS = RB * 16;
  float* slab = a.ws + (size_t)sp * ROWS * Ncols;
#pragma unroll
  for (int t = 0; t < NTW; ++t)
    if (tw0 + t < nt && tw0 + t < NTC)
#pragma unroll
      for (int r = 0; r < RBW; ++r)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int row = (rbw0 + r) * 16 + 4 * (lane >> 4) + e;
          if (row < a.M) slab[(size_t)row * Ncols + (tb + tw0 + t) * 16 + (lane & 15)] = acc[t][r][e];
        }
}

// ---- 33..128-row weight streams, second form (k_gemm_wrow): each wave owns ONE weight tile over the workgroup's K
// range and streams its fragments straight into registers DW k-steps ahead (a register ring, compiler-counted loads,
// ~DW KiB in flight per wave), while the X rows of the k-step are staged once per workgroup through LDS, already
// split into bf16 hi / lo (row block r loaded and converted by wave r): per k-step a workgroup ingests its tiles' 1 KiB
// fragments from HBM and ONE copy of the k-step's X from L2 -- k_gemm_rows (waves split the rows) pulled every tile
// through an LDS-DMA ring of at most ~60 KiB in flight and read X fp32 per wave.  One barrier per k-step (the X slot
// double-buffered); no cross-wave reduction; partial tiles into split sp's slab, k_gemm_reduce runs the epilogue.
template <int NWV, int RB, int DW, int DXS>
__global__ __launch_bounds__(NWV * 64) void k_gemm_wrow(GemmArgs a, int G) {
  static_assert(DW % DXS == 0 && DW % 2 == 0 && RB <= NWV, "k_gemm_wrow: ring shapes");
  __shared__ bf16x8 xhi[2][RB][64], xlo[2][RB][64];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;   // (uniform: SGPR offsets)
  const int KS = a.K >> 5;
  const int total = a.S * G, per_x = (total + 7) >> 3;
  const int wgi = (int)(blockIdx.x & 7) * per_x + (int)(blockIdx.x >> 3);
  if (wgi >= total) return;
  const int sp = wgi / G, gx = wgi - sp * G;
  const int tile = gx * NWV + wave;
  const bool live = tile < a.ntiles;
  const int kb = (int)((long)KS * sp / a.S), ke = (int)((long)KS * (sp + 1) / a.S);
  const int nk = ke - kb;
  // weight fragments through a buffer descriptor: k-steps past the split or a tile past ntiles address beyond its
  // range, which the hardware drops (zeros, no memory access)
  const unsigned long long wbase = (unsigned long long)a.Wp;
  const __amdgpu_buffer_rsrc_t srd = __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<void*>(((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(wbase >> 32)) << 32) |
                              (unsigned)__builtin_amdgcn_readfirstlane((unsigned)wbase)),
      (short)0, __builtin_amdgcn_readfirstlane(a.ntiles * KS * 1024), 0x00020000);
  const int voff = lane * 16;
  const int beyond = a.ntiles * KS * 1024;
  auto ldw = [&](int i) -> bf16x8 {
    const int so = (live && i < nk) ? (tile * KS + kb + i) * 1024 : beyond;
    return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(srd, voff, so, 2));
  };
  // X staging: wave r < RB loads row block r's fragment of each k-step (lane: row 16 r + (l & 15), 8 columns)
  const bool stager = wave < RB;
  const int xrow = min(wave * 16 + (lane & 15), a.M - 1);
  const float* xp = reinterpret_cast<const float*>(a.X) + (size_t)xrow * a.ldx + 8 * (lane >> 4) + (size_t)kb * 32;
  auto ldx2 = [&](int i, float4 (&q)[2]) {
    if (stager && i < nk) {
      q[0] = reinterpret_cast<const float4*>(xp + (size_t)i * 32)[0];
      q[1] = reinterpret_cast<const float4*>(xp + (size_t)i * 32)[1];
    }
  };
  bf16x8 wq[DW];
  float4 xq[DXS][2];
#pragma unroll
  for (int j = 0; j < DW; ++j) wq[j] = ldw(j);
#pragma unroll
  for (int j = 0; j < DXS; ++j) ldx2(j, xq[j]);
  f32x4 acc[RB];
#pragma unroll
  for (int r = 0; r < RB; ++r) acc[r] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int i0 = 0; i0 < nk; i0 += DW) {
#pragma unroll
    for (int j = 0; j < DW; ++j) {
      const int i = i0 + j;
      if (i < nk) {          // workgroup-uniform
      const int sl = j & 1;  // (i0 is a multiple of DW, which is even)
      if (stager) {          // X of k-step i, split once into bf16 hi / lo for every wave
        const float4 q0 = xq[j % DXS][0], q1 = xq[j % DXS][1];
        const float f[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
        bf16x8 h8, l8;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const __bf16 h = (__bf16)f[e];
          h8[e] = h;
          l8[e] = (__bf16)(f[e] - (float)h);
        }
        xhi[sl][wave][lane] = h8;
        xlo[sl][wave][lane] = l8;
      }
      ldx2(i + DXS, xq[j % DXS]);
      __syncthreads();   // k-step i's X visible; every wave is past k-step i - 2's reads of this slot
      const bf16x8 w = wq[j];
      wq[j] = ldw(i + DW);
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        acc[r] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xhi[sl][r][lane], w, acc[r], 0, 0, 0);
        acc[r] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xlo[sl][r][lane], w, acc[r], 0, 0, 0);
      }
      }
    }
  }
  if (!live) return;
  const int Ncols = a.ntiles * 16;
  float* slab = a.ws + (size_t)sp * (RB * 16) * Ncols;
#pragma unroll
  for (int r = 0; r < RB; ++r)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int row = r * 16 + 4 * (lane >> 4) + e;
      if (row < a.M) slab[(size_t)row * Ncols + tile * 16 + (lane & 15)] = acc[r][e];
    }
}

// in-launch split-K merge: 0 off, 1 every eligible split, 2 (default) splits of small weights only -- measured
// (profiles/r02t_*): the TTS down (8.7 MB) 184.8 -> 181.5 us per AR step, the Qwen2 down (136 MB) slower
// (LLM stage 3313 -> 3340 us: every one of its 224 workgroups drains write-through partials before exiting),
// and so were the speech encoder's 32-row FFN-down LayerNorm producers (encoder stage 1594 -> 1624 us), which
// keep the reduce launch.
// -1 = FO_GEMM_MERGE (0-2) decides at first use.
int g_merge = -1;
inline int merge_mode() {
  if (g_merge < 0) {
    const char* e = getenv("FO_GEMM_MERGE");
    g_merge = (e && e[0] >= '0' && e[0] <= '2') ? e[0] - '0' : 2;
  }
  return g_merge;
}
int g_xs = -1;  // X-stationary kernel for eligible M <= 16 GEMMs: -1 = FO_GEMM_XS (default on), 0 off, 1 on
inline bool xs_mode() {
  if (g_xs < 0) {
    const char* e = getenv("FO_GEMM_XS");
    g_xs = (e && e[0] == '0') ? 0 : 1;
  }
  return g_xs == 1;
}
// 65..128-row GEMMs on the split-K weight streams as two row halves (FO_GEMM_ROW_SPLIT=0: the 64-row tile kernels)
const bool g_row_split = [] {
  const char* e = getenv("FO_GEMM_ROW_SPLIT");
  return !(e && e[0] == '0');
}();
// paged K / V appended by the RoPE epilogues rounded to bf16 (the values a bf16 cache would hold; storage stays fp32):
// the A/B of a bf16 KV against the fp32 default (FO_KV_BF16=1 or fo_set_kv_bf16)
int g_kv_bf16 = [] {
  const char* e = getenv("FO_KV_BF16");
  return (e && e[0] == '1') ? 1 : 0;
}();
// 65..128-row GEMMs on the >= 128 MB weight streams take k_gemm_rows (FO_GEMM_ROWS=0: the row halves above)
// (probe, fo_gemm_set_rows: 2 = k_gemm_wrow, one tile per wave)
int g_rows = [] {
  const char* e = getenv("FO_GEMM_ROWS");
  return (e && e[0] == '0') ? 0 : 1;
}();
// weights of at least this many MiB take the 17..64-row split-K stream (fo_gemm_set_xsk_min_mb: probes)
int g_xsk_min_mb = [] {
  const char* e = getenv("FO_XSK_MIN_MB");
  return e ? atoi(e) : 128;
}();
// 33..48-row split-K stream shape: 5 k-steps per wave and 2 units in flight (K split 3 ways on the Qwen2 gate/up
// instead of 4, 15 on the down instead of 19: a quarter fewer partial-slab bytes); FO_XSK_RB3=4: the round-4 shape
// (4 k-steps, 3 units).  Measured (scripts/gemm_mid_probe.py, profiles/r05ze_xsk_rb3_ab.txt): gate/up at 40 / 48
// rows 73.0 / 74.8 -> 69.6 / 70.0 us, down 40.8 / 41.9 -> 38.9 / 40.3 us
const int g_xsk_rb3 = [] {
  const char* e = getenv("FO_XSK_RB3");
  return e ? atoi(e) : 5;
}();
int g_xsk = -1;  // X-stationary split-K kernel for eligible 17..64-row GEMMs: -1 = FO_GEMM_XSK (default on)
inline bool xsk_mode() {
  if (g_xsk < 0) {
    const char* e = getenv("FO_GEMM_XSK");
    g_xsk = (e && e[0] == '0') ? 0 : 1;
  }
  return g_xsk == 1;
}
// K split of the 8-tile long-K weight stream (Qwen2 down: 28 column groups x S workgroups); -1 = FO_DOWN_S
// (4-16) decides at first use, default 8 (224 workgroups)
int g_down_s = -1;
inline int down_split() {
  if (g_down_s < 0) {
    const char* e = getenv("FO_DOWN_S");
    const int v = e ? atoi(e) : 0;
    g_down_s = (v >= 4 && v <= 16) ? v : 8;
  }
  return g_down_s;
}
// tiles per workgroup of that stream: 7 (default: 32 column groups x 8 = 256 workgroups, one per CU) or 8 (28
// groups, 224 workgroups); FO_DOWN_NT.  r03s (one call): down alone 30.1 -> 29.8 us at 16 rows, the LLM stage
// 3264 -> 3256 us, the bench 193.0 / 192.9x -> 194.3 / 195.2x; 8 x 9 (252 workgroups) and 7 x 9 (288) are slower
// (31.3, 40.9 us; profiles/r03s_down_tiles_ab.txt)
int g_down_nt = -1;
inline int down_tiles() {
  if (g_down_nt < 0) {
    const char* e = getenv("FO_DOWN_NT");
    g_down_nt = (e && atoi(e) == 8) ? 8 : 7;
  }
  return g_down_nt;
}
int g_num_cus = 0;
inline int num_cus() {
  if (!g_num_cus) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) ==
        hipSuccess && n > 0)
      g_num_cus = n;
    else
      g_num_cus = 256;
  }
  return g_num_cus;
}

// Pack W[N][K] (row-major, f32 or bf16, row stride ldw) into fragment order, writing tile t
// of the source to destination tile (tile_base + t * tile_stride).
__global__ void k_pack(const void* W, int src_bf16, int N, int K, int ldw, bf16_t* out, int KSp,
                       int tile_base, int tile_stride, int ntiles_src) {
  const size_t total = (size_t)ntiles_src * KSp * 64;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int lane = i & 63;
    const size_t rest = i >> 6;
    const int ks = rest % KSp;
    const int t = rest / KSp;
    const int row = t * 16 + (lane & 15);
    const int k0 = ks * 32 + 8 * (lane >> 4);
    bf16_t v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = k0 + j;
      float f = 0.f;
      if (row < N && k < K) {
        if (src_bf16) f = bf2f(reinterpret_cast<const bf16_t*>(W)[(size_t)row * ldw + k]);
        else f = reinterpret_cast<const float*>(W)[(size_t)row * ldw + k];
      }
      v[j] = f2bf(f);
    }
    const size_t dt = (size_t)tile_base + (size_t)t * tile_stride;
    bf16_t* d = out + ((dt * KSp + ks) * 64 + lane) * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) d[j] = v[j];
  }
}

}  // namespace

extern "C" {

int fo_gemm_pick_split(int M, int N_tiles_groups, int K) {
  const int KS = K >> 5;
  const int mt = (M + 63) / 64;
  const int blocks = N_tiles_groups * mt;
  // Measured on MI355X (scripts/gemm_sweep.py): every cross-workgroup split adds ~8 us of slab
  // round trip + ordered reduction, more than it buys for any hot-path shape with >= 56 column
  // tiles; split only when the grid is tiny.
  int S = blocks >= 48 ? 1 : (64 + blocks - 1) / blocks;
  int smax = KS / 16;
  if (smax < 1) smax = 1;
  if (S > smax) S = smax;
  if (S > 16) S = 16;
  if (S < 1) S = 1;
  return S;
}

long long fo_gemm_workspace_floats(int M, int N, int K, int swiglu) {
  const int ntiles = swiglu ? 2 * ((N + 15) / 16) : (N + 15) / 16;
  const int NT = swiglu ? 2 : 1;
  const int S = fo_gemm_pick_split(M, ntiles / NT, K);
  const int RB = M <= 16 ? 1 : (M <= 32 ? 2 : 4);
  const int mt = (M + RB * 16 - 1) / (RB * 16);
  return S > 1 ? (long long)S * mt * RB * 16 * ntiles * 16 : 0;
}

// Y = act(X @ W^T + bias) (+Y if residual).  X bf16 [M][ldx], K % 32 == 0.
// swiglu != 0: Wp holds interleaved (gate, up) tile pairs, Y[m][n] = silu(gate) * up, n < N.
static int gemm_impl(const void* X, int x_f32, int ldx, int M, int K, const void* Wp, int N, int swiglu,
                     const float* bias, const float* scale, const float* shift, void* Y, int ldy, int out_bf16,
                     int act, int residual, float* ws, long long ws_floats, int* counters, int splitk,
                     const float* rstats, int rgroups, float reps, float* sout, const float* gnext, float* yg,
                     int* sgroups, const GemmArgs* rope, hipStream_t stream, const float* lnw = nullptr,
                     const float* lnb = nullptr, float lneps = 0.f, float* sout1 = nullptr,
                     const float* rstats1 = nullptr) {
  // the packed buffers armed for this launch are consumed whatever happens below (one launch each)
  const PackArm xpk = g_xpk, ypk = g_ypk, yp32k = g_yp32k, xp32k = g_xp32k;
  g_xpk = g_ypk = g_yp32k = g_xp32k = PackArm{};
  FO_REQUIRE(M > 0 && N > 0 && K > 0, "fo_gemm: bad shape M=%d N=%d K=%d", M, N, K);
  FO_PACK_FITS(xpk, K, M, "fo_gemm (packed X)");
  FO_PACK_FITS(xp32k, K, M, "fo_gemm (fp32 packed X)");
  FO_PACK_FITS(ypk, N, M, "fo_gemm (packed output)");
  FO_PACK_FITS(yp32k, N, M, "fo_gemm (fp32 packed output)");
  FO_REQUIRE(!rstats || rgroups > 0, "fo_gemm: row statistics without a group count");
  FO_REQUIRE(!sout || (!swiglu && !out_bf16 && (!yg || gnext)), "fo_gemm: row statistics need fp32 non-SwiGLU output");
  FO_REQUIRE((K & 31) == 0, "fo_gemm: K=%d must be a multiple of 32", K);
  FO_REQUIRE(ldx >= K, "fo_gemm: ldx=%d < K=%d", ldx, K);
  FO_REQUIRE(ldy >= N, "fo_gemm: ldy=%d < N=%d", ldy, N);
  FO_REQUIRE(!(swiglu && (bias || scale)), "fo_gemm: swiglu with bias/affine unsupported");
  FO_REQUIRE(!scale == !shift, "fo_gemm: scale and shift go together");
  // 65..128 rows on the large weight streams (a duplex tick whose sessions start a turn: the 5-token chat prefix on
  // top of the 4 chunk rows; 8 x 9 = 72 rows): two X-stationary split-K launches on the two row halves (33..64 rows
  // each) instead of 64-row tiles, which stream the whole weight once per row tile at ~1.4-2.5 TB/s (r05i duplex
  // table: gate/up 193.8 us, down 110.4 us per layer at 72 rows).  Both halves take k_gemm_xsk, so their row
  // statistics have the same group count ((N + 255) / 256) and the halves' rows tile the [M][groups] layout.
  // 65..128 rows on the large weight streams: k_gemm_rows (the weights once) when its split-K slabs fit the workspace
  bool rows_ok = false;
  int rows_S = 1, rows_tp = 0, rows_G = 0;
  {
    const int nt_all = (swiglu ? 2 : 1) * ((N + 15) / 16);
    const long long wb = (long long)nt_all * 16 * K * 2;
    // (>= 16 MiB: the Qwen2 q|k|v -- RoPE + paged-KV append in the reduce -- and o too, which at 128 rows ran 64-row
    // tiles re-reading the weights per row tile (q|k|v 80 us, r06q) or two row halves (o 2 x 22.8 us))
    if (g_rows && M > (g_rows == 4 ? 32 : 64) && M <= 128 && x_f32 && !lnw && !sout1 && !rstats1 && splitk <= 1 &&
        wb >= (16ll << 20) && (ldx % 4) == 0 && ((unsigned long long)X & 15) == 0 && !xpk.p0 && !xp32k.p0 &&
        !g_force_nt &&
        !g_force_nw && (!swiglu || nt_all % 2 == 0)) {
      const int cus = num_cus();
      if (g_rows >= 5) {   // (probes 5 / 6) the one-K-pass 10-tile partition
        const int units = nt_all / 2, per = (units + cus - 1) / cus;
        rows_tp = 2 * per;
        rows_G = (units + per - 1) / per;
        rows_S = 1;
      } else if (g_rows != 2) {   // k_gemm_rows: the waves split the rows.  The workgroup's X (all rows over its K range)
        // comes through the CU beside its weights, so K is split until a workgroup's tiles carry about as many bytes
        // as its X: gate/up 3 K thirds x 14 (gate, up) pairs (28 tiles), one round of <= 256 workgroups; down 16 K
        // slices x 14 tiles (profiles/r06o_gemm_rows_split.txt, r06p: gate/up at 128 rows 129.4 us on one K pass of
        // 10 tiles, 102.7-110.0 on K halves of 20, 101.9 on thirds; down 68.9 on 8 slices of 7 tiles, 59.6-63.9)
        const int ks = M <= 64 ? 2 : 3;
        if (swiglu) {
          const int units = nt_all / 2, per = (ks * units + cus - 1) / cus;
          rows_tp = 2 * per;
          rows_G = (units + per - 1) / per;
          rows_S = ks;
        } else {
          rows_tp = nt_all % 14 == 0 ? 14 : 16;
          rows_G = (nt_all + rows_tp - 1) / rows_tp;
          rows_S = max(1, min(16, cus / rows_G));
        }
      } else {             // (probe) k_gemm_wrow: one tile per wave; gate/up 10 waves (5 pairs), one K pass; long-K 14 / 8
        rows_tp = swiglu ? ((nt_all / 2) % 5 == 0 ? 10 : 8) : (nt_all % 14 == 0 ? 14 : 8);
        rows_G = (nt_all + rows_tp - 1) / rows_tp;
        rows_S = swiglu ? 1 : max(1, min(16, cus / rows_G));
      }
      const long long need = (long long)rows_S * 128 * nt_all * 16;
      rows_ok = rows_tp <= (swiglu ? 30 : 16) && need <= ws_floats && ws != nullptr &&
                (K >> 5) >= rows_S;
    }
  }
  {
    const long long wb = (long long)(swiglu ? 2 : 1) * ((N + 15) / 16) * 16 * K * 2;
    const bool big = wb >= ((long long)g_xsk_min_mb << 20) || (K >= 8192 && wb >= (32ll << 20));
    // (and the plain >= 8 MB projections -- the Qwen2 o: 57.0 us on 64-row tiles at 72 rows -- whose halves take
    // the one-row-tile split-K kernels + k_gemm_reduce, the same statistics groups)
    const bool mid_w = !swiglu && wb >= (8ll << 20);
    if (!rows_ok && M > 64 && M <= 128 && x_f32 && !lnw && !rope && !sout1 && !rstats1 && splitk <= 1 && (big || mid_w) &&
        xsk_mode() && !g_force_nt && !g_force_nw && !xpk.p0 && !ypk.p0 && !yp32k.p0 && !xp32k.p0 && (K >> 5) >= 56 &&
        (ldx % 4) == 0 && ((swiglu ? 2 : 1) * ((N + 15) / 16)) % 2 == 0 && g_row_split) {
      const int M0 = (M + 1) / 2, grp = (N + 255) / 256;
      int sg = 0;
      for (int h = 0; h < 2; ++h) {
        const int r0 = h ? M0 : 0, Mh = h ? M - M0 : M0;
        const size_t yb = (size_t)r0 * ldy * (out_bf16 ? 2 : 4);
        int sgh = 0;
        const int rc = gemm_impl(static_cast<const char*>(X) + (size_t)r0 * ldx * 4, x_f32, ldx, Mh, K, Wp, N, swiglu,
                                 bias, scale, shift, static_cast<char*>(Y) + yb, ldy, out_bf16, act, residual, ws,
                                 ws_floats, counters, splitk, rstats ? rstats + (size_t)r0 * rgroups : nullptr, rgroups,
                                 reps, sout ? sout + (size_t)r0 * grp : nullptr, gnext,
                                 yg ? yg + (size_t)r0 * ldy : nullptr, &sgh, nullptr, stream);
        if (rc) return rc;
        FO_REQUIRE(!sout || sgh == grp, "fo_gemm: row halves wrote %d statistics groups, expected %d", sgh, grp);
        sg = sgh;
      }
      if (sgroups) *sgroups = sg;
      return 0;
    }
  }
  GemmArgs a;
  a.X = X;
  a.scale = scale;
  a.shift = shift;
  a.Wp = (const bf16_t*)Wp;
  a.bias = bias;
  a.Y = Y;
  a.ws = ws;
  a.counters = counters;
  a.ldx = ldx;
  a.ldy = ldy;
  a.M = M;
  a.K = K;
  a.N = N;
  a.act = act;
  a.out_bf16 = out_bf16;
  a.residual = residual;
  a.sout = sout;
  a.gnext = gnext;
  a.yg = yg;
  a.rstats = rstats;
  a.rgroups = rgroups;
  a.reps = reps;
  a.ntiles = (swiglu ? 2 : 1) * ((N + 15) / 16);
  a.rpos = a.rslot = nullptr;
  a.rcos = a.rsin = nullptr;
  a.rq = a.rk = a.rv = nullptr;
  a.rH = a.rKVH = a.rhd = a.rPS = 0;
  a.rkvb = 0;
  a.lnw = lnw;
  a.lnb = lnb;
  a.lneps = lneps;
  a.sout1 = sout1;
  a.rstats1 = rstats1;
  a.trc = g_trc;
  a.xph = reinterpret_cast<const bf16x8*>(xpk.p0);
  a.xpl = reinterpret_cast<const bf16x8*>(xpk.p1);
  a.ypkh = reinterpret_cast<bf16_t*>(const_cast<void*>(ypk.p0));
  a.ypkl = reinterpret_cast<bf16_t*>(const_cast<void*>(ypk.p1));
  a.yp32 = reinterpret_cast<float*>(const_cast<void*>(yp32k.p0));
  a.xp32 = reinterpret_cast<const float*>(xp32k.p0);
  FO_REQUIRE(!a.xp32 || (lnw && M <= 64), "fo_gemm: the fp32 packed X is read by LayerNorm-on-load launches only");
  FO_REQUIRE(!a.yp32 || (M <= 64 && !swiglu && !rope), "fo_gemm: fp32 packed output needs <= 64 plain rows");
  a.prb = (M + 15) / 16;
  FO_REQUIRE(!a.xph || (x_f32 && M <= 64 && !lnw), "fo_gemm: packed X needs fp32 X of <= 64 rows");
  FO_REQUIRE(!a.ypkh || (M <= 64 && !swiglu && !rope), "fo_gemm: packed output needs <= 64 plain rows");
  FO_REQUIRE(!sout1 || sout, "fo_gemm: row sums come with the sums of squares");
  if (lnw) {
    FO_REQUIRE(lnb && x_f32 && M <= 64 && !swiglu && rstats && rstats1 && rgroups > 0 && rgroups <= 64 && !rope &&
               ldx % 4 == 0,
               "fo_gemm_ln: fp32 X, M <= 64, producer statistics, plain epilogue only (M=%d K=%d)", M, K);
  }
  if (rope) {
    FO_REQUIRE(!swiglu && !sout && !residual && !out_bf16 && act == 0 && !scale, "fo_gemm_qkv_rope: plain epilogue only");
    FO_REQUIRE(rope->rhd % 32 == 0 && N == (rope->rH + 2 * rope->rKVH) * rope->rhd,
               "fo_gemm_qkv_rope: N=%d != (H + 2 KVH) * hd with hd %% 32 == 0", N);
    a.rpos = rope->rpos;
    a.rslot = rope->rslot;
    a.rcos = rope->rcos;
    a.rsin = rope->rsin;
    a.rq = rope->rq;
    a.rk = rope->rk;
    a.rv = rope->rv;
    a.rH = rope->rH;
    a.rKVH = rope->rKVH;
    a.rhd = rope->rhd;
    a.rPS = rope->rPS;
    a.rkvb = g_kv_bf16;
  }
  if (rows_ok) {
    a.S = rows_S;
    a.counters = nullptr;
    if (sgroups) *sgroups = (N + 255) / 256;
    const int total = rows_S * rows_G;
    const dim3 grid(8 * ((total + 7) / 8));
    // (instantiated tile counts: the Qwen2 gate/up's 14 pairs and down's 14 tiles per workgroup, else the next size)
#define FO_ROWS(NWV_, RPW_, NTC_, DW_, DX_, PR_, XL_)                                                                  \
  do {                                                                                                                \
    if (g_rows == 3 && PR_ == 0) /* (probe 3: the split consumer map, r06y: 79.3 vs 76.8 us, kept off) */            \
      hipLaunchKernelGGL((k_gemm_rows<NWV_, RPW_, NTC_, DW_, DX_, false, PR_, XL_, 1>), grid, dim3(NWV_ * 64), 0,       \
                         stream, a, rows_G, rows_tp);                                                                 \
    else                                                                                                              \
      hipLaunchKernelGGL((k_gemm_rows<NWV_, RPW_, NTC_, DW_, DX_, false, PR_, XL_, 0>), grid, dim3(NWV_ * 64), 0,       \
                         stream, a, rows_G, rows_tp);                                                                 \
  } while (0)
#define FO_WROW(NWV_, DW_, DXS_) \
  hipLaunchKernelGGL((k_gemm_wrow<NWV_, 8, DW_, DXS_>), grid, dim3(NWV_ * 64), 0, stream, a, rows_G)
    if (g_rows >= 5) {   // (probes 5 / 6: the 10-tile gate/up without X loads -- WRONG results: the weight ring's
                         // rate at 7 vs 11 k-steps of depth)
      if (g_rows == 5) FO_ROWS(8, 1, 10, 7, 1, 1, 1);
      else FO_ROWS(8, 1, 10, 11, 1, 1, 1);
    } else if (g_rows == 2) {   // (probe) k_gemm_wrow
      if (rows_tp == 10) FO_WROW(10, 12, 4);
      else if (rows_tp == 14) FO_WROW(14, 8, 4);
      else FO_WROW(8, 12, 4);
    } else if (swiglu && rows_tp > 20) {
      // the weights and X the same number of k-steps ahead: vmcnt retires in order, so the wait for a k-step's X also
      // waits for every weight load issued before it -- an X lead shorter than the weights' caps their depth at it
      // (r06w: 7 or 11 k-steps of weights alone, 85 us either way; with X 1 ahead the ring held ~1 k-step)
      FO_ROWS(8, 1, 30, 2, 2, 0, 1);
    } else if (swiglu) {
      FO_ROWS(8, 1, 20, 3, 3, 0, 1);
    } else if (rows_tp == 14) {
      FO_ROWS(8, 1, 14, 4, 4, 0, 1);
    } else {
      FO_ROWS(8, 1, 16, 3, 3, 0, 1);
    }
#undef FO_WROW
#undef FO_ROWS
    int rc = fo::check_launch("fo_gemm/rows");
    if (rc) return rc;
    launch_reduce(a, swiglu, 128, N, M, stream);
    fo::count_launch(FO_L_GEMM_ROWS);
    fo::count_launch(FO_L_GEMM_REDUCE);
    return fo::check_launch("fo_gemm/rows reduce");
  }
  // X-stationary persistent weight stream (k_gemm_xs) for the M <= 16 rows of a listen chunk / text step on
  // K = 3584 layers (Qwen2 q|k|v, o, gate/up, lm_head): no split, no LayerNorm-on-load
  // Measured (scripts/gemm_xs_ab.py, graph-replayed over weight copies beyond the Infinity Cache): gate/up
  // + SwiGLU 56.1 -> 48.4 us at 16 rows, 47.4 -> 45.5 us at 8; lm_head equal (169.5 vs 169.9 us); the
  // 26-33 MB o and q|k|v projections slower (one unit per workgroup: 12.3 -> 15.1, 18.7 -> 20.4 us), so
  // only the SwiGLU pair takes this path.
  if (x_f32 && M <= 16 && !lnw && K == XS_NW * XS_KPW * 32 && (a.ntiles % 2) == 0 && splitk <= 1 && xs_mode() &&
      !g_force_nt && !g_force_nw && swiglu && (long long)a.ntiles * 16 * K >= (64ll << 20) && ldx % 4 == 0) {
    const int units = a.ntiles / 2;
    // as many workgroups as it takes for every one to get the same (ceil) number of units: 1184 gate/up
    // pairs -> 237 x 5 (not 256 with 4 or 5: the 5-unit CUs would set the time); a CU can pull more than
    // its 1/256 share of the HBM stream, so the idle CUs cost nothing
    const int per = (units + num_cus() - 1) / num_cus();
    const int G = (units + per - 1) / per;
    a.S = 1;
    if (sgroups) *sgroups = units;
    if (sout) FO_REQUIRE(!swiglu && !rope, "fo_gemm: statistics with a paired epilogue");
    switch (xs_variant()) {
      case 1: hipLaunchKernelGGL((k_gemm_xs<XS_NW, XS_KPW, 1>), dim3(G), dim3(XS_NW * 64), 0, stream, a, units); break;
      case 2: hipLaunchKernelGGL((k_gemm_xs<XS_NW, XS_KPW, 2>), dim3(G), dim3(XS_NW * 64), 0, stream, a, units); break;
      case 3: hipLaunchKernelGGL((k_gemm_xs<8, 14>), dim3(G), dim3(8 * 64), 0, stream, a, units); break;
      case 4: hipLaunchKernelGGL((k_gemm_xs<8, 14, 4>), dim3(G), dim3(8 * 64), 0, stream, a, units); break;
      default: hipLaunchKernelGGL((k_gemm_xs<XS_NW, XS_KPW>), dim3(G), dim3(XS_NW * 64), 0, stream, a, units);
    }
    fo::count_launch(FO_L_GEMM_XS);
    if (a.xph) fo::count_launch(FO_L_GEMM_XP);
    return fo::check_launch("fo_gemm/xs");
  }
  // 17..64 rows on large weights (duplex ticks: 8 sessions x 4 framing-B tokens, the assistant prefix 8 x 5, prefixed
  // first chunks): the X-stationary stream with K split over workgroups (k_gemm_xsk) + k_gemm_reduce
  // only the weight streams: >= 64 MB (Qwen2 gate/up, down) or long-K >= 16 MB (the speech encoder's subsampling
  // output linear, 19,456 x 1024 = 40 MB: 48.8 us per chunk on the split-K grid kernel, r04i); on the 26-33 MB
  // q|k|v / o the one-row-tile kernels below are faster (r04d probe: o 14.8 vs 18.5 us, q|k|v 19.2 vs 24.4 us at 32 rows)
  const long long wbytes0 = (long long)a.ntiles * 16 * K * 2;
  const bool big_w0 = wbytes0 >= ((long long)g_xsk_min_mb << 20) || (K >= 8192 && wbytes0 >= (32ll << 20));
  if (x_f32 && M > 16 && M <= 64 && !lnw && (a.ntiles % 2) == 0 && splitk <= 1 && xsk_mode() && !g_force_nt &&
      !g_force_nw && big_w0 && ldx % 4 == 0 && !sout1 && (K >> 5) >= 56) {
    const int RBk = (M + 15) / 16;
    // 8 waves x KPW k-steps of X per split (hi in VGPRs, lo in LDS: KPW shrinks as the row blocks grow), UA units of
    // weights in flight per wave (~28 KiB, k_gemm_xs's depth); every split has work (K >= 56 k-steps)
    const int NWk = 8, KPWk = RBk == 2 ? 7 : (RBk == 3 ? (g_xsk_rb3 == 5 ? 5 : 4) : 3);
    const int KSk = K >> 5;
    const int S = (KSk + NWk * KPWk - 1) / (NWk * KPWk);
    const int units = a.ntiles / 2;
    const int per_split = max(1, num_cus() / S);
    const int per = (units + per_split - 1) / per_split;
    const int G = (units + per - 1) / per;
    const long long need = (long long)S * RBk * 16 * a.ntiles * 16;
    FO_REQUIRE(ws && need <= ws_floats, "fo_gemm/xsk: split-K workspace too small (%lld > %lld)", need, ws_floats);
    a.S = S;
    a.counters = nullptr;
    if (sgroups) *sgroups = (N + 255) / 256;
    const dim3 grid(8 * ((S * G + 7) / 8));
    if (RBk == 2) hipLaunchKernelGGL((k_gemm_xsk<8, 7, 2, 2>), grid, dim3(512), 0, stream, a, units, G);
    else if (RBk == 3 && KPWk == 5) hipLaunchKernelGGL((k_gemm_xsk<8, 5, 3, 2>), grid, dim3(512), 0, stream, a, units, G);
    else if (RBk == 3) hipLaunchKernelGGL((k_gemm_xsk<8, 4, 3, 3>), grid, dim3(512), 0, stream, a, units, G);
    else hipLaunchKernelGGL((k_gemm_xsk<8, 3, 4, 4>), grid, dim3(512), 0, stream, a, units, G);
    int rc = fo::check_launch("fo_gemm/xsk");
    if (rc) return rc;
    launch_reduce(a, swiglu, RBk * 16, N, M, stream);
    fo::count_launch(FO_L_GEMM_XSK);
    fo::count_launch(FO_L_GEMM_REDUCE);
    if (a.ypkh) fo::count_launch(FO_L_GEMM_YPACK);
    if (a.yp32) fo::count_launch(FO_L_GEMM_YPACK32);
    return fo::check_launch("fo_gemm/xsk reduce");
  }
  // mid-size row counts on large weights (the Qwen2 prefills of a turn: assistant prefix, the first
  // chunk with its chat prefix, the system prompt; 17..64 rows): one row tile of ceil(M/16) row blocks
  // against 4-tile column groups, so X (fp32, re-read by every column group) costs about what the
  // weights do, and no grid of 64-row tiles streams X four times per weight byte
  // (small weights with 33..64 rows -- the duplex encoder at 8 sessions x 7 frames -- take the same
  // one-row-tile kernels with single-tile column groups instead of 64-row tiles on 64 workgroups)
  const bool big_w = (long long)a.ntiles * 16 * K >= (8ll << 20);
  const bool mid = x_f32 && !lnw && M > 16 && M <= 64 && (big_w || M > 32);
  const int RB = mid ? (M + 15) / 16 : (M <= 16 ? 1 : (M <= 32 ? 2 : 4));
  const int mt = (M + RB * 16 - 1) / (RB * 16);
  // tiles per workgroup: the activation rows are re-read by every workgroup, so workgroups that
  // cover more output columns read X fewer times per weight byte (measured, gemm_sweep.py)
  int NT = swiglu ? 2 : 1;
  int S_auto = 0;
  int launch_pipe = 0, nw_pref = 0;
  const int KS = K >> 5;
  if (mid) {
    NT = big_w ? (a.ntiles % 4 == 0 ? 4 : 2) : (swiglu ? 2 : 1);
  } else if (RB == 1) {
    // measured policy (gemm_sweep.py, gemm_graph_sweep.py): wide layers (>= 1024 tiles: Qwen2 gate/up, lm_head) take 4
    // tiles per workgroup; long-K layers (Qwen2 down) 4 tiles and a 4-way K split; mid-size grids
    // (> 256 tiles: Qwen2 qkv) 2 tiles; small ones 1
    if (a.ntiles >= 1024) NT = 4;
    // Qwen2 down (592 k-steps, 224 tiles): 7 tiles x 8-way K split, pipelined (32 x 8 = 256 workgroups; 8 tiles: 224): the
    // activation rows are read by a quarter as many column groups as with 4 tiles x 4 ways; 31.7 -> 29.7 us at 16
    // rows, 29.7 -> 28.7 us at 8, reduce launch included (profiles/r03g_down_sweep.txt)
    else if (KS >= 256 && a.ntiles >= 128) {
      NT = a.ntiles % 8 == 0 ? 8 : 4;
      if (down_tiles() == 7 && a.ntiles % 7 == 0) NT = 7;
      S_auto = NT >= 7 ? down_split() : 4;
    }
    else if (KS >= 128 && a.ntiles <= 64) S_auto = 4;  // narrow long-K (TTS down): 10.9 -> 8.2 us in a graph
    else if (a.ntiles > 256) NT = 2;
    // small SwiGLU pairs over 512+ tiles (the TTS gate/up, 608 tiles, 17.4 MB): 2 pairs per workgroup on 8
    // waves keeps the grid within one round of the 256 CUs (152 instead of 304 workgroups): 7.83 -> 7.16 us
    // graph-replayed (profiles/r02s_tts_gemm_sweep.txt)
    if (swiglu && a.ntiles >= 512 && a.ntiles < 1024 && (long long)a.ntiles * 16 * K < (32ll << 20) &&
        a.ntiles % 4 == 0) {
      NT = 4;
      nw_pref = 8;
    }
    // Pipelined weight stream, 2-step groups (policy measured in the turn bench, A/B twice in one
    // call: 388-390 -> 383-386 ms/turn, p50 first PCM 50 -> 48.5 ms).  Isolated (scripts/
    // gemm_gu_sweep.py, gemm_pipe_ab.py; two alternating weight copies): gate/up at <= 8 rows on 2
    // tiles x 8 waves 50.5 -> 44.4 us, down 32.0 -> 29.5 us, lm_head 177 -> 172 us.  Gate/up at 9-16
    // rows keeps the plain 4-tile loop: pipelined with a 2-way K split it is faster alone (53.8 ->
    // 51.2 us) but made the pipelined listen stage slower (turn 388 -> 408 ms).
    const int pm = pipe_mode();
    if (x_f32 && pm != 0 && pm != 3) {
      launch_pipe = pm;   // sweeps: every one-row-tile fp32-X GEMM
    } else if (x_f32 && (long long)a.ntiles * 16 * K >= (32ll << 20) && pm != 0) {
      if (pm != 3) launch_pipe = pm;
      else if (!swiglu || M <= 8) launch_pipe = 2;
      if (pm == 3 && swiglu && M <= 8 && !g_force_nt && !g_force_nw) {
        NT = 2;
        nw_pref = 8;
      }
    }
    if (g_force_nt) NT = g_force_nt;
    FO_REQUIRE(NT == 1 || NT == 2 || NT == 4 || NT == 8 || (NT == 7 && !swiglu), "fo_gemm: tiles per workgroup %d", NT);
    FO_REQUIRE(!swiglu || NT >= 2, "fo_gemm: swiglu needs tile pairs");
    if (a.ntiles % NT) NT = swiglu ? 2 : 1;
  } else if (RB == 2) {
    // speech-encoder shapes (M = 32): narrow long-K layers (FFN w_2, subsampling out) split K 4 ways
    if (!swiglu && a.ntiles <= 64 && KS >= 96) S_auto = 4;
    if (g_force_nt == 1 || g_force_nt == 2) NT = swiglu ? 2 : g_force_nt;
    if (a.ntiles % NT) NT = swiglu ? 2 : 1;
  }
  int nw_pref4 = 0;
  if (RB == 4 && g_force_nt && x_f32 && !lnw && !rope) {   // sweeps (fo_gemm_tune): forced tiles per workgroup
    NT = g_force_nt;
    if (swiglu && NT < 2) NT = 2;
    if (a.ntiles % NT) NT = swiglu ? 2 : 1;
  } else if (RB == 4 && !mid && x_f32 && !lnw && M > 64) {
    // 64-row tiles (prefills of 65+ rows: the AR decoder's sentence prefill at 8 sessions x 32-40 sub-token rows, the
    // speech encoder's im2col convolutions).  Measured (scripts/gemm_big_sweep.py, profiles/r04q_gemm_big_sweep.txt):
    // 8 waves splitting K inside the workgroup everywhere but the K = 32 conv1 (4); 4 column tiles per X read when
    // that still gives >= 128 workgroups or K is long (then split K over workgroups until the grid nears 256); else
    // one tile (pair) per workgroup.  AR prefill down 67.8 -> 26.3 us, gate/up 56.2 -> 40.3 us, q|k|v 20.3 -> 16.4,
    // o 12.2 -> 10.4; conv2 130.9 -> 89.6 us, conv1 28.5 -> 15.3 us
    nw_pref4 = KS <= 2 ? 4 : 8;
    const int wg4 = a.ntiles / 4 * mt;
    if (a.ntiles % 4 == 0 && KS > 2 && (wg4 >= 128 || KS >= 128)) {
      NT = 4;
      if (KS >= 128) S_auto = (KS >= 256 || wg4 * 4 <= 256) ? 4 : (wg4 * 2 <= 256 ? 2 : 1);
    } else {
      NT = swiglu ? 2 : 1;
    }
  }
  // the epilogue rotates the (i, i + hd/2) tile pair a workgroup holds; a 17..64-row RoPE projection on large
  // weights (the Qwen2 q|k|v of a duplex tick or a prefill) keeps the 4-tile column groups of the plain path and
  // always splits K, so k_gemm_reduce (which pairs the tiles itself) runs that epilogue: one X read per 4 tiles
  // instead of per pair (r04g trace: the 2-tile split q|k|v 33.9 + 5 us at 33..48 rows)
  const bool rope4 = rope && mid && NT == 4 && splitk <= 1 && !g_force_nt;
  if (rope && !rope4) NT = 2;
  if (lnw && NT > 2) NT = 2;
  const int groups = a.ntiles / NT;
  if (mid) {  // split K: 2 ways on wide layers (Qwen2 gate/up), until the grid covers the chip on narrow ones
    S_auto = groups >= 192 ? (big_w ? 2 : 1) : (256 + groups - 1) / groups;
    if (S_auto > 4) S_auto = 4;
    if (S_auto > KS / 16) S_auto = KS / 16 > 0 ? KS / 16 : 1;
  }
  int S = splitk > 0 ? splitk : (S_auto && !g_force_nt ? S_auto : (mid ? 1 : fo_gemm_pick_split(M, groups, K)));
  if (rstats && !lnw && !mid) S = 1;  // (split RMSNorm consumers: k_gemm_reduce applies the rstd)
  if (S > (K >> 5)) S = K >> 5;
  if (rope4 && S < 2) S = 2;   // the pair epilogue needs the reduce launch
  a.S = S;
  if (S > 1) {
    const long long need = (long long)S * mt * RB * 16 * a.ntiles * 16;
    FO_REQUIRE(ws && need <= ws_floats, "fo_gemm: split-K workspace too small (%lld > %lld)", need, ws_floats);
  }
  dim3 grid(groups, mt, S);
  // one-row-tile plain splits merge inside the launch (last split to arrive sums and finishes; tickets in
  // the caller's zeroed counters, left zeroed); otherwise k_gemm_reduce follows
  const bool small_w = (long long)a.ntiles * 16 * K < (32ll << 20);
  const bool merged = S > 1 && counters && RB == 1 && !a.sout1 && !swiglu && !lnw && !mid &&
                      (merge_mode() == 1 || (merge_mode() == 2 && small_w));
  a.counters = merged ? counters : nullptr;
  if (merged) FO_REQUIRE((long long)groups * mt <= (1 << 20), "fo_gemm: too many tiles for the merge tickets");
  if (sgroups) *sgroups = (S > 1 && !merged) ? (N + 255) / 256 : groups;
  const bool wstream = (long long)a.ntiles * 16 * K >= (32ll << 20);
  const long long wgs = (long long)groups * mt * S;
  if (lnw) {
    const int nw = wgs <= 128 ? 16 : 8;
    dim3 blk(nw * 64);
#define FO_LN(NT_, RB_, NW_) hipLaunchKernelGGL((k_gemm_ln<NT_, RB_, NW_>), grid, blk, 0, stream, a)
    if (RB == 1) {
      if (NT == 2) { if (nw == 16) FO_LN(2, 1, 16); else FO_LN(2, 1, 8); }
      else { if (nw == 16) FO_LN(1, 1, 16); else FO_LN(1, 1, 8); }
    } else if (RB == 2) {
      if (NT == 2) { if (nw == 16) FO_LN(2, 2, 16); else FO_LN(2, 2, 8); }
      else { if (nw == 16) FO_LN(1, 2, 16); else FO_LN(1, 2, 8); }
    } else {   // 33..64 rows (the duplex encoder: 8 sessions x 7 framing-B frames): 2 k-steps in flight per wave
      if (NT == 2) hipLaunchKernelGGL((k_gemm_ln<2, 4, 8, 2>), grid, dim3(512), 0, stream, a);
      else hipLaunchKernelGGL((k_gemm_ln<1, 4, 8, 4>), grid, dim3(512), 0, stream, a);
    }
#undef FO_LN
  } else if (mid) {
    // 2 k-steps in flight per wave keep the RB x NT accumulators and fragments within 4 waves / SIMD
    const int nw = (NT == 4 || wgs >= 384) ? 4 : 8;
#define FO_MID(NT_, RB_, NW_, SW_) launch_mid<NT_, RB_, NW_, SW_>(grid, a, stream)
#define FO_MID_RB(NT_, NW_, SW_) { if (RB == 2) FO_MID(NT_, 2, NW_, SW_); else if (RB == 3) FO_MID(NT_, 3, NW_, SW_); else FO_MID(NT_, 4, NW_, SW_); }
    if (swiglu) {
      if (NT == 4) FO_MID_RB(4, 4, true) else if (nw == 4) FO_MID_RB(2, 4, true) else FO_MID_RB(2, 8, true)
    } else if (NT == 1) {
      if (nw == 4) FO_MID_RB(1, 4, false) else FO_MID_RB(1, 8, false)
    } else {
      if (NT == 4) FO_MID_RB(4, 4, false) else if (nw == 4) FO_MID_RB(2, 4, false) else FO_MID_RB(2, 8, false)
    }
#undef FO_MID_RB
#undef FO_MID
  } else if (RB == 1) {
    // measured (scripts/gemm_sweep.py, MI355X): one workgroup per CU wants 16 waves, a couple per
    // CU 8, many 4; 4 k-steps in flight per wave is the sweet spot everywhere on the hot path
    int nw = wgs <= 160 ? 16 : (wgs <= 256 ? (NT == 1 ? 16 : 8) : ((NT == 4 || wgs >= 1024) ? 4 : 8));
    if (nw_pref) nw = nw_pref;
    if (g_force_nw) nw = g_force_nw;
    g_launch_pipe = launch_pipe;
    g_launch_u = g_force_u ? g_force_u : 4;
    if (swiglu) {
      if (NT == 8) launch_nw<8, 1, true>(nw, wstream, x_f32, grid, a, stream);
      else if (NT == 4) launch_nw<4, 1, true>(nw, wstream, x_f32, grid, a, stream);
      else launch_nw<2, 1, true>(nw, wstream, x_f32, grid, a, stream);
    } else {
      if (NT == 8) launch_nw<8, 1, false>(nw, wstream, x_f32, grid, a, stream);
      else if (NT == 7) launch_nw<7, 1, false>(nw, wstream, x_f32, grid, a, stream);
      else if (NT == 4) launch_nw<4, 1, false>(nw, wstream, x_f32, grid, a, stream);
      else if (NT == 2) launch_nw<2, 1, false>(nw, wstream, x_f32, grid, a, stream);
      else launch_nw<1, 1, false>(nw, wstream, x_f32, grid, a, stream);
    }
  } else if (RB == 2) {
    int nw = wgs <= 128 ? 16 : 8;
    if (g_force_nw) nw = g_force_nw;
    if (swiglu) launch_nw<2, 2, true>(nw, wstream, x_f32, grid, a, stream);
    else if (NT == 2) launch_nw<2, 2, false>(nw, wstream, x_f32, grid, a, stream);
    else launch_nw<1, 2, false>(nw, wstream, x_f32, grid, a, stream);
  } else {
    if (x_f32) {
      // 64-row tiles (prefills of 65+ rows, im2col convolutions): waves split K inside the workgroup (nw4), the
      // column tiles per workgroup share each X read; fo_gemm_tune forces (waves, tiles) for sweeps
      int nw4 = nw_pref4 ? nw_pref4 : 4;
      if (g_force_nw) nw4 = g_force_nw;
#define FO_B4(NT_, NW_, SW_) launch_gemm<NT_, 4, NW_, 2, SW_>(wstream, x_f32, grid, a, stream)
      if (swiglu) {
        if (NT == 8) FO_B4(8, 4, true);
        else if (NT == 4) { if (nw4 >= 8) FO_B4(4, 8, true); else FO_B4(4, 4, true); }
        else { if (nw4 >= 16) FO_B4(2, 16, true); else if (nw4 == 8) FO_B4(2, 8, true); else FO_B4(2, 4, true); }
      } else if (NT == 8) FO_B4(8, 4, false);
      else if (NT == 4) { if (nw4 >= 8) FO_B4(4, 8, false); else FO_B4(4, 4, false); }
      else if (NT == 2) { if (nw4 >= 16) FO_B4(2, 16, false); else if (nw4 == 8) FO_B4(2, 8, false); else FO_B4(2, 4, false); }
      else { if (nw4 >= 16) FO_B4(1, 16, false); else if (nw4 == 8) FO_B4(1, 8, false); else FO_B4(1, 4, false); }
#undef FO_B4
    } else {
      if (swiglu) launch_gemm<2, 4, 4, 4, true>(wstream, x_f32, grid, a, stream);
      else if (NT == 4) launch_gemm<4, 4, 4, 4, false>(wstream, x_f32, grid, a, stream);
      else if (NT == 2) launch_gemm<2, 4, 4, 4, false>(wstream, x_f32, grid, a, stream);
      else launch_gemm<1, 4, 4, 4, false>(wstream, x_f32, grid, a, stream);
    }
  }
  const bool pipe_k = RB == 1 && x_f32 && (launch_pipe || (g_launch_u != 4 && NT <= 2));
  g_launch_pipe = 0;
  g_launch_u = 4;
  fo::count_launch(lnw ? FO_L_GEMM_LN : (mid ? FO_L_GEMM_MID : (pipe_k ? FO_L_GEMM_PIPE : FO_L_GEMM_OTHER)));
  if (lnw && a.xp32) fo::count_launch(FO_L_GEMM_XP32);
  if (a.xph && x_f32 && !lnw && !swiglu && !pipe_k) fo::count_launch(FO_L_GEMM_XP);
  if (rope4) fo::count_launch(FO_L_GEMM_ROPE4);
  if (a.ypkh) fo::count_launch(FO_L_GEMM_YPACK);
  if (a.yp32) fo::count_launch(FO_L_GEMM_YPACK32);
  if (S > 1 && !merged) {
    int rc = fo::check_launch("fo_gemm/split");
    if (rc) return rc;
    launch_reduce(a, swiglu, mt * RB * 16, N, M, stream);
    fo::count_launch(FO_L_GEMM_REDUCE);
  }
  return fo::check_launch("fo_gemm");
}

int fo_gemm(const void* X, int x_f32, int ldx, int M, int K, const void* Wp, int N, int swiglu, const float* bias,
            const float* scale, const float* shift, void* Y, int ldy, int out_bf16, int act, int residual, float* ws,
            long long ws_floats, int* counters, int splitk, hipStream_t stream) {
  return gemm_impl(X, x_f32, ldx, M, K, Wp, N, swiglu, bias, scale, shift, Y, ldy, out_bf16, act, residual, ws,
                   ws_floats, counters, splitk, nullptr, 0, 0.f, nullptr, nullptr, nullptr, nullptr, nullptr, stream);
}

int fo_gemm_rms(const void* X, int x_f32, int ldx, int M, int K, const void* Wp, int N, int swiglu, const float* bias,
                void* Y, int ldy, int act, int residual, float* ws, long long ws_floats, int* counters, int splitk,
                const float* rstats, int rgroups, float eps, float* sout, const float* gnext, float* yg,
                int* sgroups, hipStream_t stream) {
  return gemm_impl(X, x_f32, ldx, M, K, Wp, N, swiglu, bias, nullptr, nullptr, Y, ldy, 0, act, residual, ws,
                   ws_floats, counters, splitk, rstats, rgroups, eps, sout, gnext, yg, sgroups, nullptr, stream);
}

int fo_gemm_ln(const float* X, int ldx, int M, int K, const void* Wp, int N, const float* bias, const float* lnw,
               const float* lnb, float eps, const float* rsum, const float* rsumsq, int rgroups, float* Y, int ldy,
               int act, float* ws, long long ws_floats, int splitk, hipStream_t stream) {
  FO_REQUIRE(lnw && lnb && rsum && rsumsq, "fo_gemm_ln: LayerNorm weight, bias and row statistics required");
  return gemm_impl(X, 1, ldx, M, K, Wp, N, 0, bias, nullptr, nullptr, Y, ldy, 0, act, 0, ws, ws_floats, nullptr,
                   splitk, rsumsq, rgroups, 0.f, nullptr, nullptr, nullptr, nullptr, nullptr, stream, lnw, lnb, eps,
                   nullptr, rsum);
}

int fo_gemm_rowstats(const void* X, int x_f32, int ldx, int M, int K, const void* Wp, int N, const float* bias,
                     float* Y, int ldy, int act, int residual, float* ws, long long ws_floats, int* counters,
                     int splitk, float* rsum, float* rsumsq, int* sgroups, hipStream_t stream) {
  FO_REQUIRE(rsum && rsumsq, "fo_gemm_rowstats: statistics buffers required");
  return gemm_impl(X, x_f32, ldx, M, K, Wp, N, 0, bias, nullptr, nullptr, Y, ldy, 0, act, residual, ws, ws_floats,
                   counters, splitk, nullptr, 0, 0.f, rsumsq, nullptr, nullptr, sgroups, nullptr, stream, nullptr,
                   nullptr, 0.f, rsum, nullptr);
}

int fo_gemm_qkv_rope(const void* X, int x_f32, int ldx, int M, int K, const void* Wp, int N, const float* bias,
                     float* ws, long long ws_floats, int* counters, int splitk, const float* rstats, int rgroups,
                     float eps, const int* pos, const int* slot, const float* cos_t, const float* sin_t, float* q_out,
                     float* kc, float* vc, int H, int KVH, int hd, int PS, hipStream_t stream) {
  FO_REQUIRE(pos && slot && cos_t && sin_t && q_out && kc && vc && PS > 0 && H > 0 && KVH > 0,
             "fo_gemm_qkv_rope: missing rope/cache arguments");
  GemmArgs r;
  r.rpos = pos;
  r.rslot = slot;
  r.rcos = cos_t;
  r.rsin = sin_t;
  r.rq = q_out;
  r.rk = kc;
  r.rv = vc;
  r.rH = H;
  r.rKVH = KVH;
  r.rhd = hd;
  r.rPS = PS;
  return gemm_impl(X, x_f32, ldx, M, K, Wp, N, 0, bias, nullptr, nullptr, q_out, N, 0, 0, 0, ws, ws_floats, counters,
                   splitk, rstats, rgroups, eps, nullptr, nullptr, nullptr, nullptr, &r, stream);
}

// Software-pipelining mode of the one-row-tile weight-stream GEMMs (k_gemm_wpipe): 0 off, 1 U k-steps,
// 2 two k-steps, 3 the default policy.  PROCESS-GLOBAL library state (not per thread or per stream):
// meant for sweeps and tests, which restore the previous mode.  Returns the previous mode (>= 0).
int fo_gemm_set_pipe(int on) {
  FO_REQUIRE(on >= 0 && on <= 3, "fo_gemm_set_pipe: 0 (off), 1 (U k-steps), 2 (2 k-steps) or 3 (policy)");
  const int prev = g_pipe;
  g_pipe = on;
  return prev;
}

// X-stationary kernel switch for the eligible M <= 16 GEMMs (k_gemm_xs): 0 off, 1 on.  Process-global
// (sweeps, A/B); returns the previous setting.  Unset, FO_GEMM_XS (default on) decides.
int fo_gemm_set_xsk_min_mb(int mb) {
  FO_REQUIRE(mb >= 0, "fo_gemm_set_xsk_min_mb: %d", mb);
  const int prev = g_xsk_min_mb;
  g_xsk_min_mb = mb;
  return prev;
}

int fo_set_kv_bf16(int on) {
  FO_REQUIRE(on == 0 || on == 1, "fo_set_kv_bf16: 0 or 1");
  const int prev = g_kv_bf16;
  g_kv_bf16 = on;
  return prev;
}

int fo_gemm_set_rows(int on) {
  FO_REQUIRE(on >= 0 && on <= 6,
             "fo_gemm_set_rows: 0 (row halves), 1 (k_gemm_rows), probes 2 (k_gemm_wrow), 3 (split consumer map), "
             "4 (from 33 rows), 5 / 6 (the weight ring alone)");
  const int prev = g_rows;
  g_rows = on;
  return prev;
}

int fo_gemm_set_xs(int on) {
  FO_REQUIRE(on == 0 || on == 1, "fo_gemm_set_xs: 0 or 1");
  const int prev = xs_mode() ? 1 : 0;
  g_xs = on;
  return prev;
}

int fo_gemm_set_merge(int on) {
  FO_REQUIRE(on >= 0 && on <= 2, "fo_gemm_set_merge: 0, 1 or 2");
  const int prev = merge_mode();
  g_merge = on;
  return prev;
}

int fo_gemm_set_xs_variant(int v) {
  FO_REQUIRE(v >= 0 && v <= 4, "fo_gemm_set_xs_variant: 0 (shipped), 1 (no reduction: wrong results), 2 (default "
             "cache policy), 3 (round 4's 8 waves x 14 k-steps), 4 (8 x 14, barrier-free reduction)");
  const int prev = xs_variant();
  g_xs_var = v;
  return prev;
}

int fo_probe_seam(const float* xo, int M, const void* wo, const float* bo, float* x, const float* gnext, float* yg,
                  float* sout, const void* wgu, int n_gu_out, float* h, float eps, int* ready, int* ready_timeout,
                  void* trace, int mode, hipStream_t s) {
  // mode 0: the seam launch (o + gate/up); 1: its o workgroups alone; 2: its gate/up workgroups alone (ready must
  // already hold n_o)
  constexpr int K = 3584, NO = 3584;
  FO_REQUIRE(M >= 1 && M <= 16 && n_gu_out % 16 == 0 && mode >= 0 && mode <= 2 && ready && ready_timeout,
             "fo_probe_seam: M=%d (1..16), gate/up outputs %d (a multiple of 16), mode %d", M, n_gu_out, mode);
  GemmArgs ao{};
  ao.X = xo; ao.Wp = reinterpret_cast<const bf16_t*>(wo); ao.bias = bo; ao.Y = x; ao.ldx = K; ao.ldy = NO;
  ao.M = M; ao.K = K; ao.N = NO; ao.ntiles = NO / 16; ao.S = 1; ao.residual = 1; ao.gnext = gnext; ao.yg = yg;
  ao.sout = sout;
  GemmArgs ag{};
  ag.X = yg; ag.Wp = reinterpret_cast<const bf16_t*>(wgu); ag.Y = h; ag.ldx = NO; ag.ldy = n_gu_out; ag.M = M;
  ag.K = K; ag.N = n_gu_out; ag.ntiles = 2 * n_gu_out / 16; ag.S = 1; ag.rstats = sout; ag.rgroups = NO / 32;
  ag.reps = eps;
  const int n_o = NO / 32, units = n_gu_out / 16;
  const int per = (units + num_cus() - 1) / num_cus(), G = (units + per - 1) / per;
  unsigned long long* trc = reinterpret_cast<unsigned long long*>(trace);
  if (mode == 0) hipLaunchKernelGGL(k_seam_o_gu, dim3(n_o + G), dim3(512), 0, s, ao, ag, n_o, units, G, ready,
                                    ready_timeout, trc);
  else if (mode == 1) hipLaunchKernelGGL(k_seam_o_gu, dim3(n_o), dim3(512), 0, s, ao, ag, n_o, units, G, ready,
                                         ready_timeout, trc);
  else hipLaunchKernelGGL(k_seam_o_gu, dim3(G), dim3(512), 0, s, ao, ag, 0, units, G, ready, ready_timeout, trc);
  return fo::check_launch("fo_probe_seam");
}

int fo_gemm_set_trace(void* trace) {
  FO_REQUIRE(FO_GEMM_TRACE || !trace,
             "fo_gemm_set_trace: this library is built without the GEMM clock hook (make probe -> fo/libfo_hip_probe.so, "
             "loaded with FO_LIB_PATH)");
  g_trc = reinterpret_cast<unsigned long long*>(trace);
  return 0;
}

int fo_gemm_set_xpack(const void* hi, const void* lo, int cols, int cap_rb) {
  return arm_pack(g_xpk, hi, lo, true, cols, cap_rb, "fo_gemm_set_xpack");
}

int fo_gemm_set_ypack32(void* p, int cols, int cap_rb) {
  return arm_pack(g_yp32k, p, nullptr, false, cols, cap_rb, "fo_gemm_set_ypack32");
}

int fo_gemm_set_xpack32(const void* p, int cols, int cap_rb) {
  return arm_pack(g_xp32k, p, nullptr, false, cols, cap_rb, "fo_gemm_set_xpack32");
}

int fo_gemm_set_ypack(void* hi, void* lo, int cols, int cap_rb) {
  return arm_pack(g_ypk, hi, lo, true, cols, cap_rb, "fo_gemm_set_ypack");
}

int fo_gemm_set_u(int u) {
  FO_REQUIRE(u == 0 || u == 4 || u == 7 || u == 8, "fo_gemm_set_u: u must be 0/4/7/8");
  g_force_u = u;
  return 0;
}

int fo_gemm_tune(int nw, int nt) {
  FO_REQUIRE(nw == 0 || nw == 4 || nw == 8 || nw == 16, "fo_gemm_tune: nw must be 0/4/8/16");
  FO_REQUIRE(nt == 0 || nt == 1 || nt == 2 || nt == 4 || nt == 7 || nt == 8, "fo_gemm_tune: nt must be 0/1/2/4/7/8");
  g_force_nw = nw;
  g_force_nt = nt;
  return 0;
}

long long fo_pack_weight_elems(int N, int K) { return (long long)((N + 15) / 16) * 16 * ((K + 31) / 32) * 32; }

// Pack W[N][K] into fragment order at tile offset tile_base with stride tile_stride (tiles of 16 rows).
int fo_pack_weight(const void* W, int src_bf16, int N, int K, int ldw, void* out, int tile_base, int tile_stride,
                   hipStream_t stream) {
  FO_REQUIRE(N > 0 && K > 0 && ldw >= K, "fo_pack_weight: bad shape");
  const int KSp = (K + 31) / 32;
  const int nt = (N + 15) / 16;
  const size_t total = (size_t)nt * KSp * 64;
  int blocks = (int)((total + 255) / 256);
  if (blocks > 65535) blocks = 65535;
  hipLaunchKernelGGL(k_pack, dim3(blocks), dim3(256), 0, stream, W, src_bf16, N, K, ldw, (bf16_t*)out, KSp,
                     tile_base, tile_stride, nt);
  return fo::check_launch("fo_pack_weight");
}

}  // extern "C"
