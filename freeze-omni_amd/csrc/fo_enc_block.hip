// The attention half of a speech-encoder block in ONE launch (models/encoder/transformer.py:103-118
// TransformerLayer.infer with normalize_before, concat_after False; MultiHeadedAttention.infer with rel-pos and the
// left-chunk ring, models/encoder/attention.py:407-459):
//
//   x  += linear_out( relpos_attention( q|k|v = linear_qkv( LayerNorm1(x) ), ring ) )
//
// One workgroup per (session b, head hh), 16 waves:
//  * the head's slice of linear_out (d x dk) is loaded into registers at the start, while everything else runs;
//  * LayerNorm1 of the session's T rows (a wave per row) into LDS, then 12 waves each compute one 16-column tile of
//    the head's q / k / v (K = d on the matrix cores, the normalised rows split into bf16 hi + lo as they are read,
//    +bias) into LDS;
//  * the rel-pos attention of k_relpos_fused over the ring + the chunk's new rows (which are also appended to the
//    ring), scores (q + u) K^T + (q + v) P^T, softmax, P.V -- out of LDS;
//  * o_h = att_h . Wout[:, hh dk : (hh + 1) dk]^T, an N = d partial per head, published to a slab; the last head to
//    finish for a session (agent-scope release / acquire ticket) sums the h partials in head order (deterministic),
//    adds linear_out's bias and the residual, writes x in place and the rows' sums / sums of squares (one statistics
//    group: the next LayerNorm-on-load GEMM, feed_forward.w_1, reads them).
// Workgroups of one head share an XCD (their weight slices come from its L2).  Replaces fo_gemm_ln (q|k|v) +
// fo_relpos_attention_fused + fo_gemm_rowstats (out): three launches and their hand-offs per block.
#include "fo_common.h"

namespace {

constexpr int EB_NW = 16;            // waves per workgroup
constexpr int EB_NT = EB_NW * 64;
constexpr int EB_DK = 64;            // head size (the real and tiny encoders)
constexpr int EB_TMAX = 8;           // rows per session (framing A: 4, framing B: 7)
constexpr int EB_LMAX = 96;          // ring + chunk keys staged in LDS
constexpr int EB_DMAX = 1024;        // model width (the normalised rows are staged in LDS)

struct EncBlockArgs {
  float* x;                 // [B*T][d] residual stream, updated in place
  const float* lnw;         // LayerNorm1 weight / bias [d]
  const float* lnb;
  float ln_eps;
  const bf16x8* wqkv;       // linear_q|k|v packed [3d/16][d/32][64][8]
  const float* bqkv;        // [3d]
  float* kr;                // ring K / V [slots][cap][d]
  float* vr;
  int cap;
  const int* meta;          // [start B][len B][ring B][pstart B]
  const float* ptab;        // [positions][d]: linear_pos(sinusoid(p)) of this layer
  const float* bu;          // pos_bias_u / pos_bias_v [h][dk]
  const float* bv;
  const bf16x8* wout;       // linear_out packed [d/16][d/32][64][8]
  const float* bout;        // [d]
  float* part;              // [B][h][T][d] head partials
  int* tickets;             // [B], zeroed, left zeroed
  float* ssum;              // [B*T] row sums / sums of squares of the updated x
  float* ssq;
  const float* qkv;         // QKV_IN: the chunk's q|k|v rows [B*T][ldq] (+ bias) from the LayerNorm-on-load GEMM
  int ldq;
  int B, T, d, h;
  float scale;
};

__device__ __forceinline__ void split_hl(const float* f, bf16x8& hi, bf16x8& lo) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const __bf16 hv = (__bf16)f[e];
    hi[e] = hv;
    lo[e] = (__bf16)(f[e] - (float)hv);
  }
}

// OT: 16-column out-projection tiles per wave (d / 16 / EB_NW).  QKV_IN: q|k|v come from the GEMM's output (a.qkv)
// instead of LayerNorm1 + linear_q|k|v in this launch (the attention, linear_out and residual half only)
template <int OT, bool QKV_IN>
__global__ __launch_bounds__(EB_NT) void k_enc_attn_block(EncBlockArgs a) {
  constexpr int KP = EB_DK + 4;
  __shared__ float xn_s[EB_TMAX][EB_DMAX];   // LayerNorm1(x) of the session's rows
  __shared__ float nq_s[3][EB_TMAX][EB_DK];   // the chunk's q + u / k / v rows of this head (+ bias)
  __shared__ float qv_s[EB_TMAX][EB_DK];      // q + v
  __shared__ float k_s[EB_LMAX][KP];
  __shared__ float v_s[EB_LMAX][KP];
  __shared__ float p_s[EB_LMAX][KP];
  __shared__ float sc_s[EB_TMAX][EB_LMAX];
  __shared__ float att_s[EB_TMAX][EB_DK];
  __shared__ int last_s;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  // (session, head) from an XCD-aware 1-D grid: workgroup id % 8 == head % 8
  const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
  const int hh = xcd + 8 * (slot / a.B), b = slot % a.B;
  if (hh >= a.h) return;
  const int T = a.T, d = a.d, KS = d >> 5;
  const int row0 = b * T;
  // ---- the head's linear_out slice: wave w owns output tiles w*OT .. +OT, both k-steps of the head
  bf16x8 wo[OT][2];
#pragma unroll
  for (int t = 0; t < OT; ++t)
#pragma unroll
    for (int k = 0; k < 2; ++k)
      wo[t][k] = __builtin_nontemporal_load(a.wout + ((size_t)(wave * OT + t) * KS + 2 * hh + k) * 64 + lane);
  // ---- q | k | v: wave w < 12 -> matrix w / 4 (q, k, v), tile w % 4 of the head's 64 columns; its first group of
  // weight fragments is requested before the LayerNorm so it lands while the norm runs
  constexpr int G = 8;   // k-steps of weights in flight per group
  const int mat = wave >> 2, qt = wave & 3;
  const bf16x8* bp = QKV_IN ? nullptr : a.wqkv + (size_t)(mat * (d >> 4) + hh * (EB_DK >> 4) + qt) * KS * 64 + lane;
  bf16x8 wf[G];
  if (QKV_IN) {   // the head's q|k|v rows (+ the u / v position biases on q)
    for (int e = tid; e < T * EB_DK; e += EB_NT) {
      const int i = e / EB_DK, c = e % EB_DK;
      const float* src = a.qkv + (size_t)(row0 + i) * a.ldq + hh * EB_DK + c;
      const float q = src[0];
      nq_s[0][i][c] = q + a.bu[hh * EB_DK + c];
      qv_s[i][c] = q + a.bv[hh * EB_DK + c];
      nq_s[1][i][c] = src[d];
      nq_s[2][i][c] = src[2 * d];
    }
  } else if (wave < 12) {
#pragma unroll
    for (int j = 0; j < G; ++j) wf[j] = __builtin_nontemporal_load(bp + (size_t)j * 64);
  }
  // ---- LayerNorm1 of the session's rows (a wave per row; d / 256 float4 per lane, kept in registers)
  if (!QKV_IN && wave < T) {
    const float* xr = a.x + (size_t)(row0 + wave) * d;
    float4 v[EB_DMAX / 256];
    float s = 0.f, s2 = 0.f;
#pragma unroll
    for (int q = 0; q < EB_DMAX / 256; ++q) {
      const int c = lane * 4 + q * 256;
      v[q] = c < d ? *reinterpret_cast<const float4*>(xr + c) : make_float4(0.f, 0.f, 0.f, 0.f);
      s += v[q].x + v[q].y + v[q].z + v[q].w;
      s2 += v[q].x * v[q].x + v[q].y * v[q].y + v[q].z * v[q].z + v[q].w * v[q].w;
    }
    s = wave_sum(s);
    s2 = wave_sum(s2);
    const float mean = s / (float)d;
    const float rstd = 1.0f / sqrtf(fmaxf(s2 / (float)d - mean * mean, 0.f) + a.ln_eps);
#pragma unroll
    for (int q = 0; q < EB_DMAX / 256; ++q) {
      const int c = lane * 4 + q * 256;
      if (c < d) {
        const float4 w4 = *reinterpret_cast<const float4*>(a.lnw + c), b4 = *reinterpret_cast<const float4*>(a.lnb + c);
        *reinterpret_cast<float4*>(&xn_s[wave][c]) =
            make_float4((v[q].x - mean) * rstd * w4.x + b4.x, (v[q].y - mean) * rstd * w4.y + b4.y,
                        (v[q].z - mean) * rstd * w4.z + b4.z, (v[q].w - mean) * rstd * w4.w + b4.w);
      }
    }
  }
  __syncthreads();
  if (!QKV_IN && wave < 12) {
    const int r = min(lane & 15, T - 1);   // rows >= T: computed from a valid row, never kept
    const float* xr = &xn_s[r][8 * (lane >> 4)];
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int k0 = 0; k0 < KS; k0 += G) {
      bf16x8 wn[G];
      if (k0 + G < KS) {   // the next group in flight while this one computes
#pragma unroll
        for (int j = 0; j < G; ++j) wn[j] = __builtin_nontemporal_load(bp + (size_t)(k0 + G + j) * 64);
      }
#pragma unroll
      for (int j = 0; j < G; ++j) {
        const float4 x0 = *reinterpret_cast<const float4*>(xr + (k0 + j) * 32);
        const float4 x1 = *reinterpret_cast<const float4*>(xr + (k0 + j) * 32 + 4);
        const float f[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
        bf16x8 hi, lo;
        split_hl(f, hi, lo);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(hi, wf[j], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(lo, wf[j], acc, 0, 0, 0);
      }
      if (k0 + G < KS) {
#pragma unroll
        for (int j = 0; j < G; ++j) wf[j] = wn[j];
      }
    }
    // D: row 4 (lane >> 4) + i, column lane & 15
    const int col = qt * 16 + (lane & 15);
    const float bias = a.bqkv[mat * d + hh * EB_DK + col];
    const float pu = mat == 0 ? a.bu[hh * EB_DK + col] : 0.f, pv = mat == 0 ? a.bv[hh * EB_DK + col] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int rr = 4 * (lane >> 4) + i;
      if (rr < T) {
        nq_s[mat][rr][col] = acc[i] + bias + pu;
        if (mat == 0) qv_s[rr][col] = acc[i] + bias + pv;
      }
    }
  }
  __syncthreads();
  // ---- rel-pos attention (k_relpos_fused's arithmetic): keys = ring rows (old) + the chunk's new rows
  const int* meta = a.meta;
  const int st = meta[b], Lold = meta[a.B + b], ps = meta[3 * a.B + b];
  const size_t rb = (size_t)meta[2 * a.B + b];
  const int Lk = Lold + T;
  const int hd0 = hh * EB_DK;
  for (int e = tid; e < Lk * (EB_DK / 4); e += EB_NT) {
    const int j = e / (EB_DK / 4), c = (e % (EB_DK / 4)) * 4;
    float4 kk, vv;
    if (j < Lold) {
      const size_t ro = (rb * a.cap + (st + j) % a.cap) * d + hd0 + c;
      kk = *reinterpret_cast<const float4*>(a.kr + ro);
      vv = *reinterpret_cast<const float4*>(a.vr + ro);
    } else {   // the chunk's new rows: from LDS, and appended to the ring
      kk = *reinterpret_cast<const float4*>(&nq_s[1][j - Lold][c]);
      vv = *reinterpret_cast<const float4*>(&nq_s[2][j - Lold][c]);
      const size_t ro = (rb * a.cap + (st + j) % a.cap) * d + hd0 + c;
      *reinterpret_cast<float4*>(a.kr + ro) = kk;
      *reinterpret_cast<float4*>(a.vr + ro) = vv;
    }
    const float4 pp = *reinterpret_cast<const float4*>(a.ptab + (size_t)(ps + j) * d + hd0 + c);
    *reinterpret_cast<float4*>(&k_s[j][c]) = kk;
    *reinterpret_cast<float4*>(&v_s[j][c]) = vv;
    *reinterpret_cast<float4*>(&p_s[j][c]) = pp;
  }
  __syncthreads();
  for (int e = tid; e < T * Lk; e += EB_NT) {
    const int i = e / Lk, j = e - (e / Lk) * Lk;
    float s1 = 0.f, s2 = 0.f;
#pragma unroll 4
    for (int c = 0; c < EB_DK; c += 4) {
      const float4 u4 = *reinterpret_cast<const float4*>(&nq_s[0][i][c]);
      const float4 w4 = *reinterpret_cast<const float4*>(&qv_s[i][c]);
      const float4 k4 = *reinterpret_cast<const float4*>(&k_s[j][c]);
      const float4 p4 = *reinterpret_cast<const float4*>(&p_s[j][c]);
      s1 += u4.x * k4.x + u4.y * k4.y + u4.z * k4.z + u4.w * k4.w;
      s2 += w4.x * p4.x + w4.y * p4.y + w4.z * p4.z + w4.w * p4.w;
    }
    sc_s[i][j] = (s1 + s2) * a.scale;
  }
  __syncthreads();
  if (wave < T) {
    const int i = wave;
    float m = -INFINITY;
    for (int j = lane; j < Lk; j += 64) m = fmaxf(m, sc_s[i][j]);
    m = wave_max(m);
    float sum = 0.f;
    for (int j = lane; j < Lk; j += 64) {
      const float e = expf(sc_s[i][j] - m);
      sc_s[i][j] = e;
      sum += e;
    }
    sum = wave_sum(sum);
    const float r = 1.f / sum;
    for (int j = lane; j < Lk; j += 64) sc_s[i][j] *= r;
  }
  __syncthreads();
  for (int e = tid; e < T * EB_DK; e += EB_NT) {
    const int i = e / EB_DK, c = e % EB_DK;
    float acc = 0.f;
    for (int j = 0; j < Lk; ++j) acc += sc_s[i][j] * v_s[j][c];
    att_s[i][c] = acc;
  }
  __syncthreads();
  // ---- o_h partial: att (T x dk, rows >= T zero) . Wout slice^T, wave w -> output tiles w*OT ..
  bf16x8 ah[2], al[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    float f[8];
    const int r = lane & 15;
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] = r < T ? att_s[r][k * 32 + 8 * (lane >> 4) + e] : 0.f;
    split_hl(f, ah[k], al[k]);
  }
  float* pb = a.part + ((size_t)b * a.h + hh) * T * d;
#pragma unroll
  for (int t = 0; t < OT; ++t) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[k], wo[t][k], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[k], wo[t][k], acc, 0, 0, 0);
    }
    const int n = (wave * OT + t) * 16 + (lane & 15);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int rr = 4 * (lane >> 4) + i;
      if (rr < T) pb[(size_t)rr * d + n] = acc[i];
    }
  }
  // ---- publish the partial; the session's last head merges (release / acquire ticket, as the split merge)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int old = __hip_atomic_fetch_add(a.tickets + b, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last_s = old == a.h - 1;
  }
  __syncthreads();
  if (!last_s) return;
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(a.tickets + b, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  // x += bias + sum_h partials: every thread takes float4 columns of the session's rows; the partials come from
  // other XCDs' workgroups (a memory-side round trip each), so all h loads of an element are issued together, then
  // summed in head order (deterministic).  The updated rows are also kept in LDS (xn_s is free) for the statistics.
  const int D4 = d >> 2;
  const float* pb0 = a.part + (size_t)b * a.h * T * d;
  for (int e = tid; e < T * D4; e += EB_NT) {
    const int r = e / D4, c = (e - r * D4) * 4;
    const float4 xo = *reinterpret_cast<const float4*>(a.x + (size_t)(row0 + r) * d + c);
    float4 acc = *reinterpret_cast<const float4*>(a.bout + c);
    for (int g0 = 0; g0 < a.h; g0 += 16) {
      float4 pv[16];
#pragma unroll
      for (int j = 0; j < 16; ++j)
        pv[j] = g0 + j < a.h ? *reinterpret_cast<const float4*>(pb0 + ((size_t)(g0 + j) * T + r) * d + c)
                             : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        acc.x += pv[j].x;
        acc.y += pv[j].y;
        acc.z += pv[j].z;
        acc.w += pv[j].w;
      }
    }
    const float4 xv = make_float4(xo.x + acc.x, xo.y + acc.y, xo.z + acc.z, xo.w + acc.w);
    *reinterpret_cast<float4*>(a.x + (size_t)(row0 + r) * d + c) = xv;
    *reinterpret_cast<float4*>(&xn_s[r][c]) = xv;
  }
  __syncthreads();
  if (wave < T) {   // a wave per row: the updated row's sum and sum of squares
    const int r = wave;
    float s = 0.f, s2 = 0.f;
    for (int c = lane * 4; c < d; c += 256) {
      const float4 xv = *reinterpret_cast<const float4*>(&xn_s[r][c]);
      s += xv.x + xv.y + xv.z + xv.w;
      s2 += xv.x * xv.x + xv.y * xv.y + xv.z * xv.z + xv.w * xv.w;
    }
    s = wave_sum(s);
    s2 = wave_sum(s2);
    if (lane == 0) {
      a.ssum[row0 + r] = s;
      a.ssq[row0 + r] = s2;
    }
  }
}

int launch(const EncBlockArgs& a, hipStream_t s, bool qkv_in, const char* what) {
  const int grid = 8 * a.B * ((a.h + 7) / 8);
  const int ot = a.d / 16 / EB_NW;
#define FO_EB_LAUNCH(OT_)                                                                                  \
  if (qkv_in) hipLaunchKernelGGL((k_enc_attn_block<OT_, true>), dim3(grid), dim3(EB_NT), 0, s, a);       \
  else hipLaunchKernelGGL((k_enc_attn_block<OT_, false>), dim3(grid), dim3(EB_NT), 0, s, a);
  if (ot == 4) { FO_EB_LAUNCH(4) }
  else if (ot == 2) { FO_EB_LAUNCH(2) }
  else if (ot == 1) { FO_EB_LAUNCH(1) }
  else FO_REQUIRE(false, "%s: d=%d needs d / 256 in {1, 2, 4}", what, a.d);
#undef FO_EB_LAUNCH
  fo::count_launch(FO_L_ENC_BLOCK);
  return fo::check_launch(what);
}

}  // namespace

extern "C" {

int fo_enc_attn_block(float* x, int B, int T, int d, int h, const float* lnw, const float* lnb, float ln_eps,
                      const void* wqkv, const float* bqkv, float* kr, float* vr, int cap, const int* meta,
                      const float* ptab, const float* bu, const float* bv, const void* wout, const float* bout,
                      float scale, float* part, int* tickets, float* ssum, float* ssq, hipStream_t s) {
  FO_REQUIRE(B > 0 && T >= 1 && T <= EB_TMAX && h > 0 && d == h * EB_DK && (d % (16 * EB_NW)) == 0 &&
                 d <= EB_DMAX && cap + T <= EB_LMAX,
             "fo_enc_attn_block: B=%d T=%d d=%d h=%d cap=%d (head size %d, T <= %d, d a multiple of %d, ring + "
             "chunk <= %d keys)", B, T, d, h, cap, EB_DK, EB_TMAX, 16 * EB_NW, EB_LMAX);
  FO_REQUIRE(x && lnw && lnb && wqkv && bqkv && kr && vr && meta && ptab && bu && bv && wout && bout && part &&
                 tickets && ssum && ssq, "fo_enc_attn_block: null argument");
  EncBlockArgs a{x, lnw, lnb, ln_eps, reinterpret_cast<const bf16x8*>(wqkv), bqkv, kr, vr, cap, meta, ptab, bu, bv,
                 reinterpret_cast<const bf16x8*>(wout), bout, part, tickets, ssum, ssq, nullptr, 0, B, T, d, h, scale};
  return launch(a, s, false, "fo_enc_attn_block");
}

int fo_enc_attn_out(const float* qkv, int ldq, float* x, int B, int T, int d, int h, float* kr, float* vr, int cap,
                    const int* meta, const float* ptab, const float* bu, const float* bv, const void* wout,
                    const float* bout, float scale, float* part, int* tickets, float* ssum, float* ssq,
                    hipStream_t s) {
  FO_REQUIRE(B > 0 && T >= 1 && T <= EB_TMAX && h > 0 && d == h * EB_DK && (d % (16 * EB_NW)) == 0 &&
                 d <= EB_DMAX && cap + T <= EB_LMAX && ldq >= 3 * d,
             "fo_enc_attn_out: B=%d T=%d d=%d h=%d cap=%d ldq=%d (head size %d, T <= %d, d a multiple of %d, ring + "
             "chunk <= %d keys, ldq >= 3d)", B, T, d, h, cap, ldq, EB_DK, EB_TMAX, 16 * EB_NW, EB_LMAX);
  FO_REQUIRE(qkv && x && kr && vr && meta && ptab && bu && bv && wout && bout && part && tickets && ssum && ssq,
             "fo_enc_attn_out: null argument");
  EncBlockArgs a{x, nullptr, nullptr, 0.f, nullptr, nullptr, kr, vr, cap, meta, ptab, bu, bv,
                 reinterpret_cast<const bf16x8*>(wout), bout, part, tickets, ssum, ssq, qkv, ldq, B, T, d, h, scale};
  return launch(a, s, true, "fo_enc_attn_out");
}

}  // extern "C"
