// Attention for the Freeze-Omni hot path.
//
// 1. Decoder attention over a paged KV cache (Qwen2 in AudioLLM, Llama layers of the AR speech
//    decoder).  Reference: transformers Qwen2Attention/LlamaAttention reached from
//    models/audioLLM.py:482 and models/decoder/decoder.py:294-312 (DynamicCache concat per layer).
//    Here the cache is a pool of fixed-size pages per layer, laid out [page][kv_head][slot][hd]
//    (fp32) so one head's keys in a page are contiguous; sequences own block tables, so a
//    shared system prompt is shared pages and growth never copies.
//    Ragged batch: every token carries (sequence, absolute position); causal mode lets a query
//    see keys at positions <= its own, full mode (the reference's eager attention with
//    attention_mask=None / all-ones masks, decoder.py:140,175,302) sees the whole sequence.
//    Work items group a sequence's batch tokens (x the GQA group of query heads sharing one kv
//    head) so its keys are read once per kv head; split-KV over key ranges sized from each item's
//    own key count at run time, merged in the same launch by the last split to finish (or, without
//    a ticket buffer, static splits merged by a combine kernel).
// 2. Encoder rel-pos attention over a per-user ring buffer (models/encoder/attention.py:407-459):
//    scores = ((q+u).K^T + (q+v).P^T)/sqrt(dk), no mask, no rel_shift; P rows come from a
//    table of linear_pos(sinusoid(position)) precomputed at load for every position.
#include "fo_common.h"

namespace {

__global__ __launch_bounds__(256) void k_rope_kv_write(const float* qkv, int ldq, int T, int H, int KVH, int hd,
                                                       const int* pos, const int* slot, const float* cos_t,
                                                       const float* sin_t, float* q_out, float* kc, float* vc,
                                                       int PS) {
  const int t = blockIdx.x;
  const int half = hd >> 1;
  const float* row = qkv + (size_t)t * ldq;
  const int p = pos[t];
  const float* cs = cos_t + (size_t)p * half;
  const float* sn = sin_t + (size_t)p * half;
  const int sl = slot[t];
  const int page = sl / PS, off = sl % PS;
  // q heads then k heads: rotate pairs (i, i + hd/2)
  for (int e = threadIdx.x; e < (H + KVH) * half; e += blockDim.x) {
    const int h = e / half, i = e % half;
    const float* src = row + (size_t)h * hd;  // q heads [0,H), k heads [H, H+KVH) are contiguous
    const float x1 = src[i], x2 = src[i + half];
    const float c = cs[i], s = sn[i];
    const float o1 = x1 * c - x2 * s;
    const float o2 = x2 * c + x1 * s;
    if (h < H) {
      q_out[(size_t)t * H * hd + (size_t)h * hd + i] = o1;
      q_out[(size_t)t * H * hd + (size_t)h * hd + i + half] = o2;
    } else {
      float* d = kc + (((size_t)page * KVH + (h - H)) * PS + off) * hd;
      d[i] = o1;
      d[i + half] = o2;
    }
  }
  const float* vsrc = row + (size_t)(H + KVH) * hd;
  for (int e = threadIdx.x; e < KVH * hd; e += blockDim.x) {
    const int h = e / hd, i = e % hd;
    vc[(((size_t)page * KVH + h) * PS + off) * hd + i] = vsrc[e];
  }
}

struct AttnArgs {
  const float* q;          // [T][H*hd], rotated
  const int* items;        // [n_items][3]: sequence, first token, token count (a sequence's tokens are contiguous)
  const int* tok_nvis;     // keys visible to each query token (causal: own cache index + 1; full: all)
  const int* block_table;  // [S][maxb]
  const float* kc;
  const float* vc;
  float* part_ml;  // [T*H][nsplit][2]   (nsplit > 1)
  float* part_o;   // [T*H][nsplit][hd]  (nsplit > 1)
  float* out;      // [T][H*hd]
  int H, KVH, PS, maxb, nsplit;
  float scale;
  // in-launch merge: a work item uses min(nsplit, ceil(keys / kps)) splits, chosen from its own key
  // count at run time (one captured graph serves a context as it grows); the last split to finish
  // (arrival ticket cnt[item][kv head], reset by that split) merges the partials -- no combine launch
  int* cnt;        // nullable: static nsplit splits + k_attn_combine
  int kps;
  int tnu;         // items NULL: tokens per item (item b = sequence b, tokens b*tnu .. b*tnu + tnu - 1)
};

constexpr int KT = 64;      // keys per LDS tile (one key per lane in the score phase)
constexpr int MAXPG = 256;  // pages of one split staged in LDS (fo_attn_nsplit keeps splits <= 4096 keys)

// fp32 -> bf16 hi + lo: two bf16 operands whose sum carries ~16 mantissa bits
__device__ __forceinline__ void split8(const float* f, bf16x8& hi, bf16x8& lo) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const __bf16 h = (__bf16)f[i];
    hi[i] = h;
    lo[i] = (__bf16)(f[i] - (float)h);
  }
}

// sum / max over the 16 lanes of a row group (lanes l, l^1, l^2, l^4, l^8)
__device__ __forceinline__ float row16_max(float v) {
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float row16_sum(float v) {
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Split `sp` of work item `it` has written its partial (part_o / part_ml): publish it and take an
// arrival ticket; the split that draws ns - 1 merges all ns partials of the item's R rows with
// k_attn_combine's arithmetic and resets the ticket for the next launch.  Protocol: every wave drains
// its stores, lane 0 releases at agent scope before the relaxed ticket add, the merging split acquires
// at agent scope before reading (correct for any placement of the splits over XCDs).
// last_s / w_s: the kernel's existing LDS (no second __shared__ object for the flag).
template <int HD>
__device__ void attn_arrive_and_merge(const AttnArgs& a, int it, int kvh, int ns, int t0, int R, int G,
                                      int& last_s, float* w_s) {
  const int tid = threadIdx.x;
  int* ticket = a.cnt + (size_t)it * a.KVH + kvh;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int old = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last_s = old == ns - 1;
  }
  __syncthreads();
  if (!last_s) return;
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  // per row: split weights exp(m_q - M) (0 for empty splits) and 1 / l into LDS (w_s: [16][KT + 4],
  // the kernel's P tile, ns <= KT), then every (row, d) sums its ns partials with independent loads
  for (int r = tid; r < R; r += blockDim.x) {
    const size_t th = (size_t)(t0 + r / G) * a.H + kvh * G + r % G;
    const float* ml = a.part_ml + th * a.nsplit * 2;
    float M = -INFINITY;
    for (int q = 0; q < ns; ++q)
      if (ml[2 * q + 1] > 0.f) M = fmaxf(M, ml[2 * q]);
    float l = 0.f;
    for (int q = 0; q < ns; ++q) {
      const float ls = ml[2 * q + 1];
      const float w = ls > 0.f ? expf(ml[2 * q] - M) : 0.f;
      if (ls > 0.f) l += ls * w;
      w_s[r * (KT + 4) + q] = w;
    }
    w_s[r * (KT + 4) + KT] = 1.f / l;
  }
  __syncthreads();
  for (int e = tid; e < R * HD; e += blockDim.x) {
    const int r = e / HD, d = e - (e / HD) * HD;
    const size_t th = (size_t)(t0 + r / G) * a.H + kvh * G + r % G;
    const float* po = a.part_o + th * a.nsplit * HD + d;
    const float* w = w_s + r * (KT + 4);
    float o = 0.f;
    for (int q = 0; q < ns; ++q)
      if (w[q] != 0.f) o += po[(size_t)q * HD] * w[q];
    a.out[th * HD + d] = o * w[KT];
  }
}

// One work item = up to 16 query rows (a sequence's batch tokens x the GQA group sharing one kv head)
// against that kv head, over split `sp` of the sequence's keys, on the matrix cores:
//   S = Q K^T   (A = Q rows, B = K rows read straight from the paged cache in B-fragment order)
//   O = P V     (A = P through LDS, B = V staged in LDS as [key][d])
// 64-key tiles, one 16-key column block per wave; K and V of the next tile are loaded into registers
// while the current tile computes.  Every fp32 operand is split into bf16 hi + lo and each product
// uses three MFMAs (hi*hi + hi*lo + lo*hi), so scores and outputs keep ~fp32 accuracy.  Online
// softmax per row with the running max exchanged across the 4 waves through LDS.
template <int HD, int NW = 4>
__global__ __launch_bounds__(NW * 64) void k_attn_mfma(AttnArgs a) {
  constexpr int KT = 16 * NW;           // keys per tile: one 16-key column block per wave
  constexpr int NTH = NW * 64;
  constexpr int DC = HD / 32;            // 32-wide d chunks (score k-steps)
  constexpr int NTILE = HD / 16;         // 16-wide d tiles of the output
  constexpr int NTW = (NTILE + NW - 1) / NW;   // output tiles per wave
  constexpr int VP = HD + 2;             // V row pitch: the 4 key groups of a B fragment hit distinct banks
  constexpr int VL = KT * HD / 4 / NTH;  // float4 of V per thread per tile
  __shared__ float v_s[KT][VP];
  __shared__ float p_s[16][KT + 4];
  __shared__ float mx_s[NW][16];
  __shared__ float l_s[NW][16];
  __shared__ int nvis_s[16];
  __shared__ int pg_s[MAXPG];

  const int it = blockIdx.x, kvh = blockIdx.y, sp = blockIdx.z;
  // items NULL: a uniform batch (tnu tokens per sequence, in sequence order) -- no item-table round trip
  const int seq = a.items ? a.items[3 * it] : it, t0 = a.items ? a.items[3 * it + 1] : it * a.tnu;
  const int tn = a.items ? a.items[3 * it + 2] : a.tnu;
  const int G = a.H / a.KVH;
  const int R = tn * G;  // <= 16
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int grp = lane >> 4, col = lane & 15;
  const int* bt = a.block_table + (size_t)seq * a.maxb;
  // this lane's q row slices, requested before anything that waits (they depend only on t0)
  float4 qraw[2 * DC];
  {
    const int r = col < R ? col : R - 1;
    const float* qr = a.q + ((size_t)(t0 + r / G) * a.H + kvh * G + r % G) * HD + 8 * grp;
#pragma unroll
    for (int c = 0; c < DC; ++c) {
      qraw[2 * c] = *reinterpret_cast<const float4*>(qr + 32 * c);
      qraw[2 * c + 1] = *reinterpret_cast<const float4*>(qr + 32 * c + 4);
    }
  }
  // a block-table row that fits is staged whole, requested together with the key counts (no wait for
  // this split's page range first); longer rows stage the split's pages once the range is known
  const bool whole = a.maxb <= MAXPG;
  if (whole)
    for (int i = tid; i < a.maxb; i += NTH) pg_s[i] = bt[i];
  int Lmax = 0;
  for (int i = 0; i < tn; ++i) Lmax = max(Lmax, a.tok_nvis[t0 + i]);
  int ns = a.nsplit;
  if (a.cnt) {
    ns = min(ns, max(1, (Lmax + a.kps - 1) / a.kps));
    if (sp >= ns) return;  // beyond this item's splits: never counted, never read
  }
  const int per = ((Lmax + ns - 1) / ns + KT - 1) / KT * KT;
  const int c0 = sp * per, c1 = min(Lmax, c0 + per);
  if (c0 >= c1) {  // empty split: neutral partial
    for (int r = tid; r < R; r += NTH) {
      const size_t o = ((size_t)(t0 + r / G) * a.H + kvh * G + r % G) * a.nsplit + sp;
      a.part_ml[o * 2] = -INFINITY;
      a.part_ml[o * 2 + 1] = 0.f;
    }
    if (a.cnt) attn_arrive_and_merge<HD>(a, it, kvh, ns, t0, R, G, nvis_s[0], &p_s[0][0]);
    return;
  }
  const int pb0 = c0 / a.PS, npg = (c1 - 1) / a.PS - pb0 + 1;
  if (npg > MAXPG || (whole && (c1 - 1) / a.PS >= a.maxb)) {  // host contract broken: poison, never read wrong keys
    for (int r = tid; r < R; r += NTH) a.out[((size_t)(t0 + r / G) * a.H + kvh * G + r % G) * HD] = NAN;
    return;
  }
  const int pb = whole ? 0 : pb0;  // pg_s holds pages pb..
  if (!whole)
    for (int i = tid; i < npg; i += NTH) pg_s[i] = bt[pb + i];
  if (tid < 16) nvis_s[tid] = tid < R ? a.tok_nvis[t0 + tid / G] : 0;

  // Q as A fragments: row = col (lane & 15), d = 32 c + 8 grp; rows >= R are zero
  bf16x8 qh[DC], ql[DC];
  {
#pragma unroll
    for (int c = 0; c < DC; ++c) {
      float f[8];
      const float4 x0 = qraw[2 * c];
      const float4 x1 = qraw[2 * c + 1];
      const float sc = col < R ? a.scale : 0.f;
      f[0] = x0.x * sc; f[1] = x0.y * sc; f[2] = x0.z * sc; f[3] = x0.w * sc;
      f[4] = x1.x * sc; f[5] = x1.y * sc; f[6] = x1.z * sc; f[7] = x1.w * sc;
      split8(f, qh[c], ql[c]);
    }
  }
  __syncthreads();  // pg_s, nvis_s

  const size_t head_off = (size_t)kvh * a.PS * HD;
  const size_t page_sz = (size_t)a.KVH * a.PS * HD;
  float4 kA[2 * DC], vA[VL], kB[2 * DC], vB[VL];   // two tiles' K / V in flight (ping-pong)
  // K: this lane's key (16 per wave) x its 8-wide d slices; V: cooperative 16-B rows for LDS
#define FO_ATTN_LOAD(kreg, vreg, K0)                                                                      \
  {                                                                                                       \
    const int pk = min((K0) + 16 * wave + col, c1 - 1);                                                   \
    const float* kr = a.kc + (size_t)pg_s[pk / a.PS - pb] * page_sz + head_off + (size_t)(pk % a.PS) * HD \
                      + 8 * grp;                                                                          \
    _Pragma("unroll") for (int c = 0; c < DC; ++c) {                                                      \
      kreg[2 * c] = *reinterpret_cast<const float4*>(kr + 32 * c);                                        \
      kreg[2 * c + 1] = *reinterpret_cast<const float4*>(kr + 32 * c + 4);                                \
    }                                                                                                     \
    _Pragma("unroll") for (int i = 0; i < VL; ++i) {                                                      \
      const int e = tid + NTH * i, j = e / (HD / 4), d4 = e % (HD / 4);                                   \
      const int pv = min((K0) + j, c1 - 1);                                                               \
      vreg[i] = *reinterpret_cast<const float4*>(a.vc + (size_t)pg_s[pv / a.PS - pb] * page_sz + head_off \
                                                 + (size_t)(pv % a.PS) * HD + d4 * 4);                    \
    }                                                                                                     \
  }

  float m_run[4], l_lane[4];
  f32x4 acc[NTW];
#pragma unroll
  for (int i = 0; i < 4; ++i) { m_run[i] = -INFINITY; l_lane[i] = 0.f; }
#pragma unroll
  for (int n = 0; n < NTW; ++n) acc[n] = f32x4{0.f, 0.f, 0.f, 0.f};

  // tile t's loads are issued while tile t - 1 computes and two tiles are in flight from the start, so a
  // 256-key split waits for one round of memory, not two
  FO_ATTN_LOAD(kA, vA, c0)
  if (c0 + KT < c1) FO_ATTN_LOAD(kB, vB, c0 + KT)
  auto tile = [&](float4 (&kreg)[2 * DC], float4 (&vreg)[VL], const int k0) {
    __syncthreads();  // the previous tile's p_s / v_s readers are done
#pragma unroll
    for (int i = 0; i < VL; ++i) {
      const int e = tid + NTH * i, j = e / (HD / 4), d4 = e % (HD / 4);
      *reinterpret_cast<float2*>(&v_s[j][d4 * 4]) = make_float2(vreg[i].x, vreg[i].y);
      *reinterpret_cast<float2*>(&v_s[j][d4 * 4 + 2]) = make_float2(vreg[i].z, vreg[i].w);
    }
    bf16x8 kh[DC], kl[DC];
#pragma unroll
    for (int c = 0; c < DC; ++c) {
      const float f[8] = {kreg[2 * c].x, kreg[2 * c].y, kreg[2 * c].z, kreg[2 * c].w,
                          kreg[2 * c + 1].x, kreg[2 * c + 1].y, kreg[2 * c + 1].z, kreg[2 * c + 1].w};
      split8(f, kh[c], kl[c]);
    }
    if (k0 + 2 * KT < c1) FO_ATTN_LOAD(kreg, vreg, k0 + 2 * KT)
    // S[r = 4 grp + i][key = k0 + 16 wave + col]
    f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < DC; ++c) {
      s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qh[c], kh[c], s, 0, 0, 0);
      s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qh[c], kl[c], s, 0, 0, 0);
      s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ql[c], kh[c], s, 0, 0, 0);
    }
    const int key = k0 + 16 * wave + col;
    bool valid[4];
    float mw[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      valid[i] = key < c1 && key < nvis_s[4 * grp + i];
      mw[i] = row16_max(valid[i] ? s[i] : -INFINITY);
    }
    if (col == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) mx_s[wave][4 * grp + i] = mw[i];
    }
    __syncthreads();
    float alpha[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = 4 * grp + i;
      float tm = mx_s[0][r];
#pragma unroll
      for (int w = 1; w < NW; ++w) tm = fmaxf(tm, mx_s[w][r]);
      const float mn = fmaxf(m_run[i], tm);
      alpha[i] = (m_run[i] == mn) ? 1.f : expf(m_run[i] - mn);
      m_run[i] = mn;
      const float p = valid[i] ? expf(s[i] - mn) : 0.f;
      l_lane[i] = l_lane[i] * alpha[i] + p;
      p_s[r][16 * wave + col] = p;
    }
    __syncthreads();  // p_s and v_s complete
    // O[r][d] += P[r][:] V[:][d] for this wave's d tiles
#pragma unroll
    for (int n = 0; n < NTW; ++n) {
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[n][i] *= alpha[i];
    }
#pragma unroll
    for (int kc = 0; kc < KT / 32; ++kc) {
      bf16x8 ph, pl;
      {
        const float4 x0 = *reinterpret_cast<const float4*>(&p_s[col][32 * kc + 8 * grp]);
        const float4 x1 = *reinterpret_cast<const float4*>(&p_s[col][32 * kc + 8 * grp + 4]);
        const float f[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
        split8(f, ph, pl);
      }
#pragma unroll
      for (int n = 0; n < NTW; ++n) {
        const int dt = wave + NW * n;
        if (dt < NTILE) {
          float f[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) f[e] = v_s[32 * kc + 8 * grp + e][16 * dt + col];
          bf16x8 vh, vl;
          split8(f, vh, vl);
          acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ph, vh, acc[n], 0, 0, 0);
          acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ph, vl, acc[n], 0, 0, 0);
          acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pl, vh, acc[n], 0, 0, 0);
        }
      }
    }
  };
  for (int k0 = c0; k0 < c1; k0 += 2 * KT) {
    tile(kA, vA, k0);
    if (k0 + KT < c1) tile(kB, vB, k0 + KT);
  }
#undef FO_ATTN_LOAD
  // row sums: 16 lanes of the row group, then the 4 waves
  float lw[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) lw[i] = row16_sum(l_lane[i]);
  if (col == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) l_s[wave][4 * grp + i] = lw[i];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = 4 * grp + i;
    if (r >= R) continue;
    float l = l_s[0][r];
#pragma unroll
    for (int w = 1; w < NW; ++w) l += l_s[w][r];
    const size_t th = (size_t)(t0 + r / G) * a.H + kvh * G + r % G;
#pragma unroll
    for (int n = 0; n < NTW; ++n) {
      const int dt = wave + NW * n;
      if (dt >= NTILE) continue;
      const int d = 16 * dt + col;
      if (ns == 1) {
        a.out[th * HD + d] = acc[n][i] / l;
      } else {
        a.part_o[(th * a.nsplit + sp) * HD + d] = acc[n][i];
      }
    }
    if (ns > 1 && wave == 0 && col == 0) {
      a.part_ml[(th * a.nsplit + sp) * 2] = m_run[i];
      a.part_ml[(th * a.nsplit + sp) * 2 + 1] = l;
    }
  }
  if (a.cnt && ns > 1) attn_arrive_and_merge<HD>(a, it, kvh, ns, t0, R, G, nvis_s[0], &p_s[0][0]);
}

// Single-row decode attention (the AR speech decoder's step, models/decoder/decoder.py:341-349: one
// token per session, one query head per kv head): one work group per (session, head) reads the
// session's keys once, in fp32 -- scores one key per thread (16-B loads of the key row), block
// max / sum, then P.V with the waves on interleaved keys, a float4 of the row per lane.  No MFMA tile would be
// more than 1/16 full here, and no split / merge round trip is needed at <= 4096 keys.
constexpr int DEC_MAXK = MAXPG * 16;
constexpr int DEC_NW = 8, DEC_NT = DEC_NW * 64;  // 8 waves: a key per thread up to 512 keys
template <int HD>
__global__ __launch_bounds__(DEC_NT) void k_attn_decode(AttnArgs a) {
  static_assert(HD % 4 == 0 && HD <= 128, "decode attention: head_dim");
  __shared__ float s_s[DEC_MAXK];
  __shared__ float q_s[HD];
  __shared__ float acc_s[DEC_NW][HD];
  __shared__ float red_s[DEC_NW];
  __shared__ int pg_s[MAXPG];
  const int it = blockIdx.x, h = blockIdx.y;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  // items == NULL: the dense decode batch (item b = sequence b = token b), nothing to look up first
  const int seq = a.items ? a.items[3 * it] : it, t0 = a.items ? a.items[3 * it + 1] : it;
  // the visible-key count, the whole block-table row and q are requested together (none waits on
  // another); pages past the session's keys are staged but never dereferenced
  const int L = a.tok_nvis[t0];
  const int* bt = a.block_table + (size_t)seq * a.maxb;
  const int nb = a.maxb < MAXPG ? a.maxb : MAXPG;
  for (int i = tid; i < nb; i += DEC_NT) pg_s[i] = bt[i];
  const float* qr = a.q + ((size_t)t0 * a.H + h) * HD;
  for (int d = tid; d < HD; d += DEC_NT) q_s[d] = qr[d] * a.scale;
  float* orow = a.out + ((size_t)t0 * a.H + h) * HD;
  if (L > DEC_MAXK || (L + a.PS - 1) / a.PS > nb) {  // host contract broken: poison, never read wrong keys
    if (tid < HD) orow[tid] = NAN;
    return;
  }
  __syncthreads();
  const size_t page_sz = (size_t)a.KVH * a.PS * HD, head_off = (size_t)h * a.PS * HD;
  // P.V layout: HD/4 lanes per key (one float4 of the V row each), 64/(HD/4) keys per wave-instruction,
  // the waves on interleaved keys.  The first NPF rounds of V rows are loaded here, in flight together
  // with the K rows, so the P.V pass after the softmax waits on no memory for up to 256-512 keys.
  constexpr int LPK = HD / 4, KPW = 64 / LPK, VSTR = DEC_NW * KPW;
  constexpr int NPF = 512 / VSTR < 16 ? 512 / VSTR : 16;
  const int sub = lane / LPK, l4 = lane % LPK;
  float4 vpf[NPF];
#pragma unroll
  for (int i = 0; i < NPF; ++i) {
    const int j = wave * KPW + sub + i * VSTR;
    if (j < L)
      vpf[i] = *reinterpret_cast<const float4*>(a.vc + (size_t)pg_s[j / a.PS] * page_sz + head_off +
                                                (size_t)(j % a.PS) * HD + 4 * l4);
  }
  float mx = -INFINITY;
  for (int j = tid; j < L; j += DEC_NT) {
    const float* kr = a.kc + (size_t)pg_s[j / a.PS] * page_sz + head_off + (size_t)(j % a.PS) * HD;
    float s = 0.f;
#pragma unroll
    for (int d = 0; d < HD; d += 4) {
      const float4 k4 = *reinterpret_cast<const float4*>(kr + d);
      s += q_s[d] * k4.x + q_s[d + 1] * k4.y + q_s[d + 2] * k4.z + q_s[d + 3] * k4.w;
    }
    s_s[j] = s;
    mx = fmaxf(mx, s);
  }
  mx = wave_max(mx);
  if (lane == 0) red_s[wave] = mx;
  __syncthreads();
  mx = red_s[0];
#pragma unroll
  for (int w = 1; w < DEC_NW; ++w) mx = fmaxf(mx, red_s[w]);
  float sum = 0.f;
  for (int j = tid; j < L; j += DEC_NT) {
    const float p = expf(s_s[j] - mx);
    s_s[j] = p;
    sum += p;
  }
  sum = block_sum<DEC_NW>(sum, red_s);  // its barriers also publish s_s
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int i = 0; i < NPF; ++i) {
    const int j = wave * KPW + sub + i * VSTR;
    if (j < L) {
      const float p = s_s[j];
      acc.x += p * vpf[i].x;
      acc.y += p * vpf[i].y;
      acc.z += p * vpf[i].z;
      acc.w += p * vpf[i].w;
    }
  }
#pragma unroll 8
  for (int j = wave * KPW + sub + NPF * VSTR; j < L; j += VSTR) {
    const float p = s_s[j];
    const float4 v = *reinterpret_cast<const float4*>(a.vc + (size_t)pg_s[j / a.PS] * page_sz + head_off +
                                                      (size_t)(j % a.PS) * HD + 4 * l4);
    acc.x += p * v.x;
    acc.y += p * v.y;
    acc.z += p * v.z;
    acc.w += p * v.w;
  }
#pragma unroll
  for (int o = LPK; o < 64; o <<= 1) {
    acc.x += __shfl_xor(acc.x, o, 64);
    acc.y += __shfl_xor(acc.y, o, 64);
    acc.z += __shfl_xor(acc.z, o, 64);
    acc.w += __shfl_xor(acc.w, o, 64);
  }
  if (sub == 0) *reinterpret_cast<float4*>(&acc_s[wave][4 * l4]) = acc;
  __syncthreads();
  for (int d = tid; d < HD; d += DEC_NT) {
    float o = 0.f;
#pragma unroll
    for (int w = 0; w < DEC_NW; ++w) o += acc_s[w][d];
    orow[d] = o / sum;
  }
}

// merge split partials: grid (T, H)
__global__ void k_attn_combine(AttnArgs a, int hd) {
  const int t = blockIdx.x, h = blockIdx.y;
  const size_t base = ((size_t)t * a.H + h) * a.nsplit;
  float M = -INFINITY;
  for (int s = 0; s < a.nsplit; ++s)
    if (a.part_ml[(base + s) * 2 + 1] > 0.f) M = fmaxf(M, a.part_ml[(base + s) * 2]);
  float l = 0.f;
  for (int s = 0; s < a.nsplit; ++s) {
    const float ls = a.part_ml[(base + s) * 2 + 1];
    if (ls > 0.f) l += ls * expf(a.part_ml[(base + s) * 2] - M);
  }
  for (int dd = threadIdx.x; dd < hd; dd += blockDim.x) {
    float o = 0.f;
    for (int s = 0; s < a.nsplit; ++s) {
      const float ls = a.part_ml[(base + s) * 2 + 1];
      if (ls > 0.f) o += a.part_o[(base + s) * hd + dd] * expf(a.part_ml[(base + s) * 2] - M);
    }
    a.out[((size_t)t * a.H + h) * hd + dd] = o / l;
  }
}

// ------------------------------------------------------------------ encoder rel-pos attention
__global__ void k_enc_kv_write(const float* k, const float* v, int ldkv, int B, int T, int d, const int* start,
                               const int* len, const int* ring, int cap, float* kr, float* vr) {
  const long long total = (long long)B * T * d;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(e % d);
    const int i = (int)((e / d) % T);
    const int b = (int)(e / ((long long)T * d));
    const int slot = (start[b] + len[b] + i) % cap;
    const size_t rb = ring ? (size_t)ring[b] : (size_t)b;
    kr[(rb * cap + slot) * d + c] = k[((size_t)b * T + i) * ldkv + c];
    vr[(rb * cap + slot) * d + c] = v[((size_t)b * T + i) * ldkv + c];
  }
}

template <int TMAX, int LMAX>
__global__ __launch_bounds__(256) void k_relpos_attn(const float* q, int ldq, const float* kr, const float* vr,
                                                     int cap, const int* start, const int* len, const int* ring,
                                                     const float* ptab,
                                                     const int* pstart, const float* bu, const float* bv, int T,
                                                     int h, int dk, float scale, float* out, int ldo) {
  extern __shared__ float smem[];
  float* qu = smem;                     // [T][dk]
  float* qv = qu + TMAX * dk;           // [T][dk]
  float* sc = qv + TMAX * dk;           // [T][LMAX]
  const int b = blockIdx.x, hh = blockIdx.y;
  const int d = h * dk;
  const size_t rb = ring ? (size_t)ring[b] : (size_t)b;
  const int Lk = len[b] + T;
  const int st = start[b];
  const int ps = pstart[b];
  for (int e = threadIdx.x; e < T * dk; e += blockDim.x) {
    const int i = e / dk, c = e % dk;
    const float x = q[((size_t)b * T + i) * ldq + hh * dk + c];
    qu[i * dk + c] = x + bu[hh * dk + c];
    qv[i * dk + c] = x + bv[hh * dk + c];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < T * Lk; e += blockDim.x) {
    const int i = e / Lk, j = e % Lk;
    const int slot = (st + j) % cap;
    const float* kk = kr + (rb * cap + slot) * d + hh * dk;
    const float* pp = ptab + (size_t)(ps + j) * d + hh * dk;
    float s1 = 0.f, s2 = 0.f;
    for (int c = 0; c < dk; ++c) {
      s1 += qu[i * dk + c] * kk[c];
      s2 += qv[i * dk + c] * pp[c];
    }
    sc[i * LMAX + j] = (s1 + s2) * scale;
  }
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int i = wave; i < T; i += blockDim.x / 64) {
    float m = -INFINITY;
    for (int j = lane; j < Lk; j += 64) m = fmaxf(m, sc[i * LMAX + j]);
    m = wave_max(m);
    float s = 0.f;
    for (int j = lane; j < Lk; j += 64) {
      const float e = expf(sc[i * LMAX + j] - m);
      sc[i * LMAX + j] = e;
      s += e;
    }
    s = wave_sum(s);
    const float r = 1.f / s;
    for (int j = lane; j < Lk; j += 64) sc[i * LMAX + j] *= r;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < T * dk; e += blockDim.x) {
    const int i = e / dk, c = e % dk;
    float acc = 0.f;
    for (int j = 0; j < Lk; ++j) {
      const int slot = (st + j) % cap;
      acc += sc[i * LMAX + j] * vr[(rb * cap + slot) * d + hh * dk + c];
    }
    out[((size_t)b * T + i) * ldo + hh * dk + c] = acc;
  }
}

// Fused ring append + rel-pos attention for one (user, head): the chunk's new K/V rows come straight
// from the QKV GEMM output and are written into the user's ring (MultiHeadedAttention.infer's
// cat-and-trim, models/encoder/attention.py:415-428) while every key/value/position row this head
// needs is staged in LDS with 16-B coalesced loads; scores, softmax and P.V then run out of LDS.
__global__ __launch_bounds__(256) void k_relpos_fused(const float* qkv, int ldq, float* kr, float* vr, int cap,
                                                      const int* start, const int* len, const int* ring,
                                                      const float* ptab, const int* pstart, const float* bu,
                                                      const float* bv, int T, int h, int dk, float scale, float* out,
                                                      int ldo) {
  extern __shared__ float smem[];
  const int KP = dk + 4;  // padded rows: lanes on consecutive keys hit distinct banks
  float* k_s = smem;                  // [cap][KP]
  float* v_s = k_s + cap * KP;        // [cap][KP]
  float* p_s = v_s + cap * KP;        // [cap][KP]
  float* qu = p_s + cap * KP;         // [T][dk]
  float* qv = qu + T * dk;            // [T][dk]
  float* sc = qv + T * dk;            // [T][cap]
  const int b = blockIdx.x, hh = blockIdx.y;
  const int d = h * dk;
  const size_t rb = ring ? (size_t)ring[b] : (size_t)b;
  const int Lold = len[b], Lk = Lold + T;
  const int st = start[b];
  const int ps = pstart[b];
  const int D4 = dk / 4;
  for (int e = threadIdx.x; e < Lk * D4; e += blockDim.x) {
    const int j = e / D4, c = (e % D4) * 4;
    const size_t ro = (rb * cap + (st + j) % cap) * d + hh * dk + c;
    float4 kk, vv;
    if (j < Lold) {
      kk = *reinterpret_cast<const float4*>(kr + ro);
      vv = *reinterpret_cast<const float4*>(vr + ro);
    } else {
      const float* src = qkv + ((size_t)b * T + (j - Lold)) * ldq + hh * dk + c;
      kk = *reinterpret_cast<const float4*>(src + d);
      vv = *reinterpret_cast<const float4*>(src + 2 * d);
      *reinterpret_cast<float4*>(kr + ro) = kk;
      *reinterpret_cast<float4*>(vr + ro) = vv;
    }
    *reinterpret_cast<float4*>(k_s + j * KP + c) = kk;
    *reinterpret_cast<float4*>(v_s + j * KP + c) = vv;
    *reinterpret_cast<float4*>(p_s + j * KP + c) =
        *reinterpret_cast<const float4*>(ptab + (size_t)(ps + j) * d + hh * dk + c);
  }
  for (int e = threadIdx.x; e < T * dk; e += blockDim.x) {
    const int i = e / dk, c = e % dk;
    const float x = qkv[((size_t)b * T + i) * ldq + hh * dk + c];
    qu[i * dk + c] = x + bu[hh * dk + c];
    qv[i * dk + c] = x + bv[hh * dk + c];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < T * Lk; e += blockDim.x) {
    const int i = e / Lk, j = e % Lk;
    const float* kk = k_s + j * KP;
    const float* pp = p_s + j * KP;
    const float* a1 = qu + i * dk;
    const float* a2 = qv + i * dk;
    float s1 = 0.f, s2 = 0.f;
    for (int c = 0; c < dk; c += 4) {
      const float4 k4 = *reinterpret_cast<const float4*>(kk + c), p4 = *reinterpret_cast<const float4*>(pp + c);
      const float4 u4 = *reinterpret_cast<const float4*>(a1 + c), w4 = *reinterpret_cast<const float4*>(a2 + c);
      s1 += u4.x * k4.x + u4.y * k4.y + u4.z * k4.z + u4.w * k4.w;
      s2 += w4.x * p4.x + w4.y * p4.y + w4.z * p4.z + w4.w * p4.w;
    }
    sc[i * cap + j] = (s1 + s2) * scale;
  }
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int i = wave; i < T; i += blockDim.x / 64) {
    float m = -INFINITY;
    for (int j = lane; j < Lk; j += 64) m = fmaxf(m, sc[i * cap + j]);
    m = wave_max(m);
    float sum = 0.f;
    for (int j = lane; j < Lk; j += 64) {
      const float e = expf(sc[i * cap + j] - m);
      sc[i * cap + j] = e;
      sum += e;
    }
    sum = wave_sum(sum);
    const float r = 1.f / sum;
    for (int j = lane; j < Lk; j += 64) sc[i * cap + j] *= r;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < T * dk; e += blockDim.x) {
    const int i = e / dk, c = e % dk;
    const float* pr = sc + i * cap;
    float acc = 0.f;
    for (int j = 0; j < Lk; ++j) acc += pr[j] * v_s[j * KP + c];
    out[((size_t)b * T + i) * ldo + hh * dk + c] = acc;
  }
}

// waves per work group of the multi-row MFMA attention at head_dim 128 (the Qwen2 listen / text rows): 8 (default:
// 128-key tiles, so a 128-key split loads in one round instead of two) or 4 (64-key tiles); FO_ATTN_NW.  r03t
// (scripts/attn_kps_sweep.py, 8 sessions, graph-replayed): 2 tokens x 200 keys 18.0 -> 15.2 us, 400 keys 21.2 ->
// 17.7 us, 1 token x 200 keys 15.9 -> 13.8 us (profiles/r03t_attn_nw_ab.txt)
int g_attn_nw = -1;
inline int attn_waves() {
  if (g_attn_nw < 0) {
    const char* e = getenv("FO_ATTN_NW");
    g_attn_nw = (e && atoi(e) == 4) ? 4 : 8;   // (16 waves: 128 VGPRs a lane, 109 spilled -- not built)
  }
  return g_attn_nw;
}

inline int grid_for(long long n) {
  long long g = (n + 255) / 256;
  return (int)(g > 8192 ? 8192 : (g < 1 ? 1 : g));
}

}  // namespace

extern "C" {

int fo_attn_nsplit(int max_keys, int n_items, int KVH) {
  // enough work groups to cover the chip (~2 per CU) while every split keeps >= one 64-key tile
  const int by_keys = (max_keys + KT - 1) / KT;
  const int wgs = n_items * KVH;
  int ns = (512 + wgs - 1) / wgs;
  if (ns > by_keys) ns = by_keys;
  if (ns > 32) ns = 32;
  const int need = (max_keys + MAXPG * 16 - 1) / (MAXPG * 16);  // every split within the LDS page table
  if (ns < need) ns = need;
  return ns < 1 ? 1 : ns;
}

int fo_rope_kv_write(const float* qkv, int ldq, int T, int H, int KVH, int hd, const int* pos, const int* slot,
                     const float* cos_t, const float* sin_t, float* q_out, float* kc, float* vc, int PS,
                     hipStream_t s) {
  FO_REQUIRE(T > 0 && (hd % 2) == 0, "fo_rope_kv_write: bad shape");
  hipLaunchKernelGGL(k_rope_kv_write, dim3(T), dim3(256), 0, s, qkv, ldq, T, H, KVH, hd, pos, slot, cos_t, sin_t,
                     q_out, kc, vc, PS);
  return fo::check_launch("fo_rope_kv_write");
}

// q [T][H*hd] -> out [T][H*hd].  items [n_items][3] (sequence, first token, tokens), or NULL for a uniform batch
// (item b = sequence b = tokens b*T/n_items .. (b+1)*T/n_items - 1), with
// tokens * (H/KVH) <= max_rows <= 64; part_ml >= T*H*nsplit*2 and part_o >= T*H*nsplit*hd floats
// when nsplit > 1.  tickets (nullable): n_items*KVH zero-initialised ints; then each item takes
// min(nsplit, ceil(keys / keys_per_split)) splits and the last one merges them in this launch (the
// tickets are left zeroed); without tickets nsplit static splits are merged by a second launch.
int fo_attention(const float* q, int T, const int* items, int n_items, int max_rows, const int* tok_nvis,
                 const int* block_table, int maxb, int PS, const float* kc, const float* vc, int H, int KVH, int hd,
                 float scale, int nsplit, float* part_ml, float* part_o, float* out, int* tickets,
                 int keys_per_split, hipStream_t s) {
  FO_REQUIRE(T > 0 && n_items > 0 && KVH > 0 && H % KVH == 0, "fo_attention: bad shape");
  FO_REQUIRE(items || T % n_items == 0, "fo_attention: items NULL needs T / n_items tokens per item");
  FO_REQUIRE(hd == 32 || hd == 64 || hd == 128, "fo_attention: head_dim %d unsupported", hd);
  FO_REQUIRE(max_rows >= 1 && max_rows <= 16, "fo_attention: %d query rows per item (max 16)", max_rows);
  FO_REQUIRE(nsplit >= 1 && (nsplit == 1 || (part_ml && part_o)), "fo_attention: bad split buffers");
  FO_REQUIRE(!tickets || keys_per_split >= KT, "fo_attention: keys_per_split %d < %d", keys_per_split, KT);
  AttnArgs a{q, items, tok_nvis, block_table, kc, vc, part_ml, part_o, out, H, KVH, PS, maxb, nsplit, scale,
             tickets, keys_per_split, items ? 1 : T / n_items};
  if (max_rows == 1 && (long long)maxb * PS <= DEC_MAXK) {  // one query row per (session, head): decode kernel
    dim3 g1(n_items, H);
    if (hd == 128) hipLaunchKernelGGL((k_attn_decode<128>), g1, dim3(DEC_NT), 0, s, a);
    else if (hd == 64) hipLaunchKernelGGL((k_attn_decode<64>), g1, dim3(DEC_NT), 0, s, a);
    else hipLaunchKernelGGL((k_attn_decode<32>), g1, dim3(DEC_NT), 0, s, a);
    return fo::check_launch("fo_attention/decode");
  }
  dim3 grid(n_items, KVH, nsplit);
  if (hd == 128 && attn_waves() == 8) hipLaunchKernelGGL((k_attn_mfma<128, 8>), grid, dim3(512), 0, s, a);
  else if (hd == 128) hipLaunchKernelGGL((k_attn_mfma<128>), grid, dim3(256), 0, s, a);
  else if (hd == 64) hipLaunchKernelGGL((k_attn_mfma<64>), grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL((k_attn_mfma<32>), grid, dim3(256), 0, s, a);
  int rc = fo::check_launch("fo_attention/rows");
  if (rc || nsplit == 1 || tickets) return rc;
  hipLaunchKernelGGL(k_attn_combine, dim3(T, H), dim3(hd < 64 ? 64 : hd), 0, s, a, hd);
  return fo::check_launch("fo_attention/combine");
}

int fo_enc_kv_write(const float* k, const float* v, int ldkv, int B, int T, int d, const int* start, const int* len,
                    const int* ring, int cap, float* kr, float* vr, hipStream_t s) {
  const long long n = (long long)B * T * d;
  hipLaunchKernelGGL(k_enc_kv_write, dim3(grid_for(n)), dim3(256), 0, s, k, v, ldkv, B, T, d, start, len, ring, cap,
                     kr, vr);
  return fo::check_launch("fo_enc_kv_write");
}

int fo_relpos_attention_fused(const float* qkv, int ldq, float* kr, float* vr, int cap, const int* start,
                              const int* len, const int* ring, const float* ptab, const int* pstart, const float* bu,
                              const float* bv, int B, int T, int h, int dk, float scale, float* out, int ldo,
                              hipStream_t s) {
  FO_REQUIRE(T >= 1 && T <= cap && dk % 4 == 0 && (ldq % 4) == 0, "fo_relpos_attention_fused: T=%d dk=%d", T, dk);
  const size_t lds = (size_t)(3 * cap * (dk + 4) + 2 * T * dk + T * cap) * sizeof(float);
  FO_REQUIRE(lds <= 160 * 1024, "fo_relpos_attention_fused: ring of %d x %d exceeds LDS", cap, dk);
  hipLaunchKernelGGL(k_relpos_fused, dim3(B, h), dim3(256), lds, s, qkv, ldq, kr, vr, cap, start, len, ring, ptab,
                     pstart, bu, bv, T, h, dk, scale, out, ldo);
  return fo::check_launch("fo_relpos_attention_fused");
}

int fo_relpos_attention(const float* q, int ldq, const float* kr, const float* vr, int cap, const int* start,
                        const int* len, const int* ring, const float* ptab, const int* pstart, const float* bu,
                        const float* bv, int B, int T, int h, int dk, float scale, float* out, int ldo,
                        hipStream_t s) {
  FO_REQUIRE(T <= 8 && cap + T <= 264, "fo_relpos_attention: T=%d cap=%d too large", T, cap);
  const size_t lds = (size_t)(2 * 8 * dk + 8 * 264) * sizeof(float);
  FO_REQUIRE(lds <= 65536, "fo_relpos_attention: dk too large");
  hipLaunchKernelGGL((k_relpos_attn<8, 264>), dim3(B, h), dim3(256), lds, s, q, ldq, kr, vr, cap, start, len, ring,
                     ptab, pstart, bu, bv, T, h, dk, scale, out, ldo);
  return fo::check_launch("fo_relpos_attention");
}

}  // extern "C"
