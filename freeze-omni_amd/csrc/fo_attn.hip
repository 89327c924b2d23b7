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
//    head) so its keys are read once per kv head; split-KV over key ranges when the grid would
//    otherwise not cover the chip, merged by a combine kernel.
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
};

constexpr int KT = 64;      // keys per LDS tile (one key per lane in the score phase)
constexpr int MAXPG = 256;  // pages of one split staged in LDS (fo_attn_nsplit keeps splits <= 4096 keys)

// One work item = up to RMAX query rows (tokens x GQA group) of ONE sequence against one kv head,
// over split `sp` of that sequence's keys.  K/V tiles of 64 keys are loaded with 16-B coalesced
// loads into registers one tile ahead (the next tile's loads are in flight while the current tile
// is computed), staged through LDS, and consumed by all rows: a sequence's keys cross HBM once per
// kv head no matter how many of its tokens are in the batch.  Online softmax per row (a row's
// 64 scores of a tile are one wave's 64 lanes); fp32 throughout.
template <int HD, int RMAX>
__global__ __launch_bounds__(256) void k_attn_rows(AttnArgs a) {
  constexpr int KP = HD + 4;          // padded K row: lanes j read k_s[j][d..d+3] conflict-free
  constexpr int D4 = HD / 4;
  constexpr int LPT = KT * D4 / 256;  // float4 per thread per tile (K and V each)
  constexpr int RG = 256 / HD;        // row groups in the PV phase (thread owns column tid % HD)
  constexpr int NACC = RMAX / RG;
  constexpr int RPW = RMAX / 4;       // rows per wave in the score phase
  __shared__ float q_s[RMAX][HD];
  __shared__ float k_s[KT][KP];
  __shared__ float v_s[KT][HD];
  __shared__ float p_s[RMAX][KT + 4];
  __shared__ float alpha_s[RMAX];
  __shared__ float ml_s[RMAX][2];
  __shared__ int nvis_s[RMAX];
  __shared__ int pg_s[MAXPG];

  const int it = blockIdx.x, kvh = blockIdx.y, sp = blockIdx.z;
  const int seq = a.items[3 * it], t0 = a.items[3 * it + 1], tn = a.items[3 * it + 2];
  const int G = a.H / a.KVH;
  const int R = tn * G;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  int Lmax = 0;
  for (int i = 0; i < tn; ++i) Lmax = max(Lmax, a.tok_nvis[t0 + i]);
  const int per = ((Lmax + a.nsplit - 1) / a.nsplit + KT - 1) / KT * KT;
  const int c0 = sp * per, c1 = min(Lmax, c0 + per);
  if (c0 >= c1) {  // empty split: neutral partial
    for (int r = tid; r < R; r += 256) {
      const size_t o = ((size_t)(t0 + r / G) * a.H + kvh * G + r % G) * a.nsplit + sp;
      a.part_ml[o * 2] = -INFINITY;
      a.part_ml[o * 2 + 1] = 0.f;
    }
    return;
  }
  for (int e = tid; e < RMAX * D4; e += 256) {  // rows >= R duplicate row R-1 (never output)
    const int r = e / D4, d4 = e % D4, rr = min(r, R - 1);
    float4 v = *reinterpret_cast<const float4*>(a.q + ((size_t)(t0 + rr / G) * a.H + kvh * G + rr % G) * HD + d4 * 4);
    v.x *= a.scale; v.y *= a.scale; v.z *= a.scale; v.w *= a.scale;
    *reinterpret_cast<float4*>(&q_s[r][d4 * 4]) = v;
  }
  if (tid < RMAX) nvis_s[tid] = tid < R ? a.tok_nvis[t0 + tid / G] : 0;

  // the split's block-table slice goes to LDS once, so tile loads never wait on a dependent global load
  const int* bt = a.block_table + (size_t)seq * a.maxb;
  const int pb = c0 / a.PS, npg = (c1 - 1) / a.PS - pb + 1;
  if (npg > MAXPG) {  // host contract broken (split wider than 4096 keys): poison rather than read wrong keys
    for (int r = tid; r < R; r += 256) a.out[((size_t)(t0 + r / G) * a.H + kvh * G + r % G) * HD] = NAN;
    return;
  }
  for (int i = tid; i < npg; i += 256) pg_s[i] = bt[pb + i];
  __syncthreads();
  const size_t head_off = (size_t)kvh * a.PS * HD;
  const size_t page_sz = (size_t)a.KVH * a.PS * HD;
  float4 kreg[LPT], vreg[LPT];
  // K/V tile [k0, k0 + 64) into registers.  A macro, not a lambda (a captured array would live in
  // scratch).  Full tiles load branch-free (a per-element "load or zero" makes hipcc wait vmcnt(0)
  // per load); only the split's last, partial tile takes the guarded path.
#define FO_ATTN_LOAD_TILE(K0)                                                                              \
  if ((K0) + KT <= c1) {                                                                                   \
    _Pragma("unroll") for (int i = 0; i < LPT; ++i) {                                                      \
      const int e = tid + 256 * i, j = e / D4, d4 = e % D4, p = (K0) + j;                                  \
      const size_t off = (size_t)pg_s[p / a.PS - pb] * page_sz + head_off + (size_t)(p % a.PS) * HD + d4 * 4; \
      kreg[i] = *reinterpret_cast<const float4*>(a.kc + off);                                              \
      vreg[i] = *reinterpret_cast<const float4*>(a.vc + off);                                              \
    }                                                                                                      \
  } else {                                                                                                 \
    _Pragma("unroll") for (int i = 0; i < LPT; ++i) {                                                      \
      const int e = tid + 256 * i, j = e / D4, d4 = e % D4, p = (K0) + j;                                  \
      if (p < c1) {                                                                                        \
        const size_t off = (size_t)pg_s[p / a.PS - pb] * page_sz + head_off + (size_t)(p % a.PS) * HD + d4 * 4; \
        kreg[i] = *reinterpret_cast<const float4*>(a.kc + off);                                            \
        vreg[i] = *reinterpret_cast<const float4*>(a.vc + off);                                            \
      } else {                                                                                             \
        kreg[i] = make_float4(0.f, 0.f, 0.f, 0.f);                                                         \
        vreg[i] = kreg[i];                                                                                 \
      }                                                                                                    \
    }                                                                                                      \
  }
  float m_run[RPW], l_run[RPW], acc[NACC];
#pragma unroll
  for (int i = 0; i < RPW; ++i) { m_run[i] = -INFINITY; l_run[i] = 0.f; }
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = 0.f;
  const int d = tid % HD, rg = tid / HD;

  FO_ATTN_LOAD_TILE(c0)
  for (int k0 = c0; k0 < c1; k0 += KT) {
    __syncthreads();  // readers of the previous tile are done (first pass: q_s / nvis_s visible)
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int e = tid + 256 * i, j = e / D4, d4 = e % D4;
      *reinterpret_cast<float4*>(&k_s[j][d4 * 4]) = kreg[i];
      *reinterpret_cast<float4*>(&v_s[j][d4 * 4]) = vreg[i];
    }
    if (k0 + KT < c1) {
      FO_ATTN_LOAD_TILE(k0 + KT)
    }
    __syncthreads();
    const int nk = min(KT, c1 - k0);
    // scores: wave w owns rows w, w+4, ...; lane = key.  Rows go in blocks of 4 with a wave-uniform
    // guard, and the inner loops are branch-free so LDS reads batch instead of serialising.
    float sc[RPW];
#pragma unroll
    for (int ib = 0; ib < RPW; ib += 4) {
#pragma unroll
      for (int u = 0; u < 4; ++u) sc[ib + u] = 0.f;
      if (wave + 4 * ib < R) {
#pragma unroll 4
        for (int d4 = 0; d4 < D4; ++d4) {
          const float4 kk = *reinterpret_cast<const float4*>(&k_s[lane][d4 * 4]);
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const float4 qq = *reinterpret_cast<const float4*>(&q_s[wave + 4 * (ib + u)][d4 * 4]);
            sc[ib + u] += qq.x * kk.x + qq.y * kk.y + qq.z * kk.z + qq.w * kk.w;
          }
        }
      }
    }
    // online softmax per row (a row's 64 scores are this wave's 64 lanes)
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      const int r = wave + 4 * i;
      if (r < R) {
        const bool valid = lane < nk && k0 + lane < nvis_s[r];
        const float x = valid ? sc[i] : -INFINITY;
        const float mo = m_run[i];
        const float mn = fmaxf(mo, wave_max(x));
        const float p = valid ? expf(x - mn) : 0.f;
        const float al = (mo == mn) ? 1.f : expf(mo - mn);
        l_run[i] = l_run[i] * al + p;  // per-lane partial; reduced once after the last tile
        m_run[i] = mn;
        p_s[r][lane] = p;
        if (lane == 0) alpha_s[r] = al;
      }
    }
    __syncthreads();
    // PV: thread owns column d for rows rg, rg+RG, ...; keys in steps of 4 (p_s rows are 16-B aligned;
    // keys past nk have p = 0 and zero V)
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] *= alpha_s[min(rg + RG * i, RMAX - 1)];
    for (int j = 0; j < nk; j += 4) {
      const float v0 = v_s[j][d], v1 = v_s[j + 1][d], v2 = v_s[j + 2][d], v3 = v_s[j + 3][d];
#pragma unroll
      for (int ib = 0; ib < NACC; ib += 4) {
        if (rg + RG * ib < R) {
#pragma unroll
          for (int u = 0; u < 4 && ib + u < NACC; ++u) {
            const float4 pp = *reinterpret_cast<const float4*>(&p_s[rg + RG * (ib + u)][j]);
            acc[ib + u] += pp.x * v0 + pp.y * v1 + pp.z * v2 + pp.w * v3;
          }
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < RPW; ++i) {
    const int r = wave + 4 * i;
    if (r < R) {
      const float l = wave_sum(l_run[i]);
      if (lane == 0) {
        ml_s[r][0] = m_run[i];
        ml_s[r][1] = l;
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < NACC; ++i) {
    const int r = rg + RG * i;
    if (r < R) {
      const size_t th = (size_t)(t0 + r / G) * a.H + kvh * G + r % G;
      if (a.nsplit == 1) {
        a.out[th * HD + d] = acc[i] / ml_s[r][1];
      } else {
        a.part_o[(th * a.nsplit + sp) * HD + d] = acc[i];
        if (d == 0) {
          a.part_ml[(th * a.nsplit + sp) * 2] = ml_s[r][0];
          a.part_ml[(th * a.nsplit + sp) * 2 + 1] = ml_s[r][1];
        }
      }
    }
  }
}

#undef FO_ATTN_LOAD_TILE

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

// q [T][H*hd] -> out [T][H*hd].  items [n_items][3] (sequence, first token, tokens) with
// tokens * (H/KVH) <= max_rows <= 64; part_ml >= T*H*nsplit*2 and part_o >= T*H*nsplit*hd floats
// when nsplit > 1.
int fo_attention(const float* q, int T, const int* items, int n_items, int max_rows, const int* tok_nvis,
                 const int* block_table, int maxb, int PS, const float* kc, const float* vc, int H, int KVH, int hd,
                 float scale, int nsplit, float* part_ml, float* part_o, float* out, hipStream_t s) {
  FO_REQUIRE(T > 0 && n_items > 0 && KVH > 0 && H % KVH == 0, "fo_attention: bad shape");
  FO_REQUIRE(hd == 32 || hd == 64 || hd == 128, "fo_attention: head_dim %d unsupported", hd);
  FO_REQUIRE(max_rows >= 1 && max_rows <= 64, "fo_attention: %d query rows per item (max 64)", max_rows);
  FO_REQUIRE(nsplit >= 1 && (nsplit == 1 || (part_ml && part_o)), "fo_attention: bad split buffers");
  AttnArgs a{q, items, tok_nvis, block_table, kc, vc, part_ml, part_o, out, H, KVH, PS, maxb, nsplit, scale};
  dim3 grid(n_items, KVH, nsplit);
  const bool small = max_rows <= 16;
  if (hd == 128) {
    if (small) hipLaunchKernelGGL((k_attn_rows<128, 16>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((k_attn_rows<128, 64>), grid, dim3(256), 0, s, a);
  } else if (hd == 64) {
    if (small) hipLaunchKernelGGL((k_attn_rows<64, 16>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((k_attn_rows<64, 64>), grid, dim3(256), 0, s, a);
  } else {
    if (small) hipLaunchKernelGGL((k_attn_rows<32, 16>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((k_attn_rows<32, 64>), grid, dim3(256), 0, s, a);
  }
  int rc = fo::check_launch("fo_attention/rows");
  if (rc || nsplit == 1) return rc;
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
