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
//    Split-KV: grid (token, kv_head, split) computes partial softmax statistics per chunk of CH
//    keys for the G query heads sharing that kv head; a combine kernel merges them.
// 2. Encoder rel-pos attention over a per-user ring buffer (models/encoder/attention.py:407-459):
//    scores = ((q+u).K^T + (q+v).P^T)/sqrt(dk), no mask, no rel_shift; P rows come from a
//    table of linear_pos(sinusoid(position)) precomputed at load for every position.
#include "fo_common.h"

namespace {

constexpr int CH = 256;  // keys per split

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
  const float* q;
  const int* tok_seq;
  const int* tok_nvis;  // keys visible to each query token (causal: own cache index + 1; full: all)
  const int* block_table;
  const float* kc;
  const float* vc;
  float* part_ml;  // [T][H][nsplit][2]
  float* part_o;   // [T][H][nsplit][hd]
  float* out;      // [T][H*hd]
  int H, KVH, hd, PS, maxb, nsplit;
  float scale;
};

__device__ __forceinline__ int visible_keys(const AttnArgs& a, int t) { return a.tok_nvis[t]; }

template <int HD, int GMAX>
__global__ __launch_bounds__(256) void k_attn_split(AttnArgs a) {
  constexpr int LPK = HD / 8;         // lanes per key (8 dims per lane)
  constexpr int KPW = 64 / LPK;       // keys per wave per iteration
  constexpr int PARTS = 256 / HD;     // key partitions in the PV phase
  __shared__ float q_s[GMAX][HD];
  __shared__ float sc[GMAX][CH];
  __shared__ float ml_s[GMAX][2];
  __shared__ float o_s[PARTS][GMAX][HD];
  const int t = blockIdx.x, kvh = blockIdx.y, sp = blockIdx.z;
  const int G = a.H / a.KVH;
  const int L = visible_keys(a, t);
  const int c0 = sp * CH;
  const int n = min(CH, L - c0);
  const size_t pidx = ((size_t)t * a.H + (size_t)kvh * G) * a.nsplit + sp;
  if (n <= 0) return;  // combine reads only splits < ceil(L / CH)
  const int seq = a.tok_seq[t];
  const int* bt = a.block_table + (size_t)seq * a.maxb;
  for (int e = threadIdx.x; e < G * HD; e += 256) {
    const int g = e / HD, d = e % HD;
    q_s[g][d] = a.q[(size_t)t * a.H * HD + (size_t)(kvh * G + g) * HD + d];
  }
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int kl = lane / LPK, d0 = (lane % LPK) * 8;
  for (int base = wave * KPW; base < n; base += 4 * KPW) {
    const int j = base + kl;
    float part[GMAX];
#pragma unroll
    for (int g = 0; g < GMAX; ++g) part[g] = 0.f;
    if (j < n) {
      const int p = c0 + j;
      const float* kr = a.kc + (((size_t)bt[p / a.PS] * a.KVH + kvh) * a.PS + (p % a.PS)) * HD + d0;
      const float4 k0 = reinterpret_cast<const float4*>(kr)[0];
      const float4 k1 = reinterpret_cast<const float4*>(kr)[1];
      const float kv[8] = {k0.x, k0.y, k0.z, k0.w, k1.x, k1.y, k1.z, k1.w};
#pragma unroll
      for (int g = 0; g < GMAX; ++g)
        if (g < G) {
#pragma unroll
          for (int i = 0; i < 8; ++i) part[g] += q_s[g][d0 + i] * kv[i];
        }
    }
#pragma unroll
    for (int g = 0; g < GMAX; ++g) {
      float v = part[g];
#pragma unroll
      for (int o = LPK / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
      if (g < G && j < n && (lane % LPK) == 0) sc[g][j] = v * a.scale;
    }
  }
  __syncthreads();
  // per-head max / exp / sum over the chunk
  for (int g = wave; g < G; g += 4) {
    float m = -INFINITY;
    for (int j = lane; j < n; j += 64) m = fmaxf(m, sc[g][j]);
    m = wave_max(m);
    float s = 0.f;
    for (int j = lane; j < n; j += 64) {
      const float e = expf(sc[g][j] - m);
      sc[g][j] = e;
      s += e;
    }
    s = wave_sum(s);
    if (lane == 0) {
      ml_s[g][0] = m;
      ml_s[g][1] = s;
    }
  }
  __syncthreads();
  // PV
  {
    const int d = threadIdx.x % HD, part = threadIdx.x / HD;
    float acc[GMAX];
#pragma unroll
    for (int g = 0; g < GMAX; ++g) acc[g] = 0.f;
    for (int j = part; j < n; j += PARTS) {
      const int p = c0 + j;
      const float v = a.vc[(((size_t)bt[p / a.PS] * a.KVH + kvh) * a.PS + (p % a.PS)) * HD + d];
#pragma unroll
      for (int g = 0; g < GMAX; ++g)
        if (g < G) acc[g] += sc[g][j] * v;
    }
#pragma unroll
    for (int g = 0; g < GMAX; ++g)
      if (g < G) o_s[part][g][d] = acc[g];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < G * HD; e += 256) {
    const int g = e / HD, d = e % HD;
    float v = 0.f;
#pragma unroll
    for (int p = 0; p < PARTS; ++p) v += o_s[p][g][d];
    a.part_o[(pidx + (size_t)g * a.nsplit) * HD + d] = v;
  }
  if (threadIdx.x < G) {
    a.part_ml[(pidx + (size_t)threadIdx.x * a.nsplit) * 2 + 0] = ml_s[threadIdx.x][0];
    a.part_ml[(pidx + (size_t)threadIdx.x * a.nsplit) * 2 + 1] = ml_s[threadIdx.x][1];
  }
}

__global__ void k_attn_combine(AttnArgs a) {
  const int t = blockIdx.x, h = blockIdx.y;
  const int L = visible_keys(a, t);
  const int ns = (L + CH - 1) / CH;
  const size_t base = ((size_t)t * a.H + h) * a.nsplit;
  float M = -INFINITY;
  for (int s = 0; s < ns; ++s) M = fmaxf(M, a.part_ml[(base + s) * 2]);
  float l = 0.f;
  for (int s = 0; s < ns; ++s) l += a.part_ml[(base + s) * 2 + 1] * expf(a.part_ml[(base + s) * 2] - M);
  for (int d = threadIdx.x; d < a.hd; d += blockDim.x) {
    float o = 0.f;
    for (int s = 0; s < ns; ++s) o += a.part_o[(base + s) * a.hd + d] * expf(a.part_ml[(base + s) * 2] - M);
    a.out[(size_t)t * a.H * a.hd + (size_t)h * a.hd + d] = o / l;
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

int fo_attn_nsplit(int max_keys) { return (max_keys + CH - 1) / CH; }

int fo_rope_kv_write(const float* qkv, int ldq, int T, int H, int KVH, int hd, const int* pos, const int* slot,
                     const float* cos_t, const float* sin_t, float* q_out, float* kc, float* vc, int PS,
                     hipStream_t s) {
  FO_REQUIRE(T > 0 && (hd % 2) == 0, "fo_rope_kv_write: bad shape");
  hipLaunchKernelGGL(k_rope_kv_write, dim3(T), dim3(256), 0, s, qkv, ldq, T, H, KVH, hd, pos, slot, cos_t, sin_t,
                     q_out, kc, vc, PS);
  return fo::check_launch("fo_rope_kv_write");
}

// q [T][H*hd] -> out [T][H*hd]; part_ml >= T*H*nsplit*2 floats, part_o >= T*H*nsplit*hd floats.
int fo_attention(const float* q, int T, const int* tok_seq, const int* tok_nvis, const int* block_table, int maxb,
                 int PS, const float* kc, const float* vc, int H, int KVH, int hd, float scale, int nsplit,
                 float* part_ml, float* part_o, float* out, hipStream_t s) {
  FO_REQUIRE(T > 0 && H % KVH == 0, "fo_attention: bad heads");
  FO_REQUIRE(H / KVH <= 8, "fo_attention: GQA group %d > 8 unsupported", H / KVH);
  FO_REQUIRE(hd == 32 || hd == 64 || hd == 128, "fo_attention: head_dim %d unsupported", hd);
  AttnArgs a{q, tok_seq, tok_nvis, block_table, kc, vc, part_ml, part_o, out, H, KVH, hd, PS, maxb, nsplit, scale};
  dim3 grid(T, KVH, nsplit);
  if (hd == 128) hipLaunchKernelGGL((k_attn_split<128, 8>), grid, dim3(256), 0, s, a);
  else if (hd == 64) hipLaunchKernelGGL((k_attn_split<64, 8>), grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL((k_attn_split<32, 8>), grid, dim3(256), 0, s, a);
  int rc = fo::check_launch("fo_attention/split");
  if (rc) return rc;
  hipLaunchKernelGGL(k_attn_combine, dim3(T, H), dim3(hd < 64 ? 64 : hd), 0, s, a);
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
