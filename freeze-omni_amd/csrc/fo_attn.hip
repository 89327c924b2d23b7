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
#include <type_traits>

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

#include "fo_attn_rows.h"

template <int HD, int NW = 4, int RT = 1, bool TR = false>
__global__ __launch_bounds__(NW * 64) void k_attn_mfma(AttnArgs a) {
  if constexpr (TR) {
#pragma nounroll
    for (int rep = 0; rep < (a.reps > 1 ? a.reps : 1); ++rep) {
      attn_rows_body<HD, NW, RT, TR>(a, blockIdx.x, blockIdx.y, blockIdx.z);
      __syncthreads();
    }
  } else {
    attn_rows_body<HD, NW, RT, TR>(a, blockIdx.x, blockIdx.y, blockIdx.z);
  }
}

// Single-row decode attention (the AR speech decoder's step, models/decoder/decoder.py:341-349: one
// token per session, one query head per kv head): one work group per (session, head) reads the
// session's keys once, in fp32 -- scores one key per thread (16-B loads of the key row), block
// max / sum, then P.V with the waves on interleaved keys, a float4 of the row per lane.  No MFMA tile would be
// more than 1/16 full here, and no split / merge round trip is needed at <= 4096 keys.
constexpr int DEC_MAXK = MAXPG * 16;
constexpr int DEC_NW = 8, DEC_NT = DEC_NW * 64;  // 8 waves: a key per thread up to 512 keys
// One (work item, head) of the decode attention; the normalised output row is left in o_s[HD] (LDS, visible to
// every thread after the call) and, unless to_lds_only, stored to out (+ the packed copy when armed).  Returns
// false when the host contract is broken (the row is then NaN, stored and in o_s).
template <int HD>
__device__ bool attn_decode_row(const AttnArgs& a, const int it, const int h, float* o_s, bool to_lds_only) {
  static_assert(HD % 4 == 0 && HD <= 128, "decode attention: head_dim");
  __shared__ float s_s[DEC_MAXK];
  __shared__ float q_s[HD];
  __shared__ float acc_s[DEC_NW][HD];
  __shared__ float red_s[DEC_NW];
  __shared__ int pg_s[MAXPG];
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
    for (int d = tid; d < HD; d += DEC_NT) {
      o_s[d] = NAN;
      if (to_lds_only) continue;
      orow[d] = NAN;   // (and the packed copy the next GEMM reads, when armed)
      if (a.oph) xpack_store(a.oph, a.opl, t0, h * HD + d, NAN, a.prb);
    }
    __syncthreads();
    return false;
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
  // the wave's keys, lanes LPK apart (lane_xor: no LDS round trip)
  auto xadd = [&](auto off) {
    constexpr int O = decltype(off)::value;
    if constexpr (O >= LPK && O < 64) {
      acc.x += lane_xor<O>(acc.x);
      acc.y += lane_xor<O>(acc.y);
      acc.z += lane_xor<O>(acc.z);
      acc.w += lane_xor<O>(acc.w);
    }
  };
  xadd(std::integral_constant<int, 8>{});
  xadd(std::integral_constant<int, 16>{});
  xadd(std::integral_constant<int, 32>{});
  if (sub == 0) *reinterpret_cast<float4*>(&acc_s[wave][4 * l4]) = acc;
  __syncthreads();
  for (int d = tid; d < HD; d += DEC_NT) {
    float o = 0.f;
#pragma unroll
    for (int w = 0; w < DEC_NW; ++w) o += acc_s[w][d];
    o_s[d] = o / sum;
    if (to_lds_only) continue;
    orow[d] = o / sum;
    if (a.oph) xpack_store(a.oph, a.opl, t0, h * HD + d, o / sum, a.prb);
  }
  __syncthreads();
  return true;
}

template <int HD>
__global__ __launch_bounds__(DEC_NT) void k_attn_decode(AttnArgs a) {
  __shared__ float o_s[HD];
  attn_decode_row<HD>(a, blockIdx.x, blockIdx.y, o_s, false);
}

// The AR speech decoder's attention fused with its o projection, residual add and the next RMSNorm's statistics
// (models/decoder/decoder.py:341-349 through LlamaAttention.o_proj + the residual of LlamaDecoderLayer): o is a
// sum over heads, o[s] = sum_h att[s][h] . Wo[:, h*HD:(h+1)*HD]^T, so each (session, head) workgroup multiplies its
// own attention row by its head's slice of the packed o weight (N x HD, loaded into registers at the start, while the
// attention runs) and publishes an N-wide partial; the last head to arrive for a session (agent-scope release /
// acquire ticket, as the split merge) sums the H partials in head order (deterministic), adds the residual and
// writes x (in place), yg = x * gamma_next and the row's sum of squares (one statistics group) -- the next
// gate/up GEMM's RMSNorm-on-load input.  Workgroups of one head are dealt to one XCD (its L2 serves the head's
// slice to every session).  For o slices of <= 128 KiB per head (the 896-wide decoder; not Qwen2's 3584 x 128).
struct AttnOArgs {
  const bf16x8* wo;   // packed [N/16][K/32][64][8], K = H * HD
  float* part;        // [S][H][N]
  int* tickets;       // [S] zeroed, left zeroed
  float* x;           // [S][ldx] residual stream, updated in place
  const float* gnext; // [N]
  float* yg;          // [S][ldx]
  float* sout;        // [S]
  int N, ldx, KS;     // KS = K / 32
};
constexpr int AO_TILES = 8;   // 16-column tiles per wave (8 waves: up to 128 * 8 = 1024 columns)
template <int HD>
__global__ __launch_bounds__(DEC_NT) void k_attn_decode_o(AttnArgs a, AttnOArgs o) {
  constexpr int KPH = HD / 32;   // k-steps per head
  __shared__ float o_s[HD];
  __shared__ float red_s[DEC_NW];
  __shared__ int last_s;
  const int S = gridDim.x / (8 * ((a.H + 7) / 8));
  const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
  const int h = xcd + 8 * (slot / S), it = slot % S;
  if (h >= a.H) return;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int ntiles = (o.N + 15) / 16;
  // this head's o weight fragments: wave w owns tiles w*AO_TILES .. +AO_TILES, both of the head's k-steps
  bf16x8 wf[AO_TILES][KPH];
#pragma unroll
  for (int t = 0; t < AO_TILES; ++t) {
    const int tile = wave * AO_TILES + t;
#pragma unroll
    for (int k = 0; k < KPH; ++k)
      if (tile < ntiles) wf[t][k] = __builtin_nontemporal_load(o.wo + ((size_t)tile * o.KS + h * KPH + k) * 64 + lane);
  }
  attn_decode_row<HD>(a, it, h, o_s, true);
  // A fragments of the attention row (row 0 of a 16-row block; the other rows zero), fp32 split into hi + lo
  bf16x8 ah[KPH], al[KPH];
#pragma unroll
  for (int k = 0; k < KPH; ++k) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float v = (lane & 15) == 0 ? o_s[k * 32 + 8 * (lane >> 4) + e] : 0.f;
      const __bf16 hv = (__bf16)v;
      ah[k][e] = hv;
      al[k][e] = (__bf16)(v - (float)hv);
    }
  }
  const int s = a.items ? a.items[3 * it + 1] : it;   // this item's token (decode: one per sequence)
  float* prow = o.part + ((size_t)s * a.H + h) * o.N;
#pragma unroll
  for (int t = 0; t < AO_TILES; ++t) {
    const int tile = wave * AO_TILES + t;
    if (tile >= ntiles) break;   // wave-uniform
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < KPH; ++k) {
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[k], wf[t][k], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[k], wf[t][k], acc, 0, 0, 0);
    }
    const int n = tile * 16 + lane;
    if (lane < 16 && n < o.N) prow[n] = acc[0];   // D row 0: lanes 0..15, element 0
  }
  // publish the partial and take the session's ticket (the split-merge protocol of attn_arrive_and_merge)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int old = __hip_atomic_fetch_add(o.tickets + s, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last_s = old == a.H - 1;
  }
  __syncthreads();
  if (!last_s) return;
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(o.tickets + s, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  const float* ps = o.part + (size_t)s * a.H * o.N;
  float ssq = 0.f;
  for (int n = tid; n < o.N; n += DEC_NT) {
    // the H partials come from other XCDs' workgroups (a memory-side round trip each): all loads of a group of 16
    // heads are issued together, then summed in head order (deterministic)
    float v = 0.f;
    for (int h0 = 0; h0 < a.H; h0 += 16) {
      float pv[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) pv[j] = h0 + j < a.H ? ps[(size_t)(h0 + j) * o.N + n] : 0.f;
#pragma unroll
      for (int j = 0; j < 16; ++j) v += pv[j];
    }
    const size_t off = (size_t)s * o.ldx + n;
    const float y = o.x[off] + v;
    o.x[off] = y;
    o.yg[off] = y * o.gnext[n];
    ssq += y * y;
  }
  ssq = block_sum<DEC_NW>(ssq, red_s);
  if (tid == 0) o.sout[s] = ssq;
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
                                                      int ldo, uint16_t* oph, uint16_t* opl, int prb) {
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
  // staging: each thread's key / value / position rows (up to RB_ per batch) are all loaded before any of them
  // is stored to LDS -- one dependent memory round trip per batch instead of one per row (a chunk's new rows come
  // from the q|k|v output through the same branch-free loads and are then appended to the ring)
  constexpr int RB_ = 8;
  // the chunk's query rows (+ the u / v position biases), at most 2 per thread, ride in the first batch
  float qx[2], qbu[2], qbv[2];
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int e = threadIdx.x + r * 256;
    const int i = e < T * dk ? e / dk : 0, c = e < T * dk ? e % dk : 0;
    qx[r] = qkv[((size_t)b * T + i) * ldq + hh * dk + c];
    qbu[r] = bu[hh * dk + c];
    qbv[r] = bv[hh * dk + c];
  }
  for (int e0 = 0; e0 < Lk * D4; e0 += RB_ * 256) {
    typedef float v4f __attribute__((ext_vector_type(4)));   // (a native vector: the arrays stay in VGPRs)
    v4f kk[RB_], vv[RB_], pp[RB_];
#pragma unroll
    for (int q = 0; q < RB_; ++q) {
      const int e = e0 + q * 256 + threadIdx.x;
      const bool on = e < Lk * D4;
      const int j = on ? e / D4 : 0, c = on ? (e % D4) * 4 : 0;
      const bool old_row = j < Lold;
      const size_t ro = (rb * cap + (st + j) % cap) * d + hh * dk + c;
      const float* src = qkv + ((size_t)b * T + (old_row ? 0 : j - Lold)) * ldq + hh * dk + c;
      kk[q] = *reinterpret_cast<const v4f*>(old_row ? kr + ro : src + d);
      vv[q] = *reinterpret_cast<const v4f*>(old_row ? vr + ro : src + 2 * d);
      pp[q] = *reinterpret_cast<const v4f*>(ptab + (size_t)(ps + j) * d + hh * dk + c);
    }
#pragma unroll
    for (int q = 0; q < RB_; ++q) {
      const int e = e0 + q * 256 + threadIdx.x;
      if (e < Lk * D4) {
        const int j = e / D4, c = (e % D4) * 4;
        if (j >= Lold) {   // the chunk's new rows enter the ring
          const size_t ro = (rb * cap + (st + j) % cap) * d + hh * dk + c;
          *reinterpret_cast<v4f*>(kr + ro) = kk[q];
          *reinterpret_cast<v4f*>(vr + ro) = vv[q];
        }
        *reinterpret_cast<v4f*>(k_s + j * KP + c) = kk[q];
        *reinterpret_cast<v4f*>(v_s + j * KP + c) = vv[q];
        *reinterpret_cast<v4f*>(p_s + j * KP + c) = pp[q];
      }
    }
  }
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int e = threadIdx.x + r * 256;
    if (e < T * dk) {
      qu[e] = qx[r] + qbu[r];
      qv[e] = qx[r] + qbv[r];
    }
  }
  for (int e = threadIdx.x + 512; e < T * dk; e += blockDim.x) {   // (T * dk > 512: not used at dk 64, T <= 8)
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
    if (oph) xpack_store(oph, opl, b * T + i, hh * dk + c, acc, prb);   // the out projection's packed input
  }
}

// k_relpos_fused over C consecutive chunks of the same users in ONE launch (the offline listen's grouped encoder,
// SpeechEncoderEngine.run(chunks=C)): per (user, head) the chunks run in order, each with its own ring / position
// metadata (meta[chunk][start B | len B | ring B | pstart B], host_meta after the chunks before it) and the chunk's
// rows of the group's q|k|v output (chunk-major: row (j * B + b) * T + i).  The ring rows that chunks < j of this
// launch appended are read from their q|k|v rows, never re-read from the ring this launch writes (so no global
// write-then-read inside the launch); every chunk still appends its rows to the ring for the launches after it.
// Chunk j sees exactly the left context the sequential per-chunk launches give it.
// k_relpos_fused over C consecutive chunks of the same users in ONE launch (the offline listen's grouped encoder,
// SpeechEncoderEngine.run(chunks=C)): one workgroup per (user, head, chunk), all chunks at once -- chunk j's context is
// the ring as it was before the launch (meta[chunk][start B | len B | ring B | pstart B]: host_meta after the chunks
// before it) plus the k / v columns of the earlier chunks' q|k|v rows (chunk-major: row (j * B + b) * T + i), which the
// group's q|k|v GEMM has already produced; nothing is read from ring slots this launch's appends
// (k_relpos_chunks_append, the next launch) will write.  Chunk j sees exactly the left context the sequential
// per-chunk launches give it.
__global__ __launch_bounds__(256) void k_relpos_chunks(const float* qkv, int ldq, float* kr, float* vr, int cap,
                                                       const int* meta, int B, int C, const float* ptab,
                                                       const float* bu, const float* bv, int T, int h, int dk,
                                                       float scale, float* out, int ldo) {
  extern __shared__ float smem[];
  const int KP = dk + 4;
  float* k_s = smem;
  float* v_s = k_s + cap * KP;
  float* p_s = v_s + cap * KP;
  float* qu = p_s + cap * KP;
  float* qv = qu + T * dk;
  float* sc = qv + T * dk;
  const int b = blockIdx.x, hh = blockIdx.y;
  const int d = h * dk;
  const int D4 = dk / 4;
  typedef float v4f __attribute__((ext_vector_type(4)));
  constexpr int RB_ = 8;
  {
    const int jc = blockIdx.z;
    const int* m = meta + (size_t)jc * 4 * B;
    const size_t rb = (size_t)m[2 * B + b];
    const int Lold = m[B + b], Lk = Lold + T;
    const int st = m[b];
    const int ps = m[3 * B + b];
    const size_t row0 = ((size_t)jc * B + b) * T;   // this chunk's first q|k|v row
    float qx[2], qbu[2], qbv[2];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int e = threadIdx.x + r * 256;
      const int i = e < T * dk ? e / dk : 0, c = e < T * dk ? e % dk : 0;
      qx[r] = qkv[(row0 + i) * ldq + hh * dk + c];
      qbu[r] = bu[hh * dk + c];
      qbv[r] = bv[hh * dk + c];
    }
    for (int e0 = 0; e0 < Lk * D4; e0 += RB_ * 256) {
      v4f kk[RB_], vv[RB_], pp[RB_];
#pragma unroll
      for (int q = 0; q < RB_; ++q) {
        const int e = e0 + q * 256 + threadIdx.x;
        const bool on = e < Lk * D4;
        const int j = on ? e / D4 : 0, c = on ? (e % D4) * 4 : 0;
        // row j of the context: the chunk's own (j >= Lold), one an earlier chunk of this launch appended (age <
        // jc * T), or one in the ring from before the launch
        const int age = Lold - 1 - j;
        const float* src;
        const float* ksrc;
        const float* vsrc;
        if (j >= Lold) {
          src = qkv + (row0 + (j - Lold)) * ldq + hh * dk + c;
          ksrc = src + d;
          vsrc = src + 2 * d;
        } else if (age < jc * T) {
          const int jj = jc - 1 - age / T, t = T - 1 - age % T;
          src = qkv + (((size_t)jj * B + b) * T + t) * ldq + hh * dk + c;
          ksrc = src + d;
          vsrc = src + 2 * d;
        } else {
          const size_t ro = (rb * cap + (st + j) % cap) * d + hh * dk + c;
          ksrc = kr + ro;
          vsrc = vr + ro;
        }
        kk[q] = *reinterpret_cast<const v4f*>(ksrc);
        vv[q] = *reinterpret_cast<const v4f*>(vsrc);
        pp[q] = *reinterpret_cast<const v4f*>(ptab + (size_t)(ps + j) * d + hh * dk + c);
      }
#pragma unroll
      for (int q = 0; q < RB_; ++q) {
        const int e = e0 + q * 256 + threadIdx.x;
        if (e < Lk * D4) {
          const int j = e / D4, c = (e % D4) * 4;
          *reinterpret_cast<v4f*>(k_s + j * KP + c) = kk[q];
          *reinterpret_cast<v4f*>(v_s + j * KP + c) = vv[q];
          *reinterpret_cast<v4f*>(p_s + j * KP + c) = pp[q];
        }
      }
    }
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int e = threadIdx.x + r * 256;
      if (e < T * dk) {
        qu[e] = qx[r] + qbu[r];
        qv[e] = qx[r] + qbv[r];
      }
    }
    for (int e = threadIdx.x + 512; e < T * dk; e += blockDim.x) {
      const int i = e / dk, c = e % dk;
      const float x = qkv[(row0 + i) * ldq + hh * dk + c];
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
      float mx = -INFINITY;
      for (int j = lane; j < Lk; j += 64) mx = fmaxf(mx, sc[i * cap + j]);
      mx = wave_max(mx);
      float sum = 0.f;
      for (int j = lane; j < Lk; j += 64) {
        const float e = expf(sc[i * cap + j] - mx);
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
      out[(row0 + i) * ldo + hh * dk + c] = acc;
    }
  }
}

// The ring appends of a listen group's C chunks, after k_relpos_chunks has read the ring: chunk j's T rows (k, v
// columns of its q|k|v rows) at its sequential positions (start_j + len_j + t) % cap -- consecutive over the chunks, so
// the ring ends as C sequential appends leave it (C * T <= cap).
__global__ void k_relpos_chunks_append(const float* qkv, int ldq, float* kr, float* vr, int cap, const int* meta, int B,
                                       int C, int T, int d) {
  const int D4 = d / 4;
  const long long n = (long long)C * B * T * D4;
  typedef float v4f __attribute__((ext_vector_type(4)));
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(e % D4) * 4;
    const long long r = e / D4;          // q|k|v row: (jc * B + b) * T + t
    const int t = (int)(r % T);
    const int b = (int)((r / T) % B);
    const int jc = (int)(r / ((long long)T * B));
    const int* m = meta + (size_t)jc * 4 * B;
    const size_t rb = (size_t)m[2 * B + b];
    const size_t ro = (rb * cap + (m[b] + m[B + b] + t) % cap) * d + c;
    const float* src = qkv + (size_t)r * ldq + c;
    *reinterpret_cast<v4f*>(kr + ro) = *reinterpret_cast<const v4f*>(src + d);
    *reinterpret_cast<v4f*>(vr + ro) = *reinterpret_cast<const v4f*>(src + 2 * d);
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
thread_local unsigned long long* g_attn_trc = nullptr;   // fo_attention_set_trace (probes)

// query rows one attention work item may carry (fo_attn_max_rows): 32 on the 8-wave head-dim-128 kernel
inline int attn_max_rows(int hd) { return hd == 128 && attn_waves() == 8 ? 32 : 16; }

// fo_attention_set_opack: the next launch's packed output and its extent (columns, allocated row blocks)
thread_local uint16_t* g_oph = nullptr;
thread_local uint16_t* g_opl = nullptr;
thread_local int g_op_cols = 0, g_op_rb = 0;

inline int grid_for(long long n) {
  long long g = (n + 255) / 256;
  return (int)(g > 8192 ? 8192 : (g < 1 ? 1 : g));
}

}  // namespace

extern "C" {

int fo_attention_set_opack(void* hi, void* lo, int cols, int cap_rb) {
  g_oph = g_opl = nullptr;
  g_op_cols = g_op_rb = 0;
  FO_REQUIRE((hi == nullptr) == (lo == nullptr), "fo_attention_set_opack: both halves or neither");
  if (!hi) return 0;
  FO_REQUIRE(cols > 0 && (cols & 31) == 0 && cap_rb >= 1 && cap_rb <= 4,
             "fo_attention_set_opack: cols %d (a multiple of 32) and 1..4 row blocks (%d) required", cols, cap_rb);
  g_oph = reinterpret_cast<uint16_t*>(hi);
  g_opl = reinterpret_cast<uint16_t*>(lo);
  g_op_cols = cols;
  g_op_rb = cap_rb;
  return 0;
}

// Decode attention (one token per sequence, items NULL or one per token) fused with the o projection + residual
// + next-norm statistics (k_attn_decode_o above).  Arguments as fo_attention's decode form, plus: wo packed o weight
// (N x H*hd), part >= T * H * N floats, tickets T zeroed ints (left zeroed), x [T][ldx] residual (updated), gnext
// [N], yg [T][ldx], sout [T] (one statistics group per row).
int fo_attention_o(const float* q, int T, const int* items, const int* tok_nvis, const int* block_table, int maxb,
                   int PS, const float* kc, const float* vc, int H, int hd, float scale, const void* wo, int N,
                   float* part, int* tickets, float* x, int ldx, const float* gnext, float* yg, float* sout,
                   hipStream_t s) {
  FO_REQUIRE(T > 0 && H > 0 && hd == 64 && N > 0 && N <= 16 * AO_TILES * DEC_NW && ldx >= N,
             "fo_attention_o: T=%d H=%d hd=%d N=%d (N <= %d)", T, H, hd, N, 16 * AO_TILES * DEC_NW);
  FO_REQUIRE((long long)maxb * PS <= DEC_MAXK, "fo_attention_o: %d keys per sequence exceed %d", maxb * PS, DEC_MAXK);
  FO_REQUIRE(wo && part && tickets && x && gnext && yg && sout, "fo_attention_o: null argument");
  AttnArgs a{q, items, tok_nvis, block_table, kc, vc, nullptr, nullptr, nullptr, H, H, PS, maxb, 1, scale,
             nullptr, 0, 1, nullptr, nullptr, 1};
  AttnOArgs o{reinterpret_cast<const bf16x8*>(wo), part, tickets, x, gnext, yg, sout, N, ldx, H * hd / 32};
  const int grid = 8 * T * ((H + 7) / 8);
  hipLaunchKernelGGL((k_attn_decode_o<64>), dim3(grid), dim3(DEC_NT), 0, s, a, o);
  fo::count_launch(FO_L_ATTN_O);
  return fo::check_launch("fo_attention_o");
}

int fo_attn_max_rows(int hd) { return attn_max_rows(hd); }

int fo_attention_set_trace(void* trace) {
  g_attn_trc = reinterpret_cast<unsigned long long*>(trace);
  return 0;
}

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
  uint16_t *oph = g_oph, *opl = g_opl;   // the armed packed output is consumed by this launch whatever happens
  const int op_cols = g_op_cols, op_rb = g_op_rb;
  g_oph = g_opl = nullptr;
  g_op_cols = g_op_rb = 0;
  FO_REQUIRE(T > 0 && n_items > 0 && KVH > 0 && H % KVH == 0, "fo_attention: bad shape");
  FO_REQUIRE(!oph || (op_cols == H * hd && op_rb * 16 >= T),
             "fo_attention: packed output of %d columns x %d row blocks armed for %d x %d tokens", op_cols, op_rb,
             H * hd, T);
  FO_REQUIRE(items || T % n_items == 0, "fo_attention: items NULL needs T / n_items tokens per item");
  FO_REQUIRE(hd == 32 || hd == 64 || hd == 128, "fo_attention: head_dim %d unsupported", hd);
  // up to 32 query rows per item on the 8-wave head-dim-128 kernel (two row tiles share every K / V load: a duplex
  // tick's 4 tokens x 7 query heads per kv head read the session's keys once, not twice), 16 elsewhere
  const int rows_max = attn_max_rows(hd);
  FO_REQUIRE(max_rows >= 1 && max_rows <= rows_max, "fo_attention: %d query rows per item (max %d)", max_rows,
             rows_max);
  FO_REQUIRE(nsplit >= 1 && (nsplit == 1 || (part_ml && part_o)), "fo_attention: bad split buffers");
  FO_REQUIRE(!tickets || keys_per_split >= 32, "fo_attention: keys_per_split %d < 32", keys_per_split);
  // the in-launch merge reads the partials back through 32-bit buffer offsets (ld_sc1)
  FO_REQUIRE(!tickets || nsplit == 1 || (long long)T * H * nsplit * hd * 4 < (1ll << 31),
             "fo_attention: %d tokens x %d heads x %d splits of partials exceed the merge's 2 GiB window", T, H, nsplit);
  AttnArgs a{q, items, tok_nvis, block_table, kc, vc, part_ml, part_o, out, H, KVH, PS, maxb, nsplit, scale,
             tickets, keys_per_split, items ? 1 : T / n_items, oph, opl, (T + 15) / 16, g_attn_trc,
             g_attn_trc && getenv("FO_ATTN_TRACE_REPS") ? atoi(getenv("FO_ATTN_TRACE_REPS")) : 1};
  const bool dec = max_rows == 1 && (long long)maxb * PS <= DEC_MAXK;
  FO_REQUIRE(!a.oph || (T <= 64 && (dec || nsplit == 1 || tickets)),
             "fo_attention: packed output needs <= 64 tokens and no combine launch");
  if (dec) {  // one query row per (session, head): decode kernel
    dim3 g1(n_items, H);
    if (hd == 128) hipLaunchKernelGGL((k_attn_decode<128>), g1, dim3(DEC_NT), 0, s, a);
    else if (hd == 64) hipLaunchKernelGGL((k_attn_decode<64>), g1, dim3(DEC_NT), 0, s, a);
    else hipLaunchKernelGGL((k_attn_decode<32>), g1, dim3(DEC_NT), 0, s, a);
    fo::count_launch(FO_L_ATTN_DECODE);
    if (a.oph) fo::count_launch(FO_L_ATTN_OPACK);
    return fo::check_launch("fo_attention/decode");
  }
  dim3 grid(n_items, KVH, nsplit);
  // splits under 64 keys (the text step's short contexts spread over more CUs: a split's K / V arrive at one CU's
  // memory parallelism) take the 2-wave form with 32-key tiles
  const bool small = hd == 128 && tickets && keys_per_split < 64 && max_rows <= 16 && !a.trc;
  if (small) hipLaunchKernelGGL((k_attn_mfma<128, 2>), grid, dim3(128), 0, s, a);
  else if (hd == 128 && attn_waves() == 8 && max_rows > 16) hipLaunchKernelGGL((k_attn_mfma<128, 8, 2>), grid, dim3(512), 0, s, a);
  else if (hd == 128 && attn_waves() == 8 && a.trc) hipLaunchKernelGGL((k_attn_mfma<128, 8, 1, true>), grid, dim3(512), 0, s, a);
  else if (hd == 128 && attn_waves() == 8) hipLaunchKernelGGL((k_attn_mfma<128, 8>), grid, dim3(512), 0, s, a);
  else if (hd == 128) hipLaunchKernelGGL((k_attn_mfma<128>), grid, dim3(256), 0, s, a);
  else if (hd == 64) hipLaunchKernelGGL((k_attn_mfma<64>), grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL((k_attn_mfma<32>), grid, dim3(256), 0, s, a);
  fo::count_launch(FO_L_ATTN_MFMA);
  if (a.oph) fo::count_launch(FO_L_ATTN_OPACK);
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
  uint16_t *oph = g_oph, *opl = g_opl;   // consumed by this launch whatever happens
  const int op_cols = g_op_cols, op_rb = g_op_rb;
  g_oph = g_opl = nullptr;
  g_op_cols = g_op_rb = 0;
  FO_REQUIRE(!oph || (op_cols == h * dk && op_rb * 16 >= B * T),
             "fo_relpos_attention_fused: packed output of %d columns x %d row blocks armed for %d x %d rows", op_cols,
             op_rb, h * dk, B * T);
  FO_REQUIRE(T >= 1 && T <= cap && dk % 4 == 0 && (ldq % 4) == 0, "fo_relpos_attention_fused: T=%d dk=%d", T, dk);
  const size_t lds = (size_t)(3 * cap * (dk + 4) + 2 * T * dk + T * cap) * sizeof(float);
  FO_REQUIRE(lds <= 160 * 1024, "fo_relpos_attention_fused: ring of %d x %d exceeds LDS", cap, dk);
  hipLaunchKernelGGL(k_relpos_fused, dim3(B, h), dim3(256), lds, s, qkv, ldq, kr, vr, cap, start, len, ring, ptab,
                     pstart, bu, bv, T, h, dk, scale, out, ldo, oph, opl, (B * T + 15) / 16);
  fo::count_launch(FO_L_RELPOS);
  if (oph) fo::count_launch(FO_L_ATTN_OPACK);
  return fo::check_launch("fo_relpos_attention_fused");
}

int fo_relpos_attention_chunks(const float* qkv, int ldq, float* kr, float* vr, int cap, const int* meta, int B, int C,
                               const float* ptab, const float* bu, const float* bv, int T, int h, int dk, float scale,
                               float* out, int ldo, hipStream_t s) {
  FO_REQUIRE(B >= 1 && C >= 1 && T >= 1 && T <= cap && dk % 4 == 0 && (ldq % 4) == 0,
             "fo_relpos_attention_chunks: B=%d C=%d T=%d dk=%d", B, C, T, dk);
  FO_REQUIRE(C * T <= cap, "fo_relpos_attention_chunks: %d chunks of %d frames exceed the ring (%d)", C, T, cap);
  const size_t lds = (size_t)(3 * cap * (dk + 4) + 2 * T * dk + T * cap) * sizeof(float);
  FO_REQUIRE(lds <= 160 * 1024, "fo_relpos_attention_chunks: ring of %d x %d exceeds LDS", cap, dk);
  hipLaunchKernelGGL(k_relpos_chunks, dim3(B, h, C), dim3(256), lds, s, qkv, ldq, kr, vr, cap, meta, B, C, ptab, bu,
                     bv, T, h, dk, scale, out, ldo);
  fo::count_launch(FO_L_RELPOS);
  int rc = fo::check_launch("fo_relpos_attention_chunks");
  if (rc) return rc;
  const long long n = (long long)C * B * T * (h * dk / 4);
  hipLaunchKernelGGL(k_relpos_chunks_append, dim3(grid_for(n)), dim3(256), 0, s, qkv, ldq, kr, vr, cap, meta, B, C, T,
                     h * dk);
  return fo::check_launch("fo_relpos_attention_chunks/append");
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
