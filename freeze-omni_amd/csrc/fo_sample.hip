// Token selection for the text decoder (AudioLLM._post_decode, models/audioLLM.py:431-477) and the
// AR speech decoder (models/decoder/decoder.py:353-359): temperature, top-k renormalisation,
// top-p nucleus, multinomial draw.  top_k == 1 is the deterministic argmax (parity mode; the
// reference's softmax -> topk(1) -> multinomial collapses to it).  One workgroup per row.
// top_k in 1..64 takes k block arg-max passes (the AR decoder's hot path); top_k == 0 (the
// reference's "no top-k filtering") and top_k > 64 take the whole-vocabulary radix path
// (sample_row_general).
// Random draws use a counter-based splitmix64 stream (seed, row, step): not bit-identical to
// torch.multinomial (documented in DESIGN.md), identical for top_k == 1.
#include "fo_common.h"

namespace {

constexpr int KMAXS = 64;

__device__ __forceinline__ uint64_t smix(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  uint64_t z = x;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

constexpr int NOIDX = 0x7fffffff;

// arg-max order: does candidate (v2, i2) replace (v1, i1)?  Larger value, ties -> smaller index; any
// candidate replaces "none yet" (i1 == NOIDX), so a row of NaN / -inf still yields an index inside the
// table (the caller gathers an embedding row with it); a NaN never replaces a number and a number always
// replaces a NaN, so one NaN does not win over the real maximum of the rest of the row.
__device__ __forceinline__ bool amax_better(float v2, int i2, float v1, int i1) {
  if (i2 == NOIDX) return false;
  if (i1 == NOIDX) return true;
  if (v2 != v2) return false;
  if (v1 != v1) return true;
  return v2 > v1 || (v2 == v1 && i2 < i1);
}

// logits the reference cannot sample from: torch.multinomial raises on the NaN probabilities a NaN or +inf
// logit (or a row of -inf) gives after the softmax (models/audioLLM.py:455-476, models/decoder/decoder.py:355-359)
__device__ __forceinline__ bool bad_logit(float x) { return x != x || x == INFINITY; }

// block arg-max over v[0..n) excluding indices already in `taken`; ties -> smallest index.
// *bad (nullable): set when the scanned values hold a NaN or +inf (block-uniform result).
__device__ void block_argmax(const float* v, int n, const int* taken, int ntaken, int ban, float* bv, int* bi,
                             float& mval, int& midx, int* bad = nullptr) {
  float best = -INFINITY;
  int besti = NOIDX;
  int b = 0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const float x = v[i];
    bool skip = (i == ban);
    for (int q = 0; q < ntaken; ++q) skip |= (taken[q] == i);
    if (!skip) {
      b |= bad_logit(x);
      if (amax_better(x, i, best, besti)) {
        best = x;
        besti = i;
      }
    }
  }
  if (bad) *bad = __syncthreads_or(b);
  bv[threadIdx.x] = best;
  bi[threadIdx.x] = besti;
  __syncthreads();
  for (int o = blockDim.x / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      const float v2 = bv[threadIdx.x + o];
      const int i2 = bi[threadIdx.x + o];
      if (amax_better(v2, i2, bv[threadIdx.x], bi[threadIdx.x])) {
        bv[threadIdx.x] = v2;
        bi[threadIdx.x] = i2;
      }
    }
    __syncthreads();
  }
  mval = bv[0];
  midx = bi[0];
  __syncthreads();
}

// First pass of the split arg-max (fo_sample with a workspace, top_k == 1 rows over a large vocabulary:
// the text decoder's 152,064-wide lm_head rows): workgroup (c, row) reduces chunk c of the row to
// (max, index, bad) so the row is read by ~75 workgroups at HBM rate instead of by one.
constexpr int AMAX_CH = 2048;  // logits per chunk (256 threads x 8)
struct AmaxPart {
  float v;
  int i;
  int bad;
  int pad;
};
__global__ __launch_bounds__(256) void k_argmax_part(const float* logits, int ld, int V, int ban, AmaxPart* parts,
                                                     int nc) {
  __shared__ float sv[256];
  __shared__ int si[256];
  const int c = blockIdx.x, row = blockIdx.y;
  const float* lg = logits + (size_t)row * ld;
  const int i0 = c * AMAX_CH + threadIdx.x * 8;
  float best = -INFINITY;
  int besti = NOIDX, b = 0;
  if (i0 + 8 <= V && (ld & 3) == 0) {
    const float4 p0 = reinterpret_cast<const float4*>(lg + i0)[0];
    const float4 p1 = reinterpret_cast<const float4*>(lg + i0)[1];
    const float f[8] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w};
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (i0 + j != ban) {
        b |= bad_logit(f[j]);
        if (amax_better(f[j], i0 + j, best, besti)) {
          best = f[j];
          besti = i0 + j;
        }
      }
  } else {
    for (int j = 0; j < 8; ++j) {
      const int i = i0 + j;
      if (i >= V || i == ban) continue;
      const float x = lg[i];
      b |= bad_logit(x);
      if (amax_better(x, i, best, besti)) {
        best = x;
        besti = i;
      }
    }
  }
  b = __syncthreads_or(b);
  sv[threadIdx.x] = best;
  si[threadIdx.x] = besti;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o && amax_better(sv[threadIdx.x + o], si[threadIdx.x + o], sv[threadIdx.x], si[threadIdx.x])) {
      sv[threadIdx.x] = sv[threadIdx.x + o];
      si[threadIdx.x] = si[threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) parts[(size_t)row * nc + c] = AmaxPart{sv[0], si[0], b, 0};
}

// The next decode step's input, produced by the sampler itself (AR speech decoder step,
// models/decoder/decoder.py:341-367: embed(id) -> first LlamaRMSNorm): the drawn id is recorded into
// a history row, its embedding row becomes the residual stream x, and the first layer's RMSNorm of
// it goes to h -- three launches of the step folded into the sampler.
struct NextInput {
  int* hist;            // [*][hist_ld]: hist[hist_row[0] * hist_ld + row] = id (host-mapped, read lazily)
  const int* hist_row;
  int hist_ld;
  const bf16_t* emb;    // [vocab][emb_ld] bf16 embedding table
  long long emb_ld;
  int D;
  float* x;             // [B][ldx] residual stream
  int ldx;
  const float* gamma;   // first RMSNorm weight
  float eps;
  float* h;             // [B][ldh] RMSNorm(x) * gamma
  int ldh;
  // the captured AR step's metadata block [pos B][slot B][nvis B][step B][key B][hist_row 1][block table B x
  // maxb] (nullable): this row's entries advance to the next step once the row is drawn (positions,
  // visible keys, step + 1; the slot from the block table on the device), and the history row is the row's step
  int* meta;
  int B, maxb, PS;
};

struct SampleSmem {
  float bv[1024];
  int bi[1024];
  int taken[KMAXS];
  float tv[KMAXS];
  // general path
  unsigned long long hist[256];
  float wf[16];
  int wi[16];
  int si[4];
  unsigned int su[4];
  float sf[4];
};

// order-preserving float -> uint32 (larger float, larger key)
__device__ __forceinline__ uint32_t fkey(float x) {
  const uint32_t u = __float_as_uint(x);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__device__ __forceinline__ unsigned long long shfl_up_u64(unsigned long long v, int o) {
  const uint32_t lo = __shfl_up((uint32_t)v, o, 64), hi = __shfl_up((uint32_t)(v >> 32), o, 64);
  return ((unsigned long long)hi << 32) | lo;
}
__device__ __forceinline__ unsigned long long shfl_u64(unsigned long long v, int l) {
  const uint32_t lo = __shfl((uint32_t)v, l, 64), hi = __shfl((uint32_t)(v >> 32), l, 64);
  return ((unsigned long long)hi << 32) | lo;
}

// Wave 0 only: walking the 256 bins from the top, the first bin whose inclusive cumulative exceeds
// thr; returns it (or -1: everything fits) and the cumulative above it in *above.
__device__ int desc_bin_search(const unsigned long long* h, unsigned long long thr, unsigned long long* above) {
  const int l = threadIdx.x;
  unsigned long long v[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = h[255 - 4 * l - j];
  const unsigned long long tot = v[0] + v[1] + v[2] + v[3];
  unsigned long long inc = tot;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned long long y = shfl_up_u64(inc, o);
    if (l >= o) inc += y;
  }
  const unsigned long long ball = __ballot(inc > thr);
  if (ball == 0ull) return -1;
  const int L = __ffsll((long long)ball) - 1;
  unsigned long long c = inc - tot;
  int b = 0;
  for (int j = 0; j < 4; ++j) {  // resolve inside this lane's 4 bins (only lane L's answer is used)
    if (c + v[j] > thr) {
      b = 255 - 4 * l - j;
      break;
    }
    c += v[j];
  }
  *above = shfl_u64(c, L);
  return __shfl(b, L, 64);
}

__device__ float block_max1024(float v, SampleSmem& sm) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) sm.wf[w] = v;
  __syncthreads();
  float t = sm.wf[0];
#pragma unroll
  for (int i = 1; i < 16; ++i) t = fmaxf(t, sm.wf[i]);
  return t;
}

// exclusive scan of one float per thread over the block (fixed order: deterministic); returns the
// exclusive prefix and the block total in *total
__device__ float block_exscan1024(float v, SampleSmem& sm, float* total) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  float inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float y = __shfl_up(inc, o, 64);
    if (l >= o) inc += y;
  }
  __syncthreads();
  if (l == 63) sm.wf[w] = inc;
  __syncthreads();
  float base = 0.f, all = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    if (i < w) base += sm.wf[i];
    all += sm.wf[i];
  }
  *total = all;
  return base + inc - v;
}

__device__ int block_exscan1024_int(int v, SampleSmem& sm, int* total) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  int inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(inc, o, 64);
    if (l >= o) inc += y;
  }
  __syncthreads();
  if (l == 63) sm.wi[w] = inc;
  __syncthreads();
  int base = 0, all = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    if (i < w) base += sm.wi[i];
    all += sm.wi[i];
  }
  *total = all;
  return base + inc - v;
}

// The general rule of AudioLLM._post_decode for one row (top_k = 0: no top-k; top_k >= V: no top-k;
// any top_p), over the whole vocabulary without sorting it:
//   * top-k: 4-pass radix select of the k-th largest logit (8-bit digits, integer bin counts); ties at
//     the threshold are taken in index order;
//   * top-p: the reference keeps the longest sorted prefix whose inclusive cumsum is <= top_p (only the
//     first token when it alone exceeds top_p).  That prefix is {logit >= t*} for a threshold t* found
//     by the same radix descent over bin SUMS of exp((x - max) / T) in 32.32 fixed point (integer LDS
//     atomics, so the set does not depend on the order of the adds); a tie group at t* is kept whole
//     or not at all;
//   * the draw: u * Z over the kept set in index order (per-thread contiguous chunks + a block scan).
// Returns the drawn id; writes the kept-set distribution e_i / Z (the reference's pre-multinomial
// `probs`) to probs when non-null.
__device__ int sample_row_general(const float* lg, int V, int k, float T, float tp, int ban, float u01,
                                  float* probs, float* max_out, int* bad_out, SampleSmem& sm) {
  const int tid = threadIdx.x;
  const float invT = 1.f / T;
  float m = -INFINITY;
  int nallowed = 0, bad = 0;
  for (int i = tid; i < V; i += 1024)
    if (i != ban) {
      const float x = lg[i];
      bad |= bad_logit(x);
      m = fmaxf(m, x);
      ++nallowed;
    }
  bad = __syncthreads_or(bad);
  m = block_max1024(m, sm);
  *max_out = m;
  *bad_out = bad || !(m > -INFINITY);
  {
    int total;
    block_exscan1024_int(nallowed, sm, &total);
    nallowed = total;
  }
  // ---- top-k threshold
  const bool topk = k > 0 && k < nallowed;
  uint32_t Kk = 0u;
  int cut = V;  // ties at Kk with index <= cut are kept
  if (topk) {
    uint32_t prefix = 0u, mask = 0u;
    unsigned long long remaining = (unsigned long long)k;
    for (int level = 0; level < 4; ++level) {
      const int shift = 24 - 8 * level;
      for (int b = tid; b < 256; b += 1024) sm.hist[b] = 0ull;
      __syncthreads();
      for (int i = tid; i < V; i += 1024) {
        if (i == ban) continue;
        const uint32_t key = fkey(lg[i]);
        if ((key & mask) == prefix) atomicAdd(&sm.hist[(key >> shift) & 255u], 1ull);
      }
      __syncthreads();
      if (tid < 64) {
        unsigned long long above = 0ull;
        const int b = desc_bin_search(sm.hist, remaining - 1ull, &above);  // first bin reaching `remaining`
        if (tid == 0) {
          sm.su[0] = prefix | ((uint32_t)b << shift);
          sm.su[1] = (uint32_t)(remaining - above);
        }
      }
      __syncthreads();
      prefix = sm.su[0];
      remaining = sm.su[1];
      mask |= 255u << shift;
      __syncthreads();
    }
    Kk = prefix;
    const int need = (int)remaining;  // ties at Kk to keep, in index order
    const int C = (V + 1023) / 1024;
    const int lo = tid * C, hi = min(V, lo + C);
    int cnt = 0;
    for (int i = lo; i < hi; ++i) cnt += (i != ban && fkey(lg[i]) == Kk);
    int tot;
    const int ex = block_exscan1024_int(cnt, sm, &tot);
    if (tid == 0) sm.si[0] = V;
    __syncthreads();
    if (ex < need && need <= ex + cnt) {
      int c = ex;
      for (int i = lo; i < hi; ++i)
        if (i != ban && fkey(lg[i]) == Kk && ++c == need) {
          sm.si[0] = i;
          break;
        }
    }
    __syncthreads();
    cut = sm.si[0];
  }
  auto kept_k = [&](int i, uint32_t key) {
    return i != ban && (!topk || key > Kk || (key == Kk && i <= cut));
  };
  // ---- top-p threshold (fixed-point sums of e_i)
  uint32_t Kp = 0u;
  if (tp > 0.f) {
    for (int b = tid; b < 256; b += 1024) sm.hist[b] = 0ull;
    __syncthreads();
    // Z in fixed point: one bin-free pass (summed into hist[0] with integer atomics)
    unsigned long long zl = 0ull;
    for (int i = tid; i < V; i += 1024) {
      const float x = lg[i];
      const uint32_t key = fkey(x);
      if (kept_k(i, key)) zl += (unsigned long long)(expf((x - m) * invT) * 4294967296.0f);
    }
    atomicAdd(&sm.hist[0], zl);
    __syncthreads();
    const unsigned long long Zfix = sm.hist[0];
    const unsigned long long thr_all = (unsigned long long)((double)tp * (double)Zfix);
    __syncthreads();
    uint32_t prefix = 0u, mask = 0u;
    unsigned long long above_all = 0ull;
    bool all_fit = false;
    for (int level = 0; level < 4 && !all_fit; ++level) {
      const int shift = 24 - 8 * level;
      for (int b = tid; b < 256; b += 1024) sm.hist[b] = 0ull;
      __syncthreads();
      for (int i = tid; i < V; i += 1024) {
        const float x = lg[i];
        const uint32_t key = fkey(x);
        if ((key & mask) == prefix && kept_k(i, key))
          atomicAdd(&sm.hist[(key >> shift) & 255u], (unsigned long long)(expf((x - m) * invT) * 4294967296.0f));
      }
      __syncthreads();
      if (tid < 64) {
        unsigned long long above = 0ull;
        const int b = desc_bin_search(sm.hist, thr_all - above_all, &above);
        if (tid == 0) {
          sm.si[1] = b;
          sm.su[2] = (uint32_t)above;
          sm.su[3] = (uint32_t)(above >> 32);
        }
      }
      __syncthreads();
      const int b = sm.si[1];
      if (b < 0) {
        all_fit = true;  // the whole prefix range fits with what is above it
      } else {
        prefix |= (uint32_t)b << shift;
        mask |= 255u << shift;
        above_all += ((unsigned long long)sm.su[3] << 32) | sm.su[2];
      }
      __syncthreads();
    }
    Kp = all_fit ? prefix : prefix + 1u;  // exact group at `prefix` does not fit
  }
  // ---- kept-set normaliser, in index order, and the draw
  const int C = (V + 1023) / 1024;
  const int lo = tid * C, hi = min(V, lo + C);
  float s = 0.f;
  for (int i = lo; i < hi; ++i) {
    const float x = lg[i];
    const uint32_t key = fkey(x);
    if (kept_k(i, key) && key >= Kp) s += expf((x - m) * invT);
  }
  float Z;
  const float ex = block_exscan1024(s, sm, &Z);
  int argmax_only = 0;
  if (!(Z > 0.f)) {  // top-p kept nothing (a tie group at the top larger than top_p): the first token only
    argmax_only = 1;
  }
  if (tid == 0) sm.si[2] = -1;
  __syncthreads();
  if (argmax_only) {
    int best = 0x7fffffff;
    for (int i = tid; i < V; i += 1024)
      if (i != ban && lg[i] == m && i < best) best = i;
    sm.bi[tid] = best;
    __syncthreads();
    for (int o = 512; o > 0; o >>= 1) {
      if (tid < o) sm.bi[tid] = min(sm.bi[tid], sm.bi[tid + o]);
      __syncthreads();
    }
    const int pick = sm.bi[0];
    if (probs)
      for (int i = tid; i < V; i += 1024) probs[i] = i == pick ? 1.f : 0.f;
    __syncthreads();
    return pick;
  }
  const float target = u01 * Z;
  if (s > 0.f && ex <= target && target < ex + s) {
    float c = ex;
    int last = -1;
    for (int i = lo; i < hi; ++i) {
      const float x = lg[i];
      const uint32_t key = fkey(x);
      if (kept_k(i, key) && key >= Kp) {
        last = i;
        c += expf((x - m) * invT);
        if (target < c) break;
      }
    }
    sm.si[2] = last;  // exactly one thread's range holds the target
  }
  __syncthreads();
  if (tid == 0 && sm.si[2] < 0) {  // rounding put the target at/after the total: the last kept token
    int pick = -1;
    for (int i = V - 1; i >= 0 && pick < 0; --i) {
      const uint32_t key = fkey(lg[i]);
      if (kept_k(i, key) && key >= Kp) pick = i;
    }
    sm.si[2] = pick;
  }
  __syncthreads();
  const int pick = sm.si[2];
  if (probs) {
    const float iz = 1.f / Z;
    for (int i = tid; i < V; i += 1024) {
      const float x = lg[i];
      const uint32_t key = fkey(x);
      probs[i] = (kept_k(i, key) && key >= Kp) ? expf((x - m) * invT) * iz : 0.f;
    }
  }
  __syncthreads();
  return pick;
}

template <bool NEXT>
__global__ __launch_bounds__(1024) void k_sample(const float* logits, int ld, int V, const int* top_k_rows,
                                                 const float* temp_rows, const float* top_p_rows,
                                                 unsigned long long seed, const int* step_rows, const int* key_rows, int ban_id,
                                                 int* out_ids, float* out_val, float* out_probs, int ldp,
                                                 NextInput nx, const AmaxPart* parts, int nc, int* err) {
  __shared__ SampleSmem sm;
  const int row = blockIdx.x;
  const float* lg = logits + (size_t)row * ld;
  float* probs = out_probs ? out_probs + (size_t)row * ldp : nullptr;
  const int k = top_k_rows ? top_k_rows[row] : 1;
  const float T = temp_rows ? temp_rows[row] : 1.f;
  const float tp = top_p_rows ? top_p_rows[row] : 0.f;
  const uint64_t st = step_rows ? (uint64_t)step_rows[row] : 0ull;
  const uint64_t key = key_rows ? (uint64_t)key_rows[row] : (uint64_t)row;  // stream id: session, not batch row
  const float u01 = (float)(uint32_t)(smix(seed ^ (0x9E37ull * (key + 1)) + st) >> 40) * (1.0f / 16777216.0f);
  const int allowed = V - ((ban_id >= 0 && ban_id < V) ? 1 : 0);
  int bad = 0;
  if (parts && k == 1 && !probs) {
    // arg-max from the split first pass (k_argmax_part): reduce the row's nc chunk results
    float best = -INFINITY;
    int besti = NOIDX, b = 0;
    for (int c = threadIdx.x; c < nc; c += blockDim.x) {
      const AmaxPart p = parts[(size_t)row * nc + c];
      b |= p.bad;
      if (amax_better(p.v, p.i, best, besti)) {
        best = p.v;
        besti = p.i;
      }
    }
    bad = __syncthreads_or(b);
    sm.bv[threadIdx.x] = best;
    sm.bi[threadIdx.x] = besti;
    __syncthreads();
    for (int o = blockDim.x / 2; o > 0; o >>= 1) {
      if (threadIdx.x < o && amax_better(sm.bv[threadIdx.x + o], sm.bi[threadIdx.x + o], sm.bv[threadIdx.x],
                                         sm.bi[threadIdx.x])) {
        sm.bv[threadIdx.x] = sm.bv[threadIdx.x + o];
        sm.bi[threadIdx.x] = sm.bi[threadIdx.x + o];
      }
      __syncthreads();
    }
    const float mv = sm.bv[0];
    const int pick = (unsigned)sm.bi[0] < (unsigned)V ? sm.bi[0] : 0;
    bad = bad || !(mv > -INFINITY);
    __syncthreads();
    if (threadIdx.x == 0) {
      out_ids[row] = pick;
      if (out_val) out_val[row] = mv;
      sm.si[0] = pick;
    }
    __syncthreads();
  } else if (k >= 1 && k <= KMAXS && k < allowed) {
    // small top-k: k block arg-max passes, then the top-p / draw over the (sorted) k candidates
    for (int q = 0; q < k; ++q) {
      float mv;
      int i;
      block_argmax(lg, V, sm.taken, q, ban_id, sm.bv, sm.bi, mv, i, q == 0 ? &bad : nullptr);
      if (q == 0) bad = bad || !(mv > -INFINITY);
      if (threadIdx.x == 0) {
        sm.taken[q] = (unsigned)i < (unsigned)V ? i : 0;
        sm.tv[q] = mv;
      }
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      int pick = sm.taken[0];
      int keep = 1;
      float z = 1.f;
      if (k > 1) {
        float* p = sm.bv + 1024 - KMAXS;   // (LDS, free after the arg-max passes: a per-thread array would live in scratch)
        z = 0.f;
        for (int q = 0; q < k; ++q) {  // softmax over the (sorted) top-k = renormalised top-k probs
          p[q] = expf((sm.tv[q] - sm.tv[0]) / T);
          z += p[q];
        }
        keep = k;
        if (tp > 0.f) {  // reference rule: drop sorted tokens whose cumsum > top_p; if that drops
          float c = 0.f;  // the first one, keep only the first (models/audioLLM.py:464-474)
          keep = 0;
          for (int q = 0; q < k; ++q) {
            c += p[q] / z;
            if (c <= tp) keep = q + 1;
            else break;
          }
          if (keep == 0) keep = 1;
          z = 0.f;
          for (int q = 0; q < keep; ++q) z += p[q];
        }
        const float u = u01 * z;
        float c = 0.f;
        pick = sm.taken[keep - 1];
        for (int q = 0; q < keep; ++q) {
          c += p[q];
          if (u < c) {
            pick = sm.taken[q];
            break;
          }
        }
        for (int q = 0; q < keep; ++q) sm.bv[q] = p[q] / z;
      } else {
        sm.bv[0] = 1.f;
      }
      sm.si[0] = pick;
      sm.si[1] = keep;
    }
    __syncthreads();
    if (probs) {
      for (int i = threadIdx.x; i < V; i += 1024) probs[i] = 0.f;
      __syncthreads();
      if (threadIdx.x < sm.si[1]) probs[sm.taken[threadIdx.x]] = sm.bv[threadIdx.x];
    }
    if (threadIdx.x == 0) {
      out_ids[row] = sm.si[0];
      if (out_val) out_val[row] = sm.tv[0];
    }
  } else {
    float mv;
    int pick = sample_row_general(lg, V, k, T, tp, ban_id, u01, probs, &mv, &bad, sm);
    if ((unsigned)pick >= (unsigned)V) pick = 0;  // never an out-of-table id (NaN rows)
    if (threadIdx.x == 0) {
      out_ids[row] = pick;
      if (out_val) out_val[row] = mv;
      sm.si[0] = pick;
    }
    __syncthreads();
  }
  // a row the reference could not sample from: flag it for the host (which raises, as torch.multinomial
  // does); the id above is still a valid table index, so nothing downstream addresses outside memory
  if (bad && err && threadIdx.x == 0) *err = 1;
  if constexpr (NEXT) {
    __syncthreads();
    // an id outside the table (a NaN row through the general path) must never address memory: row 0
    const int id = (unsigned)sm.si[0] < (unsigned)V ? sm.si[0] : 0;
    if (threadIdx.x == 0 && nx.hist) {
      const int hr = nx.meta ? nx.meta[3 * nx.B + row] : nx.hist_row[0];  // meta: the row's own step (no shared word)
      nx.hist[(size_t)hr * nx.hist_ld + row] = id;
    }
    if (threadIdx.x == 0 && nx.meta) {
      int* m = nx.meta;
      const int B = nx.B, L = m[2 * B + row], pg = L / nx.PS;
      m[row] += 1;
      m[2 * B + row] = L + 1;
      m[3 * B + row] += 1;
      m[B + row] = (pg < nx.maxb ? m[5 * B + 1 + row * nx.maxb + pg] : 0) * nx.PS + L % nx.PS;
      if (row == 0) m[5 * B] += 1;
    }
    const bf16_t* er = nx.emb + (size_t)id * nx.emb_ld;
    float* xr = nx.x + (size_t)row * nx.ldx;
    // same per-thread float4 sums and wave order as k_rmsnorm's 256-thread block (threads >= 256 add
    // zeros), so h is bit-identical to the gather + rmsnorm launches it replaces
    float s = 0.f;
    if (threadIdx.x < 256) {
      for (int i = threadIdx.x * 4; i < nx.D; i += 1024) {
        const float4 v = make_float4(bf2f(er[i]), bf2f(er[i + 1]), bf2f(er[i + 2]), bf2f(er[i + 3]));
        *reinterpret_cast<float4*>(xr + i) = v;
        s += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
      }
    }
    s = block_sum<16>(s, sm.bv);
    const float r = rsqrtf(s / (float)nx.D + nx.eps);
    if (threadIdx.x < 256) {
      float* hr = nx.h + (size_t)row * nx.ldh;
      for (int i = threadIdx.x * 4; i < nx.D; i += 1024) {
        const float4 v = make_float4(bf2f(er[i]), bf2f(er[i + 1]), bf2f(er[i + 2]), bf2f(er[i + 3]));
        const float4 g = *reinterpret_cast<const float4*>(nx.gamma + i);
        *reinterpret_cast<float4*>(hr + i) = make_float4(g.x * (v.x * r), g.y * (v.y * r), g.z * (v.z * r),
                                                         g.w * (v.w * r));
      }
    }
  }
}

// Repetition penalty of the AR speech decoder (models/decoder/decoder.py:348-351): every entry of the
// last W generated ids (SOS included) divides its logit by `penalty`.  The reference iterates
// set(generated_tokens[0][-W:]) over 0-d tensors, whose hash is their identity, so a token present
// k times in the window is divided k times; this kernel keeps that multiplicity.  win [B][W] is a
// per-row ring indexed by step % W: the step's input id (the last generated id) is stored first.
// One lane per row, divisions in window order (x / p each time, as the reference's in-place /=).
__global__ __launch_bounds__(64) void k_penalty(float* logits, int ld, int B, int V, const int* ids, int* win, int W,
                                                const int* step_rows, float penalty) {
  const int row = blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= B) return;
  const int st = step_rows[row];
  int* w = win + (size_t)row * W;
  w[st % W] = ids[row];
  const int n = st + 1 < W ? st + 1 : W;
  float* lg = logits + (size_t)row * ld;
  for (int j = 0; j < n; ++j) {
    const int t = w[j];
    if (t >= 0 && t < V) lg[t] = lg[t] / penalty;
  }
}

}  // namespace

extern "C" {

// logits [B][ld] fp32.  top_k/temp/top_p/step are per-row device arrays (nullable: k=1, T=1, p=0, step 0).
// ban_id >= 0 excludes one token (benchmark policy: EOS masked until a fixed response length).
// err (nullable): set to 1 (never cleared here) when a row cannot be sampled by the reference's rule.
// ws (nullable, >= fo_sample_ws_floats(B, V) floats): rows with top_k == 1 over V >= 8192 take the split
// arg-max (k_argmax_part over 2048-logit chunks, then the per-row reduction), one HBM pass at chip rate.
long long fo_sample_ws_floats(int B, int V) {
  const int nc = (V + AMAX_CH - 1) / AMAX_CH;
  return (long long)B * nc * (sizeof(AmaxPart) / sizeof(float));
}

int fo_sample(const float* logits, int ld, int B, int V, const int* top_k, const float* temperature,
              const float* top_p, unsigned long long seed, const int* step, const int* key, int ban_id, int* out_ids,
              float* out_maxlogit, int* err, float* ws, long long ws_floats, hipStream_t s) {
  FO_REQUIRE(B > 0 && V > 0 && (ld >= V || ld == 0), "fo_sample: bad shape B=%d V=%d ld=%d (0: one row for all)", B, V,
             ld);
  NextInput nx{};
  AmaxPart* parts = nullptr;
  const int nc = (V + AMAX_CH - 1) / AMAX_CH;
  if (ws && V >= 8192 && nc <= 1024) {
    FO_REQUIRE(ws_floats >= fo_sample_ws_floats(B, V), "fo_sample: workspace of %lld floats < %lld", ws_floats,
               fo_sample_ws_floats(B, V));
    parts = reinterpret_cast<AmaxPart*>(ws);
    hipLaunchKernelGGL(k_argmax_part, dim3(nc, B), dim3(256), 0, s, logits, ld, V, ban_id, parts, nc);
    const int rc = fo::check_launch("fo_sample/argmax_part");
    if (rc) return rc;
  }
  hipLaunchKernelGGL(k_sample<false>, dim3(B), dim3(1024), 0, s, logits, ld, V, top_k, temperature, top_p, seed, step,
                     key, ban_id, out_ids, out_maxlogit, nullptr, 0, nx, parts, nc, err);
  return fo::check_launch("fo_sample");
}

// fo_sample that also writes each row's sampling distribution (the reference's pre-multinomial `probs`,
// models/audioLLM.py:455-476) to probs [B][ldp] (ldp >= V).
int fo_sample_probs(const float* logits, int ld, int B, int V, const int* top_k, const float* temperature,
                    const float* top_p, unsigned long long seed, const int* step, const int* key, int ban_id,
                    int* out_ids, float* probs, int ldp, int* err, hipStream_t s) {
  FO_REQUIRE(B > 0 && V > 0 && probs && ldp >= V, "fo_sample_probs: bad shape B=%d V=%d ldp=%d", B, V, ldp);
  NextInput nx{};
  hipLaunchKernelGGL(k_sample<false>, dim3(B), dim3(1024), 0, s, logits, ld, V, top_k, temperature, top_p, seed, step,
                     key, ban_id, out_ids, nullptr, probs, ldp, nx, nullptr, 0, err);
  return fo::check_launch("fo_sample_probs");
}

// fo_sample, then for every row: hist[hist_row[0] * hist_ld + row] = id (hist nullable),
// x[row] = emb[id] (bf16 -> fp32, D % 4 == 0) and h[row] = RMSNorm(x[row]) * gamma.
int fo_sample_embed(const float* logits, int ld, int B, int V, const int* top_k, const float* temperature,
                    const float* top_p, unsigned long long seed, const int* step, const int* key, int ban_id,
                    int* out_ids, int* hist, const int* hist_row, int hist_ld, const void* emb, long long emb_ld,
                    int D, float* x, int ldx, const float* gamma, float eps, float* h, int ldh, int* meta, int maxb,
                    int PS, int* err, hipStream_t s) {
  FO_REQUIRE(B > 0 && V > 0 && D > 0 && (D % 4) == 0 && D <= 4096, "fo_sample_embed: bad shape B=%d V=%d D=%d", B, V, D);
  FO_REQUIRE(emb && x && gamma && h && (!hist || ((hist_row || meta) && hist_ld >= B)), "fo_sample_embed: missing buffers");
  FO_REQUIRE((ldx % 4) == 0 && (ldh % 4) == 0, "fo_sample_embed: row strides must be float4-aligned");
  FO_REQUIRE(!meta || (maxb > 0 && PS > 0 && step == meta + 3 * B && key == meta + 4 * B),
             "fo_sample_embed: meta must be the decode block whose step / key rows are passed");
  NextInput nx{hist, hist_row, hist_ld, (const bf16_t*)emb, emb_ld, D, x, ldx, gamma, eps, h, ldh, meta, B, maxb, PS};
  hipLaunchKernelGGL(k_sample<true>, dim3(B), dim3(1024), 0, s, logits, ld, V, top_k, temperature, top_p, seed, step,
                     key, ban_id, out_ids, nullptr, nullptr, 0, nx, nullptr, 0, err);
  return fo::check_launch("fo_sample_embed");
}

// logits[row][win ids] /= penalty once per window entry (see k_penalty); win [B][W] device ring,
// step[row] = this step's index (0 = the SOS input).
int fo_penalty(float* logits, int ld, int B, int V, const int* ids, int* win, int W, const int* step, float penalty,
               hipStream_t s) {
  FO_REQUIRE(B > 0 && V > 0 && W > 0 && ld >= V, "fo_penalty: bad shape B=%d V=%d W=%d", B, V, W);
  FO_REQUIRE(logits && ids && win && step && penalty > 0.f, "fo_penalty: missing buffers or penalty <= 0");
  hipLaunchKernelGGL(k_penalty, dim3((B + 63) / 64), dim3(64), 0, s, logits, ld, B, V, ids, win, W, step, penalty);
  return fo::check_launch("fo_penalty");
}

}  // extern "C"
