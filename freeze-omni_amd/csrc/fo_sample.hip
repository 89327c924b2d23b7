// Token selection for the text decoder (AudioLLM._post_decode, models/audioLLM.py:431-477) and the
// AR speech decoder (models/decoder/decoder.py:353-359): temperature, top-k renormalisation,
// top-p nucleus, multinomial draw.  top_k == 1 is the deterministic argmax (parity mode; the
// reference's softmax -> topk(1) -> multinomial collapses to it).  One workgroup per row.
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

// block arg-max over v[0..n) excluding indices already in `taken`; ties -> smallest index
__device__ void block_argmax(const float* v, int n, const int* taken, int ntaken, int ban, float* bv, int* bi,
                             float& mval, int& midx) {
  float best = -INFINITY;
  int besti = 0x7fffffff;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const float x = v[i];
    bool skip = (i == ban);
    for (int q = 0; q < ntaken; ++q) skip |= (taken[q] == i);
    if (!skip && (x > best || (x == best && i < besti))) {
      best = x;
      besti = i;
    }
  }
  bv[threadIdx.x] = best;
  bi[threadIdx.x] = besti;
  __syncthreads();
  for (int o = blockDim.x / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      const float v2 = bv[threadIdx.x + o];
      const int i2 = bi[threadIdx.x + o];
      if (v2 > bv[threadIdx.x] || (v2 == bv[threadIdx.x] && i2 < bi[threadIdx.x])) {
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
};

template <bool NEXT>
__global__ __launch_bounds__(1024) void k_sample(const float* logits, int ld, int V, const int* top_k_rows,
                                                 const float* temp_rows, const float* top_p_rows,
                                                 unsigned long long seed, const int* step_rows, const int* key_rows, int ban_id,
                                                 int* out_ids, float* out_val, NextInput nx) {
  __shared__ float bv[1024];
  __shared__ int bi[1024];
  __shared__ int taken[KMAXS];
  __shared__ float tv[KMAXS];
  const int row = blockIdx.x;
  const float* lg = logits + (size_t)row * ld;
  int k = top_k_rows ? top_k_rows[row] : 1;
  if (k < 1) k = 1;
  if (k > KMAXS) k = KMAXS;
  for (int q = 0; q < k; ++q) {
    float m;
    int i;
    block_argmax(lg, V, taken, q, ban_id, bv, bi, m, i);
    if (threadIdx.x == 0) {
      taken[q] = i;
      tv[q] = m;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    int pick = taken[0];
    if (k > 1) {
      const float T = temp_rows ? temp_rows[row] : 1.f;
      const float tp = top_p_rows ? top_p_rows[row] : 0.f;
      float p[KMAXS];
      float z = 0.f;
      for (int q = 0; q < k; ++q) {  // softmax over the (sorted) top-k = renormalised top-k probs
        p[q] = expf((tv[q] - tv[0]) / T);
        z += p[q];
      }
      int keep = k;
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
      const uint64_t st = step_rows ? (uint64_t)step_rows[row] : 0ull;
      const uint64_t key = key_rows ? (uint64_t)key_rows[row] : (uint64_t)row;  // stream id: session, not batch row
      const float u = (float)(uint32_t)(smix(seed ^ (0x9E37ull * (key + 1)) + st) >> 40) *
                      (1.0f / 16777216.0f) * z;
      float c = 0.f;
      pick = taken[keep - 1];
      for (int q = 0; q < keep; ++q) {
        c += p[q];
        if (u < c) {
          pick = taken[q];
          break;
        }
      }
    }
    out_ids[row] = pick;
    if (out_val) out_val[row] = tv[0];
    if (NEXT) {
      taken[0] = pick;
      if (nx.hist) nx.hist[(size_t)nx.hist_row[0] * nx.hist_ld + row] = pick;
    }
  }
  if constexpr (NEXT) {
    __syncthreads();
    const int id = taken[0];
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
    s = block_sum<16>(s, bv);
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
int fo_sample(const float* logits, int ld, int B, int V, const int* top_k, const float* temperature,
              const float* top_p, unsigned long long seed, const int* step, const int* key, int ban_id, int* out_ids,
              float* out_maxlogit, hipStream_t s) {
  FO_REQUIRE(B > 0 && V > 0, "fo_sample: bad shape");
  NextInput nx{};
  hipLaunchKernelGGL(k_sample<false>, dim3(B), dim3(1024), 0, s, logits, ld, V, top_k, temperature, top_p, seed, step,
                     key, ban_id, out_ids, out_maxlogit, nx);
  return fo::check_launch("fo_sample");
}

// fo_sample, then for every row: hist[hist_row[0] * hist_ld + row] = id (hist nullable),
// x[row] = emb[id] (bf16 -> fp32, D % 4 == 0) and h[row] = RMSNorm(x[row]) * gamma.
int fo_sample_embed(const float* logits, int ld, int B, int V, const int* top_k, const float* temperature,
                    const float* top_p, unsigned long long seed, const int* step, const int* key, int ban_id,
                    int* out_ids, int* hist, const int* hist_row, int hist_ld, const void* emb, long long emb_ld,
                    int D, float* x, int ldx, const float* gamma, float eps, float* h, int ldh, hipStream_t s) {
  FO_REQUIRE(B > 0 && V > 0 && D > 0 && (D % 4) == 0 && D <= 4096, "fo_sample_embed: bad shape B=%d V=%d D=%d", B, V, D);
  FO_REQUIRE(emb && x && gamma && h && (!hist || (hist_row && hist_ld >= B)), "fo_sample_embed: missing buffers");
  FO_REQUIRE((ldx % 4) == 0 && (ldh % 4) == 0, "fo_sample_embed: row strides must be float4-aligned");
  NextInput nx{hist, hist_row, hist_ld, (const bf16_t*)emb, emb_ld, D, x, ldx, gamma, eps, h, ldh};
  hipLaunchKernelGGL(k_sample<true>, dim3(B), dim3(1024), 0, s, logits, ld, V, top_k, temperature, top_p, seed, step,
                     key, ban_id, out_ids, nullptr, nx);
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
