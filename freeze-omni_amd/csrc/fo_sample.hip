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

__global__ __launch_bounds__(1024) void k_sample(const float* logits, int ld, int V, const int* top_k_rows,
                                                 const float* temp_rows, const float* top_p_rows,
                                                 unsigned long long seed, const int* step_rows, const int* key_rows, int ban_id,
                                                 int* out_ids, float* out_val) {
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
  hipLaunchKernelGGL(k_sample, dim3(B), dim3(1024), 0, s, logits, ld, V, top_k, temperature, top_p, seed, step, key,
                     ban_id, out_ids, out_maxlogit);
  return fo::check_launch("fo_sample");
}

}  // extern "C"
