// Memory-bound helper kernels of the hot path: synthetic-weight fill, RMSNorm/LayerNorm,
// embedding / row gathers, im2col for the conv front ends, the dialog-state head.
// All loads are 16-B vectorised where the row layout allows (MI355X Guideline 13).
#include "fo_common.h"

namespace {

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  uint64_t z = x;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// oracle/weights.py hash_uniform, bit-exact: (2u-1) * scale + center with two IEEE roundings
// (no FMA contraction), then bf16 RNE.
__global__ void k_fill_hash(void* out, int out_bf16, long long n, uint64_t key, float center, float scale) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const uint64_t v = splitmix64(key + (uint64_t)i);
    const float u = (float)(uint32_t)(v >> 40) * (1.0f / 16777216.0f);
    const float t = __fadd_rn(__fmul_rn(2.0f, u), -1.0f);
    const float w = __fadd_rn(__fmul_rn(t, scale), center);
    const bf16_t b = f2bf(w);
    if (out_bf16) reinterpret_cast<bf16_t*>(out)[i] = b;
    else reinterpret_cast<float*>(out)[i] = bf2f(b);
  }
}

// one row per block, 256 threads
__global__ __launch_bounds__(256) void k_rmsnorm(const float* x, int ldx, int D, const float* w, float eps,
                                                 float* out, int ldo, int round_fp16) {
  __shared__ float red[4];
  const float* xr = x + (size_t)blockIdx.x * ldx;
  float* o = out + (size_t)blockIdx.x * ldo;
  float s = 0.f;
  for (int i = threadIdx.x * 4; i < D; i += 1024) {
    const float4 v = *reinterpret_cast<const float4*>(xr + i);
    s += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  s = block_sum<4>(s, red);
  const float r = rsqrtf(s / (float)D + eps);
  for (int i = threadIdx.x * 4; i < D; i += 1024) {
    float4 v = *reinterpret_cast<const float4*>(xr + i);
    const float4 g = *reinterpret_cast<const float4*>(w + i);
    float h0 = v.x * r, h1 = v.y * r, h2 = v.z * r, h3 = v.w * r;
    if (round_fp16) {
      h0 = round_f16(h0);
      h1 = round_f16(h1);
      h2 = round_f16(h2);
      h3 = round_f16(h3);
    }
    *reinterpret_cast<float4*>(o + i) = make_float4(g.x * h0, g.y * h1, g.z * h2, g.w * h3);
  }
}

__global__ __launch_bounds__(256) void k_layernorm(const float* x, int ldx, int D, const float* w, const float* b,
                                                   float eps, float* out, int ldo, int act) {
  __shared__ float red[4];
  const float* xr = x + (size_t)blockIdx.x * ldx;
  float* o = out + (size_t)blockIdx.x * ldo;
  float s = 0.f;
  for (int i = threadIdx.x; i < D; i += 256) s += xr[i];
  const float mean = block_sum<4>(s, red) / (float)D;
  float q = 0.f;
  for (int i = threadIdx.x; i < D; i += 256) {
    const float d = xr[i] - mean;
    q += d * d;
  }
  const float var = block_sum<4>(q, red) / (float)D;
  const float r = 1.0f / sqrtf(var + eps);
  for (int i = threadIdx.x; i < D; i += 256) {
    o[i] = apply_act((xr[i] - mean) * r * w[i] + b[i], act);
  }
}

// out[m] = table[idx[m]] for f32 or bf16 tables; optional fp16 rounding (the reference's .half()).
__global__ void k_gather_rows(const void* table, int table_bf16, long long ld_tab, const int* idx, int M, int D,
                              float* out, int ldo, const int* out_rows, int round_fp16) {
  const int m = blockIdx.x;
  if (m >= M) return;
  const long long r = idx ? idx[m] : m;
  const long long orow = out_rows ? out_rows[m] : m;
  for (int i = threadIdx.x; i < D; i += blockDim.x) {
    float v = table_bf16 ? bf2f(reinterpret_cast<const bf16_t*>(table)[r * ld_tab + i])
                         : reinterpret_cast<const float*>(table)[r * ld_tab + i];
    if (round_fp16) v = round_f16(v);
    out[(size_t)orow * ldo + i] = v;
  }
}

// 3x3 / stride-2 im2col.  in[b][c][h][w] addressed by strides (sb, sc, sh, sw); out row
// (b, ho, wo) -> columns c*9 + i*3 + j, zero-padded to ldo.  Optional global CMVN on the input
// (models/encoder/cmvn.py:24-35) applied per w index: (x - mean[w]) * istd[w].
__global__ void k_im2col_3x3s2(const float* in, int B, int C, int H, int W, long long sb, long long sc, long long sh,
                               long long sw, const float* mean, const float* istd, float* out, int ldo) {
  const int Ho = (H - 3) / 2 + 1, Wo = (W - 3) / 2 + 1;
  const long long rows = (long long)B * Ho * Wo;
  const long long total = rows * ldo;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const long long row = e / ldo;
    const int col = (int)(e % ldo);
    float v = 0.f;
    if (col < C * 9) {
      const int c = col / 9, ij = col % 9, i = ij / 3, j = ij % 3;
      const int b = (int)(row / (Ho * Wo)), rem = (int)(row % (Ho * Wo));
      const int ho = rem / Wo, wo = rem % Wo;
      const int h = 2 * ho + i, w = 2 * wo + j;
      v = in[b * sb + c * sc + h * sh + w * sw];
      if (mean) v = (v - mean[w]) * istd[w];
    }
    out[e] = v;
  }
}

// [B][t*F + f][C] -> [B*t][c*F + f]  (Conv2dSubsampling4: x.transpose(1, 2).view(b, t, c*f))
__global__ void k_tcf(const float* in, int B, int T, int F, int C, float* out) {
  const long long total = (long long)B * T * C * F;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int f = (int)(e % F);
    const int c = (int)((e / F) % C);
    const long long bt = e / ((long long)F * C);
    const int t = (int)(bt % T);
    const int b = (int)(bt / T);
    out[e] = in[((long long)b * T * F + (long long)t * F + f) * C + c];
  }
}

// Causal strided conv1d im2col with carried frames (CNNSubsampling, models/adapter.py:162-170):
// seq_b = [cache_b (KC rows) ; x_b (T rows)] of width D; out row (b, t) col c*K + j = seq_b[S*t + j][c].
__global__ void k_im2col_conv1d(const float* cache, const int* slots, const float* x, int B, int KC, int T, int D,
                                int K, int S, float* out, int ldo) {
  const int L = KC + T;
  const int To = (L - K) / S + 1;
  const long long total = (long long)B * To * ldo;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const long long row = e / ldo;
    const int col = (int)(e % ldo);
    float v = 0.f;
    if (col < D * K) {
      const int c = col / K, j = col % K;
      const int b = (int)(row / To), t = (int)(row % To);
      const int s = S * t + j;
      const long long cb = slots ? slots[b] : b;
      v = s < KC ? (cache ? cache[(cb * KC + s) * D + c] : 0.f) : x[((long long)b * T + s - KC) * D + c];
    }
    out[e] = v;
  }
}

// cache_b <- last KC rows of x_b (in place in the slot pool; requires T >= KC so no old row is read)
__global__ void k_conv_cache_update(float* cache, const int* slots, const float* x, int B, int KC, int T, int D) {
  const long long total = (long long)B * KC * D;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(e % D);
    const int r = (int)((e / D) % KC);
    const int b = (int)(e / ((long long)KC * D));
    const long long cb = slots ? slots[b] : b;
    cache[(cb * KC + r) * D + c] = x[((long long)b * T + T - KC + r) * D + c];
  }
}

// Dialog-state head (models/audioLLM.py:486-493,521-524): logits = W h + b over 4 classes for the
// selected row of each sequence; softmax over classes 0..2; writes probs[s][0..2].
// One pass over the row for all three logits, 1024 threads, every load of a 4096-wide slab issued before its use
// (the row and the three weight rows are cold: a dependent load chain per element was the launch's whole time).
__global__ __launch_bounds__(1024) void k_state_head(const float* h, int ldh, const int* rows, const float* W,
                                                     const float* bias, int D, float* probs) {
  __shared__ float red[3][16];
  const float* x = h + (size_t)rows[blockIdx.x] * ldh;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f;
  for (int base = 0; base < D; base += 4096) {
    float xv[4], w0[4], w1[4], w2[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int i = base + k * 1024 + (int)threadIdx.x;
      const bool ok = i < D;
      xv[k] = ok ? x[i] : 0.f;
      w0[k] = ok ? W[i] : 0.f;
      w1[k] = ok ? W[(size_t)D + i] : 0.f;
      w2[k] = ok ? W[2 * (size_t)D + i] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      a0 += xv[k] * w0[k];
      a1 += xv[k] * w1[k];
      a2 += xv[k] * w2[k];
    }
  }
  a0 = wave_sum(a0);
  a1 = wave_sum(a1);
  a2 = wave_sum(a2);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][w] = a0;
    red[1][w] = a1;
    red[2][w] = a2;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float lg[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      float t = bias[c];
#pragma unroll
      for (int j = 0; j < 16; ++j) t += red[c][j];
      lg[c] = t;
    }
    const float m = fmaxf(lg[0], fmaxf(lg[1], lg[2]));
    const float e0 = expf(lg[0] - m), e1 = expf(lg[1] - m), e2 = expf(lg[2] - m);
    const float z = e0 + e1 + e2;
    probs[blockIdx.x * 3 + 0] = e0 / z;
    probs[blockIdx.x * 3 + 1] = e1 / z;
    probs[blockIdx.x * 3 + 2] = e2 / z;
  }
}

__global__ void k_scale_rows(float* x, long long n, float s) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    x[i] *= s;
}

inline int grid_for(long long n, int bs = 256) {
  long long g = (n + bs - 1) / bs;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace

__global__ void k_record_ids(const int* ids, int B, int* dst, int ld, const int* row) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < B) dst[(size_t)row[0] * ld + b] = ids[b];
}

extern "C" {

int fo_fill_hash(void* out, int out_bf16, long long n, unsigned long long key, float center, float scale,
                 hipStream_t s) {
  FO_REQUIRE(out && n >= 0, "fo_fill_hash: bad args");
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_fill_hash, dim3(grid_for(n)), dim3(256), 0, s, out, out_bf16, n, (uint64_t)key, center, scale);
  return fo::check_launch("fo_fill_hash");
}

int fo_rmsnorm(const float* x, int ldx, int M, int D, const float* w, float eps, float* out, int ldo, int round_fp16,
               hipStream_t s) {
  FO_REQUIRE(M > 0 && D > 0 && (D & 3) == 0 && (ldx & 3) == 0 && (ldo & 3) == 0, "fo_rmsnorm: bad shape");
  hipLaunchKernelGGL(k_rmsnorm, dim3(M), dim3(256), 0, s, x, ldx, D, w, eps, out, ldo, round_fp16);
  return fo::check_launch("fo_rmsnorm");
}

int fo_layernorm(const float* x, int ldx, int M, int D, const float* w, const float* b, float eps, float* out, int ldo,
                 int act, hipStream_t s) {
  FO_REQUIRE(M > 0 && D > 0, "fo_layernorm: bad shape");
  FO_REQUIRE(act == FO_ACT_NONE || act == FO_ACT_RELU || act == FO_ACT_GELU, "fo_layernorm: act %d", act);
  hipLaunchKernelGGL(k_layernorm, dim3(M), dim3(256), 0, s, x, ldx, D, w, b, eps, out, ldo, act);
  return fo::check_launch("fo_layernorm");
}

int fo_gather_rows(const void* table, int table_bf16, long long ld_tab, const int* idx, int M, int D, float* out,
                   int ldo, const int* out_rows, int round_fp16, hipStream_t s) {
  FO_REQUIRE(M >= 0 && D > 0, "fo_gather_rows: bad shape");
  if (M == 0) return 0;
  hipLaunchKernelGGL(k_gather_rows, dim3(M), dim3(256), 0, s, table, table_bf16, ld_tab, idx, M, D, out, ldo, out_rows,
                     round_fp16);
  return fo::check_launch("fo_gather_rows");
}

int fo_im2col_3x3s2(const float* in, int B, int C, int H, int W, long long sb, long long sc, long long sh,
                    long long sw, const float* mean, const float* istd, float* out, int ldo, hipStream_t s) {
  FO_REQUIRE(H >= 3 && W >= 3 && ldo >= C * 9, "fo_im2col_3x3s2: bad shape");
  const long long n = (long long)B * ((H - 3) / 2 + 1) * ((W - 3) / 2 + 1) * ldo;
  hipLaunchKernelGGL(k_im2col_3x3s2, dim3(grid_for(n)), dim3(256), 0, s, in, B, C, H, W, sb, sc, sh, sw, mean, istd,
                     out, ldo);
  return fo::check_launch("fo_im2col_3x3s2");
}

int fo_tcf_permute(const float* in, int B, int T, int F, int C, float* out, hipStream_t s) {
  const long long n = (long long)B * T * F * C;
  hipLaunchKernelGGL(k_tcf, dim3(grid_for(n)), dim3(256), 0, s, in, B, T, F, C, out);
  return fo::check_launch("fo_tcf_permute");
}

int fo_im2col_conv1d(const float* cache, const int* slots, const float* x, int B, int KC, int T, int D, int K, int S,
                     float* out, int ldo, hipStream_t s) {
  FO_REQUIRE(KC + T >= K && ldo >= D * K, "fo_im2col_conv1d: bad shape");
  const int To = (KC + T - K) / S + 1;
  const long long n = (long long)B * To * ldo;
  hipLaunchKernelGGL(k_im2col_conv1d, dim3(grid_for(n)), dim3(256), 0, s, cache, slots, x, B, KC, T, D, K, S, out,
                     ldo);
  return fo::check_launch("fo_im2col_conv1d");
}

int fo_conv_cache_update(float* cache, const int* slots, const float* x, int B, int KC, int T, int D, hipStream_t s) {
  FO_REQUIRE(T >= KC, "fo_conv_cache_update: chunk T=%d shorter than the carried context %d", T, KC);
  const long long n = (long long)B * KC * D;
  hipLaunchKernelGGL(k_conv_cache_update, dim3(grid_for(n)), dim3(256), 0, s, cache, slots, x, B, KC, T, D);
  return fo::check_launch("fo_conv_cache_update");
}

int fo_state_head(const float* h, int ldh, const int* rows, int S, const float* W, const float* bias, int D,
                  float* probs, hipStream_t s) {
  FO_REQUIRE(S > 0, "fo_state_head: no rows");
  hipLaunchKernelGGL(k_state_head, dim3(S), dim3(1024), 0, s, h, ldh, rows, W, bias, D, probs);
  return fo::check_launch("fo_state_head");
}

int fo_scale(float* x, long long n, float sc, hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_scale_rows, dim3(grid_for(n)), dim3(256), 0, s, x, n, sc);
  return fo::check_launch("fo_scale");
}

// dst[row[0]][b] = ids[b]: per-step token history written by the decode graph (row index read on the
// device so one captured graph serves every step; dst may be host-mapped pinned memory).
int fo_record_ids(const int* ids, int B, int* dst, int ld, const int* row, hipStream_t s) {
  FO_REQUIRE(B > 0 && ld >= B, "fo_record_ids: bad shape");
  hipLaunchKernelGGL(k_record_ids, dim3((B + 63) / 64), dim3(64), 0, s, ids, B, dst, ld, row);
  return fo::check_launch("fo_record_ids");
}

}  // extern "C"
