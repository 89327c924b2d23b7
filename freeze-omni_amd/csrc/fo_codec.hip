// TiCodec generator (vocoder) kernels and the streaming silence cut.
//
// Reference: VQVAE.forward -> Quantizer.embed/embed_gst -> Generator.forward
// (models/decoder/ticodec/vqvae.py:37-42, models/decoder/ticodec/models.py:169-242,661-715), weight norm
// removed at load (models/decoder/llm2tts.py:28); emission rule find_min_sum_index
// (models/decoder/llm2tts.py:70-112).
// Activations are fp32 [B][C][T] (channel-major, as the reference's conv layout), weights bf16.
// conv1d: LDS-tiled direct convolution, 64 output channels x 64 samples per workgroup, 4x4
// register blocking; leaky-ReLU on the input, bias / residual / tanh fused on the output.
#include "fo_common.h"

namespace {

constexpr int CO_T = 64, T_T = 64, CI_T = 8, KMAX = 11, DMAX = 5;
constexpr int XW = T_T + DMAX * (KMAX - 1);

__global__ __launch_bounds__(256) void k_conv1d(const float* x, int Cin, int Tin, const bf16_t* w, const float* bias,
                                                int Cout, int K, int dil, int pad, float pre_slope, int pre_act,
                                                float* out, int Tout, int residual, int post_tanh) {
  __shared__ float xs[CI_T][XW];
  __shared__ float wsm[CO_T][CI_T][KMAX];
  const int b = blockIdx.z;
  const int co0 = blockIdx.y * CO_T, t0 = blockIdx.x * T_T;
  const int tc = (threadIdx.x / 16) * 4, tt = (threadIdx.x % 16) * 4;
  const int span = T_T + dil * (K - 1);
  const float* xb = x + (size_t)b * Cin * Tin;
  float acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = 0.f;
  for (int ci0 = 0; ci0 < Cin; ci0 += CI_T) {
    for (int e = threadIdx.x; e < CI_T * span; e += 256) {
      const int ci = e / span, q = e % span;
      const int ti = t0 - pad + q;
      float v = 0.f;
      if (ci0 + ci < Cin && ti >= 0 && ti < Tin) {
        v = xb[(size_t)(ci0 + ci) * Tin + ti];
        if (pre_act && v < 0.f) v *= pre_slope;
      }
      xs[ci][q] = v;
    }
    for (int e = threadIdx.x; e < CO_T * CI_T * K; e += 256) {
      const int co = e / (CI_T * K), r = e % (CI_T * K), ci = r / K, j = r % K;
      float v = 0.f;
      if (co0 + co < Cout && ci0 + ci < Cin) v = bf2f(w[((size_t)(co0 + co) * Cin + ci0 + ci) * K + j]);
      wsm[co][ci][j] = v;
    }
    __syncthreads();
    for (int ci = 0; ci < CI_T; ++ci) {
      for (int j = 0; j < K; ++j) {
        float wv[4], xv[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) wv[i] = wsm[tc + i][ci][j];
#pragma unroll
        for (int i = 0; i < 4; ++i) xv[i] = xs[ci][tt + i + j * dil];
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
          for (int c = 0; c < 4; ++c) acc[a][c] += wv[a] * xv[c];
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const int co = co0 + tc + a;
    if (co >= Cout) continue;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int t = t0 + tt + c;
      if (t >= Tout) continue;
      float v = acc[a][c] + (bias ? bias[co] : 0.f);
      const size_t o = ((size_t)b * Cout + co) * Tout + t;
      if (residual) v += out[o];
      if (post_tanh) v = tanhf(v);
      out[o] = v;
    }
  }
}

// torch ConvTranspose1d (weight [Cin][Cout][K]) with leaky-ReLU on the input.
__global__ void k_convT1d(const float* x, int Cin, int Tin, const bf16_t* w, const float* bias, int Cout, int K,
                          int stride, int pad, float pre_slope, float* out, int Tout) {
  const int b = blockIdx.z;
  const int co = blockIdx.y;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= Tout) return;
  const float* xb = x + (size_t)b * Cin * Tin;
  float acc = bias ? bias[co] : 0.f;
  const int tp = t + pad;
  int j = tp % stride;
  for (; j < K; j += stride) {
    const int ti = (tp - j) / stride;
    if (ti < 0) break;
    if (ti >= Tin) continue;
    for (int ci = 0; ci < Cin; ++ci) {
      float v = xb[(size_t)ci * Tin + ti];
      if (v < 0.f) v *= pre_slope;
      acc += v * bf2f(w[((size_t)ci * Cout + co) * K + j]);
    }
  }
  out[((size_t)b * Cout + co) * Tout + t] = acc;
}

// ids outside [0, n_codes) (the decoder's BOS/SOS/PAD specials) embed as zeros instead of reading
// out of bounds; the reference would raise IndexError there (nn.Embedding).
__global__ void k_codec_embed(const bf16_t* table, int E, int n_codes, const int* ids, int B, int T, float* out) {
  const long long total = (long long)B * E * T;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int t = (int)(e % T);
    const int c = (int)((e / T) % E);
    const int b = (int)(e / ((long long)T * E));
    const int id = ids[b * T + t];
    out[e] = (id >= 0 && id < n_codes) ? bf2f(table[(size_t)id * E + c]) : 0.f;
  }
}

// y = (y + x) or y = y * s + g[c]  (resblock sum, 1/num_kernels, global feature add)
__global__ void k_axpy(float* y, const float* x, long long n) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    y[i] += x[i];
}
__global__ void k_scale_add_channel(float* y, int B, int C, int T, float s, const float* g) {
  const long long total = (long long)B * C * T;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    float v = y[i] * s;
    if (g) {
      const int c = (int)((i / T) % C);
      const int b = (int)(i / ((long long)T * C));
      v += g[b * C + c];
    }
    y[i] = v;
  }
}

// find_min_sum_index: window sums of |x| over N samples starting at mid - N/2; argmin (first);
// then argmin |x| inside [s0, min(L, m + N + s0)).  res[0] = min window sum, res[1] = cut index.
// One work group per row (blockIdx.x: row x + blockIdx.x * ld, result res + 2 * blockIdx.x): the rows of a
// vocoder call in one launch.  A row that fits (STAGE: L <= dynamic LDS floats) is staged into LDS once, so
// the window sums' partial-chunk loops read LDS instead of issuing dependent global loads; the arithmetic
// (double prefix sums, P(b) - P(a)) is the same either way, so the result is too.
template <bool STAGE>
__global__ __launch_bounds__(1024) void k_silence_cut(const float* xg, long long ld, int L, int N, float* res) {
  extern __shared__ float xs_dyn[];
  __shared__ double cs[1025];
  __shared__ float bv[1024];
  __shared__ int bi[1024];
  xg += (size_t)blockIdx.x * ld;
  res += 2 * blockIdx.x;
  const float* x = xg;
  if constexpr (STAGE) {
    for (int i = threadIdx.x; i < L; i += 1024) xs_dyn[i] = xg[i];
    __syncthreads();
    x = xs_dyn;
  }
  const int mid = L / 2, start = mid - N / 2;
  const int nw = L - N + 1 - start;  // window count from `start`
  // prefix sums of |x| in double, 1024 threads over chunks
  const int per = (L + 1023) / 1024;
  double loc = 0.0;
  for (int i = threadIdx.x * per; i < min(L, (threadIdx.x + 1) * per); ++i) loc += fabs((double)x[i]);
  cs[threadIdx.x + 1] = loc;
  if (threadIdx.x == 0) cs[0] = 0.0;
  __syncthreads();
  // inclusive scan of the 1024 chunk sums (log-step in LDS; a serial thread-0 loop cost ~40 us)
  for (int off = 1; off < 1024; off <<= 1) {
    const double v = threadIdx.x >= off ? cs[threadIdx.x + 1 - off] : 0.0;
    __syncthreads();
    cs[threadIdx.x + 1] += v;
    __syncthreads();
  }
  // window sum at w: S(w) = P(start + w + N) - P(start + w), P(k) = sum_{i<k} |x_i|
  auto P = [&](int k) -> double {
    const int c = k / per;
    double v = cs[min(c, 1024)];
    for (int i = c * per; i < k; ++i) v += fabs((double)x[i]);
    return v;
  };
  float best = INFINITY;
  int besti = 0x7fffffff;
  for (int w = threadIdx.x; w < nw; w += 1024) {
    const float sw = (float)(P(start + w + N) - P(start + w));
    if (sw < best) {
      best = sw;
      besti = w;
    }
  }
  bv[threadIdx.x] = best;
  bi[threadIdx.x] = besti;
  __syncthreads();
  for (int o = 512; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      const float v2 = bv[threadIdx.x + o];
      const int i2 = bi[threadIdx.x + o];
      if (v2 < bv[threadIdx.x] || (v2 == bv[threadIdx.x] && i2 < bi[threadIdx.x])) {
        bv[threadIdx.x] = v2;
        bi[threadIdx.x] = i2;
      }
    }
    __syncthreads();
  }
  const float minsum = bv[0];
  const int mi = bi[0];
  const int s0 = max(0, mi + start);
  const int e0 = min(L, mi + N + s0);  // the reference adds the updated start (llm2tts.py:98-99)
  __syncthreads();
  best = INFINITY;
  besti = 0x7fffffff;
  for (int i = s0 + threadIdx.x; i < e0; i += 1024) {
    const float a = fabsf(x[i]);
    if (a < best) {
      best = a;
      besti = i;
    }
  }
  bv[threadIdx.x] = best;
  bi[threadIdx.x] = besti;
  __syncthreads();
  for (int o = 512; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      const float v2 = bv[threadIdx.x + o];
      const int i2 = bi[threadIdx.x + o];
      if (v2 < bv[threadIdx.x] || (v2 == bv[threadIdx.x] && i2 < bi[threadIdx.x])) {
        bv[threadIdx.x] = v2;
        bi[threadIdx.x] = i2;
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    res[0] = minsum;
    res[1] = (float)bi[0];
  }
}
constexpr int SC_STATIC_LDS = 1025 * 8 + 1024 * 4 * 2;
constexpr int SC_MAX_STAGE = (160 * 1024 - SC_STATIC_LDS) / 4;  // floats of a row staged in LDS

inline int grid_for(long long n) {
  long long g = (n + 255) / 256;
  return (int)(g > 8192 ? 8192 : (g < 1 ? 1 : g));
}

}  // namespace

extern "C" {

int fo_conv1d(const float* x, int B, int Cin, int Tin, const void* w, const float* bias, int Cout, int K, int dil,
              int pad, int pre_leaky, float slope, float* out, int residual, int post_tanh, hipStream_t s) {
  FO_REQUIRE(K <= KMAX && dil <= DMAX, "fo_conv1d: K=%d dil=%d exceed tile limits", K, dil);
  const int Tout = Tin + 2 * pad - dil * (K - 1);
  FO_REQUIRE(Tout > 0, "fo_conv1d: empty output");
  dim3 grid((Tout + T_T - 1) / T_T, (Cout + CO_T - 1) / CO_T, B);
  hipLaunchKernelGGL(k_conv1d, grid, dim3(256), 0, s, x, Cin, Tin, (const bf16_t*)w, bias, Cout, K, dil, pad, slope,
                     pre_leaky, out, Tout, residual, post_tanh);
  return fo::check_launch("fo_conv1d");
}

int fo_conv_transpose1d(const float* x, int B, int Cin, int Tin, const void* w, const float* bias, int Cout, int K,
                        int stride, int pad, float slope, float* out, hipStream_t s) {
  const int Tout = (Tin - 1) * stride - 2 * pad + K;
  FO_REQUIRE(Tout > 0, "fo_conv_transpose1d: empty output");
  dim3 grid((Tout + 127) / 128, Cout, B);
  hipLaunchKernelGGL(k_convT1d, grid, dim3(128), 0, s, x, Cin, Tin, (const bf16_t*)w, bias, Cout, K, stride, pad,
                     slope, out, Tout);
  return fo::check_launch("fo_conv_transpose1d");
}

int fo_codec_embed(const void* table, int E, int n_codes, const int* ids, int B, int T, float* out, hipStream_t s) {
  const long long n = (long long)B * E * T;
  hipLaunchKernelGGL(k_codec_embed, dim3(grid_for(n)), dim3(256), 0, s, (const bf16_t*)table, E, n_codes, ids, B, T,
                     out);
  return fo::check_launch("fo_codec_embed");
}

int fo_axpy(float* y, const float* x, long long n, hipStream_t s) {
  hipLaunchKernelGGL(k_axpy, dim3(grid_for(n)), dim3(256), 0, s, y, x, n);
  return fo::check_launch("fo_axpy");
}

int fo_scale_add_channel(float* y, int B, int C, int T, float sc, const float* g, hipStream_t s) {
  const long long n = (long long)B * C * T;
  hipLaunchKernelGGL(k_scale_add_channel, dim3(grid_for(n)), dim3(256), 0, s, y, B, C, T, sc, g);
  return fo::check_launch("fo_scale_add_channel");
}

int fo_silence_cut_rows(const float* x, long long ld, int rows, int L, int N, float* res, hipStream_t s) {
  FO_REQUIRE(rows >= 1 && L >= N && L / 2 - N / 2 >= 0 && (rows == 1 || ld >= L),
             "fo_silence_cut_rows: rows=%d L=%d N=%d ld=%lld", rows, L, N, ld);
  if (L <= SC_MAX_STAGE)
    hipLaunchKernelGGL((k_silence_cut<true>), dim3(rows), dim3(1024), (size_t)L * sizeof(float), s, x, ld, L, N, res);
  else
    hipLaunchKernelGGL((k_silence_cut<false>), dim3(rows), dim3(1024), 0, s, x, ld, L, N, res);
  return fo::check_launch("fo_silence_cut");
}

int fo_silence_cut(const float* x, int L, int N, float* res, hipStream_t s) {
  return fo_silence_cut_rows(x, 0, 1, L, N, res, s);
}

}  // extern "C"
