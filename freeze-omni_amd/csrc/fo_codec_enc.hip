// TiCodec encoder (VQVAE.encode, models/decoder/ticodec/vqvae.py:44-57): Encoder convs
// (models/decoder/ticodec/models.py:429-522), GroupNorm, GlobalTokenEncoder head (models.py:22-57)
// and the nearest-codebook search of Quantizer_module (models.py:531-537).  Channel-first fp32
// activations [B][C][T]; fp32 weights (weight norm removed / folded at load).  Produces voice and
// global tokens; off the speech-to-speech hot path, so the convs are direct (VALU) kernels.
#include "fo_common.h"

namespace {

// out[b][co][t] (+)= bias[co] + sum_{ci,k} w[co][ci][k] * act(x[b][ci][t*stride + k*dil - pad])
__global__ __launch_bounds__(128) void k_conv1d_ex(const float* x, int Cin, int Tin, const float* w,
                                                   const float* bias, int Cout, int K, int stride, int dil,
                                                   int pad, int pre_act, float slope, float* out, int Tout,
                                                   int residual) {
  const int b = blockIdx.z, co = blockIdx.y;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= Tout) return;
  const float* xb = x + (size_t)b * Cin * Tin;
  const float* wr = w + (size_t)co * Cin * K;
  const int t0 = t * stride - pad;
  float acc = 0.f;
  for (int ci = 0; ci < Cin; ++ci) {
    const float* xc = xb + (size_t)ci * Tin;
    const float* wc = wr + (size_t)ci * K;
    for (int k = 0; k < K; ++k) {
      const int ti = t0 + k * dil;
      if (ti < 0 || ti >= Tin) continue;
      float v = xc[ti];
      if (pre_act && v < 0.f) v *= slope;
      acc = fmaf(wc[k], v, acc);
    }
  }
  if (bias) acc += bias[co];
  float* o = out + ((size_t)b * Cout + co) * Tout + t;
  *o = residual ? *o + acc : acc;
}

// GroupNorm (torch.nn.GroupNorm, affine): one block per (group, batch); in place allowed
__global__ __launch_bounds__(256) void k_group_norm(const float* x, int C, int T, int G, const float* w,
                                                    const float* bias, float eps, float scale, float* out) {
  __shared__ float red[256];
  const int g = blockIdx.x, b = blockIdx.y;
  const int cg = C / G;
  const size_t base = ((size_t)b * C + (size_t)g * cg) * T;
  const int n = cg * T;
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s += x[base + i];
  const float mean = block_sum<4>(s, red) / (float)n;
  float v = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const float d = x[base + i] - mean;
    v += d * d;
  }
  const float rstd = rsqrtf(block_sum<4>(v, red) / (float)n + eps);
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int c = g * cg + i / T;
    out[base + i] = ((x[base + i] - mean) * rstd * w[c] + bias[c]) * scale;
  }
}

// GlobalTokenEncoder head: leaky 0.1 of the last conv -> mean over time -> Linear(C, C) -> leaky 0.1 ->
// BatchNorm1d (eval).
// One block per batch row, one thread per channel (C <= 1024).
__global__ __launch_bounds__(1024) void k_gte_head(const float* x, int C, int T, const float* lw, const float* lb,
                                                   const float* rm, const float* rv, const float* bw,
                                                   const float* bb, float bn_eps, float* out) {
  __shared__ float v[1024];
  const int b = blockIdx.x, c = threadIdx.x;
  if (c < C) {
    const float* xr = x + ((size_t)b * C + c) * T;
    float s = 0.f;
    for (int t = 0; t < T; ++t) s += xr[t] < 0.f ? xr[t] * 0.1f : xr[t];   // the last conv's leaky 0.1
    v[c] = s / (float)T;
  }
  __syncthreads();
  if (c < C) {
    float y = lb[c];
    const float* wr = lw + (size_t)c * C;
    for (int j = 0; j < C; ++j) y = fmaf(wr[j], v[j], y);
    y = y < 0.f ? y * 0.1f : y;
    out[(size_t)b * C + c] = (y - rm[c]) * rsqrtf(rv[c] + bn_eps) * bw[c] + bb[c];
  }
}

// Quantizer_module.forward for the rows (b, t) of channels [ch0, ch0 + D) of x [B][Ctot][T]:
// d_j = (|x|^2 + |e_j|^2) - 2 x.e_j, argmin (first index on ties) -> ids[(b*T + t) * ids_ld + ids_col];
// with `residual`, x -= x + (e - x) in place (the straight-through quantized value the reference
// subtracts from its residual, models.py:588-645).  One block per row; x staged in LDS.
__global__ __launch_bounds__(256) void k_vq_nearest(float* x, int Ctot, int T, int ch0, int D, const float* E,
                                                    int n_codes, int* ids, int ids_ld, int ids_col, int residual) {
  extern __shared__ float xs[];
  __shared__ float bd[256];
  __shared__ int bi[256];
  __shared__ float red[256];
  const int row = blockIdx.x;
  const int b = row / T, t = row % T;
  float* xr = x + ((size_t)b * Ctot + ch0) * T + t;
  float xx = 0.f;
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    const float v = xr[(size_t)d * T];
    xs[d] = v;
    xx += v * v;
  }
  xx = block_sum<4>(xx, red);
  float best = INFINITY;
  int besti = 0x7fffffff;
  for (int j = threadIdx.x; j < n_codes; j += blockDim.x) {
    const float* e = E + (size_t)j * D;
    float ee = 0.f, xe = 0.f;
    for (int d = 0; d < D; ++d) {
      ee = fmaf(e[d], e[d], ee);
      xe = fmaf(xs[d], e[d], xe);
    }
    const float dist = (xx + ee) - 2.f * xe;
    if (dist < best || (dist == best && j < besti)) {
      best = dist;
      besti = j;
    }
  }
  bd[threadIdx.x] = best;
  bi[threadIdx.x] = besti;
  __syncthreads();
  for (int o = blockDim.x / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      const float v2 = bd[threadIdx.x + o];
      const int i2 = bi[threadIdx.x + o];
      if (v2 < bd[threadIdx.x] || (v2 == bd[threadIdx.x] && i2 < bi[threadIdx.x])) {
        bd[threadIdx.x] = v2;
        bi[threadIdx.x] = i2;
      }
    }
    __syncthreads();
  }
  const int pick = bi[0];
  if (threadIdx.x == 0) ids[(size_t)row * ids_ld + ids_col] = pick;
  if (residual) {
    const float* e = E + (size_t)pick * D;
    for (int d = threadIdx.x; d < D; d += blockDim.x) {
      const float v = xs[d];
      xr[(size_t)d * T] = v - (v + (e[d] - v));
    }
  }
}

}  // namespace

extern "C" {

int fo_conv1d_ex(const float* x, int B, int Cin, int Tin, const float* w, const float* bias, int Cout, int K,
                 int stride, int dil, int pad, int pre_act, float slope, float* out, int residual, hipStream_t s) {
  FO_REQUIRE(B > 0 && Cin > 0 && Cout > 0 && K > 0 && stride > 0 && dil > 0 && pad >= 0,
             "fo_conv1d_ex: bad shape");
  const int Tout = (Tin + 2 * pad - dil * (K - 1) - 1) / stride + 1;
  FO_REQUIRE(Tout > 0, "fo_conv1d_ex: empty output (Tin=%d K=%d stride=%d)", Tin, K, stride);
  hipLaunchKernelGGL(k_conv1d_ex, dim3((Tout + 127) / 128, Cout, B), dim3(128), 0, s, x, Cin, Tin, w, bias, Cout,
                     K, stride, dil, pad, pre_act, slope, out, Tout, residual);
  return fo::check_launch("fo_conv1d_ex");
}

int fo_group_norm(const float* x, int B, int C, int T, int G, const float* w, const float* bias, float eps,
                  float scale, float* out, hipStream_t s) {
  FO_REQUIRE(B > 0 && G > 0 && C % G == 0 && T > 0, "fo_group_norm: C=%d not divisible by G=%d", C, G);
  hipLaunchKernelGGL(k_group_norm, dim3(G, B), dim3(256), 0, s, x, C, T, G, w, bias, eps, scale, out);
  return fo::check_launch("fo_group_norm");
}

int fo_gte_head(const float* x, int B, int C, int T, const float* lw, const float* lb, const float* rm,
                const float* rv, const float* bw, const float* bb, float bn_eps, float* out, hipStream_t s) {
  FO_REQUIRE(B > 0 && C > 0 && C <= 1024 && T > 0, "fo_gte_head: C=%d must be in 1..1024", C);
  hipLaunchKernelGGL(k_gte_head, dim3(B), dim3(((C + 63) / 64) * 64), 0, s, x, C, T, lw, lb, rm, rv, bw, bb, bn_eps,
                     out);
  return fo::check_launch("fo_gte_head");
}

int fo_vq_nearest(float* x, int B, int Ctot, int T, int ch0, int D, const float* codebook, int n_codes, int* ids,
                  int ids_ld, int ids_col, int residual, hipStream_t s) {
  FO_REQUIRE(B > 0 && T > 0 && D > 0 && ch0 >= 0 && ch0 + D <= Ctot && n_codes > 0 && D <= 8192,
             "fo_vq_nearest: bad shape");
  hipLaunchKernelGGL(k_vq_nearest, dim3(B * T), dim3(256), D * sizeof(float), s, x, Ctot, T, ch0, D, codebook,
                     n_codes, ids, ids_ld, ids_col, residual);
  return fo::check_launch("fo_vq_nearest");
}

}  // extern "C"
