// TiCodec generator convolutions on the matrix cores (channel-last activations).
//
// Reference: Generator.forward (models/decoder/ticodec/models.py:211-242) with ResBlock1
// (:59-110): conv_pre, per stage leaky -> ConvTranspose1d -> mean of dilated resblocks, conv_post.
// Every Conv1d there is an implicit GEMM  Y[co][t] = sum_{j,ci} W[co][ci][j] * x'[t + j*dil - pad][ci]
// with K = taps x Cin.  Activations live as [B][T][C] (channels contiguous) so that
//  * a workgroup stages a time window x all channels of one Cin chunk into LDS with 16-B loads,
//  * one MFMA B-fragment (8 consecutive K = 8 channels of one tap at one time step) is two 16-B LDS
//    reads, and an accumulator lane's 4 rows are 4 consecutive output channels (one 16-B store).
// Weights are packed once at load into A-fragment order [Cout/16][k-steps][64 lanes][8 bf16] with
// K ordered (Cin chunk, tap, channel) to match the staging.  fp32 activations are split into bf16
// hi + lo (two MFMAs per step), so results keep ~fp32 accuracy against bf16 weights.
// ConvTranspose1d (stride u) is u polyphase convolutions: output phase r only meets taps
// j = j0(r) + u*m, i.e. a 2-tap stride-1 conv with its own packed weights writing every u-th step.
#include "fo_common.h"

namespace {

constexpr int HALO = 56;  // >= dil * (K - 1) for K <= 11, dil <= 5

struct ConvArgs {
  const float* x;      // [B][Tin][Cin]
  const bf16_t* wp;    // packed A fragments
  const float* bias;   // [Cout] or null
  float* out;          // [B][Tout_total][Cout]
  int Cin, Tin, Cout, K, dil, pad;
  int Tq;              // outputs computed (per batch row)
  int ostride, ooff;   // output time index = q * ostride + ooff
  int Tout_total;      // time length of `out`
  int nks_c;           // k-steps per Cin chunk
  int pre_act;         // leaky ReLU on the input
  float slope;
  int residual;        // out += conv
};

template <int MTW, int NTW, int CK>
__global__ __launch_bounds__(256) void k_conv_cl(ConvArgs a) {
  constexpr int TW = 64 * NTW;     // time steps per workgroup (4 waves x 16*NTW)
  constexpr int ROWS = TW + HALO;
  constexpr int LP = CK + 4;       // padded row: 16 lanes of different rows hit distinct banks
  __shared__ float xs[ROWS][LP];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int t0 = blockIdx.x * TW;
  const int ct0 = blockIdx.y * MTW;  // first 16-channel output tile
  const int b = blockIdx.z;
  const int nchunks = a.Cin / CK;
  const int nks = nchunks * a.nks_c;
  const int span = TW + a.dil * (a.K - 1);
  const float* xb = a.x + (size_t)b * a.Tin * a.Cin;

  f32x4 acc[MTW][NTW];
#pragma unroll
  for (int m = 0; m < MTW; ++m)
#pragma unroll
    for (int n = 0; n < NTW; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  const bf16x8* wpl = reinterpret_cast<const bf16x8*>(a.wp) + lane;
  const int tl = wave * 16 * NTW + (lane & 15);  // this lane's time row (tile n adds 16 n)
  const int kq = 8 * (lane >> 4);                 // this lane's 8-wide K slice inside a step

  for (int c = 0; c < nchunks; ++c) {
    __syncthreads();
    for (int e = threadIdx.x; e < span * (CK / 4); e += 256) {
      const int row = e / (CK / 4), c4 = e % (CK / 4);
      const int ti = t0 - a.pad + row;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (ti >= 0 && ti < a.Tin) {
        v = *reinterpret_cast<const float4*>(xb + (size_t)ti * a.Cin + c * CK + c4 * 4);
        if (a.pre_act) {
          v.x = v.x < 0.f ? v.x * a.slope : v.x;
          v.y = v.y < 0.f ? v.y * a.slope : v.y;
          v.z = v.z < 0.f ? v.z * a.slope : v.z;
          v.w = v.w < 0.f ? v.w * a.slope : v.w;
        }
      }
      *reinterpret_cast<float4*>(&xs[row][c4 * 4]) = v;
    }
    __syncthreads();
    for (int s = 0; s < a.nks_c; ++s) {
      const int ks = c * a.nks_c + s;
      bf16x8 av[MTW];
#pragma unroll
      for (int m = 0; m < MTW; ++m) av[m] = wpl[((size_t)(ct0 + m) * nks + ks) * 64];
      const int kk = s * 32 + kq;
      int j = kk / CK;
      const int cil = kk - j * CK;
      if (j > a.K - 1) j = a.K - 1;  // padded K: the packed weights are zero there
      const int rb = tl + j * a.dil;
#pragma unroll
      for (int n = 0; n < NTW; ++n) {
        const float4 p0 = *reinterpret_cast<const float4*>(&xs[rb + 16 * n][cil]);
        const float4 p1 = *reinterpret_cast<const float4*>(&xs[rb + 16 * n][cil + 4]);
        const float f[8] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w};
        bf16x8 hi, lo;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const __bf16 h = (__bf16)f[i];
          hi[i] = h;
          lo[i] = (__bf16)(f[i] - (float)h);
        }
#pragma unroll
        for (int m = 0; m < MTW; ++m) {
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[m], hi, acc[m][n], 0, 0, 0);
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[m], lo, acc[m][n], 0, 0, 0);
        }
      }
    }
  }
  // C layout: row (output channel) = 4*(lane>>4) + i, column (time) = lane & 15
#pragma unroll
  for (int n = 0; n < NTW; ++n) {
    const int q = t0 + tl + 16 * n;
    if (q >= a.Tq) continue;
    const int t = q * a.ostride + a.ooff;
#pragma unroll
    for (int m = 0; m < MTW; ++m) {
      const int co = (ct0 + m) * 16 + kq / 2;  // 4*(lane>>4)
      float4 v = make_float4(acc[m][n][0], acc[m][n][1], acc[m][n][2], acc[m][n][3]);
      if (a.bias) {
        const float4 bb = *reinterpret_cast<const float4*>(a.bias + co);
        v.x += bb.x; v.y += bb.y; v.z += bb.z; v.w += bb.w;
      }
      float4* o = reinterpret_cast<float4*>(a.out + ((size_t)b * a.Tout_total + t) * a.Cout + co);
      if (a.residual) {
        const float4 r = *o;
        v.x += r.x; v.y += r.y; v.z += r.z; v.w += r.w;
      }
      *o = v;
    }
  }
}

// Pack W (conv: [Cout][Cin][K]; transposed conv: [Cin][Cout][Ktot], taps j0 + u*m of one phase,
// reversed) into A fragments with K ordered (chunk of CK channels, tap, channel), each chunk
// padded to whole 32-wide k-steps.
__global__ void k_pack_conv(const void* W, int src_bf16, int Cout, int Cin, int K, int CK, int nks_c,
                            int transposed, int Ktot, int j0, int u, bf16_t* out) {
  const int nchunks = Cin / CK;
  const size_t total = (size_t)(Cout / 16) * nchunks * nks_c * 64;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int lane = (int)(i & 63);
    const size_t rest = i >> 6;
    const int ks = (int)(rest % ((size_t)nchunks * nks_c));
    const int tile = (int)(rest / ((size_t)nchunks * nks_c));
    const int c = ks / nks_c, s = ks % nks_c;
    const int co = tile * 16 + (lane & 15);
    bf16_t v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int kk = s * 32 + 8 * (lane >> 4) + e;
      const int j = kk / CK, ci = c * CK + kk % CK;
      float f = 0.f;
      if (j < K) {
        size_t idx;
        if (transposed) {
          const int jt = j0 + u * (K - 1 - j);  // reversed phase taps
          idx = ((size_t)ci * Cout + co) * Ktot + jt;
        } else {
          idx = ((size_t)co * Cin + ci) * K + j;
        }
        f = src_bf16 ? bf2f(reinterpret_cast<const bf16_t*>(W)[idx]) : reinterpret_cast<const float*>(W)[idx];
      }
      v[e] = f2bf(f);
    }
    bf16_t* d = out + i * 8;
#pragma unroll
    for (int e = 0; e < 8; ++e) d[e] = v[e];
  }
}

// ids outside [0, n_codes) embed as zeros (see k_codec_embed in fo_codec.hip)
__global__ void k_codec_embed_cl(const bf16_t* table, int E, int n_codes, const int* ids, int BT, float* out) {
  const long long total = (long long)BT * E;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(e % E);
    const int id = ids[e / E];
    out[e] = (id >= 0 && id < n_codes) ? bf2f(table[(size_t)id * E + c]) : 0.f;
  }
}

// y[b][t][c] = y * s + g[b][c]  (1/num_kernels of the resblock sum, global-token feature)
__global__ void k_scale_add_cl(float* y, int B, int T, int C, float s, const float* g) {
  const long long total = (long long)B * T * C;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    float v = y[i] * s;
    if (g) v += g[(i / ((long long)T * C)) * C + i % C];
    y[i] = v;
  }
}

// conv_post (Cout = 1) + tanh: out[b][t] = tanh(bias + sum_{j,ci} w[ci][j] leaky(x[t + j - pad][ci]))
__global__ void k_conv_post_cl(const float* x, int B, int T, int C, const bf16_t* w, const float* bias, int K,
                               int pad, float slope, float* out) {
  const long long total = (long long)B * T;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int b = (int)(e / T), t = (int)(e % T);
    float acc = bias ? bias[0] : 0.f;
    for (int j = 0; j < K; ++j) {
      const int ti = t + j - pad;
      if (ti < 0 || ti >= T) continue;
      const float* xr = x + ((size_t)b * T + ti) * C;
      for (int ci = 0; ci < C; ++ci) {
        float v = xr[ci];
        v = v < 0.f ? v * slope : v;
        acc += v * bf2f(w[(size_t)ci * K + j]);
      }
    }
    out[e] = tanhf(acc);
  }
}

inline int grid_for(long long n) {
  long long g = (n + 255) / 256;
  return (int)(g > 8192 ? 8192 : (g < 1 ? 1 : g));
}

inline int pick_ck(int Cin) { return Cin >= 64 ? 64 : Cin; }

}  // namespace

extern "C" {

long long fo_conv_pack_elems(int Cout, int Cin, int K) {
  const int CK = pick_ck(Cin);
  const int nks_c = (K * CK + 31) / 32;
  return (long long)(Cout / 16) * (Cin / CK) * nks_c * 64 * 8;
}

// transposed == 0: W [Cout][Cin][K] conv weight.  transposed != 0: W [Cin][Cout][Ktot]
// ConvTranspose1d weight, packing phase taps j0, j0+u, ... (K of them) reversed.
int fo_pack_conv(const void* W, int src_bf16, int Cout, int Cin, int K, int transposed, int Ktot, int j0, int u,
                 void* out, hipStream_t s) {
  FO_REQUIRE(Cout % 16 == 0 && Cin >= 16 && Cin % 16 == 0 && K >= 1, "fo_pack_conv: Cout=%d Cin=%d K=%d", Cout, Cin,
             K);
  const int CK = pick_ck(Cin);
  FO_REQUIRE(Cin % CK == 0, "fo_pack_conv: Cin=%d not a multiple of %d", Cin, CK);
  const int nks_c = (K * CK + 31) / 32;
  const long long total = (long long)(Cout / 16) * (Cin / CK) * nks_c * 64;
  hipLaunchKernelGGL(k_pack_conv, dim3(grid_for(total)), dim3(256), 0, s, W, src_bf16, Cout, Cin, K, CK, nks_c,
                     transposed, Ktot, j0, u, (bf16_t*)out);
  return fo::check_launch("fo_pack_conv");
}

// Stride-1 conv on channel-last activations: x [B][Tin][Cin] -> out [B][Tout_total][Cout] at time
// q * ostride + ooff for q < Tq (Tq = Tin + 2 pad - dil (K-1) for a plain conv).
int fo_conv_cl(const float* x, int B, int Cin, int Tin, const void* wp, const float* bias, int Cout, int K, int dil,
               int pad, int Tq, int ostride, int ooff, int Tout_total, int pre_leaky, float slope, float* out,
               int residual, hipStream_t s) {
  FO_REQUIRE(Cout % 16 == 0 && Cin % 16 == 0 && Cin >= 16, "fo_conv_cl: Cout=%d Cin=%d", Cout, Cin);
  FO_REQUIRE(K >= 1 && dil >= 1 && dil * (K - 1) <= HALO, "fo_conv_cl: K=%d dil=%d beyond the LDS halo", K, dil);
  FO_REQUIRE(Tq > 0 && (long long)(Tq - 1) * ostride + ooff < Tout_total, "fo_conv_cl: output range");
  const int CK = pick_ck(Cin);
  ConvArgs a{x, (const bf16_t*)wp, bias, out, Cin, Tin, Cout, K, dil, pad, Tq, ostride, ooff, Tout_total,
             (K * CK + 31) / 32, pre_leaky, slope, residual};
  const int MTW = Cout >= 64 ? 4 : Cout / 16;
  const int NTW = 8 / MTW;
  dim3 grid((Tq + 64 * NTW - 1) / (64 * NTW), Cout / (16 * MTW), B);
  if (MTW == 4 && CK == 64) hipLaunchKernelGGL((k_conv_cl<4, 2, 64>), grid, dim3(256), 0, s, a);
  else if (MTW == 2 && CK == 64) hipLaunchKernelGGL((k_conv_cl<2, 4, 64>), grid, dim3(256), 0, s, a);
  else if (MTW == 2 && CK == 32) hipLaunchKernelGGL((k_conv_cl<2, 4, 32>), grid, dim3(256), 0, s, a);
  else if (MTW == 1 && CK == 32) hipLaunchKernelGGL((k_conv_cl<1, 8, 32>), grid, dim3(256), 0, s, a);
  else if (MTW == 1 && CK == 16) hipLaunchKernelGGL((k_conv_cl<1, 8, 16>), grid, dim3(256), 0, s, a);
  else if (MTW == 4 && CK == 32) hipLaunchKernelGGL((k_conv_cl<4, 2, 32>), grid, dim3(256), 0, s, a);
  else if (MTW == 4 && CK == 16) hipLaunchKernelGGL((k_conv_cl<4, 2, 16>), grid, dim3(256), 0, s, a);
  else if (MTW == 2 && CK == 16) hipLaunchKernelGGL((k_conv_cl<2, 4, 16>), grid, dim3(256), 0, s, a);
  else if (MTW == 1 && CK == 64) hipLaunchKernelGGL((k_conv_cl<1, 8, 64>), grid, dim3(256), 0, s, a);
  else FO_REQUIRE(false, "fo_conv_cl: no variant for Cout=%d Cin=%d", Cout, Cin);
  return fo::check_launch("fo_conv_cl");
}

int fo_codec_embed_cl(const void* table, int E, int n_codes, const int* ids, int B, int T, float* out, hipStream_t s) {
  const long long n = (long long)B * T * E;
  hipLaunchKernelGGL(k_codec_embed_cl, dim3(grid_for(n)), dim3(256), 0, s, (const bf16_t*)table, E, n_codes, ids,
                     B * T, out);
  return fo::check_launch("fo_codec_embed_cl");
}

int fo_scale_add_cl(float* y, int B, int T, int C, float sc, const float* g, hipStream_t s) {
  const long long n = (long long)B * T * C;
  hipLaunchKernelGGL(k_scale_add_cl, dim3(grid_for(n)), dim3(256), 0, s, y, B, T, C, sc, g);
  return fo::check_launch("fo_scale_add_cl");
}

int fo_conv_post_cl(const float* x, int B, int T, int C, const void* w, const float* bias, int K, int pad, float slope,
                    float* out, hipStream_t s) {
  const long long n = (long long)B * T;
  hipLaunchKernelGGL(k_conv_post_cl, dim3(grid_for(n)), dim3(256), 0, s, x, B, T, C, (const bf16_t*)w, bias, K, pad,
                     slope, out);
  return fo::check_launch("fo_conv_post_cl");
}

}  // extern "C"
