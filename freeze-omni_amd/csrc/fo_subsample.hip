// Conv2dSubsampling4 front end of the speech encoder (models/encoder/subsampling.py:67-73, with GlobalCMVN,
// models/encoder/cmvn.py:24-35), from fbank features to the input of its output Linear:
//
//   xn  = (feats - mean) * istd                                  [B][R][F]   F = 80 mel bins
//   y1  = relu(conv2d(xn, W1, 3x3, stride 2) + b1)               [B][H1][W1][C]  channel-last
//   y2  = relu(conv2d(y1, W2, 3x3, stride 2) + b2)               [B][H2][W2][C]
//   z   = y2.transpose(1, 2).view(B * H2, C * W2)                the Linear's rows: z[(b,t)][c*W2 + f]
//
// * k_sub_conv1: conv1 as a direct fp32 stencil (9 taps of one input channel) -- one thread owns 4 output channels
//   of a run of rows, its 36 weights in registers; the 9 normalised inputs of a row are shared by the whole
//   workgroup (L1 broadcast).  Replaces im2col + a K = 9 GEMM that wrote and re-read 3x the bytes.
// * k_sub_conv2: conv2 as an implicit GEMM on the matrix cores, K ordered tap-major (k = (3i + j) * C + c, the
//   weight packed from W2.permute(0, 2, 3, 1)), so a 32-wide k-step is 32 channels of ONE tap and its A rows are
//   y1 rows (b, 2 h2 + i, 2 w2 + j) read in place (no im2col buffer).  Tile 64 rows x 256 columns on 4 waves: the
//   A tile is staged through LDS once per k-step, already split into bf16 hi + lo MFMA fragments (double
//   buffered), and each wave streams its 4 column tiles' weight fragments straight from the packed layout
//   (1 KiB per tile per k-step).  K is split over S workgroups (partial slabs); the S x col-tile groups are
//   dealt to XCDs so the row tiles sharing a weight slice run on one XCD (its L2 serves the re-reads).
// * k_sub_reduce: the slabs summed in split order + bias + ReLU, written transposed into z through LDS
//   (contiguous stores of a z row segment).
#include "fo_common.h"

namespace {

constexpr int SUB_RB = 4;      // row blocks of 16 per conv2 tile (64 rows)
constexpr int SUB_NW = 4;      // waves per conv2 workgroup
constexpr int SUB_NTW = 4;     // 16-column tiles per wave (256 columns per workgroup)

__global__ __launch_bounds__(256) void k_sub_conv1(const float* __restrict__ feats, int R, int F, int H1, int W1,
                                                   int rows, int rpb, const float* __restrict__ mean,
                                                   const float* __restrict__ istd, const float* __restrict__ w1,
                                                   const float* __restrict__ b1, int C, float* __restrict__ y1) {
  const int c4 = blockIdx.y * 256 + threadIdx.x;   // this thread's 4 channels: 4 c4 .. 4 c4 + 3
  if (4 * c4 >= C) return;
  float w[4][9], bb[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
#pragma unroll
    for (int t = 0; t < 9; ++t) w[q][t] = w1[(size_t)(4 * c4 + q) * 9 + t];
    bb[q] = b1[4 * c4 + q];
  }
  const int r0 = blockIdx.x * rpb, r1 = min(rows, r0 + rpb);
  for (int row = r0; row < r1; ++row) {
    const int b = row / (H1 * W1), rem = row - b * (H1 * W1);
    const int h1 = rem / W1, w1i = rem - h1 * W1;
    const float* xr = feats + ((size_t)b * R + 2 * h1) * F + 2 * w1i;
    float xn[9];
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const int f = 2 * w1i + q;
        xn[p * 3 + q] = (xr[p * F + q] - mean[f]) * istd[f];
      }
    float4 o;
    float* op = &o.x;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float acc = bb[q];
#pragma unroll
      for (int t = 0; t < 9; ++t) acc = fmaf(w[q][t], xn[t], acc);
      op[q] = acc > 0.f ? acc : 0.f;
    }
    *reinterpret_cast<float4*>(y1 + (size_t)row * C + 4 * c4) = o;
  }
}

struct Conv2Args {
  const float* y1;      // [B][H1][W1][C]
  const bf16x8* wp;     // packed [ntiles][KS][64][8], K tap-major
  float* slab;          // [S][M][N]
  int C, H1, W1, H2, W2, M, N, ntiles, KS, S;
  int n_mt, n_nt, groups;   // row tiles, 256-column tiles, (column tile, split) groups
};

// y1 row of conv2 output row m at tap (i, j)
__device__ __forceinline__ int y1_row(const Conv2Args& a, int m, int i, int j) {
  const int b = m / (a.H2 * a.W2), rem = m - b * (a.H2 * a.W2);
  const int h2 = rem / a.W2, w2 = rem - h2 * a.W2;
  return (b * a.H1 + 2 * h2 + i) * a.W1 + 2 * w2 + j;
}

__global__ __launch_bounds__(256) void k_sub_conv2(Conv2Args a) {
  // XCD-aware decode: workgroup b runs on XCD b % 8; the groups g (a column tile x a K split) with g % 8 == xcd
  // are that XCD's, each with its n_mt row tiles
  const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
  const int g = xcd + 8 * (slot / a.n_mt), mt = slot % a.n_mt;
  if (g >= a.groups) return;
  const int nt = g % a.n_nt, sp = g / a.n_nt;
  const int ks0 = (int)((long)a.KS * sp / a.S), ks1 = (int)((long)a.KS * (sp + 1) / a.S);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int m0 = mt * (SUB_RB * 16);
  // A staging: thread t loads row (t >> 2) of the tile, 8 channels at (t & 3) * 8 of the k-step
  const int sr = threadIdx.x >> 2, sk = (threadIdx.x & 3) * 8;
  const int srow_m = min(m0 + sr, a.M - 1);   // rows >= M: computed from a valid row, never stored
  __shared__ bf16x8 As[2][SUB_RB][2][64];     // [buffer][row block][hi / lo][fragment lane]
  const int frag_lane = ((sk >> 3) << 4) | (sr & 15), frag_rb = sr >> 4;
  auto load_a = [&](int ks, float4& p0, float4& p1) {
    const int k = ks * 32, tap = k / a.C, c0 = k - tap * a.C;
    const float* src = a.y1 + (size_t)y1_row(a, srow_m, tap / 3, tap % 3) * a.C + c0 + sk;
    p0 = reinterpret_cast<const float4*>(src)[0];
    p1 = reinterpret_cast<const float4*>(src)[1];
  };
  auto store_a = [&](int buf, const float4& p0, const float4& p1) {
    const float f[8] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w};
    bf16x8 hi, lo;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const __bf16 h = (__bf16)f[e];
      hi[e] = h;
      lo[e] = (__bf16)(f[e] - (float)h);
    }
    As[buf][frag_rb][0][frag_lane] = hi;
    As[buf][frag_rb][1][frag_lane] = lo;
  };
  // this wave's column tiles (tiles past the weight are skipped: wave-uniform)
  const int t0 = nt * (SUB_NW * SUB_NTW) + wave * SUB_NTW;
  int ntw = a.ntiles - t0;
  ntw = ntw < 0 ? 0 : (ntw > SUB_NTW ? SUB_NTW : ntw);
  const bf16x8* bp = a.wp + (size_t)t0 * a.KS * 64 + lane;
  bf16x8 zero;
#pragma unroll
  for (int e = 0; e < 8; ++e) zero[e] = (__bf16)0.f;
  auto load_b = [&](int ks, bf16x8 (&bv)[SUB_NTW]) {
#pragma unroll
    for (int t = 0; t < SUB_NTW; ++t)
      bv[t] = t < ntw ? __builtin_nontemporal_load(bp + ((size_t)t * a.KS + ks) * 64) : zero;
  };
  f32x4 acc[SUB_RB][SUB_NTW];
#pragma unroll
  for (int r = 0; r < SUB_RB; ++r)
#pragma unroll
    for (int t = 0; t < SUB_NTW; ++t) acc[r][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  float4 pa0, pa1;
  bf16x8 bcur[SUB_NTW], bnext[SUB_NTW];
  load_a(ks0, pa0, pa1);
  load_b(ks0, bcur);
  store_a(0, pa0, pa1);
  __syncthreads();
  int buf = 0;
  for (int ks = ks0; ks < ks1; ++ks) {
    const bool more = ks + 1 < ks1;
    if (more) {   // next k-step's A rows and weights in flight while this one computes
      load_a(ks + 1, pa0, pa1);
      load_b(ks + 1, bnext);
    }
#pragma unroll
    for (int r = 0; r < SUB_RB; ++r) {
      const bf16x8 ah = As[buf][r][0][lane], al = As[buf][r][1][lane];
#pragma unroll
      for (int t = 0; t < SUB_NTW; ++t) {
        acc[r][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bcur[t], acc[r][t], 0, 0, 0);
        acc[r][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bcur[t], acc[r][t], 0, 0, 0);
      }
    }
    if (more) {
      store_a(buf ^ 1, pa0, pa1);   // the other buffer: its last readers finished before the previous barrier
#pragma unroll
      for (int t = 0; t < SUB_NTW; ++t) bcur[t] = bnext[t];
    }
    __syncthreads();
    buf ^= 1;
  }
  // partial tile of split sp: D layout (16x16x32): row 4 (lane >> 4) + i, column lane & 15
  float* slab = a.slab + (size_t)sp * a.M * a.N;
#pragma unroll
  for (int t = 0; t < SUB_NTW; ++t) {
    if (t >= ntw) break;
    const int n = (t0 + t) * 16 + (lane & 15);
    if (n >= a.N) continue;
#pragma unroll
    for (int r = 0; r < SUB_RB; ++r)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = m0 + r * 16 + 4 * (lane >> 4) + i;
        if (m < a.M) slab[(size_t)m * a.N + n] = acc[r][t][i];
      }
  }
}

// z[(b, h2)][c * W2 + w2] = relu(b2[c] + sum_s slab[s][(b, h2, w2)][c]); block = one (b, h2) row x 64 channels
__global__ __launch_bounds__(256) void k_sub_reduce(const float* __restrict__ slab, int S, int M, int N, int W2,
                                                    const float* __restrict__ b2, float* __restrict__ z) {
  extern __shared__ float st[];   // [W2][65]
  const int row = blockIdx.x, c0 = blockIdx.y * 64;
  const int nc = min(64, N - c0);
  const int E = W2 * 64;
  for (int e = threadIdx.x; e < E; e += 256) {
    const int w2 = e >> 6, cc = e & 63;
    float v = 0.f;
    if (cc < nc) {
      const size_t o = (size_t)(row * W2 + w2) * N + c0 + cc;
      for (int s = 0; s < S; ++s) v += slab[(size_t)s * M * N + o];
      v += b2[c0 + cc];
      v = v > 0.f ? v : 0.f;
    }
    st[w2 * 65 + cc] = v;
  }
  __syncthreads();
  float* zr = z + (size_t)row * N * W2 + (size_t)c0 * W2;
  for (int e = threadIdx.x; e < nc * W2; e += 256) {
    const int cc = e / W2, w2 = e - cc * W2;
    zr[e] = st[w2 * 65 + cc];
  }
}

}  // namespace

extern "C" {

long long fo_subsample_ws_floats(int B, int R, int F, int C) {
  const int H1 = (R - 3) / 2 + 1, W1 = (F - 3) / 2 + 1, H2 = (H1 - 3) / 2 + 1, W2 = (W1 - 3) / 2 + 1;
  const int M = B * H2 * W2;
  const int n_mt = (M + SUB_RB * 16 - 1) / (SUB_RB * 16), n_nt = (C + 255) / 256;
  int S = 256 / (n_mt * n_nt);
  S = S < 1 ? 1 : (S > 8 ? 8 : S);
  return (long long)S * M * C;
}

int fo_subsample(const float* feats, int B, int R, int F, const float* mean, const float* istd, const float* w1,
                 const float* b1, int C, float* y1, const void* w2p, const float* b2, float* z, float* ws,
                 long long ws_floats, hipStream_t s) {
  FO_REQUIRE(B > 0 && R >= 7 && F >= 7 && C > 0 && (C % 32) == 0,
             "fo_subsample: B=%d R=%d F=%d C=%d (C a multiple of 32, >= 7 frames and bins)", B, R, F, C);
  FO_REQUIRE(feats && mean && istd && w1 && b1 && y1 && w2p && b2 && z && ws, "fo_subsample: null argument");
  const int H1 = (R - 3) / 2 + 1, W1 = (F - 3) / 2 + 1, H2 = (H1 - 3) / 2 + 1, W2 = (W1 - 3) / 2 + 1;
  const int rows1 = B * H1 * W1;
  const int rpb = 8;
  hipLaunchKernelGGL(k_sub_conv1, dim3((rows1 + rpb - 1) / rpb, (C / 4 + 255) / 256), dim3(256), 0, s, feats, R, F, H1,
                     W1, rows1, rpb, mean, istd, w1, b1, C, y1);
  int rc = fo::check_launch("fo_subsample/conv1");
  if (rc) return rc;
  Conv2Args a;
  a.y1 = y1;
  a.wp = reinterpret_cast<const bf16x8*>(w2p);
  a.slab = ws;
  a.C = C;
  a.H1 = H1;
  a.W1 = W1;
  a.H2 = H2;
  a.W2 = W2;
  a.M = B * H2 * W2;
  a.N = C;
  a.ntiles = (C + 15) / 16;
  a.KS = 9 * C / 32;
  a.n_mt = (a.M + SUB_RB * 16 - 1) / (SUB_RB * 16);
  a.n_nt = (C + 255) / 256;
  int S = 256 / (a.n_mt * a.n_nt);
  S = S < 1 ? 1 : (S > 8 ? 8 : S);
  if (S > a.KS) S = a.KS;
  a.S = S;
  a.groups = a.n_nt * S;
  FO_REQUIRE((long long)S * a.M * a.N <= ws_floats, "fo_subsample: workspace of %lld floats < %lld", ws_floats,
             (long long)S * a.M * a.N);
  const int per_xcd = (a.groups + 7) / 8;
  hipLaunchKernelGGL(k_sub_conv2, dim3(8 * per_xcd * a.n_mt), dim3(256), 0, s, a);
  rc = fo::check_launch("fo_subsample/conv2");
  if (rc) return rc;
  hipLaunchKernelGGL(k_sub_reduce, dim3(B * H2, (C + 63) / 64), dim3(256), (size_t)W2 * 65 * sizeof(float), s, ws, S,
                     a.M, C, W2, b2, z);
  fo::count_launch(FO_L_SUBSAMPLE);
  return fo::check_launch("fo_subsample/reduce");
}

}  // extern "C"
