// Read-only streaming probes (measurement only, not part of the product library): what the HBM
// delivers to a given grid/access pattern, to separate the GEMM body's cost from the stream's.
//   k_read_frag<NT,NW,U>: the packed-weight access pattern of fo_gemm (one workgroup = NT 16-column
//                         tiles, NW waves dealing U-step groups of the K range, 1 KiB per wave-load)
//   k_read_lin           : grid-stride 16-B loads over a flat buffer
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;

template <int NT, int NW, int U, int IL = 0>
__global__ __launch_bounds__(NW * 64) void k_read_frag(const u32x4* w, int KS, uint32_t* out) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const u32x4* bp[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t)
    bp[t] = IL ? w + ((size_t)blockIdx.x * KS * NT + t) * 64 + lane : w + (size_t)(blockIdx.x * NT + t) * KS * 64 + lane;
  const int kstr = IL ? NT * 64 : 64;
  uint32_t acc = 0;
  const int G = KS / U;
  const int gb = G * wave / NW, ge = G * (wave + 1) / NW;
  for (int g = gb; g < ge; ++g) {
    u32x4 v[U][NT];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int t = 0; t < NT; ++t) v[u][t] = __builtin_nontemporal_load(bp[t] + (size_t)(g * U + u) * kstr);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int t = 0; t < NT; ++t) acc ^= v[u][t].x ^ v[u][t].y ^ v[u][t].z ^ v[u][t].w;
  }
  if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

__global__ void k_read_lin(const u32x4* w, long long n16, uint32_t* out) {
  uint32_t acc = 0;
  const long long stride = (long long)gridDim.x * blockDim.x;
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    const u32x4 a = __builtin_nontemporal_load(w + i), b = __builtin_nontemporal_load(w + i + stride);
    const u32x4 c = __builtin_nontemporal_load(w + i + 2 * stride), d = __builtin_nontemporal_load(w + i + 3 * stride);
    acc ^= a.x ^ b.y ^ c.z ^ d.w;
  }
  for (; i < n16; i += stride) acc ^= w[i].x;
  if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

template <int NT, int NW, int U>
static void launch_frag(const void* w, int ntiles, int KS, uint32_t* out, hipStream_t s, int il) {
  if (il) hipLaunchKernelGGL((k_read_frag<NT, NW, U, 1>), dim3(ntiles / NT), dim3(NW * 64), 0, s, (const u32x4*)w, KS, out);
  else hipLaunchKernelGGL((k_read_frag<NT, NW, U, 0>), dim3(ntiles / NT), dim3(NW * 64), 0, s, (const u32x4*)w, KS, out);
}

extern "C" {
// kind 0: linear (grid = blocks of 256); kind 1: fragment pattern with (nt, nw, u)
// Launches reps times, rotating over nbuf buffers, and returns the average time per launch in us.
double probe_time(int kind, void** bufs, int nbuf, long long bytes, int ntiles, int KS, int nt, int nw, int u,
                  int grid, int reps, void* out) {
  hipStream_t s;
  hipStreamCreate(&s);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto one = [&](int i) {
    const void* w = bufs[i % nbuf];
    if (kind == 0) {
      hipLaunchKernelGGL(k_read_lin, dim3(grid), dim3(256), 0, s, (const u32x4*)w, bytes / 16, (uint32_t*)out);
    } else {
#define FR(A, B, C) if (nt == A && nw == B && u == C) launch_frag<A, B, C>(w, ntiles, KS, (uint32_t*)out, s, kind == 2)
      FR(1, 4, 4); FR(2, 4, 4); FR(4, 4, 4); FR(1, 8, 4); FR(2, 8, 4); FR(4, 8, 4); FR(1, 16, 4); FR(2, 16, 4);
      FR(4, 16, 4); FR(4, 4, 2); FR(4, 8, 2); FR(2, 8, 8); FR(1, 16, 8); FR(8, 4, 2); FR(8, 8, 2);
      FR(8, 4, 4); FR(16, 4, 2); FR(8, 2, 4); FR(4, 4, 8); FR(4, 4, 6);
#undef FR
    }
  };
  for (int i = 0; i < nbuf; ++i) one(i);
  hipEventRecord(e0, s);
  for (int i = 0; i < reps; ++i) one(i);
  hipEventRecord(e1, s);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  hipStreamDestroy(s);
  return ms * 1e3 / reps;
}
}

// GEMM body probe: the fo_gemm main loop with knobs, to price its parts against the bare stream.
//   XM 0: fp32 X split hi/lo (2 MFMAs per fragment, as fo_gemm); 1: no X loads (register constant);
//   XM 2: bf16 X (1 MFMA); XM 3: X pre-split bf16 hi|lo in fragment order [K/32][64 lanes][16 bf16]
//   MF 0: skip the MFMAs (xor the fragments instead)
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
template <int NT, int NW, int U, int XM, int MF>
__global__ __launch_bounds__(NW * 64) void k_gemm_probe(const bf16x8* W, const float* X, int K, float* Y) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int KS = K >> 5;
  f32x4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bf16x8* bp[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t)
    bp[t] = XM == 4 ? W + ((size_t)blockIdx.x * KS * NT + t) * 64 + lane : W + (size_t)(blockIdx.x * NT + t) * KS * 64 + lane;
  const int kstr = XM == 4 ? NT * 64 : 64;
  const float* xr = X + (size_t)(lane & 15) * K + 8 * (lane >> 4);
  const bf16x8* xb = reinterpret_cast<const bf16x8*>(X) + lane * 2;
  uint32_t xx = 0;
  const int G = KS / U;
  const int gb = G * wave / NW, ge = G * (wave + 1) / NW;
  bf16x8 cst;
#pragma unroll
  for (int j = 0; j < 8; ++j) cst[j] = (__bf16)(0.001f * (lane + j));
  for (int g = gb; g < ge; ++g) {
    const int ks = g * U;
    bf16x8 bv[U][NT], ah[U], al[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int t = 0; t < NT; ++t) bv[u][t] = __builtin_nontemporal_load(bp[t] + (size_t)(ks + u) * kstr);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if constexpr (XM == 0 || XM == 4) {
        const float4 a = reinterpret_cast<const float4*>(xr + (size_t)(ks + u) * 32)[0];
        const float4 b = reinterpret_cast<const float4*>(xr + (size_t)(ks + u) * 32)[1];
        const float f[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const __bf16 h = (__bf16)f[j];
          ah[u][j] = h;
          al[u][j] = (__bf16)(f[j] - (float)h);
        }
      } else if constexpr (XM == 2) {
        ah[u] = *reinterpret_cast<const bf16x8*>(reinterpret_cast<const __bf16*>(X) + (size_t)(lane & 15) * K +
                                                 8 * (lane >> 4) + (size_t)(ks + u) * 32);
      } else if constexpr (XM == 3) {
        ah[u] = xb[(size_t)(ks + u) * 128];
        al[u] = xb[(size_t)(ks + u) * 128 + 1];
      } else {
        ah[u] = cst;
        al[u] = cst;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        if constexpr (MF) {
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[u], bv[u][t], acc[t], 0, 0, 0);
          if constexpr (XM == 0 || XM == 3 || XM == 4)
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[u], bv[u][t], acc[t], 0, 0, 0);
        } else {
          xx ^= __builtin_bit_cast(uint32_t, __builtin_shufflevector(bv[u][t], bv[u][t], 0, 1)) ^
                __builtin_bit_cast(uint32_t, __builtin_shufflevector(ah[u], al[u], 2, 11));
        }
      }
  }
  __shared__ float red[NW][NT][16][17];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) red[wave][t][4 * (lane >> 4) + i][lane & 15] = acc[t][i] + (float)(xx & 1);
  __syncthreads();
  for (int e = threadIdx.x; e < NT * 256; e += NW * 64) {
    const int t = e >> 8, r = (e >> 4) & 15, c = e & 15;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) v += red[w][t][r][c];
    Y[(size_t)r * gridDim.x * NT * 16 + (blockIdx.x * NT + t) * 16 + c] = v;
  }
}

extern "C" double probe_gemm(void** bufs, int nbuf, int ntiles, int K, int nt, int nw, int u, int xm, int mf,
                             const void* X, void* Y, int reps) {
  hipStream_t s;
  hipStreamCreate(&s);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  bool ok = false;
  auto one = [&](int i) {
    const bf16x8* w = (const bf16x8*)bufs[i % nbuf];
#define GP(A, B, C, D, E)                                                                                  \
  if (nt == A && nw == B && u == C && xm == D && mf == E) {                                                \
    hipLaunchKernelGGL((k_gemm_probe<A, B, C, D, E>), dim3(ntiles / A), dim3(B * 64), 0, s, w, (const float*)X, K, \
                       (float*)Y);                                                                         \
    ok = true;                                                                                             \
  }
#define GPX(A, B, C) GP(A, B, C, 0, 1) GP(A, B, C, 1, 1) GP(A, B, C, 2, 1) GP(A, B, C, 3, 1) GP(A, B, C, 0, 0) GP(A, B, C, 4, 1)
    GPX(4, 4, 4) GPX(4, 8, 4) GPX(1, 16, 4) GPX(2, 8, 4) GPX(8, 4, 2) GPX(8, 8, 2) GPX(1, 4, 4) GPX(2, 16, 4)
    GPX(8, 4, 4) GPX(16, 4, 1) GPX(16, 4, 2) GPX(8, 2, 4) GPX(4, 2, 4) GPX(8, 4, 3) GPX(4, 4, 6) GPX(4, 4, 8)
#undef GPX
#undef GP
  };
  for (int i = 0; i < nbuf; ++i) one(i);
  if (!ok) return -1.0;
  hipEventRecord(e0, s);
  for (int i = 0; i < reps; ++i) one(i);
  hipEventRecord(e1, s);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  hipStreamDestroy(s);
  return ms * 1e3 / reps;
}

// Software-pipelined body: the next U-step group's weight + X loads are issued before the current
// group's MFMAs, so every wave keeps a group in flight while it computes.  Separate hi / lo
// accumulators (SPL) let the two MFMAs of a fragment issue back to back.
template <int NT, int U>
struct PFrag {
  bf16x8 w[U][NT];
  float4 x[U][2];
};
template <int NT, int NW, int U, int SPL>
__global__ __launch_bounds__(NW * 64) void k_gemm_pipe(const bf16x8* W, const float* X, int K, float* Y) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int KS = K >> 5;
  f32x4 acc[NT], acl[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = acl[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bf16x8* bp[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) bp[t] = W + (size_t)(blockIdx.x * NT + t) * KS * 64 + lane;
  const float* xr = X + (size_t)(lane & 15) * K + 8 * (lane >> 4);
  const int G = KS / U;
  const int gb = G * wave / NW, ge = G * (wave + 1) / NW;
  auto load = [&](PFrag<NT, U>& f, int g) {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int t = 0; t < NT; ++t) f.w[u][t] = __builtin_nontemporal_load(bp[t] + (size_t)(g * U + u) * 64);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      f.x[u][0] = reinterpret_cast<const float4*>(xr + (size_t)(g * U + u) * 32)[0];
      f.x[u][1] = reinterpret_cast<const float4*>(xr + (size_t)(g * U + u) * 32)[1];
    }
  };
  auto compute = [&](const PFrag<NT, U>& f) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      bf16x8 h, l;
      const float v[8] = {f.x[u][0].x, f.x[u][0].y, f.x[u][0].z, f.x[u][0].w,
                          f.x[u][1].x, f.x[u][1].y, f.x[u][1].z, f.x[u][1].w};
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const __bf16 hh = (__bf16)v[j];
        h[j] = hh;
        l[j] = (__bf16)(v[j] - (float)hh);
      }
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(h, f.w[u][t], acc[t], 0, 0, 0);
        if (SPL) acl[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(l, f.w[u][t], acl[t], 0, 0, 0);
        else acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(l, f.w[u][t], acc[t], 0, 0, 0);
      }
    }
  };
  PFrag<NT, U> A, B;
  if (gb < ge) load(A, gb);
  int g = gb;
  for (; g + 1 < ge; g += 2) {
    load(B, g + 1);
    compute(A);
    if (g + 2 < ge) load(A, g + 2);
    compute(B);
  }
  if (g < ge) compute(A);
  __shared__ float red[NW][NT][16][17];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) red[wave][t][4 * (lane >> 4) + i][lane & 15] = acc[t][i] + acl[t][i];
  __syncthreads();
  for (int e = threadIdx.x; e < NT * 256; e += NW * 64) {
    const int t = e >> 8, r = (e >> 4) & 15, c = e & 15;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) v += red[w][t][r][c];
    Y[(size_t)r * gridDim.x * NT * 16 + (blockIdx.x * NT + t) * 16 + c] = v;
  }
}

extern "C" double probe_pipe(void** bufs, int nbuf, int ntiles, int K, int nt, int nw, int u, int spl,
                             const void* X, void* Y, int reps) {
  hipStream_t s;
  hipStreamCreate(&s);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  bool ok = false;
  auto one = [&](int i) {
    const bf16x8* w = (const bf16x8*)bufs[i % nbuf];
#define GP(A, B, C, D)                                                                                    \
  if (nt == A && nw == B && u == C && spl == D) {                                                          \
    hipLaunchKernelGGL((k_gemm_pipe<A, B, C, D>), dim3(ntiles / A), dim3(B * 64), 0, s, w, (const float*)X, K, \
                       (float*)Y);                                                                         \
    ok = true;                                                                                             \
  }
#define GPX(A, B, C) GP(A, B, C, 0) GP(A, B, C, 1)
    GPX(4, 4, 2) GPX(4, 4, 4) GPX(4, 8, 2) GPX(2, 8, 2) GPX(2, 8, 4) GPX(1, 16, 2) GPX(1, 16, 4) GPX(2, 16, 2)
    GPX(1, 8, 4) GPX(1, 4, 4) GPX(8, 4, 1) GPX(2, 4, 4)
#undef GPX
#undef GP
  };
  for (int i = 0; i < nbuf; ++i) one(i);
  if (!ok) return -1.0;
  hipEventRecord(e0, s);
  for (int i = 0; i < reps; ++i) one(i);
  hipEventRecord(e1, s);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  hipStreamDestroy(s);
  return ms * 1e3 / reps;
}
