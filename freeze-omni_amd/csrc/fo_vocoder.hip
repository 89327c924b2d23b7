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
#include "fo_hip.h"

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
  // epilogue: out = (conv + bias + res + res2) * oscale + gadd[b][co]; res / res2 are [B][Tout_total][Cout]
  // like out and may alias it (each element is read and written by the same lane)
  const float* res;
  const float* res2;
  float oscale;
  const float* gadd;   // [B][Cout] or null
};

// Up to CONV_MAXG convolutions of one shape class (same Cin / Cout) in one launch: blockIdx.z = b + B * g
// runs conv g on batch row b (the u polyphase components of a ConvTranspose1d; the independent dilated
// ResBlock1 chains of a stage, models/decoder/ticodec/models.py:221-238); sum != 0: every workgroup runs ALL G
// convs of its output tile into one accumulator and stores (sum_g (conv_g + bias_g + res_g + res2_g)) *
// oscale + gadd (the resblocks' last convs, whose outputs the reference averages) -- out / oscale / gadd /
// the output geometry are a[0]'s.
constexpr int CONV_MAXG = 5;
struct ConvMulti {
  ConvArgs a[CONV_MAXG];
  int B, G, sum;
  unsigned long long* trc;   // probes (fo_conv_set_trace): per workgroup {start, stage cycles, compute cycles, end}
};

constexpr int CONV_KMAX = 11;
// k-steps per Cin chunk, rounded up to even (padding k-steps carry zero weights)
__host__ __device__ constexpr int nks_per_chunk(int K, int CK) { return ((K * CK + 31) / 32 + 1) & ~1; }
__host__ __device__ constexpr int conv_wmax(int CK) { return nks_per_chunk(CONV_KMAX, CK); }

// PF: the next Cin chunk's activation window is loaded into registers while this chunk's MFMAs run (issued after the
// chunk's barrier, converted into LDS after the next one), and the weight fragments come by asm LDS-DMA
// (fo_common.h dma16) counted by hand -- the builtin's conservative waits would drain the prefetch before the first
// LDS read of the compute.  Without PF the chunk is staged, then computed (r05o: staging 56-59 % of the chunk loop).
template <int MTW, int NTW, int CK, bool TR = false, bool PF = false>   // TR: per-workgroup clocks (mc.trc, probes)
__global__ __launch_bounds__(256) void k_conv_cl(ConvMulti mc) {
  constexpr int TW = 64 * NTW;     // time steps per workgroup (4 waves x 16*NTW)
  constexpr int ROWS = TW + HALO;
  constexpr int LP = CK + 8;       // padded bf16 row (16 B): 16 lanes of different rows hit distinct banks
  // the window is split into bf16 hi + lo ONCE when staged; every k-step's B fragments are then two
  // 16-B LDS reads with no conversion (the split in the k-loop made the kernel VALU-bound)
  __shared__ __attribute__((aligned(16))) __bf16 xh[ROWS][LP];
  __shared__ __attribute__((aligned(16))) __bf16 xl[ROWS][LP];
  __shared__ __attribute__((aligned(16))) bf16_t wl[MTW * conv_wmax(CK) * 512];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int t0 = blockIdx.x * TW;
  const int ct0 = blockIdx.y * MTW;  // first 16-channel output tile
  const int g0 = mc.sum ? 0 : (int)blockIdx.z / mc.B;
  const int b = mc.sum ? (int)blockIdx.z : (int)blockIdx.z % mc.B;
  const int g1 = mc.sum ? mc.G : g0 + 1;
  if (t0 >= mc.a[g0].Tq) return;  // (polyphase components: the shorter phases' last time tile)

  f32x4 acc[MTW][NTW];
#pragma unroll
  for (int m = 0; m < MTW; ++m)
#pragma unroll
    for (int n = 0; n < NTW; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
  // (a compile-time switch: the runtime-null hook cost the product launches 2-4 %, r05zz vs r05m)
  unsigned long long* const tr =
      TR ? mc.trc + 4 * (size_t)(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z)) : nullptr;
  unsigned long long t_stage = 0, t_comp = 0;
  if (tr && threadIdx.x == 0) tr[0] = wall_clock64();

  const int tl = wave * 16 * NTW + (lane & 15);  // this lane's time row (tile n adds 16 n)
  const int kq = 8 * (lane >> 4);                 // this lane's 8-wide K slice inside a step

  for (int g = g0; g < g1; ++g) {
    const ConvArgs& a = mc.a[g];
    const int nks = (a.Cin / CK) * a.nks_c;
    const int span = TW + a.dil * (a.K - 1);
    const float* xb = a.x + (size_t)b * a.Tin * a.Cin;
    // A chunk's weight A-fragments (MTW tiles x nks_c k-steps, 1 KiB each) are copied global -> LDS
    // with 16-B LDS-DMA loads (lane-linear, exactly one fragment per wave-instruction), issued with the
    // activation loads: one memory latency per chunk, and the four waves share one copy.
    // Staging: every thread issues all of its window loads for the chunk back to back (MAXL 16-B loads,
    // one latency per chunk instead of one per loop trip), then splits them into LDS.
    constexpr int MAXL = (ROWS * (CK / 4) + 255) / 256;
    auto stage = [&](int c) {
      __syncthreads();  // the previous chunk's (or convolution's) reads are done
      for (int f = wave; f < MTW * a.nks_c; f += 4) {
        const int m = f / a.nks_c, st = f - m * a.nks_c;
        const bf16_t* src = a.wp + ((size_t)(ct0 + m) * nks + c * a.nks_c + st) * 512 + lane * 8;
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                         (__attribute__((address_space(3))) void*)&wl[f * 512], 16, 0, 0);
      }
      float4 v[MAXL];
#pragma unroll
      for (int i = 0; i < MAXL; ++i) {
        const int e = threadIdx.x + 256 * i;
        const int row = e / (CK / 4), c4 = e % (CK / 4);
        const int ti = t0 - a.pad + row;
        v[i] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (e < span * (CK / 4) && ti >= 0 && ti < a.Tin)
          v[i] = *reinterpret_cast<const float4*>(xb + (size_t)ti * a.Cin + c * CK + c4 * 4);
      }
#pragma unroll
      for (int i = 0; i < MAXL; ++i) {
        const int e = threadIdx.x + 256 * i;
        if (e >= span * (CK / 4)) break;
        const int row = e / (CK / 4), c4 = e % (CK / 4);
        float f[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
        __attribute__((ext_vector_type(4))) __bf16 h4, l4;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (a.pre_act) f[q] = f[q] < 0.f ? f[q] * a.slope : f[q];
          const __bf16 h = (__bf16)f[q];
          h4[q] = h;
          l4[q] = (__bf16)(f[q] - (float)h);
        }
        *reinterpret_cast<decltype(h4)*>(&xh[row][c4 * 4]) = h4;
        *reinterpret_cast<decltype(l4)*>(&xl[row][c4 * 4]) = l4;
      }
      __builtin_amdgcn_s_waitcnt(0);  // the LDS-DMA copies (vmcnt) too
      __syncthreads();
    };
    auto comp = [&](int s) {
      const int kk = s * 32 + kq;
      int j = kk / CK;
      const int cil = kk - j * CK;
      if (j > a.K - 1) j = a.K - 1;  // padded K: the packed weights are zero there
      const int rb = tl + j * a.dil;
      bf16x8 av[MTW];
#pragma unroll
      for (int m = 0; m < MTW; ++m) av[m] = *reinterpret_cast<const bf16x8*>(&wl[(m * a.nks_c + s) * 512 + lane * 8]);
#pragma unroll
      for (int n = 0; n < NTW; ++n) {
        const bf16x8 hi = *reinterpret_cast<const bf16x8*>(&xh[rb + 16 * n][cil]);
        const bf16x8 lo = *reinterpret_cast<const bf16x8*>(&xl[rb + 16 * n][cil]);
#pragma unroll
        for (int m = 0; m < MTW; ++m) {
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[m], hi, acc[m][n], 0, 0, 0);
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[m], lo, acc[m][n], 0, 0, 0);
        }
      }
    };
    const int nchunks = a.Cin / CK;
    if constexpr (PF) {
      float4 v[MAXL];
      auto load_x = [&](int c) {
#pragma unroll
        for (int i = 0; i < MAXL; ++i) {
          const int e = threadIdx.x + 256 * i;
          const int row = e / (CK / 4), c4 = e % (CK / 4);
          const int ti = t0 - a.pad + row;
          v[i] = make_float4(0.f, 0.f, 0.f, 0.f);
          if (e < span * (CK / 4) && ti >= 0 && ti < a.Tin)
            v[i] = *reinterpret_cast<const float4*>(xb + (size_t)ti * a.Cin + c * CK + c4 * 4);
        }
      };
      load_x(0);
      for (int c = 0; c < nchunks; ++c) {
        const unsigned long long c0 = tr ? clock64() : 0;
        __syncthreads();  // the previous chunk's (or convolution's) reads of xh / xl / wl are done
        for (int f = wave; f < MTW * a.nks_c; f += 4) {
          const int m = f / a.nks_c, st = f - m * a.nks_c;
          dma16(a.wp + ((size_t)(ct0 + m) * nks + c * a.nks_c + st) * 512 + lane * 8,
                __builtin_amdgcn_readfirstlane(lds_addr(&wl[f * 512])));
        }
#pragma unroll
        for (int i = 0; i < MAXL; ++i) {
          const int e = threadIdx.x + 256 * i;
          if (e >= span * (CK / 4)) continue;   // (no break: a fully unrolled loop keeps v in registers)
          const int row = e / (CK / 4), c4 = e % (CK / 4);
          float f[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
          __attribute__((ext_vector_type(4))) __bf16 h4, l4;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            if (a.pre_act) f[q] = f[q] < 0.f ? f[q] * a.slope : f[q];
            const __bf16 h = (__bf16)f[q];
            h4[q] = h;
            l4[q] = (__bf16)(f[q] - (float)h);
          }
          *reinterpret_cast<decltype(h4)*>(&xh[row][c4 * 4]) = h4;
          *reinterpret_cast<decltype(l4)*>(&xl[row][c4 * 4]) = l4;
        }
        wait_vm<0>();     // this wave's weight DMA (and the window loads) have landed
        __syncthreads();  // ... every wave's
        if (c + 1 < nchunks) load_x(c + 1);   // in flight under this chunk's MFMAs
        const unsigned long long c1 = tr ? clock64() : 0;
        for (int s = 0; s < a.nks_c; ++s) comp(s);
        if (tr) {
          t_stage += c1 - c0;
          t_comp += clock64() - c1;
        }
      }
    } else {
      for (int c = 0; c < nchunks; ++c) {
        const unsigned long long c0 = tr ? clock64() : 0;
        stage(c);
        const unsigned long long c1 = tr ? clock64() : 0;
        for (int s = 0; s < a.nks_c; ++s) comp(s);
        if (tr) {
          t_stage += c1 - c0;
          t_comp += clock64() - c1;
        }
      }
    }
  }
  // C layout: row (output channel) = 4*(lane>>4) + i, column (time) = lane & 15.  Every epilogue
  // operand is loaded for all tiles first (one memory latency, not one per tile), rows past Tq read
  // row Tq - 1 and are not stored.
  const ConvArgs& a = mc.a[g0];
  float4 add[NTW][MTW];
#pragma unroll
  for (int n = 0; n < NTW; ++n)
#pragma unroll
    for (int m = 0; m < MTW; ++m) add[n][m] = make_float4(0.f, 0.f, 0.f, 0.f);
  size_t off[NTW];
#pragma unroll
  for (int n = 0; n < NTW; ++n) {
    const int q = min(t0 + tl + 16 * n, a.Tq - 1);
    off[n] = ((size_t)b * a.Tout_total + (size_t)q * a.ostride + a.ooff) * a.Cout + (ct0 * 16 + kq / 2);
  }
  float4 bb[MTW];
#pragma unroll
  for (int m = 0; m < MTW; ++m) bb[m] = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int g = g0; g < g1; ++g) {
    const ConvArgs& ag = mc.a[g];
    const float* rs[2] = {ag.res, ag.res2};
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      if (!rs[r]) continue;
      float4 v[NTW][MTW];
#pragma unroll
      for (int n = 0; n < NTW; ++n)
#pragma unroll
        for (int m = 0; m < MTW; ++m) v[n][m] = *reinterpret_cast<const float4*>(rs[r] + off[n] + m * 16);
#pragma unroll
      for (int n = 0; n < NTW; ++n)
#pragma unroll
        for (int m = 0; m < MTW; ++m) {
          add[n][m].x += v[n][m].x; add[n][m].y += v[n][m].y; add[n][m].z += v[n][m].z; add[n][m].w += v[n][m].w;
        }
    }
    if (ag.bias) {
#pragma unroll
      for (int m = 0; m < MTW; ++m) {
        const float4 v = *reinterpret_cast<const float4*>(ag.bias + (ct0 + m) * 16 + kq / 2);
        bb[m].x += v.x; bb[m].y += v.y; bb[m].z += v.z; bb[m].w += v.w;
      }
    }
  }
  if (tr && threadIdx.x == 0) {
    tr[1] = t_stage;
    tr[2] = t_comp;
  }
  float4 gg[MTW];
#pragma unroll
  for (int m = 0; m < MTW; ++m) {
    const int co = (ct0 + m) * 16 + kq / 2;
    gg[m] = a.gadd ? *reinterpret_cast<const float4*>(a.gadd + (size_t)b * a.Cout + co) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int n = 0; n < NTW; ++n) {
    if (t0 + tl + 16 * n >= a.Tq) continue;
#pragma unroll
    for (int m = 0; m < MTW; ++m) {
      float4 v;
      v.x = (acc[m][n][0] + bb[m].x + add[n][m].x) * a.oscale + gg[m].x;
      v.y = (acc[m][n][1] + bb[m].y + add[n][m].y) * a.oscale + gg[m].y;
      v.z = (acc[m][n][2] + bb[m].z + add[n][m].z) * a.oscale + gg[m].z;
      v.w = (acc[m][n][3] + bb[m].w + add[n][m].w) * a.oscale + gg[m].w;
      *reinterpret_cast<float4*>(a.out + off[n] + m * 16) = v;
    }
  }
  if (tr && threadIdx.x == 0) tr[3] = wall_clock64();
}

// One ResBlock1 step with both of its convolutions in one workgroup (models/decoder/ticodec/models.py:90-110):
//   y = x + c2(leaky(c1(leaky(x))))      c1: K taps, dilation d;  c2: K taps, dilation 1;  C -> C channels
// A workgroup owns a time tile [t0, t0 + TW) of one batch row and ALL C output channels (c2 reads every channel of
// c1's output).  Phase A computes c1 on the extended rows [t0 - 8, t0 + TW + 8) (8 >= c2's half width) into LDS as
// leaky'd bf16 hi + lo, zero outside the sequence (c2's zero padding); phase B computes c2 from that LDS tile and
// adds the bias and the residual x.  The intermediate never goes to memory: per step one read of x and one write
// of y instead of x -> t1 -> y through HBM, and one launch instead of two.  Members as in ConvMulti (blockIdx.z =
// b + B * g: the stage's resblock chains side by side); sum != 0: a workgroup runs every member into one c2
// accumulator and stores (sum_g y_g) * oscale + gadd (the chains' last step and their mean, models.py:236-238).
struct PairArgs {
  const float* x;      // [B][T][C] chain input, also the residual
  const bf16_t* w1;    // c1 packed (fo_pack_conv, Cin = Cout = C)
  const float* b1;
  const bf16_t* w2;    // c2 packed
  const float* b2;
  float* out;          // [B][T][C]
  int K, dil, nks_c;
};
struct PairMulti {
  PairArgs a[CONV_MAXG];
  int B, G, sum, T;
  float slope, oscale;
  const float* gadd;   // [B][C] or null
};
constexpr int PAIR_OFF = 8;  // phase A's extra rows on each side (>= (K - 1) / 2 for K <= 11... up to 17)

template <int MTW, int NTW, int CK>
__global__ __launch_bounds__(256) void k_conv_pair(PairMulti pm) {
  constexpr int C = 16 * MTW;
  constexpr int TW = 64 * NTW;
  constexpr int R1 = TW + 2 * PAIR_OFF;       // phase A rows (a multiple of 16)
  constexpr int NT1 = R1 / 16;                // phase A time tiles
  constexpr int NA = (NT1 + 3) / 4;           // phase A tiles per wave (the last round on a few waves)
  constexpr int ROWS = R1 + HALO;             // x window rows
  constexpr int LP = CK + 8, LT = C + 8;
  __shared__ __attribute__((aligned(16))) __bf16 xh[ROWS][LP];
  __shared__ __attribute__((aligned(16))) __bf16 xl[ROWS][LP];
  __shared__ __attribute__((aligned(16))) __bf16 th[R1][LT];
  __shared__ __attribute__((aligned(16))) __bf16 tlo[R1][LT];
  __shared__ __attribute__((aligned(16))) bf16_t wl[MTW * conv_wmax(CK) * 512];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int t0 = blockIdx.x * TW;
  const int g0 = pm.sum ? 0 : (int)blockIdx.z / pm.B;
  const int b = pm.sum ? (int)blockIdx.z : (int)blockIdx.z % pm.B;
  const int g1 = pm.sum ? pm.G : g0 + 1;
  const int T = pm.T;
  const int kq = 8 * (lane >> 4);
  constexpr int NCH = C / CK;

  f32x4 acc2[MTW][NTW];
#pragma unroll
  for (int m = 0; m < MTW; ++m)
#pragma unroll
    for (int n = 0; n < NTW; ++n) acc2[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  // weights of Cin chunk c of a packed conv into wl (LDS-DMA, one fragment per wave-instruction)
  auto stage_w = [&](const bf16_t* wp, int nks_c, int c) {
    const int nks = NCH * nks_c;
    for (int f = wave; f < MTW * nks_c; f += 4) {
      const int m = f / nks_c, st = f - m * nks_c;
      const bf16_t* src = wp + ((size_t)m * nks + c * nks_c + st) * 512 + lane * 8;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)&wl[f * 512], 16, 0, 0);
    }
  };

  for (int g = g0; g < g1; ++g) {
    const PairArgs& a = pm.a[g];
    const int p1 = a.dil * (a.K - 1) / 2, p2 = (a.K - 1) / 2;
    const int span = R1 + a.dil * (a.K - 1);
    const float* xb = a.x + (size_t)b * T * C;
    // ---- phase A: c1 over rows r <-> time t0 - PAIR_OFF + r
    f32x4 acc1[MTW][NA];
#pragma unroll
    for (int m = 0; m < MTW; ++m)
#pragma unroll
      for (int i = 0; i < NA; ++i) acc1[m][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    constexpr int MAXL = (ROWS * (CK / 4) + 255) / 256;
    for (int c = 0; c < NCH; ++c) {
      __syncthreads();  // previous readers of xh / xl / wl are done
      stage_w(a.w1, a.nks_c, c);
      float4 v[MAXL];
#pragma unroll
      for (int i = 0; i < MAXL; ++i) {
        const int e = threadIdx.x + 256 * i;
        const int row = e / (CK / 4), c4 = e % (CK / 4);
        const int ti = t0 - PAIR_OFF - p1 + row;
        v[i] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (e < span * (CK / 4) && ti >= 0 && ti < T)
          v[i] = *reinterpret_cast<const float4*>(xb + (size_t)ti * C + c * CK + c4 * 4);
      }
#pragma unroll
      for (int i = 0; i < MAXL; ++i) {
        const int e = threadIdx.x + 256 * i;
        if (e >= span * (CK / 4)) break;
        const int row = e / (CK / 4), c4 = e % (CK / 4);
        float f[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
        __attribute__((ext_vector_type(4))) __bf16 h4, l4;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          f[q] = f[q] < 0.f ? f[q] * pm.slope : f[q];
          const __bf16 h = (__bf16)f[q];
          h4[q] = h;
          l4[q] = (__bf16)(f[q] - (float)h);
        }
        *reinterpret_cast<decltype(h4)*>(&xh[row][c4 * 4]) = h4;
        *reinterpret_cast<decltype(l4)*>(&xl[row][c4 * 4]) = l4;
      }
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
      for (int s = 0; s < a.nks_c; ++s) {
        const int kk = s * 32 + kq;
        int j = kk / CK;
        const int cil = kk - j * CK;
        if (j > a.K - 1) j = a.K - 1;
        bf16x8 av[MTW];
#pragma unroll
        for (int m = 0; m < MTW; ++m) av[m] = *reinterpret_cast<const bf16x8*>(&wl[(m * a.nks_c + s) * 512 + lane * 8]);
#pragma unroll
        for (int i = 0; i < NA; ++i) {
          const int n = wave + 4 * i;
          if (n >= NT1) continue;
          const int rb = n * 16 + (lane & 15) + j * a.dil;
          const bf16x8 hi = *reinterpret_cast<const bf16x8*>(&xh[rb][cil]);
          const bf16x8 lo = *reinterpret_cast<const bf16x8*>(&xl[rb][cil]);
#pragma unroll
          for (int m = 0; m < MTW; ++m) {
            acc1[m][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[m], hi, acc1[m][i], 0, 0, 0);
            acc1[m][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[m], lo, acc1[m][i], 0, 0, 0);
          }
        }
      }
    }
    // c1 output + bias -> leaky (c2's pre-activation) -> zero outside [0, T) -> bf16 hi + lo tile in LDS
    __syncthreads();  // (the previous member's phase B readers of th / tlo are done)
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int n = wave + 4 * i;
      if (n >= NT1) continue;
      const int r = n * 16 + (lane & 15);
      const int t = t0 - PAIR_OFF + r;
#pragma unroll
      for (int m = 0; m < MTW; ++m) {
        const int co = m * 16 + kq / 2;
        const float4 bb = a.b1 ? *reinterpret_cast<const float4*>(a.b1 + co) : make_float4(0.f, 0.f, 0.f, 0.f);
        float f[4] = {acc1[m][i][0] + bb.x, acc1[m][i][1] + bb.y, acc1[m][i][2] + bb.z, acc1[m][i][3] + bb.w};
        __attribute__((ext_vector_type(4))) __bf16 h4, l4;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float v = f[q] < 0.f ? f[q] * pm.slope : f[q];
          if (t < 0 || t >= T) v = 0.f;
          const __bf16 h = (__bf16)v;
          h4[q] = h;
          l4[q] = (__bf16)(v - (float)h);
        }
        *reinterpret_cast<decltype(h4)*>(&th[r][co]) = h4;
        *reinterpret_cast<decltype(l4)*>(&tlo[r][co]) = l4;
      }
    }
    // ---- phase B: c2 over the workgroup's TW rows, B operands from the c1 tile
    const int tlb = wave * 16 * NTW + (lane & 15);
    for (int c = 0; c < NCH; ++c) {
      __syncthreads();  // th / tlo complete; the previous chunk's wl readers are done
      stage_w(a.w2, a.nks_c, c);
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
      for (int s = 0; s < a.nks_c; ++s) {
        const int kk = s * 32 + kq;
        int j = kk / CK;
        const int cil = kk - j * CK;
        if (j > a.K - 1) j = a.K - 1;
        bf16x8 av[MTW];
#pragma unroll
        for (int m = 0; m < MTW; ++m) av[m] = *reinterpret_cast<const bf16x8*>(&wl[(m * a.nks_c + s) * 512 + lane * 8]);
        const int rb = PAIR_OFF - p2 + tlb + j;
#pragma unroll
        for (int n = 0; n < NTW; ++n) {
          const bf16x8 hi = *reinterpret_cast<const bf16x8*>(&th[rb + 16 * n][c * CK + cil]);
          const bf16x8 lo = *reinterpret_cast<const bf16x8*>(&tlo[rb + 16 * n][c * CK + cil]);
#pragma unroll
          for (int m = 0; m < MTW; ++m) {
            acc2[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[m], hi, acc2[m][n], 0, 0, 0);
            acc2[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[m], lo, acc2[m][n], 0, 0, 0);
          }
        }
      }
    }
  }
  // epilogue: out = (sum_g (c2_g + b2_g + x_g)) * oscale + gadd
  const int tlb = wave * 16 * NTW + (lane & 15);
  float4 add[NTW][MTW], bb[MTW];
#pragma unroll
  for (int n = 0; n < NTW; ++n)
#pragma unroll
    for (int m = 0; m < MTW; ++m) add[n][m] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int m = 0; m < MTW; ++m) bb[m] = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int g = g0; g < g1; ++g) {
    const PairArgs& a = pm.a[g];
#pragma unroll
    for (int n = 0; n < NTW; ++n) {
      const int t = min(t0 + tlb + 16 * n, T - 1);
#pragma unroll
      for (int m = 0; m < MTW; ++m) {
        const float4 v = *reinterpret_cast<const float4*>(a.x + ((size_t)b * T + t) * C + m * 16 + kq / 2);
        add[n][m].x += v.x; add[n][m].y += v.y; add[n][m].z += v.z; add[n][m].w += v.w;
      }
    }
    if (a.b2) {
#pragma unroll
      for (int m = 0; m < MTW; ++m) {
        const float4 v = *reinterpret_cast<const float4*>(a.b2 + m * 16 + kq / 2);
        bb[m].x += v.x; bb[m].y += v.y; bb[m].z += v.z; bb[m].w += v.w;
      }
    }
  }
  float* out = pm.a[g0].out;
#pragma unroll
  for (int n = 0; n < NTW; ++n) {
    const int t = t0 + tlb + 16 * n;
    if (t >= T) continue;
#pragma unroll
    for (int m = 0; m < MTW; ++m) {
      const int co = m * 16 + kq / 2;
      const float4 gg = pm.gadd ? *reinterpret_cast<const float4*>(pm.gadd + (size_t)b * C + co)
                                : make_float4(0.f, 0.f, 0.f, 0.f);
      float4 v;
      v.x = (acc2[m][n][0] + bb[m].x + add[n][m].x) * pm.oscale + gg.x;
      v.y = (acc2[m][n][1] + bb[m].y + add[n][m].y) * pm.oscale + gg.y;
      v.z = (acc2[m][n][2] + bb[m].z + add[n][m].z) * pm.oscale + gg.z;
      v.w = (acc2[m][n][3] + bb[m].w + add[n][m].w) * pm.oscale + gg.w;
      *reinterpret_cast<float4*>(out + ((size_t)b * T + t) * C + co) = v;
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
// One output per thread; the taps x channels weights sit in LDS as fp32, every input row is read as
// float4s (neighbouring threads share K-1 of their K rows, served by L1/L2).
constexpr int POST_MAXW = 4096;
__global__ __launch_bounds__(256) void k_conv_post_cl(const float* x, int B, int T, int C, const bf16_t* w,
                                                      const float* bias, int K, int pad, float slope, float* out) {
  __shared__ float ws[POST_MAXW];  // [K][C]
  for (int i = threadIdx.x; i < K * C; i += 256) ws[i] = bf2f(w[(size_t)(i % C) * K + i / C]);
  __syncthreads();
  const long long total = (long long)B * T;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int b = (int)(e / T), t = (int)(e % T);
    float acc = bias ? bias[0] : 0.f;
    for (int j = 0; j < K; ++j) {
      const int ti = t + j - pad;
      if (ti < 0 || ti >= T) continue;
      const float4* xr = reinterpret_cast<const float4*>(x + ((size_t)b * T + ti) * C);
      const float* wj = ws + j * C;
      for (int c4 = 0; c4 < C / 4; ++c4) {
        const float4 v = xr[c4];
        const float f[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) acc += (f[i] < 0.f ? f[i] * slope : f[i]) * wj[c4 * 4 + i];
      }
    }
    out[e] = tanhf(acc);
  }
}

inline int grid_for(long long n) {
  long long g = (n + 255) / 256;
  return (int)(g > 8192 ? 8192 : (g < 1 ? 1 : g));
}

// Channels per staged Cin chunk: 32, half the LDS of a 64-channel chunk (window and weight buffers), so two or
// three workgroups share a CU and one stages its chunk while another computes: 8-user call 2.11 -> 1.93 ms
// (16: 2.58 ms; profiles/r03i_vocoder_ck_ab.txt).  FO_CONV_CK=16/64 for A/B; the packing reads the same value,
// so weights packed in a process match its launches.
int g_ck_max = 0;
inline int pick_ck(int Cin) {
  if (!g_ck_max) {
    const char* e = getenv("FO_CONV_CK");
    g_ck_max = e ? atoi(e) : 32;
    if (g_ck_max != 16 && g_ck_max != 64) g_ck_max = 32;
  }
  return Cin >= g_ck_max ? g_ck_max : Cin;
}


}  // namespace

extern "C" {

long long fo_conv_pack_elems(int Cout, int Cin, int K) {
  const int CK = pick_ck(Cin);
  const int nks_c = nks_per_chunk(K, CK);
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
  const int nks_c = nks_per_chunk(K, CK);
  const long long total = (long long)(Cout / 16) * (Cin / CK) * nks_c * 64;
  hipLaunchKernelGGL(k_pack_conv, dim3(grid_for(total)), dim3(256), 0, s, W, src_bf16, Cout, Cin, K, CK, nks_c,
                     transposed, Ktot, j0, u, (bf16_t*)out);
  return fo::check_launch("fo_pack_conv");
}

// Stride-1 conv on channel-last activations: x [B][Tin][Cin] -> out [B][Tout_total][Cout] at time
// q * ostride + ooff for q < Tq (Tq = Tin + 2 pad - dil (K-1) for a plain conv), with the fused
// epilogue out = (conv + bias + res + res2) * oscale + gadd[b] (res, res2, gadd optional).
// out must not alias x (other workgroups still read the input window).
static int conv_check(const ConvArgs& a) {
  FO_REQUIRE(a.Cout % 16 == 0 && a.Cin % 16 == 0 && a.Cin >= 16, "fo_conv_cl: Cout=%d Cin=%d", a.Cout, a.Cin);
  FO_REQUIRE(a.K >= 1 && a.K <= CONV_KMAX && a.dil >= 1 && a.dil * (a.K - 1) <= HALO,
             "fo_conv_cl: K=%d dil=%d beyond the LDS halo / weight buffer", a.K, a.dil);
  FO_REQUIRE(a.Tq > 0 && (long long)(a.Tq - 1) * a.ostride + a.ooff < a.Tout_total, "fo_conv_cl: output range");
  FO_REQUIRE((const void*)a.x != (const void*)a.out, "fo_conv_cl: out aliases the input");
  return 0;
}

// One launch of mc.G convolutions (all Cin -> Cout); Tq_max: the longest output range among them.
thread_local unsigned long long* g_conv_trc = nullptr;   // fo_conv_set_trace (probes)

static int conv_launch(ConvMulti& mc, int Tq_max, hipStream_t s) {
  mc.trc = g_conv_trc;
  const int B = mc.B, Cin = mc.a[0].Cin, Cout = mc.a[0].Cout;
  const int CK = pick_ck(Cin);
  const int zg = mc.sum ? 1 : mc.G;
  int MTW = Cout >= 64 ? 4 : Cout / 16;
  int NTW = 8 / MTW;
  // short, wide stages (the first upsampling stages: Tq of a few hundred, 256-512 channels) would put
  // only ~100 workgroups on 256 CUs: take 2 x 2 tiles per wave there (more workgroups, less reuse of
  // the L2-resident weights, which costs little at these sizes)
  if (MTW == 4 && (long long)((Tq_max + 127) / 128) * (Cout / 64) * B * zg < 256) {
    MTW = 2;
    NTW = 2;
  }
  // FO_CONV_HALFT=1 (A/B probe): half the time tile on the narrow late stages (Cout <= 32: 16 or 32 channels,
  // 18k-36k steps per user) -- less LDS and fewer registers per workgroup, more workgroups per CU
  static int halft = -1;
  if (halft < 0) {
    const char* e = getenv("FO_CONV_HALFT");
    halft = (e && e[0] == '1') ? 1 : 0;
  }
  if (halft && MTW <= 2 && NTW == 8 / MTW && CK <= 32) NTW /= 2;
  dim3 grid((Tq_max + 64 * NTW - 1) / (64 * NTW), Cout / (16 * MTW), B * zg);
  if (MTW == 1 && CK == 64) grid.x = (Tq_max + 255) / 256;
  static int pf = -1;   // FO_CONV_PREFETCH=0 / 1: the staged / prefetching chunk loop (A/B)
  if (pf < 0) {
    const char* e = getenv("FO_CONV_PREFETCH");
    pf = (e && e[0] == '1') ? 1 : 0;
  }
#define FO_CONV(A, B, C)                                                                        \
  do {                                                                                          \
    if (mc.trc) hipLaunchKernelGGL((k_conv_cl<A, B, C, true, false>), grid, dim3(256), 0, s, mc); \
    else if (pf) hipLaunchKernelGGL((k_conv_cl<A, B, C, false, true>), grid, dim3(256), 0, s, mc); \
    else hipLaunchKernelGGL((k_conv_cl<A, B, C, false, false>), grid, dim3(256), 0, s, mc);      \
  } while (0)
  if (MTW == 2 && NTW == 2 && CK == 64) FO_CONV(2, 2, 64);
  else if (MTW == 2 && NTW == 2 && CK == 32) FO_CONV(2, 2, 32);
  else if (MTW == 2 && NTW == 2 && CK == 16) FO_CONV(2, 2, 16);
  else if (MTW == 1 && NTW == 4 && CK == 32) FO_CONV(1, 4, 32);
  else if (MTW == 1 && NTW == 4 && CK == 16) FO_CONV(1, 4, 16);
  else if (MTW == 4 && CK == 64) FO_CONV(4, 2, 64);
  else if (MTW == 2 && NTW == 4 && CK == 64) FO_CONV(2, 4, 64);
  else if (MTW == 2 && CK == 32) FO_CONV(2, 4, 32);
  else if (MTW == 1 && CK == 32) FO_CONV(1, 8, 32);
  else if (MTW == 1 && CK == 16) FO_CONV(1, 8, 16);
  else if (MTW == 4 && CK == 32) FO_CONV(4, 2, 32);
  else if (MTW == 4 && CK == 16) FO_CONV(4, 2, 16);
  else if (MTW == 2 && CK == 16) FO_CONV(2, 4, 16);
  else if (MTW == 1 && CK == 64) FO_CONV(1, 4, 64);
  else FO_REQUIRE(false, "fo_conv_cl: no variant for Cout=%d Cin=%d", Cout, Cin);
#undef FO_CONV
  return fo::check_launch("fo_conv_cl");
}

int fo_conv_cl(const float* x, int B, int Cin, int Tin, const void* wp, const float* bias, int Cout, int K, int dil,
               int pad, int Tq, int ostride, int ooff, int Tout_total, int pre_leaky, float slope, float* out,
               const float* res, const float* res2, float oscale, const float* gadd, hipStream_t s) {
  ConvMulti mc{};
  mc.a[0] = ConvArgs{x, (const bf16_t*)wp, bias, out, Cin, Tin, Cout, K, dil, pad, Tq, ostride, ooff, Tout_total,
                     nks_per_chunk(K, pick_ck(Cin)), pre_leaky, slope, res, res2, oscale, gadd};
  mc.B = B;
  mc.G = 1;
  mc.sum = 0;
  if (int rc = conv_check(mc.a[0])) return rc;
  return conv_launch(mc, Tq, s);
}

int fo_conv_cl_multi(const FoConvDesc* d, int G, int B, int Cin, int Cout, int sum, hipStream_t s) {
  FO_REQUIRE(d && G >= 1 && G <= CONV_MAXG && B >= 1, "fo_conv_cl_multi: G=%d (1..%d) B=%d", G, CONV_MAXG, B);
  ConvMulti mc{};
  mc.B = B;
  mc.G = G;
  mc.sum = sum ? 1 : 0;
  int tqmax = 0;
  for (int g = 0; g < G; ++g) {
    const FoConvDesc& e = d[g];
    mc.a[g] = ConvArgs{e.x, (const bf16_t*)e.wp, e.bias, e.out, Cin, e.Tin, Cout, e.K, e.dil, e.pad, e.Tq, e.ostride,
                       e.ooff, e.Tout_total, nks_per_chunk(e.K, pick_ck(Cin)), e.pre_leaky, e.slope, e.res, e.res2,
                       e.oscale, e.gadd};
    if (int rc = conv_check(mc.a[g])) return rc;
    for (int h = 0; h < G; ++h)  // another member's output must not be this one's input (no order inside a launch)
      FO_REQUIRE(h == g || (const void*)d[h].out != (const void*)e.x, "fo_conv_cl_multi: conv %d reads conv %d's output",
                 g, h);
    if (sum) FO_REQUIRE(e.Tq == d[0].Tq, "fo_conv_cl_multi: summed convs need one output range");
    tqmax = e.Tq > tqmax ? e.Tq : tqmax;
  }
  if (!sum)
    for (int g = 0; g < G; ++g)
      for (int h = g + 1; h < G; ++h)
        FO_REQUIRE(d[g].out != d[h].out || d[g].ostride > 1, "fo_conv_cl_multi: convs %d and %d write one output", g, h);
  return conv_launch(mc, tqmax, s);
}

int fo_conv_pair_multi(const FoPairDesc* d, int G, int B, int C, int T, int sum, float slope, float oscale,
                       const float* gadd, hipStream_t s) {
  FO_REQUIRE(d && G >= 1 && G <= CONV_MAXG && B >= 1 && T >= 1, "fo_conv_pair_multi: G=%d B=%d T=%d", G, B, T);
  FO_REQUIRE(C == 16 || C == 32 || C == 64, "fo_conv_pair_multi: C=%d (16, 32 or 64)", C);
  FO_REQUIRE(pick_ck(C) == (C >= 32 ? 32 : 16), "fo_conv_pair_multi: needs the default 32-channel chunks");
  PairMulti pm{};
  pm.B = B;
  pm.G = G;
  pm.sum = sum ? 1 : 0;
  pm.T = T;
  pm.slope = slope;
  pm.oscale = oscale;
  pm.gadd = gadd;
  for (int g = 0; g < G; ++g) {
    const FoPairDesc& e = d[g];
    FO_REQUIRE(e.x && e.w1 && e.w2 && e.out, "fo_conv_pair_multi: member %d lacks a pointer", g);
    FO_REQUIRE(e.K >= 1 && e.K <= CONV_KMAX && e.K % 2 == 1 && e.dil >= 1 && e.dil * (e.K - 1) <= HALO &&
               (e.K - 1) / 2 <= PAIR_OFF, "fo_conv_pair_multi: K=%d dil=%d", e.K, e.dil);
    FO_REQUIRE((const void*)e.out != (const void*)e.x, "fo_conv_pair_multi: out aliases the input");
    for (int h = 0; h < G; ++h)
      FO_REQUIRE(h == g || (const void*)d[h].out != (const void*)e.x, "fo_conv_pair_multi: member %d reads member %d's "
                 "output", g, h);
    if (!sum)
      for (int h = g + 1; h < G; ++h)
        FO_REQUIRE(d[h].out != e.out, "fo_conv_pair_multi: members %d and %d write one output", g, h);
    pm.a[g] = PairArgs{e.x, (const bf16_t*)e.w1, e.b1, (const bf16_t*)e.w2, e.b2, e.out, e.K, e.dil,
                       nks_per_chunk(e.K, pick_ck(C))};
  }
  const int zg = sum ? 1 : G;
  if (C == 16) {
    hipLaunchKernelGGL((k_conv_pair<1, 4, 16>), dim3((T + 255) / 256, 1, B * zg), dim3(256), 0, s, pm);
  } else if (C == 32) {
    hipLaunchKernelGGL((k_conv_pair<2, 2, 32>), dim3((T + 127) / 128, 1, B * zg), dim3(256), 0, s, pm);
  } else {
    hipLaunchKernelGGL((k_conv_pair<4, 2, 32>), dim3((T + 127) / 128, 1, B * zg), dim3(256), 0, s, pm);
  }
  return fo::check_launch("fo_conv_pair_multi");
}

int fo_conv_set_trace(void* trace) {
  g_conv_trc = reinterpret_cast<unsigned long long*>(trace);
  return 0;
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
  FO_REQUIRE(C % 4 == 0 && K * C <= POST_MAXW, "fo_conv_post_cl: C=%d K=%d", C, K);
  const long long n = (long long)B * T;
  hipLaunchKernelGGL(k_conv_post_cl, dim3(grid_for(n)), dim3(256), 0, s, x, B, T, C, (const bf16_t*)w, bias, K, pad,
                     slope, out);
  return fo::check_launch("fo_conv_post_cl");
}

}  // extern "C"
