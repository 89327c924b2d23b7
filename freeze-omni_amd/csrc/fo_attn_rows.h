// Multi-row paged attention body (AttnArgs, the MFMA tile loop, the in-launch split merge), shared by the
// attention launch (fo_attn.hip: k_attn_mfma) and the q|k|v projection that runs its kv group's attention in
// the same launch (fo_gemm.hip: k_gemm_qkv_attn).  Included inside each file's anonymous namespace.
#pragma once

struct AttnArgs {
  const float* q;          // [T][H*hd], rotated
  const int* items;        // [n_items][3]: sequence, first token, token count (a sequence's tokens are contiguous)
  const int* tok_nvis;     // keys visible to each query token (causal: own cache index + 1; full: all)
  const int* block_table;  // [S][maxb]
  const float* kc;
  const float* vc;
  float* part_ml;  // [T*H][nsplit][2]   (nsplit > 1)
  float* part_o;   // [T*H][nsplit][hd]  (nsplit > 1)
  float* out;      // [T][H*hd]
  int H, KVH, PS, maxb, nsplit;
  float scale;
  // in-launch merge: a work item uses min(nsplit, ceil(keys / kps)) splits, chosen from its own key
  // count at run time (one captured graph serves a context as it grows); the last split to finish
  // (arrival ticket cnt[item][kv head], reset by that split) merges the partials -- no combine launch
  int* cnt;        // nullable: static nsplit splits + k_attn_combine
  int kps;
  int tnu;         // items NULL: tokens per item (item b = sequence b, tokens b*tnu .. b*tnu + tnu - 1)
  // out also written packed for the next GEMM (<= 64 tokens; xpack_store: fo_attention_set_opack), or nullptr
  uint16_t* oph;
  uint16_t* opl;
  int prb;         // its row blocks: ceil(T / 16)
  unsigned long long* trc;   // probes (fo_attention_set_trace): per workgroup {start, staged, tiles done, stored, end,
                             // ran, loads landed}
  int reps;                  // probe build only: the body runs reps times in a row (FO_ATTN_TRACE_REPS; the stamps
                             // are the last pass's: the same code again, its instructions already fetched)
};

constexpr int KT = 64;      // keys per LDS tile (one key per lane in the score phase)
constexpr int MAXPG = 256;  // pages of one split staged in LDS (fo_attn_nsplit keeps splits <= 4096 keys)

// fp32 -> bf16 hi + lo: two bf16 operands whose sum carries ~16 mantissa bits
__device__ __forceinline__ void split8(const float* f, bf16x8& hi, bf16x8& lo) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const __bf16 h = (__bf16)f[i];
    hi[i] = h;
    lo[i] = (__bf16)(f[i] - (float)h);
  }
}

// sum / max over the 16 lanes of a row group by DPP within the 16-lane row (VALU, no LDS round trip): lanes l^1, l^2
// (quad_perm), then the other quad (row_half_mirror) and the other half (row_mirror) -- after the quad steps every lane
// of a quad holds the same value, so each step adds the same operands in the same order as the l^4 / l^8 butterfly
// (the same result bit for bit)
template <int CTRL>
__device__ __forceinline__ float dpp16(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}
__device__ __forceinline__ float row16_max(float v) {
  v = fmaxf(v, dpp16<0xB1>(v));    // quad_perm [1, 0, 3, 2]
  v = fmaxf(v, dpp16<0x4E>(v));    // quad_perm [2, 3, 0, 1]
  v = fmaxf(v, dpp16<0x141>(v));   // row_half_mirror
  return fmaxf(v, dpp16<0x140>(v));  // row_mirror
}
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp16<0xB1>(v);
  v += dpp16<0x4E>(v);
  v += dpp16<0x141>(v);
  return v + dpp16<0x140>(v);
}

// Split `sp` of work item `it` has written its partial (part_o / part_ml): publish it and take an
// arrival ticket; the split that draws ns - 1 merges all ns partials of the item's R rows with
// k_attn_combine's arithmetic and resets the ticket for the next launch.  Protocol: every wave drains
// its stores and lane 0 takes the ticket behind a workgroup barrier (correct for any placement of the splits
// over XCDs).  SC (the 8-wave kernel: one workgroup per CU): the partials were stored write-through (st_wt) and
// are read back with sc1 loads, no fences (fo_common.h); otherwise lane 0 releases at agent scope before the
// relaxed ticket add and the merging split acquires at agent scope before plain reads.
// last_s / w_s: the kernel's existing LDS (no second __shared__ object for the flag).
template <bool SC>
__device__ __forceinline__ void st_part(float* p, float v) {
  if constexpr (SC) st_wt(p, v);
  else *p = v;
}
template <int HD, bool SC>
__device__ void attn_arrive_and_merge(const AttnArgs& a, int it, int kvh, int ns, int t0, int R, int G,
                                      int& last_s, float* w_s) {
  const int tid = threadIdx.x;
  int* ticket = a.cnt + (size_t)it * a.KVH + kvh;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    if constexpr (!SC) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const int old = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last_s = old == ns - 1;
  }
  __syncthreads();
  if (!last_s) return;
  if (tid == 0) {
    if constexpr (!SC) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  const __amdgpu_buffer_rsrc_t rml = rsrc_of(a.part_ml), rpo = rsrc_of(a.part_o);
  // a partial's element: an sc1 load (SC) or a plain one after the acquire
  auto ml_at = [&](size_t off) { return SC ? ld_sc1(rml, off) : a.part_ml[off]; };
  auto po_at = [&](size_t off) { return SC ? ld_sc1(rpo, off) : a.part_o[off]; };
  // per row: split weights exp(m_q - M) (0 for empty splits) and 1 / l into LDS (w_s: [16][KT + 4], the kernel's P
  // tile, ns <= KT).  The partials were written by other XCDs' workgroups, so every read is a memory-side round trip:
  // the loads are issued in groups of MQ splits (x EU outputs per thread below) before any of them is used, and the
  // sums still run in split order (the same result bit for bit as a serial loop).
  constexpr int MQ = 8, EU = 4;
  for (int r = tid; r < R; r += blockDim.x) {
    const size_t th = (size_t)(t0 + r / G) * a.H + kvh * G + r % G;
    const size_t mlo = th * a.nsplit * 2;
    float M = -INFINITY;
    for (int q0 = 0; q0 < ns; q0 += MQ) {
      float2 v[MQ];
#pragma unroll
      for (int j = 0; j < MQ; ++j)
        v[j] = q0 + j < ns ? make_float2(ml_at(mlo + 2 * (q0 + j)), ml_at(mlo + 2 * (q0 + j) + 1)) : make_float2(0.f, 0.f);
#pragma unroll
      for (int j = 0; j < MQ; ++j)
        if (v[j].y > 0.f) M = fmaxf(M, v[j].x);
    }
    float l = 0.f;
    for (int q0 = 0; q0 < ns; q0 += MQ) {   // (second pass: cache hits)
      float2 v[MQ];
#pragma unroll
      for (int j = 0; j < MQ; ++j)
        v[j] = q0 + j < ns ? make_float2(ml_at(mlo + 2 * (q0 + j)), ml_at(mlo + 2 * (q0 + j) + 1)) : make_float2(0.f, 0.f);
#pragma unroll
      for (int j = 0; j < MQ; ++j) {
        if (q0 + j >= ns) break;
        const float w = v[j].y > 0.f ? expf(v[j].x - M) : 0.f;
        if (v[j].y > 0.f) l += v[j].y * w;
        w_s[r * (KT + 4) + q0 + j] = w;
      }
    }
    w_s[r * (KT + 4) + KT] = 1.f / l;
  }
  __syncthreads();
  const int RH = R * HD;
  for (int e0 = tid; e0 < RH; e0 += EU * blockDim.x) {
    size_t po[EU];
    const float* w[EU];
    size_t tho[EU];
    float o[EU];
#pragma unroll
    for (int u = 0; u < EU; ++u) {
      const int e = min(e0 + u * (int)blockDim.x, RH - 1);
      const int r = e / HD, d = e - (e / HD) * HD;
      const size_t th = (size_t)(t0 + r / G) * a.H + kvh * G + r % G;
      po[u] = th * a.nsplit * HD + d;
      w[u] = w_s + r * (KT + 4);
      tho[u] = th * HD + d;
      o[u] = 0.f;
    }
    for (int q0 = 0; q0 < ns; q0 += MQ) {
      float pv[EU][MQ];
#pragma unroll
      for (int u = 0; u < EU; ++u)
#pragma unroll
        for (int j = 0; j < MQ; ++j) {
          const int q = q0 + j;
          pv[u][j] = q < ns && w[u][q] != 0.f ? po_at(po[u] + (size_t)q * HD) : 0.f;
        }
#pragma unroll
      for (int u = 0; u < EU; ++u)
#pragma unroll
        for (int j = 0; j < MQ; ++j) {
          const int q = q0 + j;
          if (q < ns && w[u][q] != 0.f) o[u] += pv[u][j] * w[u][q];
        }
    }
#pragma unroll
    for (int u = 0; u < EU; ++u) {
      if (e0 + u * (int)blockDim.x >= RH) break;
      const float y = o[u] * w[u][KT];
      a.out[tho[u]] = y;
      if (a.oph) xpack_store(a.oph, a.opl, (int)(tho[u] / HD / a.H), (int)((tho[u] / HD) % a.H) * HD + (int)(tho[u] % HD),
                             y, a.prb);
    }
  }
}

// One work item = up to 16 query rows (a sequence's batch tokens x the GQA group sharing one kv head)
// against that kv head, over split `sp` of the sequence's keys, on the matrix cores:
//   S = Q K^T   (A = Q rows, B = K rows read straight from the paged cache in B-fragment order)
//   O = P V     (A = P through LDS, B = V staged in LDS as [key][d])
// 64-key tiles, one 16-key column block per wave; K and V of the next tile are loaded into registers
// while the current tile computes.  Every fp32 operand is split into bf16 hi + lo and each product
// uses three MFMAs (hi*hi + hi*lo + lo*hi), so scores and outputs keep ~fp32 accuracy.  Online
// softmax per row with the running max exchanged across the 4 waves through LDS.
// RT: 16-row query tiles per item (2: up to 32 rows share the K / V loads); TR: the probe build with per-workgroup
// clocks (a.trc) -- a compile-time switch: the runtime-null hook cost the product launches ~6 % (r05zz vs r05m)
template <int HD, int NW, int RT = 1, bool TR = false>
__device__ __forceinline__ void attn_rows_body(const AttnArgs& a, const int it, const int kvh, const int sp) {
  constexpr int KT = 16 * NW;           // keys per tile: one 16-key column block per wave
  constexpr int NTH = NW * 64;
  constexpr int DC = HD / 32;            // 32-wide d chunks (score k-steps)
  constexpr int NTILE = HD / 16;         // 16-wide d tiles of the output
  constexpr int NTW = (NTILE + NW - 1) / NW;   // output tiles per wave
  constexpr int VP = HD + 2;             // V row pitch: the 4 key groups of a B fragment hit distinct banks
  constexpr int VL = KT * HD / 4 / NTH;  // float4 of V per thread per tile
  constexpr bool SC = NW == 8;           // one workgroup per CU: the fence-free split hand-off (attn_arrive_and_merge)
  __shared__ float v_s[KT][VP];
  // (at least 64 + 4 wide: attn_arrive_and_merge reuses it as its [16][64 + 4] weight table)
  __shared__ float p_s[16 * RT][(KT > 64 ? KT : 64) + 4];
  __shared__ float mx_s[NW][16 * RT];
  __shared__ float l_s[NW][16 * RT];
  __shared__ int nvis_s[16 * RT];
  // RT > 1: the Q fragments live in LDS (every wave uses the same ones; in registers they would spill)
  constexpr bool QL = RT > 1;
  __shared__ bf16x8 qf_s[QL ? RT : 1][QL ? DC : 1][2][64];
  __shared__ int pg_s[MAXPG];

  // items NULL: a uniform batch (tnu tokens per sequence, in sequence order) -- no item-table round trip
  const int seq = a.items ? a.items[3 * it] : it, t0 = a.items ? a.items[3 * it + 1] : it * a.tnu;
  const int tn = a.items ? a.items[3 * it + 2] : a.tnu;
  const int G = a.H / a.KVH;
  const int R = tn * G;  // <= 16 RT
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int grp = lane >> 4, col = lane & 15;
  const int* bt = a.block_table + (size_t)seq * a.maxb;
  unsigned long long* const tr =
      TR ? a.trc + 32 * (size_t)(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z)) : nullptr;
  if (tr && tid == 0) tr[0] = wall_clock64();
  // a split slot past the item's own split count leaves before its q / block-table loads: a captured graph's grid
  // carries nsplit slots per item for the longest context it will see, so at short contexts most are empty (the text
  // step: 16 slots, 1-2 used).  Split 0 always runs and keeps the loads-first order below.
  if (a.cnt && sp > 0 && !(TR)) {
    int Lm = 0;
    for (int i = 0; i < tn; ++i) Lm = max(Lm, a.tok_nvis[t0 + i]);
    const int need = (Lm + MAXPG * a.PS - 1) / (MAXPG * a.PS);
    if (sp >= min(a.nsplit, max(need, max(1, (Lm + a.kps - 1) / a.kps)))) return;
  }
  // this lane's q row slices, requested before anything that waits (they depend only on t0)
  float4 qraw[RT][2 * DC];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    const int r = min(16 * rt + col, R - 1);
    const float* qr = a.q + ((size_t)(t0 + r / G) * a.H + kvh * G + r % G) * HD + 8 * grp;
#pragma unroll
    for (int c = 0; c < DC; ++c) {
      qraw[rt][2 * c] = *reinterpret_cast<const float4*>(qr + 32 * c);
      qraw[rt][2 * c + 1] = *reinterpret_cast<const float4*>(qr + 32 * c + 4);
    }
  }
  // a block-table row that fits is staged whole, requested together with the key counts (no wait for
  // this split's page range first); longer rows stage the split's pages once the range is known
  const bool whole = a.maxb <= MAXPG;
  if (whole)
    for (int i = tid; i < a.maxb; i += NTH) pg_s[i] = bt[i];
  int Lmax = 0;
  for (int i = 0; i < tn; ++i) Lmax = max(Lmax, a.tok_nvis[t0 + i]);
  int ns = a.nsplit;
  if (a.cnt) {
    // never fewer splits than keep each within the LDS page table (fo_attn_nsplit's `need` term): a large
    // keys_per_split on a long sequence would otherwise take the poison branch below
    const int need = (Lmax + MAXPG * a.PS - 1) / (MAXPG * a.PS);
    ns = min(ns, max(need, max(1, (Lmax + a.kps - 1) / a.kps)));
    if (sp >= ns) return;  // beyond this item's splits: never counted, never read
  }
  const int per = ((Lmax + ns - 1) / ns + KT - 1) / KT * KT;
  const int c0 = sp * per, c1 = min(Lmax, c0 + per);
  if (c0 >= c1) {  // empty split: neutral partial
    for (int r = tid; r < R; r += NTH) {
      const size_t o = ((size_t)(t0 + r / G) * a.H + kvh * G + r % G) * a.nsplit + sp;
      st_part<SC>(a.part_ml + o * 2, -INFINITY);
      st_part<SC>(a.part_ml + o * 2 + 1, 0.f);
    }
    if (a.cnt) attn_arrive_and_merge<HD, SC>(a, it, kvh, ns, t0, R, G, nvis_s[0], &p_s[0][0]);
    return;
  }
  const int pb0 = c0 / a.PS, npg = (c1 - 1) / a.PS - pb0 + 1;
  if (npg > MAXPG || (whole && (c1 - 1) / a.PS >= a.maxb)) {  // host contract broken: poison, never read wrong keys
    // the item's rows become NaN wherever they are read: one split writes out (and the packed copy the next GEMM
    // reads) directly; a split of several publishes a poisoned partial (m = +inf, l = 1, o = NaN: every merge weight
    // turns NaN) and still arrives, so the in-launch merge runs and the tickets stay balanced for the next launch
    if (a.nsplit == 1) {
      for (int e = tid; e < R * HD; e += NTH) {
        const int r = e / HD, d = e - r * HD;
        const size_t th = (size_t)(t0 + r / G) * a.H + kvh * G + r % G;
        a.out[th * HD + d] = NAN;
        if (a.oph) xpack_store(a.oph, a.opl, (int)(th / a.H), (int)(th % a.H) * HD + d, NAN, a.prb);
      }
      return;
    }
    for (int e = tid; e < R * HD; e += NTH) {
      const int r = e / HD, d = e - r * HD;
      const size_t th = (size_t)(t0 + r / G) * a.H + kvh * G + r % G;
      st_part<SC>(a.part_o + (th * a.nsplit + sp) * HD + d, NAN);
      if (d == 0) {
        st_part<SC>(a.part_ml + (th * a.nsplit + sp) * 2, INFINITY);
        st_part<SC>(a.part_ml + (th * a.nsplit + sp) * 2 + 1, 1.f);
      }
    }
    if (a.cnt) attn_arrive_and_merge<HD, SC>(a, it, kvh, ns, t0, R, G, nvis_s[0], &p_s[0][0]);
    return;
  }
  const int pb = whole ? 0 : pb0;  // pg_s holds pages pb..
  if (!whole)
    for (int i = tid; i < npg; i += NTH) pg_s[i] = bt[pb + i];
  if (tid < 16 * RT) nvis_s[tid] = tid < R ? a.tok_nvis[t0 + tid / G] : 0;

  // Q as A fragments: row = col (lane & 15), d = 32 c + 8 grp; rows >= R are zero
  bf16x8 qh[QL ? 1 : RT][DC], ql[QL ? 1 : RT][DC];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
#pragma unroll
    for (int c = 0; c < DC; ++c) {
      float f[8];
      const float4 x0 = qraw[rt][2 * c];
      const float4 x1 = qraw[rt][2 * c + 1];
      const float sc = 16 * rt + col < R ? a.scale : 0.f;
      f[0] = x0.x * sc; f[1] = x0.y * sc; f[2] = x0.z * sc; f[3] = x0.w * sc;
      f[4] = x1.x * sc; f[5] = x1.y * sc; f[6] = x1.z * sc; f[7] = x1.w * sc;
      if constexpr (QL) {
        bf16x8 h, l;
        split8(f, h, l);
        if (wave == 0) {
          qf_s[rt][c][0][lane] = h;
          qf_s[rt][c][1][lane] = l;
        }
      } else {
        split8(f, qh[rt][c], ql[rt][c]);
      }
    }
  }
  __syncthreads();  // pg_s, nvis_s
  if (tr && tid == 0) tr[1] = wall_clock64();

  const size_t head_off = (size_t)kvh * a.PS * HD;
  const size_t page_sz = (size_t)a.KVH * a.PS * HD;
  float4 kA[2 * DC], vA[VL], kB[2 * DC], vB[VL];   // two tiles' K / V in flight (ping-pong)
  // K: this lane's key (16 per wave) x its 8-wide d slices; V: cooperative 16-B rows for LDS
#define FO_ATTN_LOAD(kreg, vreg, K0)                                                                      \
  {                                                                                                       \
    const int pk = min((K0) + 16 * wave + col, c1 - 1);                                                   \
    const float* kr = a.kc + (size_t)pg_s[pk / a.PS - pb] * page_sz + head_off + (size_t)(pk % a.PS) * HD \
                      + 8 * grp;                                                                          \
    _Pragma("unroll") for (int c = 0; c < DC; ++c) {                                                      \
      kreg[2 * c] = *reinterpret_cast<const float4*>(kr + 32 * c);                                        \
      kreg[2 * c + 1] = *reinterpret_cast<const float4*>(kr + 32 * c + 4);                                \
    }                                                                                                     \
    _Pragma("unroll") for (int i = 0; i < VL; ++i) {                                                      \
      const int e = tid + NTH * i, j = e / (HD / 4), d4 = e % (HD / 4);                                   \
      const int pv = min((K0) + j, c1 - 1);                                                               \
      vreg[i] = *reinterpret_cast<const float4*>(a.vc + (size_t)pg_s[pv / a.PS - pb] * page_sz + head_off \
                                                 + (size_t)(pv % a.PS) * HD + d4 * 4);                    \
    }                                                                                                     \
  }

  float m_run[RT][4], l_lane[RT][4];
  f32x4 acc[RT][NTW];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
#pragma unroll
    for (int i = 0; i < 4; ++i) { m_run[rt][i] = -INFINITY; l_lane[rt][i] = 0.f; }
#pragma unroll
    for (int n = 0; n < NTW; ++n) acc[rt][n] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  // tile t's loads are issued while tile t - 1 computes and two tiles are in flight from the start, so a
  // 256-key split waits for one round of memory, not two
  FO_ATTN_LOAD(kA, vA, c0)
  if (c0 + KT < c1) FO_ATTN_LOAD(kB, vB, c0 + KT)
  if constexpr (TR) {   // probe: when this wave's first tiles have landed
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (tr && tid == 0) tr[6] = wall_clock64();
  }
  auto tile = [&](float4 (&kreg)[2 * DC], float4 (&vreg)[VL], const int k0) {
    __syncthreads();  // the previous tile's p_s / v_s readers are done
#pragma unroll
    for (int i = 0; i < VL; ++i) {
      const int e = tid + NTH * i, j = e / (HD / 4), d4 = e % (HD / 4);
      *reinterpret_cast<float2*>(&v_s[j][d4 * 4]) = make_float2(vreg[i].x, vreg[i].y);
      *reinterpret_cast<float2*>(&v_s[j][d4 * 4 + 2]) = make_float2(vreg[i].z, vreg[i].w);
    }
    bf16x8 kh[DC], kl[DC];
#pragma unroll
    for (int c = 0; c < DC; ++c) {
      const float f[8] = {kreg[2 * c].x, kreg[2 * c].y, kreg[2 * c].z, kreg[2 * c].w,
                          kreg[2 * c + 1].x, kreg[2 * c + 1].y, kreg[2 * c + 1].z, kreg[2 * c + 1].w};
      split8(f, kh[c], kl[c]);
    }
    if (tr && tid == 0 && k0 == c0) tr[7] = wall_clock64();
    if (k0 + 2 * KT < c1) FO_ATTN_LOAD(kreg, vreg, k0 + 2 * KT)
    // S[r = 16 rt + 4 grp + i][key = k0 + 16 wave + col]
    f32x4 s[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      s[rt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < DC; ++c) {
        const bf16x8 qhv = QL ? qf_s[QL ? rt : 0][QL ? c : 0][0][lane] : qh[QL ? 0 : rt][c];
        const bf16x8 qlv = QL ? qf_s[QL ? rt : 0][QL ? c : 0][1][lane] : ql[QL ? 0 : rt][c];
        s[rt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qhv, kh[c], s[rt], 0, 0, 0);
        s[rt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qhv, kl[c], s[rt], 0, 0, 0);
        s[rt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qlv, kh[c], s[rt], 0, 0, 0);
      }
    }
    const int key = k0 + 16 * wave + col;
    bool valid[RT][4];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      float mw[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        valid[rt][i] = key < c1 && key < nvis_s[16 * rt + 4 * grp + i];
        mw[i] = row16_max(valid[rt][i] ? s[rt][i] : -INFINITY);
      }
      if (col == 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) mx_s[wave][16 * rt + 4 * grp + i] = mw[i];
      }
    }
    if (tr && lane == 0 && k0 == c0) tr[16 + wave] = wall_clock64();   // each wave's arrival at the max exchange
    __syncthreads();
    if (tr && tid == 0 && k0 == c0) tr[8] = wall_clock64();
    float alpha[RT][4];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 16 * rt + 4 * grp + i;
        float tm = mx_s[0][r];
#pragma unroll
        for (int w = 1; w < NW; ++w) tm = fmaxf(tm, mx_s[w][r]);
        const float mn = fmaxf(m_run[rt][i], tm);
        alpha[rt][i] = (m_run[rt][i] == mn) ? 1.f : expf(m_run[rt][i] - mn);
        m_run[rt][i] = mn;
        const float p = valid[rt][i] ? expf(s[rt][i] - mn) : 0.f;
        l_lane[rt][i] = l_lane[rt][i] * alpha[rt][i] + p;
        p_s[r][16 * wave + col] = p;
      }
    }
    __syncthreads();  // p_s and v_s complete
    if (tr && tid == 0 && k0 == c0) tr[9] = wall_clock64();
    // O[r][d] += P[r][:] V[:][d] for this wave's d tiles (one V fragment split serves every row tile)
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int n = 0; n < NTW; ++n) {
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[rt][n][i] *= alpha[rt][i];
      }
#pragma unroll
    for (int kc = 0; kc < KT / 32; ++kc) {
      bf16x8 ph[RT], pl[RT];
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        const float4 x0 = *reinterpret_cast<const float4*>(&p_s[16 * rt + col][32 * kc + 8 * grp]);
        const float4 x1 = *reinterpret_cast<const float4*>(&p_s[16 * rt + col][32 * kc + 8 * grp + 4]);
        const float f[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
        split8(f, ph[rt], pl[rt]);
      }
#pragma unroll
      for (int n = 0; n < NTW; ++n) {
        const int dt = wave + NW * n;
        if (dt < NTILE) {
          float f[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) f[e] = v_s[32 * kc + 8 * grp + e][16 * dt + col];
          bf16x8 vh, vl;
          split8(f, vh, vl);
#pragma unroll
          for (int rt = 0; rt < RT; ++rt) {
            acc[rt][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ph[rt], vh, acc[rt][n], 0, 0, 0);
            acc[rt][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ph[rt], vl, acc[rt][n], 0, 0, 0);
            acc[rt][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pl[rt], vh, acc[rt][n], 0, 0, 0);
          }
        }
      }
    }
    if (tr && tid == 0 && k0 == c0) tr[10] = wall_clock64();
  };
  for (int k0 = c0; k0 < c1; k0 += 2 * KT) {
    tile(kA, vA, k0);
    if (k0 + KT < c1) tile(kB, vB, k0 + KT);
  }
#undef FO_ATTN_LOAD
  if (tr && tid == 0) tr[2] = wall_clock64();
  // row sums: 16 lanes of the row group, then the waves
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    float lw[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) lw[i] = row16_sum(l_lane[rt][i]);
    if (col == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) l_s[wave][16 * rt + 4 * grp + i] = lw[i];
    }
  }
  __syncthreads();
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = 16 * rt + 4 * grp + i;
    if (r >= R) continue;
    float l = l_s[0][r];
#pragma unroll
    for (int w = 1; w < NW; ++w) l += l_s[w][r];
    const size_t th = (size_t)(t0 + r / G) * a.H + kvh * G + r % G;
#pragma unroll
    for (int n = 0; n < NTW; ++n) {
      const int dt = wave + NW * n;
      if (dt >= NTILE) continue;
      const int d = 16 * dt + col;
      if (ns == 1) {
        a.out[th * HD + d] = acc[rt][n][i] / l;
        if (a.oph) xpack_store(a.oph, a.opl, (int)(th / a.H), (int)(th % a.H) * HD + d, acc[rt][n][i] / l, a.prb);
      } else {
        st_part<SC>(a.part_o + (th * a.nsplit + sp) * HD + d, acc[rt][n][i]);
      }
    }
    if (ns > 1 && wave == 0 && col == 0) {
      st_part<SC>(a.part_ml + (th * a.nsplit + sp) * 2, m_run[rt][i]);
      st_part<SC>(a.part_ml + (th * a.nsplit + sp) * 2 + 1, l);
    }
  }
  if (tr && tid == 0) tr[3] = wall_clock64();
  if (a.cnt && ns > 1) attn_arrive_and_merge<HD, SC>(a, it, kvh, ns, t0, R, G, nvis_s[0], &p_s[0][0]);
  if (tr && tid == 0) {
    tr[4] = wall_clock64();
    tr[5] = 1 + (unsigned long long)ns;   // (nonzero: this workgroup ran the tile loop)
  }
}

