/* fo_hip.h - C ABI of the Freeze-Omni MI355X hot path (libfo_hip.so).
 *
 * Conventions: every function returns 0 on success, <0 on failure (-1 HIP error,
 * -2 bad argument); fo_last_error() returns the message.  All pointers are device
 * pointers unless noted; all work is enqueued on the given hipStream_t and is
 * asynchronous.  bf16 tensors are raw uint16 storage.  No torch types cross this ABI.
 *
 * The reference (TheDoctor-JI/Freeze-Omni) is pure Python on torch/transformers, so it has
 * no FFI of its own; each entry below names the reference call site whose computation it
 * replaces.  The Python layer in freeze-omni_amd/models mirrors the reference API on top.
 */
#ifndef FO_HIP_H
#define FO_HIP_H
#include <hip/hip_runtime.h>
#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------- plumbing */
int fo_version(void);
int fo_last_error(char* buf, int len);
int fo_device_info(int dev, char* name, int len, int* n_cu, long long* hbm_bytes);
int fo_graph_begin(hipStream_t s);
int fo_graph_end(hipStream_t s, void** exec_out);
int fo_graph_launch(void* exec, hipStream_t s);
int fo_graph_destroy(void* exec);
int fo_stream_create(void** s_out);
// level > 0: the device's greatest stream priority (the speech streams, fo/ops.py engine_stream);
// level < 0: its least; 0: the default
int fo_stream_create_prio(void** s_out, int level);
int fo_stream_priority_range(int* least, int* greatest);
/* a blocking stream restricted to the CUs set in mask (nwords 32-bit words; hipExtStreamCreateWithCUMask) */
int fo_stream_create_cumask(void** s_out, const unsigned* mask, int nwords);
int fo_stream_destroy(void* s);
int fo_stream_wait_event(hipStream_t s, void* ev);
int fo_host_alloc(long long bytes, void** host_ptr, void** dev_ptr);
int fo_host_free(void* host_ptr);
int fo_event_sync(void* ev);
int fo_event_query(void* ev);
int fo_event_create(void** ev);
int fo_event_record(void* ev, hipStream_t s);
int fo_event_elapsed_ms(void* a, void* b, float* ms);
int fo_event_destroy(void* ev);

/* ---------------------------------------------------------------- linear layers
 * Replaces torch.nn.Linear under bf16 autocast on every hot-path linear:
 *   Qwen2 q/k/v/o/gate/up/down + lm_head (models/audioLLM.py:482, transformers Qwen2 layers),
 *   encoder linears (models/encoder/attention.py:411-413,433,459; :143; transformer.py:343),
 *   adapter conv/project (models/adapter.py:670,679), TTS Llama layers + out_fnn
 *   (models/decoder/decoder.py:299-311,346).
 * W is packed once by fo_pack_weight into MFMA fragment order. */
/* fo_gemm with RMSNorm fused across the residual update (Qwen2RMSNorm / LlamaRMSNorm,
 * models/audioLLM.py:479-484, models/decoder/decoder.py:142-153): a producer GEMM (sout != 0) also
 * writes per-row partial sums of squares of Y per workgroup column group (*sgroups of them) and
 * yg = Y * gnext (gamma of the next norm); a consumer GEMM (rstats != 0) takes yg as X and scales its
 * result rows by rsqrt(sum / K + eps) before bias / activation / SwiGLU. */
int fo_gemm_rms(const void* X, int x_f32, int ldx, int M, int K, const void* Wp, int N, int swiglu, const float* bias,
                void* Y, int ldy, int act, int residual, float* ws, long long ws_floats, int* counters, int splitk,
                const float* rstats, int rgroups, float eps, float* sout, const float* gnext, float* yg,
                int* sgroups, hipStream_t stream);
/* The fused q|k|v projection of a Qwen2 / Llama attention layer with bias, rotate_half RoPE and the
 * paged-KV append in the epilogue (replaces the projection + apply_rotary_pos_emb + DynamicCache.update
 * of models/audioLLM.py:482 / models/decoder/decoder.py:299-311 through transformers' Qwen2Attention /
 * LlamaAttention).  Wp packed with (i, i + hd/2) tile pairs per head; N = (H + 2 KVH) * hd.  Rows m:
 * q_out[m] = RoPE(q, pos[m]); K/V rows of kc/vc ([page][KVH][PS][hd]) at slot[m] = RoPE(k), v.
 * rstats/rgroups/eps: optional fused RMSNorm consumer (as fo_gemm_rms). */
int fo_gemm_qkv_rope(const void* X, int x_f32, int ldx, int M, int K, const void* Wp, int N, const float* bias,
                     float* ws, long long ws_floats, int* counters, int splitk, const float* rstats, int rgroups,
                     float eps, const int* pos, const int* slot, const float* cos_t, const float* sin_t, float* q_out,
                     float* kc, float* vc, int H, int KVH, int hd, int PS, hipStream_t stream);
/* Linear layer with the preceding LayerNorm applied to X as it is loaded (a speech-encoder block's
 * pre-norm + projection: norm1 -> linear_q/k/v and norm2 -> feed_forward.w_1,
 * models/encoder/transformer.py:103-130): Y = act(LN(X; lnw, lnb, eps) W^T + bias), X fp32, M <= 64.
 * Row mean / variance come from the producer GEMM's partial sums (fo_gemm_rowstats): rsum / rsumsq
 * [M][rgroups]. */
int fo_gemm_ln(const float* X, int ldx, int M, int K, const void* Wp, int N, const float* bias, const float* lnw,
               const float* lnb, float eps, const float* rsum, const float* rsumsq, int rgroups, float* Y, int ldy,
               int act, float* ws, long long ws_floats, int splitk, hipStream_t stream);
/* fo_gemm (fp32 Y) that also writes per-row partial sums of Y and Y^2 per workgroup column group
 * (*sgroups of them) for a following fo_gemm_ln (the residual-stream producers of an encoder block). */
int fo_gemm_rowstats(const void* X, int x_f32, int ldx, int M, int K, const void* Wp, int N, const float* bias,
                     float* Y, int ldy, int act, int residual, float* ws, long long ws_floats, int* counters,
                     int splitk, float* rsum, float* rsumsq, int* sgroups, hipStream_t stream);
/* sweep hook: force (waves, 16-column tiles per workgroup) of the M <= 16 GEMM kernels; 0 = automatic */
int fo_gemm_tune(int nw, int nt);
/* sweep hook: k-steps in flight per wave of the one-row-tile fp32-X grid kernel (0 = policy, 4, 7 on 16 waves, 8 on 8 waves) */
int fo_gemm_set_u(int u);
/* X-stationary persistent weight stream (k_gemm_xs) for the M <= 16 fp32-X GEMMs with K = 3584 (Qwen2 q|k|v,
 * o, gate/up, lm_head): 0 off, 1 on (default; FO_GEMM_XS=0 turns it off).  Process-global; returns the
 * previous setting. */
int fo_gemm_set_xs(int on);
/* probe hook: variant of the k_gemm_xs launch (0 shipped; 1 no cross-wave reduction -- WRONG results, a timing
 * bound; 2 default-policy weight loads; 3 round 4's 8 waves x 14 k-steps; 4 8 x 14 with the barrier-free
 * reduction).  Process-global; returns the previous one. */
int fo_gemm_set_xs_variant(int v);
/* probe hook: the weight size (MiB) from which 17..64-row fp32 GEMMs take k_gemm_xsk (default 128; long-K >= 32 MiB
 * layers always).  Process-global; returns the previous value. */
int fo_gemm_set_xsk_min_mb(int mb);
/* probe hook: 65..128-row GEMMs on >= 16 MiB weights through k_gemm_rows (1, default: the waves split the rows, the
 * weights through an LDS-DMA ring) or as two row-half launches of the <= 64-row kernels (0); probes: 2 = k_gemm_wrow
 * (one tile per wave, X staged once per workgroup), 3 = k_gemm_rows with each wave computing two row blocks for half
 * the tiles, 4 = k_gemm_rows from 33 rows, 5 / 6 = its weight ring alone (no X loads: WRONG results, timing bounds).
 * Unset, FO_GEMM_ROWS decides.  Process-global; returns the previous setting. */
int fo_gemm_set_rows(int on);
/* A/B of a bf16 paged KV (verdict r05 item 6; the reference's k_proj / v_proj outputs under torch.autocast(bf16),
 * models/pipeline.py:67-68): 1 = the q|k|v RoPE epilogues round every appended K / V element to bf16 (storage stays
 * fp32, so the numerics are a bf16 cache's and the layout is unchanged), 0 = fp32 (default).  Unset, FO_KV_BF16
 * decides.  Process-global; returns the previous setting. */
int fo_set_kv_bf16(int on);
/* probe (scripts/seam_probe.py): the Qwen2 o -> gate/up seam at <= 16 rows as one launch (k_seam_o_gu); xo [M][3584]
 * attention output, wo / wgu packed o and SwiGLU-paired gate/up weights, x the residual stream (updated), yg / sout the
 * next norm's input and partial sums of squares ([M][112]), h the SwiGLU output [M][n_gu_out]; ready: a zeroed int
 * (left at 112), ready_timeout set when the bounded poll gave up; trace: 4 wall clocks per workgroup or NULL; mode 0
 * the seam, 1 its o workgroups alone, 2 its gate/up workgroups alone. */
int fo_probe_seam(const float* xo, int M, const void* wo, const float* bo, float* x, const float* gnext, float* yg,
                  float* sout, const void* wgu, int n_gu_out, float* h, float eps, int* ready, int* ready_timeout,
                  void* trace, int mode, hipStream_t s);
/* Split-K of the one-row-tile plain GEMMs (Qwen2 / TTS down, encoder FFN w2) merged inside the launch:
 * each split stores its partial tile write-through and takes the tile's ticket in `counters` (zeroed
 * ints, left zeroed); the last split sums every partial in split order (k_gemm_reduce's order, bit for
 * bit) and runs the epilogue, so no reduce launch follows.  0: slabs + k_gemm_reduce everywhere; 1: merge
 * every eligible split; 2 (default, FO_GEMM_MERGE overrides): merge splits of weights < 32 MB (the TTS
 * down), where the reduce launch costs more than the write-through drain.  NULL counters always take the
 * two-launch form.  Process-global; returns the previous setting. */
int fo_gemm_set_merge(int on);
/* probe hook: the calling thread's following fo_gemm launches (grid kernels) write per-workgroup wall clocks
 * (100 MHz) to trace[wg * 24 + slot]: 0 start, 1 + w the end of wave w's weight stream, 17 the K reduce done,
 * 18 the epilogue issued.  nullptr turns it off (the default).  Returns 0.  The hook is compiled into the probe
 * library only (csrc: make probe -> fo/libfo_hip_probe.so); the product library refuses a non-NULL trace (-2). */
int fo_gemm_set_trace(void* trace);
/* Packed activations (fo/ops.py XPack / XPack32).  A packed buffer holds an fp32 activation of <= 64 rows in MFMA
 * A-fragment order: k-step k (32 columns), row block b (16 rows), lane l = row 16 b + (l & 15), columns 32 k +
 * 8 (l >> 4) .. + 8, i.e. [cols/32][rb][64][8] elements, where rb is the row-block count the launch uses
 * (ceil(M/16)).  Each setter arms the calling thread's NEXT matching launch only and carries the buffer's extent:
 * cols (its K, a multiple of 32) and cap_rb (the row blocks it was allocated for, 1..4).  The consuming launch
 * returns -2 (and consumes the arming) when cols differs from the K it reads / the N it writes, or when
 * cap_rb < ceil(M/16) -- a pack built for another layer or for fewer rows is refused, never read or written out of
 * bounds.  NULL pointers disarm (cols / cap_rb ignored).
 * fo_gemm_set_xpack: X given as bf16 hi / lo halves (the split a GEMM does on load, bit-identical); read by the
 *   one-row-tile and 17..64-row grid kernels (k_gemm_xp) and the <= 16-row gate/up stream (k_gemm_xs); the
 *   software-pipelined <= 8-row kernels and the 17..64-row split-K stream (k_gemm_xsk) read row-major X and ignore it.
 * fo_gemm_set_ypack: the launch (plain epilogue) also writes its next-norm input yg (stats_out) -- or, without one,
 *   its output Y -- into hi / lo as fo_gemm_set_xpack reads it.
 * fo_gemm_set_ypack32 / fo_gemm_set_xpack32: the fp32 form of the same order (exact values): the next launch writes
 *   its output Y there / the next fo_gemm_ln launch reads its X from there (LayerNorm-on-load consumers only). */
int fo_gemm_set_xpack(const void* hi, const void* lo, int cols, int cap_rb);
int fo_gemm_set_ypack(void* hi, void* lo, int cols, int cap_rb);
int fo_gemm_set_ypack32(void* p, int cols, int cap_rb);
int fo_gemm_set_xpack32(const void* p, int cols, int cap_rb);
/* the calling thread's NEXT fo_attention (<= 64 tokens, not with the separate combine launch; cols = H * hd) or
 * fo_relpos_attention_fused (<= 64 rows; cols = h * dk) launch also writes its output packed as fo_gemm_set_xpack
 * reads it, with the same extent check.  A launch whose host contract is broken (keys beyond the block table)
 * writes NaN to both the fp32 and the packed output. */
int fo_attention_set_opack(void* hi, void* lo, int cols, int cap_rb);
/* Launch counters per kernel family (tests assert which kernels a shape was routed to).  Counted on the host when
 * a launch is issued; a launch captured into a graph counts once, at capture.  fo_launch_counts copies
 * min(n, FO_LAUNCH_KINDS) counters into out (n <= 0: none) and returns FO_LAUNCH_KINDS; fo_launch_counts_reset
 * zeroes them (process-wide). */
enum FoLaunchKind {
  FO_L_GEMM_XS = 0,     /* k_gemm_xs: <= 16-row X-stationary gate/up stream */
  FO_L_GEMM_XSK = 1,    /* k_gemm_xsk: 17..64-row X-stationary split-K stream */
  FO_L_GEMM_XP = 2,     /* any GEMM launch that read packed X (fo_gemm_set_xpack) */
  FO_L_GEMM_REDUCE = 3, /* k_gemm_reduce */
  FO_L_GEMM_LN = 4,     /* k_gemm_ln: LayerNorm on load */
  FO_L_GEMM_XP32 = 5,   /* a k_gemm_ln launch that read fp32 packed X */
  FO_L_GEMM_YPACK = 6,  /* a GEMM launch that wrote packed output (ypack) */
  FO_L_GEMM_YPACK32 = 7,/* a GEMM launch that wrote fp32 packed output */
  FO_L_GEMM_MID = 8,    /* the 17..64-row one-row-tile grid kernels */
  FO_L_GEMM_ROPE4 = 9,  /* the 17..64-row RoPE q|k|v in 4-tile column groups (epilogue in the reduce) */
  FO_L_GEMM_PIPE = 10,  /* k_gemm_wpipe */
  FO_L_GEMM_OTHER = 11, /* every other GEMM launch */
  FO_L_ATTN_MFMA = 12,  /* k_attn_mfma */
  FO_L_ATTN_DECODE = 13,/* k_attn_decode */
  FO_L_ATTN_OPACK = 14, /* an attention launch that wrote packed output */
  FO_L_RELPOS = 15,     /* k_relpos_fused */
  FO_L_SUBSAMPLE = 16,  /* fo_subsample: the encoder front end (conv1 stencil + conv2 implicit GEMM + transpose) */
  FO_L_ATTN_O = 17,     /* k_attn_decode_o: decode attention + o projection + residual + next-norm statistics */
  FO_L_ENC_BLOCK = 18,  /* k_enc_attn_block: the attention half of a speech-encoder block */
  FO_L_GEMM_ROWS = 19,  /* k_gemm_rows: 65..128 rows, the waves split the rows, weights shared through an LDS ring */
  FO_LAUNCH_KINDS = 24
};
int fo_launch_counts(long long* out, int n);
int fo_launch_counts_reset(void);
/* Software-pipelined one-row-tile fp32-X weight-stream GEMMs (M <= 16, >= 32 MB of weights: the next
 * k-group's weights + X in flight during this group's MFMAs).  3 (default): the measured policy; 0: plain
 * loops; 1 / 2: every such GEMM pipelined with 4 / 2 k-steps per group (sweeps).  Unset, the
 * FO_GEMM_PIPE environment variable (0-3) decides.  Process-global state (for sweeps and tests); returns the
 * previous mode (>= 0) so callers can restore it. */
int fo_gemm_set_pipe(int on);
long long fo_pack_weight_elems(int N, int K);
int fo_pack_weight(const void* W, int src_bf16, int N, int K, int ldw, void* out, int tile_base, int tile_stride,
                   hipStream_t stream);
int fo_gemm_pick_split(int M, int n_tile_groups, int K);
long long fo_gemm_workspace_floats(int M, int N, int K, int swiglu);
/* X: bf16 (x_f32=0) or fp32 (x_f32=1, split into bf16 hi+lo MFMA passes).  Epilogue order:
 * +bias, *scale+shift (per column), activation (0 none,1 relu,2 silu,3 gelu), +Y if residual. */
int fo_gemm(const void* X, int x_f32, int ldx, int M, int K, const void* Wp, int N, int swiglu, const float* bias,
            const float* scale, const float* shift, void* Y, int ldy, int out_bf16, int act, int residual, float* ws,
            long long ws_floats, int* counters, int splitk, hipStream_t stream);

/* ---------------------------------------------------------------- memory-bound helpers (fo_elem.hip) */
/* counter-hash synthetic weights, bit-identical to oracle/weights.py hash_uniform */
int fo_fill_hash(void* out, int out_bf16, long long n, unsigned long long key, float center, float scale,
                 hipStream_t s);
/* Qwen2RMSNorm / LlamaRMSNorm (transformers, reached from models/audioLLM.py:482 and
 * models/decoder/decoder.py:299-311,343); round_fp16 mirrors the cast back to an fp16 input dtype. */
int fo_rmsnorm(const float* x, int ldx, int M, int D, const float* w, float eps, float* out, int ldo, int round_fp16,
               hipStream_t s);
/* torch.nn.LayerNorm of the speech encoder (models/encoder/transformer.py:343-346,261,278,287) and of the
 * adapter's norm: layer branch (models/adapter.py:102-103,145-149); act 0 none, 1 ReLU, 3 exact GELU. */
int fo_layernorm(const float* x, int ldx, int M, int D, const float* w, const float* b, float eps, float* out, int ldo,
                 int act, hipStream_t s);
/* embedding / row gather (wte at models/audioLLM.py:303,330; decoder embedding decoder.py:318,336) */
int fo_gather_rows(const void* table, int table_bf16, long long ld_tab, const int* idx, int M, int D, float* out,
                   int ldo, const int* out_rows, int round_fp16, hipStream_t s);
/* Conv2dSubsampling4 front end as im2col (+ fused GlobalCMVN) (models/encoder/subsampling.py:67-73,
 * models/encoder/cmvn.py:24-35) */
int fo_im2col_3x3s2(const float* in, int B, int C, int H, int W, long long sb, long long sc, long long sh,
                    long long sw, const float* mean, const float* istd, float* out, int ldo, hipStream_t s);
int fo_tcf_permute(const float* in, int B, int T, int F, int C, float* out, hipStream_t s);
/* CNNSubsampling causal strided conv1d with carried frames (models/adapter.py:112-157) */
int fo_im2col_conv1d(const float* cache, const int* slots, const float* x, int B, int KC, int T, int D, int K, int S,
                     float* out, int ldo, hipStream_t s);
int fo_conv_cache_update(float* cache, const int* slots, const float* x, int B, int KC, int T, int D, hipStream_t s);
/* dialog-state head + 3-class softmax (models/audioLLM.py:486-493) */
int fo_state_head(const float* h, int ldh, const int* rows, int S, const float* W, const float* bias, int D,
                  float* probs, hipStream_t s);
int fo_scale(float* x, long long n, float sc, hipStream_t s);
/* dst[row[0]][b] = ids[b]: the AR decode graph's token history (llm2tts.py:122-129 accumulate ids) */
int fo_record_ids(const int* ids, int B, int* dst, int ld, const int* row, hipStream_t s);

/* ---------------------------------------------------------------- attention (fo_attn.hip) */
/* number of key splits for fo_attention: ~2 work groups per CU, >= 64 keys per split, <= 32 */
/* query rows (tokens x query heads per kv head) one work item of fo_attention may carry for head size hd: 32 on the
 * 8-wave head-dim-128 kernel (two 16-row tiles sharing the K / V loads), else 16. */
int fo_attn_max_rows(int hd);
/* probe hook: per-workgroup wall clocks of the following multi-row fo_attention launches on this thread (8 slots a
 * workgroup in linear block order: start, staged, tile loop done, partials stored, end, 1 + splits); NULL stops.
 * Armed, the head-dim-128 8-wave launches run a traced instance of the kernel (the product instance has no hook);
 * other variants run untraced. */
int fo_attention_set_trace(void* trace);
int fo_attn_nsplit(int max_keys, int n_items, int KVH);
/* RoPE (rotate_half, host cos/sin tables) + paged KV append: transformers apply_rotary_pos_emb +
 * DynamicCache.update (models/audioLLM.py:416-419, models/decoder/decoder.py:146,305) */
int fo_rope_kv_write(const float* qkv, int ldq, int T, int H, int KVH, int hd, const int* pos, const int* slot,
                     const float* cos_t, const float* sin_t, float* q_out, float* kc, float* vc, int PS,
                     hipStream_t s);
/* GQA attention over paged KV for a ragged batch (transformers sdpa/eager attention reached from
 * models/audioLLM.py:482 and models/decoder/decoder.py:142-153,299-311); token t sees the first
 * tok_nvis[t] keys of its sequence (causal: own cache index + 1, full/unmasked: all).  items
 * [n_items][3] = (sequence, first token, token count), token count * H/KVH <= max_rows <= 16;
 * items may be NULL when every sequence contributes one token (n_items == T: item b = sequence b = token b).
 * Split-KV (nsplit from fo_attn_nsplit) + combine. */
int fo_attention(const float* q, int T, const int* items, int n_items, int max_rows, const int* tok_nvis,
                 const int* block_table, int maxb, int PS, const float* kc, const float* vc, int H, int KVH, int hd,
                 float scale, int nsplit, float* part_ml, float* part_o, float* out, int* tickets,
                 int keys_per_split, hipStream_t s);
/* Conv2dSubsampling4.infer up to its output Linear (models/encoder/subsampling.py:67-73) with GlobalCMVN
 * (models/encoder/cmvn.py:24-35): feats [B][R][F] fp32 -> z [B * H2][C * W2] (the Linear's input rows, the reference's
 * x.transpose(1, 2).view(b, t, c * f)), H1 = (R - 3) / 2 + 1, W1 = (F - 3) / 2 + 1, H2 / W2 likewise from H1 / W1.
 * w1 [C][9] fp32 (conv.0 weight), b1 [C]; y1: scratch [B * H1 * W1][C]; w2p: conv.2's weight [C][C][3][3] permuted to
 * [C][3][3][C] (K tap-major) and packed by fo_pack_weight; b2 [C]; ws >= fo_subsample_ws_floats(B, R, F, C) floats
 * (split-K partial slabs).  C % 32 == 0. */
long long fo_subsample_ws_floats(int B, int R, int F, int C);
int fo_subsample(const float* feats, int B, int R, int F, const float* mean, const float* istd, const float* w1,
                 const float* b1, int C, float* y1, const void* w2p, const float* b2, float* z, float* ws,
                 long long ws_floats, hipStream_t s);
/* The AR speech decoder's decode attention (one token per sequence, MHA: KVH == H, hd 64; items NULL or one per
 * token) fused with its o projection (LlamaAttention.o_proj, models/decoder/decoder.py:341-349), the layer's
 * residual add and the next RMSNorm's statistics: x[t] += sum_h att[t][h] . Wo[:, h*hd:(h+1)*hd]^T (the H head
 * partials summed in head order by the last head to finish, an agent-scope ticket), yg[t] = x[t] * gnext,
 * sout[t] = sum x[t]^2 (one statistics group, read by the next fo_gemm_rms consumer with rgroups 1).
 * wo: the o weight packed by fo_pack_weight (N <= 1024 outputs, K = H * hd); part >= T * H * N floats; tickets: T
 * zeroed ints, left zeroed. */
int fo_attention_o(const float* q, int T, const int* items, const int* tok_nvis, const int* block_table, int maxb,
                   int PS, const float* kc, const float* vc, int H, int hd, float scale, const void* wo, int N,
                   float* part, int* tickets, float* x, int ldx, const float* gnext, float* yg, float* sout,
                   hipStream_t s);
/* The attention half of a speech-encoder block in one launch (models/encoder/transformer.py:103-118 with
 * MultiHeadedAttention.infer, models/encoder/attention.py:407-459): x += linear_out(relpos_attention(linear_q|k|v(
 * LayerNorm1(x)), ring)) for B sessions x T rows, in place, plus the updated rows' sums / sums of squares (ssum, ssq:
 * [B * T], one statistics group for the next LayerNorm-on-load GEMM).  A workgroup per (session, head); head
 * partials of linear_out in part (>= B * h * T * d floats) summed in head order by the session's last head
 * (tickets: B zeroed ints, left zeroed).  wqkv: linear_q|k|v [3d][d] packed by fo_pack_weight, bqkv [3d]; wout:
 * linear_out [d][d] packed, bout [d]; kr / vr, cap, meta [start B | len B | ring B | pos start B], ptab, bu, bv as
 * fo_relpos_attention_fused.  Head size 64, T <= 8, d = 64 h a multiple of 256 and <= 1024, cap + T <= 96. */
int fo_enc_attn_block(float* x, int B, int T, int d, int h, const float* lnw, const float* lnb, float ln_eps,
                      const void* wqkv, const float* bqkv, float* kr, float* vr, int cap, const int* meta,
                      const float* ptab, const float* bu, const float* bv, const void* wout, const float* bout,
                      float scale, float* part, int* tickets, float* ssum, float* ssq, hipStream_t s);
/* fo_enc_attn_block's second half alone: q|k|v given ([B * T] rows of ldq >= 3d floats, + bias: the LayerNorm-on-load
 * GEMM's output), the rel-pos attention, linear_out, the residual and the row statistics in one launch. */
int fo_enc_attn_out(const float* qkv, int ldq, float* x, int B, int T, int d, int h, float* kr, float* vr, int cap,
                    const int* meta, const float* ptab, const float* bu, const float* bv, const void* wout,
                    const float* bout, float scale, float* part, int* tickets, float* ssum, float* ssq,
                    hipStream_t s);
/* encoder MultiHeadedAttention.infer left-chunk buffer as a ring + rel-pos scores
 * (models/encoder/attention.py:407-459) */
int fo_enc_kv_write(const float* k, const float* v, int ldkv, int B, int T, int d, const int* start, const int* len,
                    const int* ring, int cap, float* kr, float* vr, hipStream_t s);
/* enc_kv_write + relpos_attention in one launch: new K/V rows read from the QKV output (columns
 * [d, 2d) and [2d, 3d)), appended to the ring, attention over ring + new rows staged in LDS */
int fo_relpos_attention_fused(const float* qkv, int ldq, float* kr, float* vr, int cap, const int* start,
                              const int* len, const int* ring, const float* ptab, const int* pstart, const float* bu,
                              const float* bv, int B, int T, int h, int dk, float scale, float* out, int ldo,
                              hipStream_t s);
/* fo_relpos_attention_fused over C consecutive chunks of the same B users in one launch (the offline listen's grouped
 * encoder pass, SpeechEncoderEngine.run(chunks=C); replaces C sequential calls of MultiHeadedAttention.infer,
 * models/encoder/attention.py:407-459): q|k|v rows chunk-major ((j*B + b)*T + i), meta [C][start B | len B | ring B |
 * pstart B] (each chunk's ring state after the chunks before it), out rows as q|k|v.  Chunks run in order per
 * (user, head); rows an earlier chunk of the launch appended are read from its q|k|v rows. */
int fo_relpos_attention_chunks(const float* qkv, int ldq, float* kr, float* vr, int cap, const int* meta, int B, int C,
                               const float* ptab, const float* bu, const float* bv, int T, int h, int dk, float scale,
                               float* out, int ldo, hipStream_t s);
int fo_relpos_attention(const float* q, int ldq, const float* kr, const float* vr, int cap, const int* start,
                        const int* len, const int* ring, const float* ptab, const int* pstart, const float* bu,
                        const float* bv, int B, int T, int h, int dk, float scale, float* out, int ldo,
                        hipStream_t s);

/* ---------------------------------------------------------------- audio front end (fo_audio.hip) */
/* kaldi fbank (torchaudio.compliance.kaldi.fbank at bin/inference.py:77-78, AudioFeatureGating.py:65-69) */
int fo_fbank(const float* samples, int ld_s, int B, int n_samples, int wl, int ws, int nfft, const float* window,
             const float* tw_cos, const float* tw_sin, const float* mel, int nmel, float* out, int ld_b, int row0,
             const int* zero_rows, hipStream_t s);
int fo_rows_shift(float* feats, int B, int R, int ov, int D, hipStream_t s);

/* ---------------------------------------------------------------- codec (fo_codec.hip) */
/* Generator convs (models/decoder/ticodec/models.py:59-166,211-242) */
int fo_conv1d(const float* x, int B, int Cin, int Tin, const void* w, const float* bias, int Cout, int K, int dil,
              int pad, int pre_leaky, float slope, float* out, int residual, int post_tanh, hipStream_t s);
int fo_conv_transpose1d(const float* x, int B, int Cin, int Tin, const void* w, const float* bias, int Cout, int K,
                        int stride, int pad, float slope, float* out, hipStream_t s);
/* Quantizer.embed (models/decoder/ticodec/models.py:661-702) */
int fo_codec_embed(const void* table, int E, int n_codes, const int* ids, int B, int T, float* out, hipStream_t s);
int fo_axpy(float* y, const float* x, long long n, hipStream_t s);
int fo_scale_add_channel(float* y, int B, int C, int T, float sc, const float* g, hipStream_t s);
/* ---------------------------------------------------------------- vocoder on MFMA (fo_vocoder.hip)
 * Generator.forward convs (models/decoder/ticodec/models.py:59-110,211-242) as implicit GEMMs on
 * channel-last activations [B][T][C]; ConvTranspose1d as stride-u polyphase convs.  fo_conv_cl's
 * epilogue out = (conv + bias + res + res2) * oscale + gadd[b][c] folds ResBlock1's residual adds, the
 * mean over resblocks and the global-token feature (models.py:104-108,229-238) into the convs. */
long long fo_conv_pack_elems(int Cout, int Cin, int K);
int fo_pack_conv(const void* W, int src_bf16, int Cout, int Cin, int K, int transposed, int Ktot, int j0, int u,
                 void* out, hipStream_t s);
int fo_conv_cl(const float* x, int B, int Cin, int Tin, const void* wp, const float* bias, int Cout, int K, int dil,
               int pad, int Tq, int ostride, int ooff, int Tout_total, int pre_leaky, float slope, float* out,
               const float* res, const float* res2, float oscale, const float* gadd, hipStream_t s);
/* One fo_conv_cl per descriptor, G (<= 5) of them in ONE launch, all Cin -> Cout over B batch rows: the u
 * polyphase components of a ConvTranspose1d, or the independent ResBlock1 chains of a generator stage
 * (models/decoder/ticodec/models.py:221-238: the resblocks of a stage all read the upsampled x and are
 * averaged).  No descriptor may read another's output.  sum != 0: each output tile runs all G convs into one
 * accumulator and stores (sum_g (conv_g + bias_g + res_g + res2_g)) * oscale + gadd with descriptor 0's out,
 * oscale, gadd and output geometry (the resblocks' last convs and their mean, models.py:236-238). */
typedef struct FoConvDesc {
  const float* x;       /* [B][Tin][Cin] */
  const void* wp;       /* fo_pack_conv output */
  const float* bias;    /* [Cout] or NULL */
  float* out;           /* [B][Tout_total][Cout] */
  int Tin, K, dil, pad, Tq, ostride, ooff, Tout_total, pre_leaky;
  float slope;
  const float* res;     /* like out, or NULL */
  const float* res2;
  float oscale;
  const float* gadd;    /* [B][Cout] or NULL */
} FoConvDesc;
int fo_conv_cl_multi(const FoConvDesc* descs, int G, int B, int Cin, int Cout, int sum, hipStream_t s);
/* One ResBlock1 step y = x + c2(leaky(c1(leaky(x)))) per descriptor (models/decoder/ticodec/models.py:90-110;
 * c1: K taps at dilation dil, c2: K taps at dilation 1, both C -> C, "same" padding), both convolutions in one
 * workgroup (c1's output tile stays in LDS), G (<= 5) chains side by side in one launch.  C = 16, 32 or 64
 * (the generator's narrow late stages).  sum != 0: one output = (sum_g y_g) * oscale + gadd into descs[0].out
 * (the chains' last step and their mean, models.py:236-238); otherwise oscale 1 / gadd NULL. */
typedef struct FoPairDesc {
  const float* x;       /* [B][T][C], also the residual */
  const void* w1;       /* c1 (fo_pack_conv) */
  const float* b1;
  const void* w2;       /* c2 */
  const float* b2;
  float* out;           /* [B][T][C] */
  int K, dil;
} FoPairDesc;
int fo_conv_pair_multi(const FoPairDesc* descs, int G, int B, int C, int T, int sum, float slope, float oscale,
                       const float* gadd, hipStream_t s);
/* Quantizer.embed (models/decoder/ticodec/models.py:661-700), channel-last output */
/* probe hook: per-workgroup clocks of the following k_conv_cl launches on this thread ({wall start, stage cycles,
 * compute cycles, wall end} x workgroups, linear block order); NULL stops.  Armed, they run a traced instance of the
 * kernel (the product instance has no hook). */
int fo_conv_set_trace(void* trace);
int fo_codec_embed_cl(const void* table, int E, int n_codes, const int* ids, int B, int T, float* out, hipStream_t s);
/* xs / num_kernels (+ global feature, models.py:233-238), channel-last */
int fo_scale_add_cl(float* y, int B, int T, int C, float sc, const float* g, hipStream_t s);
/* leaky -> conv_post (Cout 1) -> tanh (models.py:239-241), channel-last input */
int fo_conv_post_cl(const float* x, int B, int T, int C, const void* w, const float* bias, int K, int pad, float slope,
                    float* out, hipStream_t s);

/* llm2TTS.find_min_sum_index window search (models/decoder/llm2tts.py:70-112): res = {min_sum, cut} */
int fo_silence_cut(const float* x, int L, int N, float* res, hipStream_t s);
/* the same search for `rows` rows of one vocoder call in one launch: row r at x + r * ld (ld >= L), its
   (min window sum, cut index) at res + 2 r; each row is staged in LDS when it fits (<= ~37k samples) */
int fo_silence_cut_rows(const float* x, long long ld, int rows, int L, int N, float* res, hipStream_t s);

/* ---------------------------------------------------------------- codec encoder (fo_codec_enc.hip)
 * VQVAE.encode (models/decoder/ticodec/vqvae.py:44-57).  Channel-first fp32 [B][C][T], fp32 weights. */
/* Conv1d with stride / dilation / zero padding, optional leaky pre-activation (slope) and += into out
 * (Encoder.conv_pre / ups / ResBlock1 convs / conv_post, GlobalTokenEncoder convs; models.py:22-166,429-498) */
int fo_conv1d_ex(const float* x, int B, int Cin, int Tin, const float* w, const float* bias, int Cout, int K,
                 int stride, int dil, int pad, int pre_act, float slope, float* out, int residual, hipStream_t s);
/* torch.nn.GroupNorm(G, C, eps) with affine, then * scale (Encoder.normalize, models.py:466-467,483-489) */
int fo_group_norm(const float* x, int B, int C, int T, int G, const float* w, const float* bias, float eps,
                  float scale, float* out, hipStream_t s);
/* GlobalTokenEncoder tail (models.py:32-57): leaky 0.1 of the last conv's output, mean over T, Linear + leaky 0.1, BatchNorm1d eval -> out [B][C] */
int fo_gte_head(const float* x, int B, int C, int T, const float* lw, const float* lb, const float* rm,
                const float* rv, const float* bw, const float* bb, float bn_eps, float* out, hipStream_t s);
/* Quantizer_module.forward (models.py:531-537) on channels [ch0, ch0+D) of every (b, t):
 * argmin_j (|x|^2 + |e_j|^2) - 2 x.e_j -> ids[(b*T+t)*ids_ld + ids_col]; residual: x -= x + (e - x)
 * (Quantizer.for_one_step / forward, models.py:583-645) */
int fo_vq_nearest(float* x, int B, int Ctot, int T, int ch0, int D, const float* codebook, int n_codes, int* ids,
                  int ids_ld, int ids_col, int residual, hipStream_t s);

/* ---------------------------------------------------------------- sampling (fo_sample.hip) */
/* AudioLLM._post_decode (models/audioLLM.py:431-477) / decoder top-k (models/decoder/decoder.py:353-359).
 * Draws come from a counter stream keyed by (seed, key[row] or row, step[row]).
 * err (nullable, every sampler entry): set to 1, never cleared, when a row holds a NaN or +inf logit or
 * only -inf ones -- the rows whose softmax torch.multinomial refuses (decoder.py:355-359 raises); the
 * drawn id stays inside [0, V).  The caller raises on it (Python: RuntimeError).
 * ws (nullable, >= fo_sample_ws_floats(B, V) floats): top_k == 1 rows over V >= 8192 take a split
 * arg-max (one pass over the row by ~V/2048 workgroups, then the per-row reduction). */
long long fo_sample_ws_floats(int B, int V);
int fo_sample(const float* logits, int ld, int B, int V, const int* top_k, const float* temperature,
              const float* top_p, unsigned long long seed, const int* step, const int* key, int ban_id,
              int* out_ids, float* out_maxlogit, int* err, float* ws, long long ws_floats, hipStream_t s);
/* fo_sample that also writes each row's sampling distribution -- the `probs` _post_decode hands to
 * torch.multinomial (models/audioLLM.py:455-476) -- to probs[row * ldp + i] (ldp >= V).  top_k 0 (no
 * top-k, the reference default) and top_k > 64 take a whole-vocabulary radix-select path. */
int fo_sample_probs(const float* logits, int ld, int B, int V, const int* top_k, const float* temperature,
                    const float* top_p, unsigned long long seed, const int* step, const int* key, int ban_id,
                    int* out_ids, float* probs, int ldp, int* err, hipStream_t s);
/* fo_sample fused with the next AR decode step's input (models/decoder/decoder.py:341-346: embed(id) ->
 * first LlamaRMSNorm): hist[hist_row[0] * hist_ld + row] = id (hist nullable), x[row] = emb[id] (bf16
 * table -> fp32), h[row] = RMSNorm(x[row]) * gamma.  meta (nullable): the captured step's metadata block
 * ([pos B][slot B][nvis B][step B][key B][hist_row 1][block table B x maxb]; step / key point into it): the history row is then each row's step,
 * and each row's entries advance to the next step inside this launch (no separate advance launch). */
int fo_sample_embed(const float* logits, int ld, int B, int V, const int* top_k, const float* temperature,
                    const float* top_p, unsigned long long seed, const int* step, const int* key, int ban_id,
                    int* out_ids, int* hist, const int* hist_row, int hist_ld, const void* emb, long long emb_ld,
                    int D, float* x, int ldx, const float* gamma, float eps, float* h, int ldh, int* meta, int maxb,
                    int PS, int* err, hipStream_t s);
/* Repetition penalty of the AR decode loop (models/decoder/decoder.py:348-351), applied before the
 * draw: win[row][step[row] % W] = ids[row], then logits[row][t] /= penalty for every entry t of the
 * last min(step+1, W) ids -- once per occurrence, as the reference's set() of 0-d tensors does. */
int fo_penalty(float* logits, int ld, int B, int V, const int* ids, int* win, int W, const int* step, float penalty,
               hipStream_t s);


#ifdef __cplusplus
}
#endif
#endif
