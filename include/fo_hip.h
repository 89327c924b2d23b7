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
long long fo_pack_weight_elems(int N, int K);
int fo_pack_weight(const void* W, int src_bf16, int N, int K, int ldw, void* out, int tile_base, int tile_stride,
                   hipStream_t stream);
int fo_gemm_pick_split(int M, int n_tile_groups, int K);
long long fo_gemm_workspace_floats(int M, int N, int K, int swiglu);
int fo_gemm(const void* X, int ldx, int M, int K, const void* Wp, int N, int swiglu, const float* bias, void* Y,
            int ldy, int out_bf16, int act, int residual, float* ws, long long ws_floats, int* counters, int splitk,
            hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif
