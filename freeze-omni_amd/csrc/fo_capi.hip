// C-ABI plumbing shared by every entry point: error reporting, device info, stream graphs.
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include "fo_common.h"
#include <hip/hip_ext.h>

#include <atomic>

#include "fo_hip.h"

static thread_local char g_err[1024] = {0};
static std::atomic<long long> g_launches[FO_LAUNCH_KINDS];

namespace fo {
void count_launch(int kind) {
  if (kind >= 0 && kind < FO_LAUNCH_KINDS) g_launches[kind].fetch_add(1, std::memory_order_relaxed);
}
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: launch failed: %s", what, hipGetErrorString(e));
    return -1;
  }
  return 0;
}
}  // namespace fo

extern "C" {

int fo_version(void) { return 1; }

int fo_launch_counts(long long* out, int n) {
  for (int i = 0; out && i < n && i < FO_LAUNCH_KINDS; ++i) out[i] = g_launches[i].load(std::memory_order_relaxed);
  return FO_LAUNCH_KINDS;
}
int fo_launch_counts_reset(void) {
  for (int i = 0; i < FO_LAUNCH_KINDS; ++i) g_launches[i].store(0, std::memory_order_relaxed);
  return 0;
}

// Copies the last error message of this thread into buf (always NUL-terminated).
int fo_last_error(char* buf, int len) {
  if (!buf || len <= 0) return -2;
  strncpy(buf, g_err, (size_t)len - 1);
  buf[len - 1] = 0;
  return (int)strlen(buf);
}

int fo_device_info(int dev, char* name, int len, int* n_cu, long long* hbm_bytes) {
  hipDeviceProp_t p;
  FO_HIP(hipGetDeviceProperties(&p, dev));
  if (name && len > 0) {
    snprintf(name, (size_t)len, "%s (%s)", p.name, p.gcnArchName);
  }
  if (n_cu) *n_cu = p.multiProcessorCount;
  if (hbm_bytes) *hbm_bytes = (long long)p.totalGlobalMem;
  return 0;
}

// ---- stream capture into hipGraphs: per-step launch sequences are recorded once and replayed.
int fo_graph_begin(hipStream_t s) {
  FO_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  return 0;
}
int fo_graph_end(hipStream_t s, void** exec_out) {
  hipGraph_t g;
  FO_HIP(hipStreamEndCapture(s, &g));
  hipGraphExec_t ex;
  hipError_t e = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  if (e != hipSuccess) {
    fo::set_error("hipGraphInstantiate: %s", hipGetErrorString(e));
    return -1;
  }
  *exec_out = (void*)ex;
  return 0;
}
int fo_graph_launch(void* exec, hipStream_t s) {
  FO_HIP(hipGraphLaunch((hipGraphExec_t)exec, s));
  return 0;
}
int fo_graph_destroy(void* exec) {
  FO_HIP(hipGraphExecDestroy((hipGraphExec_t)exec));
  return 0;
}

// Event-timed region helpers (the bench times kernels on the stream they run on).
int fo_event_create(void** ev) {
  hipEvent_t e;
  FO_HIP(hipEventCreate(&e));
  *ev = (void*)e;
  return 0;
}
// Blocking stream (synchronises with the legacy default stream like torch's default work does), for
// the engines' own launch sequences and graph capture (capture needs a non-null stream).
int fo_stream_create(void** s_out) {
  hipStream_t s;
  FO_HIP(hipStreamCreate(&s));
  *s_out = (void*)s;
  return 0;
}
// A blocking stream at the device's greatest scheduling priority when level > 0 (the speech streams: a
// sentence's first audio is latency-critical while the text decode beside it is throughput work), at its
// least priority when level < 0, at the default (0, clamped into the range) otherwise.
int fo_stream_create_prio(void** s_out, int level) {
  int lo = 0, hi = 0;
  FO_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
  hipStream_t s;
  FO_HIP(hipStreamCreateWithPriority(&s, hipStreamDefault, level > 0 ? hi : (level < 0 ? lo : 0)));
  *s_out = (void*)s;
  return 0;
}
// A blocking stream whose kernels run only on the CUs set in mask (nwords 32-bit words, bit i = CU i in the
// runtime's CU numbering): the listen stages' CU partition (the encoder stage on a few CUs, the Qwen2 stage on
// the rest, so no Qwen2 workgroup shares a CU with the encoder stage).
int fo_stream_create_cumask(void** s_out, const unsigned* mask, int nwords) {
  FO_REQUIRE(mask && nwords > 0, "fo_stream_create_cumask: empty mask");
  hipStream_t s;
  FO_HIP(hipExtStreamCreateWithCUMask(&s, (uint32_t)nwords, mask));
  *s_out = (void*)s;
  return 0;
}
// The device's stream priority range (least, greatest; lower numbers are greater priorities).
int fo_stream_priority_range(int* least, int* greatest) {
  FO_HIP(hipDeviceGetStreamPriorityRange(least, greatest));
  return 0;
}
// Order stream s after event ev (cross-stream dependency of the pipelined listen stages).
int fo_stream_wait_event(hipStream_t s, void* ev) {
  FO_HIP(hipStreamWaitEvent(s, (hipEvent_t)ev, 0));
  return 0;
}
int fo_stream_destroy(void* s) {
  FO_HIP(hipStreamDestroy((hipStream_t)s));
  return 0;
}
// Pinned, device-mapped host memory: kernels write it through *dev_ptr, the host reads *host_ptr
// after an event (the decode graph's token history).
int fo_host_alloc(long long bytes, void** host_ptr, void** dev_ptr) {
  void* h = nullptr;
  FO_HIP(hipHostMalloc(&h, (size_t)bytes, hipHostMallocMapped));
  void* d = nullptr;
  hipError_t e = hipHostGetDevicePointer(&d, h, 0);
  if (e != hipSuccess) {
    (void)hipHostFree(h);
    fo::set_error("hipHostGetDevicePointer: %s", hipGetErrorString(e));
    return -1;
  }
  *host_ptr = h;
  *dev_ptr = d;
  return 0;
}
int fo_host_free(void* host_ptr) {
  FO_HIP(hipHostFree(host_ptr));
  return 0;
}
int fo_event_sync(void* ev) {
  FO_HIP(hipEventSynchronize((hipEvent_t)ev));
  return 0;
}
// 1 when the event has completed, 0 while pending, <0 on error.
int fo_event_query(void* ev) {
  hipError_t e = hipEventQuery((hipEvent_t)ev);
  if (e == hipSuccess) return 1;
  if (e == hipErrorNotReady) return 0;
  fo::set_error("hipEventQuery: %s", hipGetErrorString(e));
  return -1;
}
int fo_event_record(void* ev, hipStream_t s) {
  FO_HIP(hipEventRecord((hipEvent_t)ev, s));
  return 0;
}
int fo_event_elapsed_ms(void* a, void* b, float* ms) {
  FO_HIP(hipEventSynchronize((hipEvent_t)b));
  FO_HIP(hipEventElapsedTime(ms, (hipEvent_t)a, (hipEvent_t)b));
  return 0;
}
int fo_event_destroy(void* ev) {
  FO_HIP(hipEventDestroy((hipEvent_t)ev));
  return 0;
}

}  // extern "C"
