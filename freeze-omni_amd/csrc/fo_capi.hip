// C-ABI plumbing shared by every entry point: error reporting, device info, stream graphs.
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include "fo_common.h"

static thread_local char g_err[1024] = {0};

namespace fo {
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
