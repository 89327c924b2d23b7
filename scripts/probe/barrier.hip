// Measurement only (not part of the product library): what a kernel boundary costs inside a replayed
// graph versus a grid-wide barrier inside one persistent launch, to size a one-launch TTS step.
//   k_empty            : a do-nothing kernel (graph of NK launches)
//   k_touch            : each workgroup reads 1 KiB and writes 64 B (a minimal dependent phase)
//   k_persist          : NB grid barriers in one launch (monotonic arrival counter, bounded spin:
//                        a workgroup that waits too long records an error and leaves, so the launch
//                        always drains)
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void k_empty() {}

__global__ __launch_bounds__(256) void k_touch(const float* in, float* out) {
  const float v = in[blockIdx.x * 256 + threadIdx.x];
  __shared__ float s[4];
  float r = v;
  for (int o = 32; o > 0; o >>= 1) r += __shfl_xor(r, o);
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = r;
  __syncthreads();
  if (threadIdx.x < 16) out[blockIdx.x * 16 + threadIdx.x] = s[0] + s[1] + s[2] + s[3];
}

__device__ __forceinline__ void grid_sync(unsigned* ctr, unsigned target, int* err) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned spins = 0;
    while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1u << 20) || __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
}

// work: 0 = barriers only; 1 = each phase every workgroup reads 1 KiB of `in` (phase-dependent
// offset) and writes 64 B that the next phase reads from another workgroup
__global__ __launch_bounds__(256) void k_persist(unsigned* ctr, unsigned base, int nb, int* err, int work,
                                                 const float* in, float* buf) {
  float acc = 0.f;
  for (int b = 0; b < nb; ++b) {
    if (work) {
      const int src = (blockIdx.x + b) % gridDim.x;
      acc += in[((size_t)b * gridDim.x + blockIdx.x) % (1 << 20) * 256 % (1 << 24) + threadIdx.x];
      if (threadIdx.x < 16) acc += buf[(b & 1) * gridDim.x * 16 + src * 16 + threadIdx.x];
      if (threadIdx.x < 16) buf[((b + 1) & 1) * gridDim.x * 16 + blockIdx.x * 16 + threadIdx.x] = acc;
    }
    grid_sync(ctr, base + (unsigned)(b + 1) * gridDim.x, err);
  }
  if (acc == 12345.f) buf[0] = acc;
}

static double ms_between(hipEvent_t a, hipEvent_t b) {
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  return ms;
}

extern "C" {
// graph of nk launches of `kind` (0 empty, 1 touch with `grid` workgroups); returns us per launch
double probe_graph_launch(int kind, int nk, int grid, int reps) {
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  float *in = nullptr, *out = nullptr;
  hipMalloc(&in, (size_t)grid * 256 * 4);
  hipMalloc(&out, (size_t)grid * 16 * 4);
  hipMemset(in, 0, (size_t)grid * 256 * 4);
  hipGraph_t g;
  hipGraphExec_t ge;
  hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
  for (int i = 0; i < nk; ++i) {
    if (kind == 0) hipLaunchKernelGGL(k_empty, dim3(grid), dim3(64), 0, s);
    else hipLaunchKernelGGL(k_touch, dim3(grid), dim3(256), 0, s, in, out);
  }
  hipStreamEndCapture(s, &g);
  hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipGraphLaunch(ge, s);
  hipEventRecord(a, s);
  for (int r = 0; r < reps; ++r) hipGraphLaunch(ge, s);
  hipEventRecord(b, s);
  hipEventSynchronize(b);
  const double us = ms_between(a, b) * 1000.0 / reps / nk;
  hipGraphExecDestroy(ge);
  hipGraphDestroy(g);
  hipFree(in);
  hipFree(out);
  hipEventDestroy(a);
  hipEventDestroy(b);
  hipStreamDestroy(s);
  return us;
}

// one launch of `grid` x 256 threads doing nb grid barriers; returns us per barrier (negative: a
// workgroup timed out in a barrier)
double probe_persist(int grid, int nb, int work, int reps) {
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  unsigned* ctr = nullptr;
  int* err = nullptr;
  float *in = nullptr, *buf = nullptr;
  hipMalloc(&ctr, 4);
  hipMalloc(&err, 4);
  hipMalloc(&in, (size_t)(1 << 24) * 4 + 4096);
  hipMalloc(&buf, (size_t)grid * 32 * 4);
  hipMemset(ctr, 0, 4);
  hipMemset(err, 0, 4);
  hipMemset(in, 0, (size_t)(1 << 24) * 4 + 4096);
  hipMemset(buf, 0, (size_t)grid * 32 * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  unsigned base = 0;
  hipLaunchKernelGGL(k_persist, dim3(grid), dim3(256), 0, s, ctr, base, nb, err, work, in, buf);
  base += (unsigned)nb * grid;
  hipEventRecord(a, s);
  for (int r = 0; r < reps; ++r) {
    hipLaunchKernelGGL(k_persist, dim3(grid), dim3(256), 0, s, ctr, base, nb, err, work, in, buf);
    base += (unsigned)nb * grid;
  }
  hipEventRecord(b, s);
  hipEventSynchronize(b);
  int herr = 0;
  hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost);
  const double us = ms_between(a, b) * 1000.0 / reps / nb;
  hipFree(ctr);
  hipFree(err);
  hipFree(in);
  hipFree(buf);
  hipEventDestroy(a);
  hipEventDestroy(b);
  hipStreamDestroy(s);
  return herr ? -us : us;
}
}
