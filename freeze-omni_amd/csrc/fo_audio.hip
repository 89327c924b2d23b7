// Kaldi fbank on the GPU for the streaming front end, one workgroup per (user, frame).
//
// Replaces torchaudio.compliance.kaldi.fbank as called by the reference's chunk framers
// (bin/inference.py:71-80 framing A 25/10 ms, models/AudioFeatureGating.py:54-75 framing B 16/8 ms):
// snip-edges framing, DC removal, pre-emphasis 0.97 (x[-1] = x[0]), povey window, zero pad to a
// power of two, radix-2 FFT in LDS, |X|^2, kaldi mel triangles, log(max(e, FLT_EPSILON)).
// Window, twiddle and mel tables are computed once on the host (double precision).
#include "fo_common.h"

namespace {

constexpr int NFFT_MAX = 512;

__global__ __launch_bounds__(256) void k_fbank(const float* samples, int ld_s, int wl, int ws, int nfft, int log2n,
                                               const float* window, const float* tw_cos, const float* tw_sin,
                                               const float* mel, int nmel, float* out, int ld_b, int row0,
                                               const int* zero_rows) {
  __shared__ float x[NFFT_MAX];
  __shared__ float re[NFFT_MAX];
  __shared__ float im[NFFT_MAX];
  __shared__ float red[4];
  const int b = blockIdx.x, f = blockIdx.y;
  if (zero_rows && f < zero_rows[b]) {  // first chunk after reset: carried frames are zeros
    for (int m = threadIdx.x; m < nmel; m += 256) out[(size_t)b * ld_b + (size_t)(row0 + f) * nmel + m] = 0.f;
    return;
  }
  const float* src = samples + (size_t)b * ld_s + (size_t)f * ws;
  float s = 0.f;
  for (int i = threadIdx.x; i < wl; i += 256) {
    const float v = src[i];
    x[i] = v;
    s += v;
  }
  const float mean = block_sum<4>(s, red) / (float)wl;
  // pre-emphasis + window into bit-reversed positions
  for (int i = threadIdx.x; i < nfft; i += 256) {
    float y = 0.f;
    if (i < wl) {
      const float xi = x[i] - mean;
      const float xp = (i > 0 ? x[i - 1] : x[0]) - mean;
      y = (xi - 0.97f * xp) * window[i];
    }
    const int r = (int)(__brev((unsigned)i) >> (32 - log2n));
    re[r] = y;
    im[r] = 0.f;
  }
  __syncthreads();
  for (int m = 1; m < nfft; m <<= 1) {  // butterflies of span 2m
    for (int k = threadIdx.x; k < nfft / 2; k += 256) {
      const int grp = k / m, pos = k % m;
      const int i0 = grp * 2 * m + pos, i1 = i0 + m;
      const int tidx = pos * (nfft / (2 * m));
      const float c = tw_cos[tidx], sn = tw_sin[tidx];  // exp(-2 pi i tidx / nfft)
      const float xr = re[i1] * c + im[i1] * sn;
      const float xi = im[i1] * c - re[i1] * sn;
      const float ar = re[i0], ai = im[i0];
      re[i0] = ar + xr;
      im[i0] = ai + xi;
      re[i1] = ar - xr;
      im[i1] = ai - xi;
    }
    __syncthreads();
  }
  const int nb = nfft / 2 + 1;
  for (int k = threadIdx.x; k < nb; k += 256) x[k] = re[k] * re[k] + im[k] * im[k];
  __syncthreads();
  for (int m = threadIdx.x; m < nmel; m += 256) {
    const float* row = mel + (size_t)m * nb;
    float e = 0.f;
    for (int k = 0; k < nb; ++k) e += x[k] * row[k];
    out[(size_t)b * ld_b + (size_t)(row0 + f) * nmel + m] = logf(fmaxf(e, 1.1920928955078125e-07f));
  }
}

// feats[b][0:ov] = feats[b][R-ov:R] (chunk_data_shift, bin/inference.py:66-69)
__global__ void k_rows_shift(float* feats, int B, int R, int ov, int D) {
  const long long total = (long long)B * ov * D;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(e % D);
    const int r = (int)((e / D) % ov);
    const int b = (int)(e / ((long long)ov * D));
    feats[((size_t)b * R + r) * D + c] = feats[((size_t)b * R + R - ov + r) * D + c];
  }
}

}  // namespace

extern "C" {

// samples [B][ld_s] (already scaled to int16 range); writes n_frames rows at row0 of each user's
// [R][nmel] feature block (ld_b = R*nmel floats between users).
int fo_fbank(const float* samples, int ld_s, int B, int n_samples, int wl, int ws, int nfft, const float* window,
             const float* tw_cos, const float* tw_sin, const float* mel, int nmel, float* out, int ld_b, int row0,
             const int* zero_rows, hipStream_t s) {
  FO_REQUIRE(nfft <= NFFT_MAX && (nfft & (nfft - 1)) == 0 && wl <= nfft && n_samples >= wl,
             "fo_fbank: bad framing wl=%d nfft=%d n=%d", wl, nfft, n_samples);
  const int frames = 1 + (n_samples - wl) / ws;
  int log2n = 0;
  while ((1 << log2n) < nfft) ++log2n;
  hipLaunchKernelGGL(k_fbank, dim3(B, frames), dim3(256), 0, s, samples, ld_s, wl, ws, nfft, log2n, window, tw_cos,
                     tw_sin, mel, nmel, out, ld_b, row0, zero_rows);
  return fo::check_launch("fo_fbank");
}

int fo_rows_shift(float* feats, int B, int R, int ov, int D, hipStream_t s) {
  FO_REQUIRE(R - ov >= ov, "fo_rows_shift: overlapping shift");
  const long long n = (long long)B * ov * D;
  if (n == 0) return 0;
  long long g = (n + 255) / 256;
  hipLaunchKernelGGL(k_rows_shift, dim3((int)(g > 4096 ? 4096 : g)), dim3(256), 0, s, feats, B, R, ov, D);
  return fo::check_launch("fo_rows_shift");
}

}  // extern "C"
