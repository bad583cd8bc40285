// Acoustic feature pipeline of the data loader: the FBANK + log power + delta
// features of mr_gen's AudioPreprocessor (mr_gen/utils/preprocess/audio.py:6-67) and the delta
// stacking shared with MotionPreprocessorNX (motion_nx.py:49-58), on the GPU.
//
//   spectrum   frames x [cos | sin] DFT basis (window folded in), one GEMM (gemm.hip, x6): the
//              frames are read in place from the waveform with a RowMap of stride `hop`
//   finish     THIS FILE: |X_k|^2, the triangular mel filterbank, log(max(mel, 1e-6)) and the
//              per-frame log power log(max(sum x^2, 1e-10)) over the raw (unwindowed) samples
//              (audio.py:33-35,43-56), written as one [frames, nmels + 1] row each
//   delta      THIS FILE: cat([x[d:], delta1[d-1:], delta2]) with delta1 = x[1:] - x[:-1],
//              delta2 = delta1[1:] - delta1[:-1] in the reference's operation order (audio.py:58-67)
//
// Per frame the finish step reads 2*NF spectrum floats and nfft samples and writes nmels + 1
// floats: HBM-bound, one wave per frame, the power spectrum staged in LDS for the mel dots.
#include "mrg_common.h"

namespace mrg {

static constexpr int FB_MAXF = 1025;  // n_fft <= 2048

__global__ __launch_bounds__(256) void fbank_finish_kernel(int F, int NF, int NM, const float* __restrict__ spec,
                                                           long spec_ld, const float* __restrict__ melfb,
                                                           const float* __restrict__ wave, long hop, int nfft,
                                                           int fpc, long clip_len, float* __restrict__ out,
                                                           long out_ld) {
  __shared__ float pw[4][FB_MAXF];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int f = blockIdx.x * 4 + w;
  const bool fv = f < F;
  if (fv) {
    const float* sp = spec + (long)f * spec_ld;
    for (int k = lane; k < NF; k += 64) {
      const float re = sp[k], im = sp[NF + k];
      pw[w][k] = re * re + im * im;
    }
    // log power of the raw frame (audio.py:43-56)
    const float* x = wave + (long)(f / fpc) * clip_len + (long)(f % fpc) * hop;  // clip, frame in clip
    float s = 0.0f;
    for (int n = lane; n < nfft; n += 64) s = fmaf(x[n], x[n], s);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if (lane == 0) out[(long)f * out_ld + NM] = logf(fmaxf(s, 1e-10f));
  }
  __syncthreads();
  if (fv) {
    for (int j = lane; j < NM; j += 64) {
      float m = 0.0f;
      for (int k = 0; k < NF; ++k) m = fmaf(pw[w][k], melfb[(long)k * NM + j], m);
      // log(clamp(clamp(mel, 1e-10), 1e-6)) (audio.py:22,34) = log(max(mel, 1e-6))
      out[(long)f * out_ld + j] = logf(fmaxf(m, 1e-6f));
    }
  }
}

// nclip independent sequences x [nclip][T][C] (row stride ldx) -> out [nclip][T - order][C * (order + 1)];
// out row t of a sequence:
//   order 0: x[t];  order 1: [x[t+1], x[t+1] - x[t]];
//   order 2: [x[t+2], x[t+2] - x[t+1], (x[t+2] - x[t+1]) - (x[t+1] - x[t])]
__global__ __launch_bounds__(256) void feature_delta_kernel(int nclip, int T, int C, const float* __restrict__ x,
                                                            long ldx, int order, float* __restrict__ out) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  const int rows = T - order;
  if (i >= (long)nclip * rows * C) return;
  const long row = i / C;
  const int c = i % C;
  const long n = row / rows;
  const int t = row % rows;
  const int W = C * (order + 1);
  float* o = out + row * W;
  x += n * T * ldx;
  const float x0 = x[(long)t * ldx + c];
  if (order == 0) {
    o[c] = x0;
    return;
  }
  const float x1 = x[(long)(t + 1) * ldx + c];
  if (order == 1) {
    o[c] = x1;
    o[C + c] = x1 - x0;
    return;
  }
  const float x2 = x[(long)(t + 2) * ldx + c];
  const float d1a = x1 - x0, d1b = x2 - x1;
  o[c] = x2;
  o[C + c] = d1b;
  o[2 * C + c] = d1b - d1a;
}

}  // namespace mrg

using namespace mrg;

MRG_API int mrg_fbank_finish(int F, int NF, int NM, const float* spec, long spec_ld, const float* melfb,
                             const float* wave, long hop, int nfft, int frames_per_clip, long clip_len, float* out,
                             long out_ld, hipStream_t stream) {
  MRG_REQUIRE(F >= 0 && NF > 0 && NF <= FB_MAXF && NM > 0 && nfft > 0 && hop > 0 && frames_per_clip > 0,
              "mrg_fbank_finish: bad sizes (F=%d NF=%d NM=%d nfft=%d hop=%ld fpc=%d)", F, NF, NM, nfft, hop,
              frames_per_clip);
  if (F == 0) return 0;
  fbank_finish_kernel<<<(unsigned)((F + 3) / 4), 256, 0, stream>>>(F, NF, NM, spec, spec_ld, melfb, wave, hop, nfft,
                                                                   frames_per_clip, clip_len, out, out_ld);
  return check_launch("fbank_finish_kernel");
}

MRG_API int mrg_feature_delta(int nclip, int T, int C, const float* x, long ldx, int order, float* out,
                              hipStream_t stream) {
  MRG_REQUIRE(order >= 0 && order <= 2, "mrg_feature_delta: delta_order must be 0, 1 or 2 (got %d)", order);
  MRG_REQUIRE(nclip >= 0 && T > order && C > 0, "mrg_feature_delta: %d frames cannot carry delta order %d", T, order);
  const long n = (long)nclip * (T - order) * C;
  if (n == 0) return 0;
  feature_delta_kernel<<<(unsigned)((n + 255) / 256), 256, 0, stream>>>(nclip, T, C, x, ldx, order, out);
  return check_launch("feature_delta_kernel");
}

// ---------------------------------------------------------------------------------------------
// collate_fn (lstmformer/dataloader.py:114-121: pack_sequence + pad_packed_sequence(batch_first,
// padding_value=-100)): B variable-length [len_b, F] sequences -> out [B, Tmax, F], rows past
// len_b filled with `pad`.  Sequence b's rows are read from seqs[b] (device pointer table).
__global__ __launch_bounds__(256) void pad_sequences_kernel(int B, int Tmax, int F, const float* const* seqs,
                                                            const int* lens, float pad, float* out) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  const long per = (long)Tmax * F;
  if (i >= (long)B * per) return;
  const int b = i / per;
  const long r = i - (long)b * per;
  const int t = r / F;
  out[i] = t < lens[b] ? seqs[b][r] : pad;
}

MRG_API int mrg_pad_sequences(int B, int Tmax, int F, const float* const* seqs, const int* lens, float pad,
                              float* out, hipStream_t stream) {
  MRG_REQUIRE(B >= 0 && Tmax >= 0 && F >= 0, "mrg_pad_sequences: bad sizes");
  const long n = (long)B * Tmax * F;
  if (n == 0) return 0;
  pad_sequences_kernel<<<(unsigned)((n + 255) / 256), 256, 0, stream>>>(B, Tmax, F, seqs, lens, pad, out);
  return check_launch("pad_sequences_kernel");
}
