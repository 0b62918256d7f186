// speaker.h — MI355X-native speaker encoder (ECAPA-TDNN) replacing AudioTokenizerEncoder
// (src/audio_tokenizer_encoder.{h,cpp}): log-mel front end as two f32 GEMMs (DFT basis, mel filterbank) instead of the
// reference's O(n_fft^2)-per-frame naive DFT (:96-106), then the SE-Res2Net / MFA / ASP / FC graph (:438-694) on the
// vocoder's implicit-GEMM conv kernels.  Activations are time-major [T][C] f32; every conv input is rounded to f16
// (ggml_conv_1d's F16 im2col) against the GGUF's F16 weights.
#pragma once
#include <string>
#include <vector>

#include "arena.h"
#include "gguf.h"
#include "vocoder_kernels.h"

namespace q3t {

class SpeakerEncoder {
public:
    ~SpeakerEncoder();
    // weights from the TTS GGUF (spk_enc.*) into `wa` (the context's weight blob: broadcast with it); false + error
    // when the tensors are absent or malformed
    bool load(const Gguf &g, WeightArena &wa, hipStream_t s);
    bool loaded() const { return loaded_; }
    int dim() const { return dim_; }
    int sample_rate() const { return sample_rate_; }
    // AudioTokenizerEncoder::encode (audio_tokenizer_encoder.h:107-108): samples in [-1, 1] at 24 kHz -> emb [dim()]
    bool encode(const float *samples, int n, float *emb);
    // mel spectrogram [n_frames][128] (time-major; test entry point)
    bool mel(const float *samples, int n, std::vector<float> &mel, int *n_frames);

private:
    struct Conv { uint16_t *w = nullptr; float *b = nullptr; int k = 0, ic = 0, oc = 0; };   // w [k][oc][ic]
    bool ensure(int T);
    bool upload(const float *samples, int n);   // host samples -> samples_ (grown on demand)
    bool run_mel(const float *samples_dev, int n, int F);
    // valid conv over a reflect-padded f16 copy of x[T][ldx] (pad rows each side; optional x2 added first)
    bool conv(const Conv &c, const float *x, int ldx, const float *x2, int ldx2, int T, int pad, int dil, float *y,
              int ldy, int act);
    template <class T> T *dalloc(size_t n);

    bool loaded_ = false;
    hipStream_t stream_ = nullptr;
    int dim_ = 0, sample_rate_ = 24000;
    Conv conv0_, mfa_, asp_tdnn_, asp_conv_, fc_;
    struct Blk { Conv tdnn1, tdnn2, res[7], se1, se2; } blk_[3];
    std::vector<void *> allocs_, scratch_;
    float *basis_ = nullptr, *fb_ = nullptr, *win_ = nullptr;   // DFT basis [1024][1026], filterbank [513][128], Hann
    int cap_T_ = 0, cap_n_ = 0;
    float *samples_ = nullptr;
    float *frames_ = nullptr, *spec_ = nullptr, *mag_ = nullptr, *mel_ = nullptr;
    float *x0_ = nullptr, *h_ = nullptr, *cat_ = nullptr, *y_ = nullptr, *mfa_out_ = nullptr, *blocks_ = nullptr,
          *att_ = nullptr, *att2_ = nullptr, *vec_ = nullptr;
    uint16_t *xh_ = nullptr;   // f16 conv input (reflect-padded copy / ASP [hs | mean | std])
};

}  // namespace q3t
