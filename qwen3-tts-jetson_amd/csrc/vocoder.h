// vocoder.h — MI355X-native Qwen3-TTS tokenizer decoder ("vocoder"), replacing TRTVocoderDecoder
// (src/trt_vocoder.cpp) and the GGML AudioTokenizerDecoder (src/audio_tokenizer_decoder.cpp).
#pragma once
#include <cstdlib>
#include <string>
#include <vector>

#include "arena.h"
#include "gguf.h"
#include "kernels.h"

namespace q3t {

class Vocoder {
public:
    ~Vocoder();
    bool load(const std::string &tok_gguf, hipStream_t s, bool recv_weights = false);
    WeightArena &weights() { return wa_; }
    // mode 0 = FULL (GGML decoder semantics), 1 = CHUNK40 (TRT streaming semantics)
    int64_t n_samples(int n_frames, int mode) const;
    // chunk_frames: the fixed chunk length of the chunked mode (TRTVocoderDecoder::load_engine's fixed_frames)
    bool decode(const int32_t *codes_host, int n_frames, int mode, float *pcm_host, int64_t *n_out, int chunk_frames = 40);
    // n_utt utterances through shared launches: FULL decodes run as utterance batches (every conv / attention launch
    // covers up to batch_frames() frames of utterances padded to the batch's longest; the decoder is causal end to end,
    // so each utterance's samples are exactly its own decode's); CHUNK40 decodes every chunk of every utterance as one
    // batch of independent chunk_frames-long sequences.  pcm[u] capacity >= n_samples(n_frames[u], mode)
    bool decode_batch(int n_utt, const int32_t *const *codes_host, const int *n_frames, int mode, float *const *pcm_host,
                      int64_t *n_out, int chunk_frames = 40);
    // FULL decode of device-resident codes [nb][F][16] into pcm_dev [nb][n_samples(F, 0)]; ensure(F, nb) first
    bool decode_device(const int32_t *codes_dev, int n_frames, float *pcm_dev, int64_t *n_out, hipStream_t s, int nb = 1);
    bool ensure(int n_frames, int nb = 1);
    // frames per batched launch sequence (utterances x frames); scratch grows to this (~3 MB per frame)
    int batch_frames() const { return batch_frames_; }
    void set_batch_frames(int f) { batch_frames_ = f > 0 ? f : 4096; }
    bool loaded() const { return loaded_; }
    int n_usage_normalised() const { return n_usage_; }
    // algorithmic FLOPs of one FULL decode of F frames: 2*M*K*N over every conv (per tap), transposed conv, projection
    // and the causal attention (QK^T + PV over the lower triangle), from the loaded shapes
    double decode_flops(int n_frames) const;   // codebooks divided by *.usage at load (0 for converter output)

private:
    struct Conv { uint16_t *w = nullptr; float *b = nullptr; int k = 0, ic = 0, oc = 0; };   // w: [k][oc][ic]
    struct Snake { float *a = nullptr, *ib = nullptr; int n = 0; };                          // exp(alpha), exp(-beta)
    struct Layer {
        uint16_t *qkv = nullptr, *o = nullptr, *gu = nullptr, *down = nullptr;
        float *attn_norm = nullptr, *ffn_norm = nullptr, *attn_scale = nullptr, *ffn_scale = nullptr;
    };
    struct Up {
        Conv ct;
        uint16_t *dw = nullptr, *pw1 = nullptr, *pw2 = nullptr;
        float *dw_b = nullptr, *norm_w = nullptr, *norm_b = nullptr, *gamma = nullptr, *pw1_b = nullptr, *pw2_b = nullptr;
        int dw_k = 7, pw_dim = 0;
    };
    struct Res { Snake a1, a2; Conv c1, c2; int dil = 1; };
    struct Dec { Snake snake; Conv ct; Res res[3]; int rate = 1; };

    template <class T> T *dalloc(size_t n);
    int64_t full_len(int F) const;
    bool run_conv(const Conv &c, const float *x, int T, int pad, int dil, const Snake *sn, float *y, const float *resid,
                  int act, hipStream_t s);
    bool run_convT(const Conv &c, const float *x, int T, int stride, int trim, const Snake *sn, float *y, int T_out,
                   hipStream_t s);
    // the same convs on an f16 input already snake'd by the producer's epilogue; outputs f32 y and/or
    // y16 = f16(next_snake(y)) (the next conv's input), either may be null
    bool conv16(const Conv &c, const uint16_t *xh, int T, int pad, int dil, float *y, const float *resid, uint16_t *y16,
                const Snake *next, hipStream_t s);
    bool convT16(const Conv &c, const uint16_t *xh, int T, int stride, int trim, float *y, int T_out, uint16_t *y16,
                 const Snake *next, hipStream_t s);
    bool decode_rows(const int32_t *codes_dev, int F, float *pcm_dev, int64_t *n_out, hipStream_t s);

    bool loaded_ = false;
    hipStream_t stream_ = nullptr;
    std::vector<void *> allocs_, scratch_;
    WeightArena wa_;   // every weight tensor (one blob)
    int n_usage_ = 0;
    int cb_dim_ = 0, cb_size_ = 0, hidden_ = 0, latent_ = 0, n_heads_ = 16, head_dim_ = 64, ffn_ = 0;
    uint16_t *cb_first_ = nullptr, *cb_rest_[15] = {}, *vq_first_out_ = nullptr, *vq_rest_out_ = nullptr;
    uint16_t *in_proj_ = nullptr, *out_proj_ = nullptr;
    float *in_proj_b_ = nullptr, *out_proj_b_ = nullptr, *pre_norm_ = nullptr;
    Conv pre_conv_, dec0_, dec6_;
    std::vector<Layer> layers_;
    Up up_[2];
    Dec dec_[4];
    Snake dec5_;
    // scratch (grown by ensure)
    int cap_frames_ = 0, batch_frames_ = 4096;
    size_t cap_big_ = 0, cap_ftot_ = 0, cap_pcm_ = 0;
    int nb_ = 1;   // utterances of the decode in flight (conv launches carry it as grid z)
    // the 96-channel residual units as one launch each (vocoder_resunit.hip); Q3T_VOC_FUSE=0: the two-conv form
    bool fuse_res_ = [] { const char *e = std::getenv("Q3T_VOC_FUSE"); return !(e && e[0] == '0'); }();
    float *buf_[3] = {nullptr, nullptr, nullptr};
    uint16_t *xh_ = nullptr;   // f16 (snake'd) conv input, one activation
    uint16_t *xh2_ = nullptr;  // second f16 activation: the decoder blocks ping-pong conv inputs written by epilogues
    int32_t *codes_ = nullptr;
    int *cols_ = nullptr;
    float *pcm_ = nullptr, *rope_ = nullptr;
};

}  // namespace q3t
