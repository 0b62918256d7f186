/* q3t_oracle.h — CPU restatement of the reference's per-frame decode path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library, and only as the checker / the timed CPU baseline — never as the product path.
 *
 * It restates, op by op, the GGML-CPU graphs of the reference (GGML_CUDA=OFF build):
 *   Talker step  src/tts_transformer.cpp:1376-1512     prefill  :1093-1374 (run token-by-token)
 *   CB0 logits   src/tts_transformer.cpp:2416-2495     frame loop :2342-2574
 *   Code pred.   src/tts_transformer.cpp:1514-1827,2153-2340 (+ TRT loop trt_code_predictor.cpp:484-600)
 *   Vocoder      src/audio_tokenizer_decoder.cpp:375-802 (FULL) ; src/trt_vocoder.cpp:98-170 (CHUNK40)
 *
 * Numerics (ggml_rounding = 1, default): "GGML-CPU semantics" — weights f16 as stored in the GGUF, every
 * matmul/conv input activation rounded to f16 (ggml mul_mat vec_dot_type F16, im2col F16), F16 KV caches,
 * f32 elsewhere, rms/layer-norm sums in double.  ggml_rounding = 0: pure fp32 activations and KV (used to
 * pin the restatement against the PyTorch export harness scripts/export_code_predictor.py:45-231).
 * The exact ggml internals (SIMD summation order, F16 V accumulator inside CPU flash_attn_ext, F16 GELU
 * table) are [ggml-upstream] and not pinned by any file in this container.
 */
#ifndef Q3T_ORACLE_H
#define Q3T_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    int hidden, n_layers, n_heads, n_kv, head_dim, inter, codec_vocab, n_codebooks, text_vocab, text_dim;
    int cp_layers, cp_vocab;
    float eps, rope_theta;
    int codec_pad, codec_bos, codec_eos, tts_bos, tts_eos, tts_pad, think, nothink, think_bos, think_eos;
    int has_vocoder, cb_dim, cb_size, voc_hidden, voc_latent, voc_heads, voc_layers, voc_ffn, dec_dim, up_k;
    int conv_t_k[4], rates[4];
    /* code predictor geometry (1.7B: cp_hidden != hidden, code_pred.mtp_proj projects talker-space inputs;
     * tts_transformer.cpp:370-389, 611-616, 1554-1560, 1709-1714); the 0.6B defaults are the talker's values */
    int cp_hidden, cp_inter, cp_heads, cp_kv, cp_head_dim, has_mtp;
} q3o_config;

typedef struct q3o_model q3o_model;
typedef struct q3o_kv q3o_kv;

const char *q3o_error(void);
q3o_model *q3o_load(const char *tts_gguf, const char *tok_gguf, int ggml_rounding);
void q3o_free(q3o_model *m);
void q3o_get_config(const q3o_model *m, q3o_config *c);
void q3o_set_threads(int n);

/* KV cache: which = 0 talker (n_layers), 1 code predictor (cp_layers). */
q3o_kv *q3o_kv_new(const q3o_model *m, int n_ctx, int which);
void q3o_kv_free(q3o_kv *kv);

/* one decode step of the 28-layer talker at position pos; hidden = output-normed hidden [H], logits [Vc] */
int q3o_talker_step(const q3o_model *m, q3o_kv *kv, const float *embd, int pos, float *hidden, float *logits);
/* same with only the first n_layers layers (golden-vector pinning through the 5-slot export harness) */
int q3o_talker_step_n(const q3o_model *m, q3o_kv *kv, const float *embd, int pos, int n_layers, float *hidden, float *logits);
/* text projection rows (tts_transformer.cpp:1026-1091) */
int q3o_project_text(const q3o_model *m, const int32_t *toks, int n, float *out);
/* prefill assembly (tts_transformer.cpp:1093-1231). prefill [<=10][H], trailing [max(1,n-8)][H], tts_pad [H] */
int q3o_prefill_embd(const q3o_model *m, const int32_t *toks, int n, const float *spk, int language_id,
                     float *prefill, int *prefill_len, float *trailing, int *trailing_len, float *tts_pad);
/* one code-predictor pass at pos (0..15); head<0: no lm_head; x is the pass input [H] */
int q3o_cp_pass(const q3o_model *m, q3o_kv *kv, const float *x, int pos, int head, float *hidden_out, float *logits);
/* 15 codes of one frame from the talker hidden + cb0. u15: 15 uniforms (sampling) or NULL for greedy. */
int q3o_cp_frame(const q3o_model *m, const float *hidden, int cb0, float temperature, int top_k, const float *u15,
                 int32_t *codes, float *logits_all);
/* same passes fed with the given codes15 (teacher forcing); logits_all [15][Vcp] */
int q3o_cp_frame_forced(const q3o_model *m, const float *hidden, int cb0, const int32_t *codes15, float *logits_all);
/* top-k/temperature sampling by inverse CDF (temperature<=0 => first-max argmax). keep_id>=0 survives top-k. */
int q3o_sample(const float *logits, int n, float temperature, int top_k, float u, int keep_id);
/* CB0 logit processing (tts_transformer.cpp:2417-2495) on logits in place; seen = [Vc] flags of emitted CB0s.
 * eos_mask != 0 (bench force_frames) masks EOS after the ramp. returns the token. */
int q3o_cb0_select(const q3o_model *m, float *logits, const uint8_t *seen, int frame, int n_tokens, float rep_penalty,
                   float temperature, int top_k, float u, int eos_mask);
/* deterministic uniform used by both the oracle and the HIP path */
float q3o_uniform(uint64_t seed, uint64_t utt, uint64_t frame, uint64_t cb);
/* full frame loop (tts_transformer.cpp:2342-2574). codes_out [max_len][16]. force_frames>0 masks EOS until
 * force_frames frames are produced. Returns 0 on success. step_embd_trace optional [max_len][H]. */
int q3o_generate(const q3o_model *m, const int32_t *toks, int n, const float *spk, int max_len, int language_id,
                 float rep_penalty, float temperature, int top_k, uint64_t seed, uint64_t utt, int force_frames,
                 int32_t *codes_out, int *n_frames, float *logits_trace, float *hidden_trace);
/* teacher-forced replay of forced[n_forced][16]; records the processed CB0 logits [n_forced][Vc] and the code
 * predictor logits [n_forced][15][Vcp] of every decision (greedy-parity checks with near-tie tolerance) */
int q3o_generate_forced(const q3o_model *m, const int32_t *toks, int n, const float *spk, int language_id, float rep,
                        int force_frames, const int32_t *forced, int n_forced, float *cb0_trace, float *cp_trace);
/* the same replay, tracing only frames >= from_frame (earlier frames advance the talker KV with their forced codes, no
 * selection or code-predictor work): traces hold n_forced - from_frame frames */
int q3o_generate_forced_from(const q3o_model *m, const int32_t *toks, int n, const float *spk, int language_id, float rep,
                             int force_frames, const int32_t *forced, int n_forced, int from_frame, float *cb0_trace,
                             float *cp_trace);
/* vocoder: mode 0 = FULL (audio_tokenizer_decoder.cpp), 1 = CHUNK40 (trt_vocoder.cpp:98-170).
 * pcm == NULL => only report the sample count. */
int q3o_vocoder_decode(const q3o_model *m, const int32_t *codes, int n_frames, int mode, float *pcm, int64_t *n_samples);
int64_t q3o_vocoder_len(const q3o_model *m, int n_frames, int mode);
/* speaker encoder (AudioTokenizerEncoder, src/audio_tokenizer_encoder.cpp): mel spectrogram [128][F] of 24 kHz samples
 * (mel == NULL: only *n_frames), and the ECAPA-TDNN embedding [q3o_speaker_dim] */
int q3o_mel(const q3o_model *m, const float *samples, int n, float *mel, int *n_frames);
int q3o_speaker_encode(const q3o_model *m, const float *samples, int n, float *embedding);
int q3o_speaker_dim(const q3o_model *m);
/* a tensor of either file as the model sees it (F16 weights / F32 vectors; quantised files dequantised at open), f32;
 * *src_type = the on-disk GGML type */
int q3o_tensor(const q3o_model *m, const char *name, float *out, int64_t n, int *src_type);
/* codebook i (0 = vq_first, 1..15 = vq_rest.i-1) as f32 [cb_size][cb_dim], after normalize_codebooks */
int q3o_codebook(const q3o_model *m, int i, float *out);

/* helpers exported for tests */
uint16_t q3o_f32_to_f16(float x);
float q3o_f16_to_f32(uint16_t h);
void q3o_rope_cache(float theta_base_pos, int dims, float freq_base, float *cache /*[dims]*/);

#ifdef __cplusplus
}
#endif
#endif
