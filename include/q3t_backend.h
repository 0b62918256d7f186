/* q3t_backend.h — C ABI of the MI355X-native Qwen3-TTS decode path (libq3t.so).
 *
 * Plain pointers and sizes only; every call returns Q3T_OK (0) or Q3T_ERR (-1) and leaves a message in the
 * thread-local q3t_last_error() (the reference's `bool` + get_error() convention, src/tts_transformer.h:244,
 * src/trt_code_predictor.h:85).  One q3t_ctx per GPU; calls on one context are not thread-safe, contexts on
 * different devices may be driven by different host threads.  All buffers below are HOST buffers unless the
 * name says _dev; the hot path keeps everything resident in HBM between calls.
 *
 * Interfaces replaced (reference file:line):
 *   q3t_ctx_create        TTSTransformer::load_model (src/tts_transformer.h:170, .cpp:51) +
 *                         AudioTokenizerDecoder::load_model (src/audio_tokenizer_decoder.h:165) +
 *                         TRTCodePredictor::load_engine/upload_* (src/trt_code_predictor.h:31-50)
 *   q3t_generate          TTSTransformer::generate (src/tts_transformer.h:233-241, .cpp:2342-2574)
 *   q3t_generate_stream   the same with frame_callback_t on_frames / callback_interval (src/tts_transformer.h:224,
 *                         .cpp:2517-2523, 2563-2570; caller qwen3_tts.cpp:437-463: the TRT streaming vocoder)
 *   q3t_generate_queue    continuous batching over the same path (no reference counterpart: SURVEY §7 step 9,
 *                         the serving extension of TTSTransformer::generate to more utterances than slots)
 *   q3t_comm_unique_id,   SURVEY §8(e) multi-GPU start-up (no reference counterpart: the reference is one process
 *   q3t_ctx_create_shared on one Jetson): RCCL broadcast of rank 0's packed weight blobs over xGMI
 *   q3t_ctx_create_replica, q3t_comm_allreduce_max
 *   q3t_talker_forward    TTSTransformer::forward_step (src/tts_transformer.h:189-192, .cpp:1952-2028)
 *   q3t_talker_prefill    TTSTransformer::forward_prefill (src/tts_transformer.h:196-198, .cpp:1233-1374, 1829-1920)
 *   q3t_codepred_frame    TTSTransformer::predict_codes_autoregressive (src/tts_transformer.h:203-207) /
 *                         TRTCodePredictor::run_greedy_loop / run_sampling_loop (src/trt_code_predictor.h:68-79)
 *   q3t_cb0_select        CB0 logit processing inside generate (src/tts_transformer.cpp:2417-2499)
 *   q3t_project_text      TTSTransformer::project_text_tokens (src/tts_transformer.cpp:1026-1091)
 *   q3t_prefill_embd      TTSTransformer::build_prefill_graph (src/tts_transformer.cpp:1093-1231)
 *   q3t_vocoder_decode    AudioTokenizerDecoder::decode (src/audio_tokenizer_decoder.h:173-174) [FULL] and
 *                         TRTVocoderDecoder::decode (src/trt_vocoder.h:33-34) [CHUNK40]
 *   gpu_*                 the four extern "C" wrappers of src/trt_cuda_kernels.cu:10,60,78,183
 */
#ifndef Q3T_BACKEND_H
#define Q3T_BACKEND_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define Q3T_OK 0
#define Q3T_ERR (-1)
#define Q3T_VOCODER_FULL 0    /* whole utterance, GGML decoder semantics */
#define Q3T_VOCODER_CHUNK40 1 /* independent 40-frame chunks, 1920 samples/frame (TRT streaming) */

typedef struct q3t_ctx q3t_ctx;

typedef struct q3t_config {
    int32_t hidden, n_layers, n_heads, n_kv_heads, head_dim, intermediate;
    int32_t codec_vocab, n_codebooks, text_vocab, text_dim, cp_layers, cp_vocab;
    int32_t codec_eos, has_vocoder, sample_rate, max_slots, max_ctx;
    /* code predictor geometry (tts_transformer.cpp:370-389): equal to the talker's for 0.6B; 1.7B projects every
     * code-predictor input with code_pred.mtp_proj (has_mtp = 1) */
    int32_t cp_hidden, cp_intermediate, cp_heads, cp_kv_heads, has_mtp;
} q3t_config;

/* tts_params (src/qwen3_tts.h:18-43) + generate() arguments; top_p / n_threads are unused by the reference */
typedef struct q3t_gen_params {
    int32_t max_len;            /* max_audio_tokens (frames), default 4096 */
    int32_t language_id;        /* 2050 (english) as passed by synthesize_internal, qwen3_tts.cpp:459-463 */
    float repetition_penalty;   /* 1.05 */
    float temperature;          /* 0.9; <= 0 => greedy */
    int32_t top_k;              /* 50 */
    uint64_t seed;              /* counter-based sampler seed (the reference seeds std::mt19937 from random_device) */
    int32_t force_frames;       /* bench only: EOS masked until this many frames (0 = off) */
} q3t_gen_params;

const char *q3t_last_error(void);
void q3t_default_params(q3t_gen_params *p);

/* tts_gguf may be NULL: a vocoder-only context (AudioTokenizerDecoder::load_model / TRTVocoderDecoder::load_engine
 * without a talker); the talker entry points then fail with an error.  tokenizer_gguf may be NULL: no vocoder. */
int q3t_ctx_create(const char *tts_gguf, const char *tokenizer_gguf /* may be NULL: no vocoder */, int device,
                   int max_slots, int max_ctx, q3t_ctx **out);
void q3t_ctx_destroy(q3t_ctx *ctx);

/* ---- multi-GPU (one process per GPU): rank 0 calls q3t_comm_unique_id and hands the bytes to the other ranks by any
 * host channel; every rank then calls q3t_ctx_create_shared.  Only rank 0 reads tensor bytes from the GGUF files; the
 * other ranks parse the headers, lay out identical weight blobs and receive them by ncclBroadcast (RCCL over xGMI). */
#define Q3T_COMM_ID_BYTES 128
int q3t_comm_unique_id(uint8_t *id /* [Q3T_COMM_ID_BYTES] */);
int q3t_ctx_create_shared(const char *tts_gguf, const char *tokenizer_gguf, int device, int max_slots, int max_ctx,
                          int rank, int world, const uint8_t *id, q3t_ctx **out);
/* host-only weight layout of a model file (no device touched): the byte offset of every allocation of the talker blob
 * in order (n_alloc of them; offsets may be NULL to query n_alloc, else max_n entries) and the bytes used -- what every
 * rank of q3t_ctx_create_shared computes from the GGUF headers before the broadcast (whose size check compares
 * `used` across ranks) */
int q3t_plan_weight_layout(const char *tts_gguf, uint64_t *offsets, int max_n, int *n_alloc, uint64_t *used);
/* a second context whose weight blobs are copied device-to-device from src's (same or peer device, no file reads) */
int q3t_ctx_create_replica(q3t_ctx *src, int device, int max_slots, int max_ctx, q3t_ctx **out);
/* element-wise max over the ranks of a shared context (n <= 64 host doubles; also a barrier); no-op otherwise */
int q3t_comm_allreduce_max(q3t_ctx *ctx, double *values, int n);
int q3t_get_config(const q3t_ctx *ctx, q3t_config *out);

/* ---- hot path: prefill + frame loop for n_utt utterances batched in lock-step.
 * tokens[u] -> n_tokens[u] chat-template ids; speaker[u] -> hidden floats or speaker == NULL (all or none).
 * codes: [n_utt][p->max_len][16] int32 row-major [frame][codebook]; n_frames[u] = frames produced. */
int q3t_generate(q3t_ctx *ctx, int n_utt, const int32_t *const *tokens, const int32_t *n_tokens,
                 const float *const *speaker, const q3t_gen_params *p, int32_t *codes, int32_t *n_frames);
/* streaming: on_frames(user, u, codes [n][16], n, 16) is called on the caller's thread every `interval` frames of
 * utterance u with its newest `interval` frames, and once more after the loop with the remainder (< interval
 * frames, or the frames before EOS); returning 0 stops utterance u after the frames delivered so far.  The callback
 * may call q3t_vocoder_decode on the same context (it runs behind the frames already queued).  The callback runs
 * while the generate holds its device lock (shared for batches, exclusive for one utterance): it must not start a
 * one-utterance generate on another context of the same device, and a wait in it for another thread's work on the
 * same device can be delayed up to 20 ms by a one-utterance generate queued meanwhile (devlock.h). */
typedef int (*q3t_frame_cb)(void *user, int32_t utterance, const int32_t *codes, int32_t n_frames, int32_t n_codebooks);
int q3t_generate_stream(q3t_ctx *ctx, int n_utt, const int32_t *const *tokens, const int32_t *n_tokens,
                        const float *const *speaker, const q3t_gen_params *p, int32_t *codes, int32_t *n_frames,
                        q3t_frame_cb on_frames, void *user, int32_t interval);
/* continuous batching: n_utt utterances (any number; codes [n_utt][max_len][16], n_frames [n_utt]) through
 * min(max_slots, n_utt) slots with at most max_active (<= 0: all slots) in flight.  When an utterance ends (EOS or
 * max_len) its slot is refilled with the next one between two frames (prefill of the newcomer on that slot only).
 * Sampling is keyed by the utterance's index in the call, so an utterance's codes do not depend on its slot, on when
 * it was admitted or on its neighbours.  A newcomer's prefill runs on its own stream, overlapping the other slots'
 * decoding, with the batch's kernels (>= 4 slots: the first wave's codes equal q3t_generate's). */
int q3t_generate_queue(q3t_ctx *ctx, int n_utt, const int32_t *const *tokens, const int32_t *n_tokens,
                       const float *const *speaker, const q3t_gen_params *p, int32_t *codes, int32_t *n_frames,
                       int32_t max_active);
/* tuning knob (process-wide): batches of >= min_batch slots run the projections on the matrix cores (MFMA GEMM,
 * gemm_mfma.hip) instead of the weight-streaming GEMV; 0 disables the matrix-core path.  Default 4 (env
 * Q3T_MFMA_MIN_B).  Applies to graphs captured afterwards (create contexts after changing it). */
int q3t_set_mfma_min_batch(int min_batch);
/* wait until every operation queued on the context's device has finished (hipDeviceSynchronize) */
int q3t_synchronize(q3t_ctx *ctx);
/* device time (ms) of the last q3t_generate: prefill and frame loop */
int q3t_last_timing(const q3t_ctx *ctx, double *prefill_ms, double *frames_ms);

/* replay the captured stage graph (0 = talker decode step, 1 = 16-pass code-predictor frame) `iters` times at
 * KV position `pos` for n_slots slots; *ms = mean device time per replay (an event pair around each replay on the
 * context stream: the replay's own duration, not the host-side gap between two graph launches) */
int q3t_time_stage(q3t_ctx *ctx, int stage, int n_slots, int pos, int iters, double *ms);
/* the single-slot talker step and code-predictor frame as persistent launches (persist.hip, no reference
 * counterpart: they replace the per-op graphs of TTSTransformer::forward_step / TRTCodePredictor at batch 1):
 * -1 = not in use (shapes or device not supported, another context on the device holds the persistent kernels, or
 * Q3T_PERSIST=0), 0 = in use, 1 = a launch gave up waiting on an in-launch hand-off (protocol fault; the next call
 * falls back), 2 = disabled after such a fault: the context runs the bit-identical launch-per-op graphs */
int q3t_persist_status(q3t_ctx *ctx);
/* which single-slot persistent kernels the context launches (bit mask, 0 when none): 1 = talker step on
 * role-specialised workgroups (persist_tk.hip), 2 = talker step on all-role workgroups (persist.hip k_persist<0,CH>),
 * 4 = code-predictor frame on role-specialised workgroups (persist_cp.hip), 8 = code-predictor frame on all-role
 * workgroups (persist.hip k_persist<1|2,16>) */
int q3t_persist_kernels(q3t_ctx *ctx);

/* ---- vocoder */
int64_t q3t_vocoder_num_samples(const q3t_ctx *ctx, int32_t n_frames, int mode);
/* algorithmic FLOPs of one FULL decode of n_frames (sum of 2*M*K*N over the loaded conv / projection shapes and the
 * causal attention); bench.py's MFMA-utilisation figure.  -1 without a vocoder */
double q3t_vocoder_flops(const q3t_ctx *ctx, int32_t n_frames);
int q3t_vocoder_decode(q3t_ctx *ctx, const int32_t *codes /* [n_frames][16] */, int32_t n_frames, int mode,
                       float *pcm /* [q3t_vocoder_num_samples] */, int64_t *n_samples);

/* TRTVocoderDecoder::decode (src/trt_vocoder.h:33-34) with the engine's fixed_frames: independent chunk_frames-long
 * chunks, n_frames * 1920 samples (pcm capacity); n_codebooks must be 16 */
int q3t_vocoder_decode_chunked(q3t_ctx *ctx, const int32_t *codes /* [n_frames][n_codebooks] */, int32_t n_frames,
                               int32_t n_codebooks, int32_t chunk_frames, float *pcm, int64_t *n_samples);

/* Several utterances through shared launches (the batched counterpart of q3t_vocoder_decode /
 * q3t_vocoder_decode_chunked; the reference decodes one utterance per call, qwen3_tts.cpp:518 /
 * trt_vocoder.cpp:98-170).  FULL: utterances run as batches of up to q3t_vocoder_set_batch_frames frames (default
 * 4096), each padded to its batch's longest; the decoder is causal end to end, so pcm[u] is exactly
 * q3t_vocoder_decode(codes[u]).  CHUNK40: every chunk_frames-long chunk of every utterance is one independent sequence
 * of the batch; pcm[u] equals q3t_vocoder_decode_chunked(codes[u]).  codes[u]: [n_frames[u]][16];
 * pcm[u]: capacity q3t_vocoder_num_samples(n_frames[u], mode); n_samples[u] receives its length. */
int q3t_vocoder_decode_batch(q3t_ctx *ctx, int32_t n_utt, const int32_t *const *codes, const int32_t *n_frames,
                             int mode, int32_t chunk_frames, float *const *pcm, int64_t *n_samples);
/* frames (utterances x frames) per batched vocoder launch sequence; scratch grows to ~3 MB per frame */
int q3t_vocoder_set_batch_frames(q3t_ctx *ctx, int32_t frames);

/* ---- speaker encoder (ECAPA-TDNN; the TTS GGUF's spk_enc.* tensors)
 * q3t_speaker_dim: embedding length, 0 when the model has no speaker encoder.
 * q3t_speaker_encode: AudioTokenizerEncoder::encode (src/audio_tokenizer_encoder.h:107-108): samples in [-1, 1] at
 * 24 kHz -> embedding [q3t_speaker_dim]; Q3T_ERR + q3t_last_error() when the audio is too short (< 5 mel frames).
 * q3t_speaker_mel: its log-mel front end (compute_mel_spectrogram, audio_tokenizer_encoder.cpp:281-364), time-major
 * [n_frames][128]; mel may be NULL to query *n_frames. */
int q3t_speaker_dim(const q3t_ctx *ctx);
/* a context holding only the speaker encoder (AudioTokenizerEncoder::load_model reads only spk_enc.* tensors) */
int q3t_ctx_create_speaker(const char *tts_gguf, int device, q3t_ctx **out);
int q3t_speaker_encode(q3t_ctx *ctx, const float *samples, int32_t n_samples, float *embedding);
int q3t_speaker_mel(q3t_ctx *ctx, const float *samples, int32_t n_samples, float *mel, int32_t cap_frames,
                    int32_t *n_frames);

/* ---- text tokenizer (host side; TextTokenizer, src/text_tokenizer.h:21-86 / text_tokenizer.cpp:80-349)
 * q3t_tokenizer_load reads tokenizer.ggml.tokens / merges / *_token_id from a GGUF (the TTS model file).
 * q3t_tokenizer_encode: for_tts != 0 wraps the text in the TTS template (encode_for_tts, :293-330); *n_tokens receives
 * the count, tokens may be NULL to query it, Q3T_ERR when cap is too small.
 * q3t_tokenizer_decode: bytes of the decoded text (not NUL-terminated), *n_bytes its length; text may be NULL. */
typedef struct q3t_tokenizer q3t_tokenizer;
int q3t_tokenizer_load(const char *gguf_path, q3t_tokenizer **out);
void q3t_tokenizer_free(q3t_tokenizer *tok);
int q3t_tokenizer_info(const q3t_tokenizer *tok, int32_t *vocab_size, int32_t *bos_id, int32_t *eos_id,
                       int32_t *pad_id);
int q3t_tokenizer_encode(const q3t_tokenizer *tok, const char *text, int64_t n_bytes /* < 0: NUL-terminated */,
                         int for_tts, int32_t *tokens, int32_t cap, int32_t *n_tokens);
int q3t_tokenizer_decode(const q3t_tokenizer *tok, const int32_t *tokens, int32_t n, char *text, int64_t cap,
                         int64_t *n_bytes);

/* ---- stage entry points (used by the parity tests; each syncs the context stream) */
int q3t_talker_forward(q3t_ctx *ctx, int n_slots, const float *embd /* [n][H] */, const int32_t *pos /* [n] */,
                       float *hidden /* [n][H] or NULL */, float *logits /* [n][codec_vocab] or NULL */);
/* causal prefill from position 0 (the pass q3t_generate runs): the n_rows <= 10 rows of each of n_utt utterances in one
 * pass, K/V into slots 0..n_utt-1; hidden = the final-norm hidden state of every row, logits = the codec logits of each
 * utterance's last row.  family_slots (0: n_utt) picks the kernels of a family_slots-slot decode step: every row then
 * equals q3t_talker_forward with that many slots replayed at its position, bit for bit. */
int q3t_talker_prefill(q3t_ctx *ctx, int n_utt, int n_rows, const float *embd /* [n_utt][n_rows][H] */, int family_slots,
                       float *hidden /* [n_utt][n_rows][H] or NULL */, float *logits /* [n_utt][codec_vocab] or NULL */);
int q3t_codepred_frame(q3t_ctx *ctx, int n_slots, const float *hidden /* [n][H] */, const int32_t *cb0 /* [n] */,
                       float temperature, int32_t top_k, uint64_t seed, int32_t frame,
                       int32_t *codes15 /* [n][15] */, float *logits /* [n][15][cp_vocab] or NULL */);
int q3t_cb0_select(q3t_ctx *ctx, int n_slots, const float *logits /* [n][V] */, const uint8_t *seen /* [n][V] */,
                   const int32_t *frame, const int32_t *n_tokens, const q3t_gen_params *p, int32_t *tokens);
int q3t_project_text(q3t_ctx *ctx, int n, const int32_t *tokens, float *out /* [n][H] */);
int q3t_prefill_embd(q3t_ctx *ctx, const int32_t *tokens, int n, const float *speaker, int language_id,
                     float *prefill /* [10][H] */, int32_t *prefill_len, float *trailing /* [max(1,n-8)][H] */,
                     int32_t *trailing_len, float *tts_pad /* [H] */);

/* ---- drop-in replacements of src/trt_cuda_kernels.cu (device pointers, stream = hipStream_t or NULL) */
void gpu_fp32_to_fp16(const float *in, void *out, int n, void *stream);
void gpu_argmax_f32(const float *in, int32_t *out, int n, void *stream);
void gpu_embedding_lookup_by_gpu_id(const int32_t *token_id_ptr, const float *table, float *output, int embd_dim,
                                    void *stream);
void gpu_sample_topk_f32(const float *logits, const float *rand_val, int32_t *out, float temperature, int32_t top_k,
                         int32_t vocab_size, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* Q3T_BACKEND_H */
