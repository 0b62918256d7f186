// engine.h — MI355X-native runtime of the per-frame decode path (Talker step -> CB0 -> Code Predictor ->
// step embedding), replacing the reference's TTSTransformer::generate hot loop (src/tts_transformer.cpp:2342-2574)
// and TRTCodePredictor (src/trt_code_predictor.cpp).  B utterances ("slots") advance in lock-step; every
// per-frame kernel reads positions / frame counters from device memory so one hipGraph replays every frame.
#pragma once
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "arena.h"
#include "gguf.h"
#include "kernels.h"

namespace q3t {

struct Config {
    int hidden = 1024, n_layers = 28, n_heads = 16, n_kv = 8, head_dim = 128, inter = 3072;
    int codec_vocab = 3072, n_codebooks = 16, text_vocab = 151936, text_dim = 2048;
    int cp_layers = 5, cp_vocab = 2048;
    // code predictor geometry (tts_transformer.cpp:370-389): the talker's values for 0.6B; 1.7B has its own hidden /
    // FFN width behind code_pred.mtp_proj (talker space -> code-predictor space, applied to every pass input)
    int cp_hidden = 1024, cp_inter = 3072, cp_heads = 16, cp_kv = 8;
    bool has_mtp = false;
    float eps = 1e-6f, rope_theta = 1e6f;
    int codec_pad = 2148, codec_bos = 2149, codec_eos = 2150;
    int tts_bos = 151672, tts_eos = 151673, tts_pad = 151671;
    int think = 2154, nothink = 2155, think_bos = 2156, think_eos = 2157;
};

struct GenParams {
    int max_len = 4096;
    int language_id = 2050;
    float rep_penalty = 1.05f;
    float temperature = 0.9f;
    int top_k = 50;
    uint64_t seed = 0;
    int force_frames = 0;      // bench: mask EOS until this many frames are produced
};

struct DevLayer {
    uint16_t *qkv = nullptr, *o = nullptr, *gu = nullptr, *down = nullptr;
    float *attn_norm = nullptr, *ffn_norm = nullptr, *qn = nullptr, *kn = nullptr;
};

class Vocoder;
class SpeakerEncoder;
struct PLayerW;

// Path-selection knobs, read once from the environment when a context is created (the reference's own pattern:
// QWEN3_TTS_LOW_MEM, src/qwen3_tts.cpp:125-129).  All default to the fastest path; the alternatives exist so that
// the tests can compare paths that must agree (persistent vs launch-per-op, sequential vs split attention).
//   Q3T_PERSIST=0          single-slot talker step as launch-per-phase graphs instead of the persistent kernel
//   Q3T_PERSIST_CP=0       single-slot code-predictor frame as per-op launches
//   Q3T_PERSIST_CPB=0      batched (matrix-core) code-predictor frame as per-op launches (persist_cpb.hip otherwise)
//   Q3T_PERSIST_TKB=0      batched (matrix-core) talker step as per-op launches (persist_tkb.hip otherwise)
//   Q3T_CP_FUSED_ATTN=0    code-predictor attention as its own launch (the arithmetic the persistent frame reproduces)
//   Q3T_FUSED_SELECT=0     token selection as standalone launches
//   Q3T_CP_DEFER_SELECT=0  code-predictor tokens selected in the head launch
//   Q3T_ATTN_SPLIT=1       batched attention always split-K (k_attn) instead of k_attn_seq at >= 16 slots
//   Q3T_PERSIST_FAULT_AT=n test hook: the n-th persistent launch of the context flags a hand-off fault
// Development-only knobs (Q3T_TALKER_LAYERS, Q3T_PERSIST_PROF, ...) exist only in a -DQ3T_DEV build.
struct Options {
    bool persist = true, persist_cp = true, cp_fused_attn = true, fused_select = true, defer_cp_select = true;
    bool cp_qkv_table = true;   // Q3T_CP_QKV_TABLE: the persistent code-predictor frame reads layer 0's QKV rows from a table
    bool cp_roles = true;       // Q3T_CP_ROLES: that frame on role-specialised workgroups (persist_cp.hip)
    bool mm_cp_table = true;    // Q3T_MM_CP_TABLE: batched code predictor, layer 0 of passes 1..15 from the QKV table
    bool fold_advance = true;   // Q3T_FOLD_ADVANCE: the single-slot role talker kernel advances pos / frame (no k_advance)
    bool tk_roles = true;       // Q3T_TK_ROLES: the 1-slot talker step on role-specialised workgroups (persist_tk.hip)
    bool cpb = true;            // Q3T_PERSIST_CPB: the batched (2..64-slot) code-predictor frame as one persistent launch
    bool tkb = true;            // Q3T_PERSIST_TKB: the batched (16..64-policy-slot) talker step as one persistent launch
    bool attn_split = false;
    unsigned persist_fault_at = 0;
    int poll_every = 16;   // frames between done-flag polls
    static Options from_env();
};

class Engine {
public:
    Engine();
    ~Engine();
    // recv_weights: lay out the weight arenas from the GGUF headers only; the bytes are filled afterwards by
    // copy_weights_from() or an RCCL broadcast of weight_arenas()
    // host-only weight layout of a model file (no device): allocation offsets in order, bytes used
    bool plan_layout(const std::string &tts_gguf, std::vector<size_t> &offsets, size_t &used);
    bool load(const std::string &tts_gguf, const std::string &tok_gguf, int device, int max_slots, int max_ctx,
              bool recv_weights = false);
    // the packed weight blobs (talker + code predictor + embeddings; vocoder), in broadcast order
    std::vector<WeightArena *> weight_arenas();
    const Config &cfg() const { return c_; }
    int max_slots() const { return max_slots_; }
    int device() const { return device_; }
    const std::string &tts_path() const { return tts_path_; }
    // speaker-encoder-only context (AudioTokenizerEncoder::load_model, audio_tokenizer_encoder.cpp: only the
    // spk_enc.* tensors of the TTS GGUF are read)
    bool load_speaker_only(const std::string &tts_gguf, int device);
    bool has_talker() const { return talker_; }
    const std::string &tok_path() const { return tok_path_; }
    int max_ctx() const { return max_ctx_; }
    hipStream_t stream() const { return stream_; }
    Vocoder *vocoder() { return voc_.get(); }
    SpeakerEncoder *speaker() { return spk_.get(); }   // null when the TTS GGUF has no spk_enc.* tensors

    // ---- hot path: prefill + frame loop for n_utt utterances (codes [n_utt][max_len][ncb])
    // on_frames (frame_callback_t, src/tts_transformer.h:224): called every `interval` frames per utterance with its
    // newest `interval` frames, plus one final flush of the remainder; returning 0 stops that utterance
    // (src/tts_transformer.cpp:2517-2523, 2563-2570)
    typedef int (*FrameCb)(void *user, int slot, const int32_t *codes, int n_frames, int n_codebooks);
    bool generate(int n_utt, const int32_t *const *tokens, const int *n_tokens, const float *const *speaker,
                  const GenParams &gp, int32_t *codes, int *n_frames, FrameCb on_frames = nullptr,
                  void *user = nullptr, int interval = 40);
    // continuous batching: n_utt utterances (any number) through min(max_slots, n_utt) slots, at
    // most max_active of them at a time.  A slot whose utterance ended (EOS or max_len) is refilled with the next
    // queued utterance between two frames: its text rows are projected, its prefill rows assembled and replayed
    // token by token through a single-slot talker step on that slot's KV region while the other slots wait, and its
    // state (position, frame, EOS, repetition set, codes) is reset.  Sampling streams are keyed by the utterance's
    // index in the call (utt id), so an utterance's codes do not depend on its slot, its admission frame or the
    // other utterances in flight (the S-slot decode step never mixes tokens); on the matrix-core path (>= 4 slots) the
    // admission prefill runs the batch's kernels for its one slot, so the first wave's codes equal generate()'s.
    bool generate_queue(int n_utt, const int32_t *const *tokens, const int *n_tokens, const float *const *speaker,
                        const GenParams &gp, int32_t *codes, int *n_frames, int max_active);
    // fill this context's weight arenas (laid out with recv_weights) from another context's, device to device
    bool copy_weights_from(Engine &src);
    // after the weight arenas of a receiving context were filled by a broadcast: build what is derived from the weights
    // (the persistent code-predictor frame's per-token tables)
    bool finish_weights();

    // ---- stage entry points (host buffers) used by the parity tests
    bool talker_prefill(int n_utt, int n_rows, const float *embd, int family_slots, float *hidden, float *logits);
    bool talker_forward(int S, const float *embd, const int *pos, float *hidden, float *logits);
    bool codepred_frame(int S, const float *hidden, const int *cb0, float temperature, int top_k, uint64_t seed,
                        int frame, int32_t *codes15, float *logits_all);
    bool cb0_select_host(int S, const float *logits, const uint8_t *seen, const int *frame, const int *n_tokens,
                         const GenParams &gp, int *tokens);
    bool project_text(int n, const int32_t *toks, float *out);
    bool prefill_embd(const int32_t *toks, int n, const float *spk, int language_id, float *prefill, int *prefill_len,
                      float *trailing, int *trailing_len, float *tts_pad);

    // replay the captured talker-step (or code-predictor frame) graph `iters` times at position `pos` for S slots and
    // report the mean device time per replay (HIP events on the context stream)
    bool time_stage(int stage, int S, int pos, int iters, double *ms);

    // true if a persistent launch gave up waiting on a hand-off (never expected: a protocol fault)
    bool persist_fault_hook(int S, int n_launches);   // Q3T_PERSIST_FAULT_AT test hook (host side)
    unsigned persist_launches_ = 0;
    bool persist_error();
    bool persist_enabled() const { return persist_ || persist_cp_ || cpb_ || tkb_; }
    int persist_kernels() const {   // q3t_persist_kernels
        return (persist_ ? (tk_roles_ ? 1 : 2) : 0) | (persist_cp_ ? (cp_roles_ && cp_qkvtab_ ? 4 : 8) : 0) | (cpb_ ? 16 : 0) | (tkb_ ? 32 : 0);
    }
    // runs with S slots launch a persistent grid (the 1-slot kernels, or the batched code-predictor frame): they hold the
    // device lock exclusively (devlock.h)
    bool persist_exclusive(int S) const { return ((persist_ || persist_cp_) && S == 1) || ((cpb_ || tkb_) && S > 1); }
    bool persist_fell_back() const { return persist_fallback_; }
#ifdef Q3T_DEV
    // development hook: copy a device state buffer to the host (0 K cache, 1 V cache, 2 qkv, 3 attention output)
    bool debug_read(int which, void *dst, size_t bytes);
#endif

    // profiling hooks for bench.py: last generate() timings
    double last_prefill_ms = 0, last_frames_ms = 0;

private:
    bool upload_weights(const Gguf &g);
    bool parse_config(const Gguf &g);
    bool layout_weights(const Gguf &g);
    bool upload_weights_rest();
    bool alloc_state();
    bool setup_persist();
    // after a persistent launch flagged a fault: drain the stream, clear the hand-off state, drop the captured graphs
    // and continue on the launch-per-op graphs (the reference's permanent-fallback pattern, tts_transformer.cpp:2176-2182)
    bool persist_recover();
    struct StreamState {   // per utterance, kept across a fallback re-run so no chunk is delivered twice
        std::vector<int> delivered, stop_at;
    };
    bool generate_once(int n_utt, const int32_t *const *tokens, const int *n_tokens, const float *const *speaker,
                       const GenParams &gp, int32_t *codes, int *n_frames, FrameCb on_frames, void *user, int interval,
                       StreamState &st, bool *fault);
    bool generate_queue_once(int n_utt, const int32_t *const *tokens, const int *n_tokens, const float *const *speaker,
                             const GenParams &gp, int32_t *codes, int *n_frames, int max_active, bool *faulted);
    // host scratch kept across calls (a per-call hipFree / hipHostFree synchronises the whole device)
    struct PinnedChunk { size_t cap = 0; int32_t *codes = nullptr; hipEvent_t ev = nullptr; };
    std::vector<PinnedChunk> chunk_pool_;   // streaming chunks of generate()
    void *pin_ = nullptr, *qout_ = nullptr;
    size_t pin_cap_ = 0, qout_cap_ = 0;
    bool ensure_pinned(size_t bytes);
    bool ensure_qout(size_t bytes);
    bool enqueue_talker_step(int S, hipStream_t s);
    bool enqueue_talker(int S, hipStream_t s, bool gather_input, bool select_next, bool prenormed = false,
                        bool *fold_advance = nullptr);
    SelectSpec select_spec(int mode, const GenParams &gp, int frame_offset, int step) const;
    bool enqueue_cp_frame(int S, hipStream_t s, float *logits_host = nullptr, bool talker_next = false);
    bool enqueue_frame(int S, hipStream_t s);
    bool enqueue_text_projection(int n_rows, hipStream_t s);
    bool graph_for(std::map<int, hipGraphExec_t> &cache, int S, bool (Engine::*fn)(int, hipStream_t));
    bool graph_for_key(std::map<int, hipGraphExec_t> &cache, int key, int S, bool (Engine::*fn)(int, hipStream_t));
    int policy_slots_ = 0;         // > 0: the batched stacks choose kernels as for this many slots (queue graphs)
    bool set_slot_state(int S, const std::vector<int> &pos, const std::vector<int> &frame);
    // causal prefill (one pass over the prompt rows of n_utt utterances, K/V written into slots pf_slot_[u])
    bool ensure_prefill();
    bool enqueue_prefill_rows(int key, hipStream_t s);
    bool prefill(int n_utt, int plen, const float *src, int S_main, hipStream_t s);
    std::map<int, hipGraphExec_t> g_prefill_;
    float *pf_x_ = nullptr, *pf_qkv_ = nullptr, *pf_parts_ = nullptr, *pf_hid_ = nullptr, *pf_logits_ = nullptr;
    uint16_t *pf_xn_ = nullptr, *pf_attn_ = nullptr, *pf_hmlp_ = nullptr;
    int *pf_slot_ = nullptr, *slot_iota_ = nullptr;
    // continuous batching: admission batches on their own stream (their prefill on the prefill scratch), then
    // activation of each slot on the main stream between two frames
    bool alloc_admission();
    bool admit_batch(const std::vector<int> &tgt, const std::vector<int> &utt, const int32_t *const *tokens,
                     const int *n_tokens, const float *const *speaker, const GenParams &gp, int plen, hipStream_t as,
                     int *tgt_h, std::vector<int> &trailing_len);
    bool activate_slot(int slot, uint64_t utt, int trailing_len, int n_tok, const GenParams &gp, int plen, int *state_h);
    bool enqueue_text_projection(int n_rows, hipStream_t s, const int *idx, uint16_t *hbuf, float *out);
    hipStream_t astream_ = nullptr;
    float *aprefill_ = nullptr, *ahidden_ = nullptr, *alogits_ = nullptr, *aproj_out_ = nullptr;
    uint16_t *aproj_h_ = nullptr;
    int *aproj_idx_ = nullptr;
    RowRecipe *arecipe_ = nullptr;
    int aproj_cap_ = 0;
    int q_slots_ = 0;              // slot count of the running queue (the batch the admissions reproduce)

    Config c_;
    Config cpc_;                         // the code predictor's layer geometry (c_ with the cp_* values)
    bool mm_ok_ = true;                  // the batched matrix-core stack supports this model's shapes
    int fam1_ = 0;                       // !mm_ok_: every projection runs the vector kernels with a 1-slot K split
    bool use_mm(int S) const { return mm_ok_ && S >= gemm_mfma_min_batch(); }
    uint16_t *mtp_ = nullptr;            // code_pred.mtp_proj [cp_hidden][hidden] (1.7B)
    float *mtp_b_ = nullptr;             // its bias (optional)
    bool cp_project(int S, const float *x_talker, int ldx, hipStream_t s);   // cpx_ = mtp_proj . x + b
    std::string tts_path_, tok_path_;
    bool talker_ = true;   // false: vocoder-only context
    int device_ = 0, max_slots_ = 0, max_ctx_ = 0, max_trailing_ = 0;
    hipStream_t stream_ = nullptr;
    std::vector<void *> allocs_;
    WeightArena wa_;
    template <class T> T *dalloc(size_t n);

    // weights
    std::vector<DevLayer> L_, CP_;
    uint16_t *text_embd_ = nullptr, *fc1_ = nullptr, *fc2_ = nullptr, *codec_embd_ = nullptr, *codec_head_ = nullptr;
    float *fc1_b_ = nullptr, *fc2_b_ = nullptr, *out_norm_ = nullptr, *cp_out_norm_ = nullptr;
    std::vector<uint16_t *> cp_embd_, cp_head_;
    uint16_t **tabs16_dev_ = nullptr;   // codec_embd + code_pred.codec_embd[0..14]
    float *rope_ = nullptr;
    int rope_len_ = 0;

    // activations / state (sized for max_slots)
    float *x_ = nullptr, *qkv_ = nullptr, *logits_ = nullptr, *hidden_ = nullptr, *cpx_ = nullptr, *cp_in1_ = nullptr;
    float *cp_logits_ = nullptr, *part_ = nullptr;
    unsigned *ticket_ = nullptr;   // split-attention arrival counters [S][n_kv]
    unsigned *sel_ticket_ = nullptr;   // fused head+select arrival counters [S]
    uint16_t *attn_ = nullptr, *hmlp_ = nullptr;
    uint16_t *xn_ = nullptr;      // batched path: normalised f16 activations (resid_norm output)
    float *parts_ = nullptr;      // batched path: split-K partial slabs [4][S][H]
    uint16_t *kc_ = nullptr, *vc_ = nullptr, *cpkc_ = nullptr, *cpvc_ = nullptr;
    int *pos_ = nullptr, *frame_ = nullptr, *done_ = nullptr, *token_ = nullptr, *tokens_ = nullptr;
    int *n_tokens_ = nullptr, *force_ = nullptr, *trailing_len_ = nullptr, *cp_pos_ = nullptr;
    uint8_t *seen_ = nullptr;
    uint64_t *utt_ = nullptr;
    uint64_t *seed_dev_ = nullptr;   // the sampling seed read by the captured selections (SelectSpec::seed_dev)
    uint64_t seed_host_ = 0;
    bool set_seed(uint64_t seed, hipStream_t s);
    float *trailing_ = nullptr, *tts_pad_ = nullptr, *prefill_ = nullptr;
    int32_t *codes_ = nullptr;
    int codes_max_len_ = 0;
    // text projection scratch
    int *proj_idx_ = nullptr;
    uint16_t *proj_h_ = nullptr;
    float *proj_out_ = nullptr;
    int proj_cap_ = 0;
    RowRecipe *recipe_ = nullptr;
    int recipe_cap_ = 0;
    GenParams gp_;   // parameters baked into the captured frame graph
    Options opt_;
    int poll_every_ = 16;
    bool fused_select_ = true;
    bool cp_fused_attn_ = true;
    bool defer_cp_select_ = true;
    bool persist_ = true;
    bool persist_fallback_ = false;   // persistent kernels disabled after a flagged fault
    PLayerW *pl_dev_ = nullptr, *pl_cp_dev_ = nullptr;
    const uint16_t **heads_dev_ = nullptr;
    float *cp_qkvtab_ = nullptr;         // persistent code-predictor frame: layer 0's QKV row per table token
    float *cp_projtab_ = nullptr;        // 1.7B: mtp_proj . f16(table row) + b per table token (f32, code-predictor space)
    std::shared_ptr<struct CpTables> cp_tables_;   // the two tables above, shared by every context of this device
                                                   // that loaded the same weight file (engine.cpp, table registry)
    bool build_cp_proj_table();
    bool build_cp_qkv_table();
    bool build_persist_tables();
    bool tables_built_ = false;
    bool persist_cp_ = false;
    bool cp_roles_ = false;    // the 1-slot code-predictor frame runs persist_cp.hip
    bool tk_roles_ = false;    // the 1-slot talker step runs persist_tk.hip
    bool cpb_ = false;         // the batched code-predictor frame runs persist_cpb.hip (use_cpb)
    uint8_t *cpb_state_ = nullptr;
    bool setup_cpb();
    bool use_cpb(int S) const;
    bool tkb_ = false;         // the batched talker step runs persist_tkb.hip (use_tkb)
    uint8_t *tkb_state_ = nullptr;
    bool setup_tkb();
    bool use_tkb(int S) const;
    uint8_t *pstate_ = nullptr;
    int *table_iota_ = nullptr;   // 0..codec_vocab-1: the table builds' token ids
    uint64_t *pprof_ = nullptr;   // Q3T_DEV + Q3T_PERSIST_PROF: persistent-step timeline

    bool enqueue_cp_only(int S, hipStream_t s) { return enqueue_cp_frame(S, s); }
    std::map<int, hipGraphExec_t> g_talker_, g_frame_, g_cp_;
    std::unique_ptr<Vocoder> voc_;
    std::unique_ptr<SpeakerEncoder> spk_;
};

}  // namespace q3t
