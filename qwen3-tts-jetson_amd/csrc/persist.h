// persist.h — the persistent talker decode step (persist.hip): the whole 28-layer Talker step plus the codec head and
// the fused CB0 selection of ONE slot as a single launch of one workgroup per CU, replacing the 141-launch graph of
// enqueue_talker at batch 1 (src/tts_transformer.cpp:1376-1512 build_step_graph + :2416-2499 CB0 processing).
//
// Inside the launch, every dependency edge (x -> QKV -> attention -> O -> x' -> gate/up -> h -> down -> x) is a
// vector of data-tagged granules: {32-bit payload, 32-bit tag} written by ONE 8-byte agent-scope (sc1) store and
// polled by the consumers with sc1 loads until every tag matches (MI355X_MICROARCH.md, handoff-1to1 / allgather rows;
// no flags, no fences, no grid barrier).  Tags are ((seq * 1024 + phase) << 1) | 1 with `seq` a device word bumped
// by the last workgroup of every launch, so a granule of an earlier launch or layer can never match.  Weights and
// K/V rows do not depend on the edge: each phase's weight loads are issued as soon as the previous phase's input has
// arrived, so they stream while the chain waits.
#pragma once
#include "kernels.h"

namespace q3t {

constexpr int PROF_PH = 448;   // timeline phases recorded per workgroup (5 per layer + head)
constexpr int PROF_WG = 512;   // timeline rows (workgroups; persist_tk.hip runs up to 505)

struct PLayerW {
    const uint16_t *qkv, *o, *gu, *down;
    const float *attn_norm, *ffn_norm, *qn, *kn;
};

struct PersistParams {
    const PLayerW *L = nullptr;   // device array [n_layers]
    int n_layers = 0;
    float eps = 1e-6f;
    // layer-0 input: x_in (f32 [1024], written before the launch) or the step-embedding gather (GatherSum, NT = 16)
    int gather = 0;
    const float *x_in = nullptr;
    GatherSum gs;
    // attention (talker KV layout [layer][slot][kv][n_ctx][128], slot 0)
    const float *rope = nullptr;
    const int *pos = nullptr;
    uint16_t *kc = nullptr, *vc = nullptr;
    size_t kv_layer = 0;
    int n_ctx = 0;
    float *part = nullptr;        // [8][32][2][130] split partials
    unsigned *ticket = nullptr;   // [8] split arrival counters (zero between layers)
    // head: hidden = rms(x) * out_norm (f32, side output), logits = head . f16(hidden) (f32 [V], sc1 stores)
    const uint16_t *head = nullptr;
    const float *out_norm = nullptr;
    float *hidden = nullptr, *logits = nullptr;
    SelectSpec sel;               // SEL_CB0 of the next frame, or SEL_NONE
    // hand-off state (persist_alloc)
    uint64_t *gx = nullptr, *gx2 = nullptr, *gqkv = nullptr, *gattn = nullptr, *gh = nullptr;
    uint64_t *gpart = nullptr;     // [8][32][264] attention split partials (granules)
    uint64_t *gop = nullptr;       // [4][1024] O-projection K-slice partial rows (granules, persist_tk.hip)
    uint64_t *gtok = nullptr;      // [16] code-predictor tokens of the launch (granules)
    uint64_t *glog = nullptr;      // [3072] head logits (granules): the selecting workgroup gathers them
    const uint16_t *const *heads = nullptr;   // code-predictor frame: device array of the 15 lm_heads
    // code-predictor frame (optional): layer 0's raw QKV row of every table token, f32 [3072 + 14 * 2048][4096] (pass 1:
    // codec_embd rows, pass p >= 2: code_pred.codec_embd[p-2] rows), computed with the per-op QKV GEMV's arithmetic
    // (persist_qkv_table_rows): passes 1..15 then skip layer 0's norm + QKV phase and its edge
    const float *qkvtab = nullptr;
    // code-predictor frame (1.7B): the pass inputs of passes 1..15 as projected f32 rows [3072 + 14 * 2048][1024] in
    // place of the f16 table rows (gs.tabs), same row order as qkvtab; x_in is then the projected pass-0 input
    const float *xtab = nullptr;
    // frame graph (k_tk_roles only): after its commit the selecting workgroup advances slot 0 exactly as k_advance
    // would (pos + 1, frame + 1 unless done), so the frame needs no k_advance launch.  Null: no advance (stage replays,
    // talker_forward)
    int *adv_pos = nullptr, *adv_frame = nullptr;
    const int *adv_done = nullptr;
    uint64_t *prof = nullptr;      // development timeline [256][PROF_PH][4] (null = off)
    int roles_split = 0;           // persist_tk.hip: attention splits per kv group (set by the launcher)
    unsigned *seq = nullptr, *head_ticket = nullptr, *err = nullptr;
};

// shapes the persistent step supports: H 1024, 16 q / 8 kv heads of 128, I 3072, V 3072, one workgroup per CU on a
// 256-CU device, n_ctx <= 32 * 256 (split chunk of 64..256 positions)
bool persist_supported(int hidden, int n_heads, int n_kv, int head_dim, int inter, int vocab, int n_ctx, int n_cu);
// residency check: every k_persist instantiation the context may launch fits one workgroup per CU on `device`
// (hipOccupancyMaxActiveBlocksPerMultiprocessor with the kernel's LDS request) and the device has >= 256 CUs, so the
// 256-workgroup grid is co-resident when nothing else occupies the device (MI355X_MICROARCH.md, Residency)
bool persist_resident(int device, int n_ctx, bool cp_frame);
bool persist_resident_cp(int device);   // the code-predictor frame alone (a talker the step kernel does not cover)
size_t persist_state_bytes();                    // granule buffers + counters (zeroed once at allocation)
void persist_carve(uint8_t *base, PersistParams &p);   // point the hand-off buffers into a zeroed state block
bool persist_talker_step(const PersistParams &p, hipStream_t s);
// the 16-pass code-predictor frame of one slot as one launch (same hand-off protocol): p.L = the 5 code-predictor
// layers, x_in = the talker hidden state, gs.tok = the frame's codes (CB0 in column 0), gs.tabs = the 16 embedding
// tables, kc/vc = the 16-position code-predictor caches, heads = lm_head[0..14], out_norm, logits [2048],
// sel = SEL_CP (step set per pass)
bool persist_cp_frame(const PersistParams &p, hipStream_t s);
// the same frame with role-specialised workgroups (persist_cp.hip): 0.6B shapes with the layer-0 QKV table
// (p.qkvtab) and 5 code-predictor layers; bit-identical to persist_cp_frame and the launch-per-op graph
bool persist_cp_roles(const PersistParams &p, hipStream_t s);
bool persist_cp_roles_resident(int device);
// the talker step with role-specialised workgroups (persist_tk.hip): the 0.6B shapes, contexts up to 64 x 4 x 3
// positions; bit-identical to persist_talker_step and the launch-per-op graph
bool persist_tk_roles(const PersistParams &p, hipStream_t s);
bool persist_tk_roles_supported(int n_ctx);
bool persist_tk_roles_resident(int device, int n_ctx);
int persist_chunk(int n_ctx);                    // positions per attention split workgroup
size_t persist_qkv_table_rows();                 // rows of PersistParams::qkvtab (3072 + 14 * 2048)

// ------------------------------------------------------------------ the batched code-predictor frame (persist_cpb.hip)
// 1..64 slots, 0.6B code-predictor shapes, the launch-per-op matrix-core family of up to 64 slots (split-K 4): the whole
// 16-pass frame of every slot as one persistent launch, bit-identical to enqueue_cp_frame's decoder_stack_mm graph
struct CpbParams {
    const PLayerW *L = nullptr;                  // device array [5]
    const uint16_t *const *heads = nullptr;      // device array of the 15 lm_heads
    const uint16_t *const *tabs = nullptr;       // device array [16]: codec_embd, code_pred.codec_embd[0..14]
    const float *out_norm = nullptr;             // code-predictor output norm
    const float *qkvtab = nullptr;               // layer 0's raw QKV row per table token (Engine::build_cp_qkv_table)
    const float *x_in = nullptr;                 // [S][1024] talker hidden state (pass 0 input)
    const float *rope = nullptr;
    const int *pos = nullptr;                    // [16][pos_ld] position of pass p per slot
    int pos_ld = 0;
    uint16_t *kc = nullptr, *vc = nullptr;       // [5][pos_ld][8][16][128] f16
    size_t kv_layer = 0;
    float *logits = nullptr;                     // [S][2048]
    SelectSpec sel;                              // SEL_CP (step set per pass), sel.tokens = the frame codes [S][16]
    int S = 0;
    float eps = 1e-6f;
    // talker_next: after the last pass, the next talker step's embedding (16 table rows + trailing / pad row) into tx and
    // its layer-0 RMSNorm (tnw) into txn (k_select_embed_norm nt = 16)
    int talker_next = 0;
    float *tx = nullptr;
    uint16_t *txn = nullptr;
    const float *tnw = nullptr;
    const float *tr = nullptr, *pad = nullptr;
    const int *tr_len = nullptr, *frame = nullptr;
    int tr_ld = 0;
    uint8_t *state = nullptr;                    // cpb_state_bytes(), zeroed once
    uint64_t *prof = nullptr;                    // development timeline [256][768][4] (null = off)
};
size_t cpb_state_bytes();
bool cpb_resident(int device);                   // both instantiations fit one workgroup per CU, >= 256 CUs
bool persist_cp_batched(const CpbParams &p, hipStream_t s);
bool cpb_error(const uint8_t *state, hipStream_t s, bool *err);   // a hand-off wait gave up
bool cpb_clear(uint8_t *state, hipStream_t s);   // zero the flags and the error word

// ------------------------------------------------------------------ the batched talker step (persist_tkb.hip)
// 2..64 slots, 0.6B talker shapes (28 layers), the launch-per-op matrix-core family of >= 16 policy slots (split-K 4,
// k_attn_seq): the whole step of every slot -- 28 layers, final norm, codec head, CB0 selection -- as one persistent
// launch, bit-identical to enqueue_talker's decoder_stack_mm + head GEMM + select_tokens
struct TkbParams {
    const PLayerW *L = nullptr;                  // device array [28]
    int n_layers = 0;
    const uint16_t *head = nullptr;              // codec head [3072][1024]
    const float *out_norm = nullptr;
    const float *x_in = nullptr;                 // [S][1024] the step's input rows (the residual stream's start)
    float *hidden = nullptr;                     // [S][1024] side output: the final-normalised hidden state (f32)
    float *logits = nullptr;                     // [S][3072] (optional) the head's logits
    const float *rope = nullptr;
    const int *pos = nullptr;                    // [S]
    uint16_t *kc = nullptr, *vc = nullptr;       // [28][slot][8][n_ctx][128] f16
    size_t kv_layer = 0;
    int n_ctx = 0;
    int select = 0;                              // 1: CB0 of the next frame (sel: SEL_CB0, frame_offset 1)
    SelectSpec sel;
    int S = 0;
    float eps = 1e-6f;
    uint8_t *state = nullptr;                    // tkb_state_bytes(), zeroed once
    uint64_t *prof = nullptr;                    // development timeline [256][768][4] (null = off)
};
size_t tkb_state_bytes();
bool tkb_resident(int device);                   // both instantiations fit one workgroup per CU, >= 256 CUs
bool persist_talker_batched(const TkbParams &p, hipStream_t s);
bool tkb_error(const uint8_t *state, hipStream_t s, bool *err);   // a hand-off wait gave up
bool tkb_clear(uint8_t *state, hipStream_t s);   // zero the flags and the error word

}  // namespace q3t
