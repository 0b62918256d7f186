// kernels.h — launchers of the hand-written gfx950 kernels (kernels.hip).
#pragma once
#include "q3t_common.h"

namespace q3t {

// PRO_RMS_G1 / PRO_RMS_G16: RMSNorm over a GatherSum source (1 table row / 16 table rows + trailing-or-pad row)
// PRO_CPATT: the code predictor's whole attention (head RMSNorm + RoPE + KV append + softmax(QK^T)V over <= 16
// positions) computed in the O-projection's prologue from the raw QKV rows (GemvParams::att)
// PRO_SEL_G1: PRO_RMS_G1 whose token is first SELECTED by every workgroup from the previous head's logits
// (sel_logits, SelectSpec sel; workgroup x = 0 records it): the code predictor's selection moved off the head's
// last-arriver chain into the next pass's weight-streaming window
enum Prologue { PRO_F16 = 0, PRO_F32 = 1, PRO_RMS = 2, PRO_LN = 3, PRO_RMS_G1 = 4, PRO_RMS_G16 = 5, PRO_CPATT = 6,
                PRO_SEL_G1 = 7 };
enum Act { ACT_NONE = 0, ACT_SILU = 1, ACT_GELU = 2, ACT_SWIGLU = 3 };

// Token selection (select.h): SEL_CB0 = CB0 logit processing + selection (src/tts_transformer.cpp:2416-2499),
// SEL_CP = code-predictor token of pass step+1 (trt_code_predictor.cpp:552-592 / k_sample_topk_f32 semantics).
// Used by the standalone select launch (one 256-thread workgroup per slot) and fused into the head GEMV, where
// the last head workgroup to finish (arrival ticket) selects in the same launch.
enum SelMode { SEL_NONE = 0, SEL_CP = 1, SEL_CB0 = 2 };
struct SelectSpec {
    int mode = SEL_NONE;
    int V = 0;
    unsigned *ticket = nullptr;     // fused: [gridDim.y] arrival counters (zero between launches)
    int *tokens = nullptr;          // [S][16] frame codes (CB0: col 0; CP: col step+1)
    int32_t *codes = nullptr;       // [S][max_len][ncb]
    int max_len = 0, ncb = 16;
    const int *frame = nullptr;     // [S]
    int frame_offset = 0;           // selected token belongs to frame[s] + frame_offset
    int *done = nullptr;            // [S] frame of EOS, else -1 (slots with done >= 0 are skipped)
    float temperature = 0.f;
    int top_k = 50;
    uint64_t seed = 0;
    const uint64_t *seed_dev = nullptr;   // if set, the seed is read here (one device word: a captured graph serves
                                          // every seed; the host writes it before the frame loop)
    const uint64_t *utt = nullptr;  // [S]
    int step = 0;                   // SEL_CP: 0..14
    // SEL_CB0
    uint8_t *seen = nullptr;        // [S][V]
    const int *n_tokens = nullptr;  // [S]
    const int *force_frames = nullptr;  // [S] (bench: EOS masked while frame < force)
    int eos = 2150;
    float rep = 1.05f;
};
// standalone: logits [S][V] -> one workgroup per slot
bool select_tokens(const SelectSpec &sp, const float *logits, int S, hipStream_t s);

// f32 activation row assembled on the fly by the gather prologues:
//   PRO_RMS_G1:  x[b] = tab0[tok[b * tok_ld + tok_col0]]                       (code-predictor pass input,
//                trt_code_predictor.cpp:552-592)
//   PRO_RMS_G16: x[b] = tabs[0][tok[b][0]] + ... + tabs[15][tok[b][15]] + (frame[b] < tr_len[b] ? tr[b][frame[b]]
//                : pad[b])  (the talker step embedding, tts_transformer.cpp:2529-2553; tok_ld must be 16)
// f16 table rows converted and summed left to right in f32.
struct GatherSum {
    const int *tok = nullptr;
    int tok_ld = 16, tok_col0 = 0;
    const uint16_t *tab0 = nullptr;        // G1: the table
    const uint16_t *const *tabs = nullptr; // G16: device array of 16 tables [V][K]
    const float *tr = nullptr;             // optional f32 term: [B][tr_ld] rows of K, indexed by frame
    const int *tr_len = nullptr, *frame = nullptr;
    int tr_ld = 0;
    const float *pad = nullptr;            // [B][K]
};

// the GatherSum rows as a plain f32 buffer out[b][0..K) (nt = 1 or 16 table rows; batched path)
bool gather_sum(const GatherSum &gs, int nt, int S, int K, float *out, int ldo, hipStream_t s);

// PRO_CPATT source: one new token per slot at position pos[b] (< 16) over a 16-position F16 cache
// (scripts/export_code_predictor.py:132-231 step semantics; 16 q heads / 8 kv heads / D 128 only)
struct CpAttnSrc {
    const float *qkv = nullptr;           // [B][ld] raw Q | K | V rows of the QKV GEMV
    int ld = 0;
    const float *qn = nullptr, *kn = nullptr;  // head-norm weights [128]
    float eps = 1e-6f;
    const float *rope = nullptr;          // [pos][128] (cos, sin) pairs
    const int *pos = nullptr;             // [B]
    uint16_t *kc = nullptr, *vc = nullptr;  // this layer's cache [B][8][16][128] f16
};

// y[b][n] = epilogue( W[n][:] . f16(prologue(x[b][:])) ),  W f16 row-major [N][K]
struct GemvParams {
    const uint16_t *W = nullptr;
    int N = 0, K = 0, B = 0;
    int pro = PRO_F16;
    const void *x = nullptr;      // f16 [B][ldx] (PRO_F16) or f32 [B][ldx]
    int ldx = 0;
    const int *x_idx = nullptr;   // optional row gather: row of batch b = x_idx[b]
    const float *nw = nullptr, *nb = nullptr;  // norm weight / bias (RMS, LN)
    float eps = 1e-6f;
    GatherSum gs;                 // PRO_RMS_G1 / PRO_RMS_G16 source
    CpAttnSrc att;                // PRO_CPATT source
    SelectSpec sel;               // PRO_RMS heads: select in the last workgroup (logits -> out_f32); PRO_SEL_G1 source
    const float *sel_logits = nullptr;  // PRO_SEL_G1: [B][sel.V] logits of the previous head
    float *side_out = nullptr;    // normalized prologue rows (f32 [B][K]) written by x-block 0
    float *raw_out = nullptr;     // raw (pre-norm) f32 prologue rows [B][K] written by x-block 0
    int act = ACT_NONE;           // ACT_SWIGLU: rows interleaved in 16-row blocks [gate16 | up16]
    const float *bias = nullptr, *scale = nullptr;
    const float *resid = nullptr;  // out = resid[b][n] + (...)
    int ldr = 0;
    const float *aux = nullptr;    // out = aux[b][n] + (...)   (applied after resid)
    int lda = 0;
    float *out_f32 = nullptr;
    uint16_t *out_f16 = nullptr;
    int ldo = 0;
    int orow_mul = 1, orow_add = 0;  // output row of batch b = b*orow_mul + orow_add
    int dbg = 0;                     // microbenchmark knobs (tools/dev/kbench_mm): 1 = no activation loads, 2 = no weight loads
    // split-K partial slabs (matrix-core path, PRO_F16): grid z = ksplit K slices, slice z writes its raw partial sums
    // to parts[z][b][n] (no epilogue); resid_norm() folds them into the residual stream
    float *parts = nullptr;
    int ksplit = 1;
    bool xcd_slices = false;   // split-K tiles in XCD-aware order (gemm_mfma.hip splitk_tile)
    int mm_tt = 0;              // MFMA token tile in 32-token units for this call (0: the library default)
    // matrix-core f16 path, one token-tile row, no split-K: extra workgroups past the row tiles touch one dword per
    // 128-B line of these bytes (the NEXT projection's weights) so they are in the Infinity Cache when it runs
    const void *prefetch = nullptr;
    size_t prefetch_bytes = 0;
    bool force_mm = false;   // matrix-core path even below gemm_mfma_min_batch() (a single slot reproducing the
                             // per-token arithmetic of a batch that runs there)
    int family_b = 0;        // > 0: kernel family (vector / matrix core) and K split chosen as for a batch of
                             // family_b rows -- the per-row arithmetic of that batch, for any B (the causal prefill)
};
bool gemv(const GemvParams &p, hipStream_t s);   // routes wide batches to gemm_mfma (gemm_mfma.hip)
// matrix-core path for B >= gemm_mfma_min_batch() tokens (Q3T_MFMA_MIN_B, default 4; 0 = off): F16 / F32 / RMS / LN
// prologues, K in {256, 512, 1024, 2048, 3072} (norm prologues K <= 1024), N % 32 == 0, no fused selection
bool gemm_mfma_supported(const GemvParams &p);
bool gemm_mfma(const GemvParams &p, hipStream_t s);
int gemm_mfma_min_batch();
void gemm_mfma_set_min_batch(int b);
void gemv_set_min_blocks(int n);   // tuning hook (tools/dev/kbench)

// Qwen3 attention for one new token per slot (talker decode / unfused code-predictor pass), fused with q/k head
// RMSNorm, NEOX RoPE (host cos/sin table), F16 KV append at pos[slot] and split-K flash-decode over ATTN_CHUNK-position
// chunks; the last split to finish (agent-scope ticket) combines the partials in the same launch (attn.hip).
struct AttnParams {
    const float *qkv = nullptr;   // [S][(nH + 2 nKV) * D] f32
    const float *qn = nullptr, *kn = nullptr;  // head-norm weights [D]
    float eps = 1e-6f;
    const float *rope = nullptr;  // [max_pos][D] (cos, sin pairs)
    const int *pos = nullptr;     // [S] position of the new token
    uint16_t *kc = nullptr, *vc = nullptr;  // cache base of this layer: [S][nKV][n_ctx][D] f16
    int n_ctx = 0, S = 0, nH = 0, nKV = 0, D = 0;
    int chunk = 64;               // positions per split workgroup: 64 or 128 (batched decode: fewer, fuller splits)
    int seqk = 0;                 // 1: one workgroup per (slot, kv head) streams the whole context (k_attn_seq; many slots)
    int small = 0;                // 1: batched code predictor (n_ctx <= 16): one wave per (slot, kv head) (k_attn_small)
    int max_splits = 1;           // grid z = ceil(n_ctx / chunk)
    float *part = nullptr;        // [S][nKV][max_splits][R][D + 2] split partials (m, l, acc)
    unsigned *ticket = nullptr;   // [S][nKV] arrival counters, zero between launches
    uint16_t *out = nullptr;      // [S][nH*D] f16 (rounded attention output, the O-proj input)
    float *dbg = nullptr;         // development dump (slot 0, kv group 5, split 0)
    // k_attn_small only: slot s's raw QKV row is the per-token table row qkv_tab[tab_row0 + tab_tok[s * tab_ld +
    // tab_col]] (the code predictor's layer 0 of passes 1..15, Engine::build_cp_qkv_table) instead of qkv[s]
    const float *qkv_tab = nullptr;
    const int *tab_tok = nullptr;
    int tab_ld = 0, tab_col = 0;
    size_t tab_row0 = 0;
};
bool attn_decode(const AttnParams &p, hipStream_t s);
constexpr int ATTN_CHUNK = 64;

// Causal attention over the prompt rows of n_utt utterances in one launch (the real prefill,
// src/tts_transformer.cpp:1233-1374): row i of utterance u is token u*plen + i at position i of slot slot[u]; q / k
// head RMSNorm + NEOX RoPE at i, F16 K/V rows written to the slot's cache rows [0, plen), softmax(QK^T / sqrt(D)) V over
// positions 0..i.  One workgroup per (utterance, kv head).
constexpr int PREFILL_MAX_ROWS = 16;
struct PrefillAttnParams {
    const float *qkv = nullptr;   // [n_utt * plen][(nH + 2 nKV) * D] f32 raw QKV rows
    const float *qn = nullptr, *kn = nullptr;
    float eps = 1e-6f;
    const float *rope = nullptr;  // [pos][D] (cos, sin) pairs
    uint16_t *kc = nullptr, *vc = nullptr;   // this layer's cache base [slot][nKV][n_ctx][D] f16
    const int *slot = nullptr;    // [n_utt] cache slot of each utterance
    int n_ctx = 0, n_utt = 0, plen = 0, nH = 0, nKV = 0, D = 0;
    uint16_t *out = nullptr;      // [n_utt * plen][nH * D] f16 (the O-projection input)
};
bool prefill_attn(const PrefillAttnParams &p, hipStream_t s);
constexpr int ATTN_MAX_SPLITS = 160;   // n_ctx <= 10240



// pos[s]++, frame[s]++
bool advance(int *pos, int *frame, const int *done, int S, hipStream_t s);   // done: slots with done >= 0 stay (may be null)

// *out = t[0] + t[1] + t[2] (f32 rows or f16 table rows; null terms skipped); recipe built on the host
struct RowTerm { const void *ptr; int is_f16; };
struct RowRecipe { float *out; RowTerm t[3]; };
bool rows_recipe(const RowRecipe *recipe_dev, int n_rows, int H, hipStream_t s);
// batched residual + RMSNorm between the matrix-core projections (one workgroup per token, H <= 1024):
//   x[b] = xin[b] + parts[0][b] + ... + parts[ksplit-1][b]   (written to x when parts or xin != x)
//   xn[b] = f16((x[b] * rsqrt(mean(x[b]^2) + eps)) * nw)       (double sums, as the GEMV prologues)
//   side[b] = the same normalised row in f32 (optional: hidden_states side output)
struct ResidNorm {
    const float *xin = nullptr;
    float *x = nullptr;
    const float *parts = nullptr;
    int ksplit = 0;
    const float *nw = nullptr;
    float eps = 1e-6f;
    uint16_t *xn = nullptr;
    float *side = nullptr;
    int S = 0, H = 0;
    // optional: extra workgroups touch one dword of every 128-B line of the NEXT projection's weights (up to 256 MB)
    // while the token rows normalise, so the lines are in the Infinity Cache when that GEMM streams them
    const void *prefetch = nullptr;
    size_t prefetch_bytes = 0;
};
bool resid_norm(const ResidNorm &r, hipStream_t s);

// batched: the selection launch also prepares the NEXT stage's input (one workgroup per slot): the token selected
// for slot b, then x[b] = the GatherSum row (nt = 1: the next code-predictor pass; nt = 16: the talker step
// embedding, the selected token among its 16), then xn[b] = f16(RMSNorm(x[b]) * nw) -- k_gather_sum + k_resid_norm
// arithmetic, so the fused and the three-launch forms give the same bits
struct EmbedNorm {
    GatherSum gs;
    int nt = 0;
    float *x = nullptr;
    uint16_t *xn = nullptr;
    const float *nw = nullptr;
    float eps = 1e-6f;
    int H = 0;
};
bool select_embed_norm(const SelectSpec &sp, const float *logits, const EmbedNorm &en, int S, hipStream_t s);

// src/trt_cuda_kernels.cu drop-ins (C ABI wrappers in capi.cpp)
void launch_f32_to_f16(const float *in, uint16_t *out, int n, hipStream_t s);
void launch_argmax_f32(const float *in, int32_t *out, int n, hipStream_t s);
void launch_embed_lookup(const int32_t *tok, const float *table, float *out, int dim, hipStream_t s);
void launch_sample_topk_f32(const float *logits, const float *rand_val, int32_t *out, float temperature, int top_k, int n,
                            hipStream_t s);

}  // namespace q3t
