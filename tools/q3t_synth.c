// q3t_synth — writes synthetic Qwen3-TTS GGUF files (talker+code-predictor and tokenizer decoder)
// with the exact tensor names / shapes / dtypes the reference converters emit
// (scripts/convert_tts_to_gguf.py:42-125,289-297; scripts/convert_tokenizer_to_gguf.py:42-163,265-296).
//
// This is TEST/BENCH DATA tooling, not product code. No checkpoint exists in this environment
// (SURVEY.md §8(d)), so every weight is generated from a portable counter-based hash:
//   h   = mix(mix(seed ^ fnv1a64(name)) + index)         (mix = splitmix64 finaliser)
//   s   = sum of four 10-bit fields of h  - 2046           (integer in [-2046, 2046], ~normal)
//   val = center + s * 2^-e                                 (e chosen so std ~= the target sigma)
// Every value has <= 11 significant bits, so it is EXACT in f16 and f32: the GGUF bytes are identical
// no matter which language regenerates them.
//
// usage: q3t_synth <config: full|tiny> <out_dir> [seed] [usage]
//   writes <out_dir>/qwen3-tts-0.6b-f16.gguf and <out_dir>/qwen3-tts-tokenizer-f16.gguf
//   (the fixed file names the reference loads, src/qwen3_tts.cpp:117-118).
//   "q8_0" / "q4_0" / "q4_k" / "f32": weight dtype policy of the converters' --outtype (convert_tts_to_gguf.py:250-335,
//   convert_tokenizer_to_gguf.py:265-296; the tokenizer converter knows f32 / f16 / q8_0 only, so q4_* leave that
//   file F16).  Q8_0 / Q4_0 blocks use ggml's reference quantisers; Q4_K uses a plain min/max fit per 32-value
//   sub-block (not ggml's iterative make_qkx2_quants: any valid block decodes the same way, which is what the
//   loaders are tested on).
//   "usage": the tokenizer file also carries tok_dec.vq_{first.0,rest.N}.usage [cb_size] F32 tensors, as an
//   unconverted checkpoint would (the converter divides and drops them, convert_tokenizer_to_gguf.py:347-359);
//   loaders must apply normalize_codebooks (src/audio_tokenizer_decoder.cpp:40-73).
#define _GNU_SOURCE
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>

#define GGML_F32 0
#define GGML_F16 1
#define GGML_Q4_0 2
#define GGML_Q8_0 8
#define GGML_Q4_K 12
enum { GV_U32 = 4, GV_F32 = 6, GV_STR = 8, GV_ARR = 9 };

static uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static uint64_t fnv1a64(const char *s) {
    uint64_t h = 0xcbf29ce484222325ull;
    for (; *s; ++s) { h ^= (uint8_t)*s; h *= 0x100000001b3ull; }
    return h;
}

typedef struct {
    const char *name;
    int text_vocab, text_dim, hidden, n_layers, n_heads, n_kv, head_dim, inter, codec_vocab, n_codebooks;
    int cp_layers, cp_vocab;
    float eps, rope_theta;
    int tts_bos, tts_eos, tts_pad;
    int cb_size, cb_dim, voc_hidden, voc_latent, voc_layers, voc_heads, voc_ffn, dec_dim;
    int up_ratio, convnext_mult;
    int rates[4];
    // code predictor geometry when it differs from the talker's (1.7B: 0 = the talker's values); cp_hidden != hidden
    // adds code_pred.mtp_proj.{weight,bias} (tts_transformer.cpp:370-389, 611-616)
    int cp_hidden, cp_inter, cp_heads, cp_kv;
} cfg_t;

static const cfg_t CFG_FULL = {
    "full", 151936, 2048, 1024, 28, 16, 8, 128, 3072, 3072, 16,
    5, 2048, 1e-6f, 1000000.0f, 151672, 151673, 151671,
    2048, 256, 512, 1024, 8, 16, 1024, 1536, 2, 4, {8, 5, 4, 3}};
// the full model's widths with its first 5 talker layers only: the generator is counter-based per tensor name, so
// these are exactly the full model's first 5 layers, which tests/golden/talker5_full.npz pins (5 harness layer slots)
static const cfg_t CFG_FULL5 = {
    "full5", 151936, 2048, 1024, 5, 16, 8, 128, 3072, 3072, 16,
    5, 2048, 1e-6f, 1000000.0f, 151672, 151673, 151671,
    2048, 256, 512, 1024, 8, 16, 1024, 1536, 2, 4, {8, 5, 4, 3}};
static const cfg_t CFG_TINY1 = {
    "tiny1", 1024, 128, 256, 1, 4, 2, 64, 512, 3072, 16,
    1, 2048, 1e-6f, 1000000.0f, 1001, 1002, 1000,
    2048, 32, 64, 128, 2, 2, 128, 96, 2, 4, {8, 5, 4, 3}};
// 1.7B-shaped: talker hidden 2048 / FFN 6144, code predictor 1024 / 3072 behind code_pred.mtp_proj
static const cfg_t CFG_FULL17 = {
    "full17", 151936, 2048, 2048, 28, 16, 8, 128, 6144, 3072, 16,
    5, 2048, 1e-6f, 1000000.0f, 151672, 151673, 151671,
    2048, 256, 512, 1024, 8, 16, 1024, 1536, 2, 4, {8, 5, 4, 3}, 1024, 3072, 16, 8};
// the same relation at test size: talker 512 wide, code predictor 256 wide (different head counts too)
static const cfg_t CFG_TINY17 = {
    "tiny17", 1024, 128, 512, 3, 8, 2, 64, 1024, 3072, 16,
    3, 2048, 1e-6f, 1000000.0f, 1001, 1002, 1000,
    2048, 32, 64, 128, 2, 2, 128, 96, 2, 4, {8, 5, 4, 3}, 256, 512, 4, 2};
static const cfg_t CFG_TINY = {
    "tiny", 1024, 128, 256, 5, 4, 2, 64, 512, 3072, 16,
    5, 2048, 1e-6f, 1000000.0f, 1001, 1002, 1000,
    2048, 32, 64, 128, 2, 2, 128, 96, 2, 4, {8, 5, 4, 3}};

// ---------------------------------------------------------------- tensor catalogue
typedef struct {
    char name[96];
    int ndims;
    int64_t ne[4];
    int type;
    float center;
    int e;  // value = center + s * 2^-e
    uint64_t off;
} tens_t;

static tens_t *g_t = NULL;
static int g_nt = 0, g_cap = 0;

static int exp_for_sigma(double sigma) {
    // std of s (sum of 4 uniform 10-bit ints) = sqrt(4 * (1024^2-1)/12) = 591.3
    int e = (int)lround(log2(591.3 / sigma));
    if (e < 0) e = 0;
    if (e > 24) e = 24;
    return e;
}

static void add_t(const char *name, int ndims, int64_t n0, int64_t n1, int64_t n2, double center, double sigma) {
    if (g_nt == g_cap) { g_cap = g_cap ? g_cap * 2 : 256; g_t = realloc(g_t, sizeof(tens_t) * g_cap); }
    tens_t *t = &g_t[g_nt++];
    memset(t, 0, sizeof(*t));
    snprintf(t->name, sizeof(t->name), "%s", name);
    t->ndims = ndims;
    t->ne[0] = n0; t->ne[1] = n1; t->ne[2] = n2; t->ne[3] = 1;
    // dtype policy of the converters: 1-D -> F32, >=2-D -> F16
    t->type = ndims <= 1 ? GGML_F32 : GGML_F16;
    t->center = (float)center;
    t->e = exp_for_sigma(sigma);
}
static void add1(const char *n, int64_t a, double c, double s) { add_t(n, 1, a, 1, 1, c, s); }
// 2-D linear weight PyTorch [out, in] -> ggml ne [in, out]
static void addw(const char *n, int64_t out, int64_t in, double gain) { add_t(n, 2, in, out, 1, 0.0, gain / sqrt((double)in)); }
// conv1d weight PyTorch [oc, ic, k] -> ne [k, ic, oc]
static void addconv(const char *n, int64_t oc, int64_t ic, int64_t k, double gain) {
    add_t(n, 3, k, ic, oc, 0.0, gain / sqrt((double)(ic * k)));
}

static int cp_h(const cfg_t *c) { return c->cp_hidden ? c->cp_hidden : c->hidden; }

static void build_talker(const cfg_t *c) {
    char b[96];
    const int H0 = c->hidden;
    {
    const int H = H0;
    addw("talker.text_embd.weight", c->text_vocab, c->text_dim, 0.02 * sqrt((double)c->text_dim));
    addw("talker.text_proj.fc1.weight", c->text_dim, c->text_dim, 1.0);
    add1("talker.text_proj.fc1.bias", c->text_dim, 0.0, 0.02);
    addw("talker.text_proj.fc2.weight", H, c->text_dim, 1.0);
    add1("talker.text_proj.fc2.bias", H, 0.0, 0.02);
    addw("talker.codec_embd.weight", c->codec_vocab, H, 0.02 * sqrt((double)H) * 8.0);
    addw("talker.codec_head.weight", c->codec_vocab, H, 4.0);
    add1("talker.output_norm.weight", H, 1.0, 0.1);
    }
    for (int L = 0; L < 2; ++L) {
        const int nl = L == 0 ? c->n_layers : c->cp_layers;
        const char *p = L == 0 ? "talker" : "code_pred";
        // layer geometry: the talker's, or the code predictor's own (1.7B)
        const int H = L == 0 ? H0 : cp_h(c);
        const int nh = L == 1 && c->cp_heads ? c->cp_heads : c->n_heads, nkv = L == 1 && c->cp_kv ? c->cp_kv : c->n_kv;
        const int Dq = nh * c->head_dim, Dkv = nkv * c->head_dim;
        const int I = L == 1 && c->cp_inter ? c->cp_inter : c->inter;
        for (int i = 0; i < nl; ++i) {
#define NM(suf) (snprintf(b, sizeof b, "%s.blk.%d.%s", p, i, suf), b)
            add1(NM("attn_norm.weight"), H, 1.0, 0.1);
            addw(NM("attn_q.weight"), Dq, H, 1.0);
            addw(NM("attn_k.weight"), Dkv, H, 1.0);
            addw(NM("attn_v.weight"), Dkv, H, 1.0);
            addw(NM("attn_output.weight"), H, Dq, 0.25);
            add1(NM("attn_q_norm.weight"), c->head_dim, 1.0, 0.1);
            add1(NM("attn_k_norm.weight"), c->head_dim, 1.0, 0.1);
            add1(NM("ffn_norm.weight"), H, 1.0, 0.1);
            addw(NM("ffn_gate.weight"), I, H, 1.0);
            addw(NM("ffn_up.weight"), I, H, 1.0);
            addw(NM("ffn_down.weight"), H, I, 0.25);
#undef NM
        }
    }
    add1("code_pred.output_norm.weight", cp_h(c), 1.0, 0.1);
    const int H = H0;
    if (c->cp_hidden && c->cp_hidden != H) {   // talker space -> code-predictor space (every code-predictor input)
        addw("code_pred.mtp_proj.weight", c->cp_hidden, H, 1.0);
        add1("code_pred.mtp_proj.bias", c->cp_hidden, 0.0, 0.02);
    }
    // speaker encoder (ECAPA-TDNN) in the TTS file, as the converter writes it (convert_tts_to_gguf.py:58-124;
    // loader audio_tokenizer_encoder.cpp:185-241): conv weights [OC, IC, K] -> ne [K, IC, OC], F32 biases
#define SPK(nm, oc, ic, k, g) do { snprintf(b, sizeof b, "spk_enc.%s.weight", nm); addconv(b, oc, ic, k, g); \
                                   snprintf(b, sizeof b, "spk_enc.%s.bias", nm); add1(b, oc, 0.0, 0.02); } while (0)
    SPK("conv0", 512, 128, 5, 1.0);
    for (int i = 1; i <= 3; ++i) {
        char nm[64];
        snprintf(nm, sizeof nm, "blk.%d.tdnn1", i); SPK(nm, 512, 512, 1, 1.41);
        for (int r = 0; r < 7; ++r) { snprintf(nm, sizeof nm, "blk.%d.res2net.%d", i, r); SPK(nm, 64, 64, 3, 1.41); }
        snprintf(nm, sizeof nm, "blk.%d.tdnn2", i); SPK(nm, 512, 512, 1, 1.41);
        snprintf(nm, sizeof nm, "blk.%d.se.conv1", i); SPK(nm, 128, 512, 1, 1.41);
        snprintf(nm, sizeof nm, "blk.%d.se.conv2", i); SPK(nm, 512, 128, 1, 1.0);
    }
    SPK("mfa", 1536, 1536, 1, 1.41);
    SPK("asp.tdnn", 128, 4608, 1, 1.41);
    SPK("asp.conv", 1536, 128, 1, 1.0);
    SPK("fc", H, 3072, 1, 1.0);
#undef SPK
    for (int i = 0; i < c->n_codebooks - 1; ++i) {
        snprintf(b, sizeof b, "code_pred.codec_embd.%d.weight", i);
        addw(b, c->cp_vocab, H, 0.02 * sqrt((double)H) * 8.0);
        snprintf(b, sizeof b, "code_pred.lm_head.%d.weight", i);
        addw(b, c->cp_vocab, cp_h(c), 4.0);
    }
}

static int g_usage = 0;

static void build_tokenizer(const cfg_t *c) {
    char b[128];
    const int CD = c->cb_dim, VH = c->voc_hidden, LAT = c->voc_latent;
    add_t("tok_dec.vq_first.0.codebook", 2, CD, c->cb_size, 1, 0.0, 1.0);
    if (g_usage) {
        add1("tok_dec.vq_first.0.usage", c->cb_size, 1.5, 0.3);
        for (int i = 0; i < c->n_codebooks - 1; ++i) {
            snprintf(b, sizeof b, "tok_dec.vq_rest.%d.usage", i);
            add1(b, c->cb_size, 1.5, 0.3);
        }
    }
    add_t("tok_dec.vq_first.input_proj.weight", 3, 1, VH, CD, 0.0, 1.0 / sqrt((double)VH));
    add_t("tok_dec.vq_first.output_proj.weight", 3, 1, CD, VH, 0.0, 1.0 / sqrt((double)CD));
    for (int i = 0; i < c->n_codebooks - 1; ++i) {
        snprintf(b, sizeof b, "tok_dec.vq_rest.%d.codebook", i);
        add_t(b, 2, CD, c->cb_size, 1, 0.0, 1.0);
    }
    add_t("tok_dec.vq_rest.input_proj.weight", 3, 1, VH, CD, 0.0, 1.0 / sqrt((double)VH));
    add_t("tok_dec.vq_rest.output_proj.weight", 3, 1, CD, VH, 0.0, 0.25 / sqrt((double)CD));
    addconv("tok_dec.pre_conv.weight", LAT, VH, 3, 1.0);
    add1("tok_dec.pre_conv.bias", LAT, 0.0, 0.02);
    addw("tok_dec.pre_tfm.input_proj.weight", VH, LAT, 1.0);
    add1("tok_dec.pre_tfm.input_proj.bias", VH, 0.0, 0.02);
    for (int i = 0; i < c->voc_layers; ++i) {
#define NM(suf) (snprintf(b, sizeof b, "tok_dec.pre_tfm.blk.%d.%s", i, suf), b)
        add1(NM("attn_norm.weight"), VH, 1.0, 0.1);
        addw(NM("attn_q.weight"), LAT, VH, 1.0);
        addw(NM("attn_k.weight"), LAT, VH, 1.0);
        addw(NM("attn_v.weight"), LAT, VH, 1.0);
        addw(NM("attn_output.weight"), VH, LAT, 1.0);
        add1(NM("attn_scale"), VH, 0.25, 0.05);
        add1(NM("ffn_norm.weight"), VH, 1.0, 0.1);
        addw(NM("ffn_gate.weight"), c->voc_ffn, VH, 1.0);
        addw(NM("ffn_up.weight"), c->voc_ffn, VH, 1.0);
        addw(NM("ffn_down.weight"), VH, c->voc_ffn, 1.0);
        add1(NM("ffn_scale"), VH, 0.25, 0.05);
#undef NM
    }
    add1("tok_dec.pre_tfm.norm.weight", VH, 1.0, 0.1);
    addw("tok_dec.pre_tfm.output_proj.weight", LAT, VH, 1.0);
    add1("tok_dec.pre_tfm.output_proj.bias", LAT, 0.0, 0.02);
    for (int u = 0; u < 2; ++u) {
#define NM(suf) (snprintf(b, sizeof b, "tok_dec.upsample.%d.%s", u, suf), b)
        // ConvTranspose1d weight PyTorch [ic, oc, k] -> ne [k, oc, ic]
        add_t(NM("conv.weight"), 3, c->up_ratio, LAT, LAT, 0.0, 1.0 / sqrt((double)LAT));
        add1(NM("conv.bias"), LAT, 0.0, 0.02);
        add_t(NM("dwconv.weight"), 3, 7, 1, LAT, 0.0, 1.0 / sqrt(7.0));
        add1(NM("dwconv.bias"), LAT, 0.0, 0.02);
        add1(NM("norm.weight"), LAT, 1.0, 0.1);
        add1(NM("norm.bias"), LAT, 0.0, 0.02);
        addw(NM("pwconv1.weight"), c->convnext_mult * LAT, LAT, 1.0);
        add1(NM("pwconv1.bias"), c->convnext_mult * LAT, 0.0, 0.02);
        addw(NM("pwconv2.weight"), LAT, c->convnext_mult * LAT, 1.0);
        add1(NM("pwconv2.bias"), LAT, 0.0, 0.02);
        add1(NM("gamma"), LAT, 0.25, 0.05);
#undef NM
    }
    addconv("tok_dec.dec.0.conv.weight", c->dec_dim, LAT, 7, 1.0);
    add1("tok_dec.dec.0.conv.bias", c->dec_dim, 0.0, 0.02);
    int ch = c->dec_dim;
    for (int d = 1; d <= 4; ++d) {
        const int r = c->rates[d - 1], oc = ch / 2;
#define NM(suf) (snprintf(b, sizeof b, "tok_dec.dec.%d.%s", d, suf), b)
        add1(NM("snake.alpha"), ch, 0.0, 0.1);
        add1(NM("snake.beta"), ch, 0.0, 0.1);
        add_t(NM("conv_t.weight"), 3, 2 * r, oc, ch, 0.0, 1.0 / sqrt((double)ch * 2.0));
        add1(NM("conv_t.bias"), oc, 0.0, 0.02);
#undef NM
        for (int ri = 2; ri <= 4; ++ri) {
#define NM(suf) (snprintf(b, sizeof b, "tok_dec.dec.%d.res.%d.%s", d, ri, suf), b)
            add1(NM("act1.alpha"), oc, 0.0, 0.1);
            add1(NM("act1.beta"), oc, 0.0, 0.1);
            addconv(NM("conv1.weight"), oc, oc, 7, 1.0);
            add1(NM("conv1.bias"), oc, 0.0, 0.02);
            add1(NM("act2.alpha"), oc, 0.0, 0.1);
            add1(NM("act2.beta"), oc, 0.0, 0.1);
            addconv(NM("conv2.weight"), oc, oc, 1, 0.35);
            add1(NM("conv2.bias"), oc, 0.0, 0.02);
#undef NM
        }
        ch = oc;
    }
    add1("tok_dec.dec.5.snake.alpha", ch, 0.0, 0.1);
    add1("tok_dec.dec.5.snake.beta", ch, 0.0, 0.1);
    addconv("tok_dec.dec.6.conv.weight", 1, ch, 7, 0.3);
    add1("tok_dec.dec.6.conv.bias", 1, 0.0, 0.002);
}

// ---------------------------------------------------------------- text vocabulary (tokenizer.ggml.*)
// The converter writes vocab.json's tokens sorted by id, pads the list with "[PAD<id>]" up to text_vocab_size, and adds
// merges.txt (convert_tts_to_gguf.py:337-377, 498-547); Qwen's special tokens are not in vocab.json, so ids >= 151643
// are pads and the tokenizer falls back to its default bos / eos ids (text_tokenizer.h:13-18).  Synthetic stand-in:
// ids 0..255 are the GPT-2 byte symbols in Qwen's own order (id 13 = ".", 198 = "Ċ", 220 = "Ġ"), a word list is
// merged left to right into whole-word tokens ("Hello" at Qwen's id 9707, "assistant" at 77091, the ids of the
// reference's known-answer vector, tests/test_tokenizer.cpp:14), the rest are "[SYN<id>]" fillers.
static const char *VOCAB_WORDS[] = {
    "Hello", "assistant", "hello", "world", "the", "of", "and", "to", "in", "is", "you", "that", "it", "he", "was",
    "for", "on", "are", "as", "with", "his", "they", "at", "be", "this", "This", "have", "from", "or", "one", "had",
    "by", "word", "but", "not", "what", "all", "were", "we", "when", "your", "can", "said", "there", "use", "an",
    "each", "which", "she", "do", "how", "their", "if", "will", "up", "other", "about", "out", "many", "then", "them",
    "these", "so", "some", "her", "would", "make", "like", "him", "into", "time", "has", "look", "two", "more",
    "write", "go", "see", "number", "no", "way", "could", "people", "my", "than", "first", "water", "been", "call",
    "who", "its", "now", "find", "long", "down", "day", "did", "get", "come", "made", "may", "part", "test", "speech",
    "voice", "quick", "brown", "fox", "jumps", "over", "lazy", "dog", "The", "It", "We", "GPU", "audio", "text",
    "model", "ing", "ed", "er", "ly", "tion", "ation", "123", "2026", "!!", "...", ".\n", "\n\n"};
static char **g_vocab = NULL;
static int g_nvocab = 0, g_nmerge = 0;
static char **g_merges = NULL;
static int *g_toktype = NULL;

static void byte_sym(int b, char out[4]) {   // GPT-2 bytes_to_unicode: printable latin-1 keep their code point
    int cp;
    if ((b >= 33 && b <= 126) || (b >= 161 && b <= 172) || b >= 174) cp = b;
    else {
        int n = 0;
        for (int x = 0; x < b; ++x) n += !((x >= 33 && x <= 126) || (x >= 161 && x <= 172) || x >= 174);
        cp = 256 + n;
    }
    if (cp < 0x80) { out[0] = (char)cp; out[1] = 0; }
    else { out[0] = (char)(0xC0 | (cp >> 6)); out[1] = (char)(0x80 | (cp & 0x3F)); out[2] = 0; }
}
static int vocab_find(const char *t) {
    for (int i = 0; i < g_nvocab; ++i) if (g_vocab[i] && strcmp(g_vocab[i], t) == 0) return i;
    return -1;
}
static int g_next_id = 256;
static int vocab_add(const char *t, int want) {
    int id = vocab_find(t);
    if (id >= 0) return id;
    if (want < 0) {
        while (g_next_id < g_nvocab && (g_vocab[g_next_id] || g_next_id == 9707 || g_next_id == 77091)) ++g_next_id;
        want = g_next_id;
    }
    if (want >= g_nvocab || g_vocab[want]) return -1;
    g_vocab[want] = strdup(t);
    return want;
}
static void build_vocab(const cfg_t *c) {
    g_nvocab = c->text_vocab;
    g_vocab = calloc((size_t)g_nvocab, sizeof(char *));
    g_toktype = malloc(sizeof(int) * (size_t)g_nvocab);
    g_merges = malloc(sizeof(char *) * 8192);
    // byte symbols in Qwen order: the printable ones (by byte value), then the remapped ones
    int id = 0;
    for (int pass = 0; pass < 2; ++pass)
        for (int b = 0; b < 256; ++b) {
            const int printable = (b >= 33 && b <= 126) || (b >= 161 && b <= 172) || b >= 174;
            if (printable != (pass == 0)) continue;
            char s[4];
            byte_sym(b, s);
            g_vocab[id++] = strdup(s);
        }
    const int n_real = c->text_vocab > 151643 ? 151643 : c->text_vocab;   // ids the converter takes from vocab.json
    for (size_t w = 0; w < sizeof VOCAB_WORDS / sizeof VOCAB_WORDS[0]; ++w)
        for (int sp = 0; sp < 2; ++sp) {
            // GPT-2 symbols of (" " +) word, merged left to right
            char sym[64][8];
            int n = 0;
            if (sp) { byte_sym(' ', sym[n]); ++n; }
            for (const unsigned char *p = (const unsigned char *)VOCAB_WORDS[w]; *p && n < 63; ++p) byte_sym(*p, sym[n++]);
            char acc[512] = "";
            strcat(acc, sym[0]);
            for (int k = 1; k < n; ++k) {
                char merged[512];
                snprintf(merged, sizeof merged, "%s%s", acc, sym[k]);
                int want = -1;
                if (k == n - 1 && !sp && strcmp(VOCAB_WORDS[w], "Hello") == 0 && 9707 < n_real) want = 9707;
                if (k == n - 1 && !sp && strcmp(VOCAB_WORDS[w], "assistant") == 0 && 77091 < n_real) want = 77091;
                if (vocab_find(merged) < 0) {
                    if (g_next_id >= n_real && want < 0) break;
                    if (vocab_add(merged, want) < 0) break;
                    char m[1024];
                    snprintf(m, sizeof m, "%s %s", acc, sym[k]);
                    if (g_nmerge < 8192) g_merges[g_nmerge++] = strdup(m);
                }
                strcpy(acc, merged);
            }
        }
    for (int i = 0; i < g_nvocab; ++i) {
        if (!g_vocab[i]) {
            char b[32];
            snprintf(b, sizeof b, i < n_real ? "[SYN%d]" : "[PAD%d]", i);
            g_vocab[i] = strdup(b);
        }
        g_toktype[i] = i < n_real ? 1 : 5;   // NORMAL / UNUSED (gguf.TokenType)
    }
}

// ---------------------------------------------------------------- weight dtype policy (--outtype)
static const char *g_outtype = "f16";
static uint16_t f32_to_f16_rne(float x);
static int block_of(int type) { return type == GGML_Q4_K ? 256 : (type == GGML_Q8_0 || type == GGML_Q4_0) ? 32 : 1; }
static uint64_t type_bytes(int type, uint64_t n) {
    switch (type) {
        case GGML_F32: return n * 4;
        case GGML_F16: return n * 2;
        case GGML_Q8_0: return n / 32 * 34;
        case GGML_Q4_0: return n / 32 * 18;
        case GGML_Q4_K: return n / 256 * 144;
    }
    return 0;
}
static uint32_t file_type(void) {   // llama_ftype of the --outtype
    return strcmp(g_outtype, "f32") == 0 ? 0 : strcmp(g_outtype, "q4_0") == 0 ? 2 : strcmp(g_outtype, "q8_0") == 0 ? 7
         : strcmp(g_outtype, "q4_k") == 0 ? 15 : 1;
}
static void apply_dtype_policy(int tts_file) {
    const int want = strcmp(g_outtype, "q8_0") == 0 ? GGML_Q8_0 : strcmp(g_outtype, "q4_0") == 0 ? GGML_Q4_0
                   : strcmp(g_outtype, "q4_k") == 0 ? GGML_Q4_K : strcmp(g_outtype, "f32") == 0 ? GGML_F32 : GGML_F16;
    for (int i = 0; i < g_nt; ++i) {
        tens_t *t = &g_t[i];
        if (t->ndims <= 1) continue;   // 1-D: always F32
        if (want == GGML_F32 || want == GGML_F16) { t->type = want; continue; }
        int keep;
        if (tts_file)   // _should_quantize (convert_tts_to_gguf.py:250-274)
            keep = strstr(t->name, "_embd") || strstr(t->name, "codebook") || strstr(t->name, "_norm") ||
                   strstr(t->name, ".bias") || strstr(t->name, "lm_head") || strstr(t->name, "codec_head");
        else            // convert_tokenizer_to_gguf.py:283-294 (q8_0 only)
            keep = want != GGML_Q8_0 || strstr(t->name, "codebook") || strstr(t->name, "_norm") ||
                   strstr(t->name, "norm.") || strstr(t->name, "scale") || strstr(t->name, "alpha") ||
                   strstr(t->name, "beta");
        // gguf.quants.quantize needs whole blocks along the row: otherwise the converter falls back to F16
        t->type = (keep || t->ne[0] % block_of(want)) ? GGML_F16 : want;
    }
}
// ggml quantize_row_q8_0_ref: d = amax / 127, q = round(x / d)
static void quant_q8_0(const float *x, uint8_t *o, int64_t n) {
    for (int64_t b = 0; b < n / 32; ++b, o += 34) {
        float amax = 0.0f;
        for (int j = 0; j < 32; ++j) amax = fmaxf(amax, fabsf(x[b * 32 + j]));
        const float d = amax / 127.0f, id = d ? 1.0f / d : 0.0f;
        const uint16_t dh = f32_to_f16_rne(d);
        memcpy(o, &dh, 2);
        for (int j = 0; j < 32; ++j) o[2 + j] = (uint8_t)(int8_t)roundf(x[b * 32 + j] * id);
    }
}
// ggml quantize_row_q4_0_ref: d = (signed max-magnitude value) / -8, q = min(15, (int)(x / d + 8.5))
static void quant_q4_0(const float *x, uint8_t *o, int64_t n) {
    for (int64_t b = 0; b < n / 32; ++b, o += 18) {
        float amax = 0.0f, mx = 0.0f;
        for (int j = 0; j < 32; ++j) { const float v = x[b * 32 + j]; if (fabsf(v) > amax) { amax = fabsf(v); mx = v; } }
        const float d = mx / -8.0f, id = d ? 1.0f / d : 0.0f;
        const uint16_t dh = f32_to_f16_rne(d);
        memcpy(o, &dh, 2);
        for (int j = 0; j < 16; ++j) {
            int q0 = (int)(x[b * 32 + j] * id + 8.5f), q1 = (int)(x[b * 32 + j + 16] * id + 8.5f);
            q0 = q0 > 15 ? 15 : q0; q1 = q1 > 15 ? 15 : q1;
            o[2 + j] = (uint8_t)(q0 | (q1 << 4));
        }
    }
}
// Q4_K super-block of 256: per 32-value sub-block scale = (max - min) / 15 and offset -min, both quantised to 6 bits
// against the super-block's d / dmin, packed as ggml_get_scale_min_k4 unpacks them
static void quant_q4_k(const float *x, uint8_t *o, int64_t n) {
    for (int64_t b = 0; b < n / 256; ++b, o += 144) {
        const float *v = x + b * 256;
        float sc[8], mn[8], msc = 0.0f, mmn = 0.0f;
        for (int s = 0; s < 8; ++s) {
            float lo = v[s * 32], hi = v[s * 32];
            for (int j = 1; j < 32; ++j) { lo = fminf(lo, v[s * 32 + j]); hi = fmaxf(hi, v[s * 32 + j]); }
            if (lo > 0) lo = 0;
            sc[s] = (hi - lo) / 15.0f;
            mn[s] = -lo;
            msc = fmaxf(msc, sc[s]);
            mmn = fmaxf(mmn, mn[s]);
        }
        const float d = msc / 63.0f, dmin = mmn / 63.0f;
        const uint16_t dh = f32_to_f16_rne(d), mh = f32_to_f16_rne(dmin);
        memcpy(o, &dh, 2);
        memcpy(o + 2, &mh, 2);
        uint8_t ls[8], lm[8];
        for (int s = 0; s < 8; ++s) {
            int a = d ? (int)lroundf(sc[s] / d) : 0, c = dmin ? (int)lroundf(mn[s] / dmin) : 0;
            ls[s] = (uint8_t)(a > 63 ? 63 : a);
            lm[s] = (uint8_t)(c > 63 ? 63 : c);
        }
        uint8_t *S = o + 4;
        for (int j = 0; j < 4; ++j) {
            S[j] = (uint8_t)((ls[j] & 63) | ((ls[j + 4] >> 4) << 6));
            S[j + 4] = (uint8_t)((lm[j] & 63) | ((lm[j + 4] >> 4) << 6));
            S[j + 8] = (uint8_t)((ls[j + 4] & 15) | ((lm[j + 4] & 15) << 4));
        }
        uint8_t *Q = o + 16;
        for (int s = 0; s < 8; s += 2)
            for (int l = 0; l < 32; ++l) {
                int q[2];
                for (int u = 0; u < 2; ++u) {
                    const float step = d * ls[s + u], off = dmin * lm[s + u];
                    int t = step > 0 ? (int)lroundf((v[(s + u) * 32 + l] + off) / step) : 0;
                    q[u] = t < 0 ? 0 : t > 15 ? 15 : t;
                }
                Q[(s / 2) * 32 + l] = (uint8_t)(q[0] | (q[1] << 4));
            }
    }
}

// ---------------------------------------------------------------- GGUF v3 writer
static void w_u32(FILE *f, uint32_t v) { fwrite(&v, 4, 1, f); }
static void w_u64(FILE *f, uint64_t v) { fwrite(&v, 8, 1, f); }
static void w_str(FILE *f, const char *s) { w_u64(f, strlen(s)); fwrite(s, 1, strlen(s), f); }

typedef struct { const char *key; int type; uint32_t u; float fl; const char *s; int arr_n; const int *arr; char **sarr; } kv_t;

static uint16_t f32_to_f16_rne(float x) {
    uint32_t u; memcpy(&u, &x, 4);
    uint32_t sign = (u >> 16) & 0x8000u;
    int32_t exp = (int32_t)((u >> 23) & 0xff) - 127 + 15;
    uint32_t mant = u & 0x7fffffu;
    if (((u >> 23) & 0xff) == 0xff) return (uint16_t)(sign | 0x7c00u | (mant ? 0x200u : 0));
    if (exp >= 31) return (uint16_t)(sign | 0x7c00u);
    if (exp <= 0) {
        if (exp < -10) return (uint16_t)sign;
        mant |= 0x800000u;
        int shift = 14 - exp;
        uint32_t half = 1u << (shift - 1);
        uint32_t r = mant >> shift, rem = mant & ((1u << shift) - 1);
        if (rem > half || (rem == half && (r & 1))) r++;
        return (uint16_t)(sign | r);
    }
    uint32_t r = mant >> 13, rem = mant & 0x1fffu;
    uint32_t h = sign | ((uint32_t)exp << 10) | r;
    if (rem > 0x1000u || (rem == 0x1000u && (r & 1))) h++;
    return (uint16_t)h;
}

static float synth_value(uint64_t base, uint64_t i, float center, int e) {
    uint64_t h = mix64(base + i);
    int s = (int)(h & 1023) + (int)((h >> 10) & 1023) + (int)((h >> 20) & 1023) + (int)((h >> 30) & 1023) - 2046;
    return center + ldexpf((float)s, -e);
}

static int write_gguf(const char *path, const kv_t *kvs, int nkv, uint64_t seed) {
    FILE *f = fopen(path, "wb");
    if (!f) { perror(path); return 1; }
    const uint64_t align = 32;
    uint64_t off = 0;
    for (int i = 0; i < g_nt; ++i) {
        tens_t *t = &g_t[i];
        g_t[i].off = off;
        uint64_t n = (uint64_t)t->ne[0] * t->ne[1] * t->ne[2] * t->ne[3];
        off += type_bytes(t->type, n);
        off = (off + align - 1) / align * align;
    }
    fwrite("GGUF", 1, 4, f);
    w_u32(f, 3);
    w_u64(f, (uint64_t)g_nt);
    w_u64(f, (uint64_t)nkv);
    for (int i = 0; i < nkv; ++i) {
        w_str(f, kvs[i].key);
        w_u32(f, (uint32_t)kvs[i].type);
        if (kvs[i].type == GV_U32) w_u32(f, kvs[i].u);
        else if (kvs[i].type == GV_F32) fwrite(&kvs[i].fl, 4, 1, f);
        else if (kvs[i].type == GV_STR) w_str(f, kvs[i].s);
        else if (kvs[i].type == GV_ARR && kvs[i].sarr) {   // string array
            w_u32(f, GV_STR);
            w_u64(f, (uint64_t)kvs[i].arr_n);
            for (int j = 0; j < kvs[i].arr_n; ++j) w_str(f, kvs[i].sarr[j]);
        } else if (kvs[i].type == GV_ARR) {
            w_u32(f, GV_U32 + 1);  // INT32 array
            w_u64(f, (uint64_t)kvs[i].arr_n);
            for (int j = 0; j < kvs[i].arr_n; ++j) w_u32(f, (uint32_t)kvs[i].arr[j]);
        }
    }
    for (int i = 0; i < g_nt; ++i) {
        tens_t *t = &g_t[i];
        w_str(f, t->name);
        w_u32(f, (uint32_t)t->ndims);
        for (int d = 0; d < t->ndims; ++d) w_u64(f, (uint64_t)t->ne[d]);
        w_u32(f, (uint32_t)t->type);
        w_u64(f, t->off);
    }
    long pos = ftell(f);
    long pad = (long)((pos + align - 1) / align * align) - pos;
    static const char zeros[64] = {0};
    fwrite(zeros, 1, (size_t)pad, f);
    const uint64_t data_start = (uint64_t)ftell(f);
    const size_t CH = 1 << 22;
    void *buf = malloc(CH * 4);
    for (int i = 0; i < g_nt; ++i) {
        tens_t *t = &g_t[i];
        fseek(f, (long)(data_start + t->off), SEEK_SET);
        const uint64_t n = (uint64_t)t->ne[0] * t->ne[1] * t->ne[2] * t->ne[3];
        const uint64_t base = mix64(seed ^ fnv1a64(t->name));
        if (t->type != GGML_F16 && t->type != GGML_F32) {   // block-quantised, one row at a time
            const int64_t row = t->ne[0];
            float *x = malloc(sizeof(float) * (size_t)row);
            uint8_t *q = malloc((size_t)type_bytes(t->type, (uint64_t)row));
            for (uint64_t r = 0; r < n / (uint64_t)row; ++r) {
                for (int64_t j = 0; j < row; ++j) x[j] = synth_value(base, r * (uint64_t)row + (uint64_t)j, t->center, t->e);
                if (t->type == GGML_Q8_0) quant_q8_0(x, q, row);
                else if (t->type == GGML_Q4_0) quant_q4_0(x, q, row);
                else quant_q4_k(x, q, row);
                fwrite(q, 1, (size_t)type_bytes(t->type, (uint64_t)row), f);
            }
            free(x);
            free(q);
            continue;
        }
        for (uint64_t s0 = 0; s0 < n; s0 += CH) {
            const uint64_t m = (n - s0) < CH ? (n - s0) : CH;
            if (t->type == GGML_F16) {
                uint16_t *o = (uint16_t *)buf;
#pragma omp parallel for schedule(static)
                for (int64_t j = 0; j < (int64_t)m; ++j) o[j] = f32_to_f16_rne(synth_value(base, s0 + j, t->center, t->e));
                fwrite(o, 2, m, f);
            } else {
                float *o = (float *)buf;
#pragma omp parallel for schedule(static)
                for (int64_t j = 0; j < (int64_t)m; ++j) o[j] = synth_value(base, s0 + j, t->center, t->e);
                fwrite(o, 4, m, f);
            }
        }
    }
    // pad file end to alignment
    fseek(f, 0, SEEK_END);
    pos = ftell(f);
    pad = (long)((pos + align - 1) / align * align) - pos;
    fwrite(zeros, 1, (size_t)pad, f);
    free(buf);
    fclose(f);
    return 0;
}

int main(int argc, char **argv) {
    if (argc < 3) { fprintf(stderr, "usage: %s full|full5|tiny|tiny1|tiny17|full17 <out_dir> [seed]\n", argv[0]); return 2; }
    const cfg_t *c = strcmp(argv[1], "full") == 0 ? &CFG_FULL : strcmp(argv[1], "tiny") == 0 ? &CFG_TINY : strcmp(argv[1], "tiny1") == 0 ? &CFG_TINY1
                   : strcmp(argv[1], "tiny17") == 0 ? &CFG_TINY17 : strcmp(argv[1], "full17") == 0 ? &CFG_FULL17
                   : strcmp(argv[1], "full5") == 0 ? &CFG_FULL5 : NULL;
    if (!c) { fprintf(stderr, "unknown config %s\n", argv[1]); return 2; }
    uint64_t seed = argc > 3 ? strtoull(argv[3], NULL, 0) : 0x51E3775ull;
    g_usage = argc > 4 && strcmp(argv[4], "usage") == 0;
    if (argc > 4 && !g_usage) g_outtype = argv[4];
    char path[4096];

    build_talker(c);
    apply_dtype_policy(1);
    build_vocab(c);
    kv_t kt[] = {
        {"general.architecture", GV_STR, 0, 0, "qwen3-tts", 0, 0},
        {"general.name", GV_STR, 0, 0, c->name, 0, 0},
        {"general.file_type", GV_U32, file_type(), 0, 0, 0, 0},
        {"qwen3-tts.block_count", GV_U32, (uint32_t)c->n_layers, 0, 0, 0, 0},
        {"qwen3-tts.embedding_length", GV_U32, (uint32_t)c->hidden, 0, 0, 0, 0},
        {"qwen3-tts.feed_forward_length", GV_U32, (uint32_t)c->inter, 0, 0, 0, 0},
        {"qwen3-tts.attention.head_count", GV_U32, (uint32_t)c->n_heads, 0, 0, 0, 0},
        {"qwen3-tts.attention.head_count_kv", GV_U32, (uint32_t)c->n_kv, 0, 0, 0, 0},
        {"qwen3-tts.attention.key_length", GV_U32, (uint32_t)c->head_dim, 0, 0, 0, 0},
        {"qwen3-tts.attention.value_length", GV_U32, (uint32_t)c->head_dim, 0, 0, 0, 0},
        {"qwen3-tts.rope.freq_base", GV_F32, 0, c->rope_theta, 0, 0, 0},
        {"qwen3-tts.attention.layer_norm_rms_epsilon", GV_F32, 0, c->eps, 0, 0, 0},
        {"qwen3-tts.vocab_size", GV_U32, (uint32_t)c->codec_vocab, 0, 0, 0, 0},
        {"qwen3-tts.text_vocab_size", GV_U32, (uint32_t)c->text_vocab, 0, 0, 0, 0},
        {"qwen3-tts.text_hidden_size", GV_U32, (uint32_t)c->text_dim, 0, 0, 0, 0},
        {"qwen3-tts.num_code_groups", GV_U32, (uint32_t)c->n_codebooks, 0, 0, 0, 0},
        {"qwen3-tts.code_predictor.layer_count", GV_U32, (uint32_t)c->cp_layers, 0, 0, 0, 0},
        {"qwen3-tts.code_predictor.vocab_size", GV_U32, (uint32_t)c->cp_vocab, 0, 0, 0, 0},
        {"qwen3-tts.code_predictor.embedding_length", GV_U32, (uint32_t)cp_h(c), 0, 0, 0, 0},
        {"qwen3-tts.code_predictor.feed_forward_length", GV_U32, (uint32_t)(c->cp_inter ? c->cp_inter : c->inter), 0, 0, 0, 0},
        {"qwen3-tts.code_predictor.attention.head_count", GV_U32, (uint32_t)(c->cp_heads ? c->cp_heads : c->n_heads), 0, 0, 0, 0},
        {"qwen3-tts.code_predictor.attention.head_count_kv", GV_U32, (uint32_t)(c->cp_kv ? c->cp_kv : c->n_kv), 0, 0, 0, 0},
        {"qwen3-tts.code_predictor.attention.key_length", GV_U32, (uint32_t)c->head_dim, 0, 0, 0, 0},
        {"qwen3-tts.codec.pad_id", GV_U32, 2148, 0, 0, 0, 0},
        {"qwen3-tts.codec.bos_id", GV_U32, 2149, 0, 0, 0, 0},
        {"qwen3-tts.codec.eos_id", GV_U32, 2150, 0, 0, 0, 0},
        {"qwen3-tts.tts_bos_token_id", GV_U32, (uint32_t)c->tts_bos, 0, 0, 0, 0},
        {"qwen3-tts.tts_eos_token_id", GV_U32, (uint32_t)c->tts_eos, 0, 0, 0, 0},
        {"qwen3-tts.tts_pad_token_id", GV_U32, (uint32_t)c->tts_pad, 0, 0, 0, 0},
        {"qwen3-tts.speaker_encoder.embedding_length", GV_U32, (uint32_t)c->hidden, 0, 0, 0, 0},
        {"qwen3-tts.speaker_encoder.sample_rate", GV_U32, 24000, 0, 0, 0, 0},
        {"tokenizer.ggml.model", GV_STR, 0, 0, "gpt2", 0, 0},
        {"tokenizer.ggml.pre", GV_STR, 0, 0, "qwen2", 0, 0},
        {"tokenizer.ggml.tokens", GV_ARR, 0, 0, 0, g_nvocab, 0, g_vocab},
        {"tokenizer.ggml.token_type", GV_ARR, 0, 0, 0, g_nvocab, g_toktype},
        {"tokenizer.ggml.merges", GV_ARR, 0, 0, 0, g_nmerge, 0, g_merges},
    };
    snprintf(path, sizeof path, "%s/qwen3-tts-0.6b-f16.gguf", argv[2]);
    if (write_gguf(path, kt, (int)(sizeof kt / sizeof kt[0]), seed)) return 1;

    g_nt = 0;
    build_tokenizer(c);
    apply_dtype_policy(0);
    kv_t kk[] = {
        {"general.architecture", GV_STR, 0, 0, "qwen3-tts-tokenizer", 0, 0},
        {"general.name", GV_STR, 0, 0, c->name, 0, 0},
        {"qwen3-tts-tokenizer.num_codebooks", GV_U32, (uint32_t)c->n_codebooks, 0, 0, 0, 0},
        {"qwen3-tts-tokenizer.codebook_size", GV_U32, (uint32_t)c->cb_size, 0, 0, 0, 0},
        {"qwen3-tts-tokenizer.sample_rate", GV_U32, 24000, 0, 0, 0, 0},
        {"qwen3-tts-tokenizer.decoder.hidden_size", GV_U32, (uint32_t)c->voc_hidden, 0, 0, 0, 0},
        {"qwen3-tts-tokenizer.decoder.num_layers", GV_U32, (uint32_t)c->voc_layers, 0, 0, 0, 0},
        {"qwen3-tts-tokenizer.decoder.num_heads", GV_U32, (uint32_t)c->voc_heads, 0, 0, 0, 0},
        {"qwen3-tts-tokenizer.decoder.latent_dim", GV_U32, (uint32_t)c->voc_latent, 0, 0, 0, 0},
        {"qwen3-tts-tokenizer.upsample_rates", GV_ARR, 0, 0, 0, 4, c->rates},
    };
    snprintf(path, sizeof path, "%s/qwen3-tts-tokenizer-f16.gguf", argv[2]);
    if (write_gguf(path, kk, (int)(sizeof kk / sizeof kk[0]), seed ^ 0x70CE11ull)) return 1;
    return 0;
}
