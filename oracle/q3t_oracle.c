/* q3t_oracle.c — CPU restatement of the reference's per-frame decode path (TEST INFRASTRUCTURE ONLY).
 * See q3t_oracle.h for scope and numerics.  Every function cites the reference lines it restates.
 * Built by oracle/Makefile into oracle/_build/libq3t_oracle.so; never linked into the product.
 */
#define _GNU_SOURCE
#include "q3t_oracle.h"

#include <fcntl.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#ifdef _OPENMP
#include <omp.h>
#endif
#if defined(__F16C__) && defined(__AVX2__) && defined(__FMA__)
#include <immintrin.h>
#define Q3O_SIMD 1
#endif

static __thread char g_err[512];
const char *q3o_error(void) { return g_err; }
#define FAIL(...) do { snprintf(g_err, sizeof g_err, __VA_ARGS__); return 0; } while (0)

void q3o_set_threads(int n) {
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
#else
    (void)n;
#endif
}

/* ------------------------------------------------------------------ f16 helpers (IEEE binary16, RNE) */
float q3o_f16_to_f32(uint16_t h) {
    uint32_t s = (uint32_t)(h & 0x8000u) << 16, e = (h >> 10) & 0x1f, m = h & 0x3ff, u;
    if (e == 0) {
        if (m == 0) u = s;
        else { float f = ldexpf((float)m, -24); memcpy(&u, &f, 4); u |= s; }
    } else if (e == 31) u = s | 0x7f800000u | (m << 13);
    else u = s | ((e + 112) << 23) | (m << 13);
    float f; memcpy(&f, &u, 4); return f;
}
uint16_t q3o_f32_to_f16(float x) {
#ifdef Q3O_SIMD
    return (uint16_t)_cvtss_sh(x, 0);
#else
    uint32_t u; memcpy(&u, &x, 4);
    uint32_t sign = (u >> 16) & 0x8000u, mant = u & 0x7fffffu;
    int32_t exp = (int32_t)((u >> 23) & 0xff) - 127 + 15;
    if (((u >> 23) & 0xff) == 0xff) return (uint16_t)(sign | 0x7c00u | (mant ? 0x200u : 0));
    if (exp >= 31) return (uint16_t)(sign | 0x7c00u);
    if (exp <= 0) {
        if (exp < -10) return (uint16_t)sign;
        mant |= 0x800000u; int shift = 14 - exp; uint32_t half = 1u << (shift - 1);
        uint32_t r = mant >> shift, rem = mant & ((1u << shift) - 1);
        if (rem > half || (rem == half && (r & 1))) r++;
        return (uint16_t)(sign | r);
    }
    uint32_t r = mant >> 13, rem = mant & 0x1fffu, h = sign | ((uint32_t)exp << 10) | r;
    if (rem > 0x1000u || (rem == 0x1000u && (r & 1))) h++;
    return (uint16_t)h;
#endif
}
static inline float f16r(float x) { return q3o_f16_to_f32(q3o_f32_to_f16(x)); }

/* ------------------------------------------------------------------ GGUF reader (v2/v3) */
typedef struct { char *name; int nd; int64_t ne[4]; int type, src_type; uint64_t off; uint16_t *own; } gtensor;
typedef struct { char *key; int type; uint64_t u; double f; } gkv;
typedef struct {
    uint8_t *map; size_t size; uint64_t data_off;
    gtensor *t; int64_t nt; gkv *kv; int64_t nkv;
} gguf_t;

static int rd(const uint8_t **p, const uint8_t *end, void *dst, size_t n) {
    if ((size_t)(end - *p) < n) return 0;
    memcpy(dst, *p, n); *p += n; return 1;
}
static char *rd_str(const uint8_t **p, const uint8_t *end) {
    uint64_t n; if (!rd(p, end, &n, 8) || (uint64_t)(end - *p) < n) return NULL;
    char *s = malloc(n + 1); memcpy(s, *p, n); s[n] = 0; *p += n; return s;
}
static const size_t GTYPE_SZ[13] = {1, 1, 2, 2, 4, 4, 4, 1, 0, 0, 8, 8, 8};
static int skip_val(const uint8_t **p, const uint8_t *end, uint32_t type, gkv *out) {
    if (type == 8) { char *s = rd_str(p, end); if (!s) return 0; free(s); return 1; }
    if (type == 9) {
        uint32_t et; uint64_t n;
        if (!rd(p, end, &et, 4) || !rd(p, end, &n, 8)) return 0;
        for (uint64_t i = 0; i < n; ++i) if (!skip_val(p, end, et, NULL)) return 0;
        return 1;
    }
    if (type > 12) return 0;
    uint8_t b[8] = {0};
    if (!rd(p, end, b, GTYPE_SZ[type])) return 0;
    if (out) {
        switch (type) {
            case 0: out->u = b[0]; out->f = b[0]; break;
            case 1: out->u = (uint64_t)(int64_t)(int8_t)b[0]; out->f = (int8_t)b[0]; break;
            case 2: { uint16_t v; memcpy(&v, b, 2); out->u = v; out->f = v; } break;
            case 3: { int16_t v; memcpy(&v, b, 2); out->u = (uint64_t)(int64_t)v; out->f = v; } break;
            case 4: { uint32_t v; memcpy(&v, b, 4); out->u = v; out->f = v; } break;
            case 5: { int32_t v; memcpy(&v, b, 4); out->u = (uint64_t)(int64_t)v; out->f = v; } break;
            case 6: { float v; memcpy(&v, b, 4); out->u = (uint64_t)v; out->f = v; } break;
            case 7: out->u = b[0]; out->f = b[0]; break;
            case 10: { uint64_t v; memcpy(&v, b, 8); out->u = v; out->f = (double)v; } break;
            case 11: { int64_t v; memcpy(&v, b, 8); out->u = (uint64_t)v; out->f = (double)v; } break;
            case 12: { double v; memcpy(&v, b, 8); out->u = (uint64_t)v; out->f = v; } break;
        }
    }
    return 1;
}
/* ggml-quants.c dequantize_row_{q8_0,q4_0,q4_K} (the reference's ggml submodule, not vendored: restated from the
 * published block layouts).  Weight files of every converter dtype (convert_tts_to_gguf.py:276-335) load as if they
 * were the F16 file: quantised and 2-D+ F32 matrices become owned F16 copies, exactly as the product reader does. */
static size_t gtype_bytes(int type, int64_t n) {
    switch (type) {
        case 0: return (size_t)n * 4;
        case 1: return (size_t)n * 2;
        case 8: return n % 32 ? 0 : (size_t)(n / 32) * 34;
        case 2: return n % 32 ? 0 : (size_t)(n / 32) * 18;
        case 12: return n % 256 ? 0 : (size_t)(n / 256) * 144;
        default: return 0;
    }
}
static float rd_h(const uint8_t *p) { uint16_t h; memcpy(&h, p, 2); return q3o_f16_to_f32(h); }
static void dequant_row(int type, const uint8_t *b, float *y, int64_t n) {
    if (type == 0) { memcpy(y, b, (size_t)n * 4); return; }
    if (type == 8) {
        for (int64_t k = 0; k < n / 32; ++k, b += 34) {
            const float d = rd_h(b);
            for (int j = 0; j < 32; ++j) y[k * 32 + j] = d * (float)(int8_t)b[2 + j];
        }
    } else if (type == 2) {
        for (int64_t k = 0; k < n / 32; ++k, b += 18) {
            const float d = rd_h(b);
            for (int j = 0; j < 16; ++j) {
                y[k * 32 + j] = (float)((b[2 + j] & 15) - 8) * d;
                y[k * 32 + j + 16] = (float)((b[2 + j] >> 4) - 8) * d;
            }
        }
    } else if (type == 12) {
        for (int64_t k = 0; k < n / 256; ++k, b += 144) {
            const float d = rd_h(b), dmin = rd_h(b + 2);
            const uint8_t *sc = b + 4, *q = b + 16;
            float *o = y + k * 256;
            for (int is = 0; is < 8; is += 2, q += 32) {
                int s[2], m[2];
                for (int u = 0; u < 2; ++u) {
                    const int j = is + u;
                    if (j < 4) { s[u] = sc[j] & 63; m[u] = sc[j + 4] & 63; }
                    else { s[u] = (sc[j + 4] & 15) | ((sc[j - 4] >> 6) << 4); m[u] = (sc[j + 4] >> 4) | ((sc[j] >> 6) << 4); }
                }
                for (int l = 0; l < 32; ++l) *o++ = d * s[0] * (q[l] & 15) - dmin * m[0];
                for (int l = 0; l < 32; ++l) *o++ = d * s[1] * (q[l] >> 4) - dmin * m[1];
            }
        }
    }
}

static void gguf_close(gguf_t *g) {
    if (!g) return;
    for (int64_t i = 0; i < g->nt; ++i) { free(g->t[i].name); free(g->t[i].own); }
    for (int64_t i = 0; i < g->nkv; ++i) free(g->kv[i].key);
    free(g->t); free(g->kv);
    if (g->map) munmap(g->map, g->size);
    free(g);
}
static gguf_t *gguf_open(const char *path) {
    int fd = open(path, O_RDONLY);
    if (fd < 0) { snprintf(g_err, sizeof g_err, "cannot open %s", path); return NULL; }
    struct stat st; fstat(fd, &st);
    gguf_t *g = calloc(1, sizeof *g);
    g->size = (size_t)st.st_size;
    g->map = mmap(NULL, g->size, PROT_READ, MAP_PRIVATE, fd, 0);
    close(fd);
    if (g->map == MAP_FAILED) { g->map = NULL; gguf_close(g); snprintf(g_err, sizeof g_err, "mmap failed"); return NULL; }
    const uint8_t *p = g->map, *end = g->map + g->size;
    uint32_t ver; uint64_t alignment = 32;
    if (g->size < 24 || memcmp(p, "GGUF", 4) != 0) { gguf_close(g); snprintf(g_err, sizeof g_err, "bad magic"); return NULL; }
    p += 4; rd(&p, end, &ver, 4);
    rd(&p, end, &g->nt, 8); rd(&p, end, &g->nkv, 8);
    g->kv = calloc((size_t)g->nkv + 1, sizeof(gkv));
    for (int64_t i = 0; i < g->nkv; ++i) {
        uint32_t type;
        g->kv[i].key = rd_str(&p, end);
        if (!g->kv[i].key || !rd(&p, end, &type, 4)) { gguf_close(g); snprintf(g_err, sizeof g_err, "bad kv"); return NULL; }
        g->kv[i].type = (int)type;
        if (!skip_val(&p, end, type, &g->kv[i])) { gguf_close(g); snprintf(g_err, sizeof g_err, "bad kv value"); return NULL; }
        if (strcmp(g->kv[i].key, "general.alignment") == 0) alignment = g->kv[i].u;
    }
    g->t = calloc((size_t)g->nt + 1, sizeof(gtensor));
    for (int64_t i = 0; i < g->nt; ++i) {
        uint32_t nd = 0, type = 0;
        g->t[i].name = rd_str(&p, end);
        if (!g->t[i].name || !rd(&p, end, &nd, 4) || nd > 4) { gguf_close(g); snprintf(g_err, sizeof g_err, "bad tensor info"); return NULL; }
        g->t[i].nd = (int)nd;
        for (int d = 0; d < 4; ++d) g->t[i].ne[d] = 1;
        for (uint32_t d = 0; d < nd; ++d) rd(&p, end, &g->t[i].ne[d], 8);
        rd(&p, end, &type, 4); g->t[i].type = (int)type;
        rd(&p, end, &g->t[i].off, 8);
    }
    uint64_t pos = (uint64_t)(p - g->map);
    g->data_off = (pos + alignment - 1) / alignment * alignment;
    for (int64_t i = 0; i < g->nt; ++i) {
        gtensor *t = &g->t[i];
        t->src_type = t->type;
        const int64_t n = t->ne[0] * t->ne[1] * t->ne[2] * t->ne[3], row = t->ne[0];
        const size_t rb = gtype_bytes(t->type, row);
        if (t->type == 1 || (t->type == 0 && t->nd == 1) || rb == 0) continue;
        if (g->data_off + t->off + gtype_bytes(t->type, n) > g->size) continue;
        t->own = malloc(sizeof(uint16_t) * (size_t)n);
        float *f = malloc(sizeof(float) * (size_t)row);
        const uint8_t *src = g->map + g->data_off + t->off;
        for (int64_t r = 0; r < n / row; ++r) {
            dequant_row(t->type, src + (size_t)r * rb, f, row);
            for (int64_t c = 0; c < row; ++c) t->own[(size_t)r * row + c] = q3o_f32_to_f16(f[c]);
        }
        free(f);
        t->type = 1;
    }
    return g;
}
static const gtensor *gfind(const gguf_t *g, const char *name) {
    for (int64_t i = 0; i < g->nt; ++i) if (strcmp(g->t[i].name, name) == 0) return &g->t[i];
    return NULL;
}
static int kv_u32(const gguf_t *g, const char *const *keys, int def) {
    for (int k = 0; keys[k]; ++k)
        for (int64_t i = 0; i < g->nkv; ++i)
            if (strcmp(g->kv[i].key, keys[k]) == 0) return (int)g->kv[i].u;
    return def;
}
static float kv_f32(const gguf_t *g, const char *const *keys, float def) {
    for (int k = 0; keys[k]; ++k)
        for (int64_t i = 0; i < g->nkv; ++i)
            if (strcmp(g->kv[i].key, keys[k]) == 0) return (float)g->kv[i].f;
    return def;
}

/* ------------------------------------------------------------------ model */
typedef struct { const uint16_t *w; int rows, cols; } mat16;   /* row-major [rows][cols] f16 (ggml ne=[cols,rows]) */
typedef struct {
    const float *attn_norm, *ffn_norm, *q_norm, *k_norm;
    mat16 q, k, v, o, gate, up, down;
} layer_t;
typedef struct { const uint16_t *w; const float *b; int oc, ic, k; } conv_t;   /* w [oc][ic][k] */
typedef struct { const uint16_t *w; const float *b; int ic, oc, k; } convT_t;  /* w [ic][oc][k] */
typedef struct { const float *alpha, *beta; int n; } snake_t;
typedef struct { const float *attn_norm, *attn_scale, *ffn_norm, *ffn_scale; mat16 q, k, v, o, gate, up, down; } vlayer_t;
typedef struct { convT_t up; conv_t dw; const float *norm_w, *norm_b, *gamma; mat16 pw1, pw2; const float *pw1_b, *pw2_b; } upblk_t;
typedef struct { snake_t a1, a2; conv_t c1, c2; int dil; } resunit_t;
typedef struct { snake_t snake; convT_t ct; resunit_t res[3]; int rate; } decblk_t;

struct q3o_model {
    q3o_config c;
    int round;
    gguf_t *gt, *gk;
    mat16 text_embd, fc1, fc2, codec_embd, codec_head;
    const float *fc1_b, *fc2_b, *out_norm, *cp_out_norm;
    layer_t *L, *CP;
    q3o_config cpc;          /* the code predictor's layer geometry (hidden / inter / heads of the CP) */
    mat16 mtp;               /* 1.7B: code_pred.mtp_proj [cp_hidden][hidden] (+ bias, optional) */
    const float *mtp_b;
    mat16 cp_embd[15], cp_head[15];
    /* vocoder */
    const uint16_t *cb_first, *cb_rest[15];
    uint16_t *cb_norm[16];   /* owned usage-normalised codebooks (NULL: the file's bytes are used) */
    mat16 vq_first_out, vq_rest_out;
    conv_t pre_conv, dec0, dec6;
    mat16 in_proj, out_proj;
    const float *in_proj_b, *out_proj_b, *pre_norm;
    vlayer_t *VL;
    upblk_t up[2];
    decblk_t dec[4];
    snake_t dec5;
    /* speaker encoder (ECAPA-TDNN), audio_tokenizer_encoder.h:29-83 */
    int has_spk;
    conv_t spk_conv0, spk_mfa, spk_asp_tdnn, spk_asp_conv, spk_fc;
    struct { conv_t tdnn1, tdnn2, res[7], se1, se2; } spk_blk[3];
};

static const void *tdata(const gguf_t *g, const gtensor *t) { return t->own ? (const void *)t->own : g->map + g->data_off + t->off; }

static int get_mat(const gguf_t *g, const char *name, int rows, int cols, mat16 *out) {
    const gtensor *t = gfind(g, name);
    if (!t) FAIL("missing tensor %s", name);
    if (t->type != 1) FAIL("tensor %s: expected F16 (type %d)", name, t->type);
    const int ok2 = (t->ne[0] == cols && t->ne[1] * t->ne[2] == rows) || (t->ne[0] == 1 && t->ne[1] == cols && t->ne[2] == rows);
    if (!ok2) FAIL("tensor %s: shape [%lld,%lld] != [%d,%d]", name,
        (long long)t->ne[0], (long long)t->ne[1], cols, rows);
    out->w = tdata(g, t); out->rows = rows; out->cols = cols; return 1;
}
static const float *get_vec(const gguf_t *g, const char *name, int n) {
    const gtensor *t = gfind(g, name);
    if (!t) { snprintf(g_err, sizeof g_err, "missing tensor %s", name); return NULL; }
    if (t->type != 0 || t->ne[0] * t->ne[1] * t->ne[2] != n) { snprintf(g_err, sizeof g_err, "tensor %s: bad f32 vec", name); return NULL; }
    return tdata(g, t);
}
#define GV(dst, g, name, n) do { if (!((dst) = get_vec(g, name, n))) return 0; } while (0)

static int load_layer(const gguf_t *g, const char *pfx, int i, const q3o_config *c, layer_t *l) {
    char b[128];
    const int H = c->hidden, Dq = c->n_heads * c->head_dim, Dkv = c->n_kv * c->head_dim;
#define N(s) (snprintf(b, sizeof b, "%s.blk.%d.%s", pfx, i, s), b)
    GV(l->attn_norm, g, N("attn_norm.weight"), H);
    GV(l->ffn_norm, g, N("ffn_norm.weight"), H);
    GV(l->q_norm, g, N("attn_q_norm.weight"), c->head_dim);
    GV(l->k_norm, g, N("attn_k_norm.weight"), c->head_dim);
    if (!get_mat(g, N("attn_q.weight"), Dq, H, &l->q)) return 0;
    if (!get_mat(g, N("attn_k.weight"), Dkv, H, &l->k)) return 0;
    if (!get_mat(g, N("attn_v.weight"), Dkv, H, &l->v)) return 0;
    if (!get_mat(g, N("attn_output.weight"), H, Dq, &l->o)) return 0;
    if (!get_mat(g, N("ffn_gate.weight"), c->inter, H, &l->gate)) return 0;
    if (!get_mat(g, N("ffn_up.weight"), c->inter, H, &l->up)) return 0;
    if (!get_mat(g, N("ffn_down.weight"), H, c->inter, &l->down)) return 0;
#undef N
    return 1;
}

static int get_conv(const gguf_t *g, const char *wname, const char *bname, conv_t *cv) {
    const gtensor *t = gfind(g, wname);
    if (!t || t->type != 1 || t->nd != 3) FAIL("bad conv %s", wname);
    cv->k = (int)t->ne[0]; cv->ic = (int)t->ne[1]; cv->oc = (int)t->ne[2]; cv->w = tdata(g, t);
    cv->b = bname ? get_vec(g, bname, cv->oc) : NULL;
    if (bname && !cv->b) return 0;
    return 1;
}
static int get_convT(const gguf_t *g, const char *wname, const char *bname, convT_t *cv) {
    const gtensor *t = gfind(g, wname);
    if (!t || t->type != 1 || t->nd != 3) FAIL("bad convT %s", wname);
    cv->k = (int)t->ne[0]; cv->oc = (int)t->ne[1]; cv->ic = (int)t->ne[2]; cv->w = tdata(g, t);
    cv->b = get_vec(g, bname, cv->oc);
    return cv->b != NULL;
}
static int get_snake(const gguf_t *g, const char *pa, const char *pb, int n, snake_t *s) {
    s->n = n;
    GV(s->alpha, g, pa, n); GV(s->beta, g, pb, n);
    return 1;
}

static int load_vocoder(q3o_model *m) {
    const gguf_t *g = m->gk;
    q3o_config *c = &m->c;
    char b[128], b2[128];
    const gtensor *t = gfind(g, "tok_dec.vq_first.0.codebook");
    if (!t || t->type != 1) FAIL("missing vq_first codebook");
    c->cb_dim = (int)t->ne[0]; c->cb_size = (int)t->ne[1];
    m->cb_first = tdata(g, t);
    for (int i = 0; i < 15; ++i) {
        snprintf(b, sizeof b, "tok_dec.vq_rest.%d.codebook", i);
        const gtensor *tr = gfind(g, b);
        if (!tr || tr->ne[0] != c->cb_dim || tr->ne[1] != c->cb_size) FAIL("bad %s", b);
        m->cb_rest[i] = tdata(g, tr);
    }
    /* normalize_codebooks (audio_tokenizer_decoder.cpp:40-73): a codebook whose *.usage tensor is present is divided
     * row by row by max(usage, 1e-5) (1/u multiplied, re-rounded to f16); converter output has no usage tensors */
    for (int i = 0; i < 16; ++i) {
        if (i == 0) snprintf(b, sizeof b, "tok_dec.vq_first.0.usage");
        else snprintf(b, sizeof b, "tok_dec.vq_rest.%d.usage", i - 1);
        const gtensor *ut = gfind(g, b);
        if (!ut) continue;
        if (ut->type != 0 || ut->ne[0] * ut->ne[1] != c->cb_size) FAIL("bad %s", b);
        const float *u = tdata(g, ut);
        const uint16_t *src = i == 0 ? m->cb_first : m->cb_rest[i - 1];
        uint16_t *dst = malloc((size_t)c->cb_size * c->cb_dim * 2);
        for (int r = 0; r < c->cb_size; ++r) {
            float uu = u[r];
            if (uu < 1e-5f) uu = 1e-5f;
            const float inv = 1.0f / uu;
            for (int d = 0; d < c->cb_dim; ++d)
                dst[(size_t)r * c->cb_dim + d] = q3o_f32_to_f16(q3o_f16_to_f32(src[(size_t)r * c->cb_dim + d]) * inv);
        }
        m->cb_norm[i] = dst;
        if (i == 0) m->cb_first = dst; else m->cb_rest[i - 1] = dst;
    }
    const gtensor *op = gfind(g, "tok_dec.vq_first.output_proj.weight");
    if (!op) FAIL("missing vq_first.output_proj");
    c->voc_hidden = (int)op->ne[2];
    if (!get_mat(g, "tok_dec.vq_first.output_proj.weight", c->voc_hidden, c->cb_dim, &m->vq_first_out)) return 0;
    if (!get_mat(g, "tok_dec.vq_rest.output_proj.weight", c->voc_hidden, c->cb_dim, &m->vq_rest_out)) return 0;
    if (!get_conv(g, "tok_dec.pre_conv.weight", "tok_dec.pre_conv.bias", &m->pre_conv)) return 0;
    c->voc_latent = m->pre_conv.oc;
    const char *hk[] = {"qwen3-tts-tokenizer.decoder.num_heads", NULL};
    c->voc_heads = kv_u32(g, hk, 16);
    if (!get_mat(g, "tok_dec.pre_tfm.input_proj.weight", c->voc_hidden, c->voc_latent, &m->in_proj)) return 0;
    GV(m->in_proj_b, g, "tok_dec.pre_tfm.input_proj.bias", c->voc_hidden);
    int nl = 0;
    while (1) { snprintf(b, sizeof b, "tok_dec.pre_tfm.blk.%d.attn_q.weight", nl); if (!gfind(g, b)) break; ++nl; }
    c->voc_layers = nl;
    snprintf(b, sizeof b, "tok_dec.pre_tfm.blk.0.ffn_gate.weight");
    const gtensor *fg = gfind(g, b);
    if (!fg) FAIL("missing pre_tfm ffn");
    c->voc_ffn = (int)fg->ne[1];
    m->VL = calloc((size_t)nl, sizeof(vlayer_t));
    for (int i = 0; i < nl; ++i) {
        vlayer_t *l = &m->VL[i];
        const int VH = c->voc_hidden, LAT = c->voc_latent;
#define N(s) (snprintf(b, sizeof b, "tok_dec.pre_tfm.blk.%d.%s", i, s), b)
        GV(l->attn_norm, g, N("attn_norm.weight"), VH);
        GV(l->attn_scale, g, N("attn_scale"), VH);
        GV(l->ffn_norm, g, N("ffn_norm.weight"), VH);
        GV(l->ffn_scale, g, N("ffn_scale"), VH);
        if (!get_mat(g, N("attn_q.weight"), LAT, VH, &l->q)) return 0;
        if (!get_mat(g, N("attn_k.weight"), LAT, VH, &l->k)) return 0;
        if (!get_mat(g, N("attn_v.weight"), LAT, VH, &l->v)) return 0;
        if (!get_mat(g, N("attn_output.weight"), VH, LAT, &l->o)) return 0;
        if (!get_mat(g, N("ffn_gate.weight"), c->voc_ffn, VH, &l->gate)) return 0;
        if (!get_mat(g, N("ffn_up.weight"), c->voc_ffn, VH, &l->up)) return 0;
        if (!get_mat(g, N("ffn_down.weight"), VH, c->voc_ffn, &l->down)) return 0;
#undef N
    }
    GV(m->pre_norm, g, "tok_dec.pre_tfm.norm.weight", c->voc_hidden);
    if (!get_mat(g, "tok_dec.pre_tfm.output_proj.weight", c->voc_latent, c->voc_hidden, &m->out_proj)) return 0;
    GV(m->out_proj_b, g, "tok_dec.pre_tfm.output_proj.bias", c->voc_latent);
    for (int u = 0; u < 2; ++u) {
        upblk_t *ub = &m->up[u];
#define N(s) (snprintf(b, sizeof b, "tok_dec.upsample.%d.%s", u, s), b)
#define N2(s) (snprintf(b2, sizeof b2, "tok_dec.upsample.%d.%s", u, s), b2)
        if (!get_convT(g, N("conv.weight"), N2("conv.bias"), &ub->up)) return 0;
        if (!get_conv(g, N("dwconv.weight"), N2("dwconv.bias"), &ub->dw)) return 0;
        const int C = ub->up.oc;
        GV(ub->norm_w, g, N("norm.weight"), C);
        GV(ub->norm_b, g, N("norm.bias"), C);
        GV(ub->gamma, g, N("gamma"), C);
        const gtensor *p1 = gfind(g, N("pwconv1.weight"));
        if (!p1) FAIL("missing pwconv1");
        const int F4 = (int)p1->ne[1];
        if (!get_mat(g, N("pwconv1.weight"), F4, C, &ub->pw1)) return 0;
        GV(ub->pw1_b, g, N("pwconv1.bias"), F4);
        if (!get_mat(g, N("pwconv2.weight"), C, F4, &ub->pw2)) return 0;
        GV(ub->pw2_b, g, N("pwconv2.bias"), C);
#undef N
#undef N2
    }
    c->up_k = m->up[0].up.k;
    if (!get_conv(g, "tok_dec.dec.0.conv.weight", "tok_dec.dec.0.conv.bias", &m->dec0)) return 0;
    c->dec_dim = m->dec0.oc;
    const int rates[4] = {8, 5, 4, 3};   /* hard-coded in the reference, audio_tokenizer_decoder.cpp:766 */
    int ch = c->dec_dim;
    for (int d = 0; d < 4; ++d) {
        decblk_t *db = &m->dec[d];
        db->rate = rates[d]; c->rates[d] = rates[d];
#define N(s) (snprintf(b, sizeof b, "tok_dec.dec.%d.%s", d + 1, s), b)
#define N2(s) (snprintf(b2, sizeof b2, "tok_dec.dec.%d.%s", d + 1, s), b2)
        if (!get_snake(g, N("snake.alpha"), N2("snake.beta"), ch, &db->snake)) return 0;
        if (!get_convT(g, N("conv_t.weight"), N2("conv_t.bias"), &db->ct)) return 0;
        c->conv_t_k[d] = db->ct.k;
        const int oc = db->ct.oc;
        for (int r = 0; r < 3; ++r) {
            resunit_t *ru = &db->res[r];
            char n1[128], n2[128];
            ru->dil = r == 0 ? 1 : r == 1 ? 3 : 9;   /* audio_tokenizer_decoder.cpp:324-328 */
            snprintf(n1, sizeof n1, "tok_dec.dec.%d.res.%d.act1.alpha", d + 1, r + 2);
            snprintf(n2, sizeof n2, "tok_dec.dec.%d.res.%d.act1.beta", d + 1, r + 2);
            if (!get_snake(g, n1, n2, oc, &ru->a1)) return 0;
            snprintf(n1, sizeof n1, "tok_dec.dec.%d.res.%d.act2.alpha", d + 1, r + 2);
            snprintf(n2, sizeof n2, "tok_dec.dec.%d.res.%d.act2.beta", d + 1, r + 2);
            if (!get_snake(g, n1, n2, oc, &ru->a2)) return 0;
            snprintf(n1, sizeof n1, "tok_dec.dec.%d.res.%d.conv1.weight", d + 1, r + 2);
            snprintf(n2, sizeof n2, "tok_dec.dec.%d.res.%d.conv1.bias", d + 1, r + 2);
            if (!get_conv(g, n1, n2, &ru->c1)) return 0;
            snprintf(n1, sizeof n1, "tok_dec.dec.%d.res.%d.conv2.weight", d + 1, r + 2);
            snprintf(n2, sizeof n2, "tok_dec.dec.%d.res.%d.conv2.bias", d + 1, r + 2);
            if (!get_conv(g, n1, n2, &ru->c2)) return 0;
        }
#undef N
#undef N2
        ch = oc;
    }
    if (!get_snake(g, "tok_dec.dec.5.snake.alpha", "tok_dec.dec.5.snake.beta", ch, &m->dec5)) return 0;
    if (!get_conv(g, "tok_dec.dec.6.conv.weight", "tok_dec.dec.6.conv.bias", &m->dec6)) return 0;
    c->has_vocoder = 1;
    return 1;
}

/* parse_config key aliases and defaults: src/tts_transformer.cpp:288-442 */
static void parse_config(const gguf_t *g, q3o_config *c) {
#define K(...) ((const char *const[]){__VA_ARGS__, NULL})
    c->text_vocab = kv_u32(g, K("qwen3-tts.text.vocab_size", "qwen3-tts.text_vocab_size"), 151936);
    c->text_dim = kv_u32(g, K("qwen3-tts.text.embedding_dim", "qwen3-tts.text_hidden_size"), 2048);
    c->hidden = kv_u32(g, K("qwen3-tts.talker.embedding_length", "qwen3-tts.embedding_length"), 1024);
    c->n_layers = kv_u32(g, K("qwen3-tts.talker.block_count", "qwen3-tts.block_count"), 28);
    c->n_heads = kv_u32(g, K("qwen3-tts.talker.attention.head_count", "qwen3-tts.attention.head_count"), 16);
    c->n_kv = kv_u32(g, K("qwen3-tts.talker.attention.head_count_kv", "qwen3-tts.attention.head_count_kv"), 8);
    c->inter = kv_u32(g, K("qwen3-tts.talker.feed_forward_length", "qwen3-tts.feed_forward_length"), 3072);
    c->head_dim = kv_u32(g, K("qwen3-tts.talker.attention.key_length", "qwen3-tts.attention.key_length"), 128);
    c->eps = kv_f32(g, K("qwen3-tts.talker.attention.layer_norm_rms_epsilon", "qwen3-tts.attention.layer_norm_rms_epsilon"), 1e-6f);
    c->rope_theta = kv_f32(g, K("qwen3-tts.talker.rope.freq_base", "qwen3-tts.rope.freq_base"), 1000000.0f);
    c->codec_vocab = kv_u32(g, K("qwen3-tts.talker.codec_vocab_size", "qwen3-tts.vocab_size"), 3072);
    c->n_codebooks = kv_u32(g, K("qwen3-tts.talker.num_codebooks", "qwen3-tts.num_code_groups"), 16);
    c->cp_layers = kv_u32(g, K("qwen3-tts.code_pred.layer_count", "qwen3-tts.code_predictor.layer_count"), 5);
    c->cp_vocab = kv_u32(g, K("qwen3-tts.code_pred.vocab_size", "qwen3-tts.code_predictor.vocab_size"), 2048);
    /* code predictor architecture, falling back to the talker's values (0.6B): tts_transformer.cpp:370-389 */
    c->cp_hidden = kv_u32(g, K("qwen3-tts.code_predictor.embedding_length"), c->hidden);
    c->cp_inter = kv_u32(g, K("qwen3-tts.code_predictor.feed_forward_length"), c->inter);
    c->cp_heads = kv_u32(g, K("qwen3-tts.code_predictor.attention.head_count"), c->n_heads);
    c->cp_kv = kv_u32(g, K("qwen3-tts.code_predictor.attention.head_count_kv"), c->n_kv);
    c->cp_head_dim = kv_u32(g, K("qwen3-tts.code_predictor.attention.key_length"), c->head_dim);
    c->codec_pad = kv_u32(g, K("qwen3-tts.codec.pad_id"), 2148);
    c->codec_bos = kv_u32(g, K("qwen3-tts.codec.bos_id"), 2149);
    c->codec_eos = kv_u32(g, K("qwen3-tts.codec.eos_id", "qwen3-tts.codec.eos_token_id"), 2150);
    c->tts_bos = kv_u32(g, K("qwen3-tts.tts_bos_token_id", "qwen3-tts.tts.bos_token_id", "qwen3-tts.tts.bos_id"), 151672);
    c->tts_eos = kv_u32(g, K("qwen3-tts.tts_eos_token_id", "qwen3-tts.tts.eos_token_id", "qwen3-tts.tts.eos_id"), 151673);
    c->tts_pad = kv_u32(g, K("qwen3-tts.tts_pad_token_id", "qwen3-tts.tts.pad_token_id", "qwen3-tts.tts.pad_id"), 151671);
    c->think = kv_u32(g, K("qwen3-tts.codec.think_id", "qwen3-tts.codec_think_id"), 2154);
    c->nothink = kv_u32(g, K("qwen3-tts.codec.nothink_id", "qwen3-tts.codec_nothink_id"), 2155);
    c->think_bos = kv_u32(g, K("qwen3-tts.codec.think_bos_id", "qwen3-tts.codec_think_bos_id"), 2156);
    c->think_eos = kv_u32(g, K("qwen3-tts.codec.think_eos_id", "qwen3-tts.codec_think_eos_id"), 2157);
#undef K
}

void q3o_free(q3o_model *m) {
    if (!m) return;
    free(m->L); free(m->CP); free(m->VL);
    for (int i = 0; i < 16; ++i) free(m->cb_norm[i]);
    gguf_close(m->gt); gguf_close(m->gk);
    free(m);
}

static float *conv1d(const q3o_model *m, const conv_t *cv, const float *x, int T, int pad, int dil, int depthwise, int *Tout);

/* ------------------------------------------------------------------ speaker encoder (audio_tokenizer_encoder.cpp) */
/* tensor names: AudioTokenizerEncoder::load_model (:185-241); conv weights ne [K, IC, OC] F16, biases F32 */
static int load_speaker_encoder(q3o_model *m) {
    const gguf_t *g = m->gt;
    char w[96], b[96];
#define SPK(cv, nm) do { snprintf(w, sizeof w, "spk_enc.%s.weight", nm); snprintf(b, sizeof b, "spk_enc.%s.bias", nm); \
                         if (!get_conv(g, w, b, &(cv))) return 0; } while (0)
    SPK(m->spk_conv0, "conv0");
    SPK(m->spk_mfa, "mfa");
    SPK(m->spk_asp_tdnn, "asp.tdnn");
    SPK(m->spk_asp_conv, "asp.conv");
    SPK(m->spk_fc, "fc");
    for (int i = 0; i < 3; ++i) {
        char nm[64];
        snprintf(nm, sizeof nm, "blk.%d.tdnn1", i + 1); SPK(m->spk_blk[i].tdnn1, nm);
        snprintf(nm, sizeof nm, "blk.%d.tdnn2", i + 1); SPK(m->spk_blk[i].tdnn2, nm);
        snprintf(nm, sizeof nm, "blk.%d.se.conv1", i + 1); SPK(m->spk_blk[i].se1, nm);
        snprintf(nm, sizeof nm, "blk.%d.se.conv2", i + 1); SPK(m->spk_blk[i].se2, nm);
        for (int r = 0; r < 7; ++r) { snprintf(nm, sizeof nm, "blk.%d.res2net.%d", i + 1, r); SPK(m->spk_blk[i].res[r], nm); }
    }
#undef SPK
    if (m->spk_conv0.ic != 128 || m->spk_conv0.oc != 512 || m->spk_mfa.ic != 1536 || m->spk_fc.ic != 3072)
        FAIL("speaker encoder: unexpected shapes");
    m->has_spk = 1;
    return 1;
}

/* librosa slaney mel filterbank (compute_mel_filterbank_slaney, :16-94), [n_mels][n_bins] */
static void spk_filterbank(float *fb, int n_mels, int n_fft, int sr, float f_min, float f_max) {
    const float f_sp = 200.0f / 3.0f, min_log_hz = 1000.0f, min_log_mel = (min_log_hz - 0.0f) / f_sp;
    const float logstep = logf(6.4f) / 27.0f;
#define HZ2MEL(hz) ((hz) < min_log_hz ? ((hz) - 0.0f) / f_sp : min_log_mel + logf((hz) / min_log_hz) / logstep)
#define MEL2HZ(mel) ((mel) < min_log_mel ? 0.0f + f_sp * (mel) : min_log_hz * expf(logstep * ((mel) - min_log_mel)))
    const float mel_min = HZ2MEL(f_min), mel_max = HZ2MEL(f_max);
    const int nb = n_fft / 2 + 1;
    float *hz = malloc(sizeof(float) * (size_t)(n_mels + 2));
    for (int i = 0; i < n_mels + 2; ++i) {
        const float mp = mel_min + (mel_max - mel_min) * i / (n_mels + 1);
        hz[i] = MEL2HZ(mp);
    }
#undef HZ2MEL
#undef MEL2HZ
    memset(fb, 0, sizeof(float) * (size_t)n_mels * nb);
    for (int mm = 0; mm < n_mels; ++mm) {
        const float fl = hz[mm], fc = hz[mm + 1], fr = hz[mm + 2], enorm = 2.0f / (fr - fl);
        for (int k = 0; k < nb; ++k) {
            const float freq = (float)k * sr / n_fft;
            if (freq >= fl && freq <= fc) { if (fc > fl) fb[(size_t)mm * nb + k] = enorm * (freq - fl) / (fc - fl); }
            else if (freq > fc && freq <= fr) { if (fr > fc) fb[(size_t)mm * nb + k] = enorm * (fr - freq) / (fr - fc); }
        }
    }
    free(hz);
}

/* compute_mel_spectrogram (:281-364): reflect pad (n_fft-hop)/2, Hann window, DFT magnitude sqrt(re^2+im^2+1e-9),
 * slaney mel, log(max(x, 1e-5)) -> mel [128][F] (channel-major).  The DFT's cos/sin terms are the reference's own
 * expressions (float angle = -2*M_PI*k*t/n), tabulated once; sums in the reference's order. */
int q3o_mel(const q3o_model *m, const float *samples, int n, float *mel, int *n_frames) {
    (void)m;
    const int NFFT = 1024, HOP = 256, WIN = 1024, NM = 128, SR = 24000, NB = NFFT / 2 + 1;
    const int pad = (NFFT - HOP) / 2, plen = n + 2 * pad;
    const int F = (plen - NFFT) / HOP + 1;
    if (n < 2 || F <= 0) FAIL("Audio too short for mel spectrogram");
    *n_frames = F;
    if (!mel) return 1;
    float *padded = malloc(sizeof(float) * (size_t)plen);
    for (int i = 0; i < plen; ++i) {
        int src = i < pad ? pad - i : i >= pad + n ? 2 * n - (i - pad) - 2 : i - pad;
        src = src < 0 ? 0 : src > n - 1 ? n - 1 : src;
        padded[i] = samples[src];
    }
    float *fb = malloc(sizeof(float) * (size_t)NM * NB), *win = calloc(NFFT, sizeof(float));
    spk_filterbank(fb, NM, NFFT, SR, 0.0f, 12000.0f);
    const int off = (NFFT - WIN) / 2;
    for (int i = 0; i < WIN; ++i) win[off + i] = 0.5f * (1.0f - cosf(2.0f * M_PI * i / WIN));
    float *ct = malloc(sizeof(float) * (size_t)NB * NFFT), *st = malloc(sizeof(float) * (size_t)NB * NFFT);
#pragma omp parallel for schedule(static)
    for (int k = 0; k < NB; ++k)
        for (int t = 0; t < NFFT; ++t) {
            const float angle = -2.0f * M_PI * k * t / NFFT;
            ct[(size_t)k * NFFT + t] = cosf(angle);
            st[(size_t)k * NFFT + t] = sinf(angle);
        }
#pragma omp parallel for schedule(dynamic)
    for (int f = 0; f < F; ++f) {
        float frame[1024], mag[513];
        for (int i = 0; i < NFFT; ++i) frame[i] = padded[(size_t)f * HOP + i] * win[i];
        for (int k = 0; k < NB; ++k) {
            float re = 0.0f, im = 0.0f;
            for (int t = 0; t < NFFT; ++t) { re += frame[t] * ct[(size_t)k * NFFT + t]; im += frame[t] * st[(size_t)k * NFFT + t]; }
            mag[k] = sqrtf(re * re + im * im + 1e-9f);
        }
        for (int mm = 0; mm < NM; ++mm) {
            float sum = 0.0f;
            for (int k = 0; k < NB; ++k) sum += fb[(size_t)mm * NB + k] * mag[k];
            mel[(size_t)mm * F + f] = logf(sum > 1e-5f ? sum : 1e-5f);
        }
    }
    free(padded); free(fb); free(win); free(ct); free(st);
    return 1;
}

/* apply_reflect_pad_1d (:366-408) of [C][T] then a "valid" conv (ggml_conv_1d, F16 im2col) + bias */
static float *spk_conv(const q3o_model *m, const conv_t *cv, const float *x, int T, int pad, int dil) {
    const int C = cv->ic, Tp = T + 2 * pad;
    float *xp = malloc(sizeof(float) * (size_t)C * Tp);
    for (int c = 0; c < C; ++c)
        for (int i = 0; i < Tp; ++i) {
            const int t = i < pad ? pad - i : i >= pad + T ? T - 2 - (i - pad - T) : i - pad;
            xp[(size_t)c * Tp + i] = x[(size_t)c * T + t];
        }
    int To;
    float *y = conv1d(m, cv, xp, Tp, 0, dil, 0, &To);
    free(xp);
    return y;   /* [oc][T] */
}
static void relu_(float *x, size_t n) { for (size_t i = 0; i < n; ++i) x[i] = x[i] > 0.0f ? x[i] : 0.0f; }
/* ggml_pool_1d AVG over the whole time axis (f32 sum / T) [ggml-upstream] */
static float mean_t(const float *x, int T) { float s = 0.0f; for (int t = 0; t < T; ++t) s += x[t]; return s / (float)T; }

/* AudioTokenizerEncoder::encode (:696-750) with build_graph (:438-694): conv0 (k5, reflect 2) + ReLU; 3 SE-Res2Net
 * blocks (dilations 2,3,4: tdnn1 + ReLU, 8 branches of 64 (branch b>=2 adds the previous branch output) through k3
 * dilated convs + ReLU, tdnn2 + ReLU, SE (mean -> conv1 + ReLU -> conv2 + sigmoid -> scale), + residual); MFA
 * (concat blocks 1..3, 1x1 1536 + ReLU); ASP (global mean/std, tdnn 4608->128 + ReLU + tanh, conv 128->1536, softmax
 * over time, weighted mean/std); FC 3072 -> E */
int q3o_speaker_encode(const q3o_model *m, const float *samples, int n, float *emb) {
    if (!m->has_spk) FAIL("No speaker encoder tensors found in model");
    int T;
    if (!q3o_mel(m, samples, n, NULL, &T)) return 0;
    float *mel = malloc(sizeof(float) * (size_t)128 * T);
    q3o_mel(m, samples, n, mel, &T);
    float *cur = spk_conv(m, &m->spk_conv0, mel, T, 2, 1);
    free(mel);
    relu_(cur, (size_t)512 * T);
    float *outs[3];
    const int dils[3] = {2, 3, 4};
    for (int blk = 0; blk < 3; ++blk) {
        const int dl = dils[blk];
        float *h = spk_conv(m, &m->spk_blk[blk].tdnn1, cur, T, 0, 1);
        relu_(h, (size_t)512 * T);
        float *cat = malloc(sizeof(float) * (size_t)512 * T);
        memcpy(cat, h, sizeof(float) * (size_t)64 * T);   /* branch 0: identity */
        float *prev = NULL, *in = malloc(sizeof(float) * (size_t)64 * T);
        for (int b = 1; b < 8; ++b) {
            for (size_t i = 0; i < (size_t)64 * T; ++i) in[i] = h[(size_t)b * 64 * T + i] + (b >= 2 ? prev[i] : 0.0f);
            float *o = spk_conv(m, &m->spk_blk[blk].res[b - 1], in, T, dl, dl);
            relu_(o, (size_t)64 * T);
            memcpy(cat + (size_t)b * 64 * T, o, sizeof(float) * (size_t)64 * T);
            free(prev);
            prev = o;
        }
        free(prev); free(in); free(h);
        float *y = spk_conv(m, &m->spk_blk[blk].tdnn2, cat, T, 0, 1);
        free(cat);
        relu_(y, (size_t)512 * T);
        float se_in[512], se_mid[128], se_out[512];
        for (int c = 0; c < 512; ++c) se_in[c] = mean_t(y + (size_t)c * T, T);
        float *s1 = spk_conv(m, &m->spk_blk[blk].se1, se_in, 1, 0, 1);
        for (int c = 0; c < 128; ++c) se_mid[c] = s1[c] > 0.0f ? s1[c] : 0.0f;
        free(s1);
        float *s2 = spk_conv(m, &m->spk_blk[blk].se2, se_mid, 1, 0, 1);
        for (int c = 0; c < 512; ++c) se_out[c] = 1.0f / (1.0f + expf(-s2[c]));
        free(s2);
        for (int c = 0; c < 512; ++c)
            for (int t = 0; t < T; ++t) y[(size_t)c * T + t] = y[(size_t)c * T + t] * se_out[c] + cur[(size_t)c * T + t];
        if (blk > 0) outs[blk - 1] = cur;
        else free(cur);
        cur = y;
    }
    outs[2] = cur;
    float *mfa_in = malloc(sizeof(float) * (size_t)1536 * T);
    /* block outputs 1, 2, 3 (outs[0..2]) concatenated on channels (:599-600) */
    for (int i = 0; i < 3; ++i) memcpy(mfa_in + (size_t)i * 512 * T, outs[i], sizeof(float) * (size_t)512 * T);
    float *hs = spk_conv(m, &m->spk_mfa, mfa_in, T, 0, 1);
    free(mfa_in); free(outs[0]); free(outs[1]); free(outs[2]);
    relu_(hs, (size_t)1536 * T);
    float *att_in = malloc(sizeof(float) * (size_t)4608 * T);
    memcpy(att_in, hs, sizeof(float) * (size_t)1536 * T);
    for (int c = 0; c < 1536; ++c) {
        const float *xc = hs + (size_t)c * T;
        const float mu = mean_t(xc, T);
        float sq = 0.0f;
        for (int t = 0; t < T; ++t) sq += xc[t] * xc[t];
        float var = sq / (float)T - mu * mu;
        var = var < 1e-12f ? 1e-12f : var > 1e10f ? 1e10f : var;
        const float sd = sqrtf(var);
        for (int t = 0; t < T; ++t) { att_in[(size_t)(1536 + c) * T + t] = mu; att_in[(size_t)(3072 + c) * T + t] = sd; }
    }
    float *a1 = spk_conv(m, &m->spk_asp_tdnn, att_in, T, 0, 1);
    free(att_in);
    for (size_t i = 0; i < (size_t)128 * T; ++i) a1[i] = tanhf(a1[i] > 0.0f ? a1[i] : 0.0f);
    float *a2 = spk_conv(m, &m->spk_asp_conv, a1, T, 0, 1);
    free(a1);
    float pooled[3072];
    for (int c = 0; c < 1536; ++c) {
        float *ac = a2 + (size_t)c * T;
        const float *xc = hs + (size_t)c * T;
        float mx = -INFINITY;
        for (int t = 0; t < T; ++t) mx = ac[t] > mx ? ac[t] : mx;
        double sum = 0.0;   /* ggml_soft_max: f32 exp, ggml_float (double) sum [ggml-upstream] */
        for (int t = 0; t < T; ++t) { ac[t] = expf(ac[t] - mx); sum += ac[t]; }
        const float inv = (float)(1.0 / sum);
        for (int t = 0; t < T; ++t) ac[t] *= inv;
        float wm = 0.0f;
        for (int t = 0; t < T; ++t) wm += ac[t] * xc[t];
        wm = (wm / (float)T) * (float)T;   /* pool AVG then scale by T (:659-661) */
        float wv = 0.0f;
        for (int t = 0; t < T; ++t) { const float d = xc[t] - wm; wv += ac[t] * (d * d); }
        wv = (wv / (float)T) * (float)T;
        wv = wv < 1e-12f ? 1e-12f : wv > 1e10f ? 1e10f : wv;
        pooled[c] = wm;
        pooled[1536 + c] = sqrtf(wv);
    }
    free(a2); free(hs);
    float *e = spk_conv(m, &m->spk_fc, pooled, 1, 0, 1);
    memcpy(emb, e, sizeof(float) * (size_t)m->spk_fc.oc);
    free(e);
    return 1;
}
int q3o_speaker_dim(const q3o_model *m) { return m->has_spk ? m->spk_fc.oc : 0; }

q3o_model *q3o_load(const char *tts_gguf, const char *tok_gguf, int ggml_rounding) {
    q3o_model *m = calloc(1, sizeof *m);
    m->round = ggml_rounding;
    m->gt = gguf_open(tts_gguf);
    if (!m->gt) { q3o_free(m); return NULL; }
    q3o_config *c = &m->c;
    parse_config(m->gt, c);
    const gguf_t *g = m->gt;
    const int H = c->hidden;
    int ok = get_mat(g, "talker.text_embd.weight", c->text_vocab, c->text_dim, &m->text_embd) &&
             get_mat(g, "talker.text_proj.fc1.weight", c->text_dim, c->text_dim, &m->fc1) &&
             get_mat(g, "talker.text_proj.fc2.weight", H, c->text_dim, &m->fc2) &&
             get_mat(g, "talker.codec_embd.weight", c->codec_vocab, H, &m->codec_embd) &&
             get_mat(g, "talker.codec_head.weight", c->codec_vocab, H, &m->codec_head) &&
             (m->fc1_b = get_vec(g, "talker.text_proj.fc1.bias", c->text_dim)) &&
             (m->fc2_b = get_vec(g, "talker.text_proj.fc2.bias", H)) &&
             (m->out_norm = get_vec(g, "talker.output_norm.weight", H)) &&
             (m->cp_out_norm = get_vec(g, "code_pred.output_norm.weight", c->cp_hidden));
    if (!ok) { q3o_free(m); return NULL; }
    m->cpc = *c;
    m->cpc.hidden = c->cp_hidden; m->cpc.inter = c->cp_inter; m->cpc.n_heads = c->cp_heads;
    m->cpc.n_kv = c->cp_kv; m->cpc.head_dim = c->cp_head_dim;
    /* code_pred.mtp_proj (1.7B, tts_transformer.cpp:611-616, 709-712): applied to every code-predictor input */
    c->has_mtp = gfind(g, "code_pred.mtp_proj.weight") != NULL;
    if (c->has_mtp) {
        if (!get_mat(g, "code_pred.mtp_proj.weight", c->cp_hidden, H, &m->mtp)) { q3o_free(m); return NULL; }
        m->mtp_b = gfind(g, "code_pred.mtp_proj.bias") ? get_vec(g, "code_pred.mtp_proj.bias", c->cp_hidden) : NULL;
        if (gfind(g, "code_pred.mtp_proj.bias") && !m->mtp_b) { q3o_free(m); return NULL; }
    } else if (c->cp_hidden != H) {
        snprintf(g_err, sizeof g_err, "code predictor hidden %d != talker hidden %d without code_pred.mtp_proj", c->cp_hidden, H);
        q3o_free(m); return NULL;
    }
    m->L = calloc((size_t)c->n_layers, sizeof(layer_t));
    m->CP = calloc((size_t)c->cp_layers, sizeof(layer_t));
    for (int i = 0; i < c->n_layers; ++i) if (!load_layer(g, "talker", i, c, &m->L[i])) { q3o_free(m); return NULL; }
    for (int i = 0; i < c->cp_layers; ++i) if (!load_layer(g, "code_pred", i, &m->cpc, &m->CP[i])) { q3o_free(m); return NULL; }
    for (int i = 0; i < c->n_codebooks - 1 && i < 15; ++i) {
        char b[96];
        snprintf(b, sizeof b, "code_pred.codec_embd.%d.weight", i);
        if (!get_mat(g, b, c->cp_vocab, H, &m->cp_embd[i])) { q3o_free(m); return NULL; }
        snprintf(b, sizeof b, "code_pred.lm_head.%d.weight", i);
        if (!get_mat(g, b, c->cp_vocab, c->cp_hidden, &m->cp_head[i])) { q3o_free(m); return NULL; }
    }
    if (tok_gguf && tok_gguf[0]) {
        m->gk = gguf_open(tok_gguf);
        if (!m->gk || !load_vocoder(m)) { q3o_free(m); return NULL; }
    }
    if (gfind(g, "spk_enc.conv0.weight") && !load_speaker_encoder(m)) { q3o_free(m); return NULL; }
    return m;
}

void q3o_get_config(const q3o_model *m, q3o_config *c) { *c = m->c; }

/* ------------------------------------------------------------------ primitive ops */
/* activation rounding at a matmul input (ggml mul_mat converts src1 to vec_dot_type F16) */
static void round_in(const q3o_model *m, const float *x, float *xr, int n) {
    if (m->round) for (int i = 0; i < n; ++i) xr[i] = f16r(x[i]);
    else memcpy(xr, x, sizeof(float) * (size_t)n);
}

static inline float dot_f16_f32(const uint16_t *w, const float *x, int n) {
#ifdef Q3O_SIMD
    __m256 a0 = _mm256_setzero_ps(), a1 = a0, a2 = a0, a3 = a0;
    int i = 0;
    for (; i + 32 <= n; i += 32) {
        a0 = _mm256_fmadd_ps(_mm256_cvtph_ps(_mm_loadu_si128((const __m128i *)(w + i))), _mm256_loadu_ps(x + i), a0);
        a1 = _mm256_fmadd_ps(_mm256_cvtph_ps(_mm_loadu_si128((const __m128i *)(w + i + 8))), _mm256_loadu_ps(x + i + 8), a1);
        a2 = _mm256_fmadd_ps(_mm256_cvtph_ps(_mm_loadu_si128((const __m128i *)(w + i + 16))), _mm256_loadu_ps(x + i + 16), a2);
        a3 = _mm256_fmadd_ps(_mm256_cvtph_ps(_mm_loadu_si128((const __m128i *)(w + i + 24))), _mm256_loadu_ps(x + i + 24), a3);
    }
    a0 = _mm256_add_ps(_mm256_add_ps(a0, a1), _mm256_add_ps(a2, a3));
    __m128 s = _mm_add_ps(_mm256_castps256_ps128(a0), _mm256_extractf128_ps(a0, 1));
    s = _mm_hadd_ps(s, s); s = _mm_hadd_ps(s, s);
    float r = _mm_cvtss_f32(s);
    for (; i < n; ++i) r += q3o_f16_to_f32(w[i]) * x[i];
    return r;
#else
    float r = 0.f;
    for (int i = 0; i < n; ++i) r += q3o_f16_to_f32(w[i]) * x[i];
    return r;
#endif
}

/* y[rows] = W · round(x)  (ggml_mul_mat, F16 weights) */
static void mul_mat_vec(const q3o_model *m, const mat16 *W, const float *x, float *y) {
    float *xr = malloc(sizeof(float) * (size_t)W->cols);
    round_in(m, x, xr, W->cols);
#pragma omp parallel for schedule(static)
    for (int r = 0; r < W->rows; ++r) y[r] = dot_f16_f32(W->w + (size_t)r * W->cols, xr, W->cols);
    free(xr);
}
static inline float dot_f32(const float *a, const float *b, int n);
/* Y[t][rows] = W · round(X[t])  for T columns (row-major X [T][cols]).  Several columns: each weight row is widened
 * to f32 once (exact) and dotted with every column by dot_f32, which sums in dot_f16_f32's order (bit-identical) */
static void mul_mat_rows(const q3o_model *m, const mat16 *W, const float *X, int T, float *Y) {
    float *xr = malloc(sizeof(float) * (size_t)W->cols * (size_t)T);
    round_in(m, X, xr, W->cols * T);
    if (T < 4) {
#pragma omp parallel for schedule(static)
        for (int r = 0; r < W->rows; ++r)
            for (int t = 0; t < T; ++t) Y[(size_t)t * W->rows + r] = dot_f16_f32(W->w + (size_t)r * W->cols, xr + (size_t)t * W->cols, W->cols);
    } else {
#pragma omp parallel
        {
            float *wr = malloc(sizeof(float) * (size_t)W->cols);
#pragma omp for schedule(static)
            for (int r = 0; r < W->rows; ++r) {
                const uint16_t *w = W->w + (size_t)r * W->cols;
                for (int c = 0; c < W->cols; ++c) wr[c] = q3o_f16_to_f32(w[c]);
                for (int t = 0; t < T; ++t) Y[(size_t)t * W->rows + r] = dot_f32(wr, xr + (size_t)t * W->cols, W->cols);
            }
            free(wr);
        }
    }
    free(xr);
}

/* ggml_rms_norm (sum in ggml_float=double) followed by ggml_mul with the weight */
static void rms_norm_w(const float *x, const float *w, float *y, int n, float eps) {
    double sum = 0.0;
    for (int i = 0; i < n; ++i) sum += (double)(x[i] * x[i]);
    const float mean = (float)(sum / n);
    const float scale = 1.0f / sqrtf(mean + eps);
    for (int i = 0; i < n; ++i) y[i] = (x[i] * scale) * (w ? w[i] : 1.0f);
}
/* ggml_norm (layer norm without affine) then * w + b */
static void layer_norm_wb(const float *x, const float *w, const float *b, float *y, int n, float eps) {
    double sum = 0.0;
    for (int i = 0; i < n; ++i) sum += (double)x[i];
    const float mean = (float)(sum / n);
    double sum2 = 0.0;
    for (int i = 0; i < n; ++i) { float v = x[i] - mean; y[i] = v; sum2 += (double)(v * v); }
    const float variance = (float)(sum2 / n);
    const float scale = 1.0f / sqrtf(variance + eps);
    for (int i = 0; i < n; ++i) y[i] = y[i] * scale * w[i] + b[i];
}
static inline float silu_f(float x) { return x / (1.0f + expf(-x)); }
/* ggml_vec_gelu_f32 with GGML_GELU_FP16 (f16 lookup of the tanh approximation) [ggml-upstream] */
static inline float gelu_ggml(float x) {
    if (x <= -10.0f) return 0.0f;
    if (x >= 10.0f) return x;
    const float v = f16r(x);
    const float g = 0.5f * v * (1.0f + tanhf(0.79788456080286535587989211986876f * v * (1.0f + 0.044715f * v * v)));
    return f16r(g);
}

/* ggml_rope_cache_init + rope_yarn with ext_factor 0, attn_factor 1 (theta *= theta_scale iteratively) */
void q3o_rope_cache(float p, int dims, float freq_base, float *cache) {
    const float theta_scale = powf(freq_base, -2.0f / (float)dims);
    float theta = p;
    for (int i0 = 0; i0 < dims; i0 += 2) {
        cache[i0 + 0] = cosf(theta);
        cache[i0 + 1] = sinf(theta);
        theta *= theta_scale;
    }
}
/* GGML_ROPE_TYPE_NEOX on one head: pairs (i, i + D/2) */
static void rope_neox(float *x, int D, const float *cache) {
    const int h = D / 2;
    for (int i = 0; i < h; ++i) {
        const float c = cache[2 * i], s = cache[2 * i + 1];
        const float x0 = x[i], x1 = x[i + h];
        x[i] = x0 * c - x1 * s;
        x[i + h] = x0 * s + x1 * c;
    }
}

/* ------------------------------------------------------------------ KV cache */
struct q3o_kv { int n_layers, n_ctx, n_kv, D; float *k, *v; };   /* [layer][pos][kv_head][D] (ggml layout) */

q3o_kv *q3o_kv_new(const q3o_model *m, int n_ctx, int which) {
    q3o_kv *kv = calloc(1, sizeof *kv);
    const q3o_config *c = which == 0 ? &m->c : &m->cpc;
    kv->n_layers = which == 0 ? m->c.n_layers : m->c.cp_layers;
    kv->n_ctx = n_ctx; kv->n_kv = c->n_kv; kv->D = c->head_dim;
    const size_t n = (size_t)kv->n_layers * n_ctx * kv->n_kv * kv->D;
    kv->k = calloc(n, sizeof(float)); kv->v = calloc(n, sizeof(float));
    return kv;
}
void q3o_kv_free(q3o_kv *kv) { if (kv) { free(kv->k); free(kv->v); free(kv); } }

/* ------------------------------------------------------------------ one Qwen3 decoder layer, one token
 * tts_transformer.cpp:1410-1494 (talker step) == :1721-1811 (CP step).  Attention of the step graph is
 * ggml_flash_attn_ext (Q->f16, K/V f16 from the cache, f32 online softmax); restated with f32 accumulation. */
static void decoder_layer_block(const q3o_model *m, const q3o_config *c, const layer_t *l, q3o_kv *kv, int il, float *x,
                                int pos0, int T);

/* f32 dot product, 4 x 8-lane accumulators combined in a fixed order (n % 8 == 0 lanes vectorised, tail scalar) */
static inline float dot_f32(const float *a, const float *b, int n) {
#ifdef Q3O_SIMD
    __m256 a0 = _mm256_setzero_ps(), a1 = a0, a2 = a0, a3 = a0;
    int i = 0;
    for (; i + 32 <= n; i += 32) {
        a0 = _mm256_fmadd_ps(_mm256_loadu_ps(a + i), _mm256_loadu_ps(b + i), a0);
        a1 = _mm256_fmadd_ps(_mm256_loadu_ps(a + i + 8), _mm256_loadu_ps(b + i + 8), a1);
        a2 = _mm256_fmadd_ps(_mm256_loadu_ps(a + i + 16), _mm256_loadu_ps(b + i + 16), a2);
        a3 = _mm256_fmadd_ps(_mm256_loadu_ps(a + i + 24), _mm256_loadu_ps(b + i + 24), a3);
    }
    a0 = _mm256_add_ps(_mm256_add_ps(a0, a1), _mm256_add_ps(a2, a3));
    __m128 s = _mm_add_ps(_mm256_castps256_ps128(a0), _mm256_extractf128_ps(a0, 1));
    s = _mm_hadd_ps(s, s); s = _mm_hadd_ps(s, s);
    float r = _mm_cvtss_f32(s);
    for (; i < n; ++i) r += a[i] * b[i];
    return r;
#else
    float r = 0.f;
    for (int i = 0; i < n; ++i) r += a[i] * b[i];
    return r;
#endif
}

/* ggml_flash_attn_ext of one token (q [nH][D], at position pos) over the cached rows 0..pos of layer il: f16-rounded
 * Q, f32 scores and online-softmax sums (double), f32 V accumulation -> att [nH][D].  `par`: heads in parallel. */
static void attend(const q3o_model *m, const q3o_config *c, const q3o_kv *kv, int il, const float *q, int pos, float *att,
                   int par) {
    const int D = c->head_dim, nH = c->n_heads, nKV = c->n_kv, rep = nH / nKV;
    const float *kc = kv->k + (size_t)il * kv->n_ctx * nKV * D, *vc = kv->v + (size_t)il * kv->n_ctx * nKV * D;
    const float scale = 1.0f / sqrtf((float)D);
    float *sc_all = malloc(sizeof(float) * (size_t)(pos + 1) * nH);
#pragma omp parallel for schedule(static) if (par)
    for (int h = 0; h < nH; ++h) {
        const int hk = h / rep;
        float *sc = sc_all + (size_t)h * (pos + 1);
        float qr[512];
        for (int d = 0; d < D; ++d) qr[d] = m->round ? f16r(q[h * D + d]) : q[h * D + d];
        float mx = -INFINITY;
        for (int j = 0; j <= pos; ++j) {
            sc[j] = dot_f32(kc + ((size_t)j * nKV + hk) * D, qr, D) * scale;
            if (sc[j] > mx) mx = sc[j];
        }
        double sum = 0.0;
        for (int j = 0; j <= pos; ++j) { sc[j] = expf(sc[j] - mx); sum += sc[j]; }
        float *o = att + h * D;
        for (int d = 0; d < D; ++d) o[d] = 0.f;
        for (int j = 0; j <= pos; ++j) {
            const float *vr = vc + ((size_t)j * nKV + hk) * D;
            for (int d = 0; d < D; ++d) o[d] += sc[j] * vr[d];
        }
        const float inv = (float)(1.0 / sum);
        for (int d = 0; d < D; ++d) o[d] *= inv;
    }
    free(sc_all);
}

/* head RMSNorms + NEOX RoPE of one token's raw q/k, then its K/V rows written to the cache (ggml_cpy -> F16) */
static void qk_norm_rope_store(const q3o_model *m, const q3o_config *c, const layer_t *l, q3o_kv *kv, int il, float *q,
                               float *k, const float *v, int pos) {
    const int D = c->head_dim, nH = c->n_heads, nKV = c->n_kv;
    float cache[512];
    q3o_rope_cache((float)pos, D, c->rope_theta, cache);
    for (int h = 0; h < nH; ++h) { rms_norm_w(q + h * D, l->q_norm, q + h * D, D, c->eps); rope_neox(q + h * D, D, cache); }
    for (int h = 0; h < nKV; ++h) { rms_norm_w(k + h * D, l->k_norm, k + h * D, D, c->eps); rope_neox(k + h * D, D, cache); }
    float *kc = kv->k + (size_t)il * kv->n_ctx * nKV * D, *vc = kv->v + (size_t)il * kv->n_ctx * nKV * D;
    for (int i = 0; i < nKV * D; ++i) {
        kc[(size_t)pos * nKV * D + i] = m->round ? f16r(k[i]) : k[i];
        vc[(size_t)pos * nKV * D + i] = m->round ? f16r(v[i]) : v[i];
    }
}

/* ------------------------------------------------------------------ one Qwen3 decoder layer, one token
 * tts_transformer.cpp:1410-1494 (talker step) == :1721-1811 (CP step).  Attention of the step graph is
 * ggml_flash_attn_ext (Q->f16, K/V f16 from the cache, f32 online softmax); restated with f32 accumulation. */
static void decoder_layer(const q3o_model *m, const q3o_config *c, const layer_t *l, q3o_kv *kv, int il, float *x, int pos) {
    decoder_layer_block(m, c, l, kv, il, x, pos, 1);
}

/* the same layer over T consecutive tokens at positions pos0..pos0+T-1 (x [T][H] in place): every weight row is read
 * once per block and reused by the T tokens, each token computed exactly as decoder_layer computes it alone (the
 * teacher-forced replay of q3o_generate_forced_from uses it for the frames it does not trace) */
static void decoder_layer_block(const q3o_model *m, const q3o_config *c, const layer_t *l, q3o_kv *kv, int il, float *x,
                                int pos0, int T) {
    const int H = c->hidden, D = c->head_dim, nH = c->n_heads, nKV = c->n_kv, I = c->inter;
    float *xn = malloc(sizeof(float) * (size_t)T * (H > I ? H : I));
    float *q = malloc(sizeof(float) * (size_t)T * nH * D), *k = malloc(sizeof(float) * (size_t)T * nKV * D);
    float *v = malloc(sizeof(float) * (size_t)T * nKV * D), *att = malloc(sizeof(float) * (size_t)T * nH * D);
    float *y = malloc(sizeof(float) * (size_t)T * H);
    float *g = malloc(sizeof(float) * (size_t)T * I), *u = malloc(sizeof(float) * (size_t)T * I);
    for (int t = 0; t < T; ++t) rms_norm_w(x + (size_t)t * H, l->attn_norm, xn + (size_t)t * H, H, c->eps);
    mul_mat_rows(m, &l->q, xn, T, q);
    mul_mat_rows(m, &l->k, xn, T, k);
    mul_mat_rows(m, &l->v, xn, T, v);
    for (int t = 0; t < T; ++t)
        qk_norm_rope_store(m, c, l, kv, il, q + (size_t)t * nH * D, k + (size_t)t * nKV * D, v + (size_t)t * nKV * D, pos0 + t);
    if (T == 1) {
        attend(m, c, kv, il, q, pos0, att, 1);
    } else {
#pragma omp parallel for schedule(dynamic)
        for (int t = 0; t < T; ++t) attend(m, c, kv, il, q + (size_t)t * nH * D, pos0 + t, att + (size_t)t * nH * D, 0);
    }
    mul_mat_rows(m, &l->o, att, T, y);
    for (size_t i = 0; i < (size_t)T * H; ++i) x[i] += y[i];
    for (int t = 0; t < T; ++t) rms_norm_w(x + (size_t)t * H, l->ffn_norm, xn + (size_t)t * H, H, c->eps);
    mul_mat_rows(m, &l->gate, xn, T, g);
    mul_mat_rows(m, &l->up, xn, T, u);
    for (size_t i = 0; i < (size_t)T * I; ++i) g[i] = silu_f(g[i]) * u[i];
    mul_mat_rows(m, &l->down, g, T, y);
    for (size_t i = 0; i < (size_t)T * H; ++i) x[i] += y[i];
    free(g); free(u); free(y); free(xn); free(q); free(k); free(v); free(att);
}

int q3o_talker_step_n(const q3o_model *m, q3o_kv *kv, const float *embd, int pos, int n_layers, float *hidden, float *logits) {
    const q3o_config *c = &m->c;
    if (pos < 0 || pos >= kv->n_ctx) FAIL("Context length exceeded");
    if (n_layers <= 0 || n_layers > c->n_layers) n_layers = c->n_layers;
    float *x = malloc(sizeof(float) * (size_t)c->hidden);
    memcpy(x, embd, sizeof(float) * (size_t)c->hidden);
    for (int il = 0; il < n_layers; ++il) decoder_layer(m, c, &m->L[il], kv, il, x, pos);
    rms_norm_w(x, m->out_norm, hidden, c->hidden, c->eps);                  /* :1498-1499 */
    if (logits) mul_mat_vec(m, &m->codec_head, hidden, logits);             /* :1503 */
    free(x);
    return 1;
}
int q3o_talker_step(const q3o_model *m, q3o_kv *kv, const float *embd, int pos, float *hidden, float *logits) {
    return q3o_talker_step_n(m, kv, embd, pos, 0, hidden, logits);
}

/* text_embd row gather -> fc1 + b -> SiLU -> fc2 + b (tts_transformer.cpp:1050-1055) */
int q3o_project_text(const q3o_model *m, const int32_t *toks, int n, float *out) {
    const q3o_config *c = &m->c;
    const int E = c->text_dim, H = c->hidden;
    float *rows = malloc(sizeof(float) * (size_t)E * n), *h1 = malloc(sizeof(float) * (size_t)E * n);
    for (int t = 0; t < n; ++t) {
        if (toks[t] < 0 || toks[t] >= c->text_vocab) { free(rows); free(h1); FAIL("text token out of range"); }
        const uint16_t *r = m->text_embd.w + (size_t)toks[t] * E;
        for (int i = 0; i < E; ++i) rows[(size_t)t * E + i] = q3o_f16_to_f32(r[i]);
    }
    mul_mat_rows(m, &m->fc1, rows, n, h1);
    for (int t = 0; t < n; ++t) for (int i = 0; i < E; ++i) h1[(size_t)t * E + i] = silu_f(h1[(size_t)t * E + i] + m->fc1_b[i]);
    mul_mat_rows(m, &m->fc2, h1, n, out);
    for (int t = 0; t < n; ++t) for (int i = 0; i < H; ++i) out[(size_t)t * H + i] += m->fc2_b[i];
    free(rows); free(h1);
    return 1;
}

static void embd_row(const mat16 *tab, int id, float *out) {
    const uint16_t *r = tab->w + (size_t)id * tab->cols;
    for (int i = 0; i < tab->cols; ++i) out[i] = q3o_f16_to_f32(r[i]);
}

/* build_prefill_graph: tts_transformer.cpp:1093-1231 */
int q3o_prefill_embd(const q3o_model *m, const int32_t *toks, int n, const float *spk, int language_id,
                     float *prefill, int *prefill_len, float *trailing, int *trailing_len, float *tts_pad) {
    const q3o_config *c = &m->c;
    const int H = c->hidden;
    if (n < 4) FAIL("Need at least 4 text tokens for prefill");
    int32_t special[3] = {c->tts_bos, c->tts_eos, c->tts_pad};
    float *sp = malloc(sizeof(float) * 3 * (size_t)H), *role = malloc(sizeof(float) * 3 * (size_t)H);
    float *first = malloc(sizeof(float) * (size_t)H), *row = malloc(sizeof(float) * (size_t)H);
    if (!q3o_project_text(m, special, 3, sp) || !q3o_project_text(m, toks, 3, role) || !q3o_project_text(m, toks + 3, 1, first)) {
        free(sp); free(role); free(first); free(row); return 0;
    }
    const float *tts_bos = sp, *tts_eos = sp + H;
    memcpy(tts_pad, sp + 2 * H, sizeof(float) * (size_t)H);
    int codec_pre[4], n_pre;
    if (language_id < 0) { codec_pre[0] = c->nothink; codec_pre[1] = c->think_bos; codec_pre[2] = c->think_eos; n_pre = 3; }
    else { codec_pre[0] = c->think; codec_pre[1] = c->think_bos; codec_pre[2] = language_id; codec_pre[3] = c->think_eos; n_pre = 4; }
    const int has_spk = spk != NULL;
    const int codec_input_len = n_pre + has_spk + 2;
    float *cin = malloc(sizeof(float) * (size_t)codec_input_len * H);
    int dst = 0;
    for (int i = 0; i < n_pre; ++i) embd_row(&m->codec_embd, codec_pre[i], cin + (size_t)(dst++) * H);
    if (has_spk) memcpy(cin + (size_t)(dst++) * H, spk, sizeof(float) * (size_t)H);
    embd_row(&m->codec_embd, c->codec_pad, cin + (size_t)(dst++) * H);
    embd_row(&m->codec_embd, c->codec_bos, cin + (size_t)(dst++) * H);
    const int overlay_len = codec_input_len - 1;
    const int plen = 3 + overlay_len + 1;
    memcpy(prefill, role, sizeof(float) * 3 * (size_t)H);
    for (int t = 0; t < overlay_len; ++t) {
        const float *ov = (t == overlay_len - 1) ? tts_bos : tts_pad;
        for (int h = 0; h < H; ++h) prefill[(size_t)(3 + t) * H + h] = ov[h] + cin[(size_t)t * H + h];
    }
    const float *bos = cin + (size_t)(codec_input_len - 1) * H;
    for (int h = 0; h < H; ++h) prefill[(size_t)(plen - 1) * H + h] = first[h] + bos[h];
    *prefill_len = plen;
    const int trailing_count = n - 9 > 0 ? n - 9 : 0;
    if (trailing_count > 0 && !q3o_project_text(m, toks + 4, trailing_count, trailing)) { free(sp); free(role); free(first); free(row); free(cin); return 0; }
    memcpy(trailing + (size_t)trailing_count * H, tts_eos, sizeof(float) * (size_t)H);
    *trailing_len = trailing_count + 1;
    free(sp); free(role); free(first); free(row); free(cin);
    return 1;
}

/* ------------------------------------------------------------------ code predictor */
/* xin: the pass input in talker space [hidden]; with code_pred.mtp_proj (1.7B) it is projected first,
 * x = mtp_proj . f16(xin) + bias (ggml_mul_mat + ggml_add, tts_transformer.cpp:1554-1560 / :1709-1714) */
int q3o_cp_pass(const q3o_model *m, q3o_kv *kv, const float *xin, int pos, int head, float *hidden_out, float *logits) {
    const q3o_config *c = &m->cpc;
    float *x = malloc(sizeof(float) * (size_t)c->hidden), *hn = malloc(sizeof(float) * (size_t)c->hidden);
    if (m->c.has_mtp) {
        mul_mat_vec(m, &m->mtp, xin, x);
        if (m->mtp_b) for (int i = 0; i < c->hidden; ++i) x[i] += m->mtp_b[i];
    } else {
        memcpy(x, xin, sizeof(float) * (size_t)c->hidden);
    }
    for (int il = 0; il < c->cp_layers; ++il) decoder_layer(m, c, &m->CP[il], kv, il, x, pos);
    rms_norm_w(x, m->cp_out_norm, hn, c->hidden, c->eps);                  /* :1815-1816 */
    if (hidden_out) memcpy(hidden_out, hn, sizeof(float) * (size_t)c->hidden);
    if (head >= 0 && logits) mul_mat_vec(m, &m->cp_head[head], hn, logits); /* :1818 */
    free(x); free(hn);
    return 1;
}

static int argmax_first(const float *x, int n) {   /* tts_transformer.cpp:2051-2061 */
    int mi = 0; float mv = x[0];
    for (int i = 1; i < n; ++i) if (x[i] > mv) { mv = x[i]; mi = i; }
    return mi;
}

/* k-th largest value (nth_element / partial_sort threshold) */
static float kth_largest(const float *x, int n, int k) {
    float *tmp = malloc(sizeof(float) * (size_t)n);
    memcpy(tmp, x, sizeof(float) * (size_t)n);
    /* quickselect for the k-th largest */
    int lo = 0, hi = n - 1, want = k - 1;
    while (lo < hi) {
        float piv = tmp[(lo + hi) / 2];
        int i = lo, j = hi;
        while (i <= j) {
            while (tmp[i] > piv) ++i;
            while (tmp[j] < piv) --j;
            if (i <= j) { float t = tmp[i]; tmp[i] = tmp[j]; tmp[j] = t; ++i; --j; }
        }
        if (want <= j) hi = j; else if (want >= i) lo = i; else break;
    }
    float r = tmp[want];
    free(tmp);
    return r;
}

/* temperature -> top-k threshold (< thr => -inf, ties survive) -> softmax -> inverse CDF with u.
 * Shared restatement of the sampling in tts_transformer.cpp:2450-2495 (CB0) / :2198-2236 (CP) and the GPU
 * sampler trt_cuda_kernels.cu:91-183: every variant keeps {x : x >= k-th largest}.  The draw itself is
 * deterministic here (u supplied), not std::mt19937 as in the reference. */
int q3o_sample(const float *logits_in, int n, float temperature, int top_k, float u, int keep_id) {
    if (temperature <= 0.0f) return argmax_first(logits_in, n);
    float *l = malloc(sizeof(float) * (size_t)n);
    for (int i = 0; i < n; ++i) l[i] = logits_in[i] / temperature;
    const float keep_v = keep_id >= 0 ? l[keep_id] : 0.f;
    if (top_k > 0 && top_k < n) {
        const float thr = kth_largest(l, n, top_k);
        for (int i = 0; i < n; ++i) if (l[i] < thr) l[i] = -INFINITY;
    }
    if (keep_id >= 0) l[keep_id] = keep_v;
    float mx = -INFINITY;
    for (int i = 0; i < n; ++i) if (l[i] > mx) mx = l[i];
    double total = 0.0;
    for (int i = 0; i < n; ++i) { l[i] = expf(l[i] - mx); total += l[i]; }
    const double target = (double)u * total;
    double cum = 0.0;
    int tok = n - 1;
    for (int i = 0; i < n; ++i) { cum += l[i]; if (cum >= target && l[i] > 0.f) { tok = i; break; } }
    free(l);
    return tok;
}

int q3o_cp_frame(const q3o_model *m, const float *hidden, int cb0, float temperature, int top_k, const float *u15,
                 int32_t *codes, float *logits_all) {
    const q3o_config *c = &m->c;
    const int H = c->hidden, V = c->cp_vocab, nsteps = c->n_codebooks - 1;
    q3o_kv *kv = q3o_kv_new(m, 16, 1);
    float *x = malloc(sizeof(float) * (size_t)H), *lg = malloc(sizeof(float) * (size_t)V);
    /* pass 0: talker hidden at pos 0 (no head); pass 1: codec_embd[cb0] at pos 1 -> lm_head[0]
     * (= the 2-token prefill, tts_transformer.cpp:2243-2288, fed token-by-token as in trt_code_predictor.cpp:552-571) */
    q3o_cp_pass(m, kv, hidden, 0, -1, NULL, NULL);
    embd_row(&m->codec_embd, cb0, x);
    for (int s = 0; s < nsteps; ++s) {
        if (s > 0) embd_row(&m->cp_embd[s - 1], codes[s - 1], x);      /* :2294-2310 */
        q3o_cp_pass(m, kv, x, s + 1, s, NULL, lg);
        if (logits_all) memcpy(logits_all + (size_t)s * V, lg, sizeof(float) * (size_t)V);
        codes[s] = q3o_sample(lg, V, temperature, top_k, u15 ? u15[s] : 0.f, -1);
    }
    free(x); free(lg);
    q3o_kv_free(kv);
    return 1;
}

/* teacher-forced code predictor: passes fed with the given codes, logits of every step recorded */
int q3o_cp_frame_forced(const q3o_model *m, const float *hidden, int cb0, const int32_t *codes15, float *logits_all) {
    const q3o_config *c = &m->c;
    const int H = c->hidden, V = c->cp_vocab;
    q3o_kv *kv = q3o_kv_new(m, 16, 1);
    float *x = malloc(sizeof(float) * (size_t)H), *lg = malloc(sizeof(float) * (size_t)V);
    q3o_cp_pass(m, kv, hidden, 0, -1, NULL, NULL);
    embd_row(&m->codec_embd, cb0, x);
    for (int s = 0; s < c->n_codebooks - 1; ++s) {
        if (s > 0) embd_row(&m->cp_embd[s - 1], codes15[s - 1], x);
        q3o_cp_pass(m, kv, x, s + 1, s, NULL, lg);
        if (logits_all) memcpy(logits_all + (size_t)s * V, lg, sizeof(float) * (size_t)V);
    }
    free(x); free(lg);
    q3o_kv_free(kv);
    return 1;
}

/* CB0 logit processing, tts_transformer.cpp:2417-2495 */
int q3o_cb0_select(const q3o_model *m, float *logits, const uint8_t *seen, int frame, int n_tokens, float rep,
                   float temperature, int top_k, float u, int eos_mask) {
    const q3o_config *c = &m->c;
    const int V = c->codec_vocab, EOS = c->codec_eos;
    for (int i = V - 1024; i < V; ++i) if (i != EOS) logits[i] = -INFINITY;
    if (rep != 1.0f)
        for (int t = 0; t < V; ++t)
            if (seen[t]) logits[t] = logits[t] > 0.0f ? logits[t] / rep : logits[t] * rep;
    const int expected = n_tokens * 4 > 20 ? n_tokens * 4 : 20;
    if (frame >= expected) {
        float ramp = (float)(frame - expected) / (float)expected;
        if (ramp > 1.0f) ramp = 1.0f;
        float mx = logits[0];
        for (int i = 1; i < V; ++i) if (logits[i] > mx) mx = logits[i];
        const float target = mx + 5.0f;
        logits[EOS] += ramp * (target - logits[EOS]);
    }
    if (eos_mask) logits[EOS] = -INFINITY;
    if (temperature <= 0.0f) return argmax_first(logits, V);
    return q3o_sample(logits, V, temperature, top_k, u, eos_mask ? -1 : EOS);
}

static uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
float q3o_uniform(uint64_t seed, uint64_t utt, uint64_t frame, uint64_t cb) {
    const uint64_t h = mix64(mix64(seed ^ (utt * 0xD1B54A32D192ED03ull)) + frame * 16ull + cb);
    return (float)(h >> 40) * (1.0f / 16777216.0f);
}

/* frame loop, tts_transformer.cpp:2342-2574.  forced != NULL: teacher forcing — the codes of each frame are
 * taken from forced[frame][16] (the decisions are still recorded: cb0_trace = processed CB0 logits fed to the
 * selection, cp_trace = [15][Vcp] code-predictor logits of each step). */
static int generate_impl(const q3o_model *m, const int32_t *toks, int n, const float *spk, int max_len, int language_id,
                         float rep, float temperature, int top_k, uint64_t seed, uint64_t utt, int force_frames,
                         const int32_t *forced, int n_forced, int32_t *codes_out, int *n_frames, float *logits_trace,
                         float *hidden_trace, float *cb0_trace, float *cp_trace, int trace_from);
int q3o_generate_forced(const q3o_model *m, const int32_t *toks, int n, const float *spk, int language_id, float rep,
                        int force_frames, const int32_t *forced, int n_forced, float *cb0_trace, float *cp_trace) {
    int nf = 0;
    int32_t *tmp = malloc(sizeof(int32_t) * 16 * (size_t)(n_forced > 0 ? n_forced : 1));
    const int r = generate_impl(m, toks, n, spk, n_forced, language_id, rep, 0.0f, 0, 0, 0, force_frames, forced, n_forced,
                                tmp, &nf, NULL, NULL, cb0_trace, cp_trace, 0);
    free(tmp);
    return r;
}
int q3o_generate_forced_from(const q3o_model *m, const int32_t *toks, int n, const float *spk, int language_id, float rep,
                             int force_frames, const int32_t *forced, int n_forced, int from_frame, float *cb0_trace,
                             float *cp_trace) {
    int nf = 0;
    int32_t *tmp = malloc(sizeof(int32_t) * 16 * (size_t)(n_forced > 0 ? n_forced : 1));
    const int r = generate_impl(m, toks, n, spk, n_forced, language_id, rep, 0.0f, 0, 0, 0, force_frames, forced, n_forced,
                                tmp, &nf, NULL, NULL, cb0_trace, cp_trace, from_frame);
    free(tmp);
    return r;
}
int q3o_generate(const q3o_model *m, const int32_t *toks, int n, const float *spk, int max_len, int language_id,
                 float rep, float temperature, int top_k, uint64_t seed, uint64_t utt, int force_frames,
                 int32_t *codes_out, int *n_frames, float *logits_trace, float *hidden_trace) {
    return generate_impl(m, toks, n, spk, max_len, language_id, rep, temperature, top_k, seed, utt, force_frames, NULL, 0,
                         codes_out, n_frames, logits_trace, hidden_trace, NULL, NULL, 0);
}
static int generate_impl(const q3o_model *m, const int32_t *toks, int n, const float *spk, int max_len, int language_id,
                         float rep, float temperature, int top_k, uint64_t seed, uint64_t utt, int force_frames,
                         const int32_t *forced, int n_forced, int32_t *codes_out, int *n_frames, float *logits_trace,
                         float *hidden_trace, float *cb0_trace, float *cp_trace, int trace_from) {
    const q3o_config *c = &m->c;
    const int H = c->hidden, V = c->codec_vocab, NCB = c->n_codebooks;
    *n_frames = 0;
    if (n < 4) FAIL("Need at least 4 text tokens for generation");
    if (max_len <= 0) return 1;
    float *prefill = malloc(sizeof(float) * 10 * (size_t)H);
    float *trailing = malloc(sizeof(float) * (size_t)(n > 9 ? n - 8 : 1) * H), *pad = malloc(sizeof(float) * (size_t)H);
    int plen, tlen;
    if (!q3o_prefill_embd(m, toks, n, spk, language_id, prefill, &plen, trailing, &tlen, pad)) return 0;
    q3o_kv *kv = q3o_kv_new(m, plen + max_len + 8, 0);
    float *hidden = malloc(sizeof(float) * (size_t)H), *logits = malloc(sizeof(float) * (size_t)V);
    float *e = malloc(sizeof(float) * (size_t)H), *row = malloc(sizeof(float) * (size_t)H);
    for (int t = 0; t < plen; ++t) q3o_talker_step(m, kv, prefill + (size_t)t * H, t, hidden, logits);
    uint8_t *seen = calloc((size_t)V, 1);
    int32_t fc[16], u15_i = 0; (void)u15_i;
    float u15[15];
    int n_past = plen, frame0 = 0;
    if (forced && trace_from > 0) {
        /* frames before trace_from: their forced codes only advance the talker, in blocks of up to 64 tokens (each
         * token computed exactly as the one-token step would compute it); hidden / logits of the last one feed frame
         * trace_from's decisions */
        int F0 = trace_from < n_forced ? trace_from : n_forced;
        if (F0 > max_len) F0 = max_len;
        for (int f = 0; f < F0; ++f)
            if (forced[(size_t)f * NCB] == c->codec_eos) { F0 = f; break; }
        const int BLK = 64;
        float *X = malloc(sizeof(float) * (size_t)BLK * H);
        for (int f0 = 0; f0 < F0; f0 += BLK) {
            const int T = F0 - f0 < BLK ? F0 - f0 : BLK;
            for (int t = 0; t < T; ++t) {
                const int f = f0 + t;
                const int32_t *fc_f = forced + (size_t)f * NCB;
                float *xt = X + (size_t)t * H;
                seen[fc_f[0]] = 1;
                memcpy(codes_out + (size_t)f * NCB, fc_f, sizeof(int32_t) * (size_t)NCB);
                embd_row(&m->codec_embd, fc_f[0], xt);
                for (int cb = 1; cb < NCB; ++cb) {
                    embd_row(&m->cp_embd[cb - 1], fc_f[cb], row);
                    for (int h = 0; h < H; ++h) xt[h] += row[h];
                }
                const float *tr = f < tlen ? trailing + (size_t)f * H : pad;
                for (int h = 0; h < H; ++h) xt[h] += tr[h];
            }
            for (int il = 0; il < c->n_layers; ++il) decoder_layer_block(m, c, &m->L[il], kv, il, X, n_past, T);
            n_past += T;
            if (f0 + T == F0) {   /* :1496-1505 on the last token */
                rms_norm_w(X + (size_t)(T - 1) * H, m->out_norm, hidden, H, c->eps);
                mul_mat_vec(m, &m->codec_head, hidden, logits);
            }
        }
        free(X);
        *n_frames = F0;
        frame0 = F0;
    }
    for (int frame = frame0; frame < max_len; ++frame) {
        if (logits_trace) memcpy(logits_trace + (size_t)frame * V, logits, sizeof(float) * (size_t)V);
        if (hidden_trace) memcpy(hidden_trace + (size_t)frame * H, hidden, sizeof(float) * (size_t)H);
        const int mask = force_frames > 0 && frame < force_frames;
        /* teacher-forced replay from trace_from: earlier frames only advance the talker (no selection, no CP) */
        const int traced = frame >= trace_from;
        int tok = 0;
        if (traced) {
            tok = q3o_cb0_select(m, logits, seen, frame, n, rep, temperature, top_k,
                                 q3o_uniform(seed, utt, (uint64_t)frame, 0), mask);
            if (cb0_trace) memcpy(cb0_trace + (size_t)(frame - trace_from) * V, logits, sizeof(float) * (size_t)V);  /* processed */
        }
        if (forced) { if (frame >= n_forced) break; tok = forced[(size_t)frame * NCB]; }
        if (tok == c->codec_eos) break;
        fc[0] = tok;
        seen[tok] = 1;
        for (int s = 0; s < NCB - 1; ++s) u15[s] = q3o_uniform(seed, utt, (uint64_t)frame, (uint64_t)s + 1);
        if (forced) {
            if (traced)
                q3o_cp_frame_forced(m, hidden, tok, forced + (size_t)frame * NCB + 1,
                                    cp_trace ? cp_trace + (size_t)(frame - trace_from) * 15 * c->cp_vocab : NULL);
            for (int s = 0; s < NCB - 1; ++s) fc[s + 1] = forced[(size_t)frame * NCB + s + 1];
        } else {
            q3o_cp_frame(m, hidden, tok, temperature, top_k, u15, fc + 1, NULL);
        }
        memcpy(codes_out + (size_t)frame * NCB, fc, sizeof(int32_t) * (size_t)NCB);
        *n_frames = frame + 1;
        if (frame + 1 >= max_len) break;
        /* step embedding, :2529-2553 */
        embd_row(&m->codec_embd, fc[0], e);
        for (int cb = 1; cb < NCB; ++cb) {
            embd_row(&m->cp_embd[cb - 1], fc[cb], row);
            for (int h = 0; h < H; ++h) e[h] += row[h];
        }
        const float *tr = frame < tlen ? trailing + (size_t)frame * H : pad;
        for (int h = 0; h < H; ++h) e[h] += tr[h];
        q3o_talker_step(m, kv, e, n_past, hidden, logits);
        n_past++;
    }
    free(prefill); free(trailing); free(pad); free(hidden); free(logits); free(e); free(row); free(seen);
    q3o_kv_free(kv);
    return 1;
}

/* ------------------------------------------------------------------ vocoder (audio_tokenizer_decoder.cpp) */
/* data layout [C][T] (ggml ne = [T, C]) */
static void snake_apply(const snake_t *s, const float *x, float *y, int T) {   /* :375-402 */
#pragma omp parallel for schedule(static)
    for (int ch = 0; ch < s->n; ++ch) {
        const float a = expf(s->alpha[ch]), ib = expf(-s->beta[ch]);
        for (int t = 0; t < T; ++t) {
            const float v = x[(size_t)ch * T + t];
            const float sn = sinf(v * a);
            y[(size_t)ch * T + t] = v + (sn * sn) * ib;
        }
    }
}
#define CG_T 16
#ifdef Q3O_SIMD
/* The conv as ggml computes it (im2col to F16, then mul_mat of the F16 kernel [OC][IC*K] with the im2col rows,
 * f32 accumulation: ggml_conv_1d / ggml_conv_transpose_1d, src/audio_tokenizer_decoder.cpp:551-620, 705-790) as a
 * register-blocked GEMM on AVX2/F16C.  The im2col matrix is never materialised: its row j = (ci, tap) is the
 * f16-rounded input row ci shifted by off[tap].  Micro-tile: 6 output channels x 16 time steps (12 ymm accumulators,
 * 2 loads + 6 broadcasts per 12 FMAs), accumulated over (ci, tap) in the order of the scalar loop below, so the
 * result is the scalar restatement's bit for bit.
 *   Y[co][t] (stored at y[co * ldy + t * sy]) = bias[co] + sum_ci sum_tap W(co, ci, tap) * X[ci][t + off[tap]]
 * wt: [ceil(OC/6)][IC][NT][6] f32 weights (rows past OC zero); x already offset to output t = 0. */
#define CG_CO 6
static void conv_gemm(const float *wt, int OC, int IC, int NT, const int *off, const float *x, size_t ldx, int n,
                      const float *bias, float *y, size_t ldy, int sy) {
    const int nct = (OC + CG_CO - 1) / CG_CO, TB = 256, ntb = (n + TB - 1) / TB;
#pragma omp parallel for collapse(2) schedule(static)
    for (int tb = 0; tb < ntb; ++tb)
        for (int ct = 0; ct < nct; ++ct) {
            const float *wc = wt + (size_t)ct * IC * NT * CG_CO;
            const int t1 = (tb + 1) * TB < n ? (tb + 1) * TB : n;
            for (int t = tb * TB; t < t1; t += CG_T) {
                const int tn = t1 - t < CG_T ? t1 - t : CG_T;
                float out[CG_CO][CG_T];
                if (tn == CG_T) {
                    __m256 a[CG_CO][2];
                    for (int c = 0; c < CG_CO; ++c) a[c][0] = a[c][1] = _mm256_setzero_ps();
                    for (int ci = 0; ci < IC; ++ci) {
                        const float *xr = x + (size_t)ci * ldx + t;
                        const float *wp = wc + (size_t)ci * NT * CG_CO;
                        for (int k = 0; k < NT; ++k, wp += CG_CO) {
                            const __m256 b0 = _mm256_loadu_ps(xr + off[k]), b1 = _mm256_loadu_ps(xr + off[k] + 8);
                            for (int c = 0; c < CG_CO; ++c) {
                                const __m256 w = _mm256_broadcast_ss(wp + c);
                                a[c][0] = _mm256_fmadd_ps(w, b0, a[c][0]);
                                a[c][1] = _mm256_fmadd_ps(w, b1, a[c][1]);
                            }
                        }
                    }
                    for (int c = 0; c < CG_CO; ++c) { _mm256_storeu_ps(out[c], a[c][0]); _mm256_storeu_ps(out[c] + 8, a[c][1]); }
                } else {   /* tail: the same order, scalar */
                    for (int c = 0; c < CG_CO; ++c)
                        for (int j = 0; j < tn; ++j) out[c][j] = 0.f;
                    for (int ci = 0; ci < IC; ++ci) {
                        const float *xr = x + (size_t)ci * ldx + t;
                        const float *wp = wc + (size_t)ci * NT * CG_CO;
                        for (int k = 0; k < NT; ++k, wp += CG_CO)
                            for (int c = 0; c < CG_CO; ++c)
                                for (int j = 0; j < tn; ++j) out[c][j] = fmaf(wp[c], xr[off[k] + j], out[c][j]);
                    }
                }
                for (int c = 0; c < CG_CO; ++c) {
                    const int co = ct * CG_CO + c;
                    if (co >= OC) break;
                    const float b = bias ? bias[co] : 0.f;
                    for (int j = 0; j < tn; ++j) y[(size_t)co * ldy + (size_t)(t + j) * sy] = out[c][j] + b;
                }
            }
        }
}
#endif

/* causal conv1d: left pad `pad`, kernel k, dilation d, stride 1 (ggml_pad_ext + ggml_conv_1d/_dw: im2col F16) */
static float *conv1d(const q3o_model *m, const conv_t *cv, const float *x, int T, int pad, int dil, int depthwise, int *Tout) {
    const int Tp = T + pad, To = Tp - dil * (cv->k - 1);
    const int C_in = depthwise ? cv->oc : cv->ic;
    float *xr = calloc((size_t)C_in * Tp + CG_T, sizeof(float));
    for (int ci = 0; ci < C_in; ++ci)
        for (int t = 0; t < T; ++t) { float v = x[(size_t)ci * T + t]; xr[(size_t)ci * Tp + pad + t] = m->round ? f16r(v) : v; }
    float *y = malloc(sizeof(float) * (size_t)cv->oc * To);
#ifdef Q3O_SIMD
    if (!depthwise) {
        const int OC = cv->oc, IC = cv->ic, K = cv->k, nct = (OC + CG_CO - 1) / CG_CO;
        float *wt = calloc((size_t)nct * IC * K * CG_CO, sizeof(float));
        for (int co = 0; co < OC; ++co)
            for (int ci = 0; ci < IC; ++ci)
                for (int k = 0; k < K; ++k)
                    wt[(((size_t)(co / CG_CO) * IC + ci) * K + k) * CG_CO + co % CG_CO] = q3o_f16_to_f32(cv->w[((size_t)co * IC + ci) * K + k]);
        int off[64];
        for (int k = 0; k < K && k < 64; ++k) off[k] = k * dil;
        if (K <= 64) {
            conv_gemm(wt, OC, IC, K, off, xr, (size_t)Tp, To, cv->b, y, (size_t)To, 1);
            free(wt);
            free(xr);
            *Tout = To;
            return y;
        }
        free(wt);
    }
#endif
    const int TB = 512;
#pragma omp parallel for schedule(dynamic)
    for (int co = 0; co < cv->oc; ++co) {
        float acc[512];
        for (int t0 = 0; t0 < To; t0 += TB) {
            const int tn = To - t0 < TB ? To - t0 : TB;
            for (int t = 0; t < tn; ++t) acc[t] = 0.f;
            const int ci0 = depthwise ? co : 0, ci1 = depthwise ? co + 1 : C_in;
            for (int ci = ci0; ci < ci1; ++ci) {
                const uint16_t *wr = cv->w + ((size_t)co * (depthwise ? 1 : cv->ic) + (depthwise ? 0 : ci)) * cv->k;
                const float *xi = xr + (size_t)ci * Tp + t0;
                for (int k = 0; k < cv->k; ++k) {
                    const float w = q3o_f16_to_f32(wr[k]);
                    const float *xs = xi + k * dil;
                    for (int t = 0; t < tn; ++t) acc[t] += w * xs[t];
                }
            }
            for (int t = 0; t < tn; ++t) y[(size_t)co * To + t0 + t] = acc[t] + (cv->b ? cv->b[co] : 0.f);
        }
    }
    free(xr);
    *Tout = To;
    return y;
}
/* ggml_conv_transpose_1d (p0 = 0, d = 1), then [trim] then + bias.  Output length (T-1)*s + K - 2*trim. */
static float *convT1d(const q3o_model *m, const convT_t *cv, const float *x, int T, int s, int trim, int *Tout) {
    const int Tfull = (T - 1) * s + cv->k, To = Tfull - 2 * trim;
    float *xr = malloc(sizeof(float) * (size_t)cv->ic * T);
    for (size_t i = 0; i < (size_t)cv->ic * T; ++i) xr[i] = m->round ? f16r(x[i]) : x[i];
    float *y = malloc(sizeof(float) * (size_t)cv->oc * To);
#ifdef Q3O_SIMD
    /* polyphase: output o' = q*s + r (o' = o + trim into the untrimmed result) takes taps k = r + m*s at input q - m,
     * added in (ic, k) order like the scatter loop below; each phase is a conv_gemm over q with offsets mmax - m
     * into the zero-padded rows */
    if (cv->k <= 64 * s) {
        const int IC = cv->ic, OC = cv->oc, K = cv->k, mmax = (K + s - 1) / s, nct = (OC + CG_CO - 1) / CG_CO;
        const size_t ld = (size_t)T + 2 * mmax + CG_T;
        float *xp = calloc((size_t)IC * ld, sizeof(float));
        for (int ic = 0; ic < IC; ++ic) memcpy(xp + (size_t)ic * ld + mmax, xr + (size_t)ic * T, sizeof(float) * (size_t)T);
        float *wt = malloc(sizeof(float) * (size_t)nct * IC * mmax * CG_CO);
        for (int r = 0; r < s; ++r) {
            const int nt = (K - r + s - 1) / s;   /* taps of this phase */
            if (nt <= 0) continue;
            /* outputs of this phase: o = q*s + r - trim in [0, To) */
            int q0 = (trim - r + s - 1) / s;
            if (q0 < 0) q0 = 0;
            const int o0 = q0 * s + r - trim;
            if (o0 >= To) continue;
            const int n = (To - o0 + s - 1) / s;
            memset(wt, 0, sizeof(float) * (size_t)nct * IC * nt * CG_CO);
            for (int oc = 0; oc < OC; ++oc)
                for (int ic = 0; ic < IC; ++ic)
                    for (int mm = 0; mm < nt; ++mm)
                        wt[(((size_t)(oc / CG_CO) * IC + ic) * nt + mm) * CG_CO + oc % CG_CO] =
                            q3o_f16_to_f32(cv->w[((size_t)ic * OC + oc) * K + r + mm * s]);
            int off[64];
            for (int mm = 0; mm < nt; ++mm) off[mm] = mmax - mm;
            /* input index q - m = (q0 + j) - m -> xp column mmax + q0 + j - m */
            conv_gemm(wt, OC, IC, nt, off, xp + q0, ld, n, cv->b, y + o0, (size_t)To, s);
        }
        free(wt);
        free(xp);
        free(xr);
        *Tout = To;
        return y;
    }
#endif
#pragma omp parallel for schedule(dynamic)
    for (int oc = 0; oc < cv->oc; ++oc) {
        float *full = calloc((size_t)Tfull, sizeof(float));
        for (int ic = 0; ic < cv->ic; ++ic) {
            const uint16_t *wr = cv->w + ((size_t)ic * cv->oc + oc) * cv->k;
            const float *xi = xr + (size_t)ic * T;
            for (int k = 0; k < cv->k; ++k) {
                const float w = q3o_f16_to_f32(wr[k]);
                for (int t = 0; t < T; ++t) full[(size_t)t * s + k] += w * xi[t];
            }
        }
        for (int t = 0; t < To; ++t) y[(size_t)oc * To + t] = full[t + trim] + cv->b[oc];
        free(full);
    }
    free(xr);
    *Tout = To;
    return y;
}
static float *transpose(const float *x, int R, int C) {   /* [R][C] -> [C][R] */
    float *y = malloc(sizeof(float) * (size_t)R * C);
    for (int r = 0; r < R; ++r) for (int c = 0; c < C; ++c) y[(size_t)c * R + r] = x[(size_t)r * C + c];
    return y;
}

/* pre-transformer layer, :412-488. x [F][VH] row-major */
static void voc_tfm_layer(const q3o_model *m, const vlayer_t *l, float *x, int F) {
    const q3o_config *c = &m->c;
    const int VH = c->voc_hidden, LAT = c->voc_latent, nh = c->voc_heads, D = LAT / nh;
    const float eps = 1e-5f;
    float *xn = malloc(sizeof(float) * (size_t)F * VH);
    float *q = malloc(sizeof(float) * (size_t)F * LAT), *k = malloc(sizeof(float) * (size_t)F * LAT), *v = malloc(sizeof(float) * (size_t)F * LAT);
    float *att = calloc((size_t)F * LAT, sizeof(float)), *y = malloc(sizeof(float) * (size_t)F * VH);
    for (int t = 0; t < F; ++t) rms_norm_w(x + (size_t)t * VH, l->attn_norm, xn + (size_t)t * VH, VH, eps);
    mul_mat_rows(m, &l->q, xn, F, q);
    mul_mat_rows(m, &l->k, xn, F, k);
    mul_mat_rows(m, &l->v, xn, F, v);
    float cache[512];
    for (int t = 0; t < F; ++t) {
        q3o_rope_cache((float)t, D, 10000.0f, cache);
        for (int h = 0; h < nh; ++h) { rope_neox(q + (size_t)t * LAT + h * D, D, cache); rope_neox(k + (size_t)t * LAT + h * D, D, cache); }
    }
    /* KQ = mul_mat(K f32, Q f32) (no rounding: both F32), scale, diag_mask_inf(0), soft_max, KQV = mul_mat(V^T f32, KQ) */
    const float scale = 1.0f / sqrtf((float)D);
#pragma omp parallel for schedule(dynamic)
    for (int hq = 0; hq < nh * F; ++hq) {
        const int h = hq / F, i = hq % F;
        float *s = malloc(sizeof(float) * (size_t)(i + 1));
        float mx = -INFINITY;
        for (int j = 0; j <= i; ++j) {
            float d = 0.f;
            for (int e = 0; e < D; ++e) d += k[(size_t)j * LAT + h * D + e] * q[(size_t)i * LAT + h * D + e];
            s[j] = d * scale;
            if (s[j] > mx) mx = s[j];
        }
        double sum = 0.0;
        for (int j = 0; j <= i; ++j) { s[j] = expf(s[j] - mx); sum += s[j]; }
        const float inv = (float)(1.0 / sum);
        for (int j = 0; j <= i; ++j) s[j] *= inv;
        for (int e = 0; e < D; ++e) {
            float a = 0.f;
            for (int j = 0; j <= i; ++j) a += v[(size_t)j * LAT + h * D + e] * s[j];
            att[(size_t)i * LAT + h * D + e] = a;
        }
        free(s);
    }
    mul_mat_rows(m, &l->o, att, F, y);
    for (int t = 0; t < F; ++t) for (int i = 0; i < VH; ++i) x[(size_t)t * VH + i] += y[(size_t)t * VH + i] * l->attn_scale[i];
    for (int t = 0; t < F; ++t) rms_norm_w(x + (size_t)t * VH, l->ffn_norm, xn + (size_t)t * VH, VH, eps);
    float *g = malloc(sizeof(float) * (size_t)F * c->voc_ffn), *u = malloc(sizeof(float) * (size_t)F * c->voc_ffn);
    mul_mat_rows(m, &l->gate, xn, F, g);
    mul_mat_rows(m, &l->up, xn, F, u);
    for (size_t i = 0; i < (size_t)F * c->voc_ffn; ++i) g[i] = silu_f(g[i]) * u[i];
    mul_mat_rows(m, &l->down, g, F, y);
    for (int t = 0; t < F; ++t) for (int i = 0; i < VH; ++i) x[(size_t)t * VH + i] += y[(size_t)t * VH + i] * l->ffn_scale[i];
    free(xn); free(q); free(k); free(v); free(att); free(y); free(g); free(u);
}

/* ConvNeXt upsample block, :490-549. x [C][T] -> returns [C][T'] */
static float *voc_upsample(const q3o_model *m, const upblk_t *ub, const float *x, int T, int *Tout) {
    int T1, T2;
    float *h = convT1d(m, &ub->up, x, T, 2, 0, &T1);
    float *d = conv1d(m, &ub->dw, h, T1, 6, 1, 1, &T2);
    const int C = ub->up.oc, F4 = ub->pw1.rows;
    float *dt = transpose(d, C, T1);                 /* [T][C] */
    float *n = malloc(sizeof(float) * (size_t)T1 * C);
    for (int t = 0; t < T1; ++t) layer_norm_wb(dt + (size_t)t * C, ub->norm_w, ub->norm_b, n + (size_t)t * C, C, 1e-6f);
    float *p1 = malloc(sizeof(float) * (size_t)T1 * F4);
    mul_mat_rows(m, &ub->pw1, n, T1, p1);
    for (int t = 0; t < T1; ++t) for (int i = 0; i < F4; ++i) p1[(size_t)t * F4 + i] = gelu_ggml(p1[(size_t)t * F4 + i] + ub->pw1_b[i]);
    mul_mat_rows(m, &ub->pw2, p1, T1, dt);
    for (int t = 0; t < T1; ++t) for (int i = 0; i < C; ++i) dt[(size_t)t * C + i] += ub->pw2_b[i];
    for (int ch = 0; ch < C; ++ch)
        for (int t = 0; t < T1; ++t) h[(size_t)ch * T1 + t] += dt[(size_t)t * C + ch] * ub->gamma[ch];
    free(d); free(dt); free(n); free(p1);
    *Tout = T1;
    return h;
}

static float *voc_decode_full(const q3o_model *m, const int32_t *codes, int F, int *Tout) {
    const q3o_config *c = &m->c;
    const int CD = c->cb_dim, VH = c->voc_hidden, LAT = c->voc_latent, NCB = c->n_codebooks;
    /* 1) RVQ lookup + output projections (:650-703) */
    float *emb = malloc(sizeof(float) * (size_t)F * CD);
    float *lat = malloc(sizeof(float) * (size_t)F * VH), *tmp = malloc(sizeof(float) * (size_t)F * VH), *acc = malloc(sizeof(float) * (size_t)F * VH);
    for (int t = 0; t < F; ++t) for (int i = 0; i < CD; ++i) emb[(size_t)t * CD + i] = q3o_f16_to_f32(m->cb_first[(size_t)codes[t * NCB] * CD + i]);
    mul_mat_rows(m, &m->vq_first_out, emb, F, lat);
    for (int cb = 0; cb < 15; ++cb) {
        for (int t = 0; t < F; ++t) for (int i = 0; i < CD; ++i) emb[(size_t)t * CD + i] = q3o_f16_to_f32(m->cb_rest[cb][(size_t)codes[t * NCB + cb + 1] * CD + i]);
        mul_mat_rows(m, &m->vq_rest_out, emb, F, cb == 0 ? acc : tmp);
        if (cb > 0) for (size_t i = 0; i < (size_t)F * VH; ++i) acc[i] += tmp[i];
    }
    for (size_t i = 0; i < (size_t)F * VH; ++i) lat[i] += acc[i];
    free(emb); free(tmp); free(acc);
    /* 2) causal pre-conv k3 (:705-718) on [VH][F] */
    float *latc = transpose(lat, F, VH);
    int T;
    float *pc = conv1d(m, &m->pre_conv, latc, F, 2, 1, 0, &T);          /* [LAT][F] */
    float *pct = transpose(pc, LAT, F);                                  /* [F][LAT] */
    free(lat); free(latc); free(pc);
    /* 3) input_proj, 8 transformer layers, norm, output_proj (:720-744) */
    float *x = malloc(sizeof(float) * (size_t)F * VH);
    mul_mat_rows(m, &m->in_proj, pct, F, x);
    for (int t = 0; t < F; ++t) for (int i = 0; i < VH; ++i) x[(size_t)t * VH + i] += m->in_proj_b[i];
    for (int i = 0; i < c->voc_layers; ++i) voc_tfm_layer(m, &m->VL[i], x, F);
    float *xn = malloc(sizeof(float) * (size_t)F * VH);
    for (int t = 0; t < F; ++t) rms_norm_w(x + (size_t)t * VH, m->pre_norm, xn + (size_t)t * VH, VH, 1e-5f);
    mul_mat_rows(m, &m->out_proj, xn, F, pct);
    for (int t = 0; t < F; ++t) for (int i = 0; i < LAT; ++i) pct[(size_t)t * LAT + i] += m->out_proj_b[i];
    float *cur = transpose(pct, F, LAT);                                 /* [LAT][F] */
    free(x); free(xn); free(pct);
    T = F;
    /* 4) two ConvNeXt upsample blocks */
    for (int u = 0; u < 2; ++u) { int T2; float *nx = voc_upsample(m, &m->up[u], cur, T, &T2); free(cur); cur = nx; T = T2; }
    /* 5) dec0 conv k7 */
    { int T2; float *nx = conv1d(m, &m->dec0, cur, T, 6, 1, 0, &T2); free(cur); cur = nx; T = T2; }
    /* 6) 4 decoder blocks (:551-620) */
    for (int d = 0; d < 4; ++d) {
        const decblk_t *db = &m->dec[d];
        float *sn = malloc(sizeof(float) * (size_t)db->snake.n * T);
        snake_apply(&db->snake, cur, sn, T);
        int T2;
        float *ct = convT1d(m, &db->ct, sn, T, db->rate, db->ct.k - db->rate, &T2);
        free(sn); free(cur); cur = ct; T = T2;
        const int C = db->ct.oc;
        for (int r = 0; r < 3; ++r) {
            const resunit_t *ru = &db->res[r];
            float *a = malloc(sizeof(float) * (size_t)C * T);
            snake_apply(&ru->a1, cur, a, T);
            int T3, T4;
            float *h1 = conv1d(m, &ru->c1, a, T, 6 * ru->dil, ru->dil, 0, &T3);
            snake_apply(&ru->a2, h1, a, T3);
            float *h2 = conv1d(m, &ru->c2, a, T3, 0, 1, 0, &T4);
            for (size_t i = 0; i < (size_t)C * T; ++i) cur[i] += h2[i];
            free(a); free(h1); free(h2);
        }
    }
    /* 7) final snake, conv k7 -> 1, tanh (:775-790) */
    float *sn = malloc(sizeof(float) * (size_t)m->dec5.n * T);
    snake_apply(&m->dec5, cur, sn, T);
    int T2;
    float *o = conv1d(m, &m->dec6, sn, T, 6, 1, 0, &T2);
    free(sn); free(cur);
    for (int t = 0; t < T2; ++t) o[t] = tanhf(o[t]);
    *Tout = T2;
    return o;
}

static int64_t full_len(const q3o_model *m, int F) {
    int64_t T = F;
    for (int u = 0; u < 2; ++u) T = (T - 1) * 2 + m->c.up_k;
    for (int d = 0; d < 4; ++d) { const int s = m->c.rates[d], K = m->c.conv_t_k[d]; T = (T - 1) * s + K - 2 * (K - s); }
    return T;
}
int q3o_tensor(const q3o_model *m, const char *name, float *out, int64_t n, int *src_type) {
    const gguf_t *g = m->gt;
    const gtensor *t = gfind(g, name);
    if (!t && m->gk) { g = m->gk; t = gfind(g, name); }
    if (!t) FAIL("missing tensor %s", name);
    const int64_t ne = t->ne[0] * t->ne[1] * t->ne[2] * t->ne[3];
    if (ne != n || (t->type != 0 && t->type != 1)) FAIL("tensor %s: %lld elements of type %d", name, (long long)ne, t->type);
    const void *d = tdata(g, t);
    for (int64_t i = 0; i < n; ++i) out[i] = t->type == 1 ? q3o_f16_to_f32(((const uint16_t *)d)[i]) : ((const float *)d)[i];
    if (src_type) *src_type = t->src_type;
    return 1;
}

int q3o_codebook(const q3o_model *m, int i, float *out) {
    if (!m->c.has_vocoder || i < 0 || i > 15) FAIL("no codebook %d", i);
    const uint16_t *cb = i == 0 ? m->cb_first : m->cb_rest[i - 1];
    for (size_t k = 0; k < (size_t)m->c.cb_size * m->c.cb_dim; ++k) out[k] = q3o_f16_to_f32(cb[k]);
    return 1;
}

int64_t q3o_vocoder_len(const q3o_model *m, int F, int mode) {
    if (F <= 0) return 0;
    return mode == 0 ? full_len(m, F) : (int64_t)F * 1920;
}

int q3o_vocoder_decode(const q3o_model *m, const int32_t *codes, int F, int mode, float *pcm, int64_t *n_samples) {
    if (!m->c.has_vocoder) FAIL("vocoder not loaded");
    *n_samples = q3o_vocoder_len(m, F, mode);
    if (!pcm || F <= 0) return 1;
    if (mode == 0) {
        int T;
        float *o = voc_decode_full(m, codes, F, &T);
        memcpy(pcm, o, sizeof(float) * (size_t)T);
        free(o);
        return 1;
    }
    /* CHUNK40: independent fixed 40-frame chunks, zero-padded codes, keep chunk_frames*1920 samples */
    const int FIX = 40, NCB = m->c.n_codebooks;
    int32_t *cc = malloc(sizeof(int32_t) * (size_t)FIX * NCB);
    int64_t out = 0;
    for (int off = 0; off < F; off += FIX) {
        const int cf = F - off < FIX ? F - off : FIX;
        memset(cc, 0, sizeof(int32_t) * (size_t)FIX * NCB);
        memcpy(cc, codes + (size_t)off * NCB, sizeof(int32_t) * (size_t)cf * NCB);
        int T;
        float *o = voc_decode_full(m, cc, FIX, &T);
        const int64_t want = (int64_t)cf * 1920;
        for (int64_t i = 0; i < want; ++i) pcm[out + i] = i < T ? o[i] : 0.f;
        out += want;
        free(o);
    }
    free(cc);
    return 1;
}
