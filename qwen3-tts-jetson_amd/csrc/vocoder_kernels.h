// vocoder_kernels.h — launchers of the vocoder (tokenizer decoder) kernels.
#pragma once
#include "q3t_common.h"

namespace q3t {

constexpr int CONV_MAX_TAPS = 7;

// SnakeBeta x + exp(-beta) sin^2(exp(alpha) x) with a = exp(alpha), ib = exp(-beta) (audio_tokenizer_decoder.cpp
// SnakeBeta).  The sine: reduce to [-0.5, 0.5] revolutions (v_rndne) and use the hardware v_sin_f32 -- ocml's sinf is
// ~30 VALU instructions with a range-reduction branch and ran twice per activation element of every residual unit;
// its result is rounded to f16 right after, so the ~1e-6 difference flips an f16 rounding only rarely.  Every kernel
// that applies SnakeBeta calls this one function, rounding each operation as written (no contraction), so a fused
// and an unfused launch sequence produce the same bits.
__device__ __forceinline__ float snake_apply(float z, float a, float ib) {
#pragma clang fp contract(off)
    const float r = (z * a) * 0.15915494309189535f;   // 1 / (2 pi)
    const float sn = __builtin_amdgcn_sinf(r - __builtin_rintf(r));
    return z + (sn * sn) * ib;
}
struct ConvTap { const uint16_t *w; int dj; };   // w: [C_out][C_in] f16 of one kernel tap; input row offset dj
// y[m*so + ob][co] = act(bias[co] + resid + sum_j sum_ci w_j[co][ci] * f16(snake(x[m + dj][ci])))
// x: [T_in][C_in] f32 (rows outside [0,T_in) read as 0 = causal zero padding); y: [T_out][C_out] f32
struct ConvParams {
    const float *x = nullptr;
    const uint16_t *xh = nullptr;   // alternative input: f16 rows [T_in][C_in] with SnakeBeta already applied (C_in % 8 == 0)
    int T_in = 0, C_in = 0;
    const float *snake_a = nullptr, *snake_ib = nullptr;   // exp(alpha), exp(-beta) per input channel (nullable)
    int n_taps = 0;
    ConvTap taps[CONV_MAX_TAPS];
    int dmin = 0, dmax = 0;
    float *y = nullptr;             // f32 output [T_out][ldy] (nullable when y16 is set)
    int C_out = 0, M = 0, so = 1, ob = 0;
    int ldy = 0;                    // row stride of y and resid (0: C_out)
    const float *bias = nullptr, *resid = nullptr;
    const float *scale = nullptr;   // per output channel, applied after the bias and before the residual
    int act = 0;   // 1 = tanh, 2 = ReLU, 3 = tanh(ReLU), 4 = GELU (ggml tanh form, f16 table); after the residual
    // optional f16 output of the same elements: y16[t][co] = f16(snake(v)) with exp(alpha) / exp(-beta) per output
    // channel (y16_a null: plain rounding) -- the NEXT conv's input, so no separate snake/round pass reads y back
    uint16_t *y16 = nullptr;
    const float *y16_a = nullptr, *y16_ib = nullptr;
    // transposed conv in one launch (multi-tile kernel): grid z = output phase phi of a stride-ct_st transposed conv
    // with ct_k taps [ct_k][C_out][C_in] at ct_w, trimmed by ct_trim; phase phi writes rows ct_st*m + phi < T_out
    // from taps k = (phi + trim) % st + j*st at input offset (phi + trim - k) / st.  taps/dmin/dmax/M/so/ob unused
    const uint16_t *ct_w = nullptr;
    int ct_k = 0, ct_st = 0, ct_trim = 0, T_out = 0;
    // utterance batch (grid z = nb x phases): nb independent sequences of the same length; utterance u's input rows
    // start xbs rows after u-1's (x / xh), its output rows (y, resid, y16) ybs rows after.  Causal padding stays
    // inside each utterance (rows outside [0, T_in) of its own segment read as 0)
    int nb = 1;
    int64_t xbs = 0, ybs = 0;
    int dev_skip = 0;   // development builds only (timing experiments): 1 weight loads, 2 window loads, 4 epilogue
    int xcd_tiles = 0;  // k_conv_mt 1-tap narrow variant: channel tiles of a row tile on one XCD (set by conv())
};
bool conv(const ConvParams &p, hipStream_t s);
// one 96-channel decoder residual unit as one launch (vocoder_resunit.hip), bit-identical to its two conv launches:
//   h = f16(snake2(conv7_dil(xh) + b1)) (kept on chip);  y = x + conv1(h) + b2;  y16 = f16(snake_next(y))
// xh / y16 are f16 [T][96] (different buffers: a tile's causal window reads rows of its neighbours), x / y f32 (may
// alias: in place; y null skips the f32 output); w1 [7][96][96], w2 [96][96] f16; nb utterances bs rows apart
struct ResUnitParams {
    const uint16_t *xh = nullptr;
    const float *x = nullptr;
    float *y = nullptr;
    uint16_t *y16 = nullptr;
    int T = 0, dil = 1;
    const uint16_t *w1 = nullptr, *w2 = nullptr;
    const float *b1 = nullptr, *a2 = nullptr, *ib2 = nullptr, *b2 = nullptr, *an = nullptr, *ibn = nullptr;
    int nb = 1;
    int64_t bs = 0;
};
bool resunit96(const ResUnitParams &p, hipStream_t s);
// out[t][c] = f16( snake(x[t][c]) ) (SnakeBeta x + exp(-beta) sin^2(exp(alpha) x), or plain rounding when a is null):
// the conv input computed ONCE per element instead of once per (output tile, tap window) inside k_conv
bool snake_f16(const float *x, const float *a, const float *ib, uint16_t *out, int64_t T, int C, hipStream_t s);
// out[t][:] = f16(norm(x[t][:])): mode 0 RMSNorm (x * scale) * w, mode 1 LayerNorm ((x - mean) * scale) * w + b;
// double sums as gemm_mfma's PRO_RMS / PRO_LN prologues (the input of a 1-tap conv used as a large-M GEMM)
bool norm_f16(const float *x, const float *w, const float *b, float eps, int mode, uint16_t *out, int T, int C,
              hipStream_t s);
// y[t] = tanh(bias + sum_j sum_ci w[j][ci] * xh[t + j - (K - 1)][ci]): the decoder's last conv (C_out = 1, K <= 8)
// nb utterances of T rows each, back to back (xh [nb][T][C], y [nb][T])
bool conv_out1(const uint16_t *xh, const uint16_t *w, const float *bias, float *y, int T, int C, int K, hipStream_t s,
               int nb = 1);
bool dwconv(const float *x, const uint16_t *w, const float *b, float *y, int T, int C, int K, hipStream_t s, int nb = 1);
// RoPE is applied to qkv's q and k columns in place; nb utterances of F frames each, causal within each
bool attn_prefill(float *qkv, const float *rope, uint16_t *out, int F, int nH, int D, hipStream_t s, int nb = 1);
bool codes_cols(const int32_t *codes, int *cols, int F, int ncb, hipStream_t s);

}  // namespace q3t
