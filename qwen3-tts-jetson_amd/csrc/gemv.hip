// gemv.hip — host dispatch of the weight-streaming GEMV (kernel: gemv_kernel.h; instantiations: gemv_inst_*.hip).
#include "kernels.h"
#include "select.h"
#include "cpatt.h"

#include <cstdlib>
#include <string>

namespace q3t {

// explicit instantiations live in gemv_inst_*.hip
template <int RPG, int BT, int KS>
void launch_pro(const GemvParams &p, int nl, dim3 grid, size_t lds, hipStream_t s);

template <int RPG, int BT>
static void launch_ks(const GemvParams &p, int ks, int nl, dim3 grid, size_t lds, hipStream_t s) {
    if (ks == 1) launch_pro<RPG, BT, 1>(p, nl, grid, lds, s);
    else if (ks == 2) launch_pro<RPG, BT, 2>(p, nl, grid, lds, s);
    else launch_pro<RPG, BT, 4>(p, nl, grid, lds, s);
}
template <int BT>
static void launch_bt(const GemvParams &p, int rpg, int ks, int nl, dim3 grid, size_t lds, hipStream_t s) {
    if (rpg == 2) launch_ks<2, BT>(p, ks, nl, grid, lds, s);
    else launch_ks<1, BT>(p, ks, nl, grid, lds, s);
}

static int g_min_blocks = [] {
#ifdef Q3T_DEV
    const char *e = std::getenv("Q3T_GEMV_MIN_BLOCKS");
    const int x = e ? std::atoi(e) : 0;
    return x > 0 ? x : 256;
#else
    return 256;
#endif
}();
static int gemv_min_blocks() { return g_min_blocks; }
// compute units of the current device (cached per device id)
static int device_cus() {
    static int cus[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (!cus[dev]) {
        int n = 0;
        cus[dev] = hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0 ? n : 256;
    }
    return cus[dev];
}
void gemv_set_min_blocks(int n) { g_min_blocks = n > 0 ? n : 256; }

bool gemv(const GemvParams &p, hipStream_t s) {
    if (p.B <= 0 || p.N <= 0) return true;
    if (gemm_mfma_supported(p)) return gemm_mfma(p, s);
    if (p.parts) { set_error("gemv: split-K slabs need the matrix-core path"); return false; }
    const bool swiglu = p.act == ACT_SWIGLU;
    if (p.K % 8 != 0 || (swiglu && p.N % 32 != 0)) {
        set_error("gemv: unsupported shape N=" + std::to_string(p.N) + " K=" + std::to_string(p.K));
        return false;
    }
    if (swiglu && p.pro != PRO_RMS) { set_error("gemv: SwiGLU needs the RMSNorm prologue"); return false; }
    const bool selg = p.pro == PRO_SEL_G1;
    if (selg && (p.sel.mode != SEL_CP || !p.sel_logits || !p.sel.tokens || p.sel.V != 2048 ||
                 (reinterpret_cast<uintptr_t>(p.sel_logits) & 15) != 0)) {
        set_error("gemv: PRO_SEL_G1 needs a code-predictor SelectSpec and the previous head's logits");
        return false;
    }
    if (!selg && p.sel.mode != SEL_NONE &&
        (p.pro != PRO_RMS || swiglu || !p.out_f32 || p.out_f16 || p.orow_mul != 1 || p.orow_add != 0 || p.ldo != p.N ||
         p.sel.V != p.N || p.N > 256 * SEL_VPT_MAX || !p.sel.ticket)) {
        set_error("gemv: fused selection needs an RMS-prologue head writing f32 logits [B][N] and a ticket buffer");
        return false;
    }
    const bool g1 = p.pro == PRO_RMS_G1 || selg, g16 = p.pro == PRO_RMS_G16;
    if (p.pro == PRO_CPATT) {
        const CpAttnSrc &A = p.att;
        if (p.K != CPA_NH * CPA_D || !A.qkv || !A.qn || !A.kn || !A.rope || !A.pos || !A.kc || !A.vc || A.ld % 4 != 0) {
            set_error("gemv: bad code-predictor attention source");
            return false;
        }
    } else if (p.pro != PRO_F16) {
        if (p.K > 4096) { set_error("gemv: f32 prologue limited to K <= 4096"); return false; }
        if (!g1 && !g16 && (p.ldx % 4 != 0 || (reinterpret_cast<uintptr_t>(p.x) & 15) != 0)) {
            set_error("gemv: f32 activation rows must be 16-byte aligned");
            return false;
        }
        if ((g1 && !(p.gs.tok && p.gs.tab0)) ||
            (g16 && !(p.gs.tok && p.gs.tabs && p.gs.tok_ld == 16 && p.gs.frame && p.gs.tr && p.gs.tr_len && p.gs.pad))) {
            set_error("gemv: bad gather-sum source");
            return false;
        }
        if ((g1 || g16) && p.K > 1024) { set_error("gemv: gather prologue limited to K <= 1024"); return false; }
        if (((p.pro == PRO_RMS || g1 || g16) && !p.nw) || (p.pro == PRO_LN && !(p.nw && p.nb))) {
            set_error("gemv: missing norm weights");
            return false;
        }
    } else if (p.ldx % 8 != 0 || (reinterpret_cast<uintptr_t>(p.x) & 15) != 0) {
        set_error("gemv: f16 activation rows must be 16-byte aligned");
        return false;
    }
    if ((p.K + 127) / 128 * 128 * 2 > 48 * 1024) { set_error("gemv: K too large for the LDS tile"); return false; }
    // batch tile: up to 8 activation rows in LDS as f16, capped at 48 KB of LDS
    int bt = p.B == 1 ? 1 : p.B == 2 ? 2 : p.B <= 4 ? 4 : 8;
    const int Kp = (p.K + 127) / 128 * 128;
    while (bt > 1 && (size_t)Kp * 2 * bt > 48 * 1024) bt /= 2;
    // family-pinned launches (the causal prefill's rows on a 1-slot step's kernels): at most 2 rows per workgroup, so
    // the 16 prompt rows spread over 8 workgroup rows instead of 2.  The tile never changes a row's arithmetic (the K
    // split comes from the family below).  16-row prefill 1.87 -> 1.39 ms (tiles 8 / 4 / 2 / 1: 1.89 / 1.51 / 1.39 /
    // 1.52 ms)
    if (p.family_b > 0) while (bt > 2) bt /= 2;
    const int gy = (p.B + bt - 1) / bt;
    const int rpg = swiglu ? 2 : 1;
    const int units = swiglu ? p.N / 2 : p.N;   // output rows (SwiGLU: gate/up pairs)
    // the K split (the only launch choice that changes a row's summation order) from the family batch's grid
    const int fb = p.family_b > 0 ? p.family_b : p.B;
    int fbt = fb == 1 ? 1 : fb == 2 ? 2 : fb <= 4 ? 4 : 8;
    while (fbt > 1 && (size_t)Kp * 2 * fbt > 48 * 1024) fbt /= 2;
    const int fgy = (fb + fbt - 1) / fbt;
    auto blocks_for = [&](int ks) { return (long)((units + (16 / ks) - 1) / (16 / ks)) * fgy; };
    int ks = 4;
    for (int c : {1, 2, 4})
        if (blocks_for(c) >= gemv_min_blocks()) { ks = c; break; }
#ifndef Q3T_GEMV_ROUNDS
#define Q3T_GEMV_ROUNDS 1
#endif
    // rows wider than 1,024 (the 1.7B talker and its codec head; never a shape the persistent kernels restate): a grid
    // of whole rounds of workgroups per CU (1.7B gate/up: 384 workgroups left half the CUs with two, 768 give all three).
    // Unlike NL below, ks changes the row's summation order: it depends on the device's CU count, fixed per device
    if (Q3T_GEMV_ROUNDS && p.K > 1024 && ks < 4 && blocks_for(ks) % device_cus() != 0) ks *= 2;
    const int nsteps = (Kp / 128 + ks - 1) / ks;
    // NL: weight loads per lane issued up front (16 only for single-row launches; launch_nl streams the rest with NL 0).
    // The loads' schedule only: the K order of every row is the same for any NL
    int nl = nsteps <= 2 ? 2 : nsteps <= 4 ? 4 : nsteps <= 8 ? 8 : (nsteps <= 16 && bt == 1) ? 16 : 0;
    if (nl == 0 && nsteps <= 24 && bt == 1 && p.pro == PRO_F16) nl = 24;
    if (bt > 2 || Kp > (nl == 24 ? 6144 : 4096)) nl = 0;
    const dim3 grid((unsigned)((units + (16 / ks) - 1) / (16 / ks)), (unsigned)gy);
    const size_t lds = (size_t)bt * Kp * 2 + 16 * rpg * bt * 4 + 8 * sizeof(double) +
                       (p.pro == PRO_CPATT ? CPA_LDS : 0) + (p.sel.mode != SEL_NONE ? sizeof(SelLds) : 0) +
                       (selg ? 8 * sizeof(int) : 0);
    if (bt == 1) launch_bt<1>(p, rpg, ks, nl, grid, lds, s);
    else if (bt == 2) launch_bt<2>(p, rpg, ks, nl, grid, lds, s);
    else if (bt == 4) launch_bt<4>(p, rpg, ks, nl, grid, lds, s);
    else launch_bt<8>(p, rpg, ks, nl, grid, lds, s);
    Q3T_HIP(hipGetLastError());
    return true;
}

}  // namespace q3t
