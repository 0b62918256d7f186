"""GPU: the src/trt_cuda_kernels.cu drop-ins (gpu_argmax_f32, gpu_sample_topk_f32, gpu_fp32_to_fp16,
gpu_embedding_lookup_by_gpu_id) called through the C ABI on device buffers, against the reference semantics
(trt_cuda_kernels.cu:16-190): first-index argmax, temperature -> top-k (`< thr` dropped, ties kept) -> softmax ->
inverse CDF.  The same selection code runs inside the fused head launches of the decode path (select.h), so the
degenerate cases (ties at the threshold, a boundary bin with > 256 keys -> radix fallback, -inf runs) live here."""
import ctypes as C
import os
import sys

import numpy as np
import pytest

from q3t_testutil import REPO, check_token

pytestmark = pytest.mark.gpu
sys.path.insert(0, os.path.join(REPO, "qwen3-tts-jetson_amd"))


@pytest.fixture(scope="module")
def dev():
    import hip_py
    if hip_py.device_count() == 0:
        pytest.skip("no GPU")
    import q3t
    lib = q3t.lib()
    lib.gpu_argmax_f32.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
    lib.gpu_sample_topk_f32.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_float, C.c_int32, C.c_int32, C.c_void_p]
    lib.gpu_fp32_to_fp16.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
    lib.gpu_embedding_lookup_by_gpu_id.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
    return hip_py, lib


def _cases(rng, V):
    yield "normal", rng.normal(0, 3, V).astype(np.float32)
    yield "ties", np.round(rng.normal(0, 2, V) * 2).astype(np.float32) / 2      # many exact ties, incl. at the top-k cut
    yield "constant", np.full(V, 1.5, np.float32)                              # boundary bin holds every key: radix fallback
    x = np.full(V, -np.inf, np.float32)
    x[rng.choice(V, 70, replace=False)] = rng.normal(0, 1, 70).astype(np.float32)
    yield "mostly-inf", x
    y = rng.normal(0, 1e-3, V).astype(np.float32) + 7.0                       # one dense bin near the max
    yield "dense", y


@pytest.mark.parametrize("V", [2048, 3072, 4096])
def test_argmax_first_index(dev, V):
    hp, lib = dev
    rng = np.random.default_rng(V)
    for name, x in _cases(rng, V):
        d, out = hp.DevBuf(x), hp.DevBuf(nbytes=4)
        lib.gpu_argmax_f32(d.p, out.p, V, None)
        assert int(out.get(np.int32, 1)[0]) == int(np.argmax(x)), name


def test_argmax_any_length(dev):
    hp, lib = dev
    x = np.random.default_rng(1).normal(0, 1, 151936).astype(np.float32)   # text-vocab sized: generic path
    x[99999] = x.max()
    d, out = hp.DevBuf(x), hp.DevBuf(nbytes=4)
    lib.gpu_argmax_f32(d.p, out.p, x.size, None)
    assert int(out.get(np.int32, 1)[0]) == int(np.argmax(x))


@pytest.mark.parametrize("V", [2048, 3072])
@pytest.mark.parametrize("top_k", [1, 50, 0])
def test_sample_topk_matches_reference_semantics(dev, V, top_k):
    hp, lib = dev
    rng = np.random.default_rng(V + top_k)
    n_tol = n = 0
    out = hp.DevBuf(nbytes=4)
    for name, x in _cases(rng, V):
        d = hp.DevBuf(x)
        for u in np.linspace(0.003, 0.997, 23):
            r = hp.DevBuf(np.array([u], np.float32))
            lib.gpu_sample_topk_f32(d.p, r.p, out.p, 0.9, top_k, V, None)
            tok = int(out.get(np.int32, 1)[0])
            assert 0 <= tok < V and np.isfinite(x[tok]), (name, u)
            n_tol += check_token(x, tok, 0.9, top_k, float(u), -1, tol_cdf=1e-4)
            n += 1
    assert n_tol <= 2, (n_tol, n)


def test_fp32_to_fp16_and_embedding_lookup(dev):
    hp, lib = dev
    x = np.random.default_rng(3).normal(0, 10, 1001).astype(np.float32)
    d, h = hp.DevBuf(x), hp.DevBuf(nbytes=1001 * 2)
    lib.gpu_fp32_to_fp16(d.p, h.p, 1001, None)
    assert np.array_equal(h.get(np.float16, 1001), x.astype(np.float16))
    table = np.random.default_rng(4).normal(0, 1, (50, 96)).astype(np.float32)
    tb, tok, o = hp.DevBuf(table), hp.DevBuf(np.array([37], np.int32)), hp.DevBuf(nbytes=96 * 4)
    lib.gpu_embedding_lookup_by_gpu_id(tok.p, tb.p, o.p, 96, None)
    assert np.array_equal(o.get(np.float32, 96), table[37])
