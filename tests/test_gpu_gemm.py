"""Decode GEMM (hpa_gemm_f32, fp32 v_mfma_f32_32x32x2_f32) vs a plain PyTorch
fp32 reference of the same op (matmul_forward, paged_infer.c:92-114) and a
float64 numpy product.  Tolerance: |gpu - f64| <= 2e-6 * sum_k |x||w| + 1e-6
(fp32 accumulation over K terms), stated per element.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _gemm(hip, x, w, b, splitk, epi):
    L = hip.lib()
    M, K = x.shape
    N = w.shape[0]
    d_x = hip.DeviceBuffer.from_array(x)
    d_w = hip.DeviceBuffer.from_array(w)
    d_b = hip.DeviceBuffer.from_array(b) if b is not None else None
    d_o = hip.DeviceBuffer(splitk * M * N * 4)
    hip.check(L.hpa_gemm_f32(d_x.ptr, K, d_w.ptr, d_b.ptr if d_b else None, d_o.ptr, N, M, N, K,
                             splitk, epi))
    hip.check(L.hpa_synchronize())
    out = d_o.download((splitk, M, N))
    return out


@pytest.mark.parametrize("M,N,K", [(64, 2304, 768), (64, 768, 3072), (3, 100, 64), (130, 96, 768),
                                   (8, 3072, 768), (64, 50257, 768), (1, 1600, 1600)])
def test_gemm_matches_fp32_reference(hip, M, N, K):
    rng = np.random.default_rng(M * 7 + N)
    x = rng.uniform(-1, 1, (M, K)).astype(np.float32)
    w = rng.uniform(-0.05, 0.05, (N, K)).astype(np.float32)
    b = rng.uniform(-0.1, 0.1, N).astype(np.float32)
    ref64 = x.astype(np.float64) @ w.astype(np.float64).T + b
    ref32 = (torch.from_numpy(x) @ torch.from_numpy(w).T + torch.from_numpy(b)).numpy()
    bound = 2e-6 * (np.abs(x).astype(np.float64) @ np.abs(w).astype(np.float64).T) + 1e-6
    # fused bias epilogue, split 1
    out = _gemm(hip, x, w, b, 1, hip.HPA_EPI_BIAS)[0]
    assert np.all(np.abs(out - ref64) <= bound)
    assert np.abs(out - ref32).max() <= 2 * bound.max()
    # the split the engine would pick, partial slabs summed
    s = hip.lib().hpa_gemm_pick_splitk(M, N, K)
    if s > 1:
        part = _gemm(hip, x, w, None, s, hip.HPA_EPI_PARTIAL)
        assert np.all(np.abs(part.sum(0, dtype=np.float64) + b - ref64) <= bound)


def test_gemm_bias_gelu_epilogue(hip):
    rng = np.random.default_rng(1)
    M, N, K = 64, 3072, 768
    x = rng.uniform(-1, 1, (M, K)).astype(np.float32)
    w = rng.uniform(-0.05, 0.05, (N, K)).astype(np.float32)
    b = rng.uniform(-0.1, 0.1, N).astype(np.float32)
    out = _gemm(hip, x, w, b, 1, hip.HPA_EPI_BIAS_GELU)[0]
    h = torch.from_numpy(x).double() @ torch.from_numpy(w).double().T + torch.from_numpy(b).double()
    ref = torch.nn.functional.gelu(h, approximate="tanh").numpy()
    assert np.abs(out - ref).max() <= 1e-5


def test_gemm_deterministic(hip):
    rng = np.random.default_rng(2)
    x = rng.uniform(-1, 1, (64, 768)).astype(np.float32)
    w = rng.uniform(-0.05, 0.05, (768, 768)).astype(np.float32)
    a = _gemm(hip, x, w, None, 6, hip.HPA_EPI_PARTIAL)
    c = _gemm(hip, x, w, None, 6, hip.HPA_EPI_PARTIAL)
    assert np.array_equal(a, c)


def test_gemm_rejects_bad_shapes(hip):
    L = hip.lib()
    d = hip.DeviceBuffer(1 << 20)
    # K not a multiple of 8 -> error code, nothing launched
    assert L.hpa_gemm_f32(d.ptr, 12, d.ptr, None, d.ptr, 16, 4, 16, 12, 1, 1) != 0
