"""K17 MFMA GEMM (csrc/nn/gemm_mfma.hip) against fp64 torch on odd shapes, every operand layout, batch
broadcasting and the fused epilogue; and the ONNX Gemm / MatMul ops on it."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _G():
    from synapseml_amd.ops import gemm as G

    return G


def _check(y, ref, dtype):
    ref = ref.double()
    err = (y.double().cpu() - ref.cpu()).abs().max().item()
    scale = max(ref.abs().max().item(), 1.0)
    tol = {torch.float32: 1e-5, torch.float16: 4e-3, torch.bfloat16: 3e-2}[dtype]
    assert err <= tol * scale, (err, scale, dtype)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16, torch.bfloat16])
@pytest.mark.parametrize("M,N,K", [(1, 1, 1), (67, 131, 97), (128, 1000, 2048), (256, 64, 64), (5, 300, 4099)])
@pytest.mark.parametrize("ta,tb", [(False, False), (False, True), (True, False), (True, True)])
def test_gemm_layouts(dtype, M, N, K, ta, tb):
    g = torch.Generator(device="cpu").manual_seed(M * 7 + N + K)
    a64 = torch.randn(M, K, generator=g, dtype=torch.float64)
    b64 = torch.randn(K, N, generator=g, dtype=torch.float64)
    # ta: A stored [K, M] and read through a transposed view; tb: B stored [N, K] (an FC weight), read as B^T
    a = a64.t().contiguous().to("cuda", dtype).t() if ta else a64.to("cuda", dtype)
    b = b64.t().contiguous().to("cuda", dtype).t() if tb else b64.to("cuda", dtype)
    y = _G().gemm(a, b)
    _check(y, a.double().cpu() @ b.double().cpu(), dtype)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
def test_gemm_epilogue(dtype):
    g = torch.Generator(device="cpu").manual_seed(3)
    M, N, K = 77, 1000, 256
    a = torch.randn(M, K, generator=g).to("cuda", dtype)
    w = torch.randn(N, K, generator=g).to("cuda", dtype)  # FC weight [out, in], read as b = w.t()
    bias = torch.randn(N, generator=g)
    c = torch.randn(M, N, generator=g).to("cuda", dtype)
    ref = 0.5 * (a.double().cpu() @ w.double().cpu().t()) + 2.0 * bias.double()
    _check(_G().gemm(a, w.t(), bias=bias, alpha=0.5, beta=2.0), ref, dtype)
    _check(_G().gemm(a, w.t(), bias=bias, alpha=0.5, beta=2.0, relu=True), ref.clamp_min(0), dtype)
    ref2 = 1.5 * (a.double().cpu() @ w.double().cpu().t()) - 0.25 * c.double().cpu()
    _check(_G().gemm(a, w.t(), c=c, alpha=1.5, beta=-0.25), ref2, dtype)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("sa,sb", [((3, 4, 33, 65), (3, 4, 65, 17)), ((2, 1, 40, 64), (1, 5, 64, 24)),
                                   ((6, 50, 96), (96, 70)), ((96,), (4, 96, 3)), ((7, 130), (130,))])
def test_matmul_broadcast(dtype, sa, sb):
    g = torch.Generator(device="cpu").manual_seed(len(sa) * 10 + len(sb))
    a = torch.randn(*sa, generator=g, dtype=torch.float64)
    b = torch.randn(*sb, generator=g, dtype=torch.float64)
    y = _G().matmul(a.to("cuda", dtype), b.to("cuda", dtype))
    ref = torch.matmul(a.to(dtype).double(), b.to(dtype).double())
    assert tuple(y.shape) == tuple(ref.shape)
    _check(y, ref, dtype)


def test_onnx_gemm_and_matmul_ops_run_on_the_mfma_gemm(monkeypatch):
    """The executor's Gemm (transB, bias, fused Relu) and MatMul go through gemm_mfma: torch.matmul is
    never called on the GPU path."""
    from synapseml_amd.onnx import ops as O

    calls = []
    real = torch.matmul
    monkeypatch.setattr(torch, "matmul", lambda *a, **k: calls.append(1) or real(*a, **k))

    class RT:
        class session:
            _nn = object()

    x = torch.randn(9, 48, device="cuda")
    w = torch.randn(20, 48, device="cuda")
    bias = torch.randn(20, device="cuda")
    y = O.OPS["Gemm"](RT, {"transB": 1, "__act": 1}, [x, w, bias])[0]
    ref = torch.relu(x.double() @ w.double().t() + bias.double())
    assert (y.double() - ref).abs().max().item() < 1e-4
    m = O.OPS["MatMul"](RT, {}, [x.reshape(3, 3, 48), w.t()])[0]
    assert (m.double() - (x.reshape(3, 3, 48).double() @ w.double().t())).abs().max().item() < 1e-4
    assert not calls


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
@pytest.mark.parametrize("C,Cout,k,stride,pad,groups", [
    (3, 64, 7, 2, 3, 1),      # the ResNet stem: 3 channels, 7x7/2
    (24, 40, 3, 1, 1, 1),     # channel counts that are not multiples of the MFMA K tile
    (1, 8, 5, 1, 2, 1),       # grayscale
    (32, 32, 3, 2, 1, 32),    # depthwise
    (32, 64, 3, 1, 1, 32),    # depthwise, multiplier 2
    (64, 128, 3, 1, 1, 4),    # grouped, wide groups (batched GEMM)
    (16, 16, 1, 1, 0, 4),     # narrow groups (direct kernel)
])
def test_general_conv_matches_torch(dtype, C, Cout, k, stride, pad, groups):
    """Convs outside the tiled implicit-GEMM kernel run on the GEMM-with-im2col (stem, odd channels,
    wide groups) or the direct NHWC kernel (depthwise / narrow groups); fused bias + ReLU + residual."""
    from synapseml_amd.ops.conv import conv2d_nhwc_general

    g = torch.Generator(device="cpu").manual_seed(C * 31 + Cout + groups)
    x = torch.randn(3, C, 23, 29, generator=g)
    w = torch.randn(Cout, C // groups, k, k, generator=g) / (k * (C // groups)) ** 0.5
    b = torch.randn(Cout, generator=g)
    ref = torch.nn.functional.conv2d(x.double(), w.double(), b.double(), stride=stride, padding=pad, groups=groups)
    res = torch.randn(ref.shape, generator=g)
    xd = x.to("cuda", dtype).contiguous(memory_format=torch.channels_last)
    wp = w.to("cuda", dtype).permute(0, 2, 3, 1).contiguous()
    for relu, r in ((0, None), (2, res), (1, res)):
        y = conv2d_nhwc_general(xd, wp, k, k, (stride, stride), (pad, pad, pad, pad), (1, 1), groups=groups,
                                bias=b.cuda(), relu=relu,
                                res=None if r is None else r.to("cuda", dtype).contiguous(memory_format=torch.channels_last))
        want = ref if r is None else (torch.relu(ref + r.double()) if relu == 2 else torch.relu(ref) + r.double())
        _check(y.float().cpu(), want, dtype)
