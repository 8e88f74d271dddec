"""MFMA implicit-GEMM convolution vs a plain fp32 PyTorch reference of the same
fused op (prologue affine+ReLU, bias, ReLU, residual, second affine output)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _ref(x, w, stride, pad, bias=None, relu=False, pro=None, res=None, post=None):
    xf = x.float()
    if pro is not None:
        xf = torch.relu(xf * pro[0].view(1, -1, 1, 1) + pro[1].view(1, -1, 1, 1))
    y = F.conv2d(xf, w.float(), None, stride, pad)
    if bias is not None:
        y = y + bias.view(1, -1, 1, 1)
    if relu:
        y = torch.relu(y)
    if res is not None:
        y = y + res.float()
    y2 = None if post is None else torch.relu(y * post[0].view(1, -1, 1, 1) + post[1].view(1, -1, 1, 1))
    return y, y2


# 0 = shape-chosen tile; BM*1000+BN = forced tile (128999 / 64999: 128x128 / 64x64 with 8 waves; 256064 /
# 128164: 256x64 / 128x64 with one wave along N, 64x64 wave tiles; 128777 / 64777 / 256777: the LDS-DMA
# staged 128x128 (8 waves) / 64x64 / 256x64 forms, swizzled unpadded LDS rows)
# 128932 / 256932 / 64932: 32x32x16 MFMA forms of 128x128 (8 waves) / 256x128 (8 waves) / 64x64 (4 waves)
# 128555 / 64555: persistent tile walk (next tile's loads behind the epilogue)
KERNELS = [0, 64064, 64999, 128064, 64128, 128128, 128999, 256128, 128256, 256064, 128164, 128777, 64777, 256777,
           128932, 256932, 64932, 128555, 64555]


@pytest.mark.parametrize("kernel", KERNELS)
def test_exact_integer_layout(kernel):
    """Small integers are exact in fp16 and fp32: any lane/row/col mapping (or LDS swizzle) error shows as a
    mismatch. Shapes leave partial tiles in M and N and padding taps on every border."""
    from synapseml_amd.ops.conv import conv2d_nhwc, pack_weight

    g = torch.Generator().manual_seed(0)
    for (B, C, H, W, Co) in ((2, 64, 9, 7, 80), (3, 128, 17, 11, 200)):
        x = torch.randint(-2, 3, (B, C, H, W), generator=g).half().cuda().contiguous(memory_format=torch.channels_last)
        w = torch.randint(-2, 3, (Co, C, 3, 3), generator=g).half().cuda()
        y = conv2d_nhwc(x, pack_weight(w, torch.float16), 3, 3, (1, 1), (1, 1), kernel=kernel)
        ref = F.conv2d(x.float(), w.float(), None, 1, 1)
        torch.testing.assert_close(y.float(), ref, rtol=0, atol=0)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("shape", [
    # B, C, H, W, Cout, k, stride, pad
    (4, 64, 56, 56, 64, 1, 1, 0),
    (4, 64, 56, 56, 256, 1, 1, 0),
    (2, 256, 28, 28, 128, 3, 1, 1),
    (2, 128, 29, 29, 128, 3, 2, 1),
    (3, 512, 14, 14, 1024, 1, 2, 0),
    (1, 2048, 7, 7, 512, 1, 1, 0),
])
def test_conv_matches_fp32_reference(dtype, shape):
    from synapseml_amd.ops.conv import conv2d_nhwc, pack_weight

    B, C, H, W, Co, k, st, pd = shape
    torch.manual_seed(1)
    x = torch.randn(B, C, H, W, device="cuda").to(dtype).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(Co, C, k, k, device="cuda") / (C * k * k) ** 0.5).to(dtype)
    bias = torch.randn(Co, device="cuda")
    ref, _ = _ref(x, w, st, pd, bias=bias, relu=True)
    tol = 2e-2 if dtype == torch.float16 else 8e-2
    for kernel in (0, 128128, 128999, 256128, 128256, 256064, 128164, 128777, 64777, 256777, 128932, 256932, 64932,
                   128555, 64555):
        y = conv2d_nhwc(x, pack_weight(w, dtype), k, k, (st, st), (pd, pd), bias=bias, relu=True, kernel=kernel)
        torch.testing.assert_close(y.float(), ref, rtol=tol, atol=tol, msg=lambda m: f"kernel {kernel}: {m}")


def test_prologue_residual_dual_output():
    from synapseml_amd.ops.conv import conv2d_nhwc, pack_weight

    torch.manual_seed(2)
    dt = torch.float16
    B, C, H, W, Co = 2, 128, 14, 14, 256
    x = torch.randn(B, C, H, W, device="cuda").to(dt).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(Co, C, 1, 1, device="cuda") / C ** 0.5).to(dt)
    pro = (torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.1)
    res = torch.randn(B, Co, H, W, device="cuda").to(dt).contiguous(memory_format=torch.channels_last)
    post = (torch.rand(Co, device="cuda") + 0.5, torch.randn(Co, device="cuda") * 0.1)
    y, y2 = conv2d_nhwc(x, pack_weight(w, dt), 1, 1, in_affine=pro, res=res, out_affine=post)
    ry, ry2 = _ref(x, w, 1, 0, pro=pro, res=res, post=post)
    torch.testing.assert_close(y.float(), ry, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(y2.float(), ry2, rtol=2e-2, atol=3e-2)
    # the same through the 8-wave 256x128 tile and the 32x32x16 MFMA forms
    for kernel in (256128, 128932, 256932, 64932, 128555, 64555):
        yq, yq2 = conv2d_nhwc(x, pack_weight(w, dt), 1, 1, in_affine=pro, res=res, out_affine=post, kernel=kernel)
        torch.testing.assert_close(yq.float(), ry, rtol=2e-2, atol=2e-2)
        torch.testing.assert_close(yq2.float(), ry2, rtol=2e-2, atol=3e-2)
    with pytest.raises(RuntimeError):  # unknown tile code
        conv2d_nhwc(x, pack_weight(w, dt), 1, 1, kernel=12345)
    # padding taps stay zero with a prologue (3x3)
    w3 = (torch.randn(64, C, 3, 3, device="cuda") / (9 * C) ** 0.5).to(dt)
    y3 = conv2d_nhwc(x, pack_weight(w3, dt), 3, 3, (1, 1), (1, 1), in_affine=pro)
    r3, _ = _ref(x, w3, 1, 1, pro=pro)
    torch.testing.assert_close(y3.float(), r3, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("shape", [(2, 256, 14, 14, 64, 1), (2, 128, 15, 13, 200, 1), (3, 512, 14, 14, 1024, 2)])
def test_glds_prologue_matches_register_path(dtype, shape):
    """The LDS-DMA form's fragment-time prologue (1x1 pre-activation layers, stride 1 or 2) against the fp32
    reference and against the register-staged tile that applies the same affine + ReLU at its LDS write."""
    from synapseml_amd.ops.conv import conv2d_nhwc, pack_weight

    B, C, H, W, Co, st = shape
    torch.manual_seed(4)
    x = torch.randn(B, C, H, W, device="cuda").to(dtype).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(Co, C, 1, 1, device="cuda") / C ** 0.5).to(dtype)
    pro = (torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.5)
    bias = torch.randn(Co, device="cuda")
    ref, _ = _ref(x, w, st, 0, bias=bias, relu=True, pro=pro)
    tol = 2e-2 if dtype == torch.float16 else 8e-2
    wp = pack_weight(w, dtype)
    yr = conv2d_nhwc(x, wp, 1, 1, (st, st), (0, 0), bias=bias, relu=True, in_affine=pro, kernel=128999)
    for kernel in (0, 128777, 64777, 256777):
        y = conv2d_nhwc(x, wp, 1, 1, (st, st), (0, 0), bias=bias, relu=True, in_affine=pro, kernel=kernel)
        torch.testing.assert_close(y.float(), ref, rtol=tol, atol=tol, msg=lambda m: f"kernel {kernel}: {m}")
        torch.testing.assert_close(y.float(), yr.float(), rtol=1e-2, atol=1e-2, msg=lambda m: f"kernel {kernel}: {m}")


@pytest.mark.parametrize("dtype,mode", [(torch.float16, None), (torch.bfloat16, None), (torch.float32, "bf16x6"),
                                        (torch.float32, "bf16x3")])
@pytest.mark.parametrize("shape", [(2, 512, 7, 7, 512, 3), (1, 1024, 14, 14, 256, 1), (3, 256, 9, 11, 200, 3)])
def test_split_k_fused_epilogue(dtype, mode, shape):
    """Split-K (few output tiles, long K): partial fp32 tiles + arrival counters, the last split sums in split
    order and runs the fused prologue / bias / ReLU / residual / dual-output epilogue."""
    from synapseml_amd.ops import native
    from synapseml_amd.ops.conv import F32_MODES, conv2d_nhwc, pack_weight, out_hw

    B, C, H, W, Co, k = shape
    pd = k // 2
    oh, ow = out_hw(H, W, k, k, (1, 1), (pd, pd), (1, 1))
    geom = [B, H, W, C, Co, k, k, 1, 1, pd, pd, 1, 1, oh, ow]
    dt_code = F32_MODES[mode] if mode else {torch.float16: 1, torch.bfloat16: 2}[dtype]
    sk, _, _ = native.load("_nn").conv_split_plan(geom, dt_code, True)
    assert sk > 1
    torch.manual_seed(3)
    x = torch.randn(B, C, H, W, device="cuda").to(dtype).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(Co, C, k, k, device="cuda") / (C * k * k) ** 0.5).to(dtype)
    pro = (torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.1)
    bias = torch.randn(Co, device="cuda")
    res = torch.randn(B, Co, oh, ow, device="cuda").to(dtype).contiguous(memory_format=torch.channels_last)
    post = (torch.rand(Co, device="cuda") + 0.5, torch.randn(Co, device="cuda") * 0.1)
    y, y2 = conv2d_nhwc(x, pack_weight(w, dtype), k, k, (1, 1), (pd, pd), bias=bias, relu=True, in_affine=pro,
                        res=res, out_affine=post, f32_mode=mode)
    ry, ry2 = _ref(x, w, 1, pd, bias=bias, relu=True, pro=pro, res=res, post=post)
    tol = {torch.float16: 2e-2, torch.bfloat16: 8e-2, torch.float32: 2e-3}[dtype]
    torch.testing.assert_close(y.float(), ry, rtol=tol, atol=tol)
    torch.testing.assert_close(y2.float(), ry2, rtol=tol, atol=1.5 * tol)
    # repeated calls reuse the caching allocator's workspace: same result (summation order fixed per split)
    y_again, _ = conv2d_nhwc(x, pack_weight(w, dtype), k, k, (1, 1), (pd, pd), bias=bias, relu=True, in_affine=pro,
                             res=res, out_affine=post, f32_mode=mode)
    assert torch.equal(y, y_again)


# ---------------------------------------------------------------- fp32 (exact f32-input 16x16x4 MFMA)
F32_KERNELS = [0, 64064, 64999, 128064, 64128, 128128]


@pytest.mark.parametrize("kernel", F32_KERNELS)
def test_fp32_exact_integer_layout(kernel):
    """fp32 form: 16-B fragments feed four MFMAs from their components; small integers make any k / lane /
    row mapping error an exact mismatch. C = 32 and 96 exercise the 32-channel K tile (not a multiple of 64)."""
    from synapseml_amd.ops.conv import conv2d_nhwc, pack_weight

    g = torch.Generator().manual_seed(3)
    for (B, C, H, W, Co, k) in ((2, 32, 9, 7, 80, 3), (3, 96, 17, 11, 200, 3), (2, 64, 8, 8, 36, 1)):
        x = torch.randint(-3, 4, (B, C, H, W), generator=g).float().cuda().contiguous(memory_format=torch.channels_last)
        w = torch.randint(-3, 4, (Co, C, k, k), generator=g).float().cuda()
        y = conv2d_nhwc(x, pack_weight(w, torch.float32), k, k, (1, 1), (k // 2, k // 2), kernel=kernel)
        ref = F.conv2d(x.cpu().double(), w.cpu().double(), None, 1, k // 2)
        torch.testing.assert_close(y.cpu().double(), ref, rtol=0, atol=0)


@pytest.mark.parametrize("shape", [
    (4, 64, 56, 56, 256, 1, 1, 0),
    (2, 256, 28, 28, 128, 3, 1, 1),
    (2, 128, 29, 29, 128, 3, 2, 1),
    (1, 2048, 7, 7, 512, 1, 1, 0),
])
def test_fp32_conv_matches_fp64_reference(shape):
    """fp32 MFMA conv (+bias, ReLU) against an fp64 host convolution: fp32-level error, no reduced-precision path
    (the exact f32 MFMA mode; the bf16x3 default has its own error gate below)."""
    from synapseml_amd.ops.conv import conv2d_nhwc, pack_weight

    B, C, H, W, Co, k, st, pd = shape
    torch.manual_seed(4)
    x = torch.randn(B, C, H, W, device="cuda").contiguous(memory_format=torch.channels_last)
    w = torch.randn(Co, C, k, k, device="cuda") / (C * k * k) ** 0.5
    bias = torch.randn(Co, device="cuda")
    ref = torch.relu(F.conv2d(x.cpu().double(), w.cpu().double(), bias.cpu().double(), st, pd))
    for kernel in (0, 64064, 128128, 64128):
        y = conv2d_nhwc(x, pack_weight(w, torch.float32), k, k, (st, st), (pd, pd), bias=bias, relu=True, kernel=kernel,
                        f32_mode="exact")
        torch.testing.assert_close(y.cpu().double(), ref, rtol=1e-5, atol=2e-5, msg=lambda m: f"kernel {kernel}: {m}")
    with pytest.raises(RuntimeError):  # the 8-wave tiles are f16/bf16 only
        conv2d_nhwc(x, pack_weight(w, torch.float32), k, k, (st, st), (pd, pd), kernel=256128, f32_mode="exact")


def test_fp32_prologue_residual_dual_output():
    from synapseml_amd.ops.conv import conv2d_nhwc, pack_weight

    torch.manual_seed(5)
    B, C, H, W, Co = 2, 128, 14, 14, 256
    x = torch.randn(B, C, H, W, device="cuda").contiguous(memory_format=torch.channels_last)
    pro = (torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.1)
    res = torch.randn(B, Co, H, W, device="cuda").contiguous(memory_format=torch.channels_last)
    post = (torch.rand(Co, device="cuda") + 0.5, torch.randn(Co, device="cuda") * 0.1)
    for k in (1, 3):
        w = torch.randn(Co, C, k, k, device="cuda") / (C * k * k) ** 0.5
        y, y2 = conv2d_nhwc(x, pack_weight(w, torch.float32), k, k, (1, 1), (k // 2, k // 2), in_affine=pro,
                            res=res, out_affine=post)
        xd = torch.relu(x.cpu().double() * pro[0].cpu().double().view(1, -1, 1, 1)
                        + pro[1].cpu().double().view(1, -1, 1, 1))
        ry = F.conv2d(xd, w.cpu().double(), None, 1, k // 2) + res.cpu().double()
        ry2 = torch.relu(ry * post[0].cpu().double().view(1, -1, 1, 1) + post[1].cpu().double().view(1, -1, 1, 1))
        torch.testing.assert_close(y.cpu().double(), ry, rtol=1e-5, atol=2e-5)
        torch.testing.assert_close(y2.cpu().double(), ry2, rtol=1e-5, atol=3e-5)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_stem_packed_form_exact(dtype):
    """Few-channel stem form (kernel=1): input padded to 4 channels, weights packed to [Cout][8][8][4] with
    zero taps, one more virtual padding row / column; small integers make any tap / pixel-pair mapping error an
    exact mismatch (ResNet stem 7x7/2 pad 3, and a 5x5/1 odd-size case)."""
    from synapseml_amd.ops.conv import conv2d_nhwc

    g = torch.Generator().manual_seed(9)
    for (B, C, H, W, Co, k, st, pd) in ((2, 3, 37, 29, 64, 7, 2, 3), (3, 3, 15, 17, 40, 5, 1, 2)):
        x = torch.randint(-2, 3, (B, C, H, W), generator=g).float()
        w = torch.randint(-2, 3, (Co, C, k, k), generator=g).float()
        ref = F.conv2d(x.double(), w.double(), None, st, pd)
        x4 = torch.empty((B, 4, H, W), dtype=dtype, device="cuda", memory_format=torch.channels_last).zero_()
        x4[:, :C] = x.to(dtype).cuda()
        wp = torch.zeros((Co, 8, 8, 4), dtype=dtype, device="cuda")
        wp[:, :k, :k, :C] = w.permute(0, 2, 3, 1).to(dtype).cuda()
        y = conv2d_nhwc(x4, wp, 8, 8, (st, st), (pd, pd, pd + 8 - k, pd + 8 - k), kernel=1)
        assert y.shape == ref.shape
        torch.testing.assert_close(y.cpu().double(), ref, rtol=0, atol=0)


# ---------------------------------------------------------------- fp32 on split bf16 planes
@pytest.mark.parametrize("mode", ["bf16x3", "bf16x6"])
@pytest.mark.parametrize("kernel", [0, 64064, 64999, 128064, 64128, 128128])
def test_fp32_split_integer_layout(mode, kernel):
    """Small integers are exact in the first bf16 plane (the others are zero): any plane / k / lane / row
    mapping error of the split form is an exact mismatch."""
    from synapseml_amd.ops.conv import conv2d_nhwc, pack_weight

    g = torch.Generator().manual_seed(3)
    for (B, C, H, W, Co, k) in ((2, 32, 9, 7, 80, 3), (3, 96, 17, 11, 200, 3), (2, 64, 8, 8, 36, 1)):
        x = torch.randint(-3, 4, (B, C, H, W), generator=g).float().cuda().contiguous(memory_format=torch.channels_last)
        w = torch.randint(-3, 4, (Co, C, k, k), generator=g).float().cuda()
        y = conv2d_nhwc(x, pack_weight(w, torch.float32), k, k, (1, 1), (k // 2, k // 2), kernel=kernel, f32_mode=mode)
        ref = F.conv2d(x.cpu().double(), w.cpu().double(), None, 1, k // 2)
        torch.testing.assert_close(y.cpu().double(), ref, rtol=0, atol=0)


@pytest.mark.parametrize("shape", [
    (4, 64, 56, 56, 256, 1, 1, 0),
    (2, 256, 28, 28, 128, 3, 1, 1),
    (2, 128, 29, 29, 128, 3, 2, 1),
    (1, 2048, 7, 7, 512, 1, 1, 0),
])
def test_fp32_split_modes_error_vs_fp64(shape):
    """Error of the three fp32 modes against an fp64 convolution, relative to max |y|: bf16x6 keeps every
    product term down to the f32 rounding level (same bound as the exact f32 MFMA), bf16x3 ~16 bits per
    product (TF32, the reference's default fp32 conv math on NVIDIA tensor cores, keeps 11)."""
    from synapseml_amd.ops.conv import conv2d_nhwc, pack_weight

    B, C, H, W, Co, k, st, pd = shape
    torch.manual_seed(4)
    x = torch.randn(B, C, H, W, device="cuda").contiguous(memory_format=torch.channels_last)
    w = torch.randn(Co, C, k, k, device="cuda") / (C * k * k) ** 0.5
    bias = torch.randn(Co, device="cuda")
    ref = torch.relu(F.conv2d(x.cpu().double(), w.cpu().double(), bias.cpu().double(), st, pd))
    scale = float(ref.abs().max())
    errs = {}
    for mode in ("exact", "bf16x6", "bf16x3"):
        y = conv2d_nhwc(x, pack_weight(w, torch.float32), k, k, (st, st), (pd, pd), bias=bias, relu=True, f32_mode=mode)
        errs[mode] = float((y.cpu().double() - ref).abs().max()) / scale
    print("max |err| / max |y|:", {m: f"{e:.2e}" for m, e in errs.items()})
    assert errs["exact"] < 2e-6
    assert errs["bf16x6"] < 2e-6
    assert errs["bf16x3"] < 5e-5


def test_fp32_split_prologue_residual_dual_output():
    from synapseml_amd.ops.conv import conv2d_nhwc, pack_weight

    torch.manual_seed(5)
    B, C, H, W, Co = 2, 128, 14, 14, 256
    x = torch.randn(B, C, H, W, device="cuda").contiguous(memory_format=torch.channels_last)
    pro = (torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.1)
    res = torch.randn(B, Co, H, W, device="cuda").contiguous(memory_format=torch.channels_last)
    post = (torch.rand(Co, device="cuda") + 0.5, torch.randn(Co, device="cuda") * 0.1)
    for k in (1, 3):
        w = torch.randn(Co, C, k, k, device="cuda") / (C * k * k) ** 0.5
        y, y2 = conv2d_nhwc(x, pack_weight(w, torch.float32), k, k, (1, 1), (k // 2, k // 2), in_affine=pro,
                            res=res, out_affine=post, f32_mode="bf16x6")
        xd = torch.relu(x.cpu().double() * pro[0].cpu().double().view(1, -1, 1, 1)
                        + pro[1].cpu().double().view(1, -1, 1, 1))
        ry = F.conv2d(xd, w.cpu().double(), None, 1, k // 2) + res.cpu().double()
        ry2 = torch.relu(ry * post[0].cpu().double().view(1, -1, 1, 1) + post[1].cpu().double().view(1, -1, 1, 1))
        torch.testing.assert_close(y.cpu().double(), ry, rtol=1e-5, atol=2e-5)
        torch.testing.assert_close(y2.cpu().double(), ry2, rtol=1e-5, atol=3e-5)


@pytest.mark.parametrize("mode", ["bf16x3", "bf16x6"])
def test_fp32_presplit_weight_planes_bitwise(mode):
    """Weights split once on the host side (split_weight) give bitwise the in-kernel split's result (same
    RNE bf16 planes, same products in the same order), with and without the prologue."""
    from synapseml_amd.ops.conv import conv2d_nhwc, pack_weight, split_weight

    torch.manual_seed(7)
    B, C, H, W, Co = 2, 96, 13, 11, 160
    x = torch.randn(B, C, H, W, device="cuda").contiguous(memory_format=torch.channels_last)
    pro = (torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.1)
    for k, kernel in ((3, 0), (1, 0), (3, 64064), (1, 128999)):
        wp = pack_weight(torch.randn(Co, C, k, k, device="cuda") / (C * k * k) ** 0.5, torch.float32)
        for ia in (None, pro):
            a = conv2d_nhwc(x, wp, k, k, (1, 1), (k // 2, k // 2), in_affine=ia, f32_mode=mode, kernel=kernel)
            b = conv2d_nhwc(x, wp, k, k, (1, 1), (k // 2, k // 2), in_affine=ia, f32_mode=mode, kernel=kernel,
                            w_planes=split_weight(wp, mode))
            torch.testing.assert_close(a, b, rtol=0, atol=0)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("geom", [
    # B, C, H, W, Cout, k, stride, pad
    (4, 3, 224, 224, 64, 7, 2, 3),   # the ResNet-50 stem
    (3, 3, 37, 29, 64, 7, 2, 3),     # partial pixel tiles, padding on every border
    (2, 4, 19, 23, 128, 5, 1, 2),    # two 64-channel tiles, C = 4
    (2, 1, 16, 16, 80, 3, 1, 1),     # a partial channel tile
    (2, 3, 33, 31, 64, 5, 1, 2),     # 3 channels, 5x5 stride 1: row runs of 15 values, odd row byte offsets
    (1, 3, 17, 9, 64, 3, 3, 0),      # 3x3 stride 3 unpadded
    (2, 3, 40, 48, 64, 7, 2, 3),     # row-staged form: 24-pixel output rows, padding both sides
    (3, 3, 24, 16, 80, 5, 1, 2),     # row-staged form, stride 1, a partial channel tile
])
def test_stem_kernel_matches_reference(dtype, geom):
    """Dedicated few-channel stem kernel (im2col rows in LDS, K padded to 160) vs the fp32 reference, with
    bias + ReLU and a residual; small integers check the layout exactly."""
    from synapseml_amd.ops.conv import pack_stem_weight, stem_conv_nhwc

    B, C, H, W, Co, k, st, pd = geom
    g = torch.Generator().manual_seed(5)
    x = torch.randint(-2, 3, (B, C, H, W), generator=g).to(dtype).cuda().contiguous(memory_format=torch.channels_last)
    w = torch.randint(-2, 3, (Co, C, k, k), generator=g).to(dtype).cuda()
    y = stem_conv_nhwc(x, pack_stem_weight(w), k, k, (st, st), (pd, pd))
    ref = F.conv2d(x.float(), w.float(), None, st, pd)
    torch.testing.assert_close(y.float(), ref.to(dtype).float(), rtol=0, atol=0)  # exact sum, one rounding
    if C == 3:  # the row-run form (SML_STEM_ROWRUN) and the 2-byte gather form agree exactly
        yw = stem_conv_nhwc(x, pack_stem_weight(w, wide=True), k, k, (st, st), (pd, pd), form=1)
        torch.testing.assert_close(yw.float(), ref.to(dtype).float(), rtol=0, atol=0)
        yg = stem_conv_nhwc(x, pack_stem_weight(w), k, k, (st, st), (pd, pd), form=1)
        torch.testing.assert_close(yg.float(), ref.to(dtype).float(), rtol=0, atol=0)
        if W % 8 == 0 and ref.shape[3] <= 128:  # the row-staged form (the default where it applies)
            yr = stem_conv_nhwc(x, pack_stem_weight(w), k, k, (st, st), (pd, pd), form=2)
            torch.testing.assert_close(yr.float(), ref.to(dtype).float(), rtol=0, atol=0)
    torch.manual_seed(6)
    xf = torch.randn(B, C, H, W, device="cuda").to(dtype).contiguous(memory_format=torch.channels_last)
    wf = (torch.randn(Co, C, k, k, device="cuda") / (C * k * k) ** 0.5).to(dtype)
    bias = torch.randn(Co, device="cuda")
    res = torch.randn_like(ref).to(dtype).contiguous(memory_format=torch.channels_last)
    y2 = stem_conv_nhwc(xf, pack_stem_weight(wf), k, k, (st, st), (pd, pd), bias=bias, relu=2, res=res)
    r2 = torch.relu(F.conv2d(xf.float(), wf.float(), bias, st, pd) + res.float())
    tol = 2e-2 if dtype == torch.float16 else 8e-2
    torch.testing.assert_close(y2.float(), r2, rtol=tol, atol=tol)
    # input affine (+ ReLU) inside the im2col: padding taps stay 0 (the affine of the padded input is not)
    sc = torch.rand(C, device="cuda") + 0.5
    sh = torch.randn(C, device="cuda")
    for in_relu in (False, True):
        y3 = stem_conv_nhwc(xf, pack_stem_weight(wf), k, k, (st, st), (pd, pd), bias=bias, in_affine=(sc, sh),
                            in_relu=in_relu)
        xa = xf.float() * sc.view(1, -1, 1, 1) + sh.view(1, -1, 1, 1)
        xa = (torch.relu(xa) if in_relu else xa).to(dtype).float()
        r3 = F.conv2d(xa, wf.float(), bias, st, pd)
        torch.testing.assert_close(y3.float(), r3, rtol=tol, atol=tol)


@pytest.mark.parametrize("mode", ["bf16x3", "bf16x6"])
@pytest.mark.parametrize("geom", [
    # B, H, W, Cout, k, stride, pad
    (3, 224, 224, 64, 7, 2, 3),   # the ResNet-50 stem
    (2, 40, 48, 64, 7, 2, 3),     # 24-pixel output rows: a partial pixel tile per wave pair
    (3, 24, 16, 80, 5, 1, 2),     # stride 1, a partial channel tile (Cout % 8 == 0)
    (2, 20, 36, 36, 3, 1, 1),     # Cout % 8 != 0: the element-store epilogue
    (1, 17, 12, 64, 3, 3, 0),     # 3x3 stride 3 unpadded
])
def test_stem_f32_kernel_matches_fp64(mode, geom):
    """fp32 stem on bf16 planes (stem_f32_kernel) vs an fp64 convolution: small integers (exact in one plane)
    check the layout bit for bit; random data stays within the tiled fp32 modes' error gate (bf16x3: 1e-5
    of max |y|; bf16x6: 1e-6), with bias + ReLU + residual and with the fused input affine (+ ReLU)."""
    from synapseml_amd.ops.conv import pack_stem_weight_f32, stem_conv_nhwc, stem_f32_supported

    B, H, W, Co, k, st, pd = geom
    g = torch.Generator().manual_seed(7)
    x = torch.randint(-3, 4, (B, 3, H, W), generator=g).float().cuda().contiguous(memory_format=torch.channels_last)
    w = torch.randint(-3, 4, (Co, 3, k, k), generator=g).float().cuda()
    assert stem_f32_supported(x, w, (st, st), (pd, pd), (1, 1), mode)
    y = stem_conv_nhwc(x, pack_stem_weight_f32(w, mode), k, k, (st, st), (pd, pd))
    ref = F.conv2d(x.double(), w.double(), None, st, pd)
    torch.testing.assert_close(y.double(), ref, rtol=0, atol=0)
    torch.manual_seed(8)
    xf = torch.randn(B, 3, H, W, device="cuda").contiguous(memory_format=torch.channels_last)
    wf = torch.randn(Co, 3, k, k, device="cuda") / (3 * k * k) ** 0.5
    bias = torch.randn(Co, device="cuda")
    res = torch.randn_like(ref.float()).contiguous(memory_format=torch.channels_last)
    gate = 1e-5 if mode == "bf16x3" else 1e-6
    wk = pack_stem_weight_f32(wf, mode)
    y2 = stem_conv_nhwc(xf, wk, k, k, (st, st), (pd, pd), bias=bias, relu=2, res=res)
    r2 = torch.relu(F.conv2d(xf.double(), wf.double(), bias.double(), st, pd) + res.double())
    assert (y2.double() - r2).abs().max().item() <= gate * r2.abs().max().item()
    sc = torch.rand(3, device="cuda") + 0.5
    sh = torch.randn(3, device="cuda")
    for in_relu in (False, True):
        y3 = stem_conv_nhwc(xf, wk, k, k, (st, st), (pd, pd), bias=bias, relu=1, in_affine=(sc, sh), in_relu=in_relu)
        xa = xf.double() * sc.double().view(1, -1, 1, 1) + sh.double().view(1, -1, 1, 1)
        xa = torch.relu(xa) if in_relu else xa
        r3 = torch.relu(F.conv2d(xa, wf.double(), bias.double(), st, pd))
        assert (y3.double() - r3).abs().max().item() <= gate * r3.abs().max().item()


_RING_GEOMS = [
    # B, H, W, Cout, k, stride, pad
    (3, 224, 224, 64, 7, 2, 3),   # the ResNet-50 stem: 14 strips of 8 output rows
    (2, 40, 48, 64, 7, 2, 3),     # a partial last strip (OH = 20), a partial pixel tile
    (2, 36, 40, 80, 5, 2, 2),     # a partial channel tile, even pad
    (2, 21, 24, 36, 3, 2, 1),     # Cout % 8 != 0 (element-store epilogue), odd H
    (1, 30, 32, 64, 8, 2, 3),     # 8 x 8 taps: K = 192, every run slot real
]


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16, torch.float32, "fp32-bf16x6"])
@pytest.mark.parametrize("geom", _RING_GEOMS)
def test_stem_ring_kernel_matches_reference(dtype, geom):
    """The strip form of the stride-2 RGB stem (input rows in an LDS ring, fragments read straight from the
    staged rows): small integers exact against the reference (f16 / bf16, and fp32 on bf16 planes), random data
    within each precision's gate, with bias + ReLU + residual and the fused input affine (+ ReLU)."""
    from synapseml_amd.ops.conv import pack_stem_weight, pack_stem_weight_f32, stem_conv_nhwc, stem_ring_ok

    B, H, W, Co, k, st, pd = geom
    mode = "bf16x6" if dtype == "fp32-bf16x6" else "bf16x3"
    dtype = torch.float32 if dtype == "fp32-bf16x6" else dtype
    f32 = dtype == torch.float32
    pack = (lambda t: pack_stem_weight_f32(t, mode, wide=True)) if f32 else (lambda t: pack_stem_weight(t, wide=True))
    g = torch.Generator().manual_seed(11)
    x = torch.randint(-3, 4, (B, 3, H, W), generator=g).to(dtype).cuda().contiguous(memory_format=torch.channels_last)
    w = torch.randint(-3, 4, (Co, 3, k, k), generator=g).to(dtype).cuda()
    assert stem_ring_ok(x, w, (st, st), (pd, pd), (1, 1), (3 if mode == "bf16x6" else 2) if f32 else 1)
    if k * k * 3 > 160:  # the Python front end's K bound (the strip form itself takes R * 24 <= 192)
        with pytest.raises(ValueError):
            stem_conv_nhwc(x, pack(w), k, k, (st, st), (pd, pd), form=3)
        return
    y = stem_conv_nhwc(x, pack(w), k, k, (st, st), (pd, pd), form=3)
    ref = F.conv2d(x.double(), w.double(), None, st, pd)
    torch.testing.assert_close(y.double(), ref.to(dtype).double(), rtol=0, atol=0)
    torch.manual_seed(12)
    xf = torch.randn(B, 3, H, W, device="cuda").to(dtype).contiguous(memory_format=torch.channels_last)
    wf = (torch.randn(Co, 3, k, k, device="cuda") / (3 * k * k) ** 0.5).to(dtype)
    bias = torch.randn(Co, device="cuda")
    res = torch.randn(ref.shape, device="cuda").to(dtype).contiguous(memory_format=torch.channels_last)
    wk = pack(wf)
    y2 = stem_conv_nhwc(xf, wk, k, k, (st, st), (pd, pd), bias=bias, relu=2, res=res, form=3)
    r2 = torch.relu(F.conv2d(xf.double(), wf.double(), bias.double(), st, pd) + res.double())
    sc = torch.rand(3, device="cuda") + 0.5
    sh = torch.randn(3, device="cuda")
    outs = [(y2, r2)]
    for in_relu in (False, True):
        y3 = stem_conv_nhwc(xf, wk, k, k, (st, st), (pd, pd), bias=bias, relu=1, in_affine=(sc, sh), in_relu=in_relu,
                            form=3)
        xa = xf.double() * sc.double().view(1, -1, 1, 1) + sh.double().view(1, -1, 1, 1)
        xa = torch.relu(xa) if in_relu else xa
        if not f32:
            xa = xa.to(dtype).double()  # the kernel rounds the affine'd input to the storage type
        outs.append((y3, torch.relu(F.conv2d(xa, wf.double(), bias.double(), st, pd))))
    for yy, rr in outs:
        if f32:
            gate = 1e-6 if mode == "bf16x6" else 1e-5
            assert (yy.double() - rr).abs().max().item() <= gate * rr.abs().max().item()
        else:
            tol = 2e-2 if dtype == torch.float16 else 8e-2
            torch.testing.assert_close(yy.double(), rr, rtol=tol, atol=tol)
    # the strip form and the row-staged form agree (f16 / bf16: both one rounding of an fp32 sum)
    if not f32 and W % 8 == 0 and ref.shape[3] <= 128 and k * k * 3 <= 160:
        yr = stem_conv_nhwc(xf, pack_stem_weight(wf), k, k, (st, st), (pd, pd), bias=bias, relu=2, res=res, form=2)
        torch.testing.assert_close(y2.float(), yr.float(), rtol=1e-2, atol=1e-2)


def test_resnet_fp32_session_stem_uses_f32_kernel():
    """An fp32 graph's 3-channel stem with its input BatchNormalization: the BN rides the bf16-plane stem
    kernel (no separate affine pass), and the output matches an fp64 reference within the fp32 conv gate."""
    import numpy as np

    from synapseml_amd.onnx import InferenceSession, proto as P
    from synapseml_amd.onnx.writer import GraphBuilder

    rng = np.random.default_rng(3)
    gb = GraphBuilder("stem32")
    gb.input("x", P.FLOAT32, ["N", 3, 64, 64])
    prm = [gb.init("s", (rng.random(3) + 0.5).astype(np.float32)),
           gb.init("t", rng.standard_normal(3).astype(np.float32)),
           gb.init("m", (rng.standard_normal(3) * 0.1).astype(np.float32)),
           gb.init("v", (rng.random(3) + 0.5).astype(np.float32))]
    xb = gb.add("BatchNormalization", ["x"] + prm, {"epsilon": 1e-5})
    w = gb.init("w", (rng.standard_normal((64, 3, 7, 7)) / 12).astype(np.float32))
    bb = gb.init("b", rng.standard_normal(64).astype(np.float32))
    c = gb.add("Conv", [xb, w, bb], {"kernel_shape": [7, 7], "pads": [3, 3, 3, 3], "strides": [2, 2]})
    gb.add("Relu", [c], out="y")
    gb.output("y", P.FLOAT32, None)
    sess = InferenceSession(gb.to_bytes(), device="cuda", precision="fp32")
    stem = [n for n in sess.nodes if sess._stem_conv_node(n)]
    assert len(stem) == 1 and stem[0].inputs[0] == "x" and len(stem[0].inputs) == 6  # the BN is the prologue
    xin = rng.standard_normal((2, 3, 64, 64)).astype(np.float32)
    y = np.asarray(sess.run(None, {"x": xin})[0], dtype=np.float64)
    it = {k: torch.from_numpy(gb.inits[k]).double().view(1, -1, 1, 1) for k in ("s", "t", "m", "v")}
    xr = (torch.from_numpy(xin).double() - it["m"]) / torch.sqrt(it["v"] + 1e-5) * it["s"] + it["t"]
    ref = torch.relu(F.conv2d(xr, torch.from_numpy(gb.inits["w"]).double(),
                              torch.from_numpy(gb.inits["b"]).double(), 2, 3)).numpy()
    assert np.abs(y - ref).max() <= 1e-5 * np.abs(ref).max()


_RESNET50_SHAPES = [  # C, H, Cout, k, stride (tools/bench_conv.py SHAPES: the 14 bottleneck layer shapes)
    (64, 56, 64, 1, 1), (64, 56, 64, 3, 1), (64, 56, 256, 1, 1), (256, 56, 64, 1, 1),
    (128, 28, 128, 3, 1), (128, 28, 512, 1, 1), (512, 28, 128, 1, 1), (256, 56, 512, 1, 2),
    (256, 14, 256, 3, 1), (256, 14, 1024, 1, 1), (1024, 14, 256, 1, 1),
    (512, 7, 512, 3, 1), (512, 7, 2048, 1, 1), (2048, 7, 512, 1, 1),
]


@pytest.mark.parametrize("shape", _RESNET50_SHAPES)
def test_fp32_default_mode_error_gate_resnet50(shape):
    """The default fp32 conv mode (bf16x3 unless SML_CONV_F32 says otherwise) stays within 1e-5 of max |y| of
    an fp64 convolution on every ResNet-50 layer shape (TF32 would be ~1e-3)."""
    from synapseml_amd.ops.conv import conv2d_nhwc, f32_mode_default, pack_weight

    C, H, Co, k, st = shape
    torch.manual_seed(sum(shape))
    x = torch.randn(2, C, H, H, device="cuda").contiguous(memory_format=torch.channels_last)
    w = torch.randn(Co, C, k, k, device="cuda") / (C * k * k) ** 0.5
    bias = torch.randn(Co, device="cuda")
    pd = k // 2
    ref = torch.relu(F.conv2d(x.cpu().double(), w.cpu().double(), bias.cpu().double(), st, pd))
    y = conv2d_nhwc(x, pack_weight(w, torch.float32), k, k, (st, st), (pd, pd), bias=bias, relu=True)
    err = float((y.cpu().double() - ref).abs().max()) / float(ref.abs().max())
    print(f1 := f"{f32_mode_default()} {shape}: max |err| / max |y| = {err:.2e}")
    assert err <= 1e-5, f1
