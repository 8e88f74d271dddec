"""Image stage tests (model: reference opencv/src/test/scala/.../ImageTransformerSuite.scala,
ImageSetAugmenterSuite.scala, core image UnrollImageSuite). OpenCV itself is not available here:
fixed-point resize / luma values are checked against hand-computed OpenCV arithmetic; GPU
kernels are checked bit-for-bit against the host path."""
import numpy as np
import pytest

from synapseml_amd.core.dataframe import DataFrame
from synapseml_amd.image import (ImageSetAugmenter, ImageTransformer, UnrollBinaryImage, UnrollImage,
                                 decode_bytes, encode_png, make_image_row, row_to_array, unroll)
from synapseml_amd.ops import native


def _df(*arrays):
    col = np.empty(len(arrays), dtype=object)
    for i, a in enumerate(arrays):
        col[i] = make_image_row(a, f"img{i}")
    return DataFrame({"image": col})


def test_png_roundtrip_bgr_order():
    a = np.random.default_rng(0).integers(0, 256, (5, 7, 3), dtype=np.uint8)
    np.testing.assert_array_equal(decode_bytes(encode_png(a)), a)
    g = np.random.default_rng(1).integers(0, 256, (5, 7, 1), dtype=np.uint8)
    np.testing.assert_array_equal(decode_bytes(encode_png(g)), g)


def test_resize_dims_and_fixed_point():
    a = np.random.default_rng(0).integers(0, 256, (40, 60, 3), dtype=np.uint8)
    out = ImageTransformer(outputCol="o").resize(15, 10).transform(_df(a))["o"][0]
    assert (out["height"], out["width"]) == (15, 10)
    img = native.load("_image")
    src = np.array([[0, 100], [200, 50]], dtype=np.uint8)[:, :, None]
    assert img.resize(src, 1, 1).reshape(-1)[0] == 88  # (0+100+200+50)/4 = 87.5 rounds up in 22-bit fixed point
    const = np.full((9, 13, 3), 77, np.uint8)
    assert (img.resize(const, 20, 7) == 77).all()
    # keep aspect ratio: shorter side -> size
    out = ImageTransformer(outputCol="o").resize(20, True).transform(_df(a))["o"][0]
    assert (out["height"], out["width"]) == (20, 30)


def test_tensor_normalization_red_image():
    red = np.zeros((8, 8, 3), np.uint8)
    red[:, :, 2] = 255
    t = ImageTransformer(outputCol="t").normalize([0.5, 0.5, 0.5], [1.0, 1.0, 1.0], 1 / 255).setDeviceType("cpu")
    v = t.transform(_df(red))["t"][0]
    assert v.shape == (3, 8, 8)
    assert np.allclose(v[0], 0.5) and np.allclose(v[1], -0.5) and np.allclose(v[2], -0.5)
    bgr = t.copy().setTensorChannelOrder("BGR").transform(_df(red))["t"][0]
    assert np.allclose(bgr[2], 0.5)
    dbl = t.copy().setTensorElementType("double").transform(_df(red))["t"][0]
    assert dbl.dtype == np.float64


def test_color_threshold_flip_blur_gaussian():
    img = native.load("_image")
    px = np.array([[[255, 0, 0], [0, 255, 0], [0, 0, 255]]], np.uint8)  # BGR blue, green, red
    gray = img.cvt_color(px, 6).reshape(-1)
    assert gray.tolist() == [29, 150, 76]
    x = np.array([[10, 100, 200]], np.uint8)[:, :, None]
    assert img.threshold(x, 100, 255, 0).reshape(-1).tolist() == [0, 0, 255]
    assert img.threshold(x, 100, 255, 1).reshape(-1).tolist() == [255, 255, 0]
    assert img.threshold(x, 100, 255, 2).reshape(-1).tolist() == [10, 100, 100]
    assert img.threshold(x, 100, 255, 3).reshape(-1).tolist() == [0, 0, 200]
    assert img.threshold(x, 100, 255, 4).reshape(-1).tolist() == [10, 100, 0]
    a = np.random.default_rng(2).integers(0, 256, (11, 9, 3), dtype=np.uint8)
    df = _df(a)
    f = ImageTransformer(outputCol="o").flip(1).transform(df)["o"][0]
    np.testing.assert_array_equal(row_to_array(f), a[:, ::-1])
    const = np.full((6, 6, 1), 40, np.uint8)
    assert (img.box_blur(const, 3, 5) == 40).all()
    # box blur interior = mean of the window
    b = img.box_blur(a, 3, 3)
    assert b[5, 4, 1] == int(np.floor(a[4:7, 3:6, 1].mean() + 0.5)) or \
        abs(int(b[5, 4, 1]) - a[4:7, 3:6, 1].mean()) <= 0.5
    k = np.asarray(img.gaussian_kernel(5, 0.0))
    np.testing.assert_allclose(k, [0.0625, 0.25, 0.375, 0.25, 0.0625])
    k2 = np.asarray(img.gaussian_kernel(7, 1.5))
    assert abs(k2.sum() - 1) < 1e-12 and k2[3] == k2.max()
    gauss = ImageTransformer(outputCol="o").gaussianKernel(5, 0).transform(df)["o"][0]
    g = row_to_array(gauss).astype(int)
    ref = sum(kk * a[min(max(3 + j - 2, 0), 10), 4, 0].astype(float) for j, kk in enumerate(k))
    assert abs(g[3, 4, 0] - ref) <= 0.5 + 1e-9


def test_center_crop_and_stage_chain():
    a = np.random.default_rng(3).integers(0, 256, (30, 40, 3), dtype=np.uint8)
    out = ImageTransformer(outputCol="o").centerCrop(10, 20).transform(_df(a))["o"][0]
    np.testing.assert_array_equal(row_to_array(out), a[10:20, 10:30])
    out = (ImageTransformer(outputCol="o").resize(30, 40).crop(1, 2, 5, 6).colorFormat(6)
           .transform(_df(a))["o"][0])
    assert (out["height"], out["width"], out["nChannels"]) == (5, 6, 1)


def test_decoding_errors_and_binary_input():
    good = encode_png(np.zeros((4, 4, 3), np.uint8))
    col = np.empty(2, dtype=object)
    col[0] = good
    col[1] = b"not an image"
    df = DataFrame({"image": col})
    with pytest.raises(Exception):
        ImageTransformer(outputCol="o").resize(2, 2).transform(df)
    out = ImageTransformer(outputCol="o").resize(2, 2).setIgnoreDecodingErrors(True).transform(df)
    assert out["o"][0]["height"] == 2 and out["o"][1] is None


def test_augmenter_and_unroll():
    a = np.random.default_rng(4).integers(1, 256, (3, 4, 3), dtype=np.uint8)
    df = _df(a)
    aug = ImageSetAugmenter(outputCol="o", flipUpDown=True).transform(df)
    assert aug.count() == 3
    np.testing.assert_array_equal(row_to_array(aug["o"][1]), a[:, ::-1])
    np.testing.assert_array_equal(row_to_array(aug["o"][2]), a[::-1])
    u = UnrollImage(outputCol="u").transform(df)["u"][0].toArray()
    np.testing.assert_array_equal(u, a.transpose(2, 0, 1).reshape(-1).astype(float))
    z = np.zeros((1, 1, 3), np.uint8)
    assert unroll(make_image_row(z)).tolist() == [256.0, 256.0, 256.0]  # reference quirk
    b = DataFrame({"image": np.array([encode_png(a)], dtype=object)})
    v = UnrollBinaryImage(outputCol="v", width=2, height=2).transform(b)["v"][0]
    assert len(v.toArray()) == 12


@pytest.mark.gpu
def test_gpu_fused_preprocess_bit_exact():
    import torch

    rng = np.random.default_rng(5)
    arrays = [rng.integers(0, 256, (h, w, c), dtype=np.uint8)
              for h, w, c in [(37, 53, 3), (224, 224, 3), (300, 120, 3), (64, 64, 3)]]
    t = (ImageTransformer(outputCol="o").resize(height=96, width=80).centerCrop(64, 64)
         .normalize([0.485, 0.456, 0.406], [0.229, 0.224, 0.225], 1 / 255))
    dev = t.device_tensors(arrays)
    assert dev is not None and dev.is_cuda and dev.shape == (4, 3, 64, 64)
    host = np.stack([t.process_host(a) for a in arrays])
    np.testing.assert_array_equal(dev.cpu().numpy(), host)
    nhwc = t.device_tensors(arrays, nhwc=True)
    np.testing.assert_array_equal(nhwc.contiguous().cpu().numpy(), host)
    half = t.device_tensors(arrays, dtype="float16")
    np.testing.assert_allclose(half.float().cpu().numpy(), host, atol=2e-3, rtol=1e-3)
    gray = [rng.integers(0, 256, (50, 40, 1), dtype=np.uint8) for _ in range(3)]
    tg = (ImageTransformer(outputCol="o").setAutoConvertToColor(True).resize(height=32, width=32)
          .normalize([0.5] * 3, [0.25] * 3, 1 / 255))
    np.testing.assert_array_equal(tg.device_tensors(gray).cpu().numpy(), np.stack([tg.process_host(a) for a in gray]))
    # end-to-end transform on the GPU path equals the CPU path
    col = np.empty(len(arrays), dtype=object)
    for i, a in enumerate(arrays):
        col[i] = make_image_row(a)
    df = DataFrame({"image": col})
    g = t.copy().setDeviceType("gpu").transform(df)["o"]
    c = t.copy().setDeviceType("cpu").transform(df)["o"]
    for x, y in zip(g, c):
        np.testing.assert_array_equal(x, y)
    del torch


@pytest.mark.gpu
def test_gpu_stage_kernels_match_host():
    import torch

    img = native.load("_image")
    rng = np.random.default_rng(6)
    B, h, w, c = 3, 31, 45, 3
    a = rng.integers(0, 256, (B, h, w, c), dtype=np.uint8)
    src = torch.from_numpy(a).cuda()
    stream = torch.cuda.current_stream().cuda_stream
    out = torch.empty((B, 20, 17, c), dtype=torch.uint8, device="cuda")
    img.resize_batch_device(src.data_ptr(), B, h, w, c, out.data_ptr(), 20, 17, stream)
    ref = np.stack([img.resize(x, 20, 17) for x in a])
    np.testing.assert_array_equal(out.cpu().numpy(), ref)
    bl = torch.empty_like(src)
    img.box_blur_batch_device(src.data_ptr(), B, h, w, c, bl.data_ptr(), 3, 5, stream)
    np.testing.assert_array_equal(bl.cpu().numpy(), np.stack([img.box_blur(x, 3, 5) for x in a]))
    k = img.gaussian_kernel(7, 1.3)
    gs = torch.empty_like(src)
    img.column_filter_batch_device(src.data_ptr(), B, h, w, c, gs.data_ptr(), k, stream)
    np.testing.assert_array_equal(gs.cpu().numpy(), np.stack([img.column_filter(x, k) for x in a]))
    th = torch.empty_like(src)
    img.threshold_device(src.data_ptr(), src.numel(), th.data_ptr(), 120.5, 200, 2, stream)
    np.testing.assert_array_equal(th.cpu().numpy(), img.threshold(a.reshape(-1, w, c), 120.5, 200, 2).reshape(a.shape))
    fl = torch.empty_like(src)
    img.flip_batch_device(src.data_ptr(), B, h, w, c, fl.data_ptr(), -1, stream)
    np.testing.assert_array_equal(fl.cpu().numpy(), a[:, ::-1, ::-1])
    gr = torch.empty((B, h, w, 1), dtype=torch.uint8, device="cuda")
    img.cvt_color_device(src.data_ptr(), B * h * w, 3, 6, gr.data_ptr(), stream)
    np.testing.assert_array_equal(gr.cpu().numpy().reshape(-1), img.cvt_color(a.reshape(-1, w, c), 6).reshape(-1))


def test_named_stage_maps_match_builder():
    from synapseml_amd.image import CenterCropImage, Flip, ImageTransformer, ResizeImage

    t = ImageTransformer().resize(height=8, width=6).centerCrop(4, 4).flip(1)
    assert t.getStages() == [ResizeImage.make(height=8, width=6), CenterCropImage.make(height=4, width=4),
                             Flip.make(flipCode=1)]


def test_reference_action_keyed_stage_list():
    """Stage maps keyed by "action" (ImageTransformerStage.stageNameKey, ImageTransformer.scala:39) as the
    reference's builder methods emit them; legacy "stageName" maps are still accepted."""
    from synapseml_amd.image.transformer import ResizeImage, stage_action

    rng = np.random.default_rng(5)
    img = rng.integers(0, 256, size=(40, 30, 3), dtype=np.uint8)
    df = _df(img)
    ref_style = [{"action": "resize", "height": 20, "width": 16},
                 {"action": "centercrop", "height": 10, "width": 8},
                 {"action": "flip", "flipCode": 1}]
    out = ImageTransformer(outputCol="out", stages=ref_style).transform(df)
    built = ImageTransformer(outputCol="out").resize(20, 16).centerCrop(10, 8).flip(1)
    assert built.getStages() == ref_style
    np.testing.assert_array_equal(row_to_array(out["out"][0]), row_to_array(built.transform(df)["out"][0]))
    legacy = [{"stageName": s["action"], **{k: v for k, v in s.items() if k != "action"}} for s in ref_style]
    out2 = ImageTransformer(outputCol="out", stages=legacy).transform(df)
    np.testing.assert_array_equal(row_to_array(out["out"][0]), row_to_array(out2["out"][0]))
    assert ResizeImage.make(height=1, width=2)["action"] == "resize"
    assert stage_action({"action": "blur"}) == "blur"
    with pytest.raises(KeyError):
        stage_action({"height": 3})


def _jpeg(a, **kw):
    import io

    from PIL import Image

    b = io.BytesIO()
    Image.fromarray(a).save(b, "JPEG", **kw)
    return b.getvalue()


def _noise_image(h, w, seed=0):
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w]
    base = np.stack([x * 255 // max(w - 1, 1), y * 255 // max(h - 1, 1), ((x + y) * 3) % 256], -1)
    return np.clip(base + rng.normal(0, 20, (h, w, 3)), 0, 255).astype(np.uint8)


@pytest.mark.parametrize("shape", [(1, 1), (7, 9), (17, 33), (224, 224), (101, 67)])
def test_native_jpeg_decoder_matches_pil(shape):
    """csrc/image/jpeg_decode.cpp reproduces libjpeg's ISLOW IDCT, fancy upsampling and YCbCr tables: the
    pixels equal PIL's decode exactly for 4:4:4 / 4:2:2 / 4:2:0, gray, restart intervals and optimised
    Huffman tables; progressive files are declined (-> PIL)."""
    import io

    from PIL import Image

    from synapseml_amd.image.schema import decode_jpeg_native

    a = _noise_image(*shape)
    files = [_jpeg(a, quality=q, subsampling=s) for q in (50, 95) for s in (0, 1, 2)]
    files += [_jpeg(a[:, :, 0]), _jpeg(a, restart_marker_blocks=3), _jpeg(a, optimize=True)]
    for d in files:
        with Image.open(io.BytesIO(d)) as im:
            ref = np.asarray(im)
        got = decode_jpeg_native(d)
        assert got is not None
        np.testing.assert_array_equal(got, ref if ref.ndim == 3 else ref[:, :, None])
    assert decode_jpeg_native(_jpeg(a, progressive=True)) is None
    d = files[0]
    assert decode_jpeg_native(d[: len(d) // 2]) is None  # truncated entropy data
    assert decode_jpeg_native(b"not a jpeg") is None


def test_pack_decoded_mixed_batch():
    """pack_decoded: native JPEGs, a progressive JPEG and a PNG (PIL; all RGB order), an image row (OpenCV
    order) and undecodable values share one buffer; every slot holds the right pixels."""
    import io

    from PIL import Image

    from synapseml_amd.image.schema import pack_decoded

    a = _noise_image(20, 30, 1)
    b = _noise_image(12, 8, 2)
    vals = [_jpeg(a), _jpeg(a, progressive=True), encode_png(b), make_image_row(b), b"garbage", None, _jpeg(b[:, :, 1])]
    buf, offs, shapes, rgb, ok = pack_decoded(vals, ignore_errors=True, threads=3)
    assert ok == [True, True, True, True, False, False, True]

    def slot(i):
        return buf[offs[i]:offs[i] + int(np.prod(shapes[i]))].reshape(shapes[i])

    with Image.open(io.BytesIO(vals[0])) as im:
        np.testing.assert_array_equal(slot(0), np.asarray(im))
    assert rgb[0] and rgb[1] and rgb[2] and not rgb[3]  # PIL decodes RGB-mode files in RGB order too
    with Image.open(io.BytesIO(vals[1])) as im:
        np.testing.assert_array_equal(slot(1), np.asarray(im))
    np.testing.assert_array_equal(slot(2), b[:, :, ::-1])  # encode_png took OpenCV order
    np.testing.assert_array_equal(slot(3), b)
    assert shapes[6] == (12, 8, 1)
    with pytest.raises(Exception):
        pack_decoded([b"garbage"], ignore_errors=False)


@pytest.mark.gpu
@pytest.mark.parametrize("c", [1, 3, 4])
def test_gpu_stage_pipeline_matches_host(c):
    """Every image-output stage list runs on the device (batched K20 launches on resident images) and is
    bit-identical to the host path (deviceType="cpu"): odd widths (row tails not a multiple of 4 bytes),
    1 / 3 / 4 channels, keepAspectRatio resize, reflected large blur / gaussian windows, threshold types,
    all flip codes, colour conversion and toTensor after the stages."""
    from synapseml_amd.image import ImageTransformer
    from synapseml_amd.image.schema import make_image_row

    rng = np.random.default_rng(11)
    imgs = [rng.integers(0, 256, (37, 53, c), dtype=np.uint8) for _ in range(5)] + \
           [rng.integers(0, 256, (64, 48, c), dtype=np.uint8) for _ in range(3)]
    df = DataFrame({"image": [make_image_row(a, f"o{i}") for i, a in enumerate(imgs)]})
    conv = {1: 8, 3: 6, 4: 3}[c]  # GRAY2BGR / BGR2GRAY / BGRA2BGR
    lists = [
        lambda t: t.resize(height=29, width=31).centerCrop(17, 19).flip(1),
        lambda t: t.resize(size=40, keep_aspect_ratio=True).crop(3, 2, 21, 23).flip(0),
        lambda t: t.blur(9, 5).threshold(100.7, 250, 1).flip(-1),
        lambda t: t.gaussianKernel(9, 2.1).threshold(90, 200, 4),
        lambda t: t.colorFormat(conv).resize(height=22, width=27),
        lambda t: t.resize(height=30, width=30).blur(3, 3).normalize([0.5] * (3 if c != 1 else 1),
                                                                     [0.25] * (3 if c != 1 else 1), 1 / 255.0),
    ]
    for build in lists:
        g = build(ImageTransformer(inputCol="image", outputCol="o", deviceType="gpu")).transform(df)["o"]
        h = build(ImageTransformer(inputCol="image", outputCol="o", deviceType="cpu")).transform(df)["o"]
        for x, y in zip(g, h):
            if isinstance(x, dict):
                assert (x["height"], x["width"], x["nChannels"]) == (y["height"], y["width"], y["nChannels"])
                assert x["data"] == y["data"] and x["origin"] == y["origin"]
            else:
                np.testing.assert_array_equal(np.asarray(x), np.asarray(y))


@pytest.mark.gpu
def test_gpu_stage_kernels_reflect_and_tails():
    """The K20 kernels on shapes that stress their tables: blur / gaussian windows larger than the image
    (repeated BORDER_REFLECT_101), 1-pixel images, row lengths with 1-3 byte tails."""
    import torch

    img = native.load("_image")
    rng = np.random.default_rng(7)
    stream = torch.cuda.current_stream().cuda_stream
    for (h, w, c) in [(1, 1, 3), (2, 3, 1), (5, 7, 3), (9, 2, 4)]:
        a = rng.integers(0, 256, (2, h, w, c), dtype=np.uint8)
        src = torch.from_numpy(a).cuda()
        bl = torch.empty_like(src)
        img.box_blur_batch_device(src.data_ptr(), 2, h, w, c, bl.data_ptr(), 11, 7, stream)
        np.testing.assert_array_equal(bl.cpu().numpy(), np.stack([img.box_blur(x, 11, 7).reshape(h, w, c) for x in a]))
        k = img.gaussian_kernel(13, 3.0)
        gs = torch.empty_like(src)
        img.column_filter_batch_device(src.data_ptr(), 2, h, w, c, gs.data_ptr(), k, stream)
        np.testing.assert_array_equal(gs.cpu().numpy(),
                                      np.stack([img.column_filter(x, k).reshape(h, w, c) for x in a]))
        rs = torch.empty((2, 3, 5, c), dtype=torch.uint8, device="cuda")
        img.resize_batch_device(src.data_ptr(), 2, h, w, c, rs.data_ptr(), 3, 5, stream)
        np.testing.assert_array_equal(rs.cpu().numpy(), np.stack([img.resize(x, 3, 5).reshape(3, 5, c) for x in a]))


def test_native_batch_copy_helpers():
    """The host side of a device batch (transformer.py): images gathered into one buffer, per-row bytes split
    out of it and a bulk copy, by the native thread team - the same bytes as the numpy copies they replace."""
    import numpy as np

    from synapseml_amd.image.transformer import _bulk_copy, _gather_images, _image_rows
    from synapseml_amd.image.schema import make_image_row

    rng = np.random.default_rng(4)
    imgs = [rng.integers(0, 256, (61, 47, 3), dtype=np.uint8) for _ in range(40)]
    srcs = [im if k % 2 else im.tobytes() for k, im in enumerate(imgs)]  # arrays and row bytes
    dst = np.zeros((48, 61, 47, 3), np.uint8)
    _gather_images(dst, [np.frombuffer(s, np.uint8).reshape(61, 47, 3) if isinstance(s, bytes) else s
                         for s in srcs])
    assert np.array_equal(dst[:40], np.stack(imgs)) and not dst[40:].any()
    strided = [im[:, ::-1] for im in imgs[:9]]  # non-contiguous: the pool fallback
    _gather_images(dst, strided)
    assert np.array_equal(dst[:9], np.stack(strided))
    _gather_images(dst, imgs)
    rows = _image_rows(dst, 40, [f"o{k}" for k in range(40)])
    for k in range(40):
        assert rows[k] == make_image_row(imgs[k], f"o{k}")
    gray = rng.integers(0, 256, (5, 33, 20), dtype=np.uint8)
    assert _image_rows(gray, 5, list("abcde"))[3] == make_image_row(gray[3], "d")
    big = rng.standard_normal((7, 3, 224, 224)).astype(np.float32)
    out = _bulk_copy(big, 6)
    assert np.array_equal(out, big[:6]) and not np.shares_memory(out, big)
