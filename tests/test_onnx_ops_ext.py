"""Extended ONNX operator set (synapseml_amd/onnx/ops_ext.py) against independent numpy / torch references.
Every case runs on the CPU; the `gpu` variants run the same graphs on the MI355X device. onnxruntime is not
installed here, so the references are the operator specifications written out in numpy (parity with ORT
itself is unpinned)."""
import math

import numpy as np
import pytest
import torch

from synapseml_amd.onnx import Graph, InferenceSession, proto as P
from synapseml_amd.onnx.graph import Node, ValueInfo
from synapseml_amd.onnx.writer import GraphBuilder


def _elem(a) -> int:
    a = np.asarray(a)
    if a.dtype == object or a.dtype.kind in "US":
        return P.STRING
    return P.ONNX_OF[a.dtype]


def run1(op_type, inputs, attrs=None, n_out=1, domain="", device="cpu", opset=None):
    """one-node graph: `inputs` = list of (name, array) ('' name = omitted optional input)"""
    b = GraphBuilder(op_type)
    names = []
    for name, arr in inputs:
        if not name:
            names.append("")
            continue
        b.input(name, _elem(arr), list(np.shape(arr)))
        names.append(name)
    outs = b.add(op_type, names, attrs or {}, out="y" if n_out == 1 else None, n_out=n_out, domain=domain)
    outs = [outs] if n_out == 1 else outs
    for o in outs:
        b.output(o, P.FLOAT32, None)
    sess = InferenceSession(b.to_bytes(opset=opset), device=device, optimization_level="NO_OPT")
    feeds = {name: arr for name, arr in inputs if name}
    return sess.run(None, feeds)


def _sub(nodes, inputs, outputs, inits=None, name="body"):
    g = Graph()
    g.name = name
    g.nodes = nodes
    g.inputs = inputs
    g.outputs = outputs
    g.initializers = dict(inits or {})
    return g


# ------------------------------------------------------------------ control flow
def test_loop_carried_scan_outputs_cond_and_outer_scope():
    # body: v' = v + i * c (c from the OUTER graph), scan out = v' * 2, cond' = v' < limit
    body = _sub([Node("Cast", ["i"], ["i_f"], {"to": P.FLOAT32}, "cast"),
                 Node("Mul", ["i_f", "c"], ["ic"], {}, "mul"),
                 Node("Add", ["v", "ic"], ["v2"], {}, "add"),
                 Node("Mul", ["v2", "two"], ["s"], {}, "dbl"),
                 Node("ReduceSum", ["v2"], ["tot"], {"keepdims": 0}, "rs"),
                 Node("Less", ["tot", "limit"], ["cond_out"], {}, "less")],
                [ValueInfo("i", elem_type=P.INT64, shape=[]), ValueInfo("cond_in", elem_type=P.BOOL, shape=[]),
                 ValueInfo("v", elem_type=P.FLOAT32, shape=[2])],
                [ValueInfo("cond_out", elem_type=P.BOOL, shape=[]), ValueInfo("v2", elem_type=P.FLOAT32, shape=[2]),
                 ValueInfo("s", elem_type=P.FLOAT32, shape=[2])],
                {"two": np.array(2.0, np.float32), "limit": np.array(40.0, np.float32)})
    b = GraphBuilder("loop")
    b.input("x", P.FLOAT32, [2])
    b.input("M", P.INT64, [])
    b.input("v0", P.FLOAT32, [2])
    c = b.add("Add", ["x", "x"], out="c")  # last explicit use is before the Loop: kept alive for the body
    b.add("Identity", ["v0"], out="vv")
    outs = b.add("Loop", ["M", "", "vv"], {"body": body}, n_out=2)
    b.output(outs[0], P.FLOAT32, None)
    b.output(outs[1], P.FLOAT32, None)
    sess = InferenceSession(b.to_bytes(), device="cpu", optimization_level="NO_OPT")
    x = np.array([1.0, 0.5], np.float32)
    v0 = np.array([0.0, 1.0], np.float32)
    for M in (3, 100):
        fin, scans = sess.run(None, {"x": x, "M": np.array(M, np.int64), "v0": v0})
        v, ref_s = v0.copy(), []
        for i in range(M):
            v = v + i * (2 * x)
            ref_s.append(v * 2)
            if not v.sum() < 40.0:
                break
        np.testing.assert_allclose(fin, v)
        np.testing.assert_allclose(scans, np.stack(ref_s))


def test_scan_forward_and_reverse():
    # state = state + x_t, output_t = state (cumulative sum); second scan input reversed
    body = _sub([Node("Add", ["st", "xt"], ["st2"], {}, "a"), Node("Add", ["st2", "yt"], ["o"], {}, "b")],
                [ValueInfo("st", elem_type=P.FLOAT32, shape=[3]), ValueInfo("xt", elem_type=P.FLOAT32, shape=[3]),
                 ValueInfo("yt", elem_type=P.FLOAT32, shape=[3])],
                [ValueInfo("st2", elem_type=P.FLOAT32, shape=[3]), ValueInfo("o", elem_type=P.FLOAT32, shape=[3])])
    rng = np.random.default_rng(0)
    X = rng.standard_normal((5, 3)).astype(np.float32)
    Y = rng.standard_normal((3, 5)).astype(np.float32)  # scanned along axis 1, reversed
    s0 = np.zeros(3, np.float32)
    fin, outs = run1("Scan", [("s0", s0), ("X", X), ("Y", Y)],
                     {"body": body, "num_scan_inputs": 2, "scan_input_axes": [0, 1], "scan_input_directions": [0, 1],
                      "scan_output_directions": [1]}, n_out=2)
    st, ref = s0.copy(), []
    for t in range(5):
        st = st + X[t]
        ref.append(st + Y[:, 4 - t])
    np.testing.assert_allclose(fin, st, rtol=1e-6)
    np.testing.assert_allclose(outs, np.stack(ref[::-1]), rtol=1e-6)


def test_sequence_ops():
    a = np.arange(6, dtype=np.float32).reshape(2, 3)
    b = GraphBuilder("seq")
    b.input("a", P.FLOAT32, [2, 3])
    s = b.add("SplitToSequence", ["a"], {"axis": 1, "keepdims": 0})
    n = b.add("SequenceLength", [s], out="n")
    s2 = b.add("SequenceInsert", [s, "a"])
    e = b.add("SequenceErase", [s2])  # drops the inserted last element
    at1 = b.add("SequenceAt", [e, "one"], out="at1")
    b.init("one", np.array(1, np.int64))
    cat = b.add("ConcatFromSequence", [e], {"axis": 0, "new_axis": 1}, out="cat")
    for o in ("n", "at1", "cat"):
        b.output(o, P.FLOAT32, None)
    n_, at1_, cat_ = InferenceSession(b.to_bytes(), device="cpu", optimization_level="NO_OPT").run(None, {"a": a})
    assert int(n_) == 3
    np.testing.assert_array_equal(at1_, a[:, 1])
    np.testing.assert_array_equal(cat_, a.T)


# ------------------------------------------------------------------ recurrent
def _sig(v):
    return 1.0 / (1.0 + np.exp(-v))


def _np_lstm(X, W, R, B, lens, h0, c0, P_, reverse):
    T, N, _ = X.shape
    H = R.shape[-1]
    Y = np.zeros((T, N, H))
    h, c = h0.copy(), c0.copy()
    Wb, Rb = B[:4 * H], B[4 * H:]
    for n in range(N):
        steps = range(lens[n] - 1, -1, -1) if reverse else range(lens[n])
        hn, cn = h[n].copy(), c[n].copy()
        for t in steps:
            z = X[t, n] @ W.T + hn @ R.T + Wb + Rb
            zi, zo, zf, zc = np.split(z, 4)
            i = _sig(zi + P_[:H] * cn)
            f = _sig(zf + P_[2 * H:] * cn)
            cn = f * cn + i * np.tanh(zc)
            o = _sig(zo + P_[H:2 * H] * cn)
            hn = o * np.tanh(cn)
            Y[t, n] = hn
        h[n], c[n] = hn, cn
    return Y, h, c


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_lstm_bidirectional_seq_lens_peepholes(device):
    rng = np.random.default_rng(1)
    T, N, I, H = 6, 3, 4, 5
    X = rng.standard_normal((T, N, I)).astype(np.float32)
    W = (rng.standard_normal((2, 4 * H, I)) * 0.4).astype(np.float32)
    R = (rng.standard_normal((2, 4 * H, H)) * 0.4).astype(np.float32)
    B = (rng.standard_normal((2, 8 * H)) * 0.1).astype(np.float32)
    lens = np.array([6, 4, 1], np.int32)
    h0 = rng.standard_normal((2, N, H)).astype(np.float32)
    c0 = rng.standard_normal((2, N, H)).astype(np.float32)
    Pp = (rng.standard_normal((2, 3 * H)) * 0.2).astype(np.float32)
    Y, Yh, Yc = run1("LSTM", [("X", X), ("W", W), ("R", R), ("B", B), ("L", lens), ("h0", h0), ("c0", c0), ("P", Pp)],
                     {"hidden_size": H, "direction": "bidirectional"}, n_out=3, device=device)
    for d in range(2):
        ry, rh, rc = _np_lstm(X.astype(np.float64), W[d], R[d], B[d], lens, h0[d], c0[d], Pp[d], d == 1)
        np.testing.assert_allclose(Y[:, d], ry, rtol=2e-5, atol=2e-5)
        np.testing.assert_allclose(Yh[d], rh, rtol=2e-5, atol=2e-5)
        np.testing.assert_allclose(Yc[d], rc, rtol=2e-5, atol=2e-5)


def test_lstm_and_gru_match_torch_layers():
    torch.manual_seed(0)
    T, N, I, H = 7, 2, 3, 4
    x = torch.randn(T, N, I)
    lstm = torch.nn.LSTM(I, H)
    ti, tf, tg, to = lstm.weight_ih_l0.detach().split(H)
    ri, rf, rg, ro = lstm.weight_hh_l0.detach().split(H)
    bi = lstm.bias_ih_l0.detach().split(H)
    bh = lstm.bias_hh_l0.detach().split(H)
    W = torch.cat([ti, to, tf, tg])[None].numpy()  # ONNX gate order i, o, f, c
    R = torch.cat([ri, ro, rf, rg])[None].numpy()
    B = torch.cat([bi[0], bi[3], bi[1], bi[2], bh[0], bh[3], bh[1], bh[2]])[None].numpy()
    Y, Yh = run1("LSTM", [("X", x.numpy()), ("W", W), ("R", R), ("B", B)], {"hidden_size": H}, n_out=2)
    ref, (rh, _) = lstm(x)
    np.testing.assert_allclose(Y[:, 0], ref.detach().numpy(), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(Yh, rh.detach().numpy(), rtol=1e-5, atol=1e-6)
    # torch GRU == ONNX GRU with linear_before_reset=1 (gate orders r, z, n vs z, r, h)
    gru = torch.nn.GRU(I, H, batch_first=True)
    xb = torch.randn(N, T, I)
    wr, wz, wn = gru.weight_ih_l0.detach().split(H)
    rr, rz, rn = gru.weight_hh_l0.detach().split(H)
    bir, biz, bin_ = gru.bias_ih_l0.detach().split(H)
    bhr, bhz, bhn = gru.bias_hh_l0.detach().split(H)
    W = torch.cat([wz, wr, wn])[None].numpy()
    R = torch.cat([rz, rr, rn])[None].numpy()
    B = torch.cat([biz, bir, bin_, bhz, bhr, bhn])[None].numpy()
    Y, Yh = run1("GRU", [("X", xb.numpy()), ("W", W), ("R", R), ("B", B)],
                 {"hidden_size": H, "linear_before_reset": 1, "layout": 1}, n_out=2)
    ref, rh = gru(xb)
    np.testing.assert_allclose(Y[:, :, 0], ref.detach().numpy(), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(Yh[:, 0], rh.detach().numpy()[0], rtol=1e-5, atol=1e-6)


def test_gru_default_reset_and_rnn_reverse():
    rng = np.random.default_rng(2)
    T, N, I, H = 5, 2, 3, 4
    X = rng.standard_normal((T, N, I)).astype(np.float32)
    W = (rng.standard_normal((1, 3 * H, I)) * 0.5).astype(np.float32)
    R = (rng.standard_normal((1, 3 * H, H)) * 0.5).astype(np.float32)
    B = (rng.standard_normal((1, 6 * H)) * 0.1).astype(np.float32)
    (Y,) = run1("GRU", [("X", X), ("W", W), ("R", R), ("B", B)], {"hidden_size": H})
    h = np.zeros((N, H))
    Wz, Wr, Wh = np.split(W[0].astype(np.float64), 3)
    Rz, Rr, Rh = np.split(R[0].astype(np.float64), 3)
    bwz, bwr, bwh, brz, brr, brh = np.split(B[0].astype(np.float64), 6)
    for t in range(T):
        z = _sig(X[t] @ Wz.T + h @ Rz.T + bwz + brz)
        r = _sig(X[t] @ Wr.T + h @ Rr.T + bwr + brr)
        hh = np.tanh(X[t] @ Wh.T + (r * h) @ Rh.T + brh + bwh)
        h = (1 - z) * hh + z * h
        np.testing.assert_allclose(Y[t, 0], h, rtol=2e-5, atol=2e-5)
    W1 = (rng.standard_normal((1, H, I)) * 0.5).astype(np.float32)
    R1 = (rng.standard_normal((1, H, H)) * 0.5).astype(np.float32)
    (Y,) = run1("RNN", [("X", X), ("W", W1), ("R", R1)], {"hidden_size": H, "direction": "reverse"})
    h = np.zeros((N, H))
    for t in reversed(range(T)):
        h = np.tanh(X[t] @ W1[0].T.astype(np.float64) + h @ R1[0].T)
        np.testing.assert_allclose(Y[t, 0], h, rtol=2e-5, atol=2e-5)


# ------------------------------------------------------------------ quantisation
def test_quantize_dequantize_per_tensor_and_axis():
    x = np.array([[-1.0, 0.25, 2.55], [0.5, 1.5, 2.5]], np.float32)
    (q,) = run1("QuantizeLinear", [("x", x), ("s", np.array(0.01, np.float32)), ("z", np.array(10, np.uint8))])
    np.testing.assert_array_equal(q, np.clip(np.rint(x / 0.01) + 10, 0, 255).astype(np.uint8))
    s = np.array([0.5, 1.0, 2.0], np.float32)
    z = np.array([-1, 0, 3], np.int8)
    (q,) = run1("QuantizeLinear", [("x", x), ("s", s), ("z", z)], {"axis": 1})
    ref = np.clip(np.rint(x / s[None]) + z[None], -128, 127).astype(np.int8)  # rint = round half to even
    np.testing.assert_array_equal(q, ref)
    (d,) = run1("DequantizeLinear", [("q", ref), ("s", s), ("z", z)], {"axis": 1})
    np.testing.assert_allclose(d, (ref.astype(np.float32) - z[None]) * s[None])


def test_dynamic_quantize_and_integer_matmuls():
    rng = np.random.default_rng(3)
    x = rng.uniform(-2, 5, (4, 6)).astype(np.float32)
    y, ys, yz = run1("DynamicQuantizeLinear", [("x", x)], n_out=3)
    scale = (max(0, x.max()) - min(0, x.min())) / 255.0
    zp = np.clip(np.rint(-min(0, x.min()) / scale), 0, 255)
    assert float(ys) == pytest.approx(scale, rel=1e-6) and int(yz) == int(zp)
    np.testing.assert_array_equal(y, np.clip(np.rint(x / np.float32(scale)) + zp, 0, 255).astype(np.uint8))
    A = rng.integers(0, 255, (5, 7)).astype(np.uint8)
    Bm = rng.integers(-128, 127, (7, 3)).astype(np.int8)
    az = np.array(12, np.uint8)
    bz = np.array([1, -2, 3], np.int8)
    (mm,) = run1("MatMulInteger", [("A", A), ("B", Bm), ("az", az), ("bz", bz)])
    ref = (A.astype(np.int64) - 12) @ (Bm.astype(np.int64) - bz[None].astype(np.int64))
    np.testing.assert_array_equal(mm, ref.astype(np.int32))
    # QLinearMatMul: requantised with round-half-even and saturation
    a_s, b_s, y_s = np.float32(0.02), np.float32(0.05), np.float32(0.3)
    (qm,) = run1("QLinearMatMul", [("A", A), ("as", np.array(a_s)), ("az", az), ("B", Bm), ("bs", np.array(b_s)),
                                   ("bz", np.array(0, np.int8)), ("ys", np.array(y_s)), ("yz", np.array(7, np.uint8))])
    acc = (A.astype(np.int64) - 12) @ Bm.astype(np.int64)
    ref = np.clip(np.rint(acc * (np.float64(a_s) * np.float64(b_s)) / np.float64(y_s)) + 7, 0, 255).astype(np.uint8)
    np.testing.assert_array_equal(qm, ref)


def test_qlinear_conv_and_conv_integer():
    rng = np.random.default_rng(4)
    x = rng.integers(0, 255, (1, 2, 5, 5)).astype(np.uint8)
    w = rng.integers(-50, 50, (3, 2, 3, 3)).astype(np.int8)
    xz, wz = 100, np.array([0, 1, -1], np.int8)
    xf = x.astype(np.int64) - xz
    wf = w.astype(np.int64) - wz[:, None, None, None]
    acc = np.zeros((1, 3, 3, 3), np.int64)
    for o in range(3):
        for i in range(3):
            for j in range(3):
                acc[0, o, i, j] = (xf[0, :, i:i + 3, j:j + 3] * wf[o]).sum()
    (ci,) = run1("ConvInteger", [("x", x), ("w", w), ("xz", np.array(xz, np.uint8)), ("wz", wz)],
                 {"kernel_shape": [3, 3]})
    np.testing.assert_array_equal(ci, acc.astype(np.int32))
    bias = np.array([10, -20, 30], np.int32)
    ws = np.array([0.01, 0.02, 0.03], np.float32)
    (qc,) = run1("QLinearConv", [("x", x), ("xs", np.array(0.05, np.float32)), ("xz", np.array(xz, np.uint8)),
                                 ("w", w), ("ws", ws), ("wz", wz), ("ys", np.array(0.5, np.float32)),
                                 ("yz", np.array(128, np.uint8)), ("b", bias)], {"kernel_shape": [3, 3]})
    mult = np.float64(np.float32(0.05)) * ws.astype(np.float64)[None, :, None, None]
    ref = np.clip(np.rint((acc + bias[None, :, None, None]) * mult / np.float64(np.float32(0.5))) + 128, 0, 255)
    np.testing.assert_array_equal(qc, ref.astype(np.uint8))


def test_qlinear_add_contrib():
    a = np.array([10, 200, 50], np.uint8)
    b = np.array([5, 5, 250], np.uint8)
    (y,) = run1("QLinearAdd", [("a", a), ("as", np.array(0.1, np.float32)), ("az", np.array(0, np.uint8)),
                               ("b", b), ("bs", np.array(0.2, np.float32)), ("bz", np.array(5, np.uint8)),
                               ("ys", np.array(0.25, np.float32)), ("yz", np.array(3, np.uint8))], domain="com.microsoft")
    f = a * np.float32(0.1) + (b.astype(np.float32) - 5) * np.float32(0.2)
    np.testing.assert_array_equal(y, np.clip(np.rint(f / np.float32(0.25)) + 3, 0, 255).astype(np.uint8))


# ------------------------------------------------------------------ tensor ops
def test_nonzero_compress_unique_eyelike_shrink():
    x = np.array([[1, 0, 3], [0, 0, 5]], np.float32)
    (nz,) = run1("NonZero", [("x", x)])
    np.testing.assert_array_equal(nz, np.array(np.nonzero(x)))
    (c,) = run1("Compress", [("x", x), ("c", np.array([False, True, True]))], {"axis": 1})
    np.testing.assert_array_equal(c, x[:, 1:])
    (c,) = run1("Compress", [("x", x), ("c", np.array([True, False, False, True]))])
    np.testing.assert_array_equal(c, [1.0, 0.0])
    u = np.array([2.0, 1.0, 1.0, 3.0, 4.0, 3.0], np.float32)
    y, idx, inv, cnt = run1("Unique", [("u", u)], {"sorted": 0}, n_out=4)  # ONNX spec example
    np.testing.assert_array_equal(y, [2.0, 1.0, 3.0, 4.0])
    np.testing.assert_array_equal(idx, [0, 1, 3, 4])
    np.testing.assert_array_equal(inv, [0, 1, 1, 2, 3, 2])
    np.testing.assert_array_equal(cnt, [1, 2, 2, 1])
    y, idx, inv, cnt = run1("Unique", [("u", u)], n_out=4)
    np.testing.assert_array_equal(y, [1.0, 2.0, 3.0, 4.0])
    np.testing.assert_array_equal(inv, [1, 0, 0, 2, 3, 2])
    (e,) = run1("EyeLike", [("x", np.zeros((3, 4), np.float32))], {"k": 1})
    np.testing.assert_array_equal(e, np.eye(3, 4, k=1))
    v = np.array([-2.0, -0.4, 0.0, 0.6, 3.0], np.float32)
    (s,) = run1("Shrink", [("v", v)], {"lambd": 0.5, "bias": 1.5})
    np.testing.assert_allclose(s, [-0.5, 0, 0, -0.9, 1.5], rtol=1e-6)


def test_reverse_sequence_mvn_groupnorm_rmsnorm_cropad():
    x = np.arange(12, dtype=np.float32).reshape(4, 3)  # [time, batch]
    (r,) = run1("ReverseSequence", [("x", x), ("l", np.array([4, 2, 1], np.int64))], {"batch_axis": 1, "time_axis": 0})
    ref = x.copy()
    ref[:4, 0] = x[:4, 0][::-1]
    ref[:2, 1] = x[:2, 1][::-1]
    np.testing.assert_array_equal(r, ref)
    rng = np.random.default_rng(5)
    t = rng.standard_normal((2, 4, 3, 3)).astype(np.float32)
    (m,) = run1("MeanVarianceNormalization", [("t", t)])
    mu = t.mean((0, 2, 3), keepdims=True)
    np.testing.assert_allclose(m, (t - mu) / (np.sqrt((t * t).mean((0, 2, 3), keepdims=True) - mu * mu) + 1e-9),
                               rtol=1e-4, atol=1e-5)
    sc = rng.standard_normal(4).astype(np.float32)
    bi = rng.standard_normal(4).astype(np.float32)
    (g,) = run1("GroupNormalization", [("t", t), ("s", sc), ("b", bi)], {"num_groups": 2, "epsilon": 1e-5})
    gt = t.reshape(2, 2, -1)
    ref = ((gt - gt.mean(-1, keepdims=True)) / np.sqrt(gt.var(-1, keepdims=True) + 1e-5)).reshape(t.shape)
    np.testing.assert_allclose(g, ref * sc[None, :, None, None] + bi[None, :, None, None], rtol=1e-4, atol=1e-5)
    h = rng.standard_normal((2, 5, 8)).astype(np.float32)
    gam = rng.standard_normal(8).astype(np.float32)
    (rm,) = run1("SimplifiedLayerNormalization", [("h", h), ("g", gam)], {"epsilon": 1e-6}, domain="com.microsoft")
    np.testing.assert_allclose(rm, h / np.sqrt((h * h).mean(-1, keepdims=True) + 1e-6) * gam, rtol=1e-5, atol=1e-6)
    img = np.arange(20, dtype=np.float32).reshape(4, 5)
    (cp,) = run1("CenterCropPad", [("img", img), ("sh", np.array([2, 7], np.int64))])
    ref = np.zeros((2, 7), np.float32)
    ref[:, 1:6] = img[1:3]
    np.testing.assert_array_equal(cp, ref)


def test_nms_onnx_example():
    boxes = np.array([[[0.0, 0.0, 1.0, 1.0], [0.0, 0.1, 1.0, 1.1], [0.0, -0.1, 1.0, 0.9], [0.0, 10.0, 1.0, 11.0],
                       [0.0, 10.1, 1.0, 11.1], [0.0, 100.0, 1.0, 101.0]]], np.float32)
    scores = np.array([[[0.9, 0.75, 0.6, 0.95, 0.5, 0.3]]], np.float32)
    (sel,) = run1("NonMaxSuppression", [("b", boxes), ("s", scores), ("m", np.array([3], np.int64)),
                                        ("i", np.array([0.5], np.float32)), ("t", np.array([0.0], np.float32))])
    np.testing.assert_array_equal(sel, [[0, 0, 3], [0, 0, 0], [0, 0, 5]])


def test_dft_windows_bitwise():
    rng = np.random.default_rng(6)
    sig = rng.standard_normal((2, 8, 1)).astype(np.float32)
    (f,) = run1("DFT", [("x", sig)], {"axis": 1}, opset={"": 17})
    ref = np.fft.fft(sig[..., 0], axis=1)
    np.testing.assert_allclose(f[..., 0], ref.real, rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(f[..., 1], ref.imag, rtol=1e-4, atol=1e-5)
    (hw,) = run1("HannWindow", [("n", np.array(8, np.int64))])
    np.testing.assert_allclose(hw, np.hanning(9)[:-1], atol=1e-6)
    (bw,) = run1("BlackmanWindow", [("n", np.array(6, np.int64))], {"periodic": 0})
    np.testing.assert_allclose(bw, np.blackman(6), atol=1e-6)
    a = np.array([12, 7], np.int32)
    (o,) = run1("BitwiseXor", [("a", a), ("b", np.array([10, 1], np.int32))])
    np.testing.assert_array_equal(o, a ^ np.array([10, 1]))


def test_string_ops_and_ml_vectorizers():
    words = np.array(["monday", "tuesday", "wednesday", "thursday"], dtype=object)
    (n,) = run1("StringNormalizer", [("w", words)], {"case_change_action": "UPPER", "stopwords": ["monday"]})
    assert list(n) == ["TUESDAY", "WEDNESDAY", "THURSDAY"]
    (m,) = run1("RegexFullMatch", [("w", words)], {"pattern": "t.*day"})
    np.testing.assert_array_equal(m, [False, True, False, True])
    cats = np.array(["a", "b", "zz"], dtype=object)
    (ids,) = run1("CategoryMapper", [("c", cats)], {"cats_strings": ["a", "b"], "cats_int64s": [5, 7],
                                                     "default_int64": -3}, domain="ai.onnx.ml")
    np.testing.assert_array_equal(ids, [5, 7, -3])
    (fv,) = run1("FeatureVectorizer", [("a", np.ones((2, 2), np.float32)), ("b", np.full((2, 3), 2, np.float32))],
                 {"inputdimensions": [3, 2]}, domain="ai.onnx.ml")
    np.testing.assert_array_equal(fv, [[1, 1, 0, 2, 2], [1, 1, 0, 2, 2]])


# ------------------------------------------------------------------ transformer contrib ops
def _ln(v, g, b, eps):
    mu = v.mean(-1, keepdims=True)
    return (v - mu) / np.sqrt(((v - mu) ** 2).mean(-1, keepdims=True) + eps) * g + b


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_skip_layernorm_attention_embed(device):
    rng = np.random.default_rng(7)
    Bsz, S, D, heads = 2, 5, 8, 2
    x = rng.standard_normal((Bsz, S, D)).astype(np.float32)
    skip = rng.standard_normal((Bsz, S, D)).astype(np.float32)
    g = rng.standard_normal(D).astype(np.float32)
    be = rng.standard_normal(D).astype(np.float32)
    bias = rng.standard_normal(D).astype(np.float32)
    y, _, _, ssum = run1("SkipLayerNormalization", [("x", x), ("s", skip), ("g", g), ("b", be), ("bias", bias)],
                         {"epsilon": 1e-5}, n_out=4, domain="com.microsoft", device=device)
    np.testing.assert_allclose(ssum, x + skip + bias, rtol=1e-6)
    np.testing.assert_allclose(y, _ln(x + skip + bias, g, be, 1e-5), rtol=1e-4, atol=1e-5)
    w = (rng.standard_normal((D, 3 * D)) * 0.3).astype(np.float32)
    wb = (rng.standard_normal(3 * D) * 0.1).astype(np.float32)
    mask = np.array([[1, 1, 1, 0, 0], [1, 1, 1, 1, 1]], np.int32)
    (att,) = run1("Attention", [("x", x), ("w", w), ("wb", wb), ("m", mask)], {"num_heads": heads},
                  domain="com.microsoft", device=device)
    qkv = x.astype(np.float64) @ w + wb
    q, k, v = np.split(qkv, 3, -1)
    hd = D // heads
    ref = np.zeros((Bsz, S, D))
    for b in range(Bsz):
        for h in range(heads):
            qs, ks, vs = (a[b][:, h * hd:(h + 1) * hd] for a in (q, k, v))
            sc = qs @ ks.T / math.sqrt(hd) + np.where(mask[b][None, :] > 0, 0.0, -10000.0)
            p = np.exp(sc - sc.max(-1, keepdims=True))
            p /= p.sum(-1, keepdims=True)
            ref[b][:, h * hd:(h + 1) * hd] = p @ vs
    np.testing.assert_allclose(att, ref, rtol=2e-4, atol=2e-5)
    (causal,) = run1("Attention", [("x", x), ("w", w), ("wb", wb)], {"num_heads": heads, "unidirectional": 1},
                     domain="com.microsoft", device=device)
    b0 = x[0].astype(np.float64) @ w + wb
    q0, k0, v0 = np.split(b0, 3, -1)
    sc = q0[:, :hd] @ k0[:, :hd].T / math.sqrt(hd)
    sc[np.triu_indices(S, 1)] = -np.inf
    p = np.exp(sc - sc.max(-1, keepdims=True))
    p /= p.sum(-1, keepdims=True)
    np.testing.assert_allclose(causal[0][:, :hd], p @ v0[:, :hd], rtol=2e-4, atol=2e-5)
    ids = rng.integers(0, 10, (Bsz, S)).astype(np.int32)
    seg = rng.integers(0, 2, (Bsz, S)).astype(np.int32)
    we = rng.standard_normal((10, D)).astype(np.float32)
    pe = rng.standard_normal((S, D)).astype(np.float32)
    se = rng.standard_normal((2, D)).astype(np.float32)
    out, mi = run1("EmbedLayerNormalization", [("ids", ids), ("seg", seg), ("we", we), ("pe", pe), ("se", se),
                                               ("g", g), ("b", be), ("m", mask)], {"epsilon": 1e-5}, n_out=2,
                   domain="com.microsoft", device=device)
    emb = we[ids] + pe[None] + se[seg]
    np.testing.assert_allclose(out, _ln(emb, g, be, 1e-5), rtol=1e-4, atol=1e-5)
    np.testing.assert_array_equal(mi, mask.sum(1))


def test_fused_matmul_and_gelus():
    rng = np.random.default_rng(8)
    a = rng.standard_normal((2, 4, 3)).astype(np.float32)
    b = rng.standard_normal((2, 5, 3)).astype(np.float32)
    (y,) = run1("FusedMatMul", [("a", a), ("b", b)], {"alpha": 0.5, "transB": 1}, domain="com.microsoft")
    np.testing.assert_allclose(y, 0.5 * a @ b.transpose(0, 2, 1), rtol=1e-5, atol=1e-6)
    v = rng.standard_normal((3, 4)).astype(np.float32)
    bias = rng.standard_normal(4).astype(np.float32)
    (fg,) = run1("FastGelu", [("v", v), ("bias", bias)], domain="com.microsoft")
    u = v + bias
    np.testing.assert_allclose(fg, 0.5 * u * (1 + np.tanh(np.sqrt(2 / np.pi) * (u + 0.044715 * u ** 3))), rtol=1e-5,
                               atol=1e-6)
    (qg,) = run1("QuickGelu", [("v", v)], domain="com.microsoft")
    np.testing.assert_allclose(qg, v / (1 + np.exp(-1.702 * v)), rtol=1e-5, atol=1e-6)


def test_random_generators_are_seeded():
    a = run1("RandomNormal", [], {"shape": [3, 4], "seed": 2.0, "mean": 1.0, "scale": 0.5})[0]
    b = run1("RandomNormal", [], {"shape": [3, 4], "seed": 2.0, "mean": 1.0, "scale": 0.5})[0]
    np.testing.assert_array_equal(a, b)
    u = run1("RandomUniformLike", [("x", np.zeros((1000,), np.float32))], {"low": 2.0, "high": 3.0, "seed": 1.0})[0]
    assert u.min() >= 2.0 and u.max() < 3.0 and abs(u.mean() - 2.5) < 0.05
