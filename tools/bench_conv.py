"""Per-layer timing: MFMA implicit-GEMM conv (fused epilogue) vs MIOpen conv + separate bias/ReLU,
ResNet-50 bottleneck shapes at batch 128, channels_last; ``--dtype fp32|fp16|bf16`` (default fp16).

Each row is also placed on the MI355X roofline: the compute floor at the dense MFMA peak (2.5 PF/s fp16 /
bf16, no sparsity; fp32 inputs run as bf16 planes) and the memory floor at 8 TB/s for the unavoidable bytes
(input + weights + output once); "%peak" is achieved / dense peak and "bound" says which floor is higher.
The ResNet-50 count of each shape weights the network total."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from synapseml_amd.ops.conv import conv2d_nhwc, pack_weight  # noqa: E402

PEAK_TFLOPS = 2500.0   # dense fp16 / bf16 MFMA (AMD's headline 5 PF includes 2:1 sparsity)
HBM_TBPS = 8.0
# occurrences of each shape below in ResNet-50 v2 (3 / 4 / 6 / 3 bottlenecks; strided / projection convs)
COUNT = [1, 3, 4, 2, 4, 4, 3, 1, 6, 6, 5, 3, 3, 2]
SHAPES = [  # C, H, Cout, k, stride
    (64, 56, 64, 1, 1), (64, 56, 64, 3, 1), (64, 56, 256, 1, 1), (256, 56, 64, 1, 1),
    (128, 28, 128, 3, 1), (128, 28, 512, 1, 1), (512, 28, 128, 1, 1), (256, 56, 512, 1, 2),
    (256, 14, 256, 3, 1), (256, 14, 1024, 1, 1), (1024, 14, 256, 1, 1),
    (512, 7, 512, 3, 1), (512, 7, 2048, 1, 1), (2048, 7, 512, 1, 1),
]


def bench(fn, iters=50):
    if "--quick" in sys.argv:
        iters = 5
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    quick = "--quick" in sys.argv
    B = 128
    dt = torch.float16
    if "--dtype" in sys.argv:
        dt = {"fp32": torch.float32, "fp16": torch.float16, "bf16": torch.bfloat16}[sys.argv[sys.argv.index("--dtype") + 1]]
    print(f"dtype {dt}")
    tot_m, tot_t, tot_floor = 0.0, 0.0, 0.0
    shapes = SHAPES[:4] if quick else SHAPES
    if "--only" in sys.argv:  # e.g. --only 1,4,8: the ResNet-50 3x3 layers (profiling runs)
        shapes = [SHAPES[int(i)] for i in sys.argv[sys.argv.index("--only") + 1].split(",")]
    for C, H, Co, k, st in shapes:
        x = torch.randn(B, C, H, H, device="cuda").to(dt).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(Co, C, k, k, device="cuda") / (C * k * k) ** 0.5).to(dt)
        wp = pack_weight(w, dt)
        bias = torch.randn(Co, device="cuda")
        pad = k // 2
        t_m = bench(lambda: conv2d_nhwc(x, wp, k, k, (st, st), (pad, pad), bias=bias, relu=True))
        wc = w.contiguous(memory_format=torch.channels_last)
        bh = bias.to(dt)
        t_t = float("nan") if "--no-ref" in sys.argv else bench(lambda: torch.relu_(F.conv2d(x, wc, bh, st, pad)))
        oh = (H + 2 * pad - k) // st + 1
        flops = 2.0 * B * oh * oh * Co * C * k * k
        esz = x.element_size()
        bytes_ = (B * H * H * C + Co * C * k * k + B * oh * oh * Co) * esz
        t_comp = flops / (PEAK_TFLOPS * 1e12) * 1e6
        t_mem = bytes_ / (HBM_TBPS * 1e12) * 1e6
        cnt = COUNT[SHAPES.index((C, H, Co, k, st))]
        tot_m += t_m * cnt
        tot_t += t_t * cnt
        tot_floor += max(t_comp, t_mem) * cnt
        tf = flops / t_m / 1e6
        print(f"C={C:5d} H={H:3d} Cout={Co:5d} k={k} s={st} x{cnt}: mfma {t_m:8.1f} us ({tf:7.1f} TF/s, "
              f"{100 * tf / PEAK_TFLOPS:5.1f}% peak; floor {max(t_comp, t_mem):6.1f} us "
              f"{'compute' if t_comp >= t_mem else 'memory'}-bound, {max(t_comp, t_mem) / t_m * 100:5.1f}% of SOL)  "
              f"miopen+bias+relu {t_t:8.1f} us ({flops / t_t / 1e6:7.1f} TF/s)  speedup {t_t / t_m:5.2f}x")
    print(f"RESNET-50 CONV TOTAL (weighted by count) mfma {tot_m:.1f} us  miopen {tot_t:.1f} us  "
          f"speedup {tot_t / tot_m:.2f}x  roofline floor {tot_floor:.1f} us ({tot_floor / tot_m * 100:.1f}% of SOL)")


if __name__ == "__main__":
    main()
