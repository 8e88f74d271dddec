"""Runs one ResNet-50 conv shape through the MFMA kernel many times (for rocprofv3 --pmc passes).
usage: python tools/conv_pmc_driver.py C H Cout k stride [iters] [kernel]; SML_PMC_DTYPE=fp32|fp16|bf16 (default fp16)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from synapseml_amd.ops.conv import conv2d_nhwc, pack_weight  # noqa: E402

C, H, Co, k, st = (int(v) for v in sys.argv[1:6])
iters = int(sys.argv[6]) if len(sys.argv) > 6 else 20
kernel = int(sys.argv[7]) if len(sys.argv) > 7 else 0
B = 128
dt = {"fp32": torch.float32, "fp16": torch.float16, "bf16": torch.bfloat16}[os.environ.get("SML_PMC_DTYPE", "fp16")]
x = torch.randn(B, C, H, H, device="cuda").to(dt).contiguous(memory_format=torch.channels_last)
w = pack_weight((torch.randn(Co, C, k, k, device="cuda") / (C * k * k) ** 0.5).to(dt), dt)
bias = torch.randn(Co, device="cuda")
for _ in range(iters):
    conv2d_nhwc(x, w, k, k, (st, st), (k // 2, k // 2), bias=bias, relu=True, kernel=kernel)
torch.cuda.synchronize()
print("done")
