"""Stem conv kernel timing probe: ResNet-50 stem (B x 3 x 224 x 224 -> 64, 7x7 / 2, pad 3) fp16 on the
dedicated kernels (2-byte gather and row-run forms), plain and with the input affine; event-timed, one JSON line per variant."""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from synapseml_amd.ops.conv import pack_stem_weight, stem_conv_nhwc  # noqa: E402


def main(batch=128, iters=20):
    x = torch.randn(batch, 3, 224, 224, device="cuda").half().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(64, 3, 7, 7, device="cuda") / 12).half()
    wk, wn = pack_stem_weight(w, wide=True), pack_stem_weight(w, wide=False)
    bias = torch.randn(64, device="cuda")
    aff = (torch.rand(3, device="cuda") + 0.5, torch.randn(3, device="cuda"))
    for name, wq, kw in (("gather", wn, {"form": 1}), ("rowstaged", wn, {"form": 2}),
                         ("rowstaged_affine", wn, {"form": 2, "in_affine": aff}), ("rowrun", wk, {})):
        for _ in range(3):
            stem_conv_nhwc(x, wq, 7, 7, (2, 2), (3, 3), bias=bias, relu=2, **kw)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            stem_conv_nhwc(x, wq, 7, 7, (2, 2), (3, 3), bias=bias, relu=2, **kw)
        e.record()
        torch.cuda.synchronize()
        print(json.dumps({"probe": "stem_conv", "variant": name, "batch": batch, "us": s.elapsed_time(e) * 1e3 / iters}))


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:]))
