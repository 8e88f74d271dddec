"""Host->device staging probe: pageable .to(), pinned DMA, and numpy copy into pinned memory with N threads."""
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

n = 256 * 3 * 224 * 224
src = np.random.default_rng(0).random(n, dtype=np.float32)
dev = torch.empty(n, dtype=torch.float32, device="cuda")
pin = torch.empty(n, dtype=torch.float32, pin_memory=True)
pn = pin.numpy()
gb = n * 4 / 1e9


def t(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


print("pageable .to(): %.1f GB/s" % (gb / t(lambda: torch.from_numpy(src).to("cuda", non_blocking=True))))
print("pageable copy_: %.1f GB/s" % (gb / t(lambda: dev.copy_(torch.from_numpy(src), non_blocking=True))))
print("pinned copy_: %.1f GB/s" % (gb / t(lambda: dev.copy_(pin, non_blocking=True))))
for th in (1, 2, 4, 8, 16):
    pool = ThreadPoolExecutor(th)
    step = -(-n // th)

    def fill():
        list(pool.map(lambda i: np.copyto(pn[i:i + step], src[i:i + step]), range(0, n, step)))

    print("copyto pinned x%d threads: %.1f GB/s" % (th, gb / t(fill)))
    pool.shutdown()
