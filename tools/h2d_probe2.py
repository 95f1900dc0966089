"""H2D bandwidth probe (GPU box): a 1.57 GB float32 batch (4096 x 96000) from
pageable / page-locked host memory, as one copy or split over 2-4 HIP
streams (torch used only as a measuring harness here)."""
import time

import torch

n = 4096 * 96000
dev = torch.device("cuda:0")
d = torch.empty(n, dtype=torch.float32, device=dev)
pageable = torch.ones(n, dtype=torch.float32)
pinned = torch.ones(n, dtype=torch.float32).pin_memory()
streams = [torch.cuda.Stream() for _ in range(4)]
for name, src in (("pageable", pageable), ("pinned", pinned)):
    for parts in (1, 2, 4):
        ts = []
        for _ in range(4):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            step = n // parts
            for k in range(parts):
                with torch.cuda.stream(streams[k]):
                    d[k * step:(k + 1) * step].copy_(src[k * step:(k + 1) * step], non_blocking=True)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        print(f"{name:9s} parts={parts}: {n * 4 / min(ts[1:]) / 1e9:6.1f} GB/s", flush=True)
