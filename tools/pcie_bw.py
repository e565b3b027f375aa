#!/usr/bin/env python3
"""Host<->HBM copy bandwidth on the GPU box (informs the C4 PCIe-inclusive
leg): pinned device-mapped host memory (fd_ed25519_hip_host_alloc) and
torch-pinned memory, H2D and D2H, 1-4 concurrent streams, 256 MB pieces."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from firedancer_amd.ed25519 import HostBuffer  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    piece = 256 << 20
    out = {}
    hb = HostBuffer(4 * piece)
    hbt = torch.from_numpy(hb.array)
    tp = torch.empty(4 * piece, dtype=torch.uint8).pin_memory()
    d = torch.empty(4 * piece, dtype=torch.uint8, device=dev)
    for name, h in (("mapped", hbt), ("torch_pinned", tp)):
        for k in (1, 2, 4):
            ss = [torch.cuda.Stream(dev) for _ in range(k)]
            for direction in ("h2d", "d2h"):
                best = 0
                for rep in range(3):
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    for i in range(4):
                        with torch.cuda.stream(ss[i % k]):
                            if direction == "h2d":
                                d[i * piece:(i + 1) * piece].copy_(h[i * piece:(i + 1) * piece], non_blocking=True)
                            else:
                                h[i * piece:(i + 1) * piece].copy_(d[i * piece:(i + 1) * piece], non_blocking=True)
                    torch.cuda.synchronize()
                    best = max(best, 4 * piece / (time.perf_counter() - t0) / 1e9)
                out[f"{name}_{direction}_{k}streams_GBps"] = round(best, 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
