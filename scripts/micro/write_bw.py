"""Achievable HBM write bandwidth on this box: torch fill_ / zero_ of large buffers (the C5 kernel
is a store stream of 36-40 B per position)."""
import torch

dev = torch.device("cuda", 0)
for gb in (4, 16):
    n = gb * (1 << 30) // 4
    x = torch.empty(n, dtype=torch.int32, device=dev)
    for name, fn in (("zero_", lambda: x.zero_()), ("fill_(1)", lambda: x.fill_(1))):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 5
        print(f"{gb} GiB {name}: {ms:.2f} ms, {x.numel() * 4 / ms / 1e6:.0f} GB/s", flush=True)
    del x
    torch.cuda.empty_cache()
