"""Torch reference rates at update sizes (fill 0 / fill 1 / copy / sum): what a plain PyTorch kernel
reaches on this HBM, for comparison with k_decode / k_scan."""
import torch, time
d = torch.device("cuda", 0)
for n in (25_610_152, 4 * 25_610_152, 16 * 25_610_152):
    x = torch.empty(n, device=d)
    y = torch.empty(n, device=d)
    for name, fn in (("fill0", lambda: x.fill_(0.0)), ("fill1", lambda: x.fill_(1.0)), ("copy", lambda: y.copy_(x)),
                     ("sum", lambda: x.sum())):
        for _ in range(5): fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50): fn()
        e1.record(); torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 50 * 1e3
        b = 4 * n * (2 if name == "copy" else 1)
        print(f"n={n} {name}: {us:.1f} us  {b / us / 1e6:.2f} TB/s")
