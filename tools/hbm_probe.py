"""Practical HBM ceilings on this GPU (diagnostic): write-only (fill_) and copy rates of
large torch tensors, timed with HIP events.  The fused CWT kernel is write-dominated
(8 B written per output point vs 8/F B read), so the fill rate is its practical roof."""
import json
import sys

import torch


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e-3


def main():
    gib = float(sys.argv[1]) if len(sys.argv) > 1 else 8.0
    n = int(gib * (1 << 30)) // 4
    x = torch.empty(n, dtype=torch.float32, device='cuda')
    y = torch.empty(n, dtype=torch.float32, device='cuda')
    t_fill = timed(lambda: x.fill_(1.0))
    t_copy = timed(lambda: y.copy_(x))
    out = {'bytes': 4 * n, 'fill_GBps': 4 * n / t_fill / 1e9, 'copy_GBps': 8 * n / t_copy / 1e9}
    print(json.dumps(out))


if __name__ == '__main__':
    main()
