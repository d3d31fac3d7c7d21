"""HBM write / copy bandwidth reference points (torch kernels) for the roofline notes."""
import torch

n = 1080 * 1920 * 64
y = torch.empty(n, dtype=torch.bfloat16, device="cuda")
x = torch.randn(n, device="cuda").to(torch.bfloat16)
yf = torch.empty(n, dtype=torch.float32, device="cuda")
for name, fn, nbytes in [("fill 265MB", lambda: y.fill_(1.0), 2 * n), ("copy 265MB", lambda: y.copy_(x), 4 * n),
                         ("zero 265MB", lambda: y.zero_(), 2 * n), ("fill f32 531MB", lambda: yf.fill_(1.0), 4 * n)]:
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    print("%-14s %.1f us  %.2f TB/s" % (name, ms * 1e3, nbytes / ms / 1e9))
