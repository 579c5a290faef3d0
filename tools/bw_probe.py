"""Dev probe: achievable HBM read bandwidth on this box for a 480 MB buffer
(torch reductions; the same bytes as one C2 launch reads)."""
import torch

x = torch.randint(0, 1 << 40, (60_000_000,), dtype=torch.int64, device="cuda")
y = x.view(torch.int32)
for name, fn in (("sum_i64", lambda: x.sum()), ("max_i32", lambda: y.max()),
                 ("copy", lambda: x.clone())):
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
    nb = x.numel() * 8 * (2 if name == "copy" else 1)
    print("%-8s %.4f ms  %.0f GB/s" % (name, ms, nb / ms / 1e6))
