"""A plain device copy (torch copy_) of the exchange's C4 / C3 send sizes: the
reference rate for k_xbuild's frame copies."""
import torch, time
x = torch.empty(371_000_000, dtype=torch.uint8, device='cuda').random_(0, 255)
y = torch.empty_like(x)
for _ in range(3): y.copy_(x)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ts = []
for _ in range(20):
    e0.record(); y.copy_(x); e1.record(); torch.cuda.synchronize(); ts.append(e0.elapsed_time(e1))
ts.sort()
t = ts[len(ts)//2] * 1e-3
print(f"torch copy 371 MB: {t*1e6:.1f} us, {2*371e6/t/1e12:.2f} TB/s (read+write)")
x2 = x[:63_000_000]; y2 = y[:63_000_000]
ts = []
for _ in range(20):
    e0.record(); y2.copy_(x2); e1.record(); torch.cuda.synchronize(); ts.append(e0.elapsed_time(e1))
ts.sort(); t = ts[len(ts)//2] * 1e-3
print(f"torch copy 63 MB: {t*1e6:.1f} us, {2*63e6/t/1e12:.2f} TB/s (read+write)")
