"""Dev tool: vendor-library calibration points for the yolov7 conv shapes (bs32 640 fp16).

1x1 convs as plain GEMMs (torch.mm -> hipBLASLt) and 3x3 convs through MIOpen (channels_last fp16),
timed with events; not part of the product path, only a yardstick for the hand-written kernels."""
import torch, sys
torch.backends.cudnn.benchmark = True
dev = 'cuda:0'
B = 32
def t(fn, it=20):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3
gemms = [(160, 256, 256), (160, 256, 128), (160, 128, 128), (80, 512, 512), (80, 512, 256), (40, 1024, 1024),
         (40, 1024, 512), (80, 256, 256), (80, 512, 128)]
for hw, k, n in gemms:
    M = B * hw * hw
    a = torch.randn(M, k, device=dev, dtype=torch.float16)
    w = torch.randn(k, n, device=dev, dtype=torch.float16)
    us = t(lambda: torch.mm(a, w))
    fl = 2 * M * k * n
    by = (M * k + M * n + k * n) * 2
    print(f'GEMM 1x1 {k:5d}->{n:5d} @{hw:3d}: {us:8.1f} us {fl/us/1e6:7.1f} TF/s {by/us/1e3:7.1f} GB/s', flush=True)
convs = [(320, 64, 64, 1), (320, 64, 128, 2), (160, 64, 64, 1), (80, 128, 128, 1), (40, 256, 256, 1), (20, 512, 512, 1),
         (80, 128, 256, 1), (40, 256, 512, 1), (20, 512, 1024, 1), (160, 128, 128, 2)]
for hw, ci, co, s in convs:
    x = torch.randn(B, ci, hw, hw, device=dev, dtype=torch.float16).to(memory_format=torch.channels_last)
    conv = torch.nn.Conv2d(ci, co, 3, s, 1).to(dev).half().to(memory_format=torch.channels_last)
    with torch.no_grad():
        us = t(lambda: conv(x))
    ho = hw // s
    fl = 2 * B * ho * ho * co * ci * 9
    print(f'MIOpen 3x3 {ci:4d}->{co:5d} s{s} @{hw:3d}: {us:8.1f} us {fl/us/1e6:7.1f} TF/s', flush=True)
