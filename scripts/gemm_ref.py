"""Library-GEMM reference point (torch.mm -> hipBLASLt / rocBLAS) for the conv layer shapes of yolov7
640 bs32 as plain GEMMs: M = 32 * H * W pixels, K = cin * k * k, N = cout (no border frame, no
epilogue, dense output).  Diagnostic only — what a vendor GEMM reaches on the same M, N, K."""
import torch

SHAPES = [  # (label, M, K, N)
    ('1x1 256->256 @160', 32 * 160 * 160, 256, 256),
    ('1x1 512->512 @80', 32 * 80 * 80, 512, 512),
    ('1x1 256->256 @80', 32 * 80 * 80, 256, 256),
    ('1x1 1024->1024 @40', 32 * 40 * 40, 1024, 1024),
    ('1x1 512->512 @40', 32 * 40 * 40, 512, 512),
    ('1x1 1024->256 @40', 32 * 40 * 40, 1024, 256),
    ('1x1 1024->1024 @20', 32 * 20 * 20, 1024, 1024),
    ('1x1 2048->512 @20', 32 * 20 * 20, 2048, 512),
    ('3x3 128->128 @80', 32 * 80 * 80, 1152, 128),
    ('3x3 256->256 @40', 32 * 40 * 40, 2304, 256),
    ('3x3 256->512 @40', 32 * 40 * 40, 2304, 512),
    ('3x3 256->256 @20', 32 * 20 * 20, 2304, 256),
    ('3x3 512->1024 @20', 32 * 20 * 20, 4608, 1024),
]


def main():
    dev = 'cuda:0'
    for label, M, K, N in SHAPES:
        a = torch.randn(M, K, device=dev, dtype=torch.float16)
        b = torch.randn(K, N, device=dev, dtype=torch.float16)
        for _ in range(5):
            torch.mm(a, b)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 30
        e0.record()
        for _ in range(n):
            torch.mm(a, b)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / n
        tf = 2.0 * M * N * K / us / 1e6
        print(f'{label:22s} M {M:7d} K {K:5d} N {N:5d}  {us:7.1f} us  {tf:6.0f} TF/s', flush=True)


if __name__ == '__main__':
    main()
