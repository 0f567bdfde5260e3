"""Read-bandwidth reference on the box: torch's own reductions over a C4-sized f64 store
(983 MB; three copies rotated so every pass streams from HBM, not the 256 MiB Infinity Cache),
timed with HIP events -- the practical read roofline the moments kernel is set against."""
import torch


def timed(fn, reps=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        fn(0)
    torch.cuda.synchronize()
    s.record()
    for i in range(reps):
        fn(i)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e-3


def main():
    dev = torch.device("cuda:0")
    n = 983_040_000 // 8
    xs = [torch.rand(n, dtype=torch.float64, device=dev) for _ in range(3)]
    outs = torch.empty(24, dtype=torch.float64, device=dev)
    for name, fn in (("sum (flat)", lambda i: xs[i % 3].sum()),
                     ("sum over rows [24, n/24]", lambda i: torch.sum(xs[i % 3].view(24, -1), dim=1, out=outs)),
                     ("copy_ into a 4th buffer (read + write)", None)):
        if fn is None:
            y = torch.empty_like(xs[0])
            t = timed(lambda i: y.copy_(xs[i % 3]))
            print(f"{name:40s} {t * 1e6:9.1f} us  {2 * n * 8 / t / 1e9:8.1f} GB/s (read + write)")
            continue
        t = timed(fn)
        print(f"{name:40s} {t * 1e6:9.1f} us  {n * 8 / t / 1e9:8.1f} GB/s read")


if __name__ == "__main__":
    main()
