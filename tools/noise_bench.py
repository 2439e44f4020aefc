"""ppf_noise_batch on many 2048-bin rows (GPU box): event-timed kernel
throughput and a digest of the outputs, to A/B the half-buffer wave FFT
(k_noise_h, PPF_NOISE_HALF=1 builds) against k_noise_w.
    PPFIT_LIB=... python tools/noise_bench.py [nrows]"""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from pulseportraiture_amd import engine
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 327680
    dev = engine.device()
    g = torch.Generator(device=dev).manual_seed(3)
    rows = torch.randn((n, 2048), device=dev, dtype=torch.float32, generator=g)
    out = engine.noise_rows(rows)
    torch.cuda.synchronize()
    ts = []
    for _ in range(7):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        out = engine.noise_rows(rows)
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    ms = ts[len(ts) // 2]
    h = hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()[:16]
    print("lib %s: %d rows of 2048 in %.3f ms (%.1f GB/s of f32 rows); digest %s" % (
        os.path.basename(os.environ.get("PPFIT_LIB", "libppfit.so")), n, ms,
        n * 2048 * 4 / ms / 1e6, h), flush=True)


if __name__ == "__main__":
    main()
