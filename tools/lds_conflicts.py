"""Bank-conflict model of the wave-FFT LDS accesses of k_xspec_w (DESIGN.md
section 3): every ds_read_b128 / ds_write_b128 the kernel issues on a wave
buffer, priced with MI355X_MICROARCH.md's LDS table (read: four 16-lane
groups, bank = (a/4) mod 64; write: eight contiguous 8-lane groups, bank =
(a/4) mod 32; one extra cycle per extra distinct 16-B slot on a bank).
    python tools/lds_conflicts.py      -> extra cycles / LDS instruction per
layout (slot map) and N, for the padded map and the XOR-swizzled one."""
import itertools

RG = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
      list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
RG += [[l + 32 for l in g] for g in RG]
WG = [list(range(8 * i, 8 * i + 8)) for i in range(8)]


def cost(addr, write):
    """extra cycles of one wave instruction; addr[lane] = 16-B slot or None"""
    groups, mod = (WG, 8) if write else (RG, 16)
    extra = 0
    for g in groups:
        per = {}
        for l in g:
            if addr[l] is None:
                continue
            per.setdefault(addr[l] % mod, set()).add(addr[l])
        if per:
            extra += max(len(v) for v in per.values()) - 1
    return extra


def plan(log2n):
    n = 1 << log2n
    r = n // 64
    lr = log2n - 6
    nfull = log2n // lr
    last = 1 << (log2n - nfull * lr)
    nst = nfull + (1 if last > 1 else 0)
    rad = [r if s < nfull else last for s in range(nst)]
    L = [1]
    for s in range(1, nst):
        L.append(L[-1] * rad[s - 1])
    return n, r, rad, L


def accesses(log2n):
    """(write?, idx[lane]) of every LDS instruction on one wave buffer for
    one row: FFT stages, the two rfft post-passes, the X stores"""
    n, r, rad, L = plan(log2n)
    out = []
    for q in range(r):
        out.append((True, [l * r + q for l in range(64)]))
    for s in range(1, len(rad)):
        nb = n // rad[s]
        for b in range(nb // 64):
            for q in range(rad[s]):
                out.append((False, [l + 64 * b + q * nb for l in range(64)]))
        for b in range(nb // 64):
            for q in range(rad[s]):
                idx = []
                for l in range(64):
                    j = l + 64 * b
                    k = j & (L[s] - 1)
                    idx.append((j - k) * rad[s] + k + q * L[s])
                out.append((True, idx))
    for _ in range(2):                      # pass 1 and pass 2 read (k, N-k)
        for i in range(n // 128):
            out.append((False, [l + 64 * i for l in range(64)]))
            out.append((False, [0 if l + 64 * i == 0 else n - l - 64 * i for l in range(64)]))
    for i in range(n // 128):
        out.append((True, [l + 64 * i for l in range(64)]))
        out.append((True, [n // 2 if l + 64 * i == 0 else n - l - 64 * i for l in range(64)]))
    return out


def writeout(log2n, slot, sl, waves=8):
    """write-out reads: thread t -> channel c = t % waves, harmonic k = t / waves
    + 64 j; channel c's buffer starts at c * sl"""
    n = 1 << log2n
    out = []
    for w in range(waves):
        for j in range((n + 1 + 63) // 64):
            a = []
            for l in range(64):
                t = 64 * w + l
                c, k = t % waves, t // waves + 64 * j
                a.append(c * sl + slot(min(k, n - 1)) if k <= n else None)
            out.append((False, a))
    return out


def pad_map(log2n):
    s = max(3, log2n - 6)
    return lambda i: i + (i >> s)


def xor_map(log2n):
    return lambda i: i ^ ((i >> 4) & 7)


def price(log2n, slot, sl):
    acc = accesses(log2n)
    ex = sum(cost([slot(i) for i in idx], w) for w, idx in acc)
    wo = writeout(log2n, slot, sl)
    exw = sum(cost(a, w) for w, a in wo)
    return ex / len(acc), exw / len(wo), (ex + exw) / (len(acc) + len(wo))


def main():
    for log2n in (7, 8, 9, 10):
        n = 1 << log2n
        s = max(3, log2n - 6)
        padded = n + (n >> s)
        print("N=%d" % n)
        print("   pad  (SL %d): fft+rfft %.3f  write-out %.3f  all %.3f" %
              ((padded + 2,) + price(log2n, pad_map(log2n), padded + 2)))
        best = min(range(n + 2, n + 34),
                   key=lambda sl: price(log2n, xor_map(log2n), sl)[2])
        print("   xor  (SL %d): fft+rfft %.3f  write-out %.3f  all %.3f" %
              ((best,) + price(log2n, xor_map(log2n), best)))


if __name__ == "__main__":
    main()
