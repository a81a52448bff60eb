"""ORACLE — test infrastructure only.  Pure-Python restatement of compressai 1.2.6's rANS coder
(cpp_exts/rans/rans_interface.cpp over ryg_rans rans64.h), used to cross-check the bytes of
mlic_amd's native coder on small streams.  compressai itself is absent from this image, so the
byte format is pinned only by this restatement of the published algorithm (parity)."""
import struct

RANS64_L = 1 << 31
PREC = 16
BYP = 4
MAXB = (1 << BYP) - 1


def encode(symbols, indexes, cdfs, lengths, offsets):
    syms = []
    for s, ci in zip(symbols, indexes):
        cdf = cdfs[ci]
        maxv = lengths[ci] - 2
        v = s - offsets[ci]
        raw = 0
        if v < 0:
            raw, v = -2 * v - 1, maxv
        elif v >= maxv:
            raw, v = 2 * (v - maxv), maxv
        syms.append((cdf[v], cdf[v + 1] - cdf[v], False))
        if v == maxv:
            nb = 0
            while (raw >> (nb * BYP)) != 0:
                nb += 1
            val = nb
            while val >= MAXB:
                syms.append((MAXB, MAXB + 1, True))
                val -= MAXB
            syms.append((val, val + 1, True))
            for j in range(nb):
                b = (raw >> (j * BYP)) & MAXB
                syms.append((b, b + 1, True))
    out = []  # words emitted back to front
    x = RANS64_L
    for start, rng, byp in reversed(syms):
        if not byp:
            x_max = ((RANS64_L >> PREC) << 32) * rng
            if x >= x_max:
                out.append(x & 0xFFFFFFFF)
                x >>= 32
            x = ((x // rng) << PREC) + (x % rng) + start
        else:
            x_max = ((RANS64_L >> 16) << 32) * (1 << (16 - BYP))
            if x >= x_max:
                out.append(x & 0xFFFFFFFF)
                x >>= 32
            x = (x << BYP) | start
    out.append(x >> 32)
    out.append(x & 0xFFFFFFFF)
    words = out[::-1]
    return struct.pack("<%dI" % len(words), *words)
