"""Host rANS coder speed on the reference fixtures' coder lists (tiled to ~4 M symbols): ns per symbol."""
import sys, time, numpy as np
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
from mlic_amd import entropy
g = np.load('tests/golden/scale_table.npz')
cdf, length, offset = g["quantized_cdf"], g["cdf_length"], g["offset"]
for fx in ("forward_MLICPP_L_192x256_r2", "forward_MLICPP_L_192x256_r5", "forward_MLICPP_L_128x192"):
    f = np.load(f'tests/golden/{fx}.npz')
    sym, idx = f["y_symbols"], f["y_indexes"]
    rep = max(1, 4_000_000 // sym.size)
    S = np.tile(sym, rep); I = np.tile(idx, rep)
    data = entropy.rans_encode(S, I, cdf, length, offset)
    best = 1e9
    for _ in range(3):
        t0 = time.perf_counter(); out = entropy.rans_decode(data, I, cdf, length, offset); dt = time.perf_counter() - t0
        best = min(best, dt)
    assert np.array_equal(out, S)
    t0 = time.perf_counter(); entropy.rans_encode(S, I, cdf, length, offset); te = time.perf_counter() - t0
    print(f"{fx}: {S.size} symbols, {8*len(data)/S.size:.3f} bits/sym, decode {1e9*best/S.size:.2f} ns/sym, encode {1e9*te/S.size:.2f} ns/sym, P(0)={np.mean(S==0):.3f}")
