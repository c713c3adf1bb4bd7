"""LDS bank conflicts of k_bnn's MFMA operand reads (csrc/potential_bnn.hip) under XOR swizzles of
the column of the H-wide row-major tiles (h1, h2 [N][H], W2 [H][H]), 64 banks of 4 bytes: the two
read patterns (16 rows x 4 consecutive columns, 4 rows x 16 consecutive columns) over every tile
of the three products at N = 100, H = 69.  Prints mean / worst lanes per bank without a swizzle,
for every swizzle 16 g(r mod 4) and a local search over periodic masks (the kernel uses
c ^ 32 (r & 1) for c < 64: 2.56 / 4 -> 1.78 / 2)."""
import itertools

import numpy as np

S, H, N = 69, 69, 100
pats = []
for rows_max, cols_max in ((N, H), (H, H)):
    for r0 in range(0, rows_max, 16):
        for s in range(0, (cols_max + 3) // 4):
            pats.append([(r0 + m, 4 * s + kq) for m in range(16) for kq in range(4)
                         if r0 + m < rows_max and 4 * s + kq < cols_max])
    for s in range(0, (rows_max + 3) // 4):
        for c0 in range(0, cols_max, 16):
            pats.append([(4 * s + kq, c0 + c) for kq in range(4) for c in range(16)
                         if 4 * s + kq < rows_max and c0 + c < cols_max])
P = len(pats)
R, C, M = np.zeros((P, 64), int), np.zeros((P, 64), int), np.zeros((P, 64), bool)
for i, p in enumerate(pats):
    for j, (r, c) in enumerate(p):
        R[i, j], C[i, j], M[i, j] = r, c, True


def cost(f):
    cc = np.where(C < 64, C ^ f[R], C)
    b = (R * S + cc) % 64 + 64 * np.arange(P)[:, None]
    cnt = np.bincount(b[M], minlength=64 * P).reshape(P, 64).max(1)
    return float(cnt.mean()), int(cnt.max())


print("no swizzle", cost(np.zeros(128, int)))
best = None
for g in itertools.product(range(4), repeat=4):
    c = cost(np.array([16 * g[r % 4] for r in range(128)]))
    if best is None or c < best[0]:
        best = (c, g)
print("best 16 g(r mod 4):", best)
print("kernel's c ^ 32 (r & 1):", cost(np.array([32 * (r & 1) for r in range(128)])))
rng = np.random.default_rng(0)
for period in (4, 8, 16):
    v = rng.integers(0, 64, period)
    cur = cost(np.array([v[r % period] for r in range(128)]))
    improved = True
    while improved:
        improved = False
        for i in range(period):
            for x in range(64):
                w = v.copy()
                w[i] = x
                c = cost(np.array([w[r % period] for r in range(128)]))
                if c < cur:
                    cur, v, improved = c, w, True
    print(f"local search, period {period}:", cur)
