"""LDS bank pattern of k_bnn_c3's three products (potential_bnn.hip): for every step of each
product's K loop, the 64 lanes' operand addresses (lane = 16 kq + l15; the k-lane permutation
k = 16 kq + s for the first 64 k, then 64 + ((K - 64) / 4) kq + (s - 16)) and the largest number of
distinct addresses that fall in one of the 64 four-byte banks.  Stride 69 for h1 / h2 (= ga2), 73
for W2.  Run by tests/test_bnn_bank_pattern.py.  usage: python scripts/bnn_bank_pattern.py"""
H, W2S = 69, 73


def kmap(kq, s, K):
    return 16 * kq + s if s < 16 else 64 + ((K - 64) // 4) * kq + (s - 16)


def ways(addrs):
    banks = {}
    for a in set(addrs):
        banks.setdefault(a % 64, set()).add(a)
    return max(len(v) for v in banks.values())


PRODUCTS = {  # name: (K, A(m, k) word address, B(k, n) word address)
    "h1 W2": (72, lambda m, k: m * H + k, lambda k, n: k * W2S + n),
    "h1^T ga2": (100, lambda m, k: k * H + m, lambda k, n: k * H + n),
    "ga2 W2^T": (72, lambda m, k: m * H + k, lambda k, n: n * W2S + k),
}


def pattern():
    """{product: (bijective k map, [(step, A ways, B ways)])}"""
    out = {}
    for name, (K, fa, fb) in PRODUCTS.items():
        steps = []
        for s in range(K // 4):
            a = [fa(l15, kmap(kq, s, K)) for kq in range(4) for l15 in range(16)]
            b = [fb(kmap(kq, s, K), l15) for kq in range(4) for l15 in range(16)]
            steps.append((s, ways(a), ways(b)))
        ks = sorted(kmap(kq, s, K) for kq in range(4) for s in range(K // 4))
        out[name] = (ks == list(range(K)), steps)
    return out


if __name__ == "__main__":
    for name, (bij, steps) in pattern().items():
        worst = [(s, a, b) for s, a, b in steps if a > 1 or b > 1]
        print(f"{name:10s} k map bijective {bij}; conflict-free steps {len(steps) - len(worst)}/{len(steps)}; "
              f"others {worst}")
