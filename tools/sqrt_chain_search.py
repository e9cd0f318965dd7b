"""How many multiplies could a better window table save in the square root's (p-3)/4
exponentiation (csrc/fp381.hpp fp_pow_pm3d4_30)?

The table must stay in registers: 8 odd powers x 13 radix-2^30 digits. For a table T of odd
exponents, the fewest windows covering (p-3)/4 is a DP over its bits (a window starts and ends
on a 1 and its value is in T; zeros between windows are free squarings). A table's build cost
is one multiply per entry that is the sum of two already-built exponents ({1, 2} to start), two
otherwise (a rough model; the chosen table's real chain is counted below). Local search from the
sliding-window table {1, 3, ..., 15} and from random tables, over odd exponents below 256.
The table csrc/fp381.hpp builds, {1, 3, 7, 9, 11, 13, 21, 255}, takes 67 windows; its chain is
a^2, a^3, a^4, a^7, a^9, a^11, a^13, a^8, a^21, a^15, four squarings to a^240, a^255: 9
multiplies + 7 squarings, against 7 + 1 for {1, 3, ..., 15} with its 79 windows.

    python3 tools/sqrt_chain_search.py
"""
import random

P = 0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab
BITS = bin((P - 3) // 4)[2:]


def windows(T, maxw=8):
    f = [0] * (len(BITS) + 1)
    for i in range(len(BITS) - 1, -1, -1):
        if BITS[i] == "0":
            f[i] = f[i + 1]
            continue
        f[i] = min((1 + f[i + w] for w in range(1, maxw + 1)
                    if i + w <= len(BITS) and BITS[i + w - 1] == "1" and int(BITS[i:i + w], 2) in T), default=10 ** 9)
    return f[0]


def build(T):
    have, c = {1, 2}, 0
    for t in sorted(T):
        if t not in have:
            c += 1 if any(t - a in have for a in have) else 2
            have.add(t)
    return c


def muls(T):  # the first window is the accumulator's initial value: no multiply
    return windows(T) - 1 + build(T)


def main():
    cur = set(range(1, 16, 2))
    odd = list(range(3, 256, 2))
    best = (muls(cur), sorted(cur))
    for seed in range(12):
        random.seed(seed)
        T = set(cur) if seed == 0 else {1, *random.sample(odd, 7)}
        c = muls(T)
        better = True
        while better:
            better = False
            for x in sorted(T - {1}):
                for y in odd:
                    if x in T and y not in T and muls((T - {x}) | {y}) < c:
                        T = (T - {x}) | {y}
                        c = muls(T)
                        better = True
        best = min(best, (c, sorted(T)))
    print(f"(p-3)/4: {len(BITS)} bits, {BITS.count('1')} ones")
    print(f"sliding-window table {{1..15 odd}}: {muls(cur)} table + window multiplies ({windows(cur)} windows)")
    print(f"best 8-entry table found: {best[0]} multiplies, table {best[1]}")
    chosen = {1, 3, 7, 9, 11, 13, 21, 255}
    print(f"chosen table {sorted(chosen)}: {windows(chosen)} windows, {windows(chosen) - 1} window multiplies "
          "+ 9 table multiplies + 7 table squarings")
    print(f"16-entry table {{1..31 odd}}: {windows(set(range(1, 32, 2)))} windows (needs 16 x 13 registers)")


if __name__ == "__main__":
    main()
