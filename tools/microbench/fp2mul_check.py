"""Checks tools/microbench/fp2mul.hip's dump: both Fp2 multiplies give a b R^-1 (R = 2^392) mod p."""
import struct
import sys

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
RINV = pow(1 << 392, -1, P)


def val(w):
    return sum(x << (28 * k) for k, x in enumerate(w))


def main(path):
    d = open(path, "rb").read()
    w = struct.unpack("<%dI" % (len(d) // 4), d)
    bad = 0
    for t in range(len(w) // 112):
        o = w[t * 112:(t + 1) * 112]
        a0, a1, b0, b1 = (val(o[14 * k:14 * k + 14]) for k in range(4))
        c0 = (a0 * b0 - a1 * b1) * RINV % P
        c1 = (a0 * b1 + a1 * b0) * RINV % P
        for base in (56, 84):
            r0, r1 = val(o[base:base + 14]), val(o[base + 14:base + 28])
            if r0 % P != c0 or r1 % P != c1 or any(x >> 28 for x in o[base:base + 28]):
                bad += 1
    print(f"fp2mul check: {bad} mismatches over {2 * (len(w) // 112)} products")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
