"""Checks the balanced 13 x 30-bit Montgomery multiply/square dump of mont30s.hip:
r 2^390 == a b (mod p), output limbs balanced."""
import struct
import sys

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
R = 1 << 390


def val(limbs):
    return sum(v << (30 * k) for k, v in enumerate(limbs))


def main(path):
    data = open(path, "rb").read()
    words = struct.unpack("<%di" % (len(data) // 4), data)
    bad = 0
    lanes = 256
    for t in range(lanes):
        w = words[t * 52:(t + 1) * 52]
        a, b, rm, rs = w[0:13], w[13:26], w[26:39], w[39:52]
        for r, want in ((rm, val(a) * val(b)), (rs, val(a) * val(a))):
            ok = (val(r) * R - want) % P == 0
            ok = ok and all(-(1 << 29) <= x < (1 << 29) for x in r[:12])
            if not ok:
                bad += 1
        ext = words[256 * 52 + t * 26:256 * 52 + t * 26 + 26]
        for r, want in ((ext[0:13], val(a) * val(b)), (ext[13:26], val(a) * val(a))):
            if (val(r) * R - want) % P != 0 or not all(-(1 << 29) <= x < (1 << 29) for x in r[:12]):
                bad += 1
    print(f"mont30s check: {bad} mismatches over {4 * lanes} products")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
