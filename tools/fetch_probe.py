"""One launch of each codec kernel at 2^20 points (after a warm-up launch), for the PMC passes of
tools/pmc_fetch_probe.sh: is the G2 kernels' read overshoot (k_g2_codec 105 B/pt fetched against
96, k_g2_check<PairingBE> 204 against 192) data being re-read, or something
the fabric counters tally that is not the record stream? Every output is checked bit-exact.

    python3 tools/fetch_probe.py            (KZGPOT_LIB selects the library build under test)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kzg-setup-powersoftau_amd"))


def main():
    import argparse

    import torch
    from kzgpot import _lib
    from kzgpot import device as D
    from kzgpot import dist as KD

    ap = argparse.ArgumentParser()
    ap.add_argument("--log2s", default="20", help="comma-separated sizes (a per-launch constant vs a per-point cost)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    res = {}
    for lg in (int(x) for x in a.log2s.split(",")):
        res[lg] = run_size(1 << lg, dev, torch, D, KD)
    print(json.dumps({"bit_exact": res, "lib": _lib.LIB_PATH}))


def run_size(n, dev, torch, D, KD):
    ok = {}
    c1, x1 = D.synth("g1", 11, 0, n, dev)
    c2, x2 = D.synth("g2", 12, 0, n, dev)
    p1 = x1.view(n, 2, 48).flip(-1).contiguous().view(-1)            # pairing-uncompressed G1
    p2 = x2.view(n, 2, 2, 48).flip(2).flip(-1).contiguous().view(-1)  # pairing-uncompressed G2
    key = torch.empty(1, dtype=torch.int64, device=dev)
    for name, op, src, rout, want, flags in (("g1_codec", "g1_decompress", c1, 96, x1, 0),
                                             ("g2_codec", "g2_decompress", c2, 192, x2, 0),
                                             ("g2_decompress_unchecked", "g2_decompress", c2, 192, x2, 1),
                                             ("g1_transcode", "g1_transcode", p1, 96, x1, 0),
                                             ("g2_transcode", "g2_transcode", p2, 192, x2, 0)):
        out = torch.empty(n * rout, dtype=torch.uint8, device=dev)
        for _ in range(2):  # the second launch is the one the summary reads (largest dispatch id)
            D.codec_dev(op, src, out, key, flags)
        torch.cuda.synchronize()
        ok[name] = bool(D.read_key(key) == KD.NO_BAD and torch.equal(out, want))
        del out
    return ok


if __name__ == "__main__":
    main()
