"""Per-phase cost of the checked codecs ("split k_g2_codec's VALU count by
phase"). On 2^20 synthetic points, for G1 and G2:

  fused     k_gX_codec                          (the default: decompress + subgroup test + emit)
  phase 1   k_gX_decompress alone               (KZGPOT_NO_SUBGROUP_CHECK: flags, x < p, square
                                                 root(s), sign rule, emit — for G2 the two Fp
                                                 exponentiations of the norm-method square root)
  split     k_gX_decompress + k_gX_check<ArkInPlace>  (KZGPOT_SPLIT_PHASES: phase 2 = the record
                                                 re-read, Montgomery conversion and the
                                                 endomorphism ladder: psi(P) = [u]P for G2)

Event-timed here; run under `rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES ...` (tools/profile_round.sh)
the per-kernel VALU instruction counts split the fused kernel's stream by phase
(tools/pmc_summary.py -> pmc_traffic.json "phases").

    python tools/codec_phases.py [--log2 20]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kzg-setup-powersoftau_amd"))

NO_CHECK, SPLIT = 0x1, 0x4


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log2", type=int, default=20)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch

    from kzgpot import device as D

    n = 1 << a.log2
    dev = torch.device("cuda", 0)
    res = {"points": n}
    for kind, rout in (("g1", 96), ("g2", 192)):
        comp, exp = D.synth(kind, 77, 0, n, dev)
        out = torch.empty(n * rout, dtype=torch.uint8, device=dev)
        key = torch.empty(1, dtype=torch.int64, device=dev)
        row = {}
        for name, flags in (("fused", 0), ("phase1", NO_CHECK), ("split", SPLIT)):
            D.codec_dev(f"{kind}_decompress", comp, out, key, flags=flags)  # warm-up
            e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            e[0].record()
            for _ in range(a.reps):
                D.codec_dev(f"{kind}_decompress", comp, out, key, flags=flags)
            e[1].record()
            torch.cuda.synchronize()
            ms = e[0].elapsed_time(e[1]) / a.reps
            row[name] = {"ms": ms, "ns_per_point": ms * 1e6 / n,
                         "bit_exact": bool(D.read_key(key) == (1 << 64) - 1 and torch.equal(out, exp))}
        row["phase2_ms_from_split"] = row["split"]["ms"] - row["phase1"]["ms"]
        res[kind] = row
    print(json.dumps(res))


if __name__ == "__main__":
    main()
