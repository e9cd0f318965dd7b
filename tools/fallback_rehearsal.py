"""Rehearse bench.py's warm-up fallback from the library gather to torch.distributed's: the first
kzgpot_decode_allgather_dev call raises (as a failing RCCL call would), the bench must finish
verified on the torch path and say so in config.gather_impl. Run at one rank with --gather-at-1:

    python tools/fallback_rehearsal.py --gather-at-1 --steps 1 --no-next-rows --no-cpu-baseline
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "kzg-setup-powersoftau_amd"))

import bench  # noqa: E402
from kzgpot import dist as KD  # noqa: E402

_orig = KD.LibComm.decode_allgather
_calls = {"n": 0}


def _failing_once(self, *a, **k):
    _calls["n"] += 1
    if _calls["n"] == 1:
        raise RuntimeError("kzgpot_decode_allgather_dev(g1_decompress) failed (-100) [injected]")
    return _orig(self, *a, **k)


KD.LibComm.decode_allgather = _failing_once
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[1:]
bench.main()
