"""PCIe-inclusive rate of the host-buffer C ABI (kzgpot_g1_decompress on pageable host memory)
against the device-resident kernel rate, on the same synthetic points.

    python tools/host_api_rate.py [--log2 25]
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kzg-setup-powersoftau_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log2", type=int, default=25)
    a = ap.parse_args()
    import torch
    import kzgpot
    from kzgpot import _lib
    from kzgpot import device as D

    dev = torch.device("cuda", 0)
    n = 1 << a.log2
    comp, exp = D.synth("g1", 0x5EED, 0, n, dev, with_expected=True)
    host_in = comp.cpu().numpy()
    want = exp.cpu().numpy().tobytes()
    del exp
    lib = _lib.load()
    out = ctypes.create_string_buffer(n * 96)
    fb = ctypes.c_int64()
    t = time.perf_counter()  # warm: two full 2^21-point chunks size both slots' staging
    lib.kzgpot_g1_decompress(host_in.ctypes.data, ctypes.c_size_t(min(n, 1 << 22)), out, 0, ctypes.byref(fb))
    first_s = time.perf_counter() - t
    t = time.perf_counter()
    rc = lib.kzgpot_g1_decompress(host_in.ctypes.data, ctypes.c_size_t(n), out, 0, ctypes.byref(fb))
    host_s = time.perf_counter() - t
    ok = rc == 0 and out.raw == want
    d_out = torch.empty(n * 96, dtype=torch.uint8, device=dev)
    key = torch.empty(1, dtype=torch.int64, device=dev)
    D.codec_dev("g1_decompress", comp, d_out, key)
    torch.cuda.synchronize()
    t = time.perf_counter()
    D.codec_dev("g1_decompress", comp, d_out, key)
    torch.cuda.synchronize()
    dev_s = time.perf_counter() - t
    print(json.dumps({"points": n, "first_call_2e22_s": first_s, "host_api_s": host_s, "host_api_points_per_s": n / host_s,
                      "device_resident_s": dev_s, "device_points_per_s": n / dev_s,
                      "pcie_overhead_frac": host_s / dev_s - 1, "bit_exact": ok, "kzgpot": kzgpot.version()}))


if __name__ == "__main__":
    main()
