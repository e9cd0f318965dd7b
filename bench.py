#!/usr/bin/env python3
"""Headline benchmark: BLS12-381 Powers-of-Tau points decompressed + checked per second.

BASELINE.json metric: "G1+G2 points decompressed+checked/sec, 2^27 BLS12-381 PoT, 1/2/4/8 GPU".
Workload (config 4): a synthetic transcript of 2^27 compressed G1 + 2^16 compressed G2 points
(valid, distinct, subgroup; ~50 % "greatest" flags), generated on the GPU and resident in HBM
before timing. One step = one pass of the hot path over the whole transcript: every point is
decompressed (Fp / Fp2 square root + sign rule), subgroup-checked and emitted as arkworks
`serialize_uncompressed` bytes — and, for N > 1 GPUs, all-gathered over RCCL into one contiguous
arkworks buffer on every rank (strong scaling: the transcript is fixed, ranks split it).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

`--gpus N > 1` without a launcher starts `torch.distributed.run` itself, as a CHILD process,
before anything touches the GPU, forwards rank 0's JSON line and exits with the child's code;
under a launcher, WORLD_SIZE != --gpus is an error. The line carries RCCL's own view of the
communicator (`rccl_nranks`, per-rank devices) so an N-GPU number is proven to be one.

Prints ONE JSON line (rank 0). `roofline` is for the dominant kernel pair (G1 decompress + G1
check), timed with HIP events on the launch stream; `valu` prices the same launches against the
cycle-weighted integer-VALU issue roof (profiles/r02_valu_mix.json); `cpu_baseline` times the C
restatement of the reference's CPU path (oracle/kzgpot_ref.c, kind "port" — the Rust reference
cannot be built here) on a bounded sample of the same points, with the reference's schedule
(decompression on num_cpus threads as num_cpus 1.13.0 counts them, the arkworks check on one
thread), and `cpu_baseline.e2e` times the reference's whole file-to-file pipeline in its own shape
beside the GPU's end-to-end rows. `next_rows.bn254_g1_decompress`
is config 5 (BN254 2^28 G1), sharded and all-gathered exactly like config 4 at N > 1.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "kzg-setup-powersoftau_amd"))

LOADER_WARM, LOADER_TIMED = 20, 10  # loader rows: ~100 ms of ramp, then 10 timed launches
HBM_PEAK_GBS = 8000.0           # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
SIMDS, CLOCK_HZ = 256 * 4, 2.4e9  # MI355X: 256 CUs x 4 SIMDs at the 2.4 GHz peak engine clock
ALG_BYTES = {"g1": 144, "g2": 288, "bn254": 96}  # bytes read + written per point
# kernel -> its name in profiles/r02_valu_mix.json (demangled; the check kernels' Src 0 = ArkInPlace)
MIX_NAMES = {"k_g1_codec": "kzgpot::k_g1_codec(",
             "k_g1_decompress": "kzgpot::k_g1_decompress(", "k_g1_check": "kzgpot::k_g1_check<(kzgpot::Src)0>",
             "k_g2_codec": "kzgpot::k_g2_codec(",
             "k_g2_decompress": "kzgpot::k_g2_decompress(", "k_g2_check": "kzgpot::k_g2_check<(kzgpot::Src)0>",
             "k_bn254_g1_decompress": "kzgpot::k_bn254_g1_decompress(",
             "k_g1_transcode": "kzgpot::k_g1_check<(kzgpot::Src)1>", "k_g2_transcode": "kzgpot::k_g2_check<(kzgpot::Src)1>"}
RECORDS = {"g1": (48, 96, "g1_decompress"), "g2": (96, 192, "g2_decompress"),
           "bn254": (32, 64, "bn254_g1_decompress")}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--g1-log2", type=int, default=27)
    ap.add_argument("--g2-log2", type=int, default=16)
    ap.add_argument("--seed", type=int, default=0x5EED)
    ap.add_argument("--no-gather", action="store_true", help="skip the RCCL all-gather (N > 1)")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL, the product path) or gloo (rehearsal)")
    ap.add_argument("--gather-impl", default="lib", choices=("lib", "torch"),
                    help="N > 1 with nccl: lib = the library's decode + RCCL all-gather (kzgpot_decode_allgather_dev, "
                         "the product path); torch = torch.distributed all_gather_into_tensor around _dev launches")
    ap.add_argument("--gather-at-1", action="store_true",
                    help="run the N > 1 sharded + gathered path with one rank (rehearses the library's RCCL path "
                         "on a one-GPU box; the number is not the N = 1 headline)")
    ap.add_argument("--gather-chunks", type=int, default=8,
                    help="N > 1: chunks per rank; each chunk's all-gather overlaps the next chunk's decode")
    ap.add_argument("--split-phases", action="store_true",
                    help="G1 and G2: decompress and check as two launches (KZGPOT_SPLIT_PHASES) instead of the fused kernels")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--oracle-sample-runs", type=int, default=64,
                    help="runs of 256 output records (+ the last 256) re-decoded by the C oracle")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-log2", type=int, default=15)
    ap.add_argument("--cpu-e2e-log2", type=int, default=12,
                    help="cpu_baseline.e2e: N of the reference-shaped CPU pipeline, file to file (0 = skip)")
    ap.add_argument("--no-next-rows", action="store_true", help="skip the SURVEY 8f rows and config 5")
    ap.add_argument("--bn254-log2", type=int, default=28, help="config 5 size (0 = skip)")
    ap.add_argument("--e2e-log2", type=int, default=21, help="end-to-end preprocess N (0 = skip)")
    ap.add_argument("--no-cli", dest="cli", action="store_false",
                    help="skip the drop-in binaries' wall-clock rows (next_rows.cli_preprocess_*)")
    ap.add_argument("--no-host-api", dest="host_api", action="store_false",
                    help="skip the host-buffer FFI rows (next_rows.host_api)")
    return ap.parse_args()


def oracle_lib():
    path = os.path.join(ROOT, "oracle", "_build", "libkzgpot_oracle.so")
    return ctypes.CDLL(path) if os.path.exists(path) else None


def affinity_cpus():
    try:
        return len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return os.cpu_count() or 1


def cgroup_v1_cpu_quota(cgroup="/proc/self/cgroup", mountinfo="/proc/self/mountinfo"):
    """ceil(cpu.cfs_quota_us / cpu.cfs_period_us) of this process's cgroup-v1 cpu controller, or None
    (no v1 cpu controller, or no quota) — what num_cpus 1.13.0 reads (/proc/self/cgroup +
    /proc/self/mountinfo). It does not read cgroup v2's cpu.max."""
    try:
        rel = next(ln.rstrip("\n").split(":", 2)[2] for ln in open(cgroup)
                   if "cpu" in ln.split(":", 2)[1].split(","))
        for ln in open(mountinfo):
            pre, post = ln.split(" - ", 1)
            f, opts = pre.split(), post.split()
            if opts[0] != "cgroup" or "cpu" not in opts[2].split(","):
                continue
            root, mnt = f[3], f[4]
            sub = rel[len(root):] if rel.startswith(root) else rel
            d = os.path.join(mnt, sub.lstrip("/"))
            quota = int(open(os.path.join(d, "cpu.cfs_quota_us")).read())
            period = int(open(os.path.join(d, "cpu.cfs_period_us")).read())
            return -(-quota // period) if quota > 0 and period > 0 else None
    except (OSError, ValueError, StopIteration, IndexError):
        pass
    return None


def num_cpus():
    """The thread count the reference's `num_cpus::get()` returns on this host (num_cpus 1.13.0, the
    version in /root/reference/Cargo.lock): min(cgroup-v1 CPU quota, affinity CPUs) when a v1 quota
    is set, else the affinity mask's CPU count. powersoftau's decompress_all sizes its chunks by it."""
    q = cgroup_v1_cpu_quota()
    return min(q, affinity_cpus()) if q else affinity_cpus()


def cgroup_v2_cpu_max():
    """This process's cgroup-v2 cpu.max ("quota period" or "max period"), recorded beside the
    thread counts: the CPU share the box actually grants, which num_cpus 1.13.0 does not see."""
    try:
        rel = next(ln.rstrip("\n").split(":", 2)[2] for ln in open("/proc/self/cgroup") if ln.startswith("0::"))
        return open(os.path.join("/sys/fs/cgroup", rel.lstrip("/"), "cpu.max")).read().strip()
    except (OSError, StopIteration):
        return None


def host_cpu():
    """The box's CPU as SURVEY §8d asks it recorded beside the baseline: model, nproc, affinity,
    and the cgroup CPU limits."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), None)
    except OSError:
        pass
    return {"cpu_model": model, "nproc": os.cpu_count(), "affinity_cpus": affinity_cpus(),
            "cgroup_v1_cpu_quota": cgroup_v1_cpu_quota(), "cgroup_v2_cpu_max": cgroup_v2_cpu_max()}


def cpu_baseline(comp1, comp2, sample_log2):
    """Reference-schedule CPU timing of the oracle restatement on a bounded sample: decompression
    on num_cpus() threads (powersoftau decompress_all, preprocess-kgz.rs:105-110), the read_g1 /
    read_g2 subgroup check + serialize on one thread (preprocess-kgz.rs:128-160)."""
    lib = oracle_lib()
    if lib is None:
        return None
    s1 = min(1 << sample_log2, comp1.numel() // 48)
    s2 = max(1, min(s1 >> 11, comp2.numel() // 96))  # keep the workload's G1:G2 ratio (2^27 : 2^16)
    h1 = bytes(comp1[: s1 * 48].cpu().numpy())
    h2 = bytes(comp2[: s2 * 96].cpu().numpy())
    cores, every = num_cpus(), affinity_cpus()
    o1 = ctypes.create_string_buffer(s1 * 96)
    o2 = ctypes.create_string_buffer(s2 * 192)
    fb = ctypes.c_int64()
    t = time.perf_counter()
    r1 = lib.oracle_g1_decompress(h1, ctypes.c_size_t(s1), o1, 0, ctypes.byref(fb), None, cores, 1)
    r2 = lib.oracle_g2_decompress(h2, ctypes.c_size_t(s2), o2, 0, ctypes.byref(fb), None, cores, 1)
    dt = time.perf_counter() - t
    # SURVEY §8d's second schedule: every stage on every CPU of the affinity mask (what a
    # parallelised reference could do)
    t = time.perf_counter()
    a1 = lib.oracle_g1_decompress(h1, ctypes.c_size_t(s1), o1, 0, ctypes.byref(fb), None, every, every)
    a2 = lib.oracle_g2_decompress(h2, ctypes.c_size_t(s2), o2, 0, ctypes.byref(fb), None, every, every)
    dt_all = time.perf_counter() - t
    # thread-count sweep of the same all-stages schedule: where the box's CPU share saturates (the
    # affinity mask can list more CPUs than the scheduler grants this process). SURVEY §8d's
    # "all-cores: every stage parallel" is the best parallel CPU, so the all-cores figure is the
    # sweep's best point with its thread count; the every-affinity-CPU run is kept beside it
    # (on the r05 box 256 threads ran 1.8x slower than 16).
    sweep = {}
    for th in sorted({4, 8, 16, 24, 32, 48, 64, 128} - {every}) + [every]:
        if th > every or th < 1:
            continue
        if th == every:
            sweep[str(th)] = (s1 + s2) / dt_all
            continue
        t = time.perf_counter()
        lib.oracle_g1_decompress(h1, ctypes.c_size_t(s1), o1, 0, ctypes.byref(fb), None, th, th)
        lib.oracle_g2_decompress(h2, ctypes.c_size_t(s2), o2, 0, ctypes.byref(fb), None, th, th)
        sweep[str(th)] = (s1 + s2) / (time.perf_counter() - t)
    best_th = max(sweep, key=lambda k: sweep[k])
    # CPUs the process effectively receives: the best rate over the 4-thread rate per thread
    per_thread = sweep.get("4", 0) / 4 if "4" in sweep else None
    return {
        "value": (s1 + s2) / dt, "unit": "points/s", "cores": cores, "kind": "port", **host_cpu(),
        "threads_decompress": cores, "threads_check": 1,
        "sample": f"{s1} G1 + {s2} G2 from the bench transcript, reference schedule "
                  f"(decompress on num_cpus = {cores} threads, arkworks subgroup check + serialize on 1 thread); "
                  f"{dt:.1f} s; rc={r1},{r2}",
        "seconds": dt,
        "all_cores": {"value": sweep[best_th], "threads": int(best_th),
                      "schedule": f"decompress and subgroup check both on {best_th} threads: the best point of the "
                                  f"thread sweep (points_per_s_by_threads) of the every-stage-parallel schedule",
                      "saturation_threads": int(best_th),
                      "effective_cpus": None if not per_thread else sweep[best_th] / per_thread,
                      "at_affinity_cpus": {"value": (s1 + s2) / dt_all, "seconds": dt_all, "threads": every,
                                           "rc": [a1, a2]},
                      "points_per_s_by_threads": sweep},
    }


def e2e_transcript(n_log2, seed, dev, D, expect_names=()):
    """A powersoftau response-layout transcript of GPU-generated valid points (as the reference's
    `powersoftau` file: 64-B hash, τG1 2N-1, τG2 N, ατG1 N, βτG1 N, βG2 1, public key) as a host
    numpy array, plus the generator's expected ark bytes of the sections named in expect_names."""
    import torch

    n = 1 << n_log2
    parts, expect = [torch.zeros(64, dtype=torch.uint8, device=dev)], {}
    for name, kind, cnt in (("tau_g1", "g1", 2 * n - 1), ("tau_g2", "g2", n), ("alpha_g1", "g1", n),
                            ("beta_g1", "g1", n), ("beta_g2", "g2", 1)):
        c, e = D.synth(kind, seed + len(parts), 0, cnt, dev, with_expected=name in expect_names)
        parts.append(c)
        if e is not None:
            expect[name] = e.cpu().numpy()
    parts.append(torch.zeros(3 * 192 + 6 * 96, dtype=torch.uint8, device=dev))
    tr = torch.cat(parts).cpu().numpy()
    return tr, expect


def cpu_e2e(n_log2, seed, dev, D, kzgpot, gpu_rows):
    """cpu_baseline.e2e: the reference's whole `main` in its own shape (oracle_preprocess_pipeline,
    oracle/kzgpot_ref.c: transcript BLAKE2b check, HashReader + decompress_all on num_cpus threads,
    the pairing-uncompressed intermediate file written and read back, read_g1 / read_g2 on one
    thread, one unbuffered write() per coordinate; preprocess-kgz.rs:32-199,
    preprocess-fastkgz.rs:129-213) file to file on a bounded N, per point beside the GPU's
    preprocess_* rows (same point count per N: 2N-1 + 3N + 1). The GPU's kzgpot_preprocess_ex
    runs on the same transcript file and its output must be byte-identical."""
    import hashlib

    import numpy as np
    from kzgpot import _lib

    lib = oracle_lib()
    if lib is None or n_log2 <= 0:
        return None
    n = 1 << n_log2
    pts = (2 * n - 1) + 3 * n + 1
    tr, _ = e2e_transcript(n_log2, seed, dev, D)
    tmpdir = tempfile.mkdtemp(prefix="kzgpot_cpu_e2e_")
    try:  # the temporary directory goes whatever happens in between
        src = os.path.join(tmpdir, "powersoftau")
        tr.tofile(src)
        digest = hashlib.blake2b(tr.tobytes()).hexdigest()
        cores = num_cpus()
        glib = _lib.load()
        rows = {}
        for mode, name in ((kzgpot.MODE_KZG, "kgz"), (kzgpot.MODE_FASTKZG, "fastkgz")):
            unc, dst, gdst = (os.path.join(tmpdir, x) for x in ("powersoftau_uncompressed", "out", "gpu_out"))
            stages = (ctypes.c_double * 5)()
            t = time.perf_counter()
            r = lib.oracle_preprocess_pipeline(src.encode(), unc.encode(), dst.encode(), ctypes.c_uint64(n), mode, cores,
                                               digest.encode(), None, stages)
            dt = time.perf_counter() - t
            sec, idx = ctypes.c_int(-1), ctypes.c_int64(-1)
            rg = glib.kzgpot_preprocess_ex(src.encode(), gdst.encode(), mode, n_log2, 1, digest.encode(), None, None,
                                           ctypes.byref(sec), ctypes.byref(idx))
            same = r == 0 and rg == 0 and np.array_equal(np.fromfile(dst, np.uint8), np.fromfile(gdst, np.uint8))
            for f in (unc, dst, gdst):
                if os.path.exists(f):
                    os.unlink(f)
            st = list(stages)
            # per-point cost of each stage, scaled to the reference's N = 2^21 (every stage is linear in N)
            scale = ((2 << 21) - 1 + 3 * (1 << 21) + 1) / pts
            gpu = gpu_rows.get(f"preprocess_{name}_e2e_file_transcript_digest") if gpu_rows else None
            rows[name] = {
                "n_log2": n_log2, "points": pts, "seconds": dt, "points_per_s": pts / dt, "rc": r,
                "threads_decompress": cores, "threads_check": 1,
                "stages_s": {"transcript_blake2b_check": st[0], "read_hash_decompress": st[1],
                             "write_uncompressed_intermediate": st[2], "read_g1_g2_subgroup_check": st[3],
                             "write_output_unbuffered": st[4]},
                "extrapolated_s_at_2e21": dt * scale,
                "output_equal_to_gpu_kzgpot_preprocess_ex": bool(same),
                "gpu_row": None if gpu is None else {"row": f"next_rows.preprocess_{name}_e2e_file_transcript_digest",
                                                     "points_per_s": gpu["points_per_s"],
                                                     "speedup_per_point": gpu["points_per_s"] / (pts / dt)}}
    finally:
        shutil.rmtree(tmpdir, ignore_errors=True)
    return {"unit": "points/s", "kind": "port", "cores": cores,
            "sample": f"N = 2^{n_log2} synthetic response transcript ({tr.size} B) file to file per mode, the "
                      "reference's pipeline shape (oracle_preprocess_pipeline); stage times linear in N",
            **rows}


def load_json(name):
    try:
        return json.load(open(os.path.join(ROOT, "profiles", name)))
    except (OSError, ValueError):
        return None


def pmc_traffic(pmc, n_g1_local):
    """HBM bytes per G1 codec launch (decompress + check) from the PMC FETCH/WRITE passes."""
    try:
        return pmc["g1_bytes_per_point"] * n_g1_local
    except (TypeError, KeyError):
        return None


def valu_roofline(pmc, mix, kernels, points, ms, clock=None):
    """Integer-VALU roof of a kernel group: PMC SQ_INSTS_VALU per wave (the instruction stream one
    lane runs for its point) x waves / the event-timed launch time, against the SIMDs' issue rate
    for THAT instruction mix — each opcode priced at its measured SIMD cycles per wave64
    instruction (tools/microbench/valu_issue.hip -> profiles/r02_valu_issue_microbench.txt;
    v_mad_u64_u32 4.4, v_add_u32 2.1, other VOP3 ~4.2), weighted by the kernel's opcode histogram
    (tools/valu_mix.py -> profiles/r02_valu_mix.json)."""
    try:
        insts = [pmc["kernels"][k]["valu_insts_per_wave"] for k in kernels]
        costs = [next(e["avg_cycles_per_valu"] for name, e in mix["kernels"].items() if MIX_NAMES[k] in name)
                 for k in kernels]
    except (TypeError, KeyError, StopIteration):
        return None
    per_pt = sum(insts)
    avg_cost = sum(i * c for i, c in zip(insts, costs)) / per_pt
    peak = SIMDS * CLOCK_HZ / avg_cost
    achieved = per_pt * (points / 64) / (ms * 1e-3)
    at_clock = {} if not clock else {
        "frac_at_measured_clock": achieved / (SIMDS * clock["mean"] * 1e6 / avg_cost), "measured_clock_mhz": clock["mean"]}
    return {"kernels": kernels, "valu_instr_per_point": per_pt, "avg_simd_cycles_per_instr": avg_cost,
            "achieved_wave_instr_per_s": achieved, "peak_wave_instr_per_s": peak, "frac": achieved / peak, **at_clock,
            "source": "instruction counts: profiles/pmc_traffic.json (SQ_INSTS_VALU); per-opcode SIMD cycles: "
                      "profiles/r02_valu_issue_microbench.txt weighted by profiles/r02_valu_mix.json; "
                      "peak = 1024 SIMDs x 2.4 GHz / avg cycles; time: this run"}


def field_ops(census, op, points, ms):
    """SURVEY §8d's Fp-multiply view of a codec kernel: its Montgomery reductions per point by kind
    (the product kernels rebuilt with fp381.hpp's counting hook, tools/fpops/fp_census.hip) x this
    run's points/s, and the fraction of the launch that those reductions would take at each
    primitive's own microbenchmarked chip-wide peak (tools/microbench/fpops_peak.hip, 2 waves per
    SIMD like the codecs). A fraction near 1 says the kernel's time is its reductions: the
    additions, normalisations, selects and memory traffic are all hidden behind them."""
    try:
        row = next(r for r in census["rows"] if r["op"] == op and r["flags"] == 0)
        peaks = {k: census["peaks_G_per_s"][k]["best_at_2_waves"] for k in row["per_point"]}
    except (TypeError, KeyError, StopIteration):
        return None
    pps = points / (ms * 1e-3)
    t_peak = sum(c / (peaks[k] * 1e9) for k, c in row["per_point"].items())
    return {"reductions_per_point": row["reductions_per_point"], "by_kind": row["per_point"],
            "reductions_per_s": row["reductions_per_point"] * pps, "peak_G_per_s": peaks,
            "reduction_time_at_peak_ns_per_point": t_peak * 1e9, "launch_ns_per_point": 1e9 / pps,
            "frac": t_peak * pps,
            "source": "counts and peaks: profiles/fp_census.json (tools/fpops/census.py, peaks "
                      + str(census.get("peaks_source")) + ", measured on another box than this run)"}


class Sharded:
    """One point stream of n records decoded across the ranks. N > 1 with the gather: block-cyclic
    (kzgpot/dist.py) in `chunks` chunks whose in-place all-gathers overlap the next chunk's
    decoding, into one contiguous arkworks buffer on every rank; otherwise one contiguous shard."""

    def __init__(self, kind, n, seed, chunks, rank, world, gather, dev, verify, comm=None, flags=0):
        import torch

        from kzgpot import device as D
        from kzgpot import dist as KD

        self.D, self.KD, self.torch = D, KD, torch
        self.kind, self.n, self.seed, self.rank, self.world, self.gather = kind, n, seed, rank, world, gather
        self.rin, self.rout, self.op = RECORDS[kind]
        self.comm, self.chunks, self.flags = (comm if gather else None), chunks, flags
        if self.comm is not None:  # the library's own decode + RCCL all-gather (kzgpot_decode_allgather_dev)
            self.blocks = KD.lib_local_ranges(n, rank, world, chunks)
        elif gather:
            b = KD.cyclic_block(n, world, chunks)
            self.blocks = [(g, b) for g in KD.owned_block_starts(n, rank, world, chunks)]
        else:
            lo, hi = KD.shard_bounds(n, rank, world)
            self.blocks = [(lo, hi - lo)]
        self.m = sum(c for _, c in self.blocks)
        parts = [D.synth(kind, seed, g, c, dev, with_expected=verify) for g, c in self.blocks]
        self.comp = torch.cat([p[0] for p in parts]) if len(parts) > 1 else parts[0][0]
        self.exps = [p[1] for p in parts]
        self.out = torch.empty((n if gather else self.m) * self.rout, dtype=torch.uint8, device=dev)
        self.keys = torch.full((len(self.blocks),), -1, dtype=torch.int64, device=dev)  # one first-bad key per launch

    def dst(self, c):
        g0, cnt = self.blocks[c]
        off = g0 if self.gather else sum(x for _, x in self.blocks[:c])
        return self.out[off * self.rout:(off + cnt) * self.rout]

    def launch(self, c, marks):
        cnt = self.blocks[c][1]
        src = self.comp[sum(x for _, x in self.blocks[:c]) * self.rin:][:cnt * self.rin]
        e = None
        if marks is not None:
            e = [self.torch.cuda.Event(enable_timing=True) for _ in range(2)]
            e[0].record()
        self.D.codec_dev(self.op, src, self.dst(c), self.keys[c:c + 1], flags=self.flags)
        if marks is not None:
            e[1].record()
            marks.append((self.kind, e))

    def step(self, marks):
        """Launch every block; returns the collective handles (wait on them before reading out)."""
        if self.comm is not None:  # one library call: decode + pipelined in-place RCCL all-gathers
            e = None
            if marks is not None:
                e = [self.torch.cuda.Event(enable_timing=True) for _ in range(2)]
                e[0].record()
            self.comm.decode_allgather(self.op, self.comp, self.n, self.chunks, self.out, self.keys[0:1], self.flags)
            if marks is not None:
                e[1].record()
                marks.append((self.kind, e))
            return []
        if self.gather:
            return self.KD.decode_gather_pipelined(lambda c, g0, dst: self.launch(c, marks), self.out, self.rout,
                                                   self.n, self.rank, self.world, len(self.blocks))
        for c in range(len(self.blocks)):
            self.launch(c, marks)
        return []

    def bad_key(self):
        if self.comm is not None:  # already global (all-reduced inside the library)
            return self.D.read_key(self.keys[0:1])
        return min(self.KD.key_with_offset(self.D.read_key(self.keys[c:c + 1]), self.blocks[c][0])
                   for c in range(len(self.blocks)))

    def verify(self):
        """Own blocks bit-exact against the generator's expected ark bytes; blocks decoded by the
        other ranks by two 64-bit checksums against their owners'."""
        torch, dist = self.torch, self.KD.dist
        ok = self.bad_key() == self.KD.NO_BAD
        for c, e in enumerate(self.exps):
            ok = ok and torch.equal(self.dst(c), e)
        if self.gather and self.world > 1:
            b = self.blocks[0][1]
            nb = self.world * self.chunks  # the exchanged blocks (a library-layout tail is every rank's own)
            mine = torch.zeros(nb, 2, dtype=torch.int64, device=self.out.device)
            w = torch.arange(1, b * self.rout // 8 + 1, dtype=torch.int64, device=self.out.device)
            for (g0, cnt), e in zip(self.blocks, self.exps):
                if cnt != b or g0 >= nb * b:
                    continue
                v = e.view(torch.int64)
                mine[g0 // cnt] = torch.stack([v.sum(), (v * w).sum()])
            dist.all_reduce(mine)  # each block has exactly one owner
            got = self.out[:nb * b * self.rout].view(torch.int64).view(nb, -1)
            ok = ok and torch.equal(torch.stack([got.sum(1), (got * w).sum(1)], 1), mine)
        self.exps = None
        return bool(ok)


def all_ok(ok, world, dev):
    import torch
    import torch.distributed as dist

    if world > 1:
        t = torch.tensor([1 if ok else 0], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        ok = bool(t.item())
    return ok


FALLBACKS = []  # gather-path fallbacks taken during warm-up (reported in the JSON line)
LAST_CLOCK = {}  # average shader clock over the last timed region (kzgpot.device.clock_mhz)


WAIT_MS = 120_000  # warm-up: kzgpot_comm_wait's watchdog (a lost collective aborts instead of hanging)


def lib_to_torch_gather(streams, err):
    """Warm-up insurance for the multi-GPU run: if kzgpot_decode_allgather_dev failed on any rank
    in-band (every collective still issued, agreed by kzgpot.dist.agree_on_failure), EVERY rank
    finishes with torch.distributed's all-gathers over the same block-cyclic layout (identical
    blocks when n splits into world x chunks equal blocks, as every bench stream does). Returns
    False if a stream cannot switch."""
    switch = [s for s in streams if s.comm is not None]
    if not switch or any(s.n % (s.world * s.chunks) for s in switch):
        return False
    for s in switch:
        s.comm = None
    FALLBACKS.append(f"library decode_allgather failed in warm-up ({err}); torch.distributed gathers")
    print(f"warning: {FALLBACKS[-1]}", file=sys.stderr)
    return True


def first_warmup_step(streams, world, dev):
    """Warm-up step 0, collective-safe: every stream is stepped even if an earlier one raised (the
    library issues all of a call's collectives even when its decode fails, so peers stay in step),
    library streams are completed through kzgpot_comm_wait (its status is the all-reduced key, the
    same on every rank), and the ranks agree on ok / fallback / abort before anything else runs."""
    import torch
    from kzgpot import dist as KD

    failed, aborted, errs = False, False, []
    for s in streams:
        try:
            for w in s.step(None):
                w.wait()
        except RuntimeError as e:
            failed = True
            errs.append(str(e))
    for s in streams:
        if s.comm is not None:
            rc, _ = s.comm.wait(s.keys[0:1], timeout_ms=WAIT_MS)
            if rc in (-101, -107):  # KZGPOT_E_DEVICE / KZGPOT_E_TIMEOUT: the communicator is aborted
                aborted = True
                errs.append(f"kzgpot_comm_wait: {rc}")
            elif rc == -106:  # KZGPOT_E_RANK_FAILED: some rank's decode failed, collectives complete
                failed = True
                errs.append("kzgpot_comm_wait: a rank failed")
    if not aborted:
        torch.cuda.synchronize()
    verdict = KD.agree_on_failure(failed, aborted, dev if world > 1 and KD.dist.get_backend() == "nccl" else "cpu")
    if verdict == "abort":
        raise RuntimeError(f"library communicator aborted in warm-up on some rank ({'; '.join(errs) or 'peer'})")
    if verdict == "fallback":
        if not lib_to_torch_gather(streams, "; ".join(errs) or "a peer rank failed"):
            raise RuntimeError(f"warm-up failed and no fallback applies ({'; '.join(errs)})")
        for s in streams:
            for w in s.step(None):
                w.wait()


def timed(streams, steps, warmup, world, dev, verify):
    """W untimed warm-up steps, (verification), then EXACTLY `steps` steps bracketed by a barrier +
    synchronize; returns (max-over-ranks seconds, per-step event marks, verified)."""
    import torch
    import torch.distributed as dist
    from kzgpot import device as D

    def step(marks):
        works = []
        for s in streams:
            works += s.step(marks)
        for w in works:
            w.wait()  # the current stream waits for the collectives

    for i in range(warmup):
        if i == 0:
            first_warmup_step(streams, world, dev)
        else:
            step(None)
    torch.cuda.synchronize()
    verified = None
    if verify:
        if warmup == 0:
            step(None)
            torch.cuda.synchronize()
        verified = all_ok(all(s.verify() for s in streams), world, dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev = []
    probe0 = D.clock_probe(dev)  # shader-clock counters at the start of the timed steps (a ~µs kernel)
    t0 = time.perf_counter()
    for _ in range(steps):
        marks = []
        step(marks)
        ev.append(marks)
    probe1 = D.clock_probe(dev)  # ... and after them, on the same stream
    torch.cuda.synchronize()
    LAST_CLOCK["mhz"] = D.clock_mhz(probe0, probe1)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, ev, verified


def loader_row(kind, src, out, key, m, what):
    """the loader kernel over m records. The GPU's clocks ramp for ~50 ms of
    sustained work after an idle spell (here the oracle check before it): 5.8-6.0 ms for the first
    launch, 4.6-4.8 ms from about the tenth on (profiles/r04n2_loader_timing.json), so the row warms
    up for LOADER_WARM launches, reports the first (cold) one, and times LOADER_TIMED launches."""
    import torch
    from kzgpot import device as D
    from kzgpot import dist as KD

    rec_b = {"g1": 96 + 104, "g2": 192 + 200}[kind]
    e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    e[2].record()
    D.codec_dev(f"{kind}_load", src, out, key)
    e[3].record()
    for _ in range(LOADER_WARM - 1):
        D.codec_dev(f"{kind}_load", src, out, key)
    e[0].record()
    for _ in range(LOADER_TIMED):
        D.codec_dev(f"{kind}_load", src, out, key)
    e[1].record()
    torch.cuda.synchronize()
    ms = e[0].elapsed_time(e[1]) / LOADER_TIMED
    gbs = rec_b * m / (ms * 1e-3) / 1e9
    return {"kernel": f"k_{kind}_load ({what} per-point work)", "points": m, "launch_ms": ms,
            "cold_launch_ms": e[2].elapsed_time(e[3]), "warm_launches": LOADER_WARM, "timed_launches": LOADER_TIMED,
            "points_per_s": m / (ms * 1e-3), "algorithmic_bytes_per_point": rec_b,
            "achieved_GBs": gbs, "peak_GBs": HBM_PEAK_GBS, "hbm_frac": gbs / HBM_PEAK_GBS,
            "all_accepted": D.read_key(key) == KD.NO_BAD}


def g2_vs_g1(g1v, g2v, g1_ms, g2_ms):
    """Clock-free efficiency of the G2 codec relative to the G1 codec launched alternately with it:
    (G2 : G1 time predicted by their VALU counts x opcode-mix cycles) / (measured G2 : G1 time).
    1.0 = G2 converts its instructions into time exactly as well as G1 does."""
    try:
        model = (g2v["valu_instr_per_point"] * g2v["avg_simd_cycles_per_instr"]) / \
                (g1v["valu_instr_per_point"] * g1v["avg_simd_cycles_per_instr"])
    except (TypeError, KeyError):
        return None
    return {"model_time_ratio": model, "measured_time_ratio": g2_ms / g1_ms, "efficiency": model / (g2_ms / g1_ms)}


def transcode_row(kind, pin, out, key, want, n):
    """SURVEY §8f row 3 (the reference's read_g1 / read_g2 loop, preprocess-kgz.rs:140-153,
    src/lib.rs:41-80): one event-timed launch of the transcode kernel over n pairing-uncompressed
    records (already warmed up by the caller), checked bit-exact, with its integer-VALU roof and
    the PMC traffic per point against the algorithmic 2 x record bytes."""
    import torch
    from kzgpot import device as D
    from kzgpot import dist as KD

    rec = 96 if kind == "g1" else 192
    e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    e[0].record()
    D.codec_dev(f"{kind}_transcode", pin, out, key)
    e[1].record()
    torch.cuda.synchronize()
    ms = e[0].elapsed_time(e[1])
    pmc = load_json("pmc_traffic.json")
    name = f"k_{kind}_transcode"
    try:
        traffic = pmc["kernels"][name]["bytes_per_point"]
    except (TypeError, KeyError):
        traffic = None
    return {"kernel": f"k_{kind}_check<PairingBE> (read_{kind}: flags, coordinates < p, curve test, subgroup, "
                      "ark emit)",
            "points": n, "launch_ms": ms, "points_per_s": n / (ms * 1e-3), "ns_per_point": ms * 1e6 / n,
            "algorithmic_bytes_per_point": 2 * rec, "pmc_bytes_per_point": traffic,
            "valu": valu_roofline(pmc, load_json("r02_valu_mix.json"), [name], n, ms),
            "verified_bit_exact": bool(D.read_key(key) == KD.NO_BAD and torch.equal(out, want))}


def gather_label(gather_impl, args):
    """What actually moved the blocks: the library's RCCL all-gather only when it ran (nccl backend,
    library communicator, no warm-up fallback); otherwise torch.distributed over the backend used."""
    if gather_impl and gather_impl.startswith("libkzgpot") and not FALLBACKS:
        return "RCCL all-gather inside libkzgpot"
    backend = "RCCL" if args.dist_backend == "nccl" else args.dist_backend
    return f"torch.distributed all-gather over {backend}"


def kernel_ms(ev, kind):
    """Average per-step event time of one kind's launches (on the launch stream)."""
    return sum(e[0].elapsed_time(e[1]) for marks in ev for k, e in marks if k == kind) / max(1, len(ev))


def oracle_sample_check(stream, runs):
    """Independent re-decode of the FULL-size output by the C oracle: `runs`
    runs of 256 records spread evenly over the whole stream plus its last 256 records (past the
    4 GiB output offset), their compressed inputs regenerated by index; bytes and accept/reject
    must equal the oracle's (the reference algorithm: pairing sqrt + ark mul_bits(r) check)."""
    lib = oracle_lib()
    if lib is None or runs <= 0:
        return None
    n, D = stream.n, stream.D
    starts = sorted(set([k * (n // runs) for k in range(runs)] + [n - 256]))
    fn = {"g1": lib.oracle_g1_decompress, "g2": lib.oracle_g2_decompress}.get(stream.kind)
    if fn is None:
        return None
    cores, ok, pts = affinity_cpus(), True, 0
    t = time.perf_counter()
    for s in starts:
        g = stream.out[s * stream.rout:(s + 256) * stream.rout]  # gathered buffer (or the N = 1 output)
        comp, _ = D.synth(stream.kind, stream.seed, s, 256, stream.out.device, with_expected=False)
        data = bytes(comp.cpu().numpy())
        want = ctypes.create_string_buffer(256 * stream.rout)
        st = ctypes.create_string_buffer(256)
        fb = ctypes.c_int64(-1)
        r = fn(data, ctypes.c_size_t(256), want, 0, ctypes.byref(fb), st, cores, cores)
        ok = ok and r == 0 and fb.value == -1 and st.raw == bytes(256) and bytes(g.cpu().numpy()) == want.raw
        pts += 256
    return {"kind": stream.kind, "points": pts, "runs": len(starts), "last_record_offset_bytes": (n - 1) * stream.rout,
            "oracle": "oracle/kzgpot_ref.c (reference algorithms: Fq sqrt a^((p-3)/4), ark mul_bits(r) subgroup)",
            "equal": bool(ok), "seconds": time.perf_counter() - t}


def host_api_rows(seed, dev, D, g1_log2=25, g2_log2=20):
    """The FFI boundary the Rust caller binds (include/kzgpot.h): kzgpot_g1_decompress /
    kzgpot_g2_decompress on PAGEABLE host buffers, as `read_g1` x N is replaced
    (src/lib.rs:41-80, preprocess-kgz.rs:140-153), timed around the C call: PCIe both ways
    included (run_host pipelines chunks of up to 2^21 points over two streams, ramping from and back
    to 2^17-point chunks at both ends of a long call: csrc/capi.hip ChunkPlan). Beside each, the same points
    device-resident (the `_dev` launch, event-timed), so the PCIe overhead is explicit. The first
    call sizes the staging and faults the output pages in; the steady-state call is the row."""
    import numpy as np
    import torch
    from kzgpot import _lib
    from kzgpot import dist as KD

    lib = _lib.load()
    rows = {}
    for kind, lg, fn, rout in (("g1", g1_log2, lib.kzgpot_g1_decompress, 96),
                               ("g2", g2_log2, lib.kzgpot_g2_decompress, 192)):
        n = 1 << lg
        comp, exp = D.synth(kind, seed, 0, n, dev, with_expected=True)
        host_in = comp.cpu().numpy()
        want = exp.cpu().numpy()
        out = np.empty(n * rout, np.uint8)  # pageable, as a Rust Vec<u8>
        fb = ctypes.c_int64()
        t = time.perf_counter()
        rc0 = fn(host_in.ctypes.data, ctypes.c_size_t(n), out.ctypes.data, 0, ctypes.byref(fb))
        first_s = time.perf_counter() - t
        out[:] = 0
        t = time.perf_counter()
        rc = fn(host_in.ctypes.data, ctypes.c_size_t(n), out.ctypes.data, 0, ctypes.byref(fb))
        host_s = time.perf_counter() - t
        ok = rc0 == 0 and rc == 0 and fb.value == -1 and np.array_equal(out, want)
        d_out = torch.empty(n * rout, dtype=torch.uint8, device=dev)
        key = torch.empty(1, dtype=torch.int64, device=dev)
        D.codec_dev(f"{kind}_decompress", comp, d_out, key)
        e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        e[0].record()
        D.codec_dev(f"{kind}_decompress", comp, d_out, key)
        e[1].record()
        torch.cuda.synchronize()
        dev_s = e[0].elapsed_time(e[1]) * 1e-3
        ok = ok and D.read_key(key) == KD.NO_BAD and torch.equal(d_out, exp)
        rows[f"{kind}_decompress"] = {
            "entry_point": f"kzgpot_{kind}_decompress (pageable host in/out, synchronous)",
            "points": n, "seconds": host_s, "points_per_s": n / host_s,
            "device_resident_s": dev_s, "device_resident_points_per_s": n / dev_s,
            "pcie_overhead_frac": host_s / dev_s - 1,
            "pcie_bytes": n * (rout + rout // 2), "first_call_s": first_s, "verified_bit_exact": bool(ok)}
        del comp, exp, d_out, host_in, want, out
        torch.cuda.empty_cache()
    return rows


def e2e_preprocess(n_log2, seed, dev, kzgpot, D, n_gpus=1):
    """Build a synthetic response transcript (powersoftau layout, GPU-generated valid points) and
    time the C ABI end to end: kzgpot_preprocess_buffer_ex (host buffers in and out, the output
    buffer pre-faulted; the Python wrapper's extra copies are not the product) without digests and
    with both, and kzgpot_preprocess_ex file to file twice — with the transcript digest only (what
    the reference computes: download_parameters' check, preprocess-kgz.rs:32-67; it never hashes
    its output) and with both digests. Each digest row states the single-stream BLAKE2b floor it
    is bound by (the bytes the longest digest covers / this box's kzgpot_blake2b rate) and its
    fraction of it. Checks the τG1 / ατG1 sections and both digests against hashlib, and the
    written files against the buffer output."""
    import hashlib

    import numpy as np
    import torch
    from kzgpot import _lib

    n = 1 << n_log2
    tr, expect = e2e_transcript(n_log2, seed, dev, D, ("tau_g1", "alpha_g1"))
    assert tr.size == kzgpot.contribution_size(n_log2)
    tr_digest = hashlib.blake2b(tr.tobytes()).hexdigest()
    lib = _lib.load()
    # the single-stream BLAKE2b rate of this box (the library's own implementation, csrc/blake2b.cpp)
    d64 = ctypes.create_string_buffer(64)
    lib.kzgpot_blake2b(tr.ctypes.data, ctypes.c_size_t(tr.size), d64)  # warm: pages touched, clocks up
    t0 = time.perf_counter()
    lib.kzgpot_blake2b(tr.ctypes.data, ctypes.c_size_t(tr.size), d64)
    b2_gbs = tr.size / (time.perf_counter() - t0) / 1e9
    out = np.ones(max(kzgpot.output_size(n_log2, m) for m in (kzgpot.MODE_KZG, kzgpot.MODE_FASTKZG)), np.uint8)
    devices = min(n_gpus, torch.cuda.device_count())  # shards map round-robin onto the visible devices
    rows = {"blake2b_single_stream": {"GBs": b2_gbs, "bytes": int(tr.size),
                                      "what": "kzgpot_blake2b over the transcript on one host thread (the floor "
                                              "of every digest row: BLAKE2b is one sequential stream per digest)"}}
    tmpdir = tempfile.mkdtemp(prefix="kzgpot_e2e_")
    src = os.path.join(tmpdir, "powersoftau")
    tr.tofile(src)
    # the file's pure read time (page cache, as the driver's box leaves it after writing it)
    t0 = time.perf_counter()
    with open(src, "rb", buffering=0) as f:
        buf = bytearray(tr.size)
        f.readinto(buf)
    read_s = time.perf_counter() - t0
    del buf
    pts = (2 * n - 1) + 3 * n + 1
    g1n = (2 * n - 1) * 96

    def floor(nbytes, secs):
        f = nbytes / (b2_gbs * 1e9)
        return {"blake2b_floor_s": f, "blake2b_floor_bytes": int(nbytes), "frac_of_blake2b_floor": f / secs}

    for mode, name in ((kzgpot.MODE_KZG, "preprocess_kgz_e2e"), (kzgpot.MODE_FASTKZG, "preprocess_fastkgz_e2e")):
        size = kzgpot.output_size(n_log2, mode)
        sec, idx = ctypes.c_int(-1), ctypes.c_int64(-1)
        shards = {"n_gpus": n_gpus, "shards": n_gpus, "distinct_devices": devices}
        # the GPU + PCIe part alone: the same call without the two BLAKE2b digests
        t0 = time.perf_counter()
        r0 = lib.kzgpot_preprocess_buffer_ex(tr.ctypes.data, tr.size, out.ctypes.data, mode, n_log2, n_gpus, None,
                                             None, None, ctypes.byref(sec), ctypes.byref(idx))
        dt0 = time.perf_counter() - t0
        ok0 = r0 == 0 and np.array_equal(out[:g1n], expect["tau_g1"]) and \
            np.array_equal(out[g1n:g1n + n * 96], expect["alpha_g1"])
        rows[name.replace("_e2e", "_buffer_no_digest")] = {
            "workload": f"N = 2^{n_log2} response transcript -> {size} B output, host buffers, {n_gpus} shard(s) "
                        "over the visible GPUs, NO digests: decode + check + PCIe only (C ABI call timed)",
            "seconds": dt0, "points": pts, "points_per_s": pts / dt0, **shards,
            "sections_verified": bool(ok0)}
        out[:] = 1
        din, dout = ctypes.create_string_buffer(129), ctypes.create_string_buffer(129)
        t0 = time.perf_counter()
        r = lib.kzgpot_preprocess_buffer_ex(tr.ctypes.data, tr.size, out.ctypes.data, mode, n_log2, n_gpus, None, din,
                                            dout, ctypes.byref(sec), ctypes.byref(idx))
        dt = time.perf_counter() - t0
        ok = r == 0 and np.array_equal(out[:g1n], expect["tau_g1"]) and \
            np.array_equal(out[g1n:g1n + n * 96], expect["alpha_g1"])
        buf_digest = hashlib.blake2b(out[:size]).hexdigest()
        ok = ok and din.value.decode() == tr_digest and dout.value.decode() == buf_digest
        rows[name] = {"workload": f"N = 2^{n_log2} response transcript ({tr.size} B) -> {size} B file, "
                                  f"host buffers, {n_gpus} shard(s), BLAKE2b of input and output (C ABI call timed)",
                      "seconds": dt, "points": pts, "points_per_s": pts / dt, **shards,
                      **floor(max(tr.size, size), dt), "gpu_pass_s": dt0,
                      "sections_verified": bool(ok),
                      "transcript_blake2b": din.value.decode()[:16] + "...",
                      "output_blake2b": dout.value.decode()[:16] + "..."}
        # file to file (the reference's contract, preprocess-kgz.rs:69-126,187-194), as the reference
        # hashes: the transcript checked against its expected digest, the output not hashed
        dst = os.path.join(tmpdir, "out")
        t0 = time.perf_counter()
        r = lib.kzgpot_preprocess_ex(src.encode(), dst.encode(), mode, n_log2, n_gpus, tr_digest.encode(), None, None,
                                     ctypes.byref(sec), ctypes.byref(idx))
        dtt = time.perf_counter() - t0
        with open(dst, "rb") as f:
            file_digest = hashlib.blake2b(f.read()).hexdigest()
        os.unlink(dst)
        rows[name + "_file_transcript_digest"] = {
            "workload": f"file to file, the reference's digest work only: kzgpot_preprocess_ex({tr.size} B transcript "
                        "-> output file, expect_transcript_digest = its BLAKE2b; no output digest), transcript "
                        "pread() behind the GPU, output pwrite() behind it",
            "seconds": dtt, "points": pts, "points_per_s": pts / dtt, **shards, **floor(tr.size, dtt),
            "gpu_pass_s": dt0, "transcript_read_s": read_s,
            "file_verified": bool(r == 0 and file_digest == buf_digest)}
        # file to file with both digests
        t0 = time.perf_counter()
        r = lib.kzgpot_preprocess_ex(src.encode(), dst.encode(), mode, n_log2, n_gpus, None, din, dout,
                                     ctypes.byref(sec), ctypes.byref(idx))
        dtf = time.perf_counter() - t0
        with open(dst, "rb") as f:
            file_digest = hashlib.blake2b(f.read()).hexdigest()
        os.unlink(dst)
        rows[name + "_file"] = {
            "workload": f"same, file to file: kzgpot_preprocess_ex({tr.size} B transcript on local disk -> output "
                        "file), transcript pread() behind the GPU, output pwrite() behind it, both digests",
            "seconds": dtf, "points_per_s": pts / dtf, **shards, "buffer_path_s": dt,
            **floor(max(tr.size, size), dtf), "gpu_pass_s": dt0,
            "transcript_read_s": read_s,
            "vs_buffer_plus_read": dtf / (dt + read_s),
            "file_verified": bool(r == 0 and file_digest == buf_digest == dout.value.decode())}
    os.unlink(src)
    os.rmdir(tmpdir)
    return rows


def cli_preprocess(n_log2):
    """The drop-in binaries as a user runs them (build/kzgpot-preprocess-{kgz,fastkgz},
    csrc/preprocess_main.cpp, in place of `cargo run --release --bin preprocess-kgz`): process start
    to exit, wall clock, on an N = 2^n_log2 response transcript on local disk, doing the reference's
    digest work (the transcript's BLAKE2b-512 checked against --expect-digest; the output not
    hashed). Runs BEFORE this process touches the GPU, so the child is never started from a process
    holding a HIP context. The transcript tiles the config-1 transcript's valid points (host-built:
    tools/e2e_breakdown.py); the output files' BLAKE2b is returned for the check against the
    library's buffer call on the same transcript once the GPU is up (verify_cli)."""
    import hashlib
    import shutil
    import subprocess

    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from e2e_breakdown import tiled_transcript

    tr = tiled_transcript(n_log2)
    digest = hashlib.blake2b(tr).hexdigest()
    tmpdir = tempfile.mkdtemp(prefix="kzgpot_cli_")
    src = os.path.join(tmpdir, "powersoftau")
    with open(src, "wb") as f:
        f.write(tr)
    rows = {"_transcript": tr}
    try:
        for mode in ("kgz", "fastkgz"):
            exe = os.path.join(ROOT, "kzg-setup-powersoftau_amd", "build", f"kzgpot-preprocess-{mode}")
            dst = os.path.join(tmpdir, "kzg_setup")
            if not os.path.exists(exe):
                rows[f"cli_preprocess_{mode}"] = {"skipped": f"{exe} not built", "_out_digest": None}
                continue
            runs = []  # two runs: the first also pays the box's cold GPU / driver start, the second is steady
            for _ in range(2):
                t0 = time.perf_counter()
                try:
                    p = subprocess.run([exe, "--n-log2", str(n_log2), "--gpus", "1", "--expect-digest", digest,
                                        "--timing"], cwd=tmpdir, capture_output=True, text=True, timeout=300)
                except subprocess.TimeoutExpired:
                    p = None
                    break
                wall = time.perf_counter() - t0
                phases = None
                for ln in (p.stdout or "").splitlines():
                    if ln.startswith("timing: main "):  # "timing: main A s after process start, library call done B s after"
                        w = ln.split()
                        main_s, done_s = float(w[2]), float(w[10])
                        phases = {"process_start_to_main_s": main_s, "library_call_s": done_s - main_s,
                                  "after_call_to_exit_s": wall - done_s,
                                  "note": "start and main from /proc/self/stat (10 ms ticks); exit = wall - call done"}
                out_digest = None
                if p.returncode == 0:
                    with open(dst, "rb") as f:
                        out_digest = hashlib.blake2b(f.read()).hexdigest()
                    os.unlink(dst)
                runs.append((wall, phases, p, out_digest))
            if p is None or not runs:
                rows[f"cli_preprocess_{mode}"] = {"skipped": "timed out after 300 s", "_out_digest": None}
                continue
            wall, phases, p, out_digest = runs[-1]
            if any(r[2].returncode != 0 or r[3] != out_digest for r in runs):
                out_digest = None  # every run must succeed with the same file
            n = 1 << n_log2
            pts = (2 * n - 1) + 3 * n + 1
            rows[f"cli_preprocess_{mode}"] = {
                "workload": f"build/kzgpot-preprocess-{mode} --n-log2 {n_log2} --gpus 1 --expect-digest <transcript "
                            f"BLAKE2b> on a {len(tr)} B transcript file: process start to exit (HIP initialisation, "
                            "transcript digest check, decode + check on the GPU, output file), as the reference's "
                            "binary is run",
                "wall_s": wall, "wall_s_each_run": [r[0] for r in runs], "points": pts, "points_per_s": pts / wall,
                "rc": p.returncode, "phases": phases,
                "stdout_tail": p.stdout.strip().splitlines()[-1:] if p.stdout else None,
                "_out_digest": out_digest}
    finally:
        shutil.rmtree(tmpdir, ignore_errors=True)
    return rows


def verify_cli(rows, n_log2, kzgpot):
    """The CLI's files against kzgpot_preprocess_buffer_ex on the same transcript (both modes)."""
    import hashlib

    import numpy as np
    from kzgpot import _lib

    tr = np.frombuffer(rows.pop("_transcript"), np.uint8)
    lib = _lib.load()
    for mode, m in (("kgz", kzgpot.MODE_KZG), ("fastkgz", kzgpot.MODE_FASTKZG)):
        row = rows[f"cli_preprocess_{mode}"]
        out = np.empty(kzgpot.output_size(n_log2, m), np.uint8)
        sec, idx = ctypes.c_int(-1), ctypes.c_int64(-1)
        r = lib.kzgpot_preprocess_buffer_ex(tr.ctypes.data, tr.size, out.ctypes.data, m, n_log2, 1, None, None, None,
                                            ctypes.byref(sec), ctypes.byref(idx))
        want = row.pop("_out_digest")
        row["file_equal_to_library_buffer_call"] = bool(r == 0 and want is not None and
                                                        want == hashlib.blake2b(out).hexdigest())
    return rows


def spawn_ranks(args) -> int:
    """`bench.py --gpus N` (N > 1) with no launcher around it: run `torch.distributed.run
    --nproc-per-node N ... bench.py <same args>` as a child process (never exec: this process has
    not touched the GPU, and must not), pass rank 0's JSON line through to stdout, everything else
    to stderr, and return the child's exit code."""
    import socket
    import subprocess

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:  # a free rendezvous port
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    import signal

    cmd = spawn_argv(args.gpus, port, sys.argv[1:])
    env = dict(os.environ, KZGPOT_BENCH_LAUNCHER="bench.py -> torch.distributed.run (child process)")
    print(f"bench.py: --gpus {args.gpus}: starting {' '.join(cmd)}", file=sys.stderr, flush=True)

    def die_with_parent():  # the launcher (and through it every rank) gets SIGTERM if this process dies
        try:
            ctypes.CDLL("libc.so.6", use_errno=True).prctl(1, signal.SIGTERM)  # PR_SET_PDEATHSIG
        except OSError:
            pass

    p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, text=True, preexec_fn=die_with_parent)

    def forward(sig, _frame):  # a timeout's SIGTERM / a ^C reaches the launcher, which stops its ranks
        p.send_signal(sig)

    for sig in (signal.SIGTERM, signal.SIGINT):
        signal.signal(sig, forward)
    for line in p.stdout:
        if line.startswith("{") and '"metric"' in line:
            sys.stdout.write(line)
            sys.stdout.flush()
        else:
            sys.stderr.write(line)
    return p.wait()


def spawn_argv(n, port, argv):
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def check_launch(gpus, environ):
    """None if this process may run the bench itself, 'spawn' if it must start the ranks, or an
    error message (a launcher whose WORLD_SIZE disagrees with --gpus)."""
    if "WORLD_SIZE" in environ:
        world = int(environ["WORLD_SIZE"])
        if world != gpus:
            return f"--gpus {gpus} but the launcher started WORLD_SIZE {world} ranks"
        return None
    return "spawn" if gpus > 1 else None


def rank_info(dev, comm):
    """This rank's device as torch and (when the library communicator exists) as RCCL sees it."""
    import socket

    import torch

    props = torch.cuda.get_device_properties(dev)
    info = {"rank": int(os.environ.get("RANK", "0")), "local_rank": int(os.environ.get("LOCAL_RANK", "0")),
            "host": socket.gethostname(), "device": dev.index, "name": props.name,
            "uuid": str(getattr(props, "uuid", "")) or None,
            "pci_bus_id": getattr(props, "pci_bus_id", None), "gcn_arch": getattr(props, "gcnArchName", None)}
    if comm is not None:
        info["rccl"] = comm.size()
    return info


def main():
    args = parse()
    launch = check_launch(args.gpus, os.environ)
    if launch == "spawn":
        sys.exit(spawn_ranks(args))
    if launch is not None:
        print(f"bench.py: {launch}", file=sys.stderr)
        sys.exit(2)
    # The one JSON line goes to the real stdout; anything native libraries print there (RCCL's
    # version banner at communicator init) is sent to stderr instead.
    sys.stdout.flush()
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # the drop-in binaries, timed as child processes before this process touches the GPU
    cli_rows = None
    if world == 1 and not args.no_next_rows and args.e2e_log2 > 0 and args.cli:
        cli_rows = cli_preprocess(args.e2e_log2)

    import torch
    import torch.distributed as dist

    # one process per GPU; ranks beyond the visible GPUs wrap around (a gloo rehearsal of the N > 1
    # path on a one-GPU box: --dist-backend gloo)
    dev = torch.device("cuda", local_rank % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)

    import kzgpot
    from kzgpot import device as D
    from kzgpot import dist as KD

    n1, n2 = 1 << args.g1_log2, 1 << args.g2_log2
    gather = (world > 1 or args.gather_at_1) and not args.no_gather
    verify = not args.no_verify
    t_gen = time.perf_counter()
    comm, gather_impl = None, None
    if gather:
        gather_impl = "torch.distributed"
        if args.gather_impl == "lib" and args.dist_backend == "nccl":
            try:
                comm = KD.LibComm(rank, world)
                gather_impl = "libkzgpot (kzgpot_decode_allgather_dev: RCCL inside the library)"
            except (OSError, RuntimeError) as e:  # reported in the line; the torch path is the same layout
                print(f"warning: library communicator unavailable ({e}); torch.distributed gathers", file=sys.stderr)
                gather_impl = f"torch.distributed (library communicator failed: {e})"
    ranks = [rank_info(dev, comm)]
    if world > 1:
        allr = [None] * world
        dist.all_gather_object(allr, ranks[0])
        ranks = allr
    g1_flags = 0x4 if args.split_phases else 0  # KZGPOT_SPLIT_PHASES (applies to G1 and G2)
    g1_kernels = ["k_g1_decompress", "k_g1_check"] if args.split_phases else ["k_g1_codec"]
    g1 = Sharded("g1", n1, args.seed, args.gather_chunks, rank, world, gather, dev, verify, comm, g1_flags)
    g2 = Sharded("g2", n2, args.seed + 1, 1, rank, world, gather, dev, verify, comm, g1_flags)  # 2^16 points: one chunk
    torch.cuda.synchronize()
    t_gen = time.perf_counter() - t_gen

    elapsed, ev, verified = timed([g1, g2], args.steps, args.warmup, world, dev, verify)
    clock = LAST_CLOCK.get("mhz")
    bad = KD.allreduce_min_key(min(g1.bad_key(), g2.bad_key()), dev) if world > 1 else min(g1.bad_key(), g2.bad_key())
    sample = None
    if verify and rank == 0 and (gather or world == 1):
        sample = oracle_sample_check(g1, args.oracle_sample_runs)
    g1_ms, g2_ms = kernel_ms(ev, "g1"), kernel_ms(ev, "g2")

    next_rows = {} if not args.no_next_rows else None
    # BN254 G1, ark compressed (32 B) -> uncompressed (64 B),
    # sharded and gathered across the ranks like config 4 (every rank takes part)
    if next_rows is not None and args.bn254_log2 > 0:
        del g1.comp
        nb = 1 << args.bn254_log2
        t_bn = time.perf_counter()
        bn = Sharded("bn254", nb, args.seed + 2, args.gather_chunks, rank, world, gather, dev, verify, comm)
        torch.cuda.synchronize()
        t_bn = time.perf_counter() - t_bn
        bn_s, bn_ev, bn_ok = timed([bn], args.steps, 1, world, dev, verify)
        bn_bad = KD.allreduce_min_key(bn.bad_key(), dev) if world > 1 else bn.bad_key()
        bn_ms = kernel_ms(bn_ev, "bn254")
        next_rows["bn254_g1_decompress"] = {
            "workload": f"config 5: 2^{args.bn254_log2} BN254 G1, ark compressed 32 B -> ark uncompressed 64 B"
                        + (f", block-cyclic shards over {world} GPUs, {gather_label(gather_impl, args)} to one "
                           f"contiguous buffer pipelined in {args.gather_chunks} chunks" if gather else ""),
            "kernel": "k_bn254_g1_decompress", "points": nb, "n_gpus": world, "steps": args.steps,
            "ms_per_step": bn_s * 1e3 / args.steps, "points_per_s": nb * args.steps / bn_s,
            "launch_ms_per_rank": bn_ms, "algorithmic_bytes_per_point": ALG_BYTES["bn254"],
            "achieved_GBs": ALG_BYTES["bn254"] * bn.m / (bn_ms * 1e-3) / 1e9, "peak_GBs": HBM_PEAK_GBS,
            "hbm_frac": ALG_BYTES["bn254"] * bn.m / (bn_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "valu": valu_roofline(load_json("pmc_traffic.json"), load_json("r02_valu_mix.json"),
                                  ["k_bn254_g1_decompress"], bn.m, bn_ms),
            "verified_bit_exact": bn_ok, "rejected_points": 0 if bn_bad == KD.NO_BAD else 1, "generate_s": t_bn}
        del bn
        torch.cuda.empty_cache()

    # SURVEY §8f rows, measured after the timed region on rank 0 only
    if next_rows is not None and rank == 0:
        m1 = g1.m
        rec1 = g1.out[:m1 * 96]  # m1 G1 ark records (any of them: all decoded and verified)
        # row 2 (loader mirror): the G1 ark records just produced -> in-memory GroupAffine
        # (deserialize_unchecked), HBM-bound
        outl = torch.empty(m1 * 104, dtype=torch.uint8, device=dev)
        keyl = torch.empty(1, dtype=torch.int64, device=dev)
        next_rows["g1_deserialize_unchecked"] = loader_row("g1", rec1, outl, keyl, m1, "load_kzg_setup")
        del outl
        # the same rows for G2 (load_fastkzg_setup's powers_of_h, src/lib.rs:209-215): every pair of
        # G1 ark records read as one G2 record (x.c0 x.c1 y.c0 y.c1 = x1 y1 x2 y2: canonical
        # coordinates, no flags), which deserialize_unchecked accepts (it checks no curve)
        m2 = m1 // 2
        outl = torch.empty(m2 * 200, dtype=torch.uint8, device=dev)
        next_rows["g2_deserialize_unchecked"] = loader_row("g2", rec1[:m2 * 192], outl, keyl, m2,
                                                           "load_fastkzg_setup")
        del outl
        # row 3 (uncompressed-input mode, the read_g1 loop alone): pairing-uncompressed records =
        # per-coordinate byte reversal of the ark records (A6 identity); decode them back
        nt = min(m1, 1 << 24)
        ark = rec1[:nt * 96]
        pin = ark.view(nt, 2, 48).flip(-1).contiguous().view(-1)
        outt = torch.empty(nt * 96, dtype=torch.uint8, device=dev)
        keyt = torch.empty(1, dtype=torch.int64, device=dev)
        D.codec_dev("g1_transcode", pin, outt, keyt)
        next_rows["g1_transcode_uncompressed"] = transcode_row("g1", pin, outt, keyt, ark, nt)
        del pin, outt
        # 2^20 G1 + 2^20 G2 (the Fp2 square-root path) on one GPU, bit-exact
        n3 = 1 << 20
        c31, x31 = D.synth("g1", args.seed + 4, 0, n3, dev, with_expected=True)
        c32, x32 = D.synth("g2", args.seed + 5, 0, n3, dev, with_expected=True)
        o31 = torch.empty(n3 * 96, dtype=torch.uint8, device=dev)
        o32 = torch.empty(n3 * 192, dtype=torch.uint8, device=dev)
        k3 = torch.empty(2, dtype=torch.int64, device=dev)
        D.codec_dev("g1_decompress", c31, o31, k3[0:1], g1_flags)
        D.codec_dev("g2_decompress", c32, o32, k3[1:2], g1_flags)
        # three pairs of launches (~17 + ~27 ms each), each launch event-timed, G1 and G2 alternating
        # so that both run under the same clock, which the shader-clock probe measures over the
        # whole interleaved region; the G2 : G1 time ratio against their VALU models' ratio is a
        # clock-free measure of how far G2 sits below G1's efficiency
        reps3 = 3
        ce = [torch.cuda.Event(enable_timing=True) for _ in range(2 * reps3 + 1)]
        p0 = D.clock_probe(dev)
        ce[0].record()
        for r in range(reps3):
            D.codec_dev("g1_decompress", c31, o31, k3[0:1], g1_flags)
            ce[2 * r + 1].record()
            D.codec_dev("g2_decompress", c32, o32, k3[1:2], g1_flags)
            ce[2 * r + 2].record()
        p1 = D.clock_probe(dev)
        torch.cuda.synchronize()
        per = {"g1": [ce[2 * r].elapsed_time(ce[2 * r + 1]) for r in range(reps3)],
               "g2": [ce[2 * r + 1].elapsed_time(ce[2 * r + 2]) for r in range(reps3)]}
        c3_clock = D.clock_mhz(p0, p1)
        g1s, g2s = per["g1"], per["g2"]
        g1c, g2c = sum(g1s) / reps3, sum(g2s) / reps3
        g1v = valu_roofline(load_json("pmc_traffic.json"), load_json("r02_valu_mix.json"),
                            ["k_g1_decompress", "k_g1_check"] if args.split_phases else ["k_g1_codec"], n3, g1c, c3_clock)
        g2v = valu_roofline(load_json("pmc_traffic.json"), load_json("r02_valu_mix.json"),
                            ["k_g2_decompress", "k_g2_check"] if args.split_phases else ["k_g2_codec"], n3, g2c, c3_clock)
        next_rows["config3_g1_g2_2e20"] = {
            "workload": "config 3: 2^20 G1 + 2^20 G2 compressed -> ark uncompressed, subgroup-checked, 1 GPU",
            "g1_ms": g1c, "g2_ms": g2c, "reps": reps3, "g1_ms_each": g1s, "g2_ms_each": g2s,
            "points_per_s": 2 * n3 / ((g1c + g2c) * 1e-3),
            "g2_ns_per_point": g2c * 1e6 / n3,
            "clock_mhz": None if c3_clock is None else c3_clock["mean"],
            "headline_clock_mhz": None if clock is None else clock["mean"],
            "g1_valu": g1v, "g2_valu": g2v,
            "g2_efficiency_vs_g1": g2_vs_g1(g1v, g2v, g1c, g2c),
            "verified_bit_exact": bool(D.read_key(k3[0:1]) == KD.NO_BAD and D.read_key(k3[1:2]) == KD.NO_BAD
                                       and torch.equal(o31, x31) and torch.equal(o32, x32))}
        # row 3, G2 (the read_g2 loop, the reference's HOT LOOP 2 for τG2): config 3's 2^20 ark G2
        # records -> pairing-uncompressed (x.c1 x.c0 y.c1 y.c0, each BE) -> decoded back
        del c31, x31, c32, o31
        pin2 = o32.view(n3, 2, 2, 48).flip(2).flip(-1).contiguous().view(-1)
        outt2 = torch.empty(n3 * 192, dtype=torch.uint8, device=dev)
        keyt2 = torch.empty(1, dtype=torch.int64, device=dev)
        D.codec_dev("g2_transcode", pin2, outt2, keyt2)
        next_rows["g2_transcode_uncompressed"] = transcode_row("g2", pin2, outt2, keyt2, x32, n3)
        del pin2, outt2, x32, o32
        # the FFI boundary: host-buffer entry points with PCIe, beside the device-resident rate
        if args.host_api:
            if hasattr(g1, "comp"):
                del g1.comp
            torch.cuda.empty_cache()
            next_rows["host_api"] = host_api_rows(args.seed + 6, dev, D)
        # row 1: end-to-end preprocess (host transcript in -> host kgz / fastkzg file out, PCIe both
        # ways, BLAKE2b of both on host threads) at the reference's N = 2^21, buffers and files; at
        # N > 1 rank 0 drives every GPU of the node (kzgpot_preprocess_ex(n_gpus = world): one shard
        # per device, preprocess-kgz.rs:162-199 / preprocess-fastkgz.rs:180-214) while the other
        # ranks wait on the host
        if args.e2e_log2 > 0:
            next_rows.update(e2e_preprocess(args.e2e_log2, args.seed + 3, dev, kzgpot, D, n_gpus=world))
        if cli_rows is not None:
            next_rows.update(verify_cli(cli_rows, args.e2e_log2, kzgpot))

    ms_per_step = elapsed * 1e3 / args.steps
    value = (n1 + n2) * args.steps / elapsed

    result = None
    if rank == 0:
        achieved = ALG_BYTES["g1"] * g1.m / (g1_ms * 1e-3) / 1e9
        pmc = load_json("pmc_traffic.json")
        result = {
            "metric": "G1+G2 points decompressed+checked/sec, 2^27 BLS12-381 PoT",
            "value": value,
            "unit": "points/s",
            "n_gpus": world,
            "rccl_nranks": (ranks[0].get("rccl") or {}).get("nranks"),
            "distinct_devices": len({(r["host"], r["uuid"] or r["pci_bus_id"] or r["device"]) for r in ranks}),
            "launcher": os.environ.get("KZGPOT_BENCH_LAUNCHER",
                                       "torch.distributed.run (external)" if "WORLD_SIZE" in os.environ else "none"),
            "ranks": ranks,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u32 (381-bit Montgomery, 14 x 28-bit limbs)",
            "data": "synthetic (GPU-generated valid subgroup points [k_i]G, 128-bit k_i; resident in HBM)",
            "config": {
                "workload": f"config 4: 2^{args.g1_log2} G1 + 2^{args.g2_log2} G2 compressed BLS12-381 "
                            "points -> arkworks uncompressed, subgroup-checked"
                            + (f", block-cyclic shards, {gather_label(gather_impl, args)} to one contiguous buffer "
                               f"pipelined in {args.gather_chunks} chunks" if gather else ""),
                "g1_points": n1, "g2_points": n2, "parallelism": f"shard{world}",
                "gather_impl": gather_impl if not FALLBACKS else FALLBACKS[0],
                "subgroup_test": "endomorphism (phi/psi), bit-exact accept/reject vs ark mul_bits(r)",
            },
            "roofline": {
                "kernel": ("k_g1_decompress + k_g1_check<ArkInPlace> (G1 codec, split launches)" if args.split_phases
                           else "k_g1_codec (G1 decompress + subgroup check + ark emit, one pass)"),
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": pmc_traffic(pmc, g1.m),
                "launch_ms": g1_ms,
                "algorithmic_bytes_per_point": ALG_BYTES["g1"],
                "note": "integer-VALU bound, not HBM: see valu",
            },
            "valu": valu_roofline(pmc, load_json("r02_valu_mix.json"), g1_kernels, g1.m, g1_ms, clock),
            "field_ops": field_ops(load_json("fp_census.json"), "g1_decompress", g1.m, g1_ms),
            "clock_mhz": None if clock is None else {
                "mean": clock["mean"], "min": min(clock["per_xcd"].values()), "max": max(clock["per_xcd"].values()),
                "xcds": len(clock["per_xcd"]),
                "source": "s_memtime / s_memrealtime of each XCD at the start and end of the timed steps "
                          "(kzgpot_synth_clock_probe); explains box-to-box spread at the same code"},
            "kernels_ms": {"g1_codec": g1_ms, "g2_codec": g2_ms},
            "verified_bit_exact": verified,
            "oracle_sample_check": sample,
            "rejected_points": 0 if bad == KD.NO_BAD else 1,
            "generate_s": t_gen,
        }
        if next_rows:
            result["next_rows"] = next_rows
        if world == 1 and not args.no_cpu_baseline:
            result["cpu_baseline"] = cpu_baseline(g1.comp if hasattr(g1, "comp") else
                                                  D.synth("g1", args.seed, 0, 1 << args.cpu_sample_log2, dev,
                                                          with_expected=False)[0],
                                                  g2.comp, args.cpu_sample_log2)
            if result["cpu_baseline"] is not None and args.cpu_e2e_log2 > 0:
                result["cpu_baseline"]["e2e"] = cpu_e2e(args.cpu_e2e_log2, args.seed + 7, dev, D, kzgpot, next_rows)
        print(json.dumps(result), file=json_out, flush=True)
    if world > 1:
        # rank 0 ran the rows after the timed region (on every GPU for the e2e rows): the others
        # wait on the rendezvous store, on the host, so no RCCL barrier kernel sits on their GPUs
        get_store = getattr(dist.distributed_c10d, "_get_default_store", None)
        store = get_store() if get_store else None
        if store is not None and rank == 0:
            store.set("kzgpot_bench_rows_done", "1")
        elif store is not None:
            import datetime
            store.wait(["kzgpot_bench_rows_done"], datetime.timedelta(minutes=30))
        dist.barrier()  # (without a store, this barrier alone waits for rank 0's rows)
        if comm is not None:
            comm.close()
        dist.destroy_process_group()
    return result


if __name__ == "__main__":
    main()
