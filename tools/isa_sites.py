"""Per-site attribution of a codec kernel's scalar, branch, wait and nop instructions (VERDICT r05
next #2: "attribute k_g2_codec's extra SALU and branches per wave against G1 to code sites").

The kernels are wave-uniform on valid points: every wave runs the same instruction stream, whose
loops have trip counts fixed by the algorithm — the square root's schedule
(bls12_381_consts.hpp SQRT_STEP_SQ: 67 window steps, 375 squarings after the 8-entry table, whose
a^240 takes a 4-squaring loop) and the |u| ladder (62 doublings; G1 runs two ladders). So the
per-wave dynamic count of each instruction class is (static count in each loop body) x (its trip
count) + (straight-line code, run once). This tool disassembles the library, finds the loops
(back-edges, including the s_getpc / s_setpc far jumps), classifies them by their body (radix-2^30
squaring: 260 v_mad_i64_i32; window step: the table lookup + f30 multiply; ladder doubling:
>= 5,000 v_mad_u64_u32 in a loop with no LDS), and prints the per-site table as JSON, with the
PMC per-wave counts beside it when a stall profile (tools/codec_stall_summary.py output) is given.

    python3 tools/isa_sites.py [--lib kzg-setup-powersoftau_amd/build/libkzgpot.so]
                               [--pmc profiles/r05a_codec_stalls.json]

Classes: valu, salu (scalar ALU incl. s_set_gpr_idx), branch (incl. far jumps), nop (s_nop),
wait (s_waitcnt), smem (scalar loads), vmem (global / buffer), lds (ds_*)."""
from __future__ import annotations

import argparse
import collections
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
sys.path.insert(0, os.path.join(ROOT, "tools"))

KERNELS = {"k_g1_codec": "_ZN6kzgpot10k_g1_codec", "k_g2_codec": "_ZN6kzgpot10k_g2_codec"}


def cat(op):
    if op.startswith("v_"):
        return "valu"
    if op == "s_nop":
        return "nop"
    if op == "s_waitcnt":
        return "wait"
    if "branch" in op or op in ("s_setpc_b64", "s_swappc_b64"):
        return "branch"
    if op.startswith(("s_load", "s_buffer_load", "s_store", "s_dcache")):
        return "smem"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    return "vmem"


def disassemble(lib):
    tmp = tempfile.mkdtemp(prefix="isa_sites_")
    try:
        dst = os.path.join(tmp, "lib.so")
        shutil.copy(lib, dst)
        subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", dst], check=True, capture_output=True, cwd=tmp)
        text = ""
        for f in sorted(os.listdir(tmp)):
            if f.endswith("gfx950"):
                text += subprocess.run([f"{LLVM}/llvm-objdump", "-d", os.path.join(tmp, f)], check=True,
                                       capture_output=True, text=True).stdout
        return text
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def parse(text, prefix):
    """[(offset, opcode, operands, branch target offset or None)] of the kernel whose symbol starts
    with prefix; far jumps (s_getpc_b64; s_add_u32 lit; s_addc_u32; s_setpc_b64) resolved."""
    ins, cur, base = [], None, None
    for ln in text.splitlines():
        m = re.match(r"^([0-9a-f]+) <(\S+)>:", ln)
        if m:
            cur = m.group(2)
            base = None
            continue
        if not cur or not cur.startswith(prefix):
            continue
        m = re.match(r"^\s+(\S+)\s+(.*?)//\s*([0-9A-F]+):\s*([0-9A-F ]+?)\s*(<\S+\+0x([0-9a-f]+)>)?\s*$", ln.rstrip())
        if m:
            a = int(m.group(3), 16)
            base = a if base is None else base
            ins.append([a - base, m.group(1), m.group(2), int(m.group(6), 16) if m.group(6) else None])
    for i, (off, op, args, tgt) in enumerate(ins):
        if op == "s_setpc_b64" and i >= 3 and ins[i - 3][1] == "s_getpc_b64":
            lit = re.search(r"0x([0-9a-f]+)", ins[i - 2][2])
            if lit:
                d = int(lit.group(1), 16)
                d = d - (1 << 32) if d >= 1 << 31 else d
                ins[i][3] = ins[i - 2][0] + d  # s_getpc_b64 yields the address of the s_add_u32
    return ins


def counts(ins, lo, hi, exclude=()):
    c, mads = collections.Counter(), collections.Counter()
    for off, op, _, _ in ins:
        if lo <= off <= hi and not any(a <= off <= b for a, b in exclude):
            c[cat(op)] += 1
            if op.startswith("v_mad_"):
                mads[op] += 1
    return c, mads


def sqrt_schedule():
    text = open(os.path.join(ROOT, "kzg-setup-powersoftau_amd", "csrc", "bls12_381_consts.hpp")).read()
    sq = [int(v) for v in re.search(r"SQRT_STEP_SQ\[SQRT_STEPS\] = \{([^}]*)\}", text).group(1).split(",")]
    return len(sq) - 1, sum(sq[1:])  # window steps after the first, squarings in them


def attribute(ins, kernel):
    """Loops of the hot path with their trip counts, exclusive counts (nested loops removed)."""
    loops = sorted({(t, off) for off, op, _, t in ins if t is not None and t <= off and cat(op) == "branch"})
    steps, squarings = sqrt_schedule()
    # each exponentiation is inlined where it is called (G2: two copies), so a copy's loops run the
    # schedule once per wave; G1's two [|u|] ladders share ONE copy of the ladder code
    ladders = 2 if kernel == "k_g1_codec" else 1
    sites = []
    for lo, hi in loops:
        nested = [(a, b) for a, b in loops if lo <= a and b <= hi and (a, b) != (lo, hi)]
        c, m = counts(ins, lo, hi, nested)
        call, mall = counts(ins, lo, hi)
        sites.append({"lo": lo, "hi": hi, "bytes": hi - lo + 4, "nested": len(nested), "excl": c, "mads": mall})
    out = []
    # radix-2^30 squaring loops (260 i64 mads, nothing nested): the one inside the window loop runs
    # the schedule's squarings; one outside it, the table's a^240 (4 iterations)
    window = [s for s in sites if s["mads"].get("v_mad_i64_i32", 0) >= 500 and s["nested"] >= 1]
    for s in sites:
        i64, u64 = s["mads"].get("v_mad_i64_i32", 0), s["mads"].get("v_mad_u64_u32", 0)
        if s["nested"] == 0 and 200 <= i64 <= 300 and u64 == 0:
            inside = any(w["lo"] <= s["lo"] and s["hi"] <= w["hi"] for w in window)
            s["site"] = "sqrt: f30 squaring loop (window steps)" if inside else "sqrt: f30 squaring loop (table a^240)"
            s["trips_per_wave"] = squarings if inside else 4
        elif s in window:
            s["site"] = "sqrt: window step (table lookup, schedule read, f30 multiply)"
            s["trips_per_wave"] = steps
        elif s["nested"] == 0 and u64 >= 2000 and s["excl"].get("lds", 0) == 0 and s["excl"].get("smem", 0) == 0:
            s["site"] = "ladder: doubling loop (jac_dbl_w, bit test, back-edge)"
            s["trips_per_wave"] = ladders * 62
        else:
            continue
        out.append(s)
    # de-duplicate loop records that share a body (several back-edges into one header): keep the
    # innermost per site and header
    seen, res = set(), []
    for s in out:
        key = (s["site"], s["lo"])
        if key in seen:
            continue
        seen.add(key)
        res.append(s)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=os.path.join(ROOT, "kzg-setup-powersoftau_amd", "build", "libkzgpot.so"))
    ap.add_argument("--pmc", default=None, help="tools/codec_stall_summary.py output (per-wave PMC counts)")
    a = ap.parse_args()
    text = disassemble(a.lib)
    pmc = json.load(open(a.pmc))["kernels"] if a.pmc else {}
    classes = ("valu", "salu", "branch", "nop", "wait", "smem", "vmem", "lds")
    res = {"lib": os.path.relpath(a.lib, ROOT), "method": __doc__.split("\n\n")[1].replace("\n", " "), "kernels": {}}
    for name, prefix in KERNELS.items():
        ins = parse(text, prefix)
        total = collections.Counter(cat(op) for _, op, _, _ in ins)
        sites = attribute(ins, name)
        rows, dyn = [], collections.Counter()
        # (the reference-mode ladder, KZGPOT_SUBGROUP_REF, reads FR_R with a scalar load: excluded)
        loop_ranges = [(s["lo"], s["hi"]) for s in sites]
        for s in sites:
            d = {k: s["excl"].get(k, 0) * s["trips_per_wave"] for k in classes}
            dyn.update(d)
            rows.append({"site": s["site"], "offset": f"0x{s['lo']:x}-0x{s['hi']:x}", "bytes": s["bytes"],
                         "trips_per_wave": s["trips_per_wave"],
                         "static_per_trip": {k: s["excl"].get(k, 0) for k in classes if s["excl"].get(k, 0)},
                         "per_wave": {k: v for k, v in d.items() if v}})
        # code outside the hot loops: the straight-line prologue / emit / ladder additions and the cold
        # paths. Its hot part runs once per wave (the 4 mixed additions 4 times): an upper bound on
        # its per-wave share is its static count (cold branches included)
        outside = collections.Counter()
        for off, op, _, _ in ins:
            if not any(lo <= off <= hi for lo, hi in loop_ranges):
                outside[cat(op)] += 1
        k = {"static_total": {c: total.get(c, 0) for c in classes}, "code_bytes": ins[-1][0] + 4 if ins else 0,
             "loop_sites": rows, "loops_per_wave": {c: dyn.get(c, 0) for c in classes},
             "outside_loops_static": {c: outside.get(c, 0) for c in classes}}
        if name in pmc:
            pw = pmc[name]["per_wave"]
            k["pmc_per_wave"] = {"valu": pw.get("valu"), "salu": pw.get("salu"), "branch": pw.get("branch"),
                                 "lds": pw.get("lds"), "smem": pw.get("smem"), "source": a.pmc}
        res["kernels"][name] = k
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
