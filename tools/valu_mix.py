"""Cycle-weighted integer-VALU roof of the codec kernels.

    python tools/valu_mix.py [--lib kzg-setup-powersoftau_amd/build/libkzgpot.so]
                             [--costs profiles/r02_valu_issue_microbench.txt]
                             [--out profiles/r02_valu_mix.json]

For every kernel in the library's gfx950 code objects:
  * the opcode histogram of its machine code (llvm-objdump), VALU opcodes only;
  * each opcode's issue cost in SIMD cycles per wave64 instruction, measured by
    tools/microbench/valu_issue.hip (the "chains=1" row at 4 waves per SIMD, chip-wide: enough
    waves that latency is hidden and the SIMD's issue rate is the limit); opcodes the
    microbenchmark does not cover take the cost of their encoding class (VOP2 2-operand 32-bit
    ALU = v_add_u32's, everything else = v_mul_lo_u32's);
  * the mix-weighted average cost = the SIMD cycles one VALU instruction of this kernel needs
    at saturation, and the register / LDS / scratch budget from the code object metadata.

bench.py turns the PMC instruction count (profiles/pmc_traffic.json) into a roof:
peak wave-instructions/s = 1024 SIMDs x 2.4 GHz / average cost.

The histogram is static (each instruction of the code counted once). The kernels are ~95 %
Montgomery multiplies/squarings whose loop bodies have the same mix as the unrolled copies, so
the static mix stands in for the dynamic one; `fp_mul` / `fp_sqr` are also reported alone
(tools/microbench/mont28.hip is not needed: the k_g1_check body is almost only those).
"""
from __future__ import annotations

import argparse
import collections
import json
import os
import re
import shutil
import subprocess
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# encoding classes for opcodes the microbenchmark does not time
VOP2_FAST = re.compile(r"^v_(add|sub|subrev|and|or|xor|lshrrev|ashrrev|max|min|mov|not|cndmask)_(u32|i32|b32)$")


def parse_costs(path):
    """opcode -> SIMD cycles per wave64 instruction (chains=1, W=4, chip-wide value)."""
    costs, op = {}, None
    for line in open(path):
        m = re.match(r"^(v_\w+)\s+W=1", line)
        if m:
            op = m.group(1)
            continue
        if op and re.match(r"^\s+chains=1\s", line):
            cells = re.findall(r"(\d+\.\d+)/\s*(\d+\.\d+)", line)
            costs[op] = float(cells[3][0])  # W=4, chip
            op = None
    return costs


def cost_of(op, costs):
    base = re.sub(r"_e(32|64)$", "", op)
    if base in costs:
        return costs[base], True
    if VOP2_FAST.match(base):
        return costs["v_add_u32"], False
    return costs["v_mul_lo_u32"], False


def extract(lib, tmp):
    dst = os.path.join(tmp, os.path.basename(lib))
    shutil.copy(lib, dst)
    subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", dst], check=True, capture_output=True)
    return sorted(os.path.join(tmp, f) for f in os.listdir(tmp) if f.endswith("gfx950"))


def kernels_of(co):
    """symbol -> list of opcodes, from the disassembly of one code object."""
    dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", co], check=True, capture_output=True, text=True).stdout
    out, cur = {}, None
    for line in dis.splitlines():
        m = re.match(r"^[0-9a-f]+ <(\S+)>:", line)
        if m:
            cur = m.group(1)
            out[cur] = []
            continue
        m = re.match(r"^\s+([sv]_\w+|ds_\w+|global_\w+|buffer_\w+|flat_\w+|scratch_\w+)", line)
        if m and cur:
            out[cur].append(m.group(1))
    return out


def metadata(co):
    """symbol -> register / memory budget from the AMDHSA metadata note (one YAML map per kernel)."""
    notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True, text=True).stdout
    keys = {".vgpr_count": "vgpr", ".agpr_count": "agpr", ".sgpr_count": "sgpr", ".group_segment_fixed_size": "lds_bytes",
            ".private_segment_fixed_size": "scratch_bytes", ".sgpr_spill_count": "sgpr_spill",
            ".vgpr_spill_count": "vgpr_spill"}
    res, cur, sym = {}, {}, None

    def flush():
        if sym:
            res[sym] = dict(cur)

    for line in notes.splitlines():
        if re.match(r"^\s*- \.", line) and (line.strip().startswith("- .agpr_count") or line.strip().startswith("- .args")):
            flush()
            cur, sym = {}, None
        t = line.strip().lstrip("- ").strip()
        for k, v in keys.items():
            if t.startswith(k + ":"):
                cur[v] = int(t.split(":")[1])
        if t.startswith(".symbol:"):
            sym = t.split(":", 1)[1].strip().removesuffix(".kd")
    flush()
    return res


def demangle(names):
    out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.splitlines()
    return dict(zip(names, out))


def waves_per_simd(md, block=256):
    vg = md.get("vgpr", 0) + md.get("agpr", 0)
    by_vgpr = 512 // max(8, -(-vg // 8) * 8) if vg else 8
    blocks_by_lds = (160 * 1024) // md["lds_bytes"] if md.get("lds_bytes") else 99
    return min(8, by_vgpr, blocks_by_lds * block // 256)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=os.path.join(ROOT, "kzg-setup-powersoftau_amd", "build", "libkzgpot.so"))
    ap.add_argument("--costs", default=os.path.join(ROOT, "profiles", "r02_valu_issue_microbench.txt"))
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r02_valu_mix.json"))
    a = ap.parse_args()
    costs = parse_costs(a.costs)
    res = {"source": "tools/valu_mix.py: static opcode histogram of each kernel's gfx950 code x per-opcode issue "
                     "cost (SIMD cycles per wave64 instruction, chains=1 / 4 waves per SIMD, chip-wide) from "
                     + os.path.relpath(a.costs, ROOT),
           "costs": costs, "kernels": {}}
    with tempfile.TemporaryDirectory() as tmp:
        for co in extract(a.lib, tmp):
            ks, md = kernels_of(co), metadata(co)
            names = demangle(list(ks))
            for sym, ops in ks.items():
                if sym not in md:
                    continue  # not a kernel entry
                valu = [o for o in ops if o.startswith("v_")]
                hist = collections.Counter(valu)
                cyc = sum(cost_of(o, costs)[0] * c for o, c in hist.items())
                uncovered = sum(c for o, c in hist.items() if not cost_of(o, costs)[1])
                name = names[sym]
                res["kernels"][name] = {
                    "valu_static": len(valu), "avg_cycles_per_valu": cyc / max(1, len(valu)),
                    "mad_u64_u32_frac": hist["v_mad_u64_u32"] / max(1, len(valu)),
                    "uncovered_opcode_frac": uncovered / max(1, len(valu)),
                    "top": dict(hist.most_common(12)), **md[sym], "waves_per_simd": waves_per_simd(md[sym])}
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    for k, e in res["kernels"].items():
        print(f"{k[:70]:70s} valu {e['valu_static']:6d}  {e['avg_cycles_per_valu']:.3f} cyc/instr  "
              f"mad {e['mad_u64_u32_frac']:.2f}  vgpr {e.get('vgpr')} lds {e.get('lds_bytes')} -> {e['waves_per_simd']} w/SIMD")


if __name__ == "__main__":
    main()
