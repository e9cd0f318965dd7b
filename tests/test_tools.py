"""CPU checks of the measurement tools whose output is committed under profiles/: the e2e stage
summary (tools/stage_summary.py) on a synthetic three-trace run, the fetch-probe summary's
request-size arithmetic (tools/fetch_probe_summary.py) and the codec stall split
(tools/codec_stall_summary.py). No GPU."""
import csv
import json
import os
import subprocess
import sys

from conftest import ROOT

TOOLS = os.path.join(ROOT, "tools")


def write_csv(path, header, rows):
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(header)
        w.writerows(rows)


def test_stage_summary_critical_path_adds_up(tmp_path):
    ms = 1_000_000
    mk = [("kzgpot.preprocess", 1, 0, 5 * ms),  # the warm-up call (skipped)
          ("kzgpot.preprocess_file", 1, 9 * ms, 130 * ms),
          ("kzgpot.preprocess", 1, 10 * ms, 110 * ms),
          ("kzgpot.section.tau_g1", 2, 11 * ms, 40 * ms),
          ("kzgpot.section.tau_g2", 2, 41 * ms, 60 * ms),
          ("kzgpot.h2d", 2, 11 * ms, 12 * ms),
          ("kzgpot.blake2b.output", 3, 20 * ms, 109 * ms),
          ("kzgpot.file_finish", 1, 111 * ms, 112 * ms)]
    write_csv(tmp_path / "run_marker_api_trace.csv",
              ["Domain", "Function", "Process_Id", "Thread_Id", "Correlation_Id", "Start_Timestamp", "End_Timestamp"],
              [["MARKER_CORE_RANGE_API", n, 1, t, i, a, b] for i, (n, t, a, b) in enumerate(mk)])
    write_csv(tmp_path / "run_kernel_trace.csv", ["Kernel_Name", "Start_Timestamp", "End_Timestamp"],
              [["kzgpot::k_g1_codec(x)", 12 * ms, 30 * ms], ["kzgpot::k_g2_codec(x)", 42 * ms, 58 * ms]])
    write_csv(tmp_path / "run_memory_copy_trace.csv", ["Direction", "Start_Timestamp", "End_Timestamp"],
              [["MEMORY_COPY_HOST_TO_DEVICE", 11 * ms, 12 * ms], ["MEMORY_COPY_DEVICE_TO_HOST", 30 * ms, 32 * ms]])
    calls = tmp_path / "calls.json"
    calls.write_text(json.dumps({"n_log2": 21, "shards": 1, "blake2b_transcript_alone_s": 0.35,
                                 "calls": [{"call": "kgz_file_digests", "seconds": 0.121, "rc": 0}]}))
    p = subprocess.run([sys.executable, os.path.join(TOOLS, "stage_summary.py"), str(tmp_path), str(calls)],
                       capture_output=True, text=True, check=True)
    (c,) = json.loads(p.stdout)["calls"]
    assert c["range_ms"] == 100.0 and c["critical_path_sum_ms"] == 100.0
    assert [n for n, _ in c["critical_path_ms"]] == ["setup", "section.tau_g1", "between sections", "section.tau_g2",
                                                   "after the last section (digest / writer drain)"]
    assert c["critical_path_ms"][-1][1] == 50.0
    assert c["last_to_finish"] == "kzgpot.blake2b.output"
    assert c["busy_ms"]["gpu.kernels"] == 34.0 and c["busy_ms"]["gpu.copy.d2h"] == 2.0
    assert c["file"]["file_call_ms"] == 121.0 and c["file"]["after_pipeline_ms"] == 20.0


def test_fetch_probe_summary_splits_request_sizes(tmp_path):
    """128-B data requests vs 64-B instruction-fetch requests: bytes_by_size counts each at its size,
    while FETCH_SIZE (every request at 64 B) x 2 over-counts the 64-B ones."""
    n = 1 << 20
    name = "kzgpot::k_g2_codec(x)"
    d = tmp_path / "lib1"
    for sub, counters in (("FETCH_SIZE", {"FETCH_SIZE": (786440 + 72077) * 64 / 1024}),
                          ("WRITE_SIZE", {"WRITE_SIZE": 192 * n / 1024}),
                          ("SQC_ICACHE_MISSES", {"SQC_ICACHE_MISSES": 1.5 * n, "SQ_INSTS_VALU": 952781 * n / 64,
                                                 "SQ_WAVES": n / 64}),
                          ("TCC_EA0_RDREQ_sum", {"TCC_EA0_RDREQ_sum": 786440 + 72077, "TCC_EA0_RDREQ_32B_sum": 0,
                                                 "TCC_EA0_RDREQ_128B_sum": 786440, "TCC_EA0_RDREQ_DRAM_sum": 858517,
                                                 "SQC_TC_INST_REQ": 8.5e7, "SQC_TC_DATA_READ_REQ": 864})):
        os.makedirs(d / sub)
        write_csv(d / sub / "run_counter_collection.csv", ["Dispatch_Id", "Grid_Size", "Kernel_Name", "Counter_Name",
                                                            "Counter_Value"],
                  [[7, n, name, k, v] for k, v in counters.items()])
    (tmp_path / "lib1.name").write_text("build/libkzgpot.so\n")
    p = subprocess.run([sys.executable, os.path.join(TOOLS, "fetch_probe_summary.py"), str(tmp_path)],
                       capture_output=True, text=True, check=True)
    row = json.loads(p.stdout)["builds"]["build/libkzgpot.so"][f"k_g2_codec @ {n}"]
    assert abs(row["rdreq"]["bytes_by_size_per_point"] - (786440 * 128 + 72077 * 64) / n) < 1e-3
    assert row["rdreq"]["64B"] == 72077 and row["write_B_per_point"] == 192.0
    assert row["fetch_B_per_point"] > row["rdreq"]["bytes_by_size_per_point"]  # the x2 correction's over-count


def test_fp_census_matches_the_documented_schedule():
    """profiles/fp_census.json (tools/fpops/census.py on the GPU) against the algorithm DESIGN §4
    describes: one (p-3)/4 exponentiation per G1 point (382 squarings + 75 multiplies on the
    radix-2^30 core: the table a, a^3, a^7, a^9, a^11, a^13, a^21, a^255 in 7 + 9, then 375 + 66, and
    the radix conversion), two per G2 point (the norm method), 2 x 62 doublings after the tripling in
    the G1 check, each with one fused multiply-plus-square reduction; and the bench's field_ops
    object computed from it."""
    import importlib.util

    census = json.load(open(os.path.join(ROOT, "profiles", "fp_census.json")))
    rows = {(r["op"], r["flags"]): r for r in census["rows"]}
    g1, g2 = rows[("g1_decompress", 0)]["per_point"], rows[("g2_decompress", 0)]["per_point"]
    assert (g1["f30_sqr"], g1["f30_mul"]) == (382, 75)
    assert (g2["f30_sqr"], g2["f30_mul"]) == (2 * 382, 2 * 75)
    assert g1["fp_mul_addsqr"] == 2 * 62
    assert rows[("g1_decompress", 1)]["per_point"].keys() >= {"f30_sqr", "f30_mul"}  # unchecked: the sqrt only
    assert rows[("g1_decompress", 1)]["reductions_per_point"] < 0.4 * rows[("g1_decompress", 0)]["reductions_per_point"]
    assert all(r["all_accepted"] and r["bit_exact"] for r in census["rows"])
    spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    fo = bench.field_ops(census, "g1_decompress", 1 << 27, 2120.0)
    assert fo["reductions_per_point"] == sum(g1.values())
    assert abs(fo["reductions_per_s"] - sum(g1.values()) * (1 << 27) / 2.12) < 1e3
    assert 0.5 < fo["frac"] < 1.5


def test_codec_stall_summary_ratios(tmp_path):
    """tools/codec_stall_summary.py (profiles/r05a_codec_stalls.json): counters summed per kernel
    over its dispatches and passes, GRBM_GUI_ACTIVE averaged over the passes that carry it, SQ_WAVES
    counted once; issue share = 4 x VALU instructions / (GRBM x 128 SIMDs per XCD)."""
    name = "kzgpot::k_g1_codec(HIP_vector_type<unsigned int, 4u> const*)"
    passes = {"p1": {"SQ_WAVE_CYCLES": 2000.0, "SQ_WAIT_ANY": 100.0, "SQ_WAIT_INST_ANY": 900.0,
                     "SQ_ACTIVE_INST_ANY": 1000.0, "SQ_ACTIVE_INST_VALU": 980.0, "GRBM_GUI_ACTIVE": 31.25},
              "p2": {"SQ_WAVES": 2.0, "SQ_INSTS_VALU": 980.0, "SQ_INSTS_SALU": 10.0, "SQ_INSTS_LDS": 4.0,
                     "GRBM_GUI_ACTIVE": 31.25},
              "p3": {"SQ_WAVES": 2.0, "SQ_THREAD_CYCLES_VALU": 980.0 * 64, "SQ_LDS_BANK_CONFLICT": 2.0,
                     "GRBM_GUI_ACTIVE": 31.25}}
    for p, counters in passes.items():
        d = tmp_path / p / "host"
        d.mkdir(parents=True)
        # two dispatches per pass, each carrying half of every counter
        write_csv(d / "run_counter_collection.csv", ["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"],
                  [[k, name, c, v / 2] for k in (1, 2) for c, v in counters.items()])
    p = subprocess.run([sys.executable, os.path.join(TOOLS, "codec_stall_summary.py"), str(tmp_path)],
                       capture_output=True, text=True, check=True)
    k = json.loads(p.stdout)["kernels"]["k_g1_codec"]
    assert k["waves"] == 2.0 and k["per_wave"]["valu"] == 490.0 and k["per_wave"]["salu"] == 5.0
    assert k["wait_any_frac"] == 0.05 and k["active_inst_any_frac"] == 0.5
    assert abs(k["simd_cycles_per_valu"] - 31.25 * 128 / 980) < 1e-12
    assert abs(k["valu_issue_frac_at_4_cycles"] - 4 * 980 / (31.25 * 128)) < 1e-12
    assert k["valu_exec_utilisation"] == 1.0 and k["lds_bank_conflict_per_lds_inst"] == 0.5


def test_isa_sites_finds_the_hot_loops():
    """tools/isa_sites.py (the per-site SALU / branch attribution committed under profiles/) on the
    built library: it must find each codec's square-root loops (a radix-2^30 squaring is 260
    v_mad_i64_i32; G2 inlines two exponentiations) and the ladder doubling loop, and the loops it
    attributes must hold most of the per-wave VALU stream (the schedule: 67 steps, 375 squarings)."""
    from conftest import PKG

    lib = os.path.join(PKG, "build", "libkzgpot.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-C", PKG, "-j", "8"], check=True)
    out = subprocess.run([sys.executable, os.path.join(TOOLS, "isa_sites.py"), "--lib", lib], capture_output=True,
                         text=True, check=True).stdout
    res = json.loads(out)["kernels"]
    for name, copies, ladder_trips in (("k_g1_codec", 1, 124), ("k_g2_codec", 2, 62)):
        sites = res[name]["loop_sites"]
        sq = [s for s in sites if s["site"].startswith("sqrt: f30 squaring loop (window")]
        win = [s for s in sites if s["site"].startswith("sqrt: window step")]
        lad = [s for s in sites if s["site"].startswith("ladder")]
        assert len(sq) == copies and len(win) == copies and len(lad) == 1, (name, [s["site"] for s in sites])
        assert all(s["trips_per_wave"] == 375 for s in sq) and all(s["trips_per_wave"] == 67 for s in win)
        assert lad[0]["trips_per_wave"] == ladder_trips
        # the loops carry the bulk of the VALU stream (PMC: 601 K / 947 K per wave)
        assert res[name]["loops_per_wave"]["valu"] > (480_000 if name == "k_g1_codec" else 800_000)
