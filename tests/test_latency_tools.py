"""CPU tests of the latency-roofline tooling: tools/latency_model.py on a synthetic
profile, tools/diag/section_isa.py on a synthetic ISA listing, and bench.py's roofline.latency_frac,
which it reports only for the library the latency model was fitted to (sha256 key, like
roofline.traffic)."""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools", "diag")]

SECTIONS = ["prologue", "plant", "y_update", "unconstrained", "qp(rest)", "u_update", "open_loop",
            "qp.check", "qp.d+z", "qp.r+t1", "qp.add", "qp.drop", "qp.warm", "qp.rotations"]


def _probe(tmp_path):
    names = ["fma_f64", "add_f64", "dpp_stage_f64", "row_sum16", "row4_sum_permlane", "bcast_readlane",
             "shfl_bpermute", "lds_handoff", "rsq_nr", "rcp_nr", "row_bcast16", "qargmin16_key", "row_argmin",
             "wave_argmin64", "uniform_branch", "ballot_branch", "lds_read_chase", "dpp_mov_pair",
             "block_prefix16_nu5", "mul_f64", "qargmin16_exact"]
    p = tmp_path / "probe.json"
    p.write_text(json.dumps({n: 10.0 for n in names}))
    return p


def _prof(tmp_path, sims=4):
    # per simulation and section: cycles in the low 48 bits, executions in the high 16
    words = np.zeros((sims, len(SECTIONS)), dtype=np.uint64)
    for k, name in enumerate(SECTIONS):
        execs = 500 if k < 7 else (700 if name == "qp.check" else 100)
        cyc = 1000 * execs
        words[:, k] = np.uint64(cyc) | (np.uint64(execs) << np.uint64(48))
    p = tmp_path / "prof.bin"
    words.tofile(p)
    return p


def test_latency_model_synthetic(tmp_path):
    probe, prof = _probe(tmp_path), _prof(tmp_path)
    out = tmp_path / "model.json"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "latency_model.py"), str(probe), str(prof),
                        "--out", str(out)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    rep = json.loads(out.read_text())
    assert rep["simulations"] == 4
    assert 0.0 < rep["latency_frac"] < 1.0
    # the QP's entry stamp (once per step) is not priced as a check: 700 - 500 executions
    assert rep["sections"]["qp.check"]["executions"] == 200.0
    assert rep["model_cycles"] <= rep["measured_cycles"]


def test_latency_model_warm_split(tmp_path):
    """r06 profile layout: 21 words per simulation, counts in the high 24 bits,
    the warm start priced per section (entry, rebuild + re-adds, gather, solve passes, drops + their
    rotations) and the old qp.warm word a near-empty remainder."""
    names = SECTIONS + ["qp.w.entry", "qp.w.rebuild", "qp.w.gather", "qp.w.solve", "qp.w.drop", "qp.w.rotations",
                        "qp.w.readds"]
    words = np.zeros((4, len(names)), dtype=np.uint64)
    for k, name in enumerate(names):
        execs = 500 if k < 7 else (700 if name == "qp.check" else 100)
        words[:, k] = np.uint64(1000 * execs) | (np.uint64(execs) << np.uint64(40))
    prof = tmp_path / "prof21.bin"
    words.tofile(prof)
    out = tmp_path / "model21.json"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "latency_model.py"), str(_probe(tmp_path)),
                        str(prof), "--out", str(out)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    rep = json.loads(out.read_text())
    sec = rep["sections"]
    assert sec["qp.check"]["executions"] == 200.0          # 40-bit split decoded
    assert sec["qp.warm"]["model"] == 0                     # split into qp.w.*
    for name in ("qp.w.entry", "qp.w.rebuild", "qp.w.gather", "qp.w.solve", "qp.w.drop"):
        assert sec[name]["model"] > 0, name
    # the warm drops and the rebuild carry their counted rotations / re-adds on top of the base chain
    assert sec["qp.w.drop"]["model"] > sec["qp.w.drop"]["chain_cycles"] * 100
    assert sec["qp.w.rebuild"]["model"] > sec["qp.w.rebuild"]["chain_cycles"] * 100


def test_section_isa_counts(tmp_path):
    from section_isa import section_counts

    asm = tmp_path / "k.s"
    asm.write_text("\n".join([
        "_Z3fooPd:",
        "\tv_add_f64 v[0:1], v[2:3], v[4:5]",
        "\t; PSTAMP PROF_PLANT",
        "\tv_mov_b32_dpp v1, v2 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf",
        "\tds_read_b64 v[2:3], v1",
        "\ts_waitcnt lgkmcnt(0)",
        "\tv_fma_f64 v[0:1], v[2:3], v[4:5], v[0:1]",
        "\t; PSTAMP PROF_YUPD",
        "\ts_endpgm",
    ]))
    rows = dict(section_counts(str(asm), "foo"))
    assert rows["PROF_PLANT #0"] == {"valu_f64": 1}
    assert rows["PROF_YUPD #0"] == {"valu_dpp": 1, "lds": 1, "wait": 1, "valu_f64": 1}


def test_bench_latency_frac_keyed_to_library(tmp_path, monkeypatch):
    import bench

    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    monkeypatch.setattr(bench, "lib_sha256", lambda: "a" * 64)
    frac, note = bench.latency_roofline()
    assert frac is None and "no latency model" in note
    (tmp_path / "profiles").mkdir()
    lat = tmp_path / "profiles" / "latency_latest.json"
    lat.write_text(json.dumps({"lib_sha256": "b" * 64, "latency_frac": 0.3}))
    frac, note = bench.latency_roofline()
    assert frac is None and "not used" in note
    lat.write_text(json.dumps({"lib_sha256": "a" * 64, "latency_frac": 0.3}))
    frac, note = bench.latency_roofline()
    assert frac == 0.3


def test_bench_workload_pmc_keyed_to_library(tmp_path, monkeypatch):
    """the other §8d lines' traffic / counter rate come from the PMC pass over bench.py
    (tools/pmc_workloads.sh) only when it profiled the loaded library"""
    import bench

    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    monkeypatch.setattr(bench, "lib_sha256", lambda: "a" * 64)
    tr, note, fc = bench.pmc_workload("shell7x5", 900.0)
    assert tr is None and fc is None and "no workload PMC" in note
    (tmp_path / "profiles").mkdir()
    p = tmp_path / "profiles" / "pmc_workloads_latest.json"
    rec = {"tag": "r99", "shell7x5": {"hbm_bytes_per_evaluation": 6.0e8, "fp64_flops_per_evaluation": 4.5e12}}
    p.write_text(json.dumps(dict(rec, lib_sha256="b" * 64)))
    tr, note, fc = bench.pmc_workload("shell7x5", 900.0)
    assert tr is None and fc is None and "not used" in note
    p.write_text(json.dumps(dict(rec, lib_sha256="a" * 64)))
    tr, note, fc = bench.pmc_workload("shell7x5", 900.0)
    assert tr == 6.0e8 and abs(fc - 5.0) < 1e-12 and "r99_pmc_workloads" in note
    tr, note, fc = bench.pmc_workload("vandevusse", 190.0)
    assert tr is None and fc is None
