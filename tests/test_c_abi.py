"""The C ABI from plain C (tests/c_abi/mpct_c_demo.c, gcc, no torch): what a MATLAB loadlibrary /
calllib or MEX host links against.  CPU: the client builds, creates the Van de Vusse NMPC scenario
from plain arrays and gets the documented error codes.  GPU: it scores three candidates through
mpct_eval_batch, and the costs equal (bit for bit) those of the Python host mirror on the same
inputs — one library, two hosts."""
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "c_abi", "mpct_c_demo.c")
EXE = os.path.join(ROOT, "tests", "c_abi", "mpct_c_demo")
CSRC = os.path.join(ROOT, "model-predictive-control-tuning_amd", "csrc")


def _build():
    subprocess.run(["gcc", "-O2", "-Wall", "-Werror", "-std=c99", "-I", os.path.join(ROOT, "include"), SRC,
                    "-L", CSRC, "-lmpct", "-Wl,-rpath," + CSRC, "-Wl,-rpath,/opt/rocm/lib", "-o", EXE], check=True)
    return EXE


def test_c_client_builds_and_validates(built):
    out = subprocess.run([_build()], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "expected error: nu*nu_max > 32" in out.stdout and out.stdout.strip().endswith("ok")
    assert "linear instance gpc_small_kernel" in out.stdout


@pytest.mark.gpu
def test_c_client_matches_python_host(built, has_gpu):
    if not has_gpu:
        pytest.skip("no GPU")
    out = subprocess.run([_build(), "eval"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    rows = re.findall(r"cand (\d) status (\d+) J1 (\S+) (\S+)", out.stdout)
    assert len(rows) == 3
    from mpct.engine import eval_batch
    from mpct.nmpc import VDV_U0, VDV_UMAX, VDV_UMIN, VDV_XMAX, VDV_XMIN, NmpcScenario, steady_state

    x0 = steady_state()
    nit = 60
    r = np.zeros((2, nit))
    r[0] = np.where(np.arange(nit) >= 9, 1.0, x0[1])
    r[1] = np.where(np.arange(nit) >= 40, 130.0, x0[2])
    sc = NmpcScenario(x0, VDV_U0, VDV_UMIN, VDV_UMAX, VDV_XMIN, VDV_XMAX, r.copy(), 31, 15)
    d = np.array([[0.09302224780430422, 0.11333840205801392], [1.0, 0.5], [0.3, 2.0]])
    lam = np.array([[0.245996189227521, 0.12310801096548595], [0.05, 0.02], [0.1, 0.1]])
    res = eval_batch(sc, [3, 12, 25], [2, 4, 7], d, lam, r[None])
    for c, (k, st, a, b) in enumerate(rows):
        assert int(st) == res.status[c]
        np.testing.assert_array_equal([float(a), float(b)], res.J1[c])


@pytest.mark.gpu
def test_c_client_linear_shell3x3_matches_python_host(built, has_gpu):
    """The linear Shell 3x3 scenario from the saved mpc object's plant (no CARIMA tables: the
    library derives them) scored by the C client equals the Python host's eval_batch on the same
    tf entries, bit for bit."""
    if not has_gpu:
        pytest.skip("no GPU")
    import json

    from mpct.engine import Scenario, eval_batch
    from mpct.lti import Tf
    from mpct.scenarios import shell3x3_xsp

    out = subprocess.run([_build(), "eval"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    rows = re.findall(r"lin (\d) status (\d+) J1 (\S+) (\S+) (\S+)", out.stdout)
    assert len(rows) == 3
    fx = json.load(open(os.path.join(ROOT, "tests", "golden", "tuning_parameters_mat.json")))["shell3x3_25jul2023"]
    ps = fx["plant_scaled_discrete"]
    P = [[Tf.make(ps["num"][i][j], ps["den"][i][j], ps["iodelay"][i][j]) for j in range(3)] for i in range(3)]
    L = np.array(fx["scale"]["L"])
    r = L[:, None] * shell3x3_xsp(500)
    mv = fx["MV"]
    umin = np.array([m["Min"] for m in mv])
    umax = np.array([m["Max"] for m in mv])
    dumax = np.array([m["RateMax"] for m in mv])
    sc = Scenario(P, P, nu=3, du_min=-dumax, du_max=dumax, u_min=umin, u_max=umax, yref=r, n2_max=30, nu_max=5,
                  Ts=4.0)
    d = np.array([fx["delta"], [0.5, 0.1, 0.01], [1.0, 1.0, 1.0]])
    lam = np.array([fx["lambda"], [0.001, 0.01, 0.002], [0.1, 0.1, 0.1]])
    res = eval_batch(sc, [30, 30, 30], [5, 5, 5], d, lam, r[None])
    for c, row in enumerate(rows):
        assert int(row[1]) == res.status[c]
        np.testing.assert_array_equal([float(x) for x in row[2:]], res.J1[c])
