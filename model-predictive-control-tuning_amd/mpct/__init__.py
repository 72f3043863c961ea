"""mpct — MI355X-native batched closed-loop GPC scoring for MPC tuning.

Host mirror of the reference's closed-loop seam (MPC-Tuning/MPC_Tuning/closedloop_toolbox.m)
and the objectives that call it (GAM_fun.m, VNS2.m), over the C ABI of libmpct.so
(include/mpct.h).  See DESIGN.md.
"""
from . import _lib
from .engine import EvalResult, MpctError, Scenario, closedloop_toolbox, eval_batch, eval_batch_device
from .lti import Tf, c2d, carima, descomp, lsim

__all__ = ["Scenario", "EvalResult", "MpctError", "eval_batch", "eval_batch_device",
           "closedloop_toolbox", "Tf", "c2d", "carima", "descomp", "lsim", "_lib"]
