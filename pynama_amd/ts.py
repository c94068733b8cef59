"""TsSolver: explicit Runge-Kutta time integration of the vorticity (SURVEY
8(f) #3).

Mirror of the reference's TsSolver (solver/ts_solver.py:3-23): a PETSc TS of
type 'rk' with RK type '5bs', ODE_EXPLICIT, times from the case's
`time-solver` block, exact final time MATCHSTEP, the problem's evalRHS as the
RHS function and its convergedStepFunction as the post-step hook.  PETSc is
not available here, so this is a restatement of TSRK (src/ts/impls/explicit/rk)
with the TSAdaptBasic step controller as PETSc 3.12 documents them:

* stages  Y_i = X + h sum_{j<i} a_ij K_j,  K_i = f(t + c_i h, Y_i)
  (first-same-as-last reuse of K_s for '5bs' / '3bs' after an accepted step);
* step    X <- X + h sum_j b_j K_j;
* error   TSAdaptChoose_Basic: the embedded solution Y = X_new - E,
  E = h sum_j (b_j - bhat_j) K_j, against X_new in TSErrorWeightedNorm2:
  sqrt(mean((E_i / (atol + rtol max(|X_new_i|, |Y_i|)))^2)), atol = rtol =
  1e-4 (PETSc's TS defaults);
* control h_new = h clip(safety err^(-1/order), 0.1, 10) with order the
  method's (phat + 1), safety 0.9; reject if err > 1 and retry with h_new;
  an attempt that fails right after a failed one uses safety x0.5
  (reject_safety) -- an attempt that passes after a rejection uses 0.9
  again; -ts_adapt_type none takes fixed steps.

The vector ops run on the device (libkle Vec); the RHS is whatever callable
the problem installs -- for BaseProblem.evalRHS one KLE solve plus the
operator chain per stage, and, as in the reference, the stage vector itself is
not read by evalRHS (it uses the problem's own vorticity).  Parity with PETSc
is unpinned (no PETSc in this environment): the tableaux are checked against
the order conditions and the integrator against exact solutions
(tests/test_ts.py, tests/test_gpu_ts.py).
"""
from fractions import Fraction as Fr

import numpy as np

from .petsc import Options, Vec

__all__ = ["TABLEAUX", "TsSolver"]


def _f(rows):
    return [[float(Fr(v)) for v in r] for r in rows]


# name: (order, embedded order, FSAL, c, A (lower triangle rows), b, bhat)
TABLEAUX = {
    # Bogacki & Shampine 3(2) (TSRK3BS)
    "3bs": (3, 2, True, _f([["0", "1/2", "3/4", "1"]])[0],
            _f([[], ["1/2"], ["0", "3/4"], ["2/9", "1/3", "4/9"]]),
            _f([["2/9", "1/3", "4/9", "0"]])[0],
            _f([["7/24", "1/4", "1/3", "1/8"]])[0]),
    # classical RK4 (TSRK4), no embedded pair
    "4": (4, 0, False, _f([["0", "1/2", "1/2", "1"]])[0],
          _f([[], ["1/2"], ["0", "1/2"], ["0", "0", "1"]]),
          _f([["1/6", "1/3", "1/3", "1/6"]])[0], None),
    # Fehlberg 5(4) (TSRK5F)
    "5f": (5, 4, False, _f([["0", "1/4", "3/8", "12/13", "1", "1/2"]])[0],
           _f([[], ["1/4"], ["3/32", "9/32"], ["1932/2197", "-7200/2197", "7296/2197"],
               ["439/216", "-8", "3680/513", "-845/4104"],
               ["-8/27", "2", "-3544/2565", "1859/4104", "-11/40"]]),
           _f([["16/135", "0", "6656/12825", "28561/56430", "-9/50", "2/55"]])[0],
           _f([["25/216", "0", "1408/2565", "2197/4104", "-1/5", "0"]])[0]),
    # Bogacki & Shampine 5(4), 8 stages, FSAL (TSRK5BS, the reference's choice)
    "5bs": (5, 4, True, _f([["0", "1/6", "2/9", "3/7", "2/3", "3/4", "1", "1"]])[0],
            _f([[], ["1/6"], ["2/27", "4/27"], ["183/1372", "-162/343", "1053/1372"],
                ["68/297", "-4/11", "42/143", "1960/3861"],
                ["597/22528", "81/352", "63099/585728", "58653/366080", "4617/20480"],
                ["174197/959244", "-30942/79937", "8152137/19744439", "666106/1039181", "-29421/29068",
                 "482048/414219"],
                ["587/8064", "0", "4440339/15491840", "24353/124800", "387/44800", "2152/5985", "7267/94080"]]),
            _f([["587/8064", "0", "4440339/15491840", "24353/124800", "387/44800", "2152/5985", "7267/94080",
                 "0"]])[0],
            _f([["2479/34992", "0", "123/416", "612941/3411720", "43/1440", "2272/6561", "79937/1113912",
                 "3293/556956"]])[0]),
}
# PETSc's names for the reference's set (ts_solver.py:4)
TABLEAUX["3"] = TABLEAUX["3bs"]


class TsSolver:
    """Same call surface as the reference's TsSolver(TS)."""

    rk_types = ["3", "5f", "5bs"]

    class ExactFinalTime:
        STEPOVER, INTERPOLATE, MATCHSTEP = 0, 1, 2

    def __init__(self, comm=None):
        self.setRKType("5bs")
        self.time = 0.0
        self.max_time = 1.0
        self.max_steps = 5000
        self.step_number = 0
        self.reject = 0
        self.dt = 0.1  # PETSc's default initial step
        self.atol = self.rtol = 1e-4
        self.adapt = "basic"
        self.safety, self.reject_safety, self.clip = 0.9, 0.5, (0.1, 10.0)
        self.dt_min, self.dt_max = 1e-20, 1e50
        self.exact_final_time = self.ExactFinalTime.MATCHSTEP
        self._rhs = self._post = None
        self._solution = None
        self.converged_reason = 0
        self.history = []  # adaptive attempts: (t, h, weighted error, accepted)

    # ------------------------------------------------------------ setup
    def setProblemType(self, t):
        pass

    def setEquationType(self, t):
        pass

    def setType(self, t):
        if t != "rk":
            raise ValueError("only explicit Runge-Kutta ('rk') is provided")

    def getType(self):
        return "rk"

    def setRKType(self, name):
        if name not in TABLEAUX:
            raise ValueError(f"unknown RK type {name!r} (have {sorted(TABLEAUX)})")
        self.rk_type = name
        self.tab = TABLEAUX[name]

    def getRKType(self):
        return self.rk_type

    def setUpTimes(self, sTime, eTime, steps):
        """ts_solver.py:12-16."""
        self.setTime(sTime)
        self.setMaxTime(eTime)
        self.setMaxSteps(steps)
        self.setExactFinalTime(self.ExactFinalTime.MATCHSTEP)

    def initSolver(self, rhsFunction, convergedStepFunction):
        """ts_solver.py:20-23."""
        self.setRHSFunction(rhsFunction)
        self.setPostStep(convergedStepFunction)
        self.setFromOptions()

    def setTime(self, t):
        self.time = float(t)

    def getTime(self):
        return self.time

    def setMaxTime(self, t):
        self.max_time = float(t)

    def getMaxTime(self):
        return self.max_time

    def setMaxSteps(self, n):
        self.max_steps = int(n)

    def getMaxSteps(self):
        return self.max_steps

    def getStepNumber(self):
        return self.step_number

    def setTimeStep(self, dt):
        self.dt = float(dt)

    def getTimeStep(self):
        return self.dt

    def setTolerances(self, rtol=None, atol=None):
        if rtol is not None:
            self.rtol = float(rtol)
        if atol is not None:
            self.atol = float(atol)

    def setExactFinalTime(self, mode):
        self.exact_final_time = mode

    def setAdaptType(self, name):
        if name not in ("basic", "none"):
            raise ValueError("adapt type must be 'basic' or 'none'")
        self.adapt = name

    def setRHSFunction(self, f, vec=None):
        self._rhs = f

    def setPostStep(self, f):
        self._post = f

    def setFromOptions(self):
        o = Options()
        if "ts_rk_type" in o:
            self.setRKType(o.getString("ts_rk_type"))
        if "ts_dt" in o:
            self.setTimeStep(float(o["ts_dt"]))
        if "ts_max_time" in o:
            self.setMaxTime(float(o["ts_max_time"]))
        if "ts_max_steps" in o:
            self.setMaxSteps(int(o["ts_max_steps"]))
        if "ts_adapt_type" in o:
            self.setAdaptType(o.getString("ts_adapt_type"))
        if "ts_rtol" in o:
            self.rtol = float(o["ts_rtol"])
        if "ts_atol" in o:
            self.atol = float(o["ts_atol"])

    def setSolution(self, u):
        self._solution = u

    def getSolution(self):
        return self._solution

    # ------------------------------------------------------------ solve
    def _wrms(self, E, Xn):
        """TSErrorWeightedNorm2(U = X_new, Y = X_new - E): the embedded
        solution's distance from the step's, weighted by both."""
        e, x = E.getArray(), Xn.getArray()
        w = e / (self.atol + self.rtol * np.maximum(np.abs(x), np.abs(x - e)))
        t = Xn.duplicate()
        t.setArray(w)
        n = Xn.getSize()
        return t.norm() / np.sqrt(max(n, 1))

    def solve(self, u):
        """Integrate u in place from getTime() to getMaxTime() (or max steps)."""
        if self._rhs is None:
            raise RuntimeError("RHS function not set (initSolver / setRHSFunction)")
        self._solution = u
        order, pembed, fsal, c, A, b, bhat = self.tab
        s = len(c)
        adaptive = self.adapt == "basic" and bhat is not None
        K = [u.duplicate() for _ in range(s)]
        Y = u.duplicate()
        Xn = u.duplicate()
        E = u.duplicate() if adaptive else None
        have_fsal = False
        eps = 1e-12 * max(1.0, abs(self.max_time))
        while self.step_number < self.max_steps and self.time < self.max_time - eps:
            h = min(self.dt, self.dt_max)
            if self.exact_final_time == self.ExactFinalTime.MATCHSTEP and self.time + h > self.max_time:
                h = self.max_time - self.time
            accept = True  # (TSStep_RK: the previous attempt's verdict, true at a step's start)
            while True:
                for i in range(s):
                    if i == 0 and fsal and have_fsal:
                        K[0], K[s - 1] = K[s - 1], K[0]  # K_s of the accepted step is K_1 of this one
                        have_fsal = False  # (a retry of this step keeps K_1 as it is)
                        continue
                    if i == 0 and fsal and not accept:
                        continue  # TSStep_RK with FSAL never recomputes stage 1: a retry reuses it
                    u.copy(Y)
                    for j in range(i):
                        if A[i][j] != 0.0:
                            Y.axpy(h * A[i][j], K[j])
                    self._rhs(self, self.time + c[i] * h, Y, K[i])
                u.copy(Xn)
                for j in range(s):
                    if b[j] != 0.0:
                        Xn.axpy(h * b[j], K[j])
                if not adaptive:
                    accept, h_next = True, self.dt
                    break
                E.set(0.0)
                for j in range(s):
                    d = b[j] - bhat[j]
                    if d != 0.0:
                        E.axpy(h * d, K[j])
                err = self._wrms(E, Xn)
                safety = self.safety
                if err > 1.0 and not accept:
                    safety *= self.reject_safety  # the last attempt also failed
                accept = err <= 1.0
                hfac = safety * (err ** (-1.0 / (pembed + 1)) if err > 0 else np.inf)
                h_next = min(max(h * min(max(hfac, self.clip[0]), self.clip[1]), self.dt_min), self.dt_max)
                self.history.append((self.time, h, err, accept))
                if accept:
                    break
                self.reject += 1
                h = h_next
            Xn.copy(u)
            self.time += h
            self.step_number += 1
            self.dt = h_next
            have_fsal = fsal
            if self._post is not None:
                self._post(self)
        self.converged_reason = 1 if self.time >= self.max_time - eps else 2
        return u
