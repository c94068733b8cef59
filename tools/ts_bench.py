"""Time-integration measurement: a few RK steps
of BaseProblem (run_case.py timeSolving) on the device.  Prints one JSON line
per case: setup / assembly time, per-step wall time, evalRHS calls, KLE
iterations per solve.  GPU tool.

  python tools/ts_bench.py            # TG-3D on config 2's mesh + cavity-2d as-is (config 1)
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pynama_amd as pa  # noqa: E402


def run(name, cfg, steps, dt, adapt="none"):
    ctx = pa.get_ctx()
    t0 = time.perf_counter()
    prob = pa.BaseProblem(cfg)
    prob.setUp()
    ctx.synchronize()
    t1 = time.perf_counter()
    prob.setUpSolver()
    ctx.synchronize()
    t2 = time.perf_counter()
    prob.setUpInitialConditions()
    ksp = prob.solverKLE.getKSP()
    calls = {"n": 0, "its": []}
    rhs = prob.evalRHS

    def counted(*a, **k):
        calls["n"] += 1
        out = rhs(*a, **k)
        calls["its"].append(ksp.getIterationNumber())
        return out

    prob.ts.initSolver(counted, prob.convergedStepFunction)
    prob.ts.setAdaptType(adapt)
    prob.ts.setTimeStep(dt)
    prob.ts.setUpTimes(0.0, steps * dt, steps)
    ctx.synchronize()
    t3 = time.perf_counter()
    prob.startSolver()
    ctx.synchronize()
    t4 = time.perf_counter()
    n = prob.ts.getStepNumber()
    print(json.dumps({"case": name, "n_dof": prob.mat.K.getSize()[0], "setup_domain_s": t1 - t0,
                      "setup_solver_s": t2 - t1, "steps": n, "s_per_step": (t4 - t3) / max(n, 1),
                      "evalRHS_calls": calls["n"], "kle_its_per_solve": calls["its"][:8],
                      "bc": list(cfg["boundary-conditions"].keys())[0]}), flush=True)


def main():
    tg = {"name": "tg3d", "material-properties": {"rho": 0.5, "mu": 0.01},
          "domain": {"ngl": 5, "box-mesh": {"nelem": [20, 16, 16], "lower": [0, 0, 0], "upper": [1, 1, 1]}},
          "boundary-conditions": {"custom-func": {"name": "taylor_green3d"}},
          "initial-conditions": {"custom-func": {"name": "taylor_green3d"}},
          "time-solver": {"start-time": 0.0, "end-time": 0.02, "max-steps": 2}}
    run("taylor-green3d, config-2 mesh (p=4, 1M DoF), TSRK 5bs, dt 0.01", tg, 2, 0.01)
    cav = {"name": "Cavity2d", "material-properties": {"rho": 0.5, "mu": 0.01},
           "domain": {"ngl": 3, "box-mesh": {"nelem": [50, 50], "lower": [0, 0], "upper": [1, 1]}},
           "time-solver": {"start-time": 0, "end-time": 0.02, "max-steps": 2},
           "boundary-conditions": {"no-slip": {"up": [2, 0], "down": [0, 0], "left": [0, 0], "right": [0, 0]}},
           "initial-conditions": {"vorticity": [0]}}
    run("cavity-2d.yaml as-is (config 1: 50x50, p=2, no-slip), TSRK 5bs, dt 0.01", cav, 2, 0.01)


if __name__ == "__main__":
    main()
