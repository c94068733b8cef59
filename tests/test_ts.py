"""CPU checks of the Runge-Kutta tableaux behind pynama_amd.ts (the restated
PETSc TSRK types '3'/'3bs', '4', '5f', '5bs'): rows sum to c, and the weights
b / bhat satisfy every order condition (rooted trees) up to the method's and
the embedded method's order.  Exact to 1e-14."""
import numpy as np
import pytest

from pynama_amd.ts import TABLEAUX


def _conditions(A, b, c):
    Ac = A @ c
    out = {1: [(b.sum(), 1.0)],
           2: [(b @ c, 1 / 2)],
           3: [(b @ c ** 2, 1 / 3), (b @ Ac, 1 / 6)],
           4: [(b @ c ** 3, 1 / 4), (b @ (c * Ac), 1 / 8), (b @ (A @ c ** 2), 1 / 12), (b @ (A @ Ac), 1 / 24)],
           5: [(b @ c ** 4, 1 / 5), (b @ (c ** 2 * Ac), 1 / 10), (b @ (c * (A @ c ** 2)), 1 / 15),
               (b @ (c * (A @ Ac)), 1 / 30), (b @ Ac ** 2, 1 / 20), (b @ (A @ c ** 3), 1 / 20),
               (b @ (A @ (c * Ac)), 1 / 40), (b @ (A @ (A @ c ** 2)), 1 / 60), (b @ (A @ (A @ Ac)), 1 / 120)]}
    return out


@pytest.mark.parametrize("name", ["3bs", "4", "5f", "5bs"])
def test_tableau_order_conditions(name):
    order, pembed, fsal, c, rows, b, bhat = TABLEAUX[name]
    s = len(c)
    A = np.zeros((s, s))
    for i, r in enumerate(rows):
        A[i, :len(r)] = r
    c, b = np.array(c), np.array(b)
    np.testing.assert_allclose(A.sum(1), c, atol=1e-14)
    conds = _conditions(A, b, c)
    for p in range(1, order + 1):
        for got, want in conds[p]:
            assert abs(got - want) < 1e-14, (name, p, got, want)
    if bhat is not None:
        bh = np.array(bhat)
        ce = _conditions(A, bh, c)
        for p in range(1, pembed + 1):
            for got, want in ce[p]:
                assert abs(got - want) < 1e-14, (name, "embedded", p, got, want)
        # the pair differs at order pembed + 1 (otherwise no error estimate)
        assert any(abs(g - w) > 1e-6 for g, w in ce[pembed + 1])
    if fsal:
        np.testing.assert_allclose(A[-1, :-1], b[:-1], atol=0)
        assert b[-1] == 0.0 and c[-1] == 1.0


def test_ts_facts_from_reference_tests():
    """The reference's own TS tests (src/tests/test_ts.py:10-19): the solver is
    'rk' / '5bs' by default, and setUpTimes sets start, final time and the
    step limit (ts_solver.py:12-16, MATCHSTEP final time)."""
    from pynama_amd.ts import TsSolver
    ts = TsSolver()
    assert ts.getType() == "rk"
    assert ts.getRKType() == "5bs"
    ts.setUpTimes(1.2, 3.4, 50)
    assert ts.getTime() == 1.2
    assert ts.getMaxTime() == 3.4
    assert ts.getMaxSteps() == 50
    assert ts.exact_final_time == TsSolver.ExactFinalTime.MATCHSTEP
    assert ts.rk_types == ["3", "5f", "5bs"]
