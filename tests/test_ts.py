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


def _trees(n):
    """Rooted trees with n nodes, each a sorted tuple of its subtrees."""
    if n == 1:
        return [()]
    out = set()

    def forests(m, maxt):  # multisets of trees with m nodes in total, non-increasing
        if m == 0:
            yield ()
            return
        for k in range(m, 0, -1):
            for t in _trees(k):
                if maxt is not None and (k, t) > maxt:
                    continue
                for rest in forests(m - k, (k, t)):
                    yield ((k, t),) + rest
    for f in forests(n - 1, None):
        out.add(tuple(sorted(t for _, t in f)))
    return sorted(out)


def _size(t):
    return 1 + sum(_size(u) for u in t)


def _gamma(t):
    g = _size(t)
    for u in t:
        g *= _gamma(u)
    return g


def test_bs54_published_coefficients_exact():
    """The Bogacki-Shampine 5(4) pair typed from the paper (tests/bs54_tableau.py,
    not the product's table): every order condition of all 17 + 8 rooted
    trees holds EXACTLY in rational arithmetic (fifth order for B, fourth for
    BHAT, BHAT fails at fifth), and pynama_amd.ts.TABLEAUX["5bs"] holds the
    nearest doubles of exactly these rationals."""
    from bs54_tableau import A, B, BHAT, C
    s = len(C)
    Af = [[A[i][j] if j < len(A[i]) else 0 for j in range(s)] for i in range(s)]

    def phi(t):  # per stage: prod over subtrees u of sum_j a_ij phi_j(u)
        v = [1] * s
        for u in t:
            pu = phi(u)
            for i in range(s):
                v[i] *= sum(Af[i][j] * pu[j] for j in range(s))
        return v

    assert all(sum(Af[i]) == C[i] for i in range(s))
    assert [len(_trees(n)) for n in range(1, 6)] == [1, 1, 2, 4, 9]
    for n in range(1, 6):
        for t in _trees(n):
            p = phi(t)
            assert sum(B[i] * p[i] for i in range(s)) * _gamma(t) == 1, ("B", t)
            if n <= 4:
                assert sum(BHAT[i] * p[i] for i in range(s)) * _gamma(t) == 1, ("BHAT", t)
    assert any(sum(BHAT[i] * p[i] for i in range(s)) * _gamma(t) != 1
               for t in _trees(5) for p in [phi(t)])
    assert Af[-1][:-1] == B[:-1] and B[-1] == 0  # first same as last
    order, pembed, fsal, c, rows, b, bhat = TABLEAUX["5bs"]
    assert (order, pembed, fsal) == (5, 4, True)
    assert c == [float(v) for v in C]
    assert rows == [[float(v) for v in r] for r in A]
    assert b == [float(v) for v in B]
    assert bhat == [float(v) for v in BHAT]


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
