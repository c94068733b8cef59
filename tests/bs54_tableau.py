"""Bogacki & Shampine's 5(4) pair, typed in as exact rationals from the
published paper (P. Bogacki, L. F. Shampine, "An efficient Runge-Kutta (4,5)
pair", Comput. Math. Appl. 32(6):15-28, 1996), the tableau PETSc registers as
TSRK5BS, the reference's integrator (ts_solver.py:3-23).  Test data only: the
tests check pynama_amd.ts.TABLEAUX["5bs"] against it and integrate with it,
so a wrong coefficient in the product's table does not cancel out."""
from fractions import Fraction as F

C = [F(0), F(1, 6), F(2, 9), F(3, 7), F(2, 3), F(3, 4), F(1), F(1)]
A = [
    [],
    [F(1, 6)],
    [F(2, 27), F(4, 27)],
    [F(183, 1372), F(-162, 343), F(1053, 1372)],
    [F(68, 297), F(-4, 11), F(42, 143), F(1960, 3861)],
    [F(597, 22528), F(81, 352), F(63099, 585728), F(58653, 366080), F(4617, 20480)],
    [F(174197, 959244), F(-30942, 79937), F(8152137, 19744439), F(666106, 1039181), F(-29421, 29068),
     F(482048, 414219)],
    [F(587, 8064), F(0), F(4440339, 15491840), F(24353, 124800), F(387, 44800), F(2152, 5985),
     F(7267, 94080)],
]
# fifth-order weights (= the last row: first same as last) and the
# fourth-order embedded weights of the error estimate
B = [F(587, 8064), F(0), F(4440339, 15491840), F(24353, 124800), F(387, 44800), F(2152, 5985),
     F(7267, 94080), F(0)]
BHAT = [F(2479, 34992), F(0), F(123, 416), F(612941, 3411720), F(43, 1440), F(2272, 6561),
        F(79937, 1113912), F(3293, 556956)]
