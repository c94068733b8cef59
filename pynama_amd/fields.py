"""Analytic Taylor-Green fields used as boundary values, initial conditions and
known answers (inputs of the hot path, not part of it).

Same fields as the reference's src/functions/taylor_green.py:4-72 (2-D),
taylor_green3d.py:4-33 (3-D) and taylor_green_3d.py:4-28 (2-D flow embedded
in 3-D), on a unit period box (Lx = Ly = Lz = 1, Uref = 1).  Velocity and
3-D vorticity are returned node-interleaved and flattened, the 2-D
vorticity as one value per node, as the reference does.
"""
from math import exp, pi

import numpy as np

TWO_PI = 2.0 * pi


class TaylorGreen2D:
    name = "taylor_green"

    @staticmethod
    def alpha(nu, t):
        return exp(-4.0 * pi ** 2 * nu * t * 2.0)

    @staticmethod
    def velocity(coords, alpha=1.0):
        x, y = TWO_PI * coords[:, 0], TWO_PI * coords[:, 1]
        return np.stack([np.cos(x) * np.sin(y) * alpha, -np.sin(x) * np.cos(y) * alpha], 1).ravel()

    @staticmethod
    def vorticity(coords, alpha=1.0):
        x, y = TWO_PI * coords[:, 0], TWO_PI * coords[:, 1]
        return -2.0 * pi * 2.0 * np.cos(x) * np.cos(y) * alpha


class TaylorGreen3D:
    name = "taylor_green3d"

    @staticmethod
    def alpha(nu, t):
        return exp(-4.0 * pi ** 2 * nu * t * 3.0)

    @staticmethod
    def velocity(coords, alpha=1.0):
        x, y, z = (TWO_PI * coords[:, d] for d in range(3))
        u = np.cos(x) * np.sin(y) * np.sin(z) * alpha
        v = np.sin(x) * np.cos(y) * np.sin(z) * alpha
        w = -2.0 * np.sin(x) * np.sin(y) * np.cos(z) * alpha
        return np.stack([u, v, w], 1).ravel()

    @staticmethod
    def vorticity(coords, alpha=1.0):
        x, y, z = (TWO_PI * coords[:, d] for d in range(3))
        wx = -2.0 * pi * 3.0 * np.sin(x) * np.cos(y) * np.cos(z) * alpha
        wy = 2.0 * pi * 3.0 * np.cos(x) * np.sin(y) * np.cos(z) * alpha
        wz = np.zeros_like(wx)  # 2 pi (Ly/Lx - Lx/Ly) = 0 on the unit box
        return np.stack([wx, wy, wz], 1).ravel()


class TaylorGreen2Din3D:
    name = "taylor_green_3d"

    @staticmethod
    def alpha(nu, t):
        return exp(-4.0 * pi ** 2 * nu * t * 2.0)

    @staticmethod
    def velocity(coords, alpha=1.0):
        x, y = TWO_PI * coords[:, 0], TWO_PI * coords[:, 1]
        u = np.cos(x) * np.sin(y) * alpha
        v = -np.sin(x) * np.cos(y) * alpha
        return np.stack([u, v, np.zeros_like(u)], 1).ravel()

    @staticmethod
    def vorticity(coords, alpha=1.0):
        x, y = TWO_PI * coords[:, 0], TWO_PI * coords[:, 1]
        wz = -2.0 * pi * 2.0 * np.cos(x) * np.cos(y) * alpha
        z = np.zeros_like(wz)
        return np.stack([z, z, wz], 1).ravel()


FUNCTIONS = {c.name: c for c in (TaylorGreen2D, TaylorGreen3D, TaylorGreen2Din3D)}


def get(name):
    try:
        return FUNCTIONS[name]
    except KeyError:
        raise ValueError(f"unknown custom-func '{name}' (have {sorted(FUNCTIONS)})")
