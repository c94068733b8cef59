"""pynama_amd -- MI355X-native KLE assembly + Krylov hot path of Pynama.

Drop-in for the reference's matrices/ (MatFS), solver/ (KleSolver, KspSolver)
and the petsc4py Mat/Vec/KSP objects they use; the compute runs in libkle.so
(hand-written HIP for gfx950).  See DESIGN.md and INTEGRATION.md.
"""
from ._lib import Error, load  # noqa: F401
from .domain import Domain  # noqa: F401
from .matrices import MatFS, MatNS, Operators  # noqa: F401
from .problem import BaseProblem, BaseProblemTest  # noqa: F401
from .ts import TsSolver  # noqa: F401
from .mesh import BoxMesh  # noqa: F401
from .runtime import COMM_WORLD, get_ctx, finalize  # noqa: F401
from .solver import KleSolver, KspSolver  # noqa: F401

__version__ = "0.1.0"
