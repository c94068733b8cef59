"""Known-byte streaming reads for calibrating rocprofv3 FETCH_SIZE on gfx950
(run under --pmc FETCH_SIZE).  Each mode reads 2 GiB once per launch."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pynama_amd as pa  # noqa: E402
import ctypes as C  # noqa: E402
from pynama_amd._lib import call  # noqa: E402

ctx = pa.get_ctx()
for mode in (1, 2, 3):
    g = C.c_double()
    call("kle_stream_bench", ctx.h, 1 << 31, 3, mode, C.byref(g))
    print("mode", mode, "GB/s", g.value, flush=True)
