"""Streaming ceilings of this GPU (verdict r04 item 2): every kle_stream_bench
mode, a few alternating repetitions each, one JSON line per mode.

  python tools/stream_ceiling.py [--gb 4] [--reps 10] [--rounds 3]

Modes (kle_core.hip kle_stream_bench): 0 copy 16 B nt stores (the bench's
copy ceiling), 1 read 16 B x4 in flight nt (the bench's read ceiling),
2/3 8-B grid-stride read nt/plain, 4 the round 1-4 read kernel, 5 read 16 B
plain, 6 read 16 B x8, 7 read 16 B x4 at 4 WGs/CU, 8 read 16 B x2 at 16
WGs/CU, 9/10 8-B reads x8/x16 in flight, 11 the round 1-4 copy, 12 copy
16 B plain stores."""
import argparse
import ctypes as C
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gb", type=float, default=4.0)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--modes", default="0,1,2,3,4,5,6,7,8,9,10,11,12")
    a = ap.parse_args()
    import pynama_amd as pa
    from pynama_amd._lib import call
    ctx = pa.get_ctx()
    modes = [int(m) for m in a.modes.split(",")]
    res = {m: [] for m in modes}
    for _ in range(a.rounds):
        for m in modes:
            nb = int(a.gb * 2 ** 30) // (2 if m in (0, 11, 12) else 1)
            g = C.c_double()
            call("kle_stream_bench", ctx.h, nb, a.reps, m, C.byref(g))
            res[m].append(g.value)
    for m in modes:
        print(json.dumps({"mode": m, "gbps_median": statistics.median(res[m]), "gbps": res[m],
                          "bytes": int(a.gb * 2 ** 30), "reps": a.reps}), flush=True)


if __name__ == "__main__":
    main()
