"""Streaming rate of a part of the CUs (kle_stream_bench mode 13: one
1024-thread workgroup per CU, 16-B nontemporal loads, 4 in flight per lane),
for 16 .. all CUs: how fast one CU streams when the others are idle (the
brick SpMV's tail)."""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import pynama_amd as pa
    from pynama_amd._lib import call
    ctx = pa.get_ctx()
    for wgs in (16, 32, 64, 128, 192, 256):
        os.environ["KLE_STREAM_WGS"] = str(wgs)
        g = C.c_double()
        call("kle_stream_bench", ctx.h, 1 << 31, 5, 13, C.byref(g))
        print(json.dumps({"workgroups": wgs, "gbps": g.value, "gbps_per_wg": g.value / wgs}), flush=True)


if __name__ == "__main__":
    main()
