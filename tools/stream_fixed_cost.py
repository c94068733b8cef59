"""Fixed cost of a plain streaming-read kernel on this GPU: k_stream_read
(libkle kle_stream_bench) over 64 MB .. 4 GB, time = a + bytes / BW fitted;
compare with the SpMV's 17 us + bytes / 6.09 TB/s (profiles/r02/slab_*.json)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np

    import pynama_amd as pa
    ctx = pa.get_ctx()
    xs, ys = [], []
    for mb in (64, 128, 256, 384, 512, 1024, 2048, 4096):
        nb = mb << 20
        g = ctx.stream_read_gbps(nb, 50)
        t_us = nb / (g * 1e9) * 1e6
        xs.append(nb / 1e9)
        ys.append(t_us)
        print(json.dumps({"bytes": nb, "gbps": g, "us": t_us}), flush=True)
    A = np.vstack([np.ones(len(xs)), xs]).T
    c, *_ = np.linalg.lstsq(A, np.array(ys), rcond=None)
    print(json.dumps({"fit_fixed_us": c[0], "fit_tbps": 1e3 / c[1]}), flush=True)


if __name__ == "__main__":
    main()
