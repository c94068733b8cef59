"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into per-launch HBM bytes
for one kernel, with the gfx950 corrections of MI355X_MICROARCH.md (HBM):
counters are in KiB; FETCH_SIZE reads 1/2 of the bytes of a coalesced
streaming read (128-B requests tallied as 64 B), so it is doubled.
Usage: python tools/pmc_traffic.py FETCH_DIR WRITE_DIR KERNEL_SUBSTR KEY [OUT]"""
import csv
import glob
import json
import os
import sys


def avg(d, sub):
    """Median counter over the dispatches of `sub`: the same kernel also runs
    once each on Krhs and Rw while the right-hand side is formed; the median
    of the (timed-loop dominated) dispatch list is the bench matrix's value."""
    f = glob.glob(os.path.join(d, "*counter_collection.csv"))[0]
    v = [float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if sub in r["Kernel_Name"]]
    v.sort()
    return v[len(v) // 2], len(v)


def main():
    fd, wd, sub, key = sys.argv[1:5]
    out = sys.argv[5] if len(sys.argv) > 5 else "profiles/traffic.json"
    fetch, nf = avg(fd, sub)
    write, nw = avg(wd, sub)
    rec = {"kernel": sub, "launches": [nf, nw], "FETCH_SIZE_KiB": fetch, "WRITE_SIZE_KiB": write,
           "fetch_bytes_corrected": fetch * 1024 * 2, "write_bytes": write * 1024,
           "hbm_bytes_per_launch": (2 * fetch + write) * 1024,
           "correction": "FETCH_SIZE x2 (gfx950 128-B requests tallied as 64 B), KiB -> B"}
    db = json.load(open(out)) if os.path.exists(out) else {}
    db[key] = rec
    json.dump(db, open(out, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
