"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into per-launch HBM bytes
of one SpMV, with the gfx950 corrections of MI355X_MICROARCH.md (HBM):
counters are in KiB; FETCH_SIZE reads 1/2 of the bytes of a coalesced
streaming read (128-B requests tallied as 64 B), so it is doubled.

  python tools/pmc_traffic.py FETCH_DIR WRITE_DIR BENCH_JSON [KEY|auto] [OUT]

(auto: the key bench.py looks the record up by, roofline.traffic_key)

BENCH_JSON is the bench.py line of the profiled run itself: its
roofline.kernel names the launches of one SpMV ("a+b": the tile kernel and
its gather, each counted once) and roofline.bytes_per_launch is the
algorithmic byte count of that kernel, stored with the record so that
bench.py can refuse a counter measured on a different kernel (a record whose
algorithmic bytes differ from the running kernel's is reported as null)."""
import csv
import glob
import json
import os
import sys


def median(d, name):
    """Median counter over the dispatches of kernel `name` (the template
    arguments included): the SpMV also runs on Krhs and Rw while the
    right-hand side is formed; the median of the (timed-loop dominated)
    dispatch list is the bench matrix's value."""
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    want = name.replace(" ", "") + "("  # (rocprofv3 names carry "void kle::" and the argument list)
    v = [float(r["Counter_Value"]) for r in csv.DictReader(open(f))
         if want in r["Kernel_Name"].replace(" ", "").replace("voidkle::", "").replace("kle::", "")]
    if not v:
        raise SystemExit(f"pmc_traffic: no dispatch of {name} in {f}")
    v.sort()
    return v[len(v) // 2], len(v)


def main():
    fd, wd, bj = sys.argv[1:4]
    key = sys.argv[4] if len(sys.argv) > 4 else "auto"
    out = sys.argv[5] if len(sys.argv) > 5 else "profiles/traffic.json"
    line = [ln for ln in open(bj) if ln.startswith("{")][-1]
    rl = json.loads(line)["roofline"]
    if key == "auto":
        key = rl["traffic_key"]
    kernels = rl["kernel"].split("+")
    parts, fetch, write, launches = {}, 0.0, 0.0, []
    for k in kernels:
        f, nf = median(fd, k)
        w, nw = median(wd, k)
        parts[k] = {"FETCH_SIZE_KiB": f, "WRITE_SIZE_KiB": w, "hbm_bytes": (2 * f + w) * 1024, "launches": [nf, nw]}
        fetch += f
        write += w
        launches.append([nf, nw])
    hbm = (2 * fetch + write) * 1024
    alg = rl["bytes_per_launch"]
    rec = {"kernel": rl["kernel"], "launches": launches, "FETCH_SIZE_KiB": fetch, "WRITE_SIZE_KiB": write,
           "fetch_bytes_corrected": fetch * 1024 * 2, "write_bytes": write * 1024,
           "hbm_bytes_per_launch": hbm, "algorithmic_bytes_per_launch": alg,
           "traffic_over_algorithmic": hbm / alg, "parts": parts,
           "source": os.path.dirname(os.path.abspath(fd)),
           "correction": "FETCH_SIZE x2 (gfx950 128-B requests tallied as 64 B), KiB -> B; "
                         "per-kernel dispatch medians of one SpMV summed"}
    db = json.load(open(out)) if os.path.exists(out) else {}
    db[key] = rec
    json.dump(db, open(out, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
