"""Summarise rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) into profiles/pmc_<config>.json.

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports half the bytes of a wide
coalesced streaming read, so read bytes = 2 * FETCH_SIZE * 1024. The same half count holds for the
small kernels' coalesced 4- and 8-byte loads: calibrated on package_frame_kernel, which reads exactly
28 B per entry (three int64 index fields and a u32 digest) and reports 14 350 kB per 1M entries =
0.50 of 29.4 MB (round 5, profiles/pmc_package4k.json). So every kernel's reads are doubled.
WRITE_SIZE is exact for 16 B/lane streaming stores (the frame kernel's 36-byte frame stores read
1.057 x their bytes). The other kernels of the call are reported beside the main one.

Each summary carries lib_sha256, the sha256 of the bookkeeper_amd/libbkdigest.so the counters were
collected on.

usage: pmc_summary.py FETCH_DIR WRITE_DIR CONFIG ALGO_BYTES_PER_LAUNCH [MAIN_KERNEL [OTHER_KERNELS]]
OTHER_KERNELS: comma-separated short names of the other kernels of the measured call (default: every
other bkd:: kernel in the trace), e.g. the verify pipeline's gate/header/plan/finish launches when the
same process also ran package calls."""
import csv, glob, hashlib, json, os, sys, time
from collections import defaultdict

LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bookkeeper_amd", "libbkdigest.so")


def load(pattern):
    """kernel short name -> counter -> list of per-dispatch values (summed over the dispatch's rows)."""
    per = defaultdict(lambda: defaultdict(float))
    names = {}
    for path in glob.glob(pattern, recursive=True):
        for row in csv.DictReader(open(path)):
            name = row.get("Kernel_Name", "")
            if "bkd::" not in name or "fill_splitmix64" in name:
                continue
            key = (path, row.get("Dispatch_Id", row.get("Correlation_Id", "")))
            per[key][row["Counter_Name"]] += float(row["Counter_Value"])
            names[key] = name.split("(")[0].replace("void ", "").split("<")[0]
    out = defaultdict(lambda: defaultdict(list))
    for key, ctrs in per.items():
        for c, v in ctrs.items():
            out[names[key]][c].append(v)
    return out


def median(v):
    v = sorted(v)
    return v[len(v) // 2] if v else 0.0


def main(fetch_dir, write_dir, config, algo_bytes, main_kernel="bkd::crc_groups_kernel", others=None):
    f = load(os.path.join(fetch_dir, "**", "*counter_collection.csv"))
    w = load(os.path.join(write_dir, "**", "*counter_collection.csv"))
    fetch_kb = median(f[main_kernel]["FETCH_SIZE"])
    write_kb = median(w[main_kernel]["WRITE_SIZE"])
    read_b = 2 * fetch_kb * 1024
    write_b = write_kb * 1024
    aux = {}
    keep = set(others.split(",")) if others else None
    for k in sorted(set(f) | set(w)):
        if k == main_kernel or (keep is not None and k not in keep):
            continue
        aux[k] = {"FETCH_SIZE_kB_median": median(f[k]["FETCH_SIZE"]),
                  "WRITE_SIZE_kB_median": median(w[k]["WRITE_SIZE"])}
    aux_b = sum((2 * a["FETCH_SIZE_kB_median"] + a["WRITE_SIZE_kB_median"]) * 1024 for a in aux.values())
    out = {"config": config, "kernel": main_kernel, "dispatches": len(f[main_kernel]["FETCH_SIZE"]),
           "FETCH_SIZE_kB_median": fetch_kb, "WRITE_SIZE_kB_median": write_kb,
           "hbm_read_bytes_per_launch": read_b, "hbm_write_bytes_per_launch": write_b,
           "hbm_bytes_per_launch": read_b + write_b + aux_b, "main_kernel_bytes_per_launch": read_b + write_b,
           "other_kernels": aux, "other_kernels_bytes_per_launch": aux_b,
           "algorithmic_bytes_per_launch": algo_bytes,
           "traffic_over_algorithmic": (read_b + write_b + aux_b) / algo_bytes,
           "correction": "every kernel: read = 2 x FETCH_SIZE x 1024 (gfx950 half count of coalesced reads, "
                         "calibrated on 16-B streaming loads and on package_frame_kernel's 4/8-B loads), "
                         "write = WRITE_SIZE x 1024",
           # provenance: the build these counters came from (bench.py attaches `traffic` only when the
           # library it times has this hash)
           "lib_sha256": hashlib.sha256(open(LIB, "rb").read()).hexdigest(),
           "collected_utc": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())}
    os.makedirs("profiles", exist_ok=True)
    json.dump(out, open(f"profiles/pmc_{config}.json", "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4]), *sys.argv[5:])
