"""Summarise rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) for the CRC kernel into
profiles/pmc_<config>.json. gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports
half the bytes of a wide coalesced streaming read, so read bytes = 2 * FETCH_SIZE * 1024;
WRITE_SIZE is exact for 16 B/lane streaming stores (our 4 B/lane digest stores are uncalibrated,
and are 0.1 % of the traffic)."""
import csv, glob, json, os, sys
from collections import defaultdict


def load(pattern):
    vals = defaultdict(list)
    for path in glob.glob(pattern, recursive=True):
        for row in csv.DictReader(open(path)):
            name = row.get("Kernel_Name", "")
            if "crc_groups_kernel" not in name:
                continue
            vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
    return vals


def main(fetch_dir, write_dir, config, algo_bytes):
    f = load(os.path.join(fetch_dir, "**", "*counter_collection.csv"))
    w = load(os.path.join(write_dir, "**", "*counter_collection.csv"))
    fetch_kb = sorted(f["FETCH_SIZE"])[len(f["FETCH_SIZE"]) // 2]
    write_kb = sorted(w["WRITE_SIZE"])[len(w["WRITE_SIZE"]) // 2]
    read_b = 2 * fetch_kb * 1024
    write_b = write_kb * 1024
    out = {"config": config, "kernel": "crc_groups_kernel", "dispatches": len(f["FETCH_SIZE"]),
           "FETCH_SIZE_kB_median": fetch_kb, "WRITE_SIZE_kB_median": write_kb,
           "hbm_read_bytes_per_launch": read_b, "hbm_write_bytes_per_launch": write_b,
           "hbm_bytes_per_launch": read_b + write_b, "algorithmic_bytes_per_launch": algo_bytes,
           "traffic_over_algorithmic": (read_b + write_b) / algo_bytes,
           "correction": "read = 2 x FETCH_SIZE x 1024 (gfx950 half-count of wide streaming reads); write = WRITE_SIZE x 1024"}
    os.makedirs("profiles", exist_ok=True)
    json.dump(out, open(f"profiles/pmc_{config}.json", "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4]))
