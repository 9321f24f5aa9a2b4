"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into per-launch HBM
bytes for one kernel (MI355X_MICROARCH.md HBM section: FETCH_SIZE and
WRITE_SIZE are KiB; on gfx950 FETCH_SIZE reports 1/2 of the bytes of wide
coalesced reads, so the read side is doubled).

usage: python tools/pmc_traffic.py <gpurun_out dir> <kernel[,kernel...]> <n> <out.json>
"""
import csv
import glob
import json
import os
import statistics
import sys


def per_dispatch(root, counter, kernel):
    vals = {}
    for path in glob.glob(os.path.join(root, f"pmc_{counter}", "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if row.get("Kernel_Name", "").split("(")[0] != kernel or row.get("Counter_Name") != counter:
                    continue
                d = row.get("Dispatch_Id")
                vals[d] = vals.get(d, 0.0) + float(row["Counter_Value"])
    return list(vals.values())


def main():
    root, kernels, n, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
    f_kib = w_kib = 0.0
    nd = []
    for kernel in kernels.split(","):  # a stage of several kernels: sum of per-kernel medians
        fetch = per_dispatch(root, "FETCH_SIZE", kernel)
        write = per_dispatch(root, "WRITE_SIZE", kernel)
        if not fetch or not write:
            raise SystemExit(f"no {kernel} rows found under {root}")
        f_kib += statistics.median(fetch)
        w_kib += statistics.median(write)
        nd.append([len(fetch), len(write)])
    kernel = kernels
    res = {
        "kernel": kernel,
        "n": n,
        "dispatches": nd,
        "fetch_size_kib_raw": f_kib,
        "write_size_kib": w_kib,
        "hbm_read_bytes_corrected": 2 * f_kib * 1024,
        "hbm_write_bytes": w_kib * 1024,
        "hbm_bytes_per_launch": 2 * f_kib * 1024 + w_kib * 1024,
        "note": "FETCH_SIZE doubled per the gfx950 calibration (wide coalesced reads); medians over dispatches",
    }
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
