"""Counter profile of bench.py's C3 device-resident round, for the line's
summary.c3_roofline (bench.load_c3_pmc).

Reads the summary tools/pmc_kernels.py wrote for `tools/gpu_session.sh pmcsec
c3_certificate_verify c3 k_cert_verify k_cert_digests k_job_count k_job_scan
k_job_place` (per (kernel, grid) medians over dispatches; FETCH_SIZE already
doubled per the gfx950 calibration), keeps the dispatches of the 10k-
certificate device round -- the grids its launcher uses for n certificates
and n_votes votes -- and writes per-round totals with the sha256 of the
committee kernels' sources and build flags (bench.c3_kernel_src_sha256;
bench.py uses the figures only while those are unchanged).

usage: python tools/pmc_c3_tie.py <pmc_kernels summary.json> <out.json> [n_certs] [votes_per_cert]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def round_grids(nc, nv):
    """Work-item grid sizes of the device round's launches (coa_committee.hip
    coa_launch_cert_verify): the certificate-digest prologue (one lane per
    certificate), the key-order sort (COA_SORT_WGS x 256, and one 1,024-thread
    scan), and k_cert_verify (header-digest blocks + the signature lanes, two
    waves per SIMD: 131,072 lanes)."""
    hdr_blocks = (nc + 255) // 256
    return {"k_cert_digests": hdr_blocks * 256, "k_job_count": 256 * 256, "k_job_scan": 1024,
            "k_job_place": 256 * 256, "k_cert_verify": hdr_blocks * 256 + 131072}


def main():
    src, dst = sys.argv[1], sys.argv[2]
    nc = int(sys.argv[3]) if len(sys.argv) > 3 else 10000
    vpc = int(sys.argv[4]) if len(sys.argv) > 4 else 67
    sys.path.insert(0, ROOT)
    import bench

    with open(src) as f:
        summ = json.load(f)["kernels"]
    grids = round_grids(nc, nc * vpc)
    res = {"n_certs": nc, "votes_per_cert": vpc, "kernel_src_sha256": bench.c3_kernel_src_sha256(),
           "command": "tools/gpu_session.sh pmcsec c3_certificate_verify c3 k_cert_verify k_cert_digests k_job_count "
                      "k_job_scan k_job_place (rocprofv3 --pmc, one counter set per pass, bench.py --sections "
                      "c3_certificate_verify)",
           "kernels": {}}
    valu = fetch = write = dur = 0.0
    for k, g in grids.items():
        e = summ.get(f"{k}@{g}")
        if e is None:
            raise SystemExit(f"no {k}@{g} in {src}")
        res["kernels"][k] = {x: e.get(x) for x in ("grid", "dispatches", "duration_us", "waves", "valu_insts",
                                                   "issue_frac", "cycles_per_valu_per_wave", "valu_active_share",
                                                   "wait_any_share", "fetch_bytes", "write_bytes")}
        valu += e["valu_insts"]
        fetch += e.get("fetch_bytes") or 0.0
        write += e.get("write_bytes") or 0.0
        dur += e["duration_us"]
    res["valu_insts_per_round"] = valu
    res["hbm_bytes_per_round"] = fetch + write
    res["fetch_bytes_per_round"] = fetch
    res["write_bytes_per_round"] = write
    res["profiled_kernel_us_per_round"] = dur
    os.makedirs(os.path.dirname(os.path.abspath(dst)), exist_ok=True)
    with open(dst, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "kernels"}))


if __name__ == "__main__":
    main()
