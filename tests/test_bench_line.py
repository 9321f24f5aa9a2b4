"""CPU tests of bench.py's output contract and its `--gpus N` launch path.

* The headline line (the LAST stdout line, which the driver parses) stays
  compact: round 5's line carried 33.7 KB of secondary sections and the
  driver recorded `parsed: null`.  Built here from that recorded run
  (profiles/r05_bench_final.json), it must fit the driver's tail and keep
  every contract key, roofline and cpu_baseline.
* `bench.py --gpus 2` without a launcher spawns two ranks (one per device,
  torchrun's environment) and rank 0 prints one line with n_gpus 2 and both
  ranks' index ranges.  The ranks here are tests/bench_rank_standin.py: the
  bench's own timed region, gather and line, with the CPU oracle standing in
  for each GPU."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import bench  # noqa: E402

RECORDED = os.path.join(ROOT, "profiles", "r05_bench_final.json")


def _recorded():
    with open(RECORDED) as f:
        return json.load(f)


def test_headline_from_recorded_run_fits_and_keeps_contract_keys():
    rec = _recorded()
    base = {k: rec[k] for k in bench.HEADLINE_KEYS if k in rec}
    base.update({k: rec[k] for k in ("kernel_ms", "verdicts_ok", "build")})
    summary = bench.summarize(rec["value"], rec["secondary"], rec["cpu_baseline"])
    line = bench.headline(base, rec["roofline"], rec["cpu_baseline"], summary,
                          ranks=[{"rank": 0, "device": 0, "index_range": [0, 65536]}],
                          secondary_path="gpurun_out/bench_secondary.json")
    s = json.dumps(line)
    assert len(s) < bench.HEADLINE_MAX_BYTES <= 16384
    for k in bench.HEADLINE_KEYS:
        assert k in line, k
    assert "secondary" not in line
    assert list(line)[-1] == "summary"
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "issue_frac", "counters"):
        assert k in line["roofline"], k
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in line["cpu_baseline"], k
    assert "by_threads" not in line["cpu_baseline"]
    assert line["summary"]["c2_verify_per_s"] == round(rec["value"], 1)
    assert line["summary"]["c3_cert_p50_ms"]["gpu_c_caller"] is not None
    assert "truncated" not in line["summary"]


def test_headline_trims_summary_never_contract_keys():
    rec = _recorded()
    base = {k: rec[k] for k in bench.HEADLINE_KEYS if k in rec}
    summary = {f"k{i}": "x" * 500 for i in range(40)}
    line = bench.headline(base, rec["roofline"], rec["cpu_baseline"], summary)
    assert len(json.dumps(line)) <= bench.HEADLINE_MAX_BYTES
    assert line["summary"].get("truncated") is True
    for k in bench.HEADLINE_KEYS:
        assert k in line


def test_rank_env_is_torchrun_shaped():
    env = bench.rank_env(1, 4, 29555, base={})
    assert env["RANK"] == env["LOCAL_RANK"] == "1"
    assert env["WORLD_SIZE"] == env["LOCAL_WORLD_SIZE"] == "4"
    assert env["MASTER_ADDR"] == "127.0.0.1" and env["MASTER_PORT"] == "29555"
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_gpus_flag_spawns_ranks(monkeypatch, capfd):
    standin = os.path.join(ROOT, "tests", "bench_rank_standin.py")
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(bench, "rank_argv", lambda argv: [sys.executable, "-u", standin] + list(argv))
    with pytest.raises(SystemExit) as e:
        bench.main(["--gpus", "2", "--steps", "3", "--warmup", "1", "--n", "4"])
    assert e.value.code == 0
    out = capfd.readouterr().out.strip().splitlines()
    line = json.loads(out[-1])
    assert line["n_gpus"] == 2
    assert line["steps"] == 3 and line["warmup"] == 1
    assert [r["rank"] for r in line["ranks"]] == [0, 1]
    assert [r["device"] for r in line["ranks"]] == [0, 1]
    assert [r["index_range"] for r in line["ranks"]] == [[0, 4], [4, 8]]
    assert line["verdicts_ok"] is True
    # value = all ranks' units / the max-over-ranks time
    assert line["value"] == pytest.approx(2 * 4 * 3 / (line["ms_per_step"] * 3e-3), rel=1e-2)


def test_gpus_flag_failing_rank_fails_the_run(monkeypatch, capfd):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(bench, "rank_argv",
                        lambda argv: [sys.executable, "-c", "import os,sys; sys.exit(3 if os.environ['RANK']=='1' "
                                                            "else 0)"])
    with pytest.raises(SystemExit) as e:
        bench.main(["--gpus", "2"])
    assert e.value.code == 3


def test_c3_roofline_from_committed_counters():
    """summary.c3_roofline: the built algorithm's INT32
    count per certificate, and -- from profiles/r06_c3_pmc.json, tied by
    sha256 to the committee kernels' sources -- VALU issue and HBM traffic
    against the algorithmic bytes of a 10k-certificate round."""
    r = bench.c3_roofline(10000, 670000, 3336, 1.25)
    assert 3.0e6 < r["alg_int32_ops_per_cert"] < 4.0e6
    assert 0.2 < r["frac"] < 0.5
    assert r["issue_frac"] is not None, r["counters"]
    assert 0.2 < r["issue_frac"] < 0.5
    assert r["traffic_bytes"] > r["alg_bytes"] > 1.5e9
    rec = _recorded()
    sec = dict(rec["secondary"])
    sec["c3_certificate_verify"] = dict(sec["c3_certificate_verify"], roofline=r)
    s = bench.summarize(rec["value"], sec, rec["cpu_baseline"])
    assert s["c3_roofline"]["issue_frac"] == r["issue_frac"]
    assert s["c3_roofline"]["traffic_ratio"] == r["traffic_ratio"]
