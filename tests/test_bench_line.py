"""bench.py's stdout line: the driver keeps only the tail of the run's
output, so the one JSON line must hold the headline in <= 4 KB and parse on its own; the
legs go to the --legs-out file and stderr.  CPU only: compact_line() is fed the full result
of a real round-3 C4 run (profiles/r03/bench_c4_r03z.json, every leg present, 46 KB) and an
inflated synthetic one."""
import copy
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

FULL = os.path.join(ROOT, "profiles", "r03", "bench_c4_r03z.json")
REQUIRED = ("metric", "value", "unit", "n_gpus", "ranks_seen", "steps", "warmup", "ms_per_step",
            "dtype", "config", "roofline", "cpu_baseline", "p50_us", "locate")


def _bench():
    import bench
    return bench


def _full():
    with open(FULL) as f:
        return json.loads(f.read().strip().splitlines()[-1])


def test_full_result_compacts_under_4k():
    b = _bench()
    res = _full()
    assert len(json.dumps(res)) > 40000 and len(res["legs"]) > 20  # the round-3 line
    line = b.compact_line(res, "gpurun_out/bench_full_n1_x.json")
    assert len(line.encode()) <= 4096
    got = json.loads(line)
    for k in REQUIRED:
        assert k in got, k
    assert got["value"] == float("%.6g" % res["value"])
    assert got["ms_per_step"] == res["ms_per_step"]
    rf = got["roofline"]
    for k in ("frac", "achieved", "alg_bytes_per_launch", "traffic", "kernel_ms_mean",
              "frac_of_random_access_ceiling"):
        assert k in rf, k
    assert abs(rf["frac"] - res["roofline"]["frac"]) <= 1e-3 * res["roofline"]["frac"]
    cb = got["cpu_baseline"]
    for k in ("value", "kind", "cores_used", "host_cores", "matches_gpu"):
        assert k in cb, k
    assert set(got["locate"]) == {"patterns_per_s", "frac"}
    assert "legs" not in got and got["legs_file"].endswith(".json")


def test_inflated_result_still_fits():
    # every optional field at its largest: long leg-error list, long strings everywhere
    b = _bench()
    res = copy.deepcopy(_full())
    res["leg_errors"] = {"leg%02d" % i: "RuntimeError: " + "x" * 500 for i in range(40)}
    res["config"]["engine"] = "e" * 3000
    res["config"]["workload"] = "w" * 300
    res["cpu_baseline"]["sample"] = "s" * 5000
    res["gather_verified"] = True
    line = b.compact_line(res, "gpurun_out/" + "f" * 300 + ".json")
    assert len(line.encode()) <= 4096
    got = json.loads(line)
    assert got["value"] and got["roofline"]["frac"] and got["gather_verified"] is True


def test_only_mode_keeps_the_leg_object():
    b = _bench()
    res = {"only": "count", "workload_key": "k", "count": {"frac": 0.2}, "legs": {}}
    assert json.loads(b.compact_line(res)) == res
