"""bench.py's compact line on a synthetic record (CPU): the tile summary's
worst-run and harness-stall fields, and that a malformed record costs only
its own summary, never the line."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def _run(p50, p99, late=0.0, gap=0.0):
    return {"p50_us": p50, "p99_us": p99, "p99_over_p50": p99 / p50, "frags_per_s": 1.0, "offered_frags_per_s": 1.0,
            "txns_per_s": 1.0, "stalls_us": {"producer_late_max": late, "tile_pass_max": 10.0, "consumer_gap_max": gap}}


def _load(runs):
    worst, clean, nst = bench.worst_of(runs)
    med = sorted(runs, key=lambda x: x["p50_us"])[1]
    return {"p50_us": med["p50_us"], "worst_p99_us": worst["p99_us"], "worst_p99_over_p50": worst["p99_over_p50"],
            "harness_stalled_runs": nst, "worst_p99_over_p50_unstalled": clean, "runs": runs}


def _tile():
    ok = [_run(1000, 1100), _run(1010, 1120), _run(990, 1090)]
    stalled = [_run(1000, 1100), _run(1000, 9000, late=5000.0), _run(1005, 1150)]
    rr_ok = {"saturated_frags_per_s": 5e7, "saturated_steady_frags_per_s": 5.2e7, "check_mismatches": 0,
             "roofline": {"frac": 0.3, "frac_steady": 0.31}, "at_50%": _load(ok), "at_80%": _load(stalled)}
    rr_ok["p99_within_2_5x_p50"] = False
    rr_ok["p99_within_2_5x_p50_unstalled"] = True
    tx = {"batch_max": 4096, "saturated_txns_per_s": 8e6, "saturated_verifies_per_s": 5e7,
          "saturated_steady_verifies_per_s": 5.1e7, "check_mismatches": 0, "at_50%": _load(ok), "at_80%": _load(ok),
          "p99_within_2_5x_p50": True, "p99_within_2_5x_p50_unstalled": True}
    return {"rows": [{"batch_max": 4096, "zero_copy": rr_ok}], "all_checks_pass": True,
            "every_row_p99_within_2_5x_p50": False, "every_row_p99_within_2_5x_p50_unstalled": True,
            "every_row_p50_nondecreasing_with_load": True, "frags_per_run": 1 << 25,
            "txn_framing": {"rows": [tx]}}


def _out(tile):
    return {"metric": "m", "value": 1.0, "unit": "verifies/s", "n_gpus": 1, "steps": 1, "warmup": 1, "ms_per_step": 1.0,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int64", "data": "synthetic",
            "config": {"workload": "w"}, "stream_tile": tile}


def test_worst_of_separates_harness_stalls():
    runs = [_run(1000, 1100), _run(1000, 9000, late=5000.0), _run(1000, 1200, gap=3000.0)]
    worst, clean, nst = bench.worst_of(runs)
    assert worst["p99_us"] == 9000 and nst == 2 and abs(clean - 1.1) < 1e-9
    worst, clean, nst = bench.worst_of([_run(1000, 9000, late=5000.0)] * 3)
    assert clean is None and nst == 3


def test_compact_line_tile_summary_fields():
    line = json.loads(bench.compact_line(_out(_tile()), "d.json"))
    st = line["stream_tile"]
    assert st["every_row_worst_p99_within_2_5x_p50"] is False
    assert st["every_row_worst_p99_within_2_5x_p50_runs_without_harness_stalls"] is True
    row = st["rows"][0]
    assert row["worst_x_80"] == 9.0 and row["stalled_runs_80"] == 1 and row["worst_x_unstalled_80"] == 1.14
    assert "stalled_runs_50" not in row
    assert st["txn_framing"][0]["worst_x_50"] == 1.11


def test_malformed_tile_record_costs_only_its_summary():
    tile = _tile()
    del tile["rows"][0]["zero_copy"]["at_80%"]
    line = json.loads(bench.compact_line(_out(tile), "d.json"))
    assert line["value"] == 1.0 and "summary_error" in line["stream_tile"]


def test_unstalled_check_fails_when_every_run_stalled():
    """A load with no stall-free run cannot pass the harness-stall view of the tail check."""
    import bench
    ok = {"worst_p99_over_p50_unstalled": 1.2}
    assert bench.unstalled_ok([ok, ok])
    assert not bench.unstalled_ok([ok, {"worst_p99_over_p50_unstalled": None}])
    assert not bench.unstalled_ok([ok, {"worst_p99_over_p50_unstalled": 2.6}])


def test_roofline_from_rocprof_and_held_clock(tmp_path, monkeypatch):
    """The line's profiler-timed DSM fraction and held clock: the committed rocprofv3 averages of the stage's
    launches, GRBM_GUI_ACTIVE / 8 XCDs over k_dsmp's duration; the traffic raw and 2x-corrected."""
    import json
    import numpy as np
    import bench
    csv = tmp_path / "r99_rocprof_kernel_stats.csv"
    csv.write_text('"Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs","StdDev"\n'
                   '"k_dsmp(unsigned int)",2,26000000,13000000.0,90,1,1,0\n'
                   '"k_ai(unsigned int)",2,1000000,500000.0,5,1,1,0\n'
                   '"k_fin(unsigned int)",2,200000,100000.0,1,1,1,0\n')
    pmc = tmp_path / "r99_pmc_latest.json"
    pmc.write_text(json.dumps({"_sigs_per_launch": 1 << 20, "k_dsmp": {
        "counters": {"GRBM_GUI_ACTIVE": 8 * 2.2e9 * 13e-3},
        "derived": {"hbm_bytes_per_launch": 2.0e10, "fetch_kb_raw": 9.0e6, "write_kb_raw": 1.0e6}},
        **{k: {"counters": {}, "derived": {"hbm_bytes_per_launch": 0.0, "fetch_kb_raw": 0.0, "write_kb_raw": 0.0}}
           for k in ("k_ai", "k_fin")}}))
    monkeypatch.setattr(bench, "rocprof_stats_path", lambda: str(csv))
    monkeypatch.setattr(bench, "pmc_summary_path", lambda: str(pmc))
    assert abs(bench.rocprof_stage_ms(["k_ai", "k_dsmp", "k_fin"])[0] - 13.6) < 1e-9
    assert abs(bench.held_clock_ghz("k_dsmp") - 2.2) < 1e-9
    n = 1 << 20
    st = np.zeros((3, n), np.uint32)
    st[0] = 250
    st[1] = 42
    st[2] = 43
    r = bench.dsm_roofline(st, 13.0, n, kernel="k_ai+k_dsmp+k_fin")
    assert abs(r["frac_rocprof"] / r["frac"] - 13.0 / 13.6) < 1e-9
    assert abs(r["frac_at_held_clock"] / r["frac"] - 2.4 / 2.2) < 1e-9
    assert r["traffic"] == 2.0e10 and r["traffic_raw"] == 1.0e7 * 1024


def test_stalled_runs_are_topped_up_and_left_out_of_the_median():
    """A producer stall on two of three paced runs: more runs until three are
    stall-free (at most TOPUP_MAX), the p50 is their median, and every run --
    stalled and extra ones too -- stays in the all-runs tail check."""
    rs = [_run(700, 800), _run(150000, 320000, late=300000.0), _run(152000, 330000, late=310000.0)]
    fresh = iter([_run(710, 790), _run(690, 770), _run(720, 800)])
    extra = bench.top_up(rs, lambda: next(fresh))
    assert extra == 2 and len(rs) == 5
    assert bench.p50_run(rs)["p50_us"] == 700                      # median of 700, 710, 690
    worst, clean, nst = bench.worst_of(rs)
    assert nst == 2 and worst["p99_us"] == 330000 and clean < 1.2  # the stalled runs still set the all-runs tail
    # at most TOPUP_MAX extra runs, then the median over whatever is clean
    rs2 = [_run(1000, 1100, late=5000.0)] * 3
    stalled = iter([_run(1000, 1100, late=5000.0)] * bench.TOPUP_MAX)
    assert bench.top_up(rs2, lambda: next(stalled)) == bench.TOPUP_MAX
    assert bench.p50_run(rs2)["p50_us"] == 1000                    # none clean: the median of all
    # three clean runs: nothing extra
    rs3 = [_run(600, 700), _run(610, 700), _run(620, 700)]
    assert bench.top_up(rs3, lambda: None) == 0 and bench.p50_run(rs3)["p50_us"] == 610
