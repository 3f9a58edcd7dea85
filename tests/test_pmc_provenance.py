"""PMC summaries and their provenance (CPU): tools/pmc_summary.py doubles every kernel's FETCH_SIZE
(gfx950's half count of coalesced reads) and stamps the library hash; bench.py attaches `traffic`
only when that stamp is the library being timed."""
import csv
import hashlib
import importlib.util
import json
import os

import pytest

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _load_summary():
    spec = importlib.util.spec_from_file_location("pmc_summary", os.path.join(HERE, "tools", "pmc_summary.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _write_csv(path, rows):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for r in rows:
            w.writerow(r)


def test_summary_doubles_every_kernels_reads_and_stamps_the_library(tmp_path, monkeypatch):
    mod = _load_summary()
    lib = tmp_path / "lib.so"
    lib.write_bytes(b"library image")
    monkeypatch.setattr(mod, "LIB", str(lib))
    main_k, other_k = "bkd::crc_groups_kernel", "bkd::plan_count_kernel"
    fetch = tmp_path / "fetch" / "x" / "pmc_counter_collection.csv"
    write = tmp_path / "write" / "x" / "pmc_counter_collection.csv"
    # three dispatches of the main kernel (median 1000 kB), one of the other (10 kB), a fill kernel ignored
    _write_csv(str(fetch), [
        {"Dispatch_Id": 1, "Kernel_Name": f"void {main_k}<8, 2>(...)", "Counter_Name": "FETCH_SIZE", "Counter_Value": 900},
        {"Dispatch_Id": 2, "Kernel_Name": f"void {main_k}<8, 2>(...)", "Counter_Name": "FETCH_SIZE", "Counter_Value": 1000},
        {"Dispatch_Id": 3, "Kernel_Name": f"void {main_k}<8, 2>(...)", "Counter_Name": "FETCH_SIZE", "Counter_Value": 1100},
        {"Dispatch_Id": 4, "Kernel_Name": f"{other_k}(...)", "Counter_Name": "FETCH_SIZE", "Counter_Value": 10},
        {"Dispatch_Id": 5, "Kernel_Name": "bkd::fill_splitmix64_kernel(...)", "Counter_Name": "FETCH_SIZE",
         "Counter_Value": 99999},
    ])
    _write_csv(str(write), [
        {"Dispatch_Id": 1, "Kernel_Name": f"void {main_k}<8, 2>(...)", "Counter_Name": "WRITE_SIZE", "Counter_Value": 4},
        {"Dispatch_Id": 4, "Kernel_Name": f"{other_k}(...)", "Counter_Name": "WRITE_SIZE", "Counter_Value": 2},
    ])
    monkeypatch.chdir(tmp_path)
    mod.main(str(tmp_path / "fetch"), str(tmp_path / "write"), "unit", 2_000_000, main_k)
    out = json.load(open(tmp_path / "profiles" / "pmc_unit.json"))
    assert out["dispatches"] == 3
    assert out["hbm_read_bytes_per_launch"] == 2 * 1000 * 1024
    assert out["hbm_write_bytes_per_launch"] == 4 * 1024
    assert out["other_kernels_bytes_per_launch"] == (2 * 10 + 2) * 1024
    assert out["hbm_bytes_per_launch"] == (2000 + 4 + 22) * 1024
    assert out["traffic_over_algorithmic"] == pytest.approx((2000 + 4 + 22) * 1024 / 2_000_000)
    assert out["lib_sha256"] == hashlib.sha256(b"library image").hexdigest()
    assert "bkd::fill_splitmix64_kernel" not in out["other_kernels"]


def test_bench_attaches_traffic_only_for_the_stamped_library(tmp_path, monkeypatch):
    import bench
    os.makedirs(tmp_path / "profiles")
    monkeypatch.setattr(bench, "HERE", str(tmp_path))
    monkeypatch.setattr(bench, "_lib_sha256", lambda: "a" * 64)
    assert bench._pmc_traffic("unit") is None  # no summary
    json.dump({"lib_sha256": "a" * 64, "hbm_bytes_per_launch": 123.0}, open(tmp_path / "profiles" / "pmc_unit.json", "w"))
    assert bench._pmc_traffic("unit") == 123.0
    json.dump({"lib_sha256": "b" * 64, "hbm_bytes_per_launch": 123.0}, open(tmp_path / "profiles" / "pmc_unit.json", "w"))
    assert bench._pmc_traffic("unit") is None  # collected on another build
    json.dump({"hbm_bytes_per_launch": 123.0}, open(tmp_path / "profiles" / "pmc_unit.json", "w"))
    assert bench._pmc_traffic("unit") is None  # unstamped


def test_committed_summaries_are_stamped_and_corrected():
    for cfg in ("uniform4k", "zipf", "verify4k", "package4k"):
        d = json.load(open(os.path.join(HERE, "profiles", f"pmc_{cfg}.json")))
        assert len(d["lib_sha256"]) == 64, cfg
        assert d["correction"].startswith("every kernel"), cfg
        assert 0.99 < d["traffic_over_algorithmic"] < 1.1, cfg
