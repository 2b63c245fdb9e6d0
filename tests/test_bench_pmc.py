"""bench.py's PMC lookup for timing scopes that span several kernels (CPU only)."""
import json
import os

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _fake():
    return {
        "_meta": {"passes": 2, "workload": "w", "input_reads": 10},
        "k_pair_coord_tile": {"traffic_bytes_per_launch": 100.0, "launches": 8},
        "k_pair_resid": {"traffic_bytes_per_launch": 10.0, "launches": 8},
        "k_resid_probe_sorted": {"traffic_bytes_per_launch": 7.0, "launches": 2},
        "k_resid_probe": {"traffic_bytes_per_launch": 30.0, "launches": 2},
        "k_sscs_vote_swar": {"traffic_bytes_per_launch": 55.0, "launches": 2},
    }


def test_scope_sums_its_kernels_by_launches():
    d = _fake()
    # 4 launches of the scope per pass: (100 * 8 + 10 * 8) / 2 passes / 4
    assert bench.scope_traffic(d, "k_pair_coord", 4) == (100.0 * 8 + 10.0 * 8) / 2 / 4
    # a scope whose kernels run on only some of its launches (k_resid_*: one launch per pass with
    # residual reads) is weighted by those launches: (7 * 2 + 30 * 2) / 2 passes / 1
    assert bench.scope_traffic(d, "k_pair_resid", 1) == (7.0 * 2 + 30.0 * 2) / 2
    # a single-kernel scope is that kernel
    assert bench.scope_traffic(d, "k_sscs_vote_swar", 1) == 55.0
    assert bench.scope_traffic(d, "k_csn", 1) is None


def test_committed_c4_pmc_gives_the_mate_search_traffic(monkeypatch):
    """The C4 line's dominant scope k_pair_coord (4 launches per step) takes its traffic from the
    committed profiles/pmc_c4_latest.json (the round-3 line carried None)."""
    path = os.path.join(ROOT, "profiles", "pmc_c4_latest.json")
    d = json.load(open(path))
    monkeypatch.setattr(bench, "_WORKLOAD", {"config": "c4", "n": d["_meta"]["input_reads"],
                                             "workload": d["_meta"]["workload"]})
    t, src = bench.pmc_traffic("k_pair_coord", 4.0)
    want = sum(d[k]["traffic_bytes_per_launch"] * d[k]["launches"] for k in ("k_pair_coord_tile", "k_pair_resid")
               if k in d) / d["_meta"]["passes"] / 4.0
    assert t is not None and abs(t - want) < 1.0
    assert "pmc_c4_latest.json" in src
    # another workload's PMC passes are not quoted
    monkeypatch.setattr(bench, "_WORKLOAD", {"config": "c4", "n": 1, "workload": "other"})
    assert bench.pmc_traffic("k_pair_coord", 4.0) == (None, None)


def test_step_traffic_leaves_out_the_upload_kernels():
    d = _fake()
    d["k_table_cols"] = {"traffic_bytes_per_launch": 1000.0, "launches": 1}
    d["k_core_pack"] = {"traffic_bytes_per_launch": 1000.0, "launches": 1}
    want = (100.0 * 8 + 10.0 * 8 + 7.0 * 2 + 30.0 * 2 + 55.0 * 2) / 2
    assert bench.step_traffic(d) == want


def test_sized_reads_sum_request_bytes_per_dispatch(tmp_path):
    """pmc_traffic.py --sized: read bytes = 32/64/128 x the size-resolved request counts, per dispatch,
    and they replace FETCH_SIZE x2 as the kernel's fetch bytes."""
    import subprocess
    import sys
    hdr = '"Dispatch_Id","Kernel_Name","Counter_Name","Counter_Value"\n'
    (tmp_path / "f.csv").write_text(hdr + '1,"k_a(int)","FETCH_SIZE",1.0\n2,"k_a(int)","FETCH_SIZE",3.0\n'
                                    '3,"k_b(int)","FETCH_SIZE",10.0\n')
    (tmp_path / "w.csv").write_text(hdr + '1,"k_a(int)","WRITE_SIZE",0.5\n2,"k_a(int)","WRITE_SIZE",0.5\n'
                                    '3,"k_b(int)","WRITE_SIZE",0.0\n')
    (tmp_path / "s.csv").write_text(hdr + '1,"k_a(int)","TCC_EA0_RDREQ_32B_sum",2\n1,"k_a(int)","TCC_EA0_RDREQ_64B_sum",1\n'
                                    '1,"k_a(int)","TCC_EA0_RDREQ_128B_sum",4\n2,"k_a(int)","TCC_EA0_RDREQ_128B_sum",8\n'
                                    '3,"k_b(int)","TCC_EA0_RDREQ_64B_sum",100\n')
    out = tmp_path / "o.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "pmc_traffic.py"), str(tmp_path / "f.csv"),
                    str(tmp_path / "w.csv"), str(out), "2", "--sized", str(tmp_path / "s.csv")], check=True,
                   capture_output=True)
    d = json.load(open(out))
    assert d["k_a"]["raw_sized_read_bytes"] == [2 * 32 + 64 + 4 * 128, 8 * 128]
    assert d["k_a"]["fetch_bytes_per_launch"] == (640 + 1024) / 2
    assert d["k_a"]["fetch_x2_bytes_per_launch"] == 2.0 * 1024 * (1 + 3) / 2
    assert d["k_a"]["traffic_bytes_per_launch"] == (640 + 1024) / 2 + 512
    assert d["k_b"]["traffic_bytes_per_launch"] == 6400
    assert d["_meta"] == {"passes": 2, "reads": "sized requests"}


def test_calibration_summary_ratios(tmp_path):
    """scripts/pmc_calib_summary.py: FETCH_SIZE x2, the size-resolved reads and WRITE_SIZE over the
    calibration kernels' known byte counts (the second round of seven dispatches is read)."""
    import subprocess
    import sys
    order = ["k_rd16", "k_rd8", "k_rd4", "k_gat16", "k_gat4", "k_wr16", "k_wr4"]
    known = [2 ** 30] * 3 + [2 ** 24 * 16, 2 ** 24 * 4] + [2 ** 30] * 2
    hdr = '"Dispatch_Id","Kernel_Name","Counter_Name","Counter_Value"\n'
    f, w, s = [hdr], [hdr], [hdr]
    for rnd in range(2):
        for i, (k, b) in enumerate(zip(order, known)):
            d = 1 + rnd * 7 + i
            rd = 0 if k.startswith("k_wr") else (b * 8 if k == "k_gat16" else b * 32 if k == "k_gat4" else b)
            wr = b if k.startswith("k_wr") else 0
            f.append('%d,"void %s<x>(int)","FETCH_SIZE",%f\n' % (d, k, rd / 2 / 1024.0))
            w.append('%d,"void %s<x>(int)","WRITE_SIZE",%f\n' % (d, k, wr / 1024.0))
            s.append('%d,"void %s<x>(int)","TCC_EA0_RDREQ_128B_sum",%d\n' % (d, k, rd // 128))
    for name, rows in (("f", f), ("w", w), ("s", s)):
        (tmp_path / (name + ".csv")).write_text("".join(rows))
    out = tmp_path / "cal.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "pmc_calib_summary.py"), str(tmp_path / "f.csv"),
                    str(tmp_path / "w.csv"), str(tmp_path / "s.csv"), str(out)], check=True, capture_output=True)
    d = json.load(open(out))
    assert d["k_rd4"]["fetch_x2_over_known"] == 1.0 and d["k_rd4"]["sized_reads_over_known"] == 1.0
    assert d["k_gat4"]["sized_reads_over_known"] == 32.0 and d["k_gat16"]["fetch_x2_over_known"] == 8.0
    assert d["k_wr16"]["write_over_known"] == 1.0 and d["k_wr16"]["fetch_x2_over_known"] == 0.0
