"""bench.py's host logic without a GPU: the GPU count that makes no HIP call (the parent of the
rank processes must not initialise the GPU), the PMC row reduction the roofline numbers come from,
and the configs leg's workloads (BASELINE.json's configs)."""
import json
import os

import bench


def test_count_gpus_reads_kfd_topology_without_hip(tmp_path, monkeypatch):
    nodes = []
    for i, simd in enumerate([0, 1024, 1024, 1024]):  # a CPU node, then three GPU nodes
        d = tmp_path / str(i)
        d.mkdir()
        (d / "properties").write_text(f"cpu_cores_count 0\nsimd_count {simd}\nmax_waves_per_simd 8\n")
        nodes.append(str(d / "properties"))
    import glob

    monkeypatch.setattr(glob, "glob", lambda pat: nodes if "kfd" in pat else [])
    for v in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    assert bench.count_gpus() == 3
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,2")
    assert bench.count_gpus() == 2


def test_pmc_reduce_takes_the_timed_frame():
    rows = []
    for did, val in [(1, 10.0), (2, 20.0), (3, 30.0), (4, 40.0)]:  # 2 frames x 2 launches
        for part in (0.5, 0.5):  # a dispatch's counter may come as several rows
            rows.append({"Dispatch_Id": str(did), "Counter_Name": "SQ_INSTS_VALU", "Counter_Value": str(val * part),
                         "Start_Timestamp": str(100 * did), "End_Timestamp": str(100 * did + 50)})
    got = bench._pmc_reduce(rows)
    assert got["launches"] == 2 and got["SQ_INSTS_VALU"] == 70.0 and got["dispatch_ns"] == 100
    assert bench._pmc_reduce([]) is None


def test_config_legs_are_the_baseline_configs():
    base = json.load(open(os.path.join(os.path.dirname(bench.__file__), "BASELINE.json")))
    assert len(base["configs"]) == 5
    legs = {(n, w, h, spp) for n, w, h, spp, _ in bench.CONFIG_LEGS}
    assert legs == {("suzanne", 1920, 1080, 512), ("cornell_cube", 800, 800, 1024), ("earth_motion", 3840, 2160, 2048)}
    for (n, w, h, spp, label), cfg in zip(bench.CONFIG_LEGS, (base["configs"][3], base["configs"][2], base["configs"][4])):
        assert f"{w}×{h}" in cfg and f"{spp}spp" in cfg, (label, cfg)
    assert bench._kernel_tag({"lds_mode": 2, "leaf_kinds": 1, "tex_kinds": 0}) == "render_kernel<false, 2, 1, 0, false, false>"


def test_kernel_tag_matches_recorded_rocprof_names():
    """Round 5's configs rooflines were null because the tag lacked the GEN template argument: the tag
    from rtw_world_kernel_name must select exactly the product kernel's rows of a recorded rocprofv3
    summary (profiles/r05/r7i_kernel_stats.csv), not the counting variant's."""
    import csv

    path = os.path.join(os.path.dirname(bench.__file__), "profiles", "r05", "r7i_kernel_stats.csv")
    rows = [{"Kernel_Name": r["Name"]} for r in csv.DictReader(open(path))]
    tag = bench._kernel_tag({"lds_mode": 1, "leaf_kinds": 0, "tex_kinds": 0, "name": "render_kernel<false, 1, 0, 0, false>"})
    got = bench._match_rows(rows, tag)
    assert len(got) == 1 and "render_kernel<false, 1, 0, 0, false>((anonymous namespace)::KArgs)" in got[0]["Kernel_Name"]
    # the round-5 tag (no GEN argument) matched nothing
    assert bench._match_rows(rows, "render_kernel<false, 1, 0, 0>") == []
    # a GEN kernel's name differs from its non-GEN sibling's, a whole-pixel kernel's from its single-sample one's
    gen = bench._kernel_tag({"lds_mode": 1, "leaf_kinds": 3, "tex_kinds": 1, "name": "render_kernel<false, 1, 3, 1, true, true>"})
    assert bench._match_rows([{"Kernel_Name": "void (anonymous namespace)::render_kernel<false, 1, 3, 1, false, true>(KArgs)"},
                              {"Kernel_Name": "void (anonymous namespace)::render_kernel<false, 1, 3, 1, true, false>(KArgs)"}],
                             gen) == []


def test_configs_pmc_notes_unmatched_rows(monkeypatch):
    """A config whose kernel has no PMC rows gets roofline None *and* a pmc_note naming what was seen."""
    rows = [{"Kernel_Name": "void render_kernel<false, 1, 1, 0, false, false>(KArgs)", "Dispatch_Id": "1",
             "Counter_Name": c, "Counter_Value": "1", "Start_Timestamp": "0", "End_Timestamp": "1"}
            for c in bench.VALU_COUNTERS + ("WRITE_SIZE", "FETCH_SIZE")]
    monkeypatch.setattr(bench, "_pmc_rows", lambda child, counters: rows)

    class A:
        max_depth, seed = 50, 1

    legs = [{"workload": "suzanne", "kernel": {"name": "render_kernel<false, 1, 1, 0, false, false>"}, "kernel_ms": 1.0,
             "colour_record_bytes": 12},
            {"workload": "earth_motion", "kernel": {"name": "render_kernel<false, 1, 3, 1, true, true>"}, "kernel_ms": 1.0,
             "colour_record_bytes": 12}]
    bench.configs_pmc(A, legs, 1228.8)
    assert legs[0]["roofline"] is not None and legs[0]["roofline"]["traffic"] is not None
    assert "lane_utilisation" in legs[0]["roofline"] and "pmc_note" not in legs[0]
    assert legs[1]["roofline"] is None and "render_kernel<false, 1, 3, 1, true, true>" in legs[1]["pmc_note"]
