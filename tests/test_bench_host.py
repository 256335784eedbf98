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
    assert bench._kernel_tag({"lds_mode": 2, "leaf_kinds": 1, "tex_kinds": 0}) == "render_kernel<false, 2, 1, 0>"
