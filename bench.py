"""Benchmark: Msamples/s of the render hot path on MI355X (BASELINE.json metric).

Workload (BASELINE configs[1]): the reference's demo world final_scene1 (demo_worlds.rs:395-463,
scene RNG seeded as main.rs:24), 1920x1080, 512 samples per pixel, max_depth 50.  One step =
one full frame: every rank renders its interleaved 8x8 tiles (rtw_render_device), then one RCCL
all-gather + untile assembles the image on rank 0 (N > 1).  `value` = W*H*spp*steps / max-over-
ranks wall time of the timed region (strong scaling: the frame is fixed, N GPUs share it).

Extra fields:
  roofline      the render kernel against its real bound, VALU instruction issue: wave-level VALU
                instructions of one timed frame (rocprofv3 --pmc SQ_INSTS_VALU pass of this same
                benchmark) / the frame's render-launch time measured live with HIP events on the
                launch stream, against 256 CUs x 4 SIMDs x 2.4 GHz / 2 cycles per wave64 VALU
                instruction (MI355X_MICROARCH.md).  Also: VALU lane utilisation, effective clock,
                the measured HBM `traffic` (and its rate against the HBM peak), and `records`: the
                SURVEY §8(d) record bytes of the traversal the timed kernel runs (its counting
                variant: the SAH walk on SAH worlds) / kernel time, against the LDS peak -- the
                node and primitive records are served from LDS (and L2), not HBM.
  thread_count  the reference's own call shape: render(.., thread_count = available_parallelism,
                ..) as main.rs:19 calls it (the plane split of rendering.rs:222-252 on the device),
                N = 1 only, against the headline's thread_count 1.
  cpu_baseline  the C restatement of the reference render loop (oracle/) in the reference's own
                scheme (ref mode: per-thread xoroshiro streams, split_work_tasks + merge_planes,
                rendering.rs:121-252) on all of this host's CPUs (nproc), N = 1 only: the
                configured frame at a reduced spp (render time is linear in spp), plus config C1
                (400x225x64) in full.
  first_frame_ms  one cold drop-in rtw_render of the configured frame (upload, tuning frame in
                chunk-major order, copy back): what a single reference-style render call costs.
  configs       N = 1 only: the other BASELINE configs on this GPU -- suzanne 1080p512 (C4),
                cornell_cube 800x800x1024 (C3), earth_motion 3840x2160x2048 (C5) -- each 1 warm-up +
                --configs-steps timed frames (HIP events on the launch stream beside the wall clock),
                with its own VALU-issue roofline, lane utilisation and HBM traffic from two PMC runs.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       (--gpus N > 1 without torchrun: starts N rank processes itself, before any GPU call)
       torchrun --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
LDS_BYTES_PER_CLK = 256  # per CU: the LDS array is 64 dwords wide per clock (MI355X_MICROARCH.md §LDS)
CLOCK_GHZ = 2.4        # MI355X peak engine clock (MI355X_MICROARCH.md)
SIMDS_PER_CU = 4       # SIMD-32 units per CU; a wave64 VALU instruction issues over 2 cycles
VALU_COUNTERS = ("SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU", "SQ_THREAD_CYCLES_VALU", "SQ_WAVE_CYCLES",
                 "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "GRBM_GUI_ACTIVE")


def alg_bytes(stats: dict, pixels: int) -> int:
    """packed-record bytes the traversal touches + the framebuffer write."""
    return (
        32 * stats["node_visits"]
        + 16 * stats["sphere_tests"]
        + 20 * stats["rect_tests"]
        + 24 * stats["box_tests"]
        + 36 * stats["triangle_tests"]
        + 64 * stats["triangle_hits"]
        + 16 * stats["material_reads"]
        + 3 * stats["texel_reads"]
        + 12 * pixels
    )


def _pmc_rows(child_args: list, counters) -> list | None:
    """The render_kernel rows of one `rocprofv3 --pmc <counters>` run of this benchmark with
    `child_args`.  None if rocprofv3 is unavailable or the pass fails."""
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile

    if not shutil.which("rocprofv3"):
        return None
    child = [sys.executable, os.path.abspath(__file__)] + child_args
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as d:
        cmd = ["rocprofv3", "--pmc", *counters, "-d", d, "-o", "pmc", "--output-format", "csv", "--"] + child
        try:
            subprocess.run(cmd, check=True, capture_output=True, timeout=600, cwd=ROOT)
        except (subprocess.SubprocessError, OSError):
            return None
        rows = []
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            rows += [r for r in csv.DictReader(open(f)) if "render_kernel" in r["Kernel_Name"]]
    return rows or None


def _pmc_reduce(rows) -> dict | None:
    """Per counter, the sum over the timed frame's render_kernel dispatches among `rows` (a warm-up
    and a timed frame with the same launch count: the last half of the dispatches; counters of one
    dispatch may come as several rows), plus that frame's dispatch time from the trace timestamps."""
    if not rows:
        return None
    ids = sorted({int(r["Dispatch_Id"]) for r in rows})
    timed = set(ids[len(ids) // 2:])  # two frames with the same launch count: the second is timed
    got: dict = {"launches": len(timed)}
    span = {}
    for r in rows:
        if int(r["Dispatch_Id"]) not in timed:
            continue
        got[r["Counter_Name"]] = got.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        span[r["Dispatch_Id"]] = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
    got["dispatch_ns"] = sum(e - s for s, e in span.values())
    return got


def _pmc_pass(args, counters) -> dict | None:
    """One PMC run of this benchmark's headline workload (1 warm-up + 1 timed frame, no extra legs)."""
    child = ["--scene", args.scene, "--width", str(args.width), "--height", str(args.height), "--spp", str(args.spp),
             "--max-depth", str(args.max_depth), "--seed", str(args.seed), "--steps", "1", "--warmup", "1",
             "--no-cpu-baseline", "--no-stats", "--no-pmc", "--no-first-frame", "--no-thread-count", "--no-configs"]
    return _pmc_reduce(_pmc_rows(child, counters))


def pmc_traffic(args) -> dict | None:
    """HBM bytes of the timed frame's render launches (MI355X_MICROARCH.md HBM section): separate
    FETCH_SIZE and WRITE_SIZE passes; both count KiB, and gfx950 reports half the bytes of wide
    coalesced reads in FETCH_SIZE, so it is doubled."""
    f = _pmc_pass(args, ["FETCH_SIZE"])
    w = _pmc_pass(args, ["WRITE_SIZE"]) if f else None
    if not f or not w or "FETCH_SIZE" not in f or "WRITE_SIZE" not in w:
        return None
    fetch = f["FETCH_SIZE"] * 1024.0 * 2.0
    write = w["WRITE_SIZE"] * 1024.0
    return {"fetch_bytes": fetch, "write_bytes": write, "bytes": fetch + write, "launches": f["launches"]}


def pmc_valu(args) -> dict | None:
    """VALU issue counters of the timed frame (one pass: 6 SQ + 1 GRBM counters)."""
    c = _pmc_pass(args, list(VALU_COUNTERS))
    if not c or any(k not in c for k in VALU_COUNTERS):
        return None
    return c


# The other BASELINE configs, on one GPU (the headline is configs[1], final_scene1 1080p512)
CONFIG_LEGS = (
    ("suzanne", 1920, 1080, 512, "C4 (BASELINE configs[3], suzanne.obj + BVH, 1080p512) on one GPU"),
    ("cornell_cube", 800, 800, 1024, "C3 (BASELINE configs[2], Cornell box + cube.obj, 800x800x1024)"),
    ("earth_motion", 3840, 2160, 2048, "C5 (BASELINE configs[4], earthmap + motion blur, 4Kx2048) on one GPU"),
)


def _kernel_tag(v: dict) -> str:
    """The render kernel's name fragment in rocprofv3's Kernel_Name for a kernel_variant() dict: the
    exact template name rtw_world_kernel_name reports (render_kernel<STATS, LDS, LK, TX, GEN, WP>), rebuilt
    from the fields for a dict without it (GEN and WP then taken as false; a wrong guess matches no row and
    configs_pmc says so)."""
    if v.get("name"):
        return v["name"]
    return f"render_kernel<false, {v['lds_mode']}, {v['leaf_kinds']}, {v['tex_kinds']}, false, false>"


def _match_rows(rows, tag: str) -> list:
    """The rows of `rows` whose Kernel_Name holds the template name `tag` exactly (the counting variant's
    render_kernel<true, ...> and other variants excluded)."""
    return [x for x in rows or [] if tag in x["Kernel_Name"]]


def render_configs(args, local_rank: int, steps: int, warmup: int, barrier) -> list:
    """`warmup` untimed + `steps` timed frames of each CONFIG_LEGS workload on this GPU (each world
    released before the next: the C5 frame's colour buffer takes up to 64 GiB)."""
    import gc

    import torch

    import raytracinginaweekend_amd as R
    from raytracinginaweekend_amd.distributed import FrameRenderer, FrameSpec

    out = []
    for name, w, h, spp, label in CONFIG_LEGS:
        world = R.demo_world(name)
        fr = FrameRenderer(world, FrameSpec(R.Size2i(w, h), spp, args.max_depth, args.seed), 0, 1, local_rank)
        for _ in range(warmup):
            fr.launch()
        barrier()
        rec = {"workload": f"{name} {w}x{h}x{spp}spp max_depth {args.max_depth}", "baseline_config": label}
        if steps > 0:
            st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t = time.perf_counter()
            st.record()
            for _ in range(steps):
                fr.launch()
            en.record()
            barrier()
            dt = (time.perf_counter() - t) / steps
            rec.update({"value": round(w * h * spp / dt / 1e6, 3), "unit": "Msamples/sec", "steps": steps,
                        "warmup": warmup, "ms_per_step": round(dt * 1e3, 3),
                        "kernel_ms": round(st.elapsed_time(en) / steps, 3)})
        lf = fr.dworld.last_frame()
        rec.update({"trace_min": lf["trace_min"],
                    "kernel": fr.dworld.kernel_variant(), "launches_per_frame": lf["launches"],
                    "work_items": "whole pixels" if lf["whole_pixel"] else "samples",
                    # the per-sample colour records the frame writes (whole-pixel items: none, the
                    # pixels themselves, 12 B each)
                    "colour_record_bytes": (w * h * 12) if lf["whole_pixel"] else (w * h * spp * 12)})
        out.append(rec)
        fr.dworld.release()
        del fr, world
        gc.collect()
    return out


def configs_pmc(args, legs: list, peak_ginstr: float) -> None:
    """PMC passes over all CONFIG_LEGS at once (a child renders 1 warm-up + 1 timed frame of each):
    the VALU issue counters with WRITE_SIZE, then FETCH_SIZE (x2, gfx950) in a second run; rows are
    told apart by the configs' kernel variants (distinct names required)."""
    child = ["--configs-child", "--max-depth", str(args.max_depth), "--seed", str(args.seed)]
    tags = [_kernel_tag(r["kernel"]) for r in legs]
    if len(set(tags)) != len(tags):
        for r in legs:
            r["roofline"] = None
            r["pmc_note"] = "configs share a kernel variant: their PMC rows cannot be told apart"
        return
    a = _pmc_rows(child, list(VALU_COUNTERS) + ["WRITE_SIZE"])
    b = _pmc_rows(child, ["FETCH_SIZE"]) if a else None
    names = sorted({x["Kernel_Name"] for x in (a or []) + (b or [])})
    for r, tag in zip(legs, tags):
        v = _pmc_reduce(_match_rows(a, tag))
        f = _pmc_reduce(_match_rows(b, tag))
        if not v or any(k not in v for k in VALU_COUNTERS) or not r.get("kernel_ms"):
            # never a silent null: say which rows were looked for and what the passes saw
            r["roofline"] = None
            r["pmc_note"] = (f"no PMC rows for {tag!r}" if a else "the VALU counter pass failed or rocprofv3 is "
                             "absent") + (f"; render kernels in the passes: {names}" if names else "")
            print(f"bench.py: configs leg {r['workload']}: {r['pmc_note']}", file=sys.stderr)
            continue
        k_s = r["kernel_ms"] * 1e-3
        achieved = v["SQ_INSTS_VALU"] / k_s / 1e9
        rl = {"bound": "valu_issue", "achieved": round(achieved, 1), "peak": round(peak_ginstr, 1),
              "unit": "G VALU wave-instr/s", "frac": round(achieved / peak_ginstr, 4),
              "insts_per_frame": int(v["SQ_INSTS_VALU"]),
              "lane_utilisation": round(v["SQ_THREAD_CYCLES_VALU"] / (64.0 * v["SQ_ACTIVE_INST_VALU"]), 4),
              "wait_any_frac": round(v["SQ_WAIT_ANY"] / v["SQ_WAVE_CYCLES"], 4),
              "pmc_launches_per_frame": v["launches"]}
        write = v.get("WRITE_SIZE", 0.0) * 1024.0
        if f and "FETCH_SIZE" in f:
            fetch = f["FETCH_SIZE"] * 1024.0 * 2.0
            rl["traffic"] = round(fetch + write)
            rl["hbm_GBps"] = round((fetch + write) / k_s / 1e9, 1)
            rl["hbm_frac"] = round((fetch + write) / k_s / 1e9 / HBM_PEAK_GBS, 5)
            rl["traffic_detail"] = {"fetch_bytes_x2": round(fetch), "write_bytes": round(write),
                                    "colour_record_bytes": r["colour_record_bytes"]}
        rl["source"] = ("rocprofv3 --pmc " + " ".join(VALU_COUNTERS) + " WRITE_SIZE, then FETCH_SIZE, on a child "
                        "rendering 1 warm-up + 1 timed frame of each config; achieved = SQ_INSTS_VALU / this leg's "
                        "kernel_ms")
        r["roofline"] = rl


def _cpu_info() -> dict:
    """nproc, the CPUs this process may run on, the cgroup CPU quota and the CPU model."""
    info = {"nproc": os.cpu_count() or 1}
    try:
        info["affinity"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        info["affinity"] = info["nproc"]
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        info["cgroup_quota_cpus"] = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        info["cgroup_quota_cpus"] = None
    info["model"] = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                info["model"] = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return info


def cpu_baseline(args) -> dict:
    """The reference algorithm in its own RNG/thread scheme (oracle ref mode, test infrastructure)
    on every CPU this process may use: the configured frame at a reduced spp (whole image, the
    reference's sample split over `threads` planes; time is linear in spp), and config C1
    (final_scene1 400x225x64, max_depth 50) in full."""
    import numpy as np

    import raytracinginaweekend_amd as R
    from oracle import pyoracle as O

    info = _cpu_info()
    usable = info["affinity"]
    if info["cgroup_quota_cpus"]:  # more threads than the quota only time-slice the same CPU time
        usable = min(usable, max(1, int(info["cgroup_quota_cpus"] + 0.5)))
    threads = args.cpu_threads or min(512, usable)

    def run(world, w, h, spp):
        out = np.zeros((w * h, 3), np.float32)
        p = R.render_params(R.Size2i(w, h), spp, args.max_depth, seed=3)
        t = time.perf_counter()
        O.render(world, p, O.RNG_REF, threads, out=out)
        return time.perf_counter() - t

    c1_dt = run(R.demo_world("final_scene1"), 400, 225, 64)  # C1 in full; also calibrates the spp below
    c1_rate = 400 * 225 * 64 / c1_dt
    spp = int(args.cpu_seconds * c1_rate / (args.width * args.height))
    spp = max(min(threads, args.spp), min(args.spp, max(1, spp)))  # every thread gets a plane
    dt = run(R.demo_world(args.scene), args.width, args.height, spp)
    rate = args.width * args.height * spp / dt / 1e6
    return {
        "value": round(rate, 4),
        "unit": "Msamples/sec",
        "cores": threads,
        "cores_note": "threads = the CPUs this process can use (affinity, capped by the cgroup CPU quota)",
        "kind": "port",
        "sample": f"{args.scene} {args.width}x{args.height} at {spp} spp (of {args.spp}; time is linear in spp), "
        f"max_depth {args.max_depth}, {dt:.1f} s; the reference's scheme (oracle ref mode: per-thread xoroshiro "
        f"streams, split_work_tasks over {threads} threads, merge_planes)",
        "nproc": info["nproc"],
        "affinity_cpus": info["affinity"],
        "cgroup_quota_cpus": info["cgroup_quota_cpus"],
        "cpu_model": info["model"],
        "c1": {"workload": "final_scene1 400x225x64spp max_depth 50 (BASELINE configs[0]), full frame",
               "seconds": round(c1_dt, 3), "Msamples_per_s": round(400 * 225 * 64 / c1_dt / 1e6, 4)},
    }


def count_gpus() -> int:
    """GPUs this process could use, counted without any HIP call (the parent of the rank processes
    must not initialise the GPU): the KFD topology's GPU nodes (simd_count > 0), narrowed by
    ROCR_VISIBLE_DEVICES / HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES when set."""
    import glob

    n = 0
    for f in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties"):
        try:
            for line in open(f):
                k, _, v = line.partition(" ")
                if k == "simd_count" and int(v) > 0:
                    n += 1
                    break
        except (OSError, ValueError):
            continue
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip()]))
    return n


def launch_ranks(args) -> int:
    """--gpus N > 1 without a launcher: one rank process per GPU, started before this process
    touches the GPU (count_gpus makes no HIP call); rank 0 prints the line."""
    import socket
    import subprocess

    n = count_gpus()
    if n < args.gpus:
        print(f"bench.py: --gpus {args.gpus} needs {args.gpus} GPUs, this node has {n}", file=sys.stderr)
        return 3
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus), LOCAL_WORLD_SIZE=str(args.gpus),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in live:  # a failed rank leaves the others waiting in a collective
                    q.terminate()
        time.sleep(0.2)
    return rc


def inproc_bench(args) -> int:
    """--inproc: the N GPUs from one process through the C ABI's multi-device path (rtw_multi_create /
    rtw_multi_render: one host thread and stream per device, the tile buffers peer-copied to GPU 0 over
    xGMI, untiled there), the way a single caller of rendering::render (main.rs:43-50) takes the node.
    A timed frame is the whole rtw_multi_render call: every partition's render, the copies, the untile."""
    devices = [int(x) for x in args.inproc_devices.split(",")] if args.inproc_devices else list(range(args.gpus))
    if not args.inproc_devices and count_gpus() < args.gpus:
        print(f"bench.py: --gpus {args.gpus} needs {args.gpus} GPUs", file=sys.stderr)
        return 3
    import torch

    import raytracinginaweekend_amd as R

    world = R.demo_world(args.scene)
    size = R.Size2i(args.width, args.height)
    p = R.render_params(size, args.spp, args.max_depth, seed=args.seed, part=(0, 0))
    mw = R.MultiDeviceWorld(world, devices)
    img = torch.empty(size.count() * 3, dtype=torch.float32, device=f"cuda:{devices[0]}")
    for _ in range(args.warmup):
        mw.render_into(p, img.data_ptr())
    t0 = time.perf_counter()
    for _ in range(args.steps):
        mw.render_into(p, img.data_ptr())
    elapsed = time.perf_counter() - t0
    if args.save:
        from raytracinginaweekend_amd.image_io import save_image

        save_image(args.save, img.cpu().numpy().reshape(-1, 3), args.width, args.height)
    value = args.width * args.height * args.spp * args.steps / elapsed / 1e6
    print(json.dumps({
        "metric": "Msamples/sec at 1920x1080x512spp; achieved HBM GB/s vs peak",
        "value": round(value, 3), "unit": "Msamples/sec", "n_gpus": len(set(devices)), "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f32",
        "data": f"synthetic: the reference's demo world {args.scene}, built as its builder does from fixed seeds",
        "config": {"workload": f"{args.scene} {args.width}x{args.height}x{args.spp}spp max_depth {args.max_depth}",
                   "parallelism": f"in-process: {len(devices)} partitions on devices {devices} (rtw_multi_render: "
                                  "one host thread per partition, peer copies to the first device, untile)"},
    }), flush=True)
    mw.release()
    return 0


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scene", default="final_scene1")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=512)
    ap.add_argument("--tile", default="8x8", help="partition tile WxH (the headline frame's; a wave takes one tile's pixels)")
    ap.add_argument("--max-depth", type=int, default=50)
    ap.add_argument("--seed", type=int, default=0x5EED)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-stats", action="store_true")
    ap.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 PMC passes (VALU counters, HBM traffic)")
    ap.add_argument("--no-traffic", action="store_true", help="skip only the HBM traffic passes")
    ap.add_argument("--no-first-frame", action="store_true")
    ap.add_argument("--no-thread-count", action="store_true", help="skip the thread_count = available_parallelism leg")
    ap.add_argument("--no-configs", action="store_true", help="skip the other BASELINE configs (C3, C4, C5 on one GPU)")
    ap.add_argument("--configs-steps", type=int, default=3, help="timed frames per config of that leg")
    ap.add_argument("--configs-child", action="store_true", help=argparse.SUPPRESS)  # the configs' PMC passes
    ap.add_argument("--thread-count-leg", type=int, default=0, help="thread_count of that leg (0: available_parallelism)")
    ap.add_argument("--stats-spp", type=int, default=128, help="spp of the counting render (scaled to --spp)")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--save", default="", help="write the rank-0 image (.ppm/.png)")
    ap.add_argument("--inproc", action="store_true",
                    help="one process drives the --gpus devices through rtw_multi_render (no ranks, no RCCL)")
    ap.add_argument("--inproc-devices", default="", help="with --inproc: an explicit device list, e.g. 0,0,0")
    args = ap.parse_args()

    if args.inproc:
        return inproc_bench(args)

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_ranks(args)
    world_size = int(os.environ.get("WORLD_SIZE", "1"))
    if world_size != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but the launcher started {world_size} ranks", file=sys.stderr)
        return 2

    import torch  # first: librtw.so then binds to the same libamdhip64.so.7 instance

    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world_size > 1:
        import torch.distributed as dist

        dist.init_process_group("nccl", device_id=dev)
        assert dist.get_world_size() == world_size

    import raytracinginaweekend_amd as R
    from raytracinginaweekend_amd.distributed import FrameRenderer, FrameSpec

    def barrier():
        torch.cuda.synchronize(dev)
        if world_size > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize(dev)

    if args.configs_child:  # a PMC pass of the configs leg: 1 warm-up + 1 profiled frame each, no line
        render_configs(args, local_rank, 1, 1, barrier)
        return 0

    world = R.demo_world(args.scene)
    spec = FrameSpec(R.Size2i(args.width, args.height), args.spp, args.max_depth, args.seed,
                     tile=tuple(int(x) for x in args.tile.lower().split("x")))
    fr = FrameRenderer(world, spec, rank, world_size, local_rank)

    for _ in range(args.warmup):
        fr.render_frame()
    barrier()

    # HIP events on the stream the render kernel is launched on (the current stream)
    starts = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for i in range(args.steps):
        starts[i].record()
        fr.launch()  # the render kernel (+ the in-order accumulation), on the current stream
        ends[i].record()
        fr.exchange()
    barrier()
    elapsed = time.perf_counter() - t0
    kernel_ms = sum(s.elapsed_time(e) for s, e in zip(starts, ends)) / args.steps

    if world_size > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())

    samples = args.width * args.height * args.spp * args.steps
    value = samples / elapsed / 1e6
    pix = fr.pixels_this_rank()

    first_frame_ms = None
    if rank == 0 and world_size == 1 and not args.no_first_frame:
        t = time.perf_counter()
        R.render(spec.size, 1, args.spp, args.max_depth, world, seed=args.seed, device=local_rank)
        first_frame_ms = round((time.perf_counter() - t) * 1e3, 1)

    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    peak_ginstr = cus * SIMDS_PER_CU * CLOCK_GHZ / 2.0  # G wave-level VALU instructions / s
    roofline = {"bound": "valu_issue", "achieved": None, "peak": round(peak_ginstr, 1), "unit": "G VALU wave-instr/s",
                "frac": None, "traffic": None,
                "kernel": fr.dworld.kernel_variant().get("name") + "; HIP events on its launch stream also span the "
                          "in-order accumulate_kernel (~1.4 % of a 1080p x 512 frame: 1.95 ms, profiles/r05/r5z_kernel_stats.csv)",
                "kernel_ms": round(kernel_ms, 3),
                "peak_basis": f"{cus} CUs x {SIMDS_PER_CU} SIMD-32 x {CLOCK_GHZ} GHz / 2 cycles per wave64 VALU instruction"}
    if not args.no_stats:
        # the counting variant is ~8x slower than the product kernel: count at a bounded spp and
        # scale to the frame's (per-sample counts do not depend on spp; samples are independent).
        # tree 1: the traversal the timed kernel runs (the SAH walk + proofs + re-traces on SAH worlds)
        sp = type(fr.params).from_buffer_copy(fr.params)
        sp.samples_per_pixel = min(args.spp, args.stats_spp)
        stats = fr.dworld.collect_stats(sp, tree=1)
        scale = args.spp / sp.samples_per_pixel
        stats = {k: int(round(v * scale)) for k, v in stats.items()}
        b = alg_bytes(stats, pix)
        lds_peak = cus * LDS_BYTES_PER_CLK * CLOCK_GHZ  # GB/s
        rate = b / (kernel_ms * 1e-3) / 1e9
        roofline["records"] = {
            "bytes_per_launch": b, "GBps": round(rate, 1), "lds_peak_GBps": round(lds_peak, 1),
            "lds_frac": round(rate / lds_peak, 4), "tree": fr.dworld.kernel_variant()["tree"],
            "counts": f"counting variant of the timed kernel's traversal at {sp.samples_per_pixel} spp, scaled x{scale:g}",
            "note": "SURVEY §8(d) record bytes (32 B per node or leaf-box visit, the primitive records, material and "
                    "texel reads, the framebuffer) / kernel time; the records come from LDS and L2, so they are "
                    "priced against the LDS array peak (256 B/clk/CU), not HBM (HBM: see traffic); approximate "
                    "where the product kernel traces cooperatively: the counting variant re-traces tied rays on "
                    "the reference tree and walks the drain's last rays (DESIGN 5.7)",
            "per_sample": {k: round(v / max(1, stats["samples"]), 3) for k, v in stats.items() if k != "samples"},
        }

    if rank == 0 and world_size == 1 and not args.no_pmc:
        v = pmc_valu(args)
        if v is not None:
            insts = v["SQ_INSTS_VALU"]
            achieved = insts / (kernel_ms * 1e-3) / 1e9
            dispatch_s = v["dispatch_ns"] * 1e-9
            roofline["achieved"] = round(achieved, 1)
            roofline["frac"] = round(achieved / peak_ginstr, 4)
            roofline["valu"] = {
                "insts_per_frame": int(insts),
                "lane_utilisation": round(v["SQ_THREAD_CYCLES_VALU"] / (64.0 * v["SQ_ACTIVE_INST_VALU"]), 4),
                "wait_any_frac": round(v["SQ_WAIT_ANY"] / v["SQ_WAVE_CYCLES"], 4),
                "effective_clock_GHz": round(v["GRBM_GUI_ACTIVE"] / 8.0 / dispatch_s / 1e9, 3) if dispatch_s > 0 else None,
                "pmc_dispatch_ms": round(dispatch_s * 1e3, 3),
                "source": "rocprofv3 --pmc " + " ".join(VALU_COUNTERS) + f" on this benchmark's timed frame "
                          f"({v['launches']} render launch(es)); lane utilisation = SQ_THREAD_CYCLES_VALU / "
                          "(64 x SQ_ACTIVE_INST_VALU); clock = GRBM_GUI_ACTIVE / 8 XCDs / dispatch time",
            }
        if not args.no_traffic:
            t = pmc_traffic(args)
            if t is not None:
                roofline["traffic"] = round(t["bytes"])
                roofline["hbm_GBps"] = round(t["bytes"] / (kernel_ms * 1e-3) / 1e9, 1)
                roofline["hbm_frac"] = round(t["bytes"] / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)
                roofline["traffic_detail"] = {
                    "fetch_bytes_x2": round(t["fetch_bytes"]), "write_bytes": round(t["write_bytes"]),
                    "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), the timed frame's "
                              f"render_kernel launches ({t['launches']})"}

    tc_leg = None
    if rank == 0 and world_size == 1 and not args.no_thread_count:
        # main.rs:19: thread_count = available_parallelism() (the CPUs this process may use, as Rust
        # reads them: affinity capped by the cgroup quota)
        info = _cpu_info()
        T = info["affinity"]
        if info["cgroup_quota_cpus"]:
            T = min(T, max(1, int(info["cgroup_quota_cpus"] + 0.5)))
        T = args.thread_count_leg or T
        spec_t = FrameSpec(spec.size, args.spp, args.max_depth, args.seed, thread_count=T)
        fr_t = FrameRenderer(world, spec_t, 0, 1, local_rank)
        fr_t.render_frame()  # warm-up (tuning, cost order)
        barrier()
        st_, en_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t = time.perf_counter()
        st_.record()
        for _ in range(2):
            fr_t.launch()
        en_.record()
        barrier()
        dt = (time.perf_counter() - t) / 2
        tc_leg = {"thread_count": T, "value": round(args.width * args.height * args.spp / dt / 1e6, 3),
                  "ms_per_step": round(dt * 1e3, 3), "kernel_ms": round(st_.elapsed_time(en_) / 2, 3),
                  "vs_thread_count_1": round(elapsed / args.steps / dt, 4),
                  "note": "render(.., thread_count, ..) as main.rs:19 calls it: split_work_tasks planes merged "
                          "as merge_planes (rendering.rs:222-252) on the device; 2 frames after a warm-up"}
        del fr_t

    configs = None
    if rank == 0 and world_size == 1 and not args.no_configs:
        configs = render_configs(args, local_rank, max(1, args.configs_steps), 1, barrier)
        if not args.no_pmc:
            configs_pmc(args, configs, peak_ginstr)

    cpu = None
    if rank == 0 and world_size == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args)

    if args.save and rank == 0:
        from raytracinginaweekend_amd.image_io import save_image

        torch.cuda.synchronize(dev)
        save_image(args.save, fr.image.cpu().numpy().reshape(-1, 3), args.width, args.height)

    if rank == 0:
        last = fr.dworld.last_frame()
        line = {
            "metric": "Msamples/sec at 1920x1080x512spp; achieved HBM GB/s vs peak",
            "value": round(value, 3),
            "unit": "Msamples/sec",
            "n_gpus": world_size,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": f"synthetic: the reference's demo world {args.scene}, built as its builder does from fixed seeds "
            "(no external data beyond the reference's own OBJ / texture assets)",
            "config": {
                "workload": f"{args.scene} {args.width}x{args.height}x{args.spp}spp max_depth {args.max_depth}",
                "width": args.width,
                "height": args.height,
                "spp": args.spp,
                "max_depth": args.max_depth,
                "partition": f"interleaved {spec.tile[0]}x{spec.tile[1]} tiles over {world_size} GPU(s)",
                "rccl_world_size": world_size,
                "trace_min": last["trace_min"],
                "kernel": fr.dworld.kernel_variant(),
                "launches_per_frame": last["launches"],
                "work_items": None if last["whole_pixel"] is None else "whole pixels" if last["whole_pixel"] else "samples",
            },
            "first_frame_ms": first_frame_ms,
            "first_frame_Msamples_s": round(args.width * args.height * args.spp / first_frame_ms / 1e3, 1)
            if first_frame_ms else None,
            "roofline": roofline,
            "thread_count_leg": tc_leg,
            "configs": configs,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)

    if world_size > 1:
        torch.distributed.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
