"""Benchmark: Msamples/s of the render hot path on MI355X (BASELINE.json metric).

Workload (BASELINE configs[1]): the reference's demo world final_scene1 (demo_worlds.rs:395-463,
scene RNG seeded as main.rs:24), 1920x1080, 512 samples per pixel, max_depth 50.  One step =
one full frame: every rank renders its interleaved 8x8 tiles (rtw_render_device), then one RCCL
all-gather + untile assembles the image on rank 0 (N > 1).  `value` = W*H*spp*steps / max-over-
ranks wall time of the timed region (strong scaling: the frame is fixed, N GPUs share it).

Extra fields:
  roofline      the render kernel's algorithmic bytes per launch (SURVEY §8(d) byte model, from
                the kernel's counting variant over this rank's partition) / its average launch
                time measured with HIP events on the launch stream; peak = 8 TB/s HBM3E.
  cpu_baseline  the C restatement of the reference render loop (oracle/) on this host's cores,
                N = 1 only, on a bounded sample of the same frame: every P-th 8x8 tile at the
                full spp (P set for ~15 s of CPU work).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
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


def pmc_traffic(args) -> dict | None:
    """HBM bytes of one render-kernel launch from rocprofv3 PMC counters (MI355X_MICROARCH.md
    HBM section): a child `rocprofv3 --pmc FETCH_SIZE` run and a separate `--pmc WRITE_SIZE` run
    of this same benchmark (1 frame, no warmup), each reading the frame's render_kernel dispatch.
    FETCH_SIZE / WRITE_SIZE are in KiB; gfx950 reports half the bytes of wide coalesced reads in
    FETCH_SIZE, so it is doubled.  None if rocprofv3 is unavailable or a pass fails."""
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile

    if not shutil.which("rocprofv3"):
        return None
    child = [sys.executable, os.path.abspath(__file__), "--scene", args.scene, "--width", str(args.width), "--height",
             str(args.height), "--spp", str(args.spp), "--max-depth", str(args.max_depth), "--seed", str(args.seed),
             "--steps", "1", "--warmup", "0", "--no-cpu-baseline", "--no-stats", "--no-traffic"]
    got = {}
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as d:
            cmd = ["rocprofv3", "--pmc", counter, "-d", d, "-o", "pmc", "--output-format", "csv", "--"] + child
            try:
                subprocess.run(cmd, check=True, capture_output=True, timeout=600, cwd=ROOT)
            except (subprocess.SubprocessError, OSError):
                return None
            rows = []
            for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
                rows += [r for r in csv.DictReader(open(f)) if "render_kernel" in r["Kernel_Name"]
                         and r["Counter_Name"] == counter]
            if not rows:
                return None
            # the child renders one frame: sum its render launches (one per <= 16 GiB of
            # per-sample colours; counters of one dispatch may come as several rows)
            got[counter] = sum(float(r["Counter_Value"]) for r in rows) * 1024.0
            got["launches"] = len({r["Dispatch_Id"] for r in rows})
    fetch = got["FETCH_SIZE"] * 2.0
    return {"fetch_bytes": fetch, "write_bytes": got["WRITE_SIZE"], "bytes": fetch + got["WRITE_SIZE"],
            "launches": got["launches"]}


def cpu_baseline(world, args) -> dict:
    """The reference algorithm on the host cores (oracle/, test infrastructure), on a bounded
    sample of the same frame: every P-th 8x8 tile (interleaved, like the GPU partition) at the
    full spp, P chosen so the sample takes about --cpu-seconds."""
    import numpy as np

    import raytracinginaweekend_amd as R
    from oracle import pyoracle as O

    threads = args.cpu_threads or min(16, os.cpu_count() or 1)
    size = R.Size2i(args.width, args.height)
    out = np.zeros((size.count(), 3), np.float32)
    n_tiles = -(-args.width // 8) * -(-args.height // 8)

    def run(parts, spp):
        p = R.render_params(size, spp, args.max_depth, seed=3, part=(0, parts))
        t = time.perf_counter()
        O.render(world, p, O.RNG_CTR, threads, out=out)
        dt = time.perf_counter() - t
        return len(range(0, n_tiles, parts)) * 64 * spp, dt

    n, dt = run(48, 16)  # calibration, ~1 s
    for _ in range(3):
        rate = n / dt
        parts = max(1, min(n_tiles, int(args.width * args.height * args.spp / (rate * args.cpu_seconds))))
        n, dt = run(parts, args.spp)
        if dt > 0.5 * args.cpu_seconds or parts == 1:
            break
    return {
        "value": round(n / dt / 1e6, 4),
        "unit": "Msamples/sec",
        "cores": threads,
        "kind": "port",
        "sample": f"{args.scene} {args.width}x{args.height} at {args.spp}spp, every {parts}th 8x8 tile "
        f"({n} samples), max_depth {args.max_depth}; C restatement of rendering.rs (oracle/), "
        f"{threads} threads over rows, {dt:.1f} s",
    }


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scene", default="final_scene1")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=512)
    ap.add_argument("--max-depth", type=int, default=50)
    ap.add_argument("--seed", type=int, default=0x5EED)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-stats", action="store_true")
    ap.add_argument("--no-traffic", action="store_true", help="skip the rocprofv3 PMC traffic passes")
    ap.add_argument("--stats-spp", type=int, default=128, help="spp of the counting render (scaled to --spp)")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--save", default="", help="write the rank-0 image (.ppm/.png)")
    args = ap.parse_args()

    import torch  # first: librtw.so then binds to the same libamdhip64.so.7 instance

    rank = int(os.environ.get("RANK", "0"))
    world_size = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world_size > 1:
        import torch.distributed as dist

        dist.init_process_group("nccl", device_id=dev)

    import raytracinginaweekend_amd as R
    from raytracinginaweekend_amd.distributed import FrameRenderer, FrameSpec

    world = R.demo_world(args.scene)
    spec = FrameSpec(R.Size2i(args.width, args.height), args.spp, args.max_depth, args.seed)
    fr = FrameRenderer(world, spec, rank, world_size, local_rank)

    def barrier():
        torch.cuda.synchronize(dev)
        if world_size > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize(dev)

    for _ in range(args.warmup):
        fr.render_frame()
    barrier()

    starts = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for i in range(args.steps):
        starts[i].record()
        fr.launch()  # the render kernel, on the current stream
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

    roofline = None
    if not args.no_stats:
        # the counting variant is ~8x slower than the product kernel: count at a bounded spp and
        # scale to the frame's (per-sample counts do not depend on spp; samples are independent)
        sp = type(fr.params).from_buffer_copy(fr.params)
        sp.samples_per_pixel = min(args.spp, args.stats_spp)
        stats = fr.dworld.collect_stats(sp)
        scale = args.spp / sp.samples_per_pixel
        stats = {k: int(round(v * scale)) for k, v in stats.items()}
        pix = fr.pixels_this_rank()
        b = alg_bytes(stats, pix)
        achieved = b / (kernel_ms * 1e-3) / 1e9
        roofline = {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": None,
            "kernel": "render_kernel<false, LDS mode> (HIP events also span the in-order accumulate_kernel)",
            "counts": f"counting variant at {min(args.spp, args.stats_spp)} spp, scaled x{args.spp / min(args.spp, args.stats_spp):g}",
            "kernel_ms": round(kernel_ms, 3),
            "alg_bytes_per_launch": b,
            "per_sample": {k: round(v / max(1, stats["samples"]), 3) for k, v in stats.items() if k != "samples"},
        }

    cpu = None
    if rank == 0 and world_size == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(world, args)
    if roofline is not None and rank == 0 and world_size == 1 and not args.no_traffic:
        t = pmc_traffic(args)
        if t is not None:
            roofline["traffic"] = round(t["bytes"])
            roofline["traffic_detail"] = {"fetch_bytes_x2": round(t["fetch_bytes"]), "write_bytes": round(t["write_bytes"]),
                                          "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, one frame's render_kernel "
                                                    f"launches ({t['launches']})"}

    if args.save and rank == 0:
        import numpy as np

        from raytracinginaweekend_amd.image_io import save_image

        torch.cuda.synchronize(dev)
        save_image(args.save, fr.image.cpu().numpy().reshape(-1, 3), args.width, args.height)

    if rank == 0:
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
                "trace_min": fr.dworld.tuned_trace_min(),
            },
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)

    if world_size > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
