"""DDGI probe-update benchmark (BASELINE.json metric: Mrays/s + probes-updated/s,
DDGI 32^3 grid x 256 rays, at 1/2/4/8 MI355X).

Workload (config C4): synthetic 10M-triangle strip soup (PCG32
seed 0xA2C05E00), 32x32x32 probes (spacing 1 m, origin 0), 256 rays/probe, the
full grid updated every step (K = N = 32768), sun light. A step = one DDGI
update (trace -> shade -> irradiance/visibility/border/offset update) of every
probe; with N GPUs the grid is split in Z-slabs (strong scaling: fixed total
work) and the atlases are all-gathered over RCCL after each update.

Besides `value`, rank 0 at N = 1 reports: the reference's own windows (K = 4096,
the node's cap, DDGINode.h:23; K = 2048, its default, DDGINode.h:31) with per-kernel
times; config C2 (Cornell 8^3 x 64) on the GPU; the CPU baseline (the oracle on the
box's host cores, one warm-up then the median of >= 5 frames, C4 and C2); the C1 AO
bake; the DDGI consumers. The roofline object's `achieved` / `frac` are the
measured HBM traffic of the dominant kernel (a rocprofv3 PMC pass of this same
library build, matched by its sha256) over that pass's own launch duration (beside
it, `frac_hip_event`: over this run's HIP-event launch time); the SURVEY
§8d algorithmic model is kept beside it as `cache_inclusive_frac` (most of its
node fetches hit L2 / Infinity Cache), with the VALU issue fractions and the
whole-update figures (roofline()).

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

`python bench.py --gpus N` with N > 1 and no WORLD_SIZE starts the N ranks itself
(torch.distributed.run as a child process, launch_decision()); it exits non-zero
when fewer than N GPUs are visible. `--dry-run` prints that decision without any
GPU call.

ARK_BENCH_REHEARSAL=1 (test infrastructure, never a measurement): the N > 1 frame loop
on ONE GPU - every rank on cuda:0, a gloo process group, the atlas all-gather staged
through host memory - so that the Z-slab ranks' code path (rendezvous, slab contexts,
overlapped exchange, barrier and max-over-ranks timing) runs on a one-GPU box; RCCL
itself refuses two ranks on one device.

Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md: 8.0 TB/s)

# Algorithmic bytes (SURVEY.md §8d model, adapted to this build's layouts)
NODE_BYTES = 80        # GpuBvh8Node (8 quantized child boxes + bases + leaf codes)
TRI_BYTES = 48         # GpuTriangle (v0, e1, e2, instance, primitive)
HIT_RECORD_BYTES = 16  # GpuHit
SURFEL_BYTES = 8       # RGBA16F surfel
# per shaded (front) hit: shading record 64 (vertex normals, instance, UVs) + instance 64
# + material 96 + 3 texel fetches 48 + 8-probe DDGI gather 8*(4*4 + 4*8) = 384
SHADE_HIT_BYTES = 64 + 64 + 96 + 48 + 384
MISS_BYTES = 16        # environment texel
SHADOW_RAY_BYTES = 32  # ShadowRay record (written by k_shadow_gen, read by k_trace_shadow)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--triangles", type=int, default=10_000_000)
    ap.add_argument("--grid", type=int, default=32)
    ap.add_argument("--rays", type=int, default=256)
    ap.add_argument("--probe-updates", type=int, default=0, help="0 = whole grid per step")
    ap.add_argument("--cpu-probes", type=int, default=512, help="C4 CPU-baseline frame: a window of this many probes")
    ap.add_argument("--cpu-frames", type=int, default=5, help="timed CPU frames (median reported) after one warm-up")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = the host cores this process may use (see cpu_cores())")
    ap.add_argument("--no-windows", action="store_true", help="skip the reference-window (K = 4096 / 2048) and C2 lines")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-ao-bake", action="store_true", help="skip the config C1 AO bake line (GPU + CPU oracle)")
    ap.add_argument("--ao-size", type=int, default=1024)
    ap.add_argument("--ao-samples", type=int, default=64)
    ap.add_argument("--ao-cpu-seconds", type=float, default=8.0)
    ap.add_argument("--no-compose", action="store_true", help="skip the DDGI consumer (lighting compose) line")
    ap.add_argument("--no-configs", action="store_true", help="skip the C5 / C3 substitute lines")
    ap.add_argument("--compose-size", default="1920x1080")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "latest_pmc.json"),
                    help="PMC traffic summary (tools/pmc_summary.py --latest); used only if its library hash matches")
    ap.add_argument("--sq", default=os.path.join(ROOT, "profiles", "latest_sq.json"),
                    help="SQ counter summary (tools/sq_summary.py --json); used only if its library hash matches")
    ap.add_argument("--sun-bvh", choices=("auto", "world", "light"), default="auto",
                    help="the sun's shadow-ray structure (ArkDdgiDesc.sun_bvh); auto = set_scene's sampled choice")
    ap.add_argument("--serial-frames", action="store_true",
                    help="no frames in flight (ARK_DDGI_FLAG_SERIAL_FRAMES): kernels do not overlap (profiling A/B)")
    ap.add_argument("--master-port", type=int, default=29517,
                    help="rendezvous port of the ranks bench.py starts itself (--gpus N > 1 without WORLD_SIZE)")
    ap.add_argument("--dry-run", action="store_true",
                    help="print the launch decision (run in this process / start N ranks / refuse) as JSON and exit; no GPU call")
    return ap.parse_args(argv)


def launch_decision(gpus, env, visible_gpus, argv, master_port=29517):
    """How `bench.py --gpus N` runs (VERDICT r05 "do this" #1), decided before any GPU
    call: ("run", N) in this process when the world size already matches (N = 1, or a
    rank of the driver's `torch.distributed.run --nproc-per-node N`); ("spawn", cmd)
    when N > 1 ranks were asked for and this process is not one of them: bench.py
    starts `torch.distributed.run` as a CHILD process (never an exec: this process has
    not touched the GPU and forwards the child's output and exit status); ("error",
    why) when the request cannot be met (more GPUs than are visible, or a WORLD_SIZE
    that disagrees with --gpus). A 1-GPU line is never printed for an N-GPU request."""
    if gpus < 1:
        return "error", f"--gpus {gpus}: at least one GPU"
    world_env = env.get("WORLD_SIZE")
    if world_env is not None:
        world = int(world_env)
        if world != gpus:
            return "error", f"WORLD_SIZE={world} but --gpus {gpus}: launch {gpus} ranks (torch.distributed.run --nproc-per-node {gpus})"
        return "run", world
    if gpus == 1:
        return "run", 1
    if visible_gpus < gpus:
        return "error", f"--gpus {gpus} but {visible_gpus} GPU(s) visible: no {gpus}-GPU line can be measured here"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr=127.0.0.1", f"--master-port={master_port}", os.path.abspath(__file__)] + list(argv)
    return "spawn", cmd


def _visible_gpus():
    """GPUs this process could use, counted without initialising the GPU (on this image
    torch.cuda.device_count() does not create a HIP context)."""
    import torch

    return torch.cuda.device_count()


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    env = os.environ
    # the launch decision first: a spawning parent must not have touched the GPU
    visible = _visible_gpus() if (args.gpus > 1 and "WORLD_SIZE" not in env) else args.gpus
    kind, what = launch_decision(args.gpus, env, visible, [a for a in argv if a != "--dry-run"], args.master_port)
    if args.dry_run:
        print(json.dumps({"decision": kind, "world_size": args.gpus if kind != "error" else None,
                          "command": what if kind == "spawn" else None, "error": what if kind == "error" else None}))
        return 0 if kind != "error" else 2
    if kind == "error":
        print(f"bench.py: {what}", file=sys.stderr)
        return 2
    if kind == "spawn":
        # stdout of rank 0 (the JSON line) and every rank's stderr pass straight through
        return subprocess.run(what, env=dict(env, HSA_ENABLE_IPC_MODE_LEGACY=env.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))).returncode
    import torch
    import torch.distributed as dist

    world = int(env.get("WORLD_SIZE", "1"))
    rank = int(env.get("RANK", "0"))
    rehearsal = env.get("ARK_BENCH_REHEARSAL") == "1"
    local_rank = 0 if rehearsal else int(env.get("LOCAL_RANK", "0"))
    device = torch.device("cuda", local_rank)
    torch.cuda.set_device(device)
    if world > 1:
        if rehearsal:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=device)

    from arkoserenderer_amd import abi
    from arkoserenderer_amd import ddgi as D
    from arkoserenderer_amd import scene as S
    from arkoserenderer_amd.collective import SlabExchange

    G = args.grid
    N = G * G * G
    K = args.probe_updates or N
    R = args.rays
    t_setup = time.time()
    scene = S.soup(args.triangles)
    grid = D.ProbeGrid((G, G, G), (1.0, 1.0, 1.0), (0.0, 0.0, 0.0))
    sun_mode = {"auto": abi.ARK_DDGI_SUN_BVH_AUTO, "world": abi.ARK_DDGI_SUN_BVH_WORLD, "light": abi.ARK_DDGI_SUN_BVH_LIGHT_SPACE}[args.sun_bvh]
    cfg = D.DDGIConfig(rays_per_probe=R, probe_updates_per_frame=K, max_rays_per_probe=R, max_probe_updates=K,
                       compute_probe_offsets=True, sun_bvh=sun_mode, serial_frames=args.serial_frames)
    exposure = dict(light_pre_exposure=1.0, ambient_illuminance=0.0, environment_brightness=1.0)
    node = D.DDGINode(cfg)
    assert node.construct(scene, grid, 10000.0, device=local_rank, shard_rank=rank, shard_count=world, **exposure)
    ctx = node.ctx
    bvh = ctx.bvh_stats()
    stream = torch.cuda.current_stream(device)
    sptr = stream.cuda_stream
    # Z-slab ranks: the all-gather of frame N runs on a side stream, overlapped with
    # frame N+1's primary traversal (collective.OverlappedSlabExchange)
    exch = None
    if world > 1:
        from arkoserenderer_amd.collective import OverlappedSlabExchange, RcclBandExchange, WindowExchange, WindowSource, torch_all_gather

        # the two bands as one RCCL group on the exchange stream itself (RcclBandExchange);
        # ARK_BENCH_TORCH_PG=1: through torch's process group instead
        band = None
        if rehearsal:
            band = SlabExchange.from_views(ctx.device_views(), rank, world, device)
            band.exchange = _host_staged(band)
            gather = _host_gather
        elif os.environ.get("ARK_BENCH_TORCH_PG") != "1":
            try:
                band = RcclBandExchange.from_views(ctx.device_views(), rank, world, device)
            except (RuntimeError, OSError, AttributeError) as e:  # no direct RCCL: the process group's all-gather
                print(f"warning: RcclBandExchange unavailable ({e}); using torch.distributed all-gather", file=sys.stderr)
        if band is None:
            band = SlabExchange.from_views(ctx.device_views(), rank, world, device)
            gather = torch_all_gather()
        elif not rehearsal:
            gather = band.all_gather
        # K < N: only the window's tiles travel (WindowExchange); K = N: the row bands
        window = WindowExchange(WindowSource(ctx), band.exchange, gather, rank, world, min(K, N // world), device)
        exch = OverlappedSlabExchange(node, window.exchange, device)
        exch.watchdog.rccl = band if isinstance(band, RcclBandExchange) else None
    setup_s = time.time() - t_setup

    frame = 0

    def step():
        nonlocal frame
        if exch is not None:
            exch.step(D.AppState(frame), sptr)
        else:
            node.execute(D.AppState(frame), sptr)
        frame += 1

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(device)

    # --- counter-instrumented update (separate kernel variant; not timed) -----
    ctx.set_counting(True)
    step()
    torch.cuda.synchronize(device)
    cnt = ctx.counters()
    ctx.set_counting(False)

    # --- per-kernel device time from HIP events on the update stream ----------
    ctx.set_timing(True)
    ktimes = []
    for _ in range(3):
        step()
        ktimes.append(ctx.last_timings())
    ctx.set_timing(False)
    torch.cuda.synchronize(device)

    # --- timed region: exactly `steps` steps -----------------------------------
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    if exch is not None:
        exch.drain()  # bounded (collective.ExchangeWatchdog): a dead peer ends the run
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    # a frame-sequencing wait that gave up inside the timed region dropped frames
    # (fail-closed, ark_ddgi_set_sequencing): that raises here, and no line is printed
    ctx.synchronize()
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    total_rays = args.steps * K * R
    total_probes = args.steps * K
    mrays = total_rays / dt / 1e6
    lib_sha = library_sha16()

    # roofline of the dominant kernel (per launch, this rank's share)
    avg = [sum(k[i] for k in ktimes) / len(ktimes) for i in range(5)]
    kernel_bytes = algorithmic_bytes(cnt, R)
    kernel_ms = {"k_trace": avg[1], "k_shade": avg[2], "k_shadow": avg[4], "k_probe_update": avg[3]}
    dom = max(kernel_ms, key=kernel_ms.get)
    ms_per_step = dt / args.steps * 1e3
    roof = roofline(args, dom, kernel_bytes, kernel_ms, ms_per_step, lib_sha, G)

    result = {
        "metric": "Mrays/s + probes-updated/s, DDGI 32^3 grid x 256 rays, at 1/2/4/8 MI355X",
        "value": round(mrays, 3),
        "unit": "Mrays/s",
        "probes_updated_per_s": round(total_probes / dt, 1),
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic",
        "config": {
            "workload": "C4: synthetic 10M-triangle strip soup, 32x32x32 probes x 256 rays, whole grid updated per step",
            "triangles": scene.triangle_count,
            "grid": G,
            "rays_per_probe": R,
            "probe_updates_per_step": K,
            "parallelism": f"zslab{world}",
            "bvh_nodes": int(bvh.node_count),
            "bvh_max_depth": int(bvh.max_depth),
            "bvh_build_ms": round(bvh.build_ms, 1),
            "sun_bvh": sun_bvh_info(bvh),
            "setup_s": round(setup_s, 2),
            "lib_sha16": lib_sha,
        },
        "roofline": roof,
        "kernels_ms": {k: round(v, 4) for k, v in kernel_ms.items()},
        "update_ms": round(avg[0], 4),
        "per_ray": per_ray(cnt),
    }

    if rank == 0 and world == 1 and not args.no_windows:
        result["reference_windows"] = reference_windows(node, ctx, torch, device, sptr, frame)
        result["c2"] = c2_line(args, torch, device)

    if rank == 0 and world == 1 and not args.no_configs:
        for name in ("c5", "c3"):
            result[name] = config_line(name, torch, device)

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(scene, grid, R, args, exposure)

    if rank == 0 and world == 1 and not args.no_ao_bake:
        result["ao_bake"] = ao_bake_c1(args, torch, device)

    if rank == 0 and world == 1 and not args.no_compose:
        result["lighting_compose"] = lighting_compose_line(args, torch, node.ctx)
        result["rt_reflections"] = rt_reflections_line(args, torch, node.ctx)

    if rank == 0:
        print(json.dumps(result), flush=True)
    node.ctx.close()
    if world > 1:
        dist.destroy_process_group()
    return 0


def _host_gather(out, mine):
    """ARK_BENCH_REHEARSAL: the all-gather through host memory over gloo (in order on the
    current stream: the copies synchronise it)."""
    import torch.distributed as dist

    parts = list(out.cpu().chunk(dist.get_world_size()))
    dist.all_gather(parts, mine.cpu())
    out.copy_(__import__("torch").cat(parts).to(out.device))


def _host_staged(band):
    """ARK_BENCH_REHEARSAL: SlabExchange's band all-gathers through host memory."""

    def exchange():
        for full, mine in band.bufs:
            _host_gather(full, mine)

    return exchange


def library_sha16() -> str:
    """sha256 (16 hex) of the HIP library this process runs: ties PMC/SQ summaries to a build."""
    from arkoserenderer_amd import abi

    path = abi.library_path()
    h = hashlib.sha256()
    with open(path, "rb") as fh:
        for chunk in iter(lambda: fh.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()[:16]


def algorithmic_bytes(cnt, R):
    """Algorithmic bytes per launch (SURVEY §8d model with this build's layouts)."""
    rays = cnt.rays
    return {
        "k_trace": NODE_BYTES * cnt.primary_node_visits + TRI_BYTES * cnt.primary_tri_tests + HIT_RECORD_BYTES * rays,
        "k_shade": HIT_RECORD_BYTES * rays + SHADE_HIT_BYTES * cnt.front_hits + MISS_BYTES * (rays - cnt.hits) + SURFEL_BYTES * rays,
        "k_shadow": NODE_BYTES * cnt.shadow_node_visits + TRI_BYTES * cnt.shadow_tri_tests + 2 * SHADOW_RAY_BYTES * cnt.shadow_rays,
        "k_probe_update": cnt.probes * (R * SURFEL_BYTES + 2 * (64 * 8 + 256 * 4) + (36 * 8 + 68 * 4) + 32),
    }


def per_ray(cnt):
    rays = max(1, cnt.rays)
    return {
        "primary_nodes": round(cnt.primary_node_visits / rays, 2),
        "primary_tris": round(cnt.primary_tri_tests / rays, 2),
        "primary_lane_util": round((cnt.primary_node_visits + cnt.primary_tri_tests) / max(1, 64 * cnt.primary_wave_steps), 3),
        "hit_frac": round(cnt.hits / rays, 4),
        "front_hit_frac": round(cnt.front_hits / rays, 4),
        "shadow_rays": round(cnt.shadow_rays / rays, 4),
        "shadow_nodes": round(cnt.shadow_node_visits / rays, 2),
        "shadow_tris": round(cnt.shadow_tri_tests / rays, 2),
    }


# rocprofv3 kernel names -> the bench's kernel keys
PMC_KERNELS = {"k_trace": ["k_trace"], "k_shade": ["k_shade"], "k_shadow": ["k_shadow_gen", "k_trace_shadow", "k_trace_shadow_sun", "k_trace_shadow_sunw"],
               "k_probe_update": ["k_probe_update"]}
# launched only for some scenes: the sun's light-space shadow traversal (a scene with a
# sun), the world-BVH shadow traversal (other lights, or no sun BVH)
PMC_OPTIONAL = {"k_trace_shadow", "k_trace_shadow_sun", "k_trace_shadow_sunw"}


# every kernel of one probe-path update (the whole-update counter figure)
PMC_PATH_KERNELS = ("k_probe_slots", "k_trace", "k_probe_offsets", "k_shadow_gen", "k_trace_shadow", "k_trace_shadow_sun", "k_trace_shadow_sunw", "k_shade", "k_probe_update")
CLOCK_GHZ = 2.4      # MI355X max engine clock (MI355X_MICROARCH.md); the VALU fractions below use it
SIMDS = 256 * 4      # 256 CUs x 4 SIMDs
WAVE64_VALU_CYCLES = 2  # a wave64 VALU instruction issues over 2 cycles on the 32-wide CDNA4 SIMD


def _load_summary(path, lib_sha, what):
    """A profiles/ summary of THIS library build (matched by sha256), or (None, why).
    PMC summaries keep the hash under config, SQ summaries at the top."""
    if not os.path.exists(path):
        return None, f"no {what} summary"
    try:
        with open(path) as fh:
            j = json.load(fh)
    except (OSError, ValueError) as e:
        return None, f"unreadable {what} summary: {e}"
    sha = j.get("config", {}).get("lib_sha16") if "config" in j else j.get("lib_sha16")
    if sha != lib_sha:
        return None, f"{what} summary {j.get('tag')} is of another build ({sha}): not used"
    return j, None


def roofline(args, dom, kernel_bytes, kernel_ms, ms_per_step, lib_sha, G):
    """The roofline object of the dominant kernel plus the whole update.

    `achieved` / `frac` are MEASURED HBM bytes: (2 FETCH_SIZE + WRITE_SIZE) x 1024 per
    launch (tools/pmc_summary.py; the gfx950 FETCH_SIZE halving of MI355X_MICROARCH.md
    §HBM) from a rocprofv3 PMC pass of this same library build, divided by that
    pass's own average launch duration; `achieved_hip_event` / `frac_hip_event` divide
    the same bytes by this run's HIP-event launch time. The SURVEY §8(d) algorithmic model (80-B nodes and 48-B
    triangles per visit, counter-instrumented visit counts) is kept beside it as
    `cache_inclusive_*`: it counts every node fetch, and most of them are L2 / Infinity
    Cache hits (LDS-cached top nodes included), so it is a cache-inclusive request
    rate, not HBM traffic. `valu_issue_frac` = VALU wave-instructions / (1024 SIMDs x
    2.4 GHz x t); `valu_simd_busy_frac` counts the 2 cycles a wave64 VALU instruction
    occupies a 32-wide SIMD."""
    t = kernel_ms[dom] * 1e-3
    alg = kernel_bytes[dom]
    roof = {
        # priced against HBM (no dense contraction, no MFMA); limited by instruction
        # issue and dependent-fetch latency (SQ counters below)
        "bound": "latency",
        "roofline": "hbm",
        "kernel": dom,
        "achieved": None,
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": None,
        "traffic": None,
        "avg_launch_ms": round(kernel_ms[dom], 4),
        "algorithmic_bytes_per_launch": int(alg),
        "cache_inclusive_achieved": round(alg / t / 1e9, 2),
        "cache_inclusive_frac": round(alg / t / 1e9 / HBM_PEAK_GBS, 4),
    }
    pm, why = _load_summary(args.pmc, lib_sha, "PMC")
    if pm is not None:
        cfg = pm.get("config", {})
        if cfg.get("triangles") != args.triangles or cfg.get("grid") != G:
            pm, why = None, f"PMC summary {pm.get('tag')} is of another workload: not used"
    if pm is not None:
        ks = [pm["kernels"].get(k) for k in PMC_KERNELS[dom] if k not in PMC_OPTIONAL or k in pm["kernels"]]
        if not ks or any(k is None or "hbm_bytes_per_launch" not in k for k in ks):
            pm, why = None, f"PMC summary {pm.get('tag')} lacks {dom}"
    if pm is not None:
        # achieved / frac: the PMC pass's bytes over the PMC pass's own average launch
        # duration (one run, self-consistent); *_hip_event: the same bytes over this
        # run's HIP-event launch time (the two runs' times differ by a few %)
        traffic = sum(k["hbm_bytes_per_launch"] for k in ks)
        t_prof = sum(k["avg_ms"] for k in ks) * 1e-3
        roof["traffic"] = int(traffic)
        roof["achieved"] = round(traffic / t_prof / 1e9, 2)
        roof["frac"] = round(traffic / t_prof / 1e9 / HBM_PEAK_GBS, 4)
        roof["traffic_source"] = pm.get("source")
        roof["traffic_profile_avg_launch_ms"] = round(t_prof * 1e3, 4)
        roof["achieved_hip_event"] = round(traffic / t / 1e9, 2)
        roof["frac_hip_event"] = round(traffic / t / 1e9 / HBM_PEAK_GBS, 4)
    else:
        roof["traffic_source"] = why
    sq, why_sq = _load_summary(args.sq, lib_sha, "SQ")
    sq_kernel = PMC_KERNELS[dom][0] if dom != "k_shadow" else "k_trace_shadow"
    k = sq.get("kernels", {}).get(sq_kernel) if sq else None
    if k is not None:
        valu = k.get("valu_insts_per_launch", 0)
        roof["valu_issue_frac"] = round(valu / (SIMDS * CLOCK_GHZ * 1e9 * t), 4)
        roof["valu_simd_busy_frac"] = round(valu * WAVE64_VALU_CYCLES / (SIMDS * CLOCK_GHZ * 1e9 * t), 4)
        roof["limiter_evidence"] = {key: k[key] for key in ("valu_active_per_wave", "wait_inst_any_per_wave", "wait_any_per_wave",
                                                             "valu_insts_per_launch", "salu_insts_per_launch", "l2_hit",
                                                             "clock_ghz_effective") if key in k} | {"source": sq.get("source")}
    else:
        roof["limiter_evidence"] = why_sq
    # the whole update ((sum B_ray + sum B_probe) / wall time of the update)
    step_alg = sum(kernel_bytes.values())
    whole = {"ms_per_step": round(ms_per_step, 4), "algorithmic_bytes_per_step": int(step_alg),
             "cache_inclusive_achieved": round(step_alg / (ms_per_step * 1e-3) / 1e9, 2),
             "cache_inclusive_frac": round(step_alg / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
             "hbm_bytes_per_step": None, "achieved": None, "frac": None}
    path = [k for k in PMC_PATH_KERNELS if k not in PMC_OPTIONAL or (pm is not None and k in pm["kernels"])]
    if pm is not None and all(k in pm["kernels"] and "hbm_bytes_per_launch" in pm["kernels"][k] for k in path):
        hbm = sum(pm["kernels"][k]["hbm_bytes_per_launch"] for k in path)
        whole.update(hbm_bytes_per_step=int(hbm), achieved=round(hbm / (ms_per_step * 1e-3) / 1e9, 2),
                     frac=round(hbm / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4))
    roof["whole_update"] = whole
    return roof


def reference_windows(node, ctx, torch, device, sptr, frame0):
    """The reference node's own rolling windows on the same C4 context: K = 4096
    (MaxNumProbeUpdates, DDGINode.h:23) and K = 2048 (m_probeUpdatesPerFrame default,
    DDGINode.h:31), 256 rays, a window advancing each frame as the node's does; two
    warm-up frames, then `reps` timed frames (wall clock) and the per-kernel HIP-event
    times of 3 more."""
    from arkoserenderer_amd import ddgi as D

    out = {}
    full = node.config.probe_updates_per_frame
    frame = frame0
    R = node.config.rays_per_probe
    for K in (4096, 2048):
        node.config.probe_updates_per_frame = K
        for _ in range(2):
            node.execute(D.AppState(frame), sptr)
            frame += 1
        torch.cuda.synchronize(device)
        reps = 20
        t0 = time.perf_counter()
        for _ in range(reps):
            node.execute(D.AppState(frame), sptr)
            frame += 1
        torch.cuda.synchronize(device)
        ms = (time.perf_counter() - t0) / reps * 1e3
        ctx.set_timing(True)
        kt = []
        for _ in range(3):
            node.execute(D.AppState(frame), sptr)
            frame += 1
            kt.append(ctx.last_timings())
        ctx.set_timing(False)
        torch.cuda.synchronize(device)
        a = [sum(k[i] for k in kt) / len(kt) for i in range(5)]
        # ms_per_frame: consecutive windows are disjoint, so frame n + 1's traversal
        # overlaps frame n's shading and update (frames in flight, ark_ddgi.h);
        # kernels_ms: the instrumented (serial) frames
        out[f"K{K}"] = {"mrays_per_s": round(K * R / ms / 1e3, 1), "probes_updated_per_s": round(K / ms * 1e3, 1), "ms_per_frame": round(ms, 4),
                        "frames_in_flight": True,
                        "kernels_ms": {"k_trace": round(a[1], 4), "k_shadow": round(a[4], 4), "k_shade": round(a[2], 4),
                                       "k_probe_update": round(a[3], 4)}}
    node.config.probe_updates_per_frame = full
    return out


def c2_line(args, torch, device):
    """Config C2: Cornell box, 8^3 probes x 64 rays, all 512 probes per
    frame, the level's exposure (preExposure 2.2e-4, env x 3000), offsets off; GPU
    wall clock over 50 frames after 5 warm-up frames."""
    from arkoserenderer_amd import ddgi as D
    from arkoserenderer_amd import scene as S

    sc, ex = S.cornell_box()
    grid = D.ProbeGrid((8, 8, 8), (0.257, 0.257, 0.257), (-0.9, 0.1, -0.9))
    cfg = D.DDGIConfig(rays_per_probe=64, probe_updates_per_frame=512, compute_probe_offsets=False, max_rays_per_probe=64, max_probe_updates=512)
    node = D.DDGINode(cfg)
    node.construct(sc, grid, ex["z_far"], device=device.index or 0, light_pre_exposure=ex["light_pre_exposure"],
                   environment_brightness=ex["environment_brightness"])
    sptr = torch.cuda.current_stream(device).cuda_stream
    for f in range(5):
        node.execute(D.AppState(f), sptr)
    torch.cuda.synchronize(device)
    reps = 50
    t0 = time.perf_counter()
    for f in range(reps):
        node.execute(D.AppState(5 + f), sptr)
    torch.cuda.synchronize(device)
    ms = (time.perf_counter() - t0) / reps * 1e3
    node.ctx.close()
    return {"workload": "C2: Cornell box (100 triangles), 8x8x8 probes x 64 rays, all probes per frame",
            "gpu_ms_per_frame": round(ms, 4), "gpu_mrays_per_s": round(512 * 64 / ms / 1e3, 1),
            "note": "32,768 rays per frame: launch-bound on the GPU (five launches)"}


def config_line(name, torch, device, steps=10, warmup=3):
    """The other GPU configs of BASELINE.json at N = 1, whole grid per step (K = N),
    with their substitutes for the scenes the reference tree lacks: C5 =
    the instanced city block for Bistro (~3 M triangles, 48x16x48 probes x 512 rays, sun
    + 4 IES spot lights: 5 shadow rays per lit hit), C3 = a 262,272-triangle strip soup
    for Sponza (Sponza.bin is missing; 24x12x24 x 256, sun + 3 IES spots). Wall clock
    over `steps` steps after `warmup` on torch's current stream (frames in flight), plus
    the per-kernel HIP-event times of 3 instrumented (serial) steps."""
    from arkoserenderer_amd import ddgi as D
    from arkoserenderer_amd import scene as S

    if name == "c5":
        sc = S.city_block()
        grid = D.ProbeGrid((48, 16, 48), (5.0, 2.5, 5.0), (2.5, 0.5, 2.5))
        R, zf = 512, 1000.0
        workload = "C5 substitute: instanced city block, 48x16x48 probes x 512 rays, sun + 4 IES spots, whole grid per step"
    else:
        sc = S.sponza_substitute()
        grid = D.ProbeGrid(*S.sponza_substitute_grid())
        R, zf = 256, 10000.0
        workload = "C3 substitute: 262,272-triangle strip soup, 24x12x24 probes x 256 rays, sun + 3 IES spots, whole grid per step"
    N = grid.probe_count()
    cfg = D.DDGIConfig(rays_per_probe=R, probe_updates_per_frame=N, max_rays_per_probe=R, max_probe_updates=N, compute_probe_offsets=True)
    node = D.DDGINode(cfg)
    t = time.time()
    node.construct(sc, grid, zf, device=device.index or 0, light_pre_exposure=1.0, ambient_illuminance=0.02, environment_brightness=1.0)
    setup = time.time() - t
    sptr = torch.cuda.current_stream(device).cuda_stream
    frame = 0
    for _ in range(warmup):
        node.execute(D.AppState(frame), sptr)
        frame += 1
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for _ in range(steps):
        node.execute(D.AppState(frame), sptr)
        frame += 1
    torch.cuda.synchronize(device)
    ms = (time.perf_counter() - t0) / steps * 1e3
    node.ctx.synchronize()
    node.ctx.set_timing(True)
    kt = []
    for _ in range(3):
        node.execute(D.AppState(frame), sptr)
        frame += 1
        kt.append(node.ctx.last_timings())
    node.ctx.set_timing(False)
    node.ctx.set_counting(True)
    node.execute(D.AppState(frame), sptr)
    torch.cuda.synchronize(device)
    c = node.ctx.counters()
    node.ctx.set_counting(False)
    a = [sum(k[i] for k in kt) / len(kt) for i in range(5)]
    bvh = node.ctx.bvh_stats()
    node.ctx.close()
    rays = N * R
    return {"workload": workload, "triangles": sc.triangle_count, "mrays_per_s": round(rays / ms / 1e3, 1),
            "probes_updated_per_s": round(N / ms * 1e3, 1), "ms_per_step": round(ms, 4), "steps": steps,
            "kernels_ms": {"k_trace": round(a[1], 4), "k_shadow": round(a[4], 4), "k_shade": round(a[2], 4), "k_probe_update": round(a[3], 4)},
            "shadow_rays_per_ray": round(c.shadow_rays / rays, 4), "primary_nodes_per_ray": round(c.primary_node_visits / rays, 2),
            "sun_bvh": sun_bvh_info(bvh), "setup_s": round(setup, 1)}


def sun_bvh_info(bvh):
    """set_scene's choice for the sun's shadow rays: the light-space BVH8 (its nodes) or
    the world BVHs, with the sampled any-hit steps per sun shadow ray of both."""
    return {"light_space": bool(bvh.sun_node_count), "sampled_steps_world": round(bvh.sun_cost_world, 2),
            "sampled_steps_light": round(bvh.sun_cost_light, 2),
            "build_ms": round(bvh.sun_build_ms, 1)}


def cpu_cores():
    """Host cores for the CPU baseline: the CPUs this process may run on
    (os.sched_getaffinity), capped at the GPU box's per-GPU CPU share where the
    box sets it (OMP_NUM_THREADS / MAX_JOBS = 16 there: nproc shows the whole
    machine), plus what the machine reports."""
    allowed = len(os.sched_getaffinity(0))
    share = None
    for var in ("OMP_NUM_THREADS", "MAX_JOBS"):
        v = os.environ.get(var)
        if v and v.isdigit() and int(v) > 0:
            share = int(v)
            break
    use = min(allowed, share) if share else allowed
    model = None
    try:
        txt = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in txt.splitlines():
            if line.startswith("Model name:"):
                model = line.split(":", 1)[1].strip()
                break
    except (OSError, subprocess.SubprocessError):
        pass
    try:
        nproc = int(subprocess.run(["nproc", "--all"], capture_output=True, text=True, timeout=10).stdout.strip())
    except (OSError, subprocess.SubprocessError, ValueError):
        nproc = os.cpu_count()
    return use, {"nproc_all": nproc, "affinity": allowed, "share": share, "model": model}


def _median_frames(orc, make_params, frames, threads):
    """One warm-up frame, then the median wall time of `frames` frames."""
    orc.update(make_params(0), threads)
    ts = []
    for f in range(1, frames + 1):
        t = time.perf_counter()
        orc.update(make_params(f), threads)
        ts.append(time.perf_counter() - t)
    return statistics.median(ts), ts


def cpu_baseline(scene, grid, R, args, exposure):
    """The CPU oracle (the C++ restatement of the reference shaders, `port`) on the
    host cores (cpu_cores()): config C4 on a window of `cpu_probes` probes of the
    same scene / grid / R (a bounded sample: one warm-up frame + the median of
    `cpu_frames` frames, all stages of the update), and config C2 whole (Cornell,
    8^3 x 64, the same protocol)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O
    from arkoserenderer_amd import ddgi as D
    from arkoserenderer_amd import scene as S

    threads, host = cpu_cores()
    threads = args.cpu_threads or threads
    k = args.cpu_probes
    cfg = D.DDGIConfig(rays_per_probe=R, probe_updates_per_frame=k, max_rays_per_probe=R, max_probe_updates=k, compute_probe_offsets=True)
    orc = O.Oracle(D.desc_for(grid, 10000.0, cfg))
    t = time.time()
    orc.set_scene(scene, threads)
    build_s = time.time() - t
    N = grid.probe_count()
    med, ts = _median_frames(orc, lambda f: D.frame_params(cfg, grid, D.AppState(f), (f * k) % N, **exposure), args.cpu_frames, threads)
    orc.close()
    res = {
        "value": round(k * R / med / 1e6, 4),
        "unit": "Mrays/s",
        "cores": threads,
        "kind": "port",
        "sample": (f"C4: windows of {k} probes x {R} rays of the same workload (rolling, K = {k}), full update incl. shading/indirect/blend; "
                   f"1 warm-up + median of {len(ts)} frames ({', '.join(f'{x:.2f}' for x in ts)} s); oracle BVH build {build_s:.1f} s excluded"),
        "probes_updated_per_s": round(k / med, 2),
        "host": host,
    }
    sc, ex = S.cornell_box()
    g2 = D.ProbeGrid((8, 8, 8), (0.257, 0.257, 0.257), (-0.9, 0.1, -0.9))
    c2cfg = D.DDGIConfig(rays_per_probe=64, probe_updates_per_frame=512, compute_probe_offsets=False, max_rays_per_probe=64, max_probe_updates=512)
    orc = O.Oracle(D.desc_for(g2, ex["z_far"], c2cfg))
    orc.set_scene(sc, threads)
    kw = dict(light_pre_exposure=ex["light_pre_exposure"], environment_brightness=ex["environment_brightness"])
    med2, ts2 = _median_frames(orc, lambda f: D.frame_params(c2cfg, g2, D.AppState(f), 0, **kw), args.cpu_frames, threads)
    orc.close()
    res["c2"] = {"value": round(512 * 64 / med2 / 1e6, 4), "unit": "Mrays/s", "cores": threads,
                 "sample": f"C2: Cornell 8^3 x 64, all 512 probes per frame; 1 warm-up + median of {len(ts2)} frames",
                 "ms_per_frame": round(med2 * 1e3, 3)}
    return res


def rt_reflections_line(args, torch, ctx):
    """The RT reflections consumer: ark_ddgi_rt_reflections at
    compose_size on the C4 scene (10M triangles) and atlases after the timed steps, a
    seeded synthetic G-buffer (10 % sky, 20 % too rough to trace) resident in HBM, one
    reflection ray per traced pixel plus its shadow ray (sun). HIP events on the
    stream the kernel runs on."""
    import numpy as np

    from arkoserenderer_amd import ddgi as D

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import reflection_inputs as RI

    W, H = (int(v) for v in args.compose_size.split("x"))
    cam = RI.camera(W, H, eye=(16.0, 16.0, -6.0), target=(16.0, 14.0, 16.0))
    g, _ = RI.gbuffer(W, H, cam, seed=5)
    dev = {k: torch.from_numpy(np.ascontiguousarray(v)).cuda() for k, v in g.items()}
    rad = torch.empty((H, W, 4), dtype=torch.int16, device="cuda")
    dirs = torch.empty((H, W, 4), dtype=torch.int16, device="cuda")
    planes = {k: dev[k].data_ptr() for k in ("depth", "material", "normal_velocity", "blue_noise")}
    planes.update(out_radiance=rad.data_ptr(), out_direction=dirs.data_ptr(), noise_width=64, noise_height=64)
    d = D.reflections_desc(W, H, cam, planes, environment_multiplier=1.0)
    ctx.synchronize()
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    for _ in range(2):
        ctx.rt_reflections(d, side.cuda_stream)
    reps = 10
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(side)
    for _ in range(reps):
        ctx.rt_reflections(d, side.cuda_stream)
    e1.record(side)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    # the pixels k_refl_setup traces, in its fp32 arithmetic: depth < 1 - 1e-6 and
    # roughness = material.r / 255 below the descriptor's no-tracing roughness
    depth_ok = g["depth"].astype(np.float32) < np.float32(1.0) - np.float32(1e-6)
    rough = g["material"][..., 0].astype(np.float32) / np.float32(255.0)
    traced = int((depth_ok & (rough < np.float32(d.no_tracing_roughness))).sum())
    return {
        "workload": f"{W}x{H} pixels ({traced} traced), synthetic G-buffer, C4 scene + atlases",
        "gpu_ms": round(ms, 4),
        "mrays_per_s": round(traced / ms / 1e3, 1),
        "note": "ray-list pipeline: setup (G-buffer -> compacted ray list) -> persistent closest-hit traversal (k_trace<ListRays>, ballot refill) -> shadow-ray list + any-hit traversal -> shading + DDGI lookup; timed over all five launches",
    }


def lighting_compose_line(args, torch, ctx):
    """The DDGI consumer: ark_ddgi_lighting_compose at
    compose_size on the C4 context's atlases after the timed steps, every flag on,
    a seeded synthetic G-buffer resident in HBM. Timed with HIP events on the stream
    the kernel runs on (torch's current stream is passed to the C-ABI)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import compose_inputs as CI
    from arkoserenderer_amd import abi

    W, H = (int(v) for v in args.compose_size.split("x"))
    g = CI.gbuffer(W, H, seed=5)
    dev = {k: torch.from_numpy(v).cuda() for k, v in g.items()}
    out = torch.empty((H, W, 4), dtype=torch.int16, device="cuda")
    cam = CI.camera(W, H, eye=(16.0, 16.0, -6.0), target=(16.0, 14.0, 16.0))
    planes = {k: t.data_ptr() for k, t in dev.items()}
    ctx.synchronize()
    torch.cuda.synchronize()
    side = torch.cuda.Stream()  # a real stream handle (the null stream would map to the ctx stream)
    stream = side.cuda_stream
    for _ in range(3):
        ctx.lighting_compose(W, H, abi.ARK_COMPOSE_DEFAULT_FLAGS, cam, planes, out.data_ptr(), stream)
    reps = 20
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(side)
    for _ in range(reps):
        ctx.lighting_compose(W, H, abi.ARK_COMPOSE_DEFAULT_FLAGS, cam, planes, out.data_ptr(), stream)
    e1.record(side)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    px = W * H
    plane_bytes = sum(v.nbytes for v in g.values()) + px * 8  # G-buffer in + RGBA16F out
    return {
        "workload": f"{W}x{H} pixels, all flags, synthetic G-buffer, C4 atlases (32^3 probes)",
        "gpu_ms": round(ms, 4),
        "mpixels_per_s": round(px / ms / 1e3, 1),
        "roofline": {"bound": "hbm", "achieved": round(plane_bytes / (ms * 1e-3) / 1e9, 1), "peak": 8000.0, "unit": "GB/s",
                     "frac": round(plane_bytes / (ms * 1e-3) / 1e9 / 8000.0, 4),
                     "algorithmic_bytes": plane_bytes, "note": "G-buffer planes + output; atlas taps (L2-resident) excluded"},
    }


def ao_bake_c1(args, torch, device):
    """Config C1: AO bake of DamagedHelmet (15,452 triangles) at
    ao_size^2 texels x ao_samples rays, on the GPU (ark_ddgi_bake_ao, wall-clock
    timed around the three passes) and on the host cores with the CPU
    oracle (the repo's own CPU AO ray path; a bounded band of rows, same rules,
    bit-identical results). Rays = covered texels x samples."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import numpy as np

    import oracle_lib as O
    from arkoserenderer_amd import abi
    from arkoserenderer_amd import ddgi as D
    from arkoserenderer_amd import scene as S
    from parity import make_desc

    W = H = args.ao_size
    n_s = args.ao_samples
    scene = S.damaged_helmet()
    grid = D.ProbeGrid((1, 1, 1), (1.0, 1.0, 1.0), (0.0, 0.0, 0.0))
    cfg = D.DDGIConfig(rays_per_probe=1, probe_updates_per_frame=1, max_rays_per_probe=1, max_probe_updates=1)
    ctx = D.DDGIContext(grid, 100.0, cfg, device=device.index or 0)
    ctx.set_scene(scene)
    ctx.bake_ao(0, W, H, n_s, False)  # warm-up (context stream)
    ctx.synchronize()
    reps = 3
    t0 = time.perf_counter()
    for _ in range(reps):
        ctx.bake_ao(0, W, H, n_s, False)
    ctx.synchronize()
    gpu_ms = (time.perf_counter() - t0) / reps * 1e3
    tri = ctx.bake_read(abi.ARK_BAKE_TRIANGLE_INDEX)
    covered = int(np.count_nonzero(tri))
    gpu_out = ctx.bake_read(abi.ARK_BAKE_OUTPUT)
    ctx.close()
    res = {"workload": f"C1: DamagedHelmet AO bake {W}x{H} texels x {n_s} samples ({covered} covered texels)",
           "gpu_mrays_s": round(covered * n_s / (gpu_ms * 1e-3) / 1e6, 2), "gpu_ms": round(gpu_ms, 3)}
    if args.no_cpu_baseline:
        return res
    threads = args.cpu_threads or cpu_cores()[0]
    orc = O.Oracle(make_desc(grid, 100.0, cfg))
    orc.set_scene(scene, threads)
    row0, rows, spent, rays, exact = 0, 4, 0.0, 0, True
    while spent < args.ao_cpu_seconds and row0 < H:
        r1 = min(H, row0 + rows)
        t = time.perf_counter()
        otri, _, out = orc.bake_ao(0, W, H, n_s, False, rows=(row0, r1), threads=threads)
        el = time.perf_counter() - t
        spent += el
        rays += int(np.count_nonzero(otri[row0:r1])) * n_s
        exact = exact and np.array_equal(out[row0:r1], gpu_out[row0:r1])
        row0 = r1
        rows = int(max(4, rows * min(4.0, args.ao_cpu_seconds / 3 / max(el, 1e-3))))
    orc.close()
    res["cpu_baseline"] = {"value": round(rays / spent / 1e6, 3), "unit": "Mrays/s", "cores": threads, "kind": "port",
                           "sample": f"rows 0..{row0 - 1} of the same bake ({rays} rays, {spent:.1f} s, parameterization passes included)",
                           "bit_exact_vs_gpu": bool(exact)}
    return res


if __name__ == "__main__":
    sys.exit(main())
