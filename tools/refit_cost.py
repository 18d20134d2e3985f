"""Cost of the per-frame instance update (ark_ddgi_set_instances) at
C4 (10 M-triangle soup, 16 instances, 32^3 x 256) and the C3 substitute: the refit's
wall time and its device part (ArkDdgiBvhStats.refit_ms), and the update throughput
before and after - one instance moved by 0.5 m, then every instance rotated by 2 deg
about y (the refit keeps the topology, so the boxes loosen with the motion).

    python tools/refit_cost.py [--config c4 c3] [--steps 5]
    python tools/refit_cost.py --continuous [--frames 300] [--config c4 c3]

--continuous (VERDICT r05 "do this" #3): the static rate, then `frames` frames that each
move one instance (ark_ddgi_set_instances_async on the update's stream, no host wait)
- the rate under motion, the background rebuilds installed meanwhile - then static
frames until the rebuilds of the final state (world BVHs and the light-space sun BVH)
are installed, and the rate again: it should be back at the static rate.
"""
import argparse
import dataclasses
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def build(name):
    from arkoserenderer_amd import ddgi as D
    from arkoserenderer_amd import scene as S
    if name == "c4":
        return S.soup(10_000_000), D.ProbeGrid((32, 32, 32), (1.0, 1.0, 1.0), (0.0, 0.0, 0.0)), 256, 10000.0
    return S.sponza_substitute(), D.ProbeGrid(*S.sponza_substitute_grid()), 256, 10000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", nargs="+", default=["c4", "c3"])
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--continuous", action="store_true", help="one instance moved every frame for --frames frames, then back to static")
    ap.add_argument("--frames", type=int, default=300)
    ap.add_argument("--no-background", action="store_true", help="ARK_DDGI_FLAG_NO_BACKGROUND_REBUILD: refits only (isolates the rebuild threads' cost)")
    ap.add_argument("--sun-turn", action="store_true", help="instead of refits: turn the sun by 10 deg, wait for the background rebuild, turn it back, wait again")
    args = ap.parse_args()
    import torch
    from arkoserenderer_amd import ddgi as D

    torch.cuda.set_device(0)
    for name in args.config:
        sc, grid, R, zf = build(name)
        N = grid.probe_count()
        cfg = D.DDGIConfig(rays_per_probe=R, probe_updates_per_frame=N, max_rays_per_probe=R, max_probe_updates=N, compute_probe_offsets=True,
                           background_rebuild=not args.no_background)
        node = D.DDGINode(cfg)
        node.construct(sc, grid, zf, light_pre_exposure=1.0, ambient_illuminance=0.02, environment_brightness=1.0)
        app = [D.AppState(0)]

        def rate(nd=None):
            nd = nd or node
            for _ in range(2):
                nd.execute(app[0])
                app[0] = D.AppState(app[0].frame_index + 1)
            nd.ctx.synchronize()
            t = time.perf_counter()
            for _ in range(args.steps):
                nd.execute(app[0])
                app[0] = D.AppState(app[0].frame_index + 1)
            nd.ctx.synchronize()
            return N * R * args.steps / (time.perf_counter() - t) / 1e6

        had_sun_bvh = node.ctx.bvh_stats().sun_node_count > 0
        out = {"config": name, "triangles": int(sc.triangle_count), "instances": int(sc.instances.size),
               "build_ms": round(node.ctx.bvh_stats().build_ms, 1), "mrays_per_s_static": round(rate(), 1)}
        if args.continuous:
            sptr = torch.cuda.current_stream().cuda_stream
            static = [out["mrays_per_s_static"], round(rate(), 1)]
            inst0 = sc.instances.copy()
            n = len(inst0)
            st0 = node.ctx.bvh_stats()
            node.ctx.synchronize()
            stream = torch.cuda.current_stream()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.frames)]
            host_refit = 0.0
            t = time.perf_counter()
            for f in range(args.frames):
                inst = inst0.copy()
                m = inst["object_to_world"].reshape(-1, 3, 4)
                m[f % n, 0, 3] += np.float32(0.3 * np.sin(0.1 * f))  # one instance a frame, back and forth
                m[(f // n) % n, 2, 3] += np.float32(0.2)               # and one left displaced for n frames
                inst["object_to_world"] = m.reshape(-1, 12)
                ev[f][0].record(stream)
                th = time.perf_counter()
                node.ctx.set_instances_async(inst, sptr)
                host_refit += time.perf_counter() - th
                ev[f][1].record(stream)
                node.execute(app[0], sptr)
                app[0] = D.AppState(app[0].frame_index + 1)
                if f % 50 == 49:
                    print(json.dumps({"frame": f + 1, "elapsed_s": round(time.perf_counter() - t, 2)}), flush=True)
            node.ctx.synchronize()
            motion_s = time.perf_counter() - t
            st1 = node.ctx.bvh_stats()
            refit_dev = sorted(e0.elapsed_time(e1) for e0, e1 in ev)
            # static again: until BVHs built from the final records (after the last refit)
            # are installed - the world BVHs and the light-space sun BVH
            t = time.perf_counter()
            while time.perf_counter() - t < 120.0 and not args.no_background:
                st = node.ctx.bvh_stats()
                if st.bvh_built_refit_version == st.refit_version and (not had_sun_bvh or st.sun_built_refit_version == st.refit_version):
                    break
                node.execute(app[0], sptr)
                app[0] = D.AppState(app[0].frame_index + 1)
                node.ctx.synchronize()
                time.sleep(0.01)
            settle_s = time.perf_counter() - t
            st2 = node.ctx.bvh_stats()
            after = [round(rate(), 1) for _ in range(2)]
            # a context built from scratch on the final transforms, measured interleaved
            # with the rebuilt one: what "back at the static rate" means for the moved scene
            fresh_node = D.DDGINode(cfg)
            fresh_node.construct(dataclasses.replace(sc, instances=inst), grid, zf, light_pre_exposure=1.0, ambient_illuminance=0.02, environment_brightness=1.0)
            fresh = []
            for _ in range(3):
                fresh.append(round(rate(fresh_node), 1))
                after.append(round(rate(), 1))
            fresh_node.ctx.close()
            out["continuous"] = {
                "frames": args.frames, "mrays_per_s_moving": round(N * R * args.frames / motion_s / 1e6, 1),
                "ms_per_frame_moving": round(motion_s / args.frames * 1e3, 4),
                "refit_device_ms": {"median": round(refit_dev[len(refit_dev) // 2], 4), "max": round(refit_dev[-1], 4)},
                "refit_host_enqueue_ms": round(host_refit / args.frames * 1e3, 4), "background_rebuild": not args.no_background,
                "built_refit_version": {"world": int(st2.bvh_built_refit_version), "sun": int(st2.sun_built_refit_version), "refits": int(st2.refit_version)},
                "installs_while_moving": {"world": int(st1.bvh_rebuilds - st0.bvh_rebuilds), "sun": int(st1.sun_rebuilds - st0.sun_rebuilds)},
                "world_rebuild_ms": round(st2.bvh_rebuild_ms, 1), "sun_rebuild_ms": round(st2.sun_build_ms, 1),
                "settled_after_s": round(settle_s, 2), "sun_bvh_installed": bool(st2.sun_node_count > 0),
                "mrays_per_s_static_before": static, "mrays_per_s_static_after": after,
                "after_vs_before": round(max(after) / max(static), 4), "mrays_per_s_fresh_build": fresh,
                "after_vs_fresh": round(sorted(after)[len(after) // 2] / sorted(fresh)[1], 4)}
            print(json.dumps(out), flush=True)
            node.ctx.close()
            continue
        if args.sun_turn:
            turns = []
            base = node.ctx.bvh_stats().sun_rebuilds
            d0 = np.array(sc.sun[1], np.float64)
            c, s_ = np.cos(np.radians(10.0)), np.sin(np.radians(10.0))
            d1 = np.array([c * d0[0] + s_ * d0[2], d0[1], -s_ * d0[0] + c * d0[2]])
            for label, d in (("turned", d1), ("back", d0)):
                node.ctx.set_lights((sc.sun[0], tuple(float(x) for x in d)), ())
                world = rate()  # the world BVHs carry the sun's rays meanwhile
                t = time.perf_counter()
                while node.ctx.bvh_stats().sun_rebuilds == base and time.perf_counter() - t < 60.0:
                    node.execute(app[0])
                    app[0] = D.AppState(app[0].frame_index + 1)
                    node.ctx.synchronize()
                base = node.ctx.bvh_stats().sun_rebuilds
                turns.append({"sun": label, "mrays_per_s_world": round(world, 1), "installed_after_s": round(time.perf_counter() - t, 2),
                              "rebuild_ms": round(node.ctx.bvh_stats().sun_build_ms, 1), "mrays_per_s_rebuilt": round(rate(), 1)})
            out["sun_turns"] = turns
            print(json.dumps(out), flush=True)
            node.ctx.close()
            continue
        inst = sc.instances.copy()
        moves = []
        inst["object_to_world"][0, 3] += 0.5
        c, s_ = np.cos(np.radians(2.0)), np.sin(np.radians(2.0))
        rot = np.array([[c, 0, s_], [0, 1, 0], [-s_, 0, c]], np.float32)
        for label in ("one_moved", "all_rotated"):
            if label == "all_rotated":
                m = inst["object_to_world"].reshape(-1, 3, 4)
                m[:] = np.einsum("ij,njk->nik", rot, m)
                inst["object_to_world"] = m.reshape(-1, 12)
            node.ctx.synchronize()
            t = time.perf_counter()
            node.ctx.set_instances(inst)
            wall = (time.perf_counter() - t) * 1e3
            st = node.ctx.bvh_stats()
            moves.append({"move": label, "set_instances_ms": round(wall, 2), "refit_ms": round(st.refit_ms, 2), "mrays_per_s": round(rate(), 1)})
        out["refits"] = moves
        # the light-space sun BVH, dropped by the refit, comes back from the background
        # rebuild (sunRebuildStep): frames until it is installed, then the rate again
        st = node.ctx.bvh_stats()
        if had_sun_bvh:
            t = time.perf_counter()
            while node.ctx.bvh_stats().sun_rebuilds == st.sun_rebuilds and time.perf_counter() - t < 60.0:
                node.execute(app[0])
                app[0] = D.AppState(app[0].frame_index + 1)
                node.ctx.synchronize()
            s2 = node.ctx.bvh_stats()
            out["sun_rebuild"] = {"installed_after_s": round(time.perf_counter() - t, 2), "rebuild_ms": round(s2.sun_build_ms, 1),
                                  "sun_nodes": int(s2.sun_node_count), "mrays_per_s": round(rate(), 1)}
        print(json.dumps(out), flush=True)
        node.ctx.close()


if __name__ == "__main__":
    main()
