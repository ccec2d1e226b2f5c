#!/usr/bin/env python3
"""bench.py — frames/s of the ORB-YGZ-SLAM front-end hot path on MI355X.

Metric (BASELINE.json): frames/sec ORB-extract + SparseImageAlign, 752x480,
1000 features, 1/2/4/8 GPUs.  Default workload = BASELINE config C5, the
offline batched-sequence mode: the 13,728 frames of EuRoC MH01..MH05
(Examples/Monocular/EuRoC_TimeStamps/MH0*.txt: 3682+3040+2700+2033+2273) as a
synthetic sequence (a rendered textured plane under a back-and-forth camera
sweep, EuRoC intrinsics; no dataset in the image), sharded contiguously over
the ranks (one process per GPU).  One "step" = the whole job over the
sequence, per rank on its shard plus a one-frame halo:
  * ORB extraction (C2: nFeatures 1000, scale 2.0, 4 levels, FAST 20/7) --
    pyramid, blur, FAST-9 cells, octree, angle + rBRIEF;
  * Hamming best/second-best of frame k against frame k-1;
  * SparseImgAlign k-1 -> k (C3: levels 3..1, 10 GN iterations), map points =
    frame k-1's keypoints back-projected on the plane;
  * the per-frame result slots (keypoints, descriptors, TCR) packed on the
    device and gathered to rank 0 over RCCL (`torch.distributed.gather`).
Frames are rendered on the device into HBM before the timed region.  `value` =
13,728 / the slowest rank's step time ("scaling": "strong": the job is fixed).
`--workload c2batch` is round 1's form instead: `--batch` frames per GPU
(weak scaling), same stages.

`--gpus N` without torchrun spawns the N ranks itself (torch.distributed.run,
127.0.0.1) before anything touches a GPU; under torchrun WORLD_SIZE must equal
--gpus, and fewer visible GPUs than --gpus is an error, never a silent N=1 run.

The JSON line also carries `roofline` (dominant kernel: algorithmic bytes per
launch / HIP-event-timed average launch duration vs 8 TB/s, plus the VALU
issue fraction from the committed PMC pass) and `cpu_baseline` (the oracle/
CPU restatement on the host cores, 1 thread and all threads, on a bounded
sample of the same workload).
"""
import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "orb-ygz-slam_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
from ygzfe.sequence import C2, C5_FRAMES, XI, C5Shard, sweep_index  # noqa: E402


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=["c5", "c2batch"], default="c5",
                    help="c5: the 13,728-frame MH01..05 sequence sharded over the ranks + RCCL gather (strong); "
                         "c2batch: --batch frames per GPU (weak)")
    ap.add_argument("--frames", type=int, default=0, help="c5 sequence length override (0 = 13,728)")
    ap.add_argument("--batch", type=int, default=1024, help="c2batch: frames per GPU")
    ap.add_argument("--cpu-sample", type=int, default=120, help="frames in the CPU-baseline sample (0 = skip)")
    ap.add_argument("--cpu-budget-s", type=float, default=20.0)
    ap.add_argument("--no-align", action="store_true")
    ap.add_argument("--graph", type=int, default=0,
                    help="1: capture one step into a HIP graph and replay it (measured: same throughput as eager launches)")
    ap.add_argument("--schedule", choices=["split", "overlap", "tail", "serial", "pipe"], default="pipe",
                    help="the timed steps' schedule. split: blur + descriptors + Hamming on a side stream "
                         "beside FAST / octree, SparseImgAlign after them; overlap: SparseImgAlign beside "
                         "orient + Hamming too; tail: the extraction on one stream, then Hamming on a side "
                         "stream beside SparseImgAlign; serial: every stage on one stream; pipe: the shard in chunks "
                         "(default 4), chunk c + 1's pyramid / FAST / octree beside chunk c's descriptors, "
                         "Hamming and SparseImgAlign.  The per-stage "
                         "roofline pass always runs serial (one kernel on the GPU at a time)")
    ap.add_argument("--chunks", type=int, default=0,
                    help="process each rank's shard in this many chunks (each its own batch), gathering a "
                         "chunk's result slots on a communication stream while the next chunk computes "
                         "(default: 4 under the pipe schedule or when N > 1, else 1 = one batch)")
    ap.add_argument("--no-undistort", action="store_true", help="skip the undistort-remap side measurement")
    ap.add_argument("--no-stage-timing", action="store_true", help="no per-stage hipEvents in the timed region")
    ap.add_argument("--no-bow", action="store_true", help="skip the DBoW2-transform side measurement")
    ap.add_argument("--no-stereo", action="store_true", help="skip the stereo-matching side measurement")
    ap.add_argument("--no-a11", action="store_true", help="skip the tracking-path searches line (row a11)")
    ap.add_argument("--no-dropin", action="store_true", help="skip the drop-in call-site timing line")
    ap.add_argument("--no-direct", action="store_true", help="skip the SearchLocalPointsDirect side measurement")
    ap.add_argument("--no-c4", action="store_true", help="skip the C4 (TUM 640x480, 2000 features) throughput line")
    ap.add_argument("--latency-frames", type=int, default=200,
                    help="single-frame latency leg: frames timed one at a time through the host C ABI (0 = skip)")
    return ap.parse_args()


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def self_launch(args):
    """`--gpus N` run directly: start N ranks with torch.distributed.run as a child
    (no GPU has been touched in this process: torch.cuda.device_count() does not
    initialise HIP on this image) and exit with its status."""
    import torch
    n_vis = torch.cuda.device_count()
    if n_vis < args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} needs {args.gpus} visible GPUs, {n_vis} visible; refusing to "
                 f"report a smaller run")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    sys.exit(subprocess.call(cmd, env=env))


def main():
    args = parse()
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        return self_launch(args)
    world = int(world_env or "1")
    if world != args.gpus:
        sys.exit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}: launch one rank per GPU")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist

    import ygzfe
    from ygzfe import dist as D
    import _scenes as S

    if torch.cuda.device_count() < max(args.gpus, local + 1):
        sys.exit(f"bench.py: rank {rank} needs GPU {local}; {torch.cuda.device_count()} visible")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
        if dist.get_world_size() != args.gpus:
            sys.exit(f"bench.py: RCCL sees {dist.get_world_size()} ranks, --gpus {args.gpus}")
        one = torch.ones(1, device=dev)
        dist.all_reduce(one)
        if int(one.item()) != args.gpus:
            sys.exit(f"bench.py: all_reduce over RCCL counted {int(one.item())} ranks, expected {args.gpus}")

    W, H, nf, sf, nl, ini, mn = C2
    n_seq = (args.frames or C5_FRAMES) if args.workload == "c5" else world * args.batch
    n_chunks = args.chunks if args.chunks > 0 else (4 if (world > 1 or args.schedule == "pipe") else 1)
    t_r = time.time()
    # the rank's whole C5 job (ygzfe/sequence.py; tests/test_gpu_c5.py runs the same object)
    shard = C5Shard(n_seq, rank, world, dev, chunks=n_chunks, schedule=args.schedule, align=not args.no_align)
    render_s = time.time() - t_r
    torch.cuda.set_stream(shard.stream)
    stream, sptr = shard.stream, shard.sptr
    batch, cap = shard.batch, shard.cap
    b0, h, F, n_own, P = shard.b0, shard.h, shard.F, shard.n_own, shard.P
    poses, sc, r3, cz = shard.poses, shard.sc, shard.r3, shard.cz
    pyr_t, counts_t, out = shard.pyr_t, shard.counts_t, shard.out
    chunks, batches, F_ext = shard.chunks, shard.batches, shard.F_ext
    S_b = shard.slot_bytes
    gather_ms = shard.gather_ms
    step = shard.step
    check_all = shard.check
    timing_all = shard.timing

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    check_all()
    if world > 1:
        dist.barrier()
    timing_all(False)  # `value`: no per-stage events inside the timed region
    run = step
    graph_ok = False
    if args.graph and world == 1 and not chunks:
        # one step captured as a HIP graph (every launch of the library, its
        # fork/join events and the side streams), replayed per step
        try:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=stream):
                step()
            g.replay()
            torch.cuda.synchronize(dev)
            batch.check()
            run = g.replay
            graph_ok = True
        except Exception as e:  # capture unsupported: eager launches
            print(f"bench: graph capture failed ({e}); eager launches", file=sys.stderr)
            torch.cuda.synchronize(dev)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    check_all()
    elapsed = D.max_over_ranks(elapsed, dev)
    # roofline: the same K steps again with hipEvents around every stage launch
    # (a stage event between two kernels adds ~10 us of dispatch gap, so they
    # stay out of the throughput run)
    stage_ms = {}
    if not args.no_stage_timing:
        # serial: each stage's events bracket one kernel that has the GPU to itself (under
        # overlap a stage's time would include its neighbour's share of the GPU)
        shard.schedule = "serial"
        timing_all(True)
        torch.cuda.synchronize(dev)
        for _ in range(args.steps):
            step(timed_gather=True)
        torch.cuda.synchronize(dev)
        stage_ms = timing_all(False)
        shard.schedule = args.schedule
        check_all()
        if gather_ms:
            stage_ms["rccl_gather"] = float(np.mean([a.elapsed_time(b) for a, b in gather_ms]))
        if world > 1:
            dist.barrier()

    ms_per_step = elapsed * 1000.0 / args.steps
    fps = n_seq / (elapsed / args.steps)

    # ------------------------------------------------ results check: rank 0 holds every frame's slot
    seq_check = None
    if rank == 0:
        full = shard.root_slots()
        hdr = full[:, :64].contiguous().view(torch.int32).cpu().numpy()
        seq_check = {"frames_at_root": int(full.shape[0]),
                     "frame_index_ok": bool(np.array_equal(hdr[:, 10], np.arange(n_seq))),
                     "frames_with_align": int(hdr[:, 11].sum()),
                     "mean_kps_at_root": round(float(hdr[:, 0].mean()), 1),
                     "slot_bytes": S_b}

    # ------------------------------------------------ roofline (dominant stage)
    counts = shard.counts().cpu().numpy()
    nvis = out[:max(P, 1), 7].contiguous().view(torch.int32).cpu().numpy() if P > 0 else np.zeros(1, np.int32)
    plan = ygzfe.orb_plan(nf, sf, nl, ini, mn, W, H)
    areas = [w * hh for w, hh in plan["sizes"]]
    if chunks:  # per-level totals over every chunk batch's last extract (lead frames included)
        cand = selk = 0
        for ch in chunks:
            if ch[3] > 0:
                cc_, ss_ = ch[4].stats(ch[1])
                cand, selk = cand + cc_, selk + ss_
    else:
        cand, selk = batch.stats(F)  # per-level totals over the F frames of the last extract
    N = float(counts.mean())
    nv = float(nvis.mean())
    ncells_tot = int(sum(plan["ncells"]))
    # algorithmic bytes per launch (per step, F frames): each intermediate crosses
    # HBM once written and once read
    # With the all-area pyramid of C2 the batch path forms levels 1..3 in the level-0 blur
    # strips (extract.hip k_blur7 fused mode): its "pyramid" stage reads level 0 once and
    # writes levels 1..3 and the blurred level 0; "blur7" is the other levels' blur.
    fused = os.environ.get("YGZFE_PYR_UNFUSED") is None and sf == 2.0 and nl <= 4 and W % 4 == 0
    alg = {
        "pyramid": F_ext * (2 * areas[0] + sum(areas[1:])) if fused else
        F_ext * sum(areas[l - 1] + areas[l] for l in range(1, nl)),
        "blur7": F_ext * 2 * sum(areas[1:] if fused else areas),
        "fast9_cells": F_ext * sum(a for a, c in zip(areas, plan["ncells"]) if c > 0) + 4 * int(cand.sum())
        + 4 * F_ext * ncells_tot,
        "octree": 4 * int(cand.sum()) + 4 * F_ext * ncells_tot + 4 * int(selk.sum()),
        "orient_rbrief": int(counts.sum()) * (961 + 512 + 4 + 60),
        "hamming_best2": int(sum(32 * (counts[i + 1] + counts[i]) + 12 * counts[i + 1] for i in range(P))),
        "sparse_align": int(P * (3 * nv * (36 + 10 * 25) + 12 * nv + 96)),
        "pack_slots": int(n_own * (2 * S_b)),
    }
    if not any(v > 0 for k, v in stage_ms.items() if k in alg):  # --no-stage-timing
        stage_ms = {k: 1e-9 for k in alg}
    dom = max((k for k in stage_ms if k in alg and stage_ms[k] > 0), key=lambda k: stage_ms[k])
    n_batches = max(1, len(batches))
    dom_ms = stage_ms[dom]
    achieved = alg[dom] / (dom_ms * 1e-3) / 1e9
    traffic = valu_frac = None
    pmc = {}
    # the newest round's PMC pass (profiles/rNN_traffic.json)
    tcands = sorted(f for f in os.listdir(os.path.join(ROOT, "profiles")) if f.endswith("_traffic.json"))
    tpath = os.path.join(ROOT, "profiles", tcands[-1]) if tcands else ""
    if tpath and os.path.exists(tpath):  # PMC FETCH_SIZE x2 + WRITE_SIZE of the same kernel (tools/run_pmc.sh)
        tj = json.load(open(tpath))
        per = tj.get("per_frame", {}).get(dom)
        if per is not None:  # scaled to this launch's frame count
            traffic = int(per["traffic_bytes"] * F / n_batches)
            valu_frac = per.get("valu_frac")
            pmc = {k: per[k] for k in ("wait_inst_frac", "wait_any_frac", "lds_conflict_per_inst") if k in per}
            pmc["source"] = os.path.basename(tpath)
        elif dom in tj.get("per_step", {}):
            traffic = tj["per_step"][dom]["traffic_bytes"]
    roof = {"kernel": dom, "bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 5), "traffic": traffic, "valu_frac": valu_frac,
            # what binds the dominant kernel below its HBM roofline: for FAST, VALU issue
            # and LDS / load latency, not HBM bandwidth (the PMC figures of the same kernel beside it)
            "binding": BINDING.get(dom, "see DESIGN.md section 4"), "pmc": pmc or None,
            # one "launch" = the stage over one batch: with chunks, each chunk's batch (its FAST = one
            # kernel per pyramid level), n_batches of them per step; stages_ms are per-step sums
            "avg_launch_ms": round(dom_ms / n_batches, 4), "alg_bytes_per_launch": int(alg[dom] / n_batches),
            "frames_per_launch": round(F_ext / n_batches, 1), "launches_per_step": n_batches,
            "stages_ms": {k: round(v, 4) for k, v in stage_ms.items()},
            "stages_gbps": {k: round(alg[k] / (stage_ms[k] * 1e-3) / 1e9, 1) for k in alg if stage_ms.get(k, 0) > 0}}
    # whole pipeline, SURVEY §8d model: (B_extract + B_align) per frame x fps
    b_extract = areas[0] + 2 * sum(areas[1:]) + 2 * sum(areas) + 60 * N
    b_align = 3 * nv * (36 + 10 * 25) + 12 * nv + 96
    pipeline_gbps = (b_extract + b_align) * (fps / world) / 1e9

    # host copies of a bounded prefix of the rendered sequence for the single-frame legs
    # and the CPU baseline (its multi-thread leg gets ~24 frames per host thread)
    n_host = 0
    if rank == 0 and world == 1:
        n_host = min(F, max(args.cpu_sample, args.latency_frames + 12, 16,
                            24 * cpu_threads() if args.cpu_sample > 0 else 0))
    frames = np.stack([batch.read_level(i, 0) for i in range(n_host)]) if n_host else None

    # ------------------------------------------------ §8(f) rank 1: undistort remap
    # (not part of the headline metric; Frame.cc:775-790 runs it ahead of the
    # pyramid on every EuRoC frame): raw frames resident in HBM -> level-0 slots
    und_line = None
    if not args.no_undistort:
        import _cameras as CAM
        ucam, udist, _ = CAM.EUROC
        und = ygzfe.Undistort(ucam, udist, W, H, device=local)
        Bu = min(F, 1024)
        raw = pyr_t.view(-1, batch.frame_pitch)[:Bu, :W * H].contiguous()  # level 0 of the first Bu frames
        for _ in range(2):
            batch.undistort_device(und, raw.data_ptr(), W * H, Bu, sptr)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = max(args.steps, 5)
        ev0.record(stream)
        for _ in range(reps):
            batch.undistort_device(und, raw.data_ptr(), W * H, Bu, sptr)
        ev1.record(stream)
        torch.cuda.synchronize(dev)
        ums = ev0.elapsed_time(ev1) / reps
        ualg = Bu * W * H * 2  # each frame read once and written once (map: cache-resident, shared)
        ugbps = ualg / (ums * 1e-3) / 1e9
        und_line = {"kernel": "remap_tiles", "frames": Bu, "frames_per_s": round(Bu / (ums * 1e-3), 1),
                    "ms_per_launch": round(ums, 4), "alg_bytes_per_launch": ualg, "achieved_gbps": round(ugbps, 1),
                    "frac": round(ugbps / HBM_PEAK_GBPS, 4), "camera": "EuRoC (Examples/Monocular/EuRoC.yaml)"}
        if frames is not None and args.cpu_sample > 0:
            import _oracle as O
            m1, m2 = O.undistort_map(ucam, udist, W, H)
            t_c = time.perf_counter()
            nrm = 0
            while nrm < 8 or time.perf_counter() - t_c < 0.5:
                O.remap_linear(frames[nrm % len(frames)], m1, m2)
                nrm += 1
            und_line["cpu_port_frames_per_s"] = round(nrm / (time.perf_counter() - t_c), 1)

    # ------------------------------------------------ §8(f) rank 2: SearchLocalPointsDirect
    direct_line = None
    if rank == 0 and world == 1 and not args.no_direct:
        direct_line = direct_leg(S, args.cpu_sample > 0)

    # ------------------------------------------------ §8(a) row a11: the tracking-path searches
    a11_line = None
    if rank == 0 and world == 1 and not args.no_a11:
        a11_line = tracking_search_leg(S, args.cpu_sample > 0)

    # ------------------------------------------------ §8(f) rank 3: stereo matching
    stereo_line = None
    if rank == 0 and world == 1 and not args.no_stereo:
        stereo_line = stereo_leg(S, dev, args.cpu_sample > 0)

    # ------------------------------------------------ §8(f) rank 4: DBoW2 transform (Frame::ComputeBoW)
    bow_line = None
    if rank == 0 and world == 1 and not args.no_bow:
        # the descriptors of an extracted batch: with chunks that is a chunk's batch (the
        # shard-wide `batch` then only owns the rendered level 0 and the slot packing)
        ext = [ch for ch in chunks if ch[3] > 0] if chunks else None
        bow_b, bow_F = (ext[0][4], ext[0][1]) if ext else (batch, F)
        bow_line = bow_leg(S, bow_b, min(bow_F, 1024), dev, stream, args.cpu_sample > 0)

    # ------------------------------------------------ C4 throughput (TUM1.yaml, batched 256 frames)
    c4_line = None
    if rank == 0 and world == 1 and not args.no_c4:
        c4_line = c4_leg(S, dev, args)

    # ------------------------------------------------ single-frame latency (rank 0, N = 1)
    lat = None
    if rank == 0 and world == 1 and args.latency_frames > 0:
        lat = latency_leg(frames, poses, sc, S, args.latency_frames)

    # ------------------------------------------------ CPU baseline (rank 0, N = 1)
    cpu = None
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        cpu = cpu_baseline(frames, r3[:n_host], cz[:n_host], S, args, sc)

    # the drop-in headers (compat/dropin) timed through the reference's own call sites
    # (tests/dropin/dropin_calls --time), beside the oracle's loops: part of the CPU-baseline
    # leg, since that program also runs the oracle (as its checker and as the CPU side)
    dropin = None
    if rank == 0 and world == 1 and args.cpu_sample > 0 and not args.no_dropin:
        dropin = dropin_leg()
    if lat is not None and cpu is not None:
        cpu_lat = cpu["ms_pyramid"] + cpu["ms_extract"] + cpu["ms_align"]
        lat["cpu_port_ms"] = round(cpu_lat, 3)
        lat["speedup_vs_cpu_port"] = round(cpu_lat / lat["median_ms"], 2)
    if rank == 0:
        wl = (f"C5 offline sequence: {n_seq} frames (EuRoC MH01..05 length) sharded over {world} GPU(s), per frame "
              f"C2 extract + dense Hamming (k vs k-1) + C3 SparseImgAlign levels 3..1, device-packed result slots "
              f"gathered to rank 0 over RCCL") if args.workload == "c5" else \
             (f"C2 batch: {args.batch} frames per GPU, extract + dense Hamming (k vs k-1) + C3 SparseImgAlign "
              f"levels 3..1 + result slots")
        line = {
            "metric": "frames/sec ORB-extract+SparseImageAlign, 752x480, 1000 feat",
            "value": round(fps, 2),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "strong" if args.workload == "c5" else "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (seeded textured-plane renders on the device, EuRoC intrinsics; no dataset)",
            "config": {"workload": wl, "sequence_frames": n_seq, "frames_per_gpu": n_own,
                       "frames_extracted_per_gpu": F_ext, "chunks": n_chunks, "image": f"{W}x{H}", "nfeatures": nf, "scale_factor": sf,
                       "nlevels": nl, "fast_th": [ini, mn], "align_pairs_per_gpu": P,
                       "mean_keypoints": round(N, 1), "mean_align_visible": round(nv, 1),
                       "mean_fast_candidates": round(float(cand.sum()) / F, 1),
                       "mean_fast_candidates_per_level": [round(float(c) / F, 1) for c in cand],
                       "mean_keypoints_per_level": [round(float(c) / F, 1) for c in selk],
                       "parallelism": f"frame-sharded x{world} (contiguous shards + 1-frame halo)",
                       "collective": (f"RCCL gather of result slots to rank 0 (torch.distributed.gather), "
                                      f"{n_chunks} chunk(s), each gathered on a communication stream while the "
                                      f"next chunk computes") if world > 1 else "none (N=1: rank 0 is the root)",
                       "schedule": (args.schedule if (args.schedule == "pipe" or not shard.chunks)
                                    else "chunked (each chunk serial)"),
                       "schedule_stage_timing": "serial",
                       "schedule_note": ("value times the steps under `schedule`; roofline.stages_ms comes from "
                                         "a separate pass of the same steps (same chunk batches) in the serial "
                                         "schedule (one kernel on the GPU at a time), so the stage times sum to "
                                         "that pass's step, not to ms_per_step"),
                       "hip_graph": graph_ok},
            "roofline": roof,
            "pipeline_gbps_model": round(pipeline_gbps, 2),
            "render_s": round(render_s, 2),
            "sequence_check": seq_check,
            "cpu_baseline": cpu,
            "latency": lat,
            "c4_batched": c4_line,
            "tracking_searches": a11_line,
            "dropin_call_sites": dropin,
            "next_rows": {"undistort_remap": und_line, "search_local_points_direct": direct_line,
                          "stereo_matches": stereo_line, "dbow2_transform": bow_line},
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


# the resource that binds each stage below its HBM roofline (measured: DESIGN.md §4)
BINDING = {
    "fast9_cells": "VALU issue + LDS/load latency (segment test on survivors, per-cell ROI staging)",
    "orient_rbrief": "LDS gather latency at 5 waves/SIMD",
    "sparse_align": "the serial Gauss-Newton chain (one pair per CU)",
    "blur7": "texture/load path",
    "octree": "LDS / barrier latency",
}


def dropin_leg():
    """The drop-in C++ headers through the reference's own call sites (Frame.cc:327-348,
    Tracking.cc:1156-1171, 1662-1674, 2171): tests/dropin/dropin_calls built and run with
    --time.  Each line: median ms per call through the drop-in (host cv::Mat / Frame /
    MapPoint in, results written back into the Frame) and the oracle's literal loops
    (1 thread).  None when the program cannot be built here."""
    import subprocess
    root = os.path.dirname(os.path.abspath(__file__))
    try:
        subprocess.run(["make", "-s", "-C", os.path.join(root, "compat"), "dropin"], check=True, timeout=240,
                       capture_output=True)
        r = subprocess.run([os.path.join(root, "compat", "build", "dropin_calls"), "--time"], capture_output=True,
                           text=True, timeout=240)
    except Exception as e:  # noqa: BLE001 -- reported, never fatal to the bench line
        return {"error": repr(e)[:200]}
    out = {"parity": "ok" if r.returncode == 0 else f"FAILED (rc {r.returncode})"}
    for ln in r.stdout.splitlines():
        f = ln.split()
        if len(f) >= 6 and f[0] == "TIMING" and f[2] == "dropin_ms":
            d = {"dropin_ms": float(f[3]), "oracle_ms": float(f[5])}
            d["speedup_vs_cpu_port"] = round(d["oracle_ms"] / d["dropin_ms"], 2) if d["dropin_ms"] > 0 else None
            for k in range(6, len(f) - 1, 2):  # extra "name value" pairs (counts, time splits)
                d[f[k]] = int(f[k + 1]) if f[k + 1].isdigit() else float(f[k + 1])
            out[f[1]] = d
    out["path"] = ("compat/dropin headers (ORBextractor.h, SparseImageAlign.h, ORBmatcherGPU.h) under the "
                   "reference's call sites, libygzfe.so underneath; CPU side: the oracle, 1 thread")
    return out


def plane_xyz(S, pose, kps, cam):
    """xyz_ref = T_ref * P_w for keypoints on the plane Z_w = PLANE_Z (the Tracking
    snapshot of the reference frame's map points), in reference-camera coordinates."""
    fx, fy, cx, cy = cam
    q, t = pose
    qi, ti = S.se3_inv(q.astype(np.float64), t.astype(np.float64))
    R_wc = np.array([S.quat_rot(qi, e) for e in np.eye(3)]).T
    d = np.stack([(kps["x"] - cx) / fx, (kps["y"] - cy) / fy, np.ones(len(kps))], 1)
    lam = (S.PLANE_Z - ti[2]) / (d @ R_wc[2])
    return np.ascontiguousarray((d * lam[:, None]).astype(np.float32))


def latency_leg(frames, poses, sc, S, n_timed, warm=10):
    """Single-frame latency, the reference's execution model (one Tracking thread,
    SURVEY.md §8d): per frame, host image -> ComputePyramid -> ORB extract ->
    keypoints + descriptors back on the host, and SparseImgAlign(prev -> cur) ->
    pose on the host, through the host C ABI (H2D and D2H included).  Both need
    only the frame's pyramid (the reference runs TrackWithSparseAlignment before
    any extraction, Tracking.cc:471 / 2145-2189), so the align is queued first
    (ygzfe_sparse_align_begin) and runs on its own stream beside the extraction;
    the frame is done when both results are on the host.  The same frames are
    also timed with the two calls back to back (`serial`).  Map points of the
    previous frame (T_ref * P_w) are formed on the host between frames, outside
    the timed region, as Tracking does."""
    import ctypes as C
    import ygzfe
    L = ygzfe.lib()
    W, H, nf, sf, nl, ini, mn = S.CONFIGS["C2"]
    ex = ygzfe.ORBextractor(nf, sf, nl, ini, mn, device=0)
    fr = [ygzfe.Frame(ex, W, H), ygzfe.Frame(ex, W, H)]
    cap = 4096
    kps = [np.zeros(cap, ygzfe.KP_DTYPE) for _ in range(2)]
    desc = [np.zeros((cap, 32), np.uint8) for _ in range(2)]
    n_out = C.c_int()
    cam = sc.camera()
    T0 = ygzfe.SE3.make()
    res = ygzfe.AlignResult()
    p = ygzfe._p
    n_frames = min(len(frames), warm + n_timed + 1)
    out = {}
    for mode in ("overlap", "serial"):
        ts, te = [], []
        prev = None
        for i in range(n_frames):
            cur = i & 1
            img = np.ascontiguousarray(frames[i])
            t0 = time.perf_counter()
            ygzfe._check(L.ygzfe_compute_pyramid(ex.h, fr[cur].h, p(img), W), "compute_pyramid")
            if prev is not None and mode == "overlap":
                pk, xyz, us = prev
                ygzfe._check(L.ygzfe_sparse_align_begin(fr[cur ^ 1].h, fr[cur].h, C.byref(cam), p(pk), p(xyz), p(us),
                                                        len(pk), 3, 1, C.byref(T0)), "sparse_align_begin")
            ygzfe._check(L.ygzfe_extract(ex.h, fr[cur].h, ygzfe.ORBSLAM_KEYPOINT, p(kps[cur]), 0, cap, p(desc[cur]),
                                         C.byref(n_out)), "extract")
            t1 = time.perf_counter()
            if prev is not None:
                if mode == "overlap":
                    ygzfe._check(L.ygzfe_sparse_align_end(fr[cur].h, C.byref(res)), "sparse_align_end")
                else:
                    pk, xyz, us = prev
                    ygzfe._check(L.ygzfe_sparse_align(fr[cur ^ 1].h, fr[cur].h, C.byref(cam), p(pk), p(xyz), p(us),
                                                      len(pk), 3, 1, C.byref(T0), C.byref(res)), "sparse_align")
            t2 = time.perf_counter()
            if i > warm:
                ts.append(t2 - t0)
                te.append(t1 - t0)
            pk = kps[cur][:n_out.value].copy()
            prev = (pk, plane_xyz(S, poses[i], pk, sc.cam), np.ones(len(pk), np.uint8))
        out[mode] = (np.array(ts) * 1e3, np.array(te) * 1e3)
    att, passed = C.c_int(), C.c_int()
    ygzfe._check(L.ygzfe_extractor_align_probe(ex.h, C.byref(att), C.byref(passed)), "align_probe")
    ts, te = out["overlap"]
    ss, se = out["serial"]
    return {"frames": len(ts), "median_ms": round(float(np.median(ts)), 4), "p90_ms": round(float(np.percentile(ts, 90)), 4),
            "median_extract_ms": round(float(np.median(te)), 4),
            "median_align_wait_ms": round(float(np.median(ts - te)), 4),
            "align_stream_probe": {"streams_created": att.value, "passed": passed.value},
            "serial": {"median_ms": round(float(np.median(ss)), 4),
                       "median_extract_ms": round(float(np.median(se)), 4),
                       "median_align_ms": round(float(np.median(ss - se)), 4)},
            "path": "host C ABI, one frame at a time: H2D 752x480 u8 -> pyramid -> [SparseImgAlign 3..1 (prev -> cur) "
                    "on its own stream | extract] -> D2H kps+desc and pose; median over frames after 10 warm-up "
                    "frames ('serial': the same calls back to back)"}


TUM1_CAM = (517.306408, 516.469215, 318.643040, 255.313989)  # Examples/RGB-D/TUM1.yaml Camera.fx/fy/cx/cy


def c4_leg(S, dev, args, B=256):
    """BASELINE config C4: TUM fr1_desk-shaped 640x480 frames, ORBextractor(2000, 1.2, 8, 20, 7)
    (Examples/RGB-D/TUM1.yaml), batched 256-frame extract + dense Hamming (k vs k-1) throughput:
    frames rendered on the device (the textured plane under the TUM intrinsics), resident in HBM,
    HIP-event timed over `--steps` repetitions after 2 warm-up passes."""
    import torch
    import ygzfe
    W, H, nf, sf, nl, ini, mn = S.CONFIGS["C4"]
    sc = S.PlaneScene(23, W, H)
    poses = [ygzfe.trajectory_pose(sweep_index(g), XI) for g in range(B)]
    b = ygzfe.Batch((nf, sf, nl, ini, mn, 0), dev.index or 0, W, H, B)
    st = torch.cuda.current_stream(dev)
    tex = torch.from_numpy(sc.tex).to(dev)
    q = torch.from_numpy(np.stack([p[0] for p in poses])).to(dev)
    t = torch.from_numpy(np.stack([p[1] for p in poses])).to(dev)
    seeds = torch.arange(50000, 50000 + B, dtype=torch.int64, device=dev)
    ygzfe.render_plane_device(tex.data_ptr(), S.TEX_W, S.TEX_H, S.TEXEL, S.PLANE_Z, TUM1_CAM, q.data_ptr(),
                              t.data_ptr(), seeds.data_ptr(), B, W, H, b.frames_ptr(), b.frame_pitch, noise_amp=2,
                              stream=st.cuda_stream)
    cap = b.kp_cap
    P = B - 1
    ri = torch.arange(0, P, dtype=torch.int32, device=dev)
    ci = ri + 1
    bi = torch.empty((P, cap), dtype=torch.int32, device=dev)
    bd, sd = torch.empty_like(bi), torch.empty_like(bi)

    def step():
        b.extract(B, st.cuda_stream)
        b.match(P, ci.data_ptr(), ri.data_ptr(), bi.data_ptr(), bd.data_ptr(), sd.data_ptr(), st.cuda_stream)

    for _ in range(2):
        step()
    torch.cuda.synchronize(dev)
    b.check()
    reps = max(args.steps, 5)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        step()
    e1.record(st)
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / reps
    b.timing(True)
    for _ in range(reps):
        step()
    torch.cuda.synchronize(dev)
    stages = b.timing(False)
    b.check()
    cand, selk = b.stats(B)
    n_kp = [b.result(i)[0].shape[0] for i in range(0, B, 32)]
    return {"config": "C4 TUM1.yaml: 640x480, nFeatures 2000, scale 1.2, 8 levels, FAST 20/7",
            "frames": B, "ms_per_step": round(ms, 4), "frames_per_s": round(B / (ms * 1e-3), 1),
            "mean_keypoints": round(float(np.mean(n_kp)), 1),
            "mean_keypoints_per_level": [round(float(c) / B, 1) for c in selk],
            "stages_ms": {k: round(v, 4) for k, v in stages.items() if v > 0},
            "path": "device-rendered frames resident in HBM; batch extract + dense Hamming (k vs k-1), HIP events"}


def bow_leg(S, batch, B, dev, stream, with_cpu, reps=10):
    """Frame::ComputeBoW (Frame.cc:495-500) with an ORBvoc-shaped synthetic vocabulary
    (k = 10, L = 6: 1,111,111 nodes, 10^6 words; the real ORBvoc.txt is absent), levelsup 4,
    over the B frames the timed region extracted (batched, HIP events), one frame through
    the host C ABI, and the oracle's restatement on one frame (1 thread)."""
    import torch
    import ygzfe
    import _vocab as V
    t0 = time.time()
    parent, is_leaf, desc, weight = V.synth_vocab(6, 10, 6)
    voc = ygzfe.Vocabulary.from_arrays(10, 6, 0, 0, parent, is_leaf, desc, weight, device=dev.index or 0)
    build_s = time.time() - t0
    cap = batch.kp_cap
    bw = torch.zeros((B, cap), dtype=torch.int32, device=dev)
    bv = torch.zeros((B, cap), dtype=torch.float64, device=dev)
    nw = torch.zeros(B, dtype=torch.int32, device=dev)
    fn = torch.zeros((B, cap), dtype=torch.int32, device=dev)
    ff = torch.zeros((B, cap), dtype=torch.int32, device=dev)
    nfv = torch.zeros(B, dtype=torch.int32, device=dev)
    args = (bw.data_ptr(), bv.data_ptr(), nw.data_ptr(), fn.data_ptr(), ff.data_ptr(), nfv.data_ptr(), stream.cuda_stream)
    torch.cuda.synchronize(dev)
    for _ in range(2):
        batch.compute_bow(voc, B, 4, *args)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        batch.compute_bow(voc, B, 4, *args)
    e1.record(stream)
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / reps
    if int(nw.min().item()) <= 0:
        raise RuntimeError("bow_leg: a frame of the batch has no BoW words (batch not extracted?)")
    _, d0 = batch.result(0)
    for _ in range(3):
        voc.transform(d0, 4)
    ts = []
    for _ in range(reps):
        t1 = time.perf_counter()
        voc.transform(d0, 4)
        ts.append(time.perf_counter() - t1)
    line = {"vocabulary": "synthetic k=10 L=6 (1111111 nodes), TF_IDF / L1", "frames": B,
            "ms_per_launch": round(ms, 4), "frames_per_s": round(B / (ms * 1e-3), 1),
            "mean_words": round(float(nw.float().mean().item()), 1),
            "single_frame_host_ms": round(float(np.median(ts)) * 1e3, 4), "vocab_build_s": round(build_s, 2),
            "path": "batched on the extracted batch (ygzfe_batch_compute_bow); single: host C ABI"}
    if with_cpu:
        import _oracle as O
        ovoc = O.Vocab(10, 6, 0, 0, parent, is_leaf, desc, weight)
        tc = []
        for _ in range(5):
            t1 = time.perf_counter()
            ovoc.transform(d0, 4)
            tc.append(time.perf_counter() - t1)
        line["cpu_port_ms_per_frame"] = round(float(np.median(tc)) * 1e3, 4)
        line["cpu_cores"] = 1
    return line


def stereo_leg(S, dev, with_cpu, n_pairs=64, reps=20):
    """Frame::ComputeStereoMatches (Frame.cc:509-682) on EuRoC-shaped rectified pairs
    (C2 extraction, baseline 0.11 m): the batched kernel over n_pairs pairs resident in
    HBM (HIP events, after the batch extract), and one pair through the host C ABI.
    CPU: the oracle's restatement, 1 thread."""
    import torch
    import ygzfe
    W, H, nf, sf, nl, ini, mn = S.CONFIGS["C2"]
    scenes = [S.stereo_scene(100 + i, W, H) for i in range(n_pairs)]
    frames = np.stack([im for d in scenes for im in (d["left"], d["right"])])
    b = ygzfe.Batch((nf, sf, nl, ini, mn, 0), dev.index or 0, W, H, len(frames))
    b.upload(frames)
    b.extract(len(frames))
    b.check()
    cap = b.kp_cap
    li = torch.arange(0, 2 * n_pairs, 2, dtype=torch.int32, device=dev)
    ri = li + 1
    ur = torch.zeros((n_pairs, cap), dtype=torch.float32, device=dev)
    dp = torch.zeros((n_pairs, cap), dtype=torch.float32, device=dev)
    mb, mbf = scenes[0]["mb"], scenes[0]["mbf"]
    st = torch.cuda.current_stream(dev)
    torch.cuda.synchronize(dev)
    for _ in range(3):
        b.stereo(n_pairs, li.data_ptr(), ri.data_ptr(), mb, mbf, ur.data_ptr(), dp.data_ptr(), st.cuda_stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        b.stereo(n_pairs, li.data_ptr(), ri.data_ptr(), mb, mbf, ur.data_ptr(), dp.data_ptr(), st.cuda_stream)
    e1.record(st)
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / reps
    kept = float((dp > 0).sum().item()) / n_pairs
    kl, dl = b.result(0)
    kr, dr = b.result(1)
    ex = ygzfe.ORBextractor(nf, sf, nl, ini, mn, device=dev.index or 0)
    fl, fr = ex.ComputePyramid(scenes[0]["left"]), ex.ComputePyramid(scenes[0]["right"])
    for _ in range(3):
        ygzfe.stereo_matches(fl, fr, kl, dl, kr, dr, mb, mbf)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        ygzfe.stereo_matches(fl, fr, kl, dl, kr, dr, mb, mbf)
        ts.append(time.perf_counter() - t0)
    line = {"pairs": n_pairs, "ms_per_launch": round(ms, 4), "pairs_per_s": round(n_pairs / (ms * 1e-3), 1),
            "mean_left_kps": round(float(np.mean([b.result(2 * i)[0].shape[0] for i in range(min(8, n_pairs))])), 1),
            "mean_depths": round(kept, 1), "single_pair_host_ms": round(float(np.median(ts)) * 1e3, 4),
            "path": "batched: frames + keypoints + descriptors resident (ygzfe_batch_stereo); single: host C ABI"}
    if with_cpu:
        import _oracle as O
        orc = O.OrbOracle(nf, sf, nl, ini, mn)
        ll, rl = orc.pyramid(scenes[0]["left"]), orc.pyramid(scenes[0]["right"])
        tc = []
        for _ in range(10):
            t0 = time.perf_counter()
            O.stereo_matches(orc, ll, rl, kl, dl, kr, dr, mb, mbf)
            tc.append(time.perf_counter() - t0)
        line["cpu_port_ms_per_pair"] = round(float(np.median(tc)) * 1e3, 4)
        line["cpu_cores"] = 1
    return line


def tracking_search_leg(S, with_cpu, reps=50):
    """Row a11 per frame, the way Tracking calls it: the current frame's keypoints and
    descriptors uploaded once (ORBmatcher_gpu.inc's set_frame), then
    SearchByProjection(CurrentFrame, LastFrame, th 7, checkOri) (ORBmatcher.cc:1218-1350,
    TrackWithMotionModel) and SearchByProjection(F, vpLocalMapPoints, th 3, nnratio 0.8)
    (ORBmatcher.cc:43-126, SearchLocalPoints) on a C2 frame pair; host C ABI (the calls the
    drop-in header makes), median over `reps` frames.  CPU: oracle/match.c's literal
    restatement of the same loops, 1 thread."""
    import ygzfe
    p = S.match_pair("C2", 0)
    bnd = (0.0, float(p["W"]), 0.0, float(p["H"]))
    Q1, qd1, ur, bl1 = S.projection_queries(p, 0, th=7.0, level_mode="mixed")
    Q2, qd2, _, bl2 = S.projection_queries(p, 10, th=3.0 * 2.5, level_mode="band")
    mf = ygzfe.MatchFrame(0)

    def gpu_frame():
        cur = mf.set(p["k1"], p["d1"], ur, bnd)
        g1, n1 = ygzfe.search_projection_best(cur, Q1, qd1, bl1, 100, True)
        g2, n2 = ygzfe.search_projection_ratio(cur, Q2, qd2, bl2, 0.8)
        return n1, n2

    for _ in range(3):
        gpu_frame()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        n1, n2 = gpu_frame()
        ts.append(time.perf_counter() - t0)
    line = {"frame_keypoints": int(len(p["k1"])), "last_frame_queries": int(len(Q1)),
            "local_map_queries": int(len(Q2)), "matches_last_frame": int(n1), "matches_local_map": int(n2),
            "median_ms": round(float(np.median(ts)) * 1e3, 4),
            "path": "host C ABI per frame: frame upload + grid, SearchByProjection(F, LastF, checkOri) + "
                    "SearchByProjection(F, localMPs, nnratio 0.8), results on the host"}
    if with_cpu:
        import _oracle as O
        tc = []
        for _ in range(10):
            t0 = time.perf_counter()
            mfr = O.mframe(p["k1"], p["d1"], ur, bnd)
            O.search_projection_best(mfr, Q1, qd1, bl1, 100, True)
            O.search_projection_ratio(mfr, Q2, qd2, bl2, 0.8)
            tc.append(time.perf_counter() - t0)
        line["cpu_port_ms"] = round(float(np.median(tc)) * 1e3, 4)
        line["cpu_cores"] = 1
        line["speedup_vs_cpu_port"] = round(line["cpu_port_ms"] / line["median_ms"], 2)
    return line


def direct_leg(S, with_cpu, reps=50):
    """Batched SearchLocalPointsDirect (Tracking.cc:2258-2410) for one current frame:
    4 keyframes, ~750 local map points with 0..5 observations each (~1750
    (point, keyframe) FindDirectProjection items), host C ABI call -> matches on the
    host; median over `reps` calls.  CPU: the oracle's sequential loop, 1 thread."""
    import ygzfe
    d = S.direct_scene(0, n_kf=4, max_obs=5)
    W, H, nf, sf, nl, ini, mn = S.CONFIGS["C2"]
    ex = ygzfe.ORBextractor(nf, sf, nl, ini, mn, device=0)
    kf = [ex.ComputePyramid(im) for im in d["kf_images"]]
    cur = ex.ComputePyramid(d["cur_image"])
    cam = d["scene"].camera()
    args = (d["item_ptr"], d["ref_index"], d["kps"], d["pt_ref"], d["T_cr"], d["px_proj"])
    for _ in range(3):
        ygzfe.search_direct_batch(kf, cur, cam, *args)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        _, m = ygzfe.search_direct_batch(kf, cur, cam, *args)
        ts.append(time.perf_counter() - t0)
    line = {"points": len(m), "items": int(d["item_ptr"][-1]), "matched": int((m >= 0).sum()),
            "median_ms": round(float(np.median(ts)) * 1e3, 4),
            "path": "host C ABI (H2D items, FindDirectProjection per item, first in-border success per point, D2H)"}
    if with_cpu:
        import _oracle as O
        orc = O.OrbOracle(nf, sf, nl, ini, mn)
        kl = [orc.pyramid(im) for im in d["kf_images"]]
        cl = orc.pyramid(d["cur_image"])
        oc = O.Cam(*d["scene"].cam)
        tc = []
        for _ in range(10):
            t0 = time.perf_counter()
            O.search_direct(orc, kl, cl, oc, *args)
            tc.append(time.perf_counter() - t0)
        line["cpu_port_ms"] = round(float(np.median(tc)) * 1e3, 4)
        line["cpu_cores"] = 1
    return line


def host_cpu_info():
    """lscpu model name and CPU counts (the whole machine, and this process's affinity)."""
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    # the cgroup's CPU bandwidth limit (cgroup v2 cpu.max "quota period"), if any: more
    # threads than that only time-slice the same CPUs
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(-(-int(q) // int(per))))
    except (OSError, ValueError):
        pass
    return model, os.cpu_count() or 1, aff, quota


def cpu_threads():
    """Threads for the CPU throughput leg: every CPU of this process's affinity (nproc),
    capped by the cgroup CPU quota when one is set."""
    _, _, aff, quota = host_cpu_info()
    return max(1, min(aff, quota) if quota else aff)


def cpu_baseline(frames, r3, cz, S, args, sc):
    """oracle/ restatement driven from C (oracle/bench.c, no per-stage Python hops):
    pyramid + ORB (C2) + Hamming vs the previous frame + SparseImgAlign 3..1 per frame.
    1 thread over the sample (the reference's single Tracking thread: per-frame latency),
    then T threads (every CPU of this process's affinity, capped by a cgroup CPU quota if
    one is set) over the same frames split in contiguous chunks (throughput).  Plus the FAST sanity check of SURVEY.md §8d:
    the restated cv::FAST vs the reference's own SSE2 FAST-10 (oracle/_ref) on test1.png."""
    import _oracle as O
    cfg = S.CONFIGS["C2"]
    model, ncpu, aff, quota = host_cpu_info()
    threads = cpu_threads()
    n1 = min(args.cpu_sample, len(frames))
    wall1, st1 = O.bench_pipeline(frames[:n1], sc.cam, S.PLANE_Z, r3[:n1], cz[:n1], cfg, 1)
    per = 1e3 / max(1, st1.frames)
    perp = 1e3 / max(1, st1.pairs)
    nmt = len(frames)
    # untimed warm pass: the first threaded run pays each thread's malloc-arena
    # first-touch page faults (measured ~6x slower per thread), not pipeline work
    O.bench_pipeline(frames[:2 * threads], sc.cam, S.PLANE_Z, r3[:2 * threads], cz[:2 * threads], cfg, threads)
    wallt, stt = O.bench_pipeline(frames, sc.cam, S.PLANE_Z, r3[:nmt], cz[:nmt], cfg, threads)
    line = {"value": round(stt.frames / wallt, 2), "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": f"{nmt} frames of the same rendered C2 sequence on {threads} threads (contiguous chunks; "
                      f"{n1} frames on 1 thread for the latency): pyramid + octree ORB + rBRIEF + Hamming vs previous "
                      f"frame + SparseImgAlign 3..1, oracle/ (gcc -O3 -march=native; FAST-9 segment test, blur and resize on vectors like OpenCV's SIMD paths, the reference's own code scalar as in the reference)",
            "cpu_model": model, "host_cpus": ncpu, "process_cpus": aff, "cgroup_cpu_quota": quota,
            "single_thread_frames_per_s": round(st1.frames / wall1, 2),
            "ms_per_frame": round(wall1 * 1e3 / max(1, st1.frames), 3),
            "ms_pyramid": round(st1.t_pyr * per, 3), "ms_extract": round(st1.t_extract * per, 3),
            "ms_hamming": round(st1.t_hamming * perp, 3), "ms_align": round(st1.t_align * perp, 3),
            # BENCH_r04's figure for the same leg: round 5's oracle refactor made it 3.861 ms
            # (accumulators through aliasing pointers); oracle/align.c keeps them in locals again
            "ms_align_r04": 1.675,
            "threads_frames_per_s": round(stt.frames / wallt, 2)}
    # FAST sanity (the CPU FAST stage must be no slower than the reference's
    # SSE2 FAST-10).  Like for like: the same FAST-10 pipeline -- detect (SSE2 variant) +
    # fast_corner_score_10 + fast_nonmax_3x3 -- restated (oracle, 16-pixel vectors) and the
    # reference's own (oracle/_ref), both timed in C over the same ROI of test1.png, same
    # survivors.  The restated cv::FAST-9 (+ cornerScore + NMS) of the C2 path is listed too.
    try:
        from PIL import Image
        img = np.array(Image.open(os.path.join(ROOT, "tests", "golden", "test1.png")))
        H, W = img.shape
        fs = {}
        for th in (75, 20):
            O.bench_fast10(img, th, 3, 3, W - 6, H - 6, reps=5)
            n10, t10 = O.bench_fast10(img, th, 3, 3, W - 6, H - 6, reps=100)
            fs[f"oracle_fast10_th{th}_ms"] = round(t10 * 1e3, 4)
            fs[f"oracle_fast10_th{th}_kept"] = int(n10)
            if O.RefFast.available():
                ref = O.RefFast()
                ref.pipeline_bench(img, th, 3, 3, W - 6, H - 6, reps=5)
                nr, tr = ref.pipeline_bench(img, th, 3, 3, W - 6, H - 6, reps=100)
                fs[f"ref_fast10_th{th}_ms"] = round(tr * 1e3, 4)
                fs[f"ref_fast10_th{th}_kept"] = int(nr)
                fs[f"oracle_no_slower_th{th}"] = bool(t10 <= tr * 1.05)
            n9, t9 = O.bench_fast9(img, th, reps=20)
            fs[f"oracle_fast9_th{th}_ms"] = round(t9 * 1e3, 4)
            fs[f"oracle_fast9_th{th}_corners"] = n9
        fs["note"] = ("fast10: detect_sse2 + score + nonmax_3x3 on test1.png's interior, restated (oracle) vs the "
                      "reference's own Thirdparty/fast (oracle/_ref), 1 thread, mean of 100; fast9: the restated "
                      "cv::FAST TYPE_9_16 + cornerScore + NMS of the C2 path (a different detector, for reference)")
        line["fast_sanity"] = fs
    except Exception as e:  # test image / reference library absent
        line["fast_sanity"] = {"skipped": str(e)}
    return line


if __name__ == "__main__":
    main()
