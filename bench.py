"""Benchmark: Mpixels/s of segment + lifting_3d on synthetic 1080p flow fields (BASELINE.json metric).

Default (weak scaling, the driver's `--gpus N --steps K --warmup W`): one step = one batch of `--batch`
synthetic 1920x1080 flow fields PER GPU pushed through the whole HIP path (blur → MST → Kruskal
replay → per-merge filters + 3D lifting → snapshots → labels), then the fixed-size 3D-box records of
every frame gathered to all ranks (RCCL all_gather over xGMI when N > 1). Inputs are generated on
device before timing (resident in HBM); frames are independent, so ranks shard frames with no
data-path collective besides the box gather ("scaling": "weak").

`--frames F` (BASELINE config 4: F = 512): a fixed job of F frames split over the N ranks (contiguous
blocks, frame f = seed f), each rank running its share in batches of at most `--batch`; one step = the
whole job ("scaling": "strong").

N > 1: run under torch.distributed.run (one process per GPU), or pass `--gpus N` alone and this script
launches torch.distributed.run itself (as a child process, before any GPU call). It never reports
fewer GPUs than asked for: a mismatch exits non-zero.

Usage: python bench.py [--gpus N --steps K --warmup W --batch B --frames F]
Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
GATHER_PER_FRAME = 64  # box records per frame in the gathered block
ROUNDS_MAX = 40        # dofs_common.h kRoundsMax (Borůvka round flags and tile census entries per frame)
ROUND_FLAG = 16        # counters: C_ACT + r = Borůvka round r found a cross-component edge

# Algorithmic (compulsory) bytes of the probed kernels, per unit:
#   k_boruvka_min4 — Borůvka pass 0 (frames of width % 4 == 0). Units: a pixel of a tile the launch
#     processes (tiles found done are skipped; dofs_batch_tile_pixels says which) reads its component
#     label (4 B) and blurred flow (8 B) = 12 B; a (tile, component) record it writes (weight 8 B,
#     index 4 B, component 4 B) = 16 B (dofs_batch_records). Neighbours' words are other pixels' reads.
#   k_boruvka_pick4 — pass 1: a record read (16 B); the component minimum it compares with is a
#     cached gather, not counted.
#   k_boruvka_min — the pixel-candidate form (other widths): pass 0 24 B, pass 1 16 B per pixel.
#   k_krt_fused — unit: a merge: its endpoints in (8 B), its node size out (4 B), two child seed words
#     of the preorder's pointer jumping out (16 B), heavy/light and path-top flags out (3 B), and one
#     16-B union-find record of the sweep read = 47 B.
#   k_replay_flow — the whole replay in one dataflow launch (round 5): its 16-byte StepIn read per merge,
#     a 32-byte replay record stored per merge the results read (size >= min_size: C_KEEP) and 24 bytes
#     published per heavy path's top (C_PATHS) = 16 M + 32 keep + 24 paths (parks' states, a few thousand a
#     batch, are not counted).
#   KPathInit — per merge its inputs (position 4, path-top flag 1, KRT children 8, light side 1, children's
#     sizes 8 = 22 B) and its 16-byte StepIn out; a pixel light child's blurred flow (8 B; N - paths of them:
#     every pixel but a path's bottom is one light child); per path top its bottom (lscan, lposr: 8 B) and
#     its state word, cursor, top and list entry (16 B) = 38 M + 8 (N - paths) + 24 paths.
#   k_pre_sweep — per merge its jump word 8, children's sizes 8, KRT children 8 and light side 1 in, its
#     position 4 out = 29 B (the tops' pushed positions, one per block top, are not counted).
BYTES = {"k_boruvka_min4": (12, 16), "k_boruvka_pick4": 16, "k_boruvka_min": (24, 16), "k_krt_fused": 47,
         "k_replay_flow": (16, 32, 24), "KPathInit": (38, 8, 24), "k_pre_sweep": 29}
PROBES = ("k_boruvka_min4", "k_boruvka_pick4", "k_krt_fused", "k_replay_flow", "k_pre_sweep", "KPathInit")
C_PATHS = 0            # counters: heavy paths
C_KEEP = 54            # counters: merges whose replay record the lean replay stores
C_FLOWERR = 58         # counters (frame 0): the dataflow replay gave up a bounded wait
INPUT_SETS = 3         # distinct resident input batches, rotated over the steps
# measurement-only knobs of the library that make results invalid (they skip work): refused
INVALID_KNOBS = ("DOFS_SKIP_B", "DOFS_SKIPMASK")


def ceil_log2(n):
    k = 0
    while (1 << k) < n:
        k += 1
    return k


def boruvka_rounds(N):
    return min(ceil_log2(N) + 2, ROUNDS_MAX - 1)


def boruvka_min_units(tile_px, counters, N):
    """(pass-0 pixels, pass-1 pixels, launches) of k_boruvka_min over one batch.

    tile_px[f][m] = pixels of frame f's tiles found done by round m's pass 0 (m >= 1): processed by
    pass 0 in rounds 1..m and by pass 1 in rounds 1..m-1. m = 0 (never found done): processed by every
    launch that ran for the frame (pass 0 of round r runs if round r - 1 found an edge, pass 1 of round
    r if round r did; dofs_pipeline.h boruvka())."""
    R = boruvka_rounds(N)
    p0 = p1 = 0
    for f in range(tile_px.shape[0]):
        act = counters[f, ROUND_FLAG:ROUND_FLAG + R] != 0
        for m in range(1, R):
            px = int(tile_px[f, m])
            p0 += px * m
            p1 += px * (m - 1)
        px = int(tile_px[f, 0])
        p0 += px * int(act[0:R - 1].sum())
        p1 += px * int(act[1:R].sum())
    return p0, p1, 2 * (R - 1)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=112, help="frames per GPU per step (--frames: per batch)")
    ap.add_argument("--frames", type=int, default=0, help="fixed job of F frames over all GPUs (config 4: 512)")
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--cpu-frames", type=int, default=1, help="frames per CPU-baseline process (0 = skip)")
    ap.add_argument("--cpu-procs", type=int, default=0, help="concurrent CPU-baseline processes (0 = auto)")
    ap.add_argument("--cpu-opt", default="O2,O0", help="oracle builds timed for the CPU baseline")
    ap.add_argument("--no-stages", action="store_true", help="skip the per-stage event timing pass")
    ap.add_argument("--no-h2d", action="store_true", help="skip the with-H2D (host input) pass")
    ap.add_argument("--probe", default=",".join(PROBES), help="kernels timed with device events (comma list)")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "r06", "pmc_kernels.json"),
                    help="PMC summary JSON (tools/pmc_kernels.py via tools/pmc_round.sh) for the roofline traffic; "
                         "used only when its lib_sha256 is the loaded library's")
    ap.add_argument("--cpu-worker", nargs=4, metavar=("OPT", "H", "W", "SEED"), help=argparse.SUPPRESS)
    return ap.parse_args(argv)


# ---- CPU baseline (oracle = the reference-faithful CPU restatement; test infrastructure) ---------------
def cpu_worker(opt, H, W, seed):
    """One frame of the faithful CPU restatement (std::multiset edge sort, std::set unions, set-copy
    snapshots), one thread; prints its seconds."""
    from oracle import binding as ob
    persp, inv, up = ob.calib()
    flow = ob.synth_flow(H, W, seed)
    t0 = time.perf_counter()
    ob.segment(flow, persp, inv, up, mode=1, opt=opt)
    print(f"{time.perf_counter() - t0:.6f}", flush=True)


def _cpu_model():
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _mem_avail_gb():
    try:
        for ln in open("/proc/meminfo"):
            if ln.startswith("MemAvailable:"):
                return int(ln.split()[1]) / 1048576
    except OSError:
        pass
    return 16.0


def cpu_baseline(a):
    """`procs` concurrent single-thread processes (the reference is single-threaded; one frame per core),
    one per host thread of this GPU's CPU share, capped by ~1.5 GB of host RAM per 1080p frame; each runs
    --cpu-frames synthetic frames of the bench workload. Runs before this process touches the GPU.

    The share: a one-GPU box of this pool is one GPU of an 8-GPU host whose `nproc` shows the whole
    machine's hardware threads (256 on the EPYC 9575F hosts) but whose harness allots 16 of them per GPU
    (its OMP_NUM_THREADS / MAX_JOBS); BASELINE.md's "nproc processes capped by RAM" on a dedicated host is
    reported beside it as an extrapolation from the measured per-frame time (`nproc_extrapolated`), and so
    is config 4's 512-frame job."""
    from oracle import binding as ob
    H, W = a.height, a.width
    share = len(os.sched_getaffinity(0))
    per_frame_gb = 1.5 * H * W / 2073600
    gpu_share = int(os.environ.get("OMP_NUM_THREADS", "16") or 16)  # the harness's per-GPU CPU share
    ram_cap = int(_mem_avail_gb() * 0.5 / per_frame_gb)
    procs = a.cpu_procs or max(1, min(gpu_share, share, ram_cap))
    out = {"unit": "Mpixels/sec", "kind": "port", "cores": procs, "nproc": os.cpu_count(), "affinity": share,
           "cpu_model": _cpu_model()}
    for opt in a.cpu_opt.split(","):
        ob.lib(opt)  # built before timing
        t0 = time.perf_counter()
        per = []
        for k in range(a.cpu_frames):  # `procs` frames at a time, one per process
            ps = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "--cpu-worker", opt, str(H), str(W),
                                    str(p * a.cpu_frames + k)], stdout=subprocess.PIPE, text=True)
                  for p in range(procs)]
            for p in ps:
                o, _ = p.communicate()
                if p.returncode != 0:
                    raise RuntimeError(f"cpu baseline worker failed ({p.returncode})")
                per.append(float(o.split()[-1]))
        wall = time.perf_counter() - t0
        frames = procs * a.cpu_frames
        per.sort()
        out[opt] = {"value": round(frames * H * W / wall / 1e6, 4), "frames": frames, "wall_s": round(wall, 2),
                    "s_per_frame": {"min": round(per[0], 2), "median": round(per[len(per) // 2], 2),
                                    "max": round(per[-1], 2)},
                    "single_core_mpix_s": round(H * W / per[len(per) // 2] / 1e6, 4)}
    first = a.cpu_opt.split(",")[0]
    out["value"] = out[first]["value"]
    med = out[first]["s_per_frame"]["median"]
    full = max(1, min(os.cpu_count() or 1, ram_cap))  # nproc processes, capped by RAM
    out["gpu_cpu_share"] = gpu_share
    out["nproc_extrapolated"] = {"procs": full, "value": round(full * H * W / med / 1e6, 3),
                                 "note": f"{full} concurrent frames at the measured median {med} s per frame "
                                         f"(nproc {os.cpu_count()}, RAM cap {ram_cap}); assumes no slowdown "
                                         f"from memory-bandwidth contention, so an upper bound"}
    out["job_512_frames_s"] = {"on_procs": round(-(-512 // procs) * med, 1),
                               "on_nproc": round(-(-512 // full) * med, 1)}
    out["sample"] = (f"{procs} concurrent processes (this GPU's CPU share) x {a.cpu_frames} synthetic {W}x{H} "
                     f"frame(s) each (seeds 0..{procs * a.cpu_frames - 1}), faithful mode (std::multiset edge sort + "
                     f"std::set unions + set-copy snapshots), one thread per process; value = {first} build; g++ "
                     + " and ".join(f"-{o}: {out[o]['wall_s']} s wall" for o in a.cpu_opt.split(","))
                     + f"; config 4's 512-frame job extrapolated: {out['job_512_frames_s']['on_procs']} s on these "
                       f"{procs} processes, {out['job_512_frames_s']['on_nproc']} s on {full} (nproc, RAM-capped)")
    return out


# ---- launcher --------------------------------------------------------------------------------------------
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def self_launch(a, argv):
    """--gpus N > 1 without a launcher: start torch.distributed.run as a child process (nothing here has
    touched the GPU) and exit with its status."""
    import torch
    n = torch.cuda.device_count()  # does not initialise the GPU on this image
    if n < a.gpus:
        print(f"bench.py: --gpus {a.gpus} but only {n} device(s) visible", file=sys.stderr)
        return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + argv
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


# ---- GPU bench -------------------------------------------------------------------------------------------
def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    a = parse(argv)
    if a.cpu_worker:
        opt, H, W, seed = a.cpu_worker
        cpu_worker(opt, int(H), int(W), int(seed))
        return 0
    bad = [k for k in INVALID_KNOBS if os.environ.get(k, "") not in ("", "0")]
    if bad:
        print(f"bench.py: {', '.join(bad)} set: these skip work and invalidate every result; refusing to run",
              file=sys.stderr)
        return 2
    world = int(os.environ.get("WORLD_SIZE", "0"))
    if world == 0:
        if a.gpus > 1:
            return self_launch(a, argv)
        world = 1
    if world != a.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {a.gpus}", file=sys.stderr)
        return 2
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    cpu = None
    if world == 1 and rank == 0 and a.cpu_frames > 0:  # before any GPU call: the workers are child processes
        cpu = cpu_baseline(a)

    import numpy as np
    import torch
    import torch.distributed as dist

    from denseopticalflowsegmentation3d_amd import runtime
    from denseopticalflowsegmentation3d_amd.abi import default_params
    from denseopticalflowsegmentation3d_amd.frames import FrameParallel, Pipelined, job_plan

    if world > 1:
        dist.init_process_group("nccl")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    H, W = a.height, a.width
    N = H * W

    ctx = runtime.Dofs(local)
    persp, inv, up = runtime.calib()
    prm = default_params()
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    fp = FrameParallel(ctx, world, GATHER_PER_FRAME)

    if a.frames:  # config 4: a fixed job split over the ranks
        mine, chunks = job_plan(a.frames, rank, world, a.batch)
        flows = torch.empty((max(len(mine), 1), H, W, 2), dtype=torch.float32, device=dev)
        # a rank without frames of its own (e.g. F = 9 on 8 GPUs: ceil(9/8) = 2 per rank leaves ranks
        # 5-7 empty) still runs every chunk, on a placeholder frame (seed F, not counted in `value`)
        runtime.synth_flow_device(flows.data_ptr(), max(len(mine), 1), H, W,
                                  seed0=mine.start if len(mine) else a.frames, stream=sh)
        frames_per_step = a.frames
        B = chunks[0][1]
    else:
        # INPUT_SETS distinct batches of fields, each resident in HBM, used in turn by consecutive steps: no
        # step sees the inputs of the step before it (a stale-state bug cannot hide behind repeated inputs)
        B = a.batch
        sets = []
        for k in range(INPUT_SETS):
            t = torch.empty((B, H, W, 2), dtype=torch.float32, device=dev)
            runtime.synth_flow_device(t.data_ptr(), B, H, W, seed0=(rank * INPUT_SETS + k) * B, stream=sh)
            sets.append(t)
        flows = sets[0]
        chunks = [(0, B)]
        frames_per_step = world * B

    # ranks with fewer real frames (F not a multiple of N) still run every chunk with n frames (the gather
    # is collective and its blocks are equal): padding positions cycle through the rank's own frames
    # (batch_view) and are not counted in `value`
    pipe = Pipelined(fp, persp, inv, up, params=prm, stream=sh)
    flush = pipe.flush

    nstep = [0]

    def step(src=None):
        if src is None:
            src = flows if a.frames else sets[nstep[0] % INPUT_SETS]
        nstep[0] += 1
        pipe.run_chunks(src, chunks)
        if a.frames:  # one step = the whole job
            flush()

    for _ in range(a.warmup):
        step()
    flush()
    checked0 = fp.checked
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ctx.probe(a.probe)
    ctx.probe_read_n(8)
    ev_step = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps + 1)]
    t0 = time.perf_counter()
    ev_step[0].record(stream)
    for k in range(a.steps):
        step()
        ev_step[k + 1].record(stream)
    flush()
    e1 = torch.cuda.Event(enable_timing=True)
    e1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    # every timed batch's records were copied through FrameParallel.collect, which fails on a batch whose
    # results are invalid (dofs_batch_records_copy: DOFS_ERR_INVALID_RESULT); this counts the batches it checked
    checked = fp.checked - checked0
    if checked != a.steps * len(chunks):
        raise RuntimeError(f"{checked} of {a.steps * len(chunks)} timed batches were checked")
    ms_ev = ev_step[0].elapsed_time(e1)
    per_step = sorted(ev_step[k].elapsed_time(ev_step[k + 1]) for k in range(a.steps))
    probes = dict(zip(a.probe.split(","), ctx.probe_read_n(8))) if a.probe else {}
    ctx.probe(None)
    t = torch.tensor([max(wall, ms_ev / 1e3)], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    value = frames_per_step * a.steps * N / elapsed / 1e6

    # roofline: algorithmic bytes of each probed kernel's launches in the timed region over their
    # device-event time (events recorded on the stream the kernel runs on). The units (processed Borůvka
    # tiles, records, long-path merges) depend on the input: each input set's census is read from one
    # extra, untimed batch of that set, and the timed region's units are the sum over its steps' sets.
    timed_sets = [(a.warmup + j) % INPUT_SETS for j in range(a.steps)] if not a.frames else [0] * a.steps
    census = {}
    for k in sorted(set(timed_sets)):
        if a.frames:
            cnt = ctx.batch_counters(chunks[-1][1])
        else:
            pipe.run_chunks(sets[k], chunks)
            flush()
            torch.cuda.synchronize()
            cnt = ctx.batch_counters(B)
        if cnt[0, C_FLOWERR]:
            raise RuntimeError("the dataflow replay gave up a bounded wait: results of the batches are invalid")
        census[k] = (cnt, ctx.tile_pixels(chunks[-1][1]), ctx.records(chunks[-1][1]))
    pmc, pmc_note = {}, "no PMC summary"
    if a.pmc and os.path.exists(a.pmc):
        import hashlib
        pj = json.load(open(a.pmc))
        sha = hashlib.sha256(open(runtime.LIB_PATH, "rb").read()).hexdigest()
        if pj.get("lib_sha256") != sha:  # counters of another build: stale, never reported
            pmc_note = f"{os.path.relpath(a.pmc, ROOT)} is for another build of libdofs_hip.so: traffic dropped"
        elif pj.get("batch") == B and pj.get("height", H) == H and pj.get("width", W) == W:
            pmc = pj.get("kernels", {})
            pmc_note = f"{os.path.relpath(a.pmc, ROOT)} (lib_sha256 {sha[:12]} matches the loaded library)"
        else:
            pmc_note = f"{os.path.relpath(a.pmc, ROOT)} is for another batch shape: traffic dropped"
    batches = a.steps * len(chunks)

    def units(name, k):
        """(algorithmic bytes of one batch of input set k, units description) for a probed kernel."""
        cnt, tiles, recs = census[k]
        if name == "k_boruvka_min4":
            p0, _, _ = boruvka_min_units(tiles, cnt, N)
            nrec = int(recs.sum())
            return p0 * BYTES[name][0] + nrec * BYTES[name][1], {"pass0_px": p0, "records": nrec}
        if name == "k_boruvka_pick4":
            nrec = int(recs.sum())
            return nrec * BYTES[name], {"records": nrec}
        if name == "k_boruvka_min":
            p0, p1, _ = boruvka_min_units(tiles, cnt, N)
            return p0 * BYTES[name][0] + p1 * BYTES[name][1], {"pass0_px": p0, "pass1_px": p1}
        M = (N - 1) * B
        paths, keep = int(cnt[:, C_PATHS].sum()), int(cnt[:, C_KEEP].sum())
        if name == "k_krt_fused":
            return BYTES[name] * M, {"merges": M}
        if name == "k_replay_flow":
            a, b, c = BYTES[name]
            return a * M + b * keep + c * paths, {"merges": M, "kept_records": keep, "paths": paths}
        if name == "KPathInit":
            a, b, c = BYTES[name]
            return a * M + b * (N * B - paths) + c * paths, {"merges": M, "paths": paths}
        if name == "k_pre_sweep":
            return BYTES[name] * M, {"merges": M}
        return None, None

    UNIT_TEXT = {"k_boruvka_min4": "12 per pixel of a processed tile + 16 per record written",
                 "k_boruvka_pick4": "16 per record read",
                 "k_boruvka_min": "24 (pass 0) / 16 (pass 1) per pixel of a processed tile",
                 "k_krt_fused": f"{BYTES['k_krt_fused']} per merge",
                 "k_replay_flow": "16 per merge (StepIn in) + 32 per stored record (size >= min_size) + 24 per "
                                  "path top published",
                 "KPathInit": "38 per merge + 8 per pixel light child + 24 per path top",
                 "k_pre_sweep": f"{BYTES['k_pre_sweep']} per merge"}
    kern = []
    for name, (ms, launches) in probes.items():
        if not launches:
            continue
        entry = {"kernel": name, "ms_per_batch": round(ms / batches, 3), "launches": launches,
                 "avg_launch_us": round(ms / launches * 1e3, 2),
                 "share_of_step": round(ms / a.steps / (elapsed * 1e3 / a.steps), 4)}
        alg = None
        if len(chunks) == 1 and units(name, timed_sets[0])[0] is not None:
            per_set = {k: units(name, k) for k in census}
            alg = sum(per_set[k][0] for k in timed_sets)
            entry["alg_bytes_per_unit"] = UNIT_TEXT[name]
            entry["units_per_batch"] = per_set[timed_sets[-1]][1]
        if alg is not None:
            ach = alg / (ms / 1e3) / 1e9
            entry.update({"achieved": round(ach, 3), "frac": round(ach / HBM_PEAK_GBS, 6),
                          "alg_bytes_per_launch": round(alg / launches)})
            pk = pmc.get(name)
            if pk and pk.get("hbm_bytes_per_launch"):
                entry["traffic"] = round(pk["hbm_bytes_per_launch"])
                entry["traffic_over_alg"] = round(pk["hbm_bytes_per_launch"] / (alg / launches), 3)
                entry["traffic_read_pattern"] = pk.get("read_pattern")
                if pk.get("hbm_read_bounds"):  # raw FETCH_SIZE (random: 64 B per request) .. x2 (streaming)
                    entry["traffic_bounds"] = [round(b + pk.get("write_size_raw_bytes", 0))
                                               for b in pk["hbm_read_bounds"]]
                if pk.get("read_bytes_by_request_size") is not None:
                    entry["read_bytes_by_request_size"] = round(pk["read_bytes_by_request_size"])
        kern.append(entry)
    kern.sort(key=lambda e: -e["ms_per_batch"])
    roof = None
    # the headline is the dominant kernel: the probed kernel with the most device time per batch
    main_k = next((e for e in kern if "achieved" in e), None)
    if main_k:
        roof = {"bound": "hbm", "achieved": main_k["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": main_k["frac"], "traffic": main_k.get("traffic"),
                "traffic_source": pmc_note + ("; rocprofv3 --pmc passes, tools/pmc_round.sh"
                                              if main_k.get("traffic") else ""),
                "kernel": main_k["kernel"], "why": "the probed kernel with the most device time per batch",
                "ms_per_batch": main_k["ms_per_batch"], "share_of_step": main_k["share_of_step"],
                "launches": main_k["launches"], "avg_launch_us": main_k["avg_launch_us"],
                "alg_bytes_per_launch": main_k["alg_bytes_per_launch"],
                "alg_bytes_per_unit": main_k["alg_bytes_per_unit"],
                "secondary": [e for e in kern if e is not main_k],
                "path_input_roofline_frac": round(frames_per_step * a.steps * N * 8 / world / elapsed / 1e9
                                                  / HBM_PEAK_GBS, 8)}
        for k in ("traffic_over_alg", "traffic_bounds", "read_bytes_by_request_size", "traffic_read_pattern"):
            if k in main_k:
                roof[k] = main_k[k]

    # with host input: each batch's flow fields copied H2D from pinned host memory on the caller stream
    # before the call (two device buffers in turn), the PCIe-inclusive rate (never `value`)
    h2d = None
    if not a.no_h2d and not a.frames:
        host = sets[0].cpu().pin_memory()
        dbuf = [torch.empty_like(sets[0]), torch.empty_like(sets[0])]
        hs = max(3, a.steps // 2)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for k in range(hs):
            d = dbuf[k & 1]
            d.copy_(host, non_blocking=True)
            step(d)
        flush()
        torch.cuda.synchronize()
        th = time.perf_counter() - t1
        h2d = {"value": round(world * B * hs * N / th / 1e6, 3), "unit": "Mpixels/sec", "steps": hs,
               "ms_per_step": round(th / hs * 1e3, 3)}
        del host

    # per-stage device-event timing of extra profiled batches (not part of the timed region)
    stages = None
    if not a.no_stages and not a.frames:
        ctx.profile(True)
        for _ in range(max(2, a.steps // 2)):
            step()
        flush()
        torch.cuda.synchronize()
        ms, nb = ctx.profile_read()
        ctx.profile(False)
        stages = {k: round(v / nb, 3) for k, v in ms.items()}

    if rank == 0:
        res = ctx.fetch(0, want_blur=False)
        med = per_step[len(per_step) // 2]
        cfg = {"workload": (f"{a.frames} synthetic {W}x{H} flow fields over {world} GPU(s) (BASELINE config 4), "
                            f"full segment + lifting_3d" if a.frames else
                            f"{W}x{H} synthetic flow, full segment + lifting_3d (BASELINE config 3 shape)"),
               "frames_per_step": frames_per_step, "frames_per_gpu_per_batch": B,
               "frames_per_sec": round(frames_per_step * a.steps / elapsed, 3),
               "parallelism": f"frame-parallel x{world}", "workspaces": ctx.batch_slots(),
               "workspace_mb_per_frame": round(ctx.workspace_bytes() / B / 1e6, 1),
               "input_sets": 1 if a.frames else INPUT_SETS,
               "dofs_env": {k: v for k, v in sorted(os.environ.items()) if k.startswith("DOFS_")},
               "replay_workers": ctx.flow_workers(),
               "timed_batches_checked": checked,
               "snapshots_frame0": int(len(res.snapshots)),
               "candidates_frame0": int(res.stats["n_candidates"])}
        out = {
            "metric": "Mpixels/sec segment+lifting_3d @1080p",
            "value": round(value, 3),
            "unit": "Mpixels/sec",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1e3, 3),
            "ms_per_step_median": round(med, 3),
            "ms_per_step_p10_p90": [round(per_step[len(per_step) // 10], 3),
                                    round(per_step[min(len(per_step) - 1, (9 * len(per_step)) // 10)], 3)],
            "higher_is_better": True,
            "scaling": "strong" if a.frames else "weak",
            "vs_baseline": None,
            "dtype": "f32+f64",
            "data": ("synthetic (on-device splitmix64 flow fields, SURVEY.md §8(d) spec"
                     + (")" if a.frames else f"; {INPUT_SETS} distinct resident batches used in turn by the steps)")),
            "config": cfg,
            "roofline": roof,
            "with_h2d": h2d,
            "stages_ms_per_batch": stages,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
