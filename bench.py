#!/usr/bin/env python3
"""Benchmark: Mrays/s of the MI355X render path on the Cornell box (config C2 of BASELINE.json:
scene 5, 500x500, 1024 spp, 32 bounces).

One step = one full render of the workload: every (pixel, sample) path traced by mrt_path_kernel,
folded per pixel in sample order (draw() semantics) and, for N > 1 GPUs, the tile shards gathered
to rank 0 over RCCL and scattered into the full framebuffer.  The image is fixed as N grows
(strong scaling); the work_queue tiles are dealt to the ranks in rounds of N, each round in its
own pseudo-random rank order (mrt_local_pixels).

Prints ONE JSON line (rank 0).  `value` = total rays traced by all ranks / max-over-ranks wall
time of the K timed steps.  `roofline` bounds the dominant kernel (mrt_path_kernel) by what limits
it, VALU issue: its VALU wave-instructions per launch (rocprofv3 SQ_INSTS_VALU per ray, committed
under profiles/, times the launch's rays) over its HIP-event-measured duration, against the issue
peak of 1024 SIMDs x 2.4 GHz / 2 cycles per wave64 instruction; beside it the measured HBM bytes
(hbm_frac) and the reference-equivalent bytes of SURVEY.md 8(d) (ref_equiv: served by caches, not
a ceiling).  `parity` compares the last timed step's image with the reference as shipped on the
same per-path streams (tests/golden fixture), after the timed region.  `cpu_baseline` times the
reference itself (oracle/_ref/mrt_ref, as shipped) on a bounded sample on this host.
"""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Mrays/sec (primary+secondary), Cornell box 32-bounce; per-pixel RMSE vs CPU"
# reference-equivalent bytes per ray: sum over the reference's tests per ray of the
# compact FP32 payload each test reads (aabb 24-32 B, rect 24 B, sphere 16 B, triangle 36 B,
# instance 20 B).  The scenes are cache-resident and the tolerance kernels replace most of those
# tests (the Cornell slab walks), so this is a reference-work rate, not an HBM ceiling.
B_RAY = {5: 256.0, 9: 434.0, 8: 1251.0, 7: 780.0, 0: 976.0}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)
# VALU issue peak: 256 CUs x 4 SIMDs, one wave64 VALU instruction per SIMD per 2 cycles
# (MI355X_MICROARCH.md: 32 lanes/cycle), at the 2.4 GHz peak engine clock
N_SIMD = 1024
CLOCK_PEAK_GHZ = 2.4
VALU_PEAK_G = N_SIMD * CLOCK_PEAK_GHZ / 2.0  # G wave-instructions/s
WORKLOAD = {5: "C2 cornell_box", 9: "C3 wt_teapot in cornell box", 8: "C4 bunny", 7: "C5 book2 final scene",
            0: "C1 random spheres"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # (20 steps: a step's fold runs beside the next step's path kernel, so the last one's is the only
    # fold the timed region waits for; 20 x 8.3 ms is still a fraction of a second)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--scene", type=int, default=5)
    ap.add_argument("--width", type=int, default=500)
    ap.add_argument("--height", type=int, default=500)
    ap.add_argument("--samples", type=int, default=1024)
    ap.add_argument("--depth", type=int, default=32)
    ap.add_argument("--tile-size", type=int, default=8,
                    help="work_queue tile edge; also the multi-GPU partition grain (tiles dealt to the ranks in permuted rounds of N)")
    ap.add_argument("--cpu-spp", type=int, default=256, help="spp of the bounded CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-quick", action="store_true", help="time the CPU baseline on the quota threads only")
    ap.add_argument("--numerics", choices=["fast", "exact"], default="fast",
                    help="numerics contract of the timed render: fast = tolerance contract (per-pixel RMSE < 1e-3 "
                         "vs the reference as shipped, tests/test_gpu_parity.py), exact = bit-for-bit the reference "
                         "built exact; the other one is timed too and reported as other_numerics")
    ap.add_argument("--no-compare-numerics", action="store_true")
    ap.add_argument("--kernel-reps", type=int, default=0,
                    help="ignored (kept for old command lines): the roofline's kernel time is now the HIP-event "
                         "time of the timed steps' own launches")
    ap.add_argument("--emulate-world", type=int, default=1,
                    help="single-GPU rehearsal: render only rank --emulate-rank's share of an N-rank job "
                         "(no collectives); used to predict per-rank step time at N GPUs")
    ap.add_argument("--emulate-rank", type=int, default=0)
    ap.add_argument("--emulate-gather", action="store_true",
                    help="with --emulate-world: also run rank 0's framebuffer scatter of all N shards each "
                         "step (the gather's device-side work; the xGMI transfer itself is not emulated)")
    ap.add_argument("--gather", choices=["capi", "torch"], default="capi",
                    help="N > 1: how the tile shards reach rank 0 -- capi (default): the C-ABI's RCCL gather "
                         "(mrt_gather_frame on a communicator from mrt_comm_init_rank; one ncclGather of the padded "
                         "shards + the device scatter, include/mrt.h), torch: miniraytracer_amd.dist.TileGather "
                         "(dist.gather + index_copy_)")
    ap.add_argument("--force-dist", action="store_true",
                    help="test hook: take the multi-rank path (process group, gather to rank 0 every step) even at "
                         "one rank -- on one GPU the C-ABI's RCCL gather then runs to itself")
    ap.add_argument("--chunk-samples", type=int, default=0,
                    help="samples per path-kernel launch (0: the library's choice)")
    ap.add_argument("--fold", choices=["auto", "lean", "full", "async"], default="auto",
                    help="mode-0 fold: async (MRT_RF_FOLD_ASYNC, one context: each render's fold on the context's "
                         "own stream, beside the next render's path kernel; C2 8.28 ms per step against 8.65 for "
                         "full), full (after its render's path kernel), lean (MRT_RF_FOLD_BEHIND, beside the other "
                         "contexts' path kernels: 8.35-8.45 ms per C2 step in most runs but 9.8-10.1 in about one "
                         "of five); auto (default) = async at one or two contexts, full with more")
    ap.add_argument("--pipeline", type=int, default=0,
                    help="render contexts used round-robin on their own HIP streams (0 = auto: 2 when a rank "
                         "traces fewer than ~100 M paths per step, else 1).  With several contexts the GPU "
                         "runs their path kernels side by side, which hides a short launch's fixed costs "
                         "(emulated 8-rank C2 share, round 6: 1.222 ms per step at 1 context, 1.102-1.114 at 2 "
                         "with the async fold, 1.123-1.137 at 3 with the full fold) but gains nothing on a full "
                         "C2 render and makes it bimodal (8.60-8.63 ms at 1 context; 8.69-8.71, and 9.3-9.4 in "
                         "2 runs of 4, at 3; DESIGN.md §4)")
    ap.add_argument("--verify", action="store_true",
                    help="after timing, rank 0 checks the assembled framebuffer of the last step against a "
                         "single-context full render, bit for bit")
    ap.add_argument("--pmc-json", default=None,
                    help="per-ray PMC figures of the workload (default: profiles/pmc_s<scene>_<W>x<H>.json, "
                         "written by tools/pmc_summary.py --bench-file)")
    ap.add_argument("--no-other-walk", action="store_true",
                    help="skip timing the general hit walk (MRT_NO_SIG=1: the linear-program interpreter) "
                         "beside a shape-specialised one")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--step-times", action="store_true",
                    help="record a HIP event after every timed step (on its stream) and report the per-step "
                         "completion intervals (median / p90 / max and where the max fell): tells a whole-run "
                         "slowdown (clock) from single-step stalls (rehearsal diagnosis)")
    return ap.parse_args()


def _cpu_quota():
    """CPUs this process may use: affinity mask, capped by a cgroup v2 cpu.max quota if one is set."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(int(q) // int(per))))
    except (OSError, ValueError):
        pass
    return n


def _has_avx512():
    try:
        return any(l.startswith("flags") and " avx512f" in l for l in open("/proc/cpuinfo"))
    except OSError:
        return False


def cpu_baseline(args):
    """The reference as shipped (multithreaded work_queue, atomic ray counter) on this host, over a
    bounded sample of the same scene, in the GPU leg's accumulation mode (-mode 0: draw(), the
    bench's render; the reference's default is draw2); its own Mrays/s formula (main.cpp:403-405).
    Timed twice: with as many threads as this process may use (affinity / cgroup quota) and with
    -threads = os.cpu_count() (every CPU the machine reports; on a shared GPU box that is more than
    the box's share, so the two differ)."""
    import oracle
    total = os.cpu_count() or 1
    quota = _cpu_quota()
    used = int(os.environ.get("MRT_CPU_THREADS", quota))
    sample = (f"scene {args.scene}, {args.width}x{args.height}, {args.cpu_spp} spp (of {args.samples}), "
              f"depth {args.depth}, -mode 0 (draw(), as the GPU leg)")
    b = oracle.ref_binary(exact=False)
    if b is not None:
        def run(threads):
            return oracle.run_ref(["-scene", args.scene, "-width", args.width, "-height", args.height, "-samples",
                                   args.cpu_spp, "-depth", args.depth, "-threads", threads, "-mode", 0], exact=False, timeout=900)
        r = run(used)
        res = {"value": round(r["mrays_per_s"], 3), "unit": "Mrays/s", "cores": used, "cores_used": used,
               "cores_total": total, "cores_quota": quota, "kind": "reference",
               "sample": sample + f", reference build oracle/_ref/mrt_ref as shipped, {r['rays']} rays in "
                                  f"{r['trace_seconds']:.2f} s on {used} threads"}
        if total != used and not args.cpu_quick:
            ra = run(total)
            res["value_all_cores"] = round(ra["mrays_per_s"], 3)
            res["sample_all_cores"] = f"-threads {total} (os.cpu_count()): {ra['rays']} rays in {ra['trace_seconds']:.2f} s"
        # -march=native on an AVX-512 host is -march=x86-64-v4: where this host has AVX-512F, that
        # build is timed as well and the faster of the two is the baseline
        v4 = oracle.ref_binary(name="mrt_ref_v4")
        if v4 is not None and not args.cpu_quick and _has_avx512():
            r4 = oracle.run_ref(["-scene", args.scene, "-width", args.width, "-height", args.height, "-samples", args.cpu_spp,
                                 "-depth", args.depth, "-threads", used, "-mode", 0], timeout=900, name="mrt_ref_v4")
            res["value_v3"] = res["value"]
            res["value_v4"] = round(r4["mrays_per_s"], 3)
            res["sample_v4"] = f"oracle/_ref/mrt_ref_v4 (-march=x86-64-v4): {r4['rays']} rays in {r4['trace_seconds']:.2f} s on {used} threads"
            if res["value_v4"] > res["value"]:
                res["value"] = res["value_v4"]
                res["sample"] = sample + (f", reference build oracle/_ref/mrt_ref_v4 as shipped with -march=x86-64-v4 (AVX-512; "
                                          f"the v3 build: {res['value_v3']} Mrays/s), {r4['rays']} rays in "
                                          f"{r4['trace_seconds']:.2f} s on {used} threads")
        res["binary"] = ref_provenance(b if res.get("value_v4") != res["value"] else oracle.ref_binary(name="mrt_ref_v4"))
        res.update(contention_free(args, used, sample))
        return res
    import miniraytracer_amd as m
    sc = m.select_scene(args.scene, args.width / args.height)
    d = oracle.desc(args.width, args.height, args.cpu_spp, depth=args.depth, threads=used)
    t0 = time.perf_counter()
    _, rays, _, _ = oracle.render(sc, d)
    dt = time.perf_counter() - t0
    return {"value": round(rays / dt / 1e6, 3), "unit": "Mrays/s", "cores": used, "cores_used": used,
            "cores_total": total, "cores_quota": quota, "kind": "port",
            "sample": sample + f", C restatement oracle/liboracle.so, {rays} rays in {dt:.2f} s"}


def ref_provenance(path):
    """Which binary the baseline ran: its sha256 now, and the recipe commit / compiler / sha256 that
    oracle/ref/build_ref.sh recorded when it built it (oracle/_ref/BUILD_INFO.json; the binaries
    travel to the GPU box untracked, /root/reference is absent there)."""
    import hashlib
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for blk in iter(lambda: f.read(1 << 20), b""):
            h.update(blk)
    out = {"path": os.path.relpath(path, ROOT), "sha256": h.hexdigest()}
    try:
        info = json.load(open(os.path.join(os.path.dirname(path), "BUILD_INFO.json")))
        out.update({k: info.get(k) for k in ("recipe", "recipe_commit", "recipe_dirty", "compiler", "built_utc")})
        out["sha256_matches_build"] = info.get("sha256", {}).get(os.path.basename(path)) == out["sha256"]
    except (OSError, ValueError) as e:
        out["build_info"] = f"unavailable: {e}"[:120]
    return out


def contention_free(args, threads, sample):
    """The reference's shared std::atomic ray counter (main.cpp:55, 68) throttles its threads (SURVEY
    0: 14.3 -> 62.5 Mrays/s on 8 cores when removed).  The contention-free figure here is the
    product's CPU backend (MRT_DEVICE_CPU: the same hot-path source compiled for the host, scalar
    code, exact contract, per-thread ray counters) on the same threads and sample: a port without
    the reference's SSE Vec3, so not the reference's own contention-free speed."""
    import miniraytracer_amd as m
    sc = m.select_scene(args.scene, args.width / args.height)
    r = m.Renderer(sc, "cpu")
    t0 = time.perf_counter()
    _, rays = r.render(m.render_desc(args.width, args.height, args.cpu_spp, depth=args.depth, threads=threads))
    dt = time.perf_counter() - t0
    return {"value_contention_free": round(rays / dt / 1e6, 3), "kind_contention_free": "port",
            "sample_contention_free": sample + f", the product's CPU backend (per-thread ray counters, scalar host build), "
                                               f"{rays} rays in {dt:.2f} s on {threads} threads"}


def pmc_path(args):
    return args.pmc_json or os.path.join(ROOT, "profiles", f"pmc_s{args.scene}_{args.width}x{args.height}.json")


def roofline(args, k_ms, rays_per_launch, numerics, kinfo):
    """Roofline of the dominant kernel from the live HIP-event kernel time and this launch's rays,
    priced by the committed rocprofv3 per-ray counters of the same workload (profiles/pmc_*.json,
    tools/pmc_summary.py): VALU wave-instructions per ray -> VALU issue rate vs its peak (the bound:
    C2's path kernel issues VALU on ~3/4 of SIMD cycles), HBM bytes per ray (2*FETCH_SIZE +
    WRITE_SIZE, MI355X_MICROARCH.md) -> hbm_frac.  Per-ray figures, so a rank's share (world > 1)
    is priced by its own rays; they do not depend on spp."""
    k_s = k_ms * 1e-3
    # the kernel's name in rocprofv3 traces: per variant the tolerance contract runs the fast, the
    # denormal-flushing or the path-exact build (mrt_launch.h kFtzVariant / kPathExact)
    from miniraytracer_amd._lib import BUILDS
    build = BUILDS[kinfo.get("build", 0)]
    kname = "mrt_path_kernel" + ("" if build == "exact" else "_" + build)
    out = {"bound": "valu", "achieved": None, "peak": round(VALU_PEAK_G, 1), "unit": "G VALU wave-instr/s", "frac": None,
           "traffic": None, "kernel": kname, "kernel_ms": round(k_ms, 3),
           "rays_per_launch": int(rays_per_launch),
           **{k: kinfo[k] for k in ("grid", "wg", "lds_bytes", "vgprs", "tree_nodes")}}
    b_ray = B_RAY.get(args.scene)
    if b_ray is not None:
        gbs = rays_per_launch * b_ray / k_s / 1e9
        out["ref_equiv"] = {"bytes_per_ray": b_ray, "GBps": round(gbs, 1), "vs_hbm_peak": round(gbs / HBM_PEAK_GBS, 4),
                            "note": "reference-equivalent bytes (SURVEY 8(d) B_ray): what the reference's tests read per ray; "
                                    "cache-served here, not an HBM ceiling"}
    p = pmc_path(args)
    if not os.path.exists(p):
        out["note"] = f"no PMC profile {os.path.relpath(p, ROOT)} for this workload: frac unmeasured"
        return out
    pmc = json.load(open(p))
    cfg = pmc.get("config") or []
    e = pmc.get("by_numerics", {}).get(numerics)
    if cfg[:3] != [args.scene, args.width, args.height] or (len(cfg) > 4 and cfg[4] != args.depth) or not e:
        out["note"] = f"{os.path.relpath(p, ROOT)} is for config {cfg}: frac unmeasured"
        return out
    out["pmc_source"] = pmc.get("source")
    vpr = e.get("valu_insts_per_ray")
    if vpr:
        ach = vpr * rays_per_launch / k_s / 1e9
        out["achieved"] = round(ach, 1)
        out["frac"] = round(ach / VALU_PEAK_G, 4)
        out["valu_insts_per_ray"] = round(vpr, 3)
    if e.get("valu_lane_util") is not None:
        out["valu_lane_util"] = round(e["valu_lane_util"], 4)
        if out["frac"] is not None:
            out["lane_frac"] = round(out["frac"] * e["valu_lane_util"], 4)  # of the lane-throughput peak
    if e.get("valu_busy") is not None:
        out["valu_busy_pmc"] = round(e["valu_busy"], 4)  # the profiler's own issue-cycle fraction
    bpr = e.get("hbm_bytes_per_ray")
    if bpr:
        out["traffic"] = round(bpr * rays_per_launch)
        out["hbm_GBps"] = round(out["traffic"] / k_s / 1e9, 1)
        out["hbm_peak"] = HBM_PEAK_GBS
        out["hbm_frac"] = round(out["hbm_GBps"] / HBM_PEAK_GBS, 5)
    return out


def visible_gpus():
    """GPUs this process may use, counted without any HIP call: KFD topology nodes with SIMDs
    (sysfs), narrowed by HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES."""
    n = 0
    base = "/sys/class/kfd/kfd/topology/nodes"
    try:
        for d in os.listdir(base):
            try:
                props = dict(line.split()[:2] for line in open(os.path.join(base, d, "properties")) if line.strip())
            except (OSError, ValueError):
                continue
            if int(props.get("simd_count", "0")) > 0:
                n += 1
    except OSError:
        pass
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip()]))
    return n


def launch_ranks(args):
    """`bench.py --gpus N` without a launcher: start N rank processes of this script (one per GPU,
    RANK/LOCAL_RANK/WORLD_SIZE set, rendezvous on 127.0.0.1), like main() spawns one thread per
    worker (main.cpp:376-382).  This parent makes no HIP call (GPUs counted from sysfs) and does
    not import torch or the package; if any rank fails, the others are stopped and its exit code
    returned (instead of the rest waiting in a collective until a timeout)."""
    import socket
    same = bool(os.environ.get("MRT_SAME_GPU"))
    ndev = visible_gpus()
    if args.gpus > ndev and not same:
        print(f"bench.py: --gpus {args.gpus} but {ndev} GPU(s) visible (set MRT_SAME_GPU=1 to rehearse "
              f"several ranks on one GPU)", file=sys.stderr)
        return 2
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    while procs:
        time.sleep(0.2)
        for p in list(procs):
            r = p.poll()
            if r is None:
                continue
            procs.remove(p)
            if r != 0:
                rc = rc or r
                for q in procs:  # a failed rank: the others would block in a collective
                    q.terminate()
                for q in procs:
                    try:
                        q.wait(timeout=20)
                    except subprocess.TimeoutExpired:
                        q.kill()
                        q.wait()
                procs = []
                break
    return rc


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args))
    if env_world is not None and int(env_world) != args.gpus and "--gpus" in " ".join(sys.argv):
        print(f"bench.py: --gpus {args.gpus} disagrees with WORLD_SIZE={env_world}", file=sys.stderr)
        sys.exit(2)
    import torch
    import torch.distributed as dist
    import miniraytracer_amd as m

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("MRT_SAME_GPU"):  # rehearsal hook: every rank on GPU 0 (one-GPU box)
        local = 0
    multi = world > 1 or args.force_dist  # the multi-rank path (process group, per-step gather)
    if multi:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if "MASTER_PORT" not in os.environ:
            import socket
            sk = socket.socket()
            sk.bind(("127.0.0.1", 0))
            os.environ["MASTER_PORT"] = str(sk.getsockname()[1])
            sk.close()
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))
        torch.cuda.set_device(local)
        backend = os.environ.get("MRT_DIST_BACKEND", "nccl")  # nccl = RCCL over xGMI; gloo: rehearsal hook
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    # scene build + upload + workspace: outside the timed region (main.cpp:309 precedes 375)
    scene = m.select_scene(args.scene, args.width / args.height)
    d_rank, d_world = rank, world
    if world == 1 and args.emulate_world > 1:
        d_rank, d_world = args.emulate_rank, args.emulate_world
    n_paths_local = len(m.local_pixels(m.render_desc(args.width, args.height, args.samples, tile_size=args.tile_size,
                                                     rank=d_rank, world=d_world))) * (int(np.sqrt(np.float32(args.samples))) ** 2)
    # contexts: several only where they pay -- a short per-rank launch (its fixed start / tail costs
    # hidden by the other contexts' kernels); a full C2 render gains nothing and turns bimodal
    # (round 6: two contexts with the async fold for the short shares -- the 8-rank C2 share 1.102-1.114
    # against 1.123-1.137 ms per step with three contexts and the full fold, and steady: step-interval
    # p90 1.11 ms against 2.2 ms, profiles/r06_ab.txt sections 6-7)
    npipe = args.pipeline if args.pipeline > 0 else (2 if n_paths_local < 100_000_000 else 1)
    rnds = [m.Renderer(scene, device=local) for _ in range(npipe)]
    rnd = rnds[0]
    # The lean fold keeps one load in flight per lane, so beside the other contexts' path kernels it
    # needs ~ns load round trips whatever the pixel count: it wins while the rank's path kernel is
    # long (C2 per-rank share, lean vs full, ms/step: 1 rank 8.36 / 8.59, 2: 4.16 / 4.30, 4: 2.19 /
    # 2.16, 8: 1.19 / 1.15; round 2) -- auto: lean from ~96 M paths per rank, with several contexts
    lean_fold = args.fold == "lean"
    # auto: one or two contexts -> each render's fold beside the next render's path kernel (C2: 8.28 vs
    # 8.65 ms per step, profiles/r05_ab.txt section 27); more contexts -> the full fold after the kernel
    async_fold = args.fold == "async" or (args.fold == "auto" and npipe <= 2)
    def desc_of(numerics):
        return m.render_desc(args.width, args.height, args.samples, depth=args.depth, tile_size=args.tile_size,
                             rank=d_rank, world=d_world, numerics=numerics, chunk_samples=args.chunk_samples,
                             flags=m._lib.RF_FOLD_BEHIND if lean_fold else (m._lib.RF_FOLD_ASYNC if async_fold else 0))

    desc = desc_of(args.numerics)
    for r in rnds:
        r.prepare(desc)
    px = m.local_pixels(desc)
    n_local = len(px)
    n_rows = n_local
    tg = eg = comm = frame = None
    if multi and args.gather == "capi" and os.environ.get("MRT_SAME_GPU"):
        args.gather = "torch"  # RCCL refuses two ranks on one device: the rehearsal gathers over torch.distributed
    if multi and args.gather == "capi":
        # the C-ABI's RCCL gather (include/mrt.h mrt_comm_*): rank 0's communicator id to every rank
        # over torch.distributed, one communicator per rank on its GPU; the shards are gathered to
        # rank 0 and scattered into `frame` by mrt_gather_frame on ONE stream (gstream below), so the
        # communicator's collectives and buffers are used in issue order
        obj = [m.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        comm = m.Comm(local, world, rank, obj[0])
        frame = torch.zeros((args.width * args.height, 4), dtype=torch.float32, device=dev) if rank == 0 else None
    elif multi:
        from miniraytracer_amd.dist import TileGather
        tg = TileGather(args.width, args.height, args.samples, args.depth, world, rank, dev, tile_size=args.tile_size)
        assert tg.n_local == n_local
        n_rows = tg.n_max  # renders write straight into the padded shard the gather sends
    elif d_world > 1 and args.emulate_gather:
        from miniraytracer_amd.dist import TileGather
        eg = TileGather(args.width, args.height, args.samples, args.depth, d_world, 0, dev, tile_size=args.tile_size)
        n_rows = eg.n_max
    # output buffers: one per context, two per context when a gather reads them (multi) so a
    # render never waits for the previous gather of its own buffer (one context, C2 on 1-2 ranks)
    nbuf = npipe * (2 if multi else 1)
    outs = [torch.zeros((n_rows, 4), dtype=torch.float32, device=dev) for _ in range(nbuf)]
    rays = torch.zeros(1, dtype=torch.int64, device=dev)  # every context adds its rays here (device atomics)
    stream = torch.cuda.current_stream(dev)
    streams = [stream] + [torch.cuda.Stream(dev) for _ in range(npipe - 1)]
    # async fold: the gather waits for a render's fold on a stream of its own, so the next render's
    # path kernel is not ordered after it
    gstream = torch.cuda.Stream(dev) if (multi and (async_fold or comm is not None)) else None

    pending = [None]
    sent = [None] * nbuf  # the gather that last read output buffer b
    it = [0]
    ctx = [rnds]  # the render contexts measure() uses (the other-walk timing swaps in its own)

    def step(d):
        # step i renders with context i % npipe on its stream; nothing orders it after step i-1's
        # kernels, so its waves start on the CUs that step i-1's finished waves leave idle
        j = it[0] % npipe
        b = it[0] % nbuf
        it[0] += 1
        with torch.cuda.stream(streams[j]):
            if sent[b] is not None:  # the gather of this buffer's previous render has read it
                sent[b].wait()
            ctx[0][j].render_device(d, outs[b].data_ptr(), rays.data_ptr(), streams[j].cuda_stream)
            if comm is not None:
                # the one RCCL collective of the data path, on the gather stream after the render
                # (after its fold on the context's own stream under the async fold)
                if async_fold:
                    ctx[0][j].join(gstream.cuda_stream)
                else:
                    gstream.wait_stream(streams[j])
                comm.gather_frame(d, outs[b].data_ptr(), frame.data_ptr() if frame is not None else 0, 0, gstream.cuda_stream)
                ev = torch.cuda.Event()
                ev.record(gstream)
                sent[b] = ev  # the next render into outs[b] waits for it
            elif multi:
                # the one RCCL collective of the data path (tile shards -> rank 0), overlapped with
                # the next render: finish the previous step's gather, then start this one's
                if pending[0] is not None:
                    tg.finish(pending[0])
                if gstream is not None:
                    ctx[0][j].join(gstream.cuda_stream)
                    with torch.cuda.stream(gstream):
                        pending[0] = sent[b] = tg.start(outs[b])
                else:
                    pending[0] = sent[b] = tg.start(outs[b])
            elif eg is not None:
                eg.scatter()  # rehearsal: rank 0's device-side share of the gather

    def drain():
        if pending[0] is not None:
            tg.finish(pending[0])
            pending[0] = None

    def note(msg):  # progress on stderr: long renders (C5 at full size) keep the log moving
        if rank == 0:
            print(f"bench.py: {msg} ({time.strftime('%H:%M:%S')})", file=sys.stderr, flush=True)

    live = [None]  # (path-kernel ms per launch, launches per render) of the last measure()
    step_times = [None]  # --step-times: the timed steps' completion intervals

    def measure(d):
        """W untimed warmup steps, then EXACTLY K steps between barrier + synchronize on both
        sides; (max-over-ranks seconds, total rays of all ranks, this rank's rays per step); the
        path kernel's HIP-event time of the timed steps in live[0]."""
        note(f"measuring numerics={'fast' if d.flags & m._lib.RF_FAST else 'exact'}")
        # setup, untimed: one render per context, so every context's first-use costs (workspace
        # first touch, first launch on its stream) are paid before the warmup steps
        for j in range(npipe):
            with torch.cuda.stream(streams[j]):
                ctx[0][j].render_device(d, outs[j].data_ptr(), rays.data_ptr(), streams[j].cuda_stream)
        torch.cuda.synchronize(dev)
        tw = time.perf_counter()
        for _ in range(args.warmup):
            step(d)
        drain()
        torch.cuda.synchronize(dev)
        # clock settle, untimed: a fresh box's GPU ramps its clock over the first few hundred ms
        # of load (measured: a first C2 run's steps 11.7 ms against 10.0 ms once warm), so
        # warmup continues until ~0.5 s of GPU work has run, whatever W is
        # (local renders, no collective: ranks may run different counts before the barrier)
        while time.perf_counter() - tw < 0.5:
            with torch.cuda.stream(streams[0]):
                ctx[0][0].render_device(d, outs[0].data_ptr(), rays.data_ptr(), streams[0].cuda_stream)
            torch.cuda.synchronize(dev)
        rays.zero_()
        if multi:
            dist.barrier()
        torch.cuda.synchronize(dev)
        note("timed steps")
        evs = []
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step(d)
            if args.step_times:
                e = torch.cuda.Event(enable_timing=True)
                e.record(streams[(it[0] - 1) % npipe])
                evs.append(e)
        drain()
        torch.cuda.synchronize(dev)
        if multi:
            dist.barrier()
        t1 = time.perf_counter()
        # the path kernel's time inside the timed region: HIP events recorded around each launch on
        # its stream by the library, read for every context's last timed render (reading them here,
        # before any untimed work, keeps the clocks of the timed region: renders timed after the
        # parity check ran on a GPU that had idled for seconds, 8.6-9.0 ms against 8.0 ms)
        kl = [c.kernel_ms() for c in ctx[0][:min(npipe, max(args.steps, 1))]]
        live[0] = (float(np.mean([ms / max(n, 1) for ms, n in kl])), max(kl[0][1], 1))
        if len(evs) > 1:  # completion intervals of consecutive steps
            iv = np.array([evs[i - 1].elapsed_time(evs[i]) for i in range(1, len(evs))])
            step_times[0] = {"median_ms": round(float(np.median(iv)), 4), "p90_ms": round(float(np.percentile(iv, 90)), 4),
                             "max_ms": round(float(iv.max()), 4), "max_at_step": int(iv.argmax()) + 1,
                             "mean_ms": round(float(iv.mean()), 4), "intervals": len(iv)}
        elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
        total_rays = rays.clone()
        if multi:
            dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
            dist.all_reduce(total_rays, op=dist.ReduceOp.SUM)
        return float(elapsed.item()), int(total_rays.item()), int(rays.item()) // max(args.steps, 1)

    desc = desc_of(args.numerics)
    secs, nrays, rays_per_step_local = measure(desc)

    def last_image():
        """The assembled framebuffer of the last timed step (rank 0; None elsewhere)."""
        if comm is not None:
            return frame.view(args.height, args.width, 4).cpu().numpy() if rank == 0 else None
        if multi:
            return tg.full.view(args.height, args.width, 4).cpu().numpy() if rank == 0 else None
        full = np.zeros((args.width * args.height, 4), dtype=np.float32)
        full[px] = outs[(it[0] - 1) % nbuf][:n_local].cpu().numpy()
        return full.reshape(args.height, args.width, 4)

    # parity of the timed render (after the timed region): the last step's image against the
    # reference as shipped on the same per-path streams, when a fixture of this exact config exists
    fixture = None
    if not args.no_parity and d_world == world:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from fixture_cmp import compare, fixture_for
        fixture = fixture_for(args.scene, args.width, args.height, desc.sqrt_samples ** 2, args.depth)

    def parity(nrays_total):
        if fixture is None or rank != 0:
            return None
        r = compare(last_image(), nrays_total // max(args.steps, 1), fixture)
        return {k: (round(v, 7) if isinstance(v, float) else v) for k, v in r.items()}

    par = parity(nrays)

    verified = None
    if args.verify and d_world == world and rank == 0:
        img = last_image()
        ref, ref_rays = m.Renderer(scene, device=local).render(
            m.render_desc(args.width, args.height, args.samples, depth=args.depth, tile_size=args.tile_size,
                          numerics=args.numerics))
        verified = bool(np.array_equal(img[..., :3].view(np.uint32), ref[..., :3].view(np.uint32))
                        and nrays == ref_rays * args.steps)

    # dominant kernel: mrt_path_kernel, HIP events of the timed steps (measure())
    k_ms, launches = live[0]
    roof = roofline(args, k_ms, rays_per_step_local / launches, args.numerics, rnd.kernel_info())

    # the other numerics contract, same protocol (reported beside the headline, never as `value`)
    other = None
    if not args.no_compare_numerics:
        alt = "exact" if args.numerics == "fast" else "fast"
        a_secs, a_rays, a_local = measure(desc_of(alt))
        a_kms, a_launches = live[0]
        a_par = parity(a_rays)
        a_roof = roofline(args, a_kms, a_local / a_launches, alt, rnd.kernel_info())
        other = {"numerics": alt, "value": round(a_rays / a_secs / 1e6, 2), "ms_per_step": round(a_secs / args.steps * 1e3, 3),
                 "kernel_ms": round(a_kms, 3), "roofline_frac": a_roof["frac"], "valu_lane_util": a_roof.get("valu_lane_util"),
                 "hbm_frac": a_roof.get("hbm_frac"), "parity": a_par}

    # the general hit walk on the same workload: the shape-specialised walks (mrt_sig.h, e.g. the
    # Cornell box's slab tests) fire only for known program shapes; this times the linear-program
    # interpreter every other scene graph of that kind runs (MRT_NO_SIG=1 at scene upload)
    other_walk = None
    if not args.no_other_walk and (rnd.kernel_info()["kernel_features"] >> 16) != 0:
        os.environ["MRT_NO_SIG"] = "1"
        try:
            gen = [m.Renderer(scene, device=local) for _ in range(npipe)]
        finally:
            del os.environ["MRT_NO_SIG"]
        for r in gen:
            r.prepare(desc)
        ctx[0] = gen
        g_secs, g_rays, g_local = measure(desc)
        g_kms, g_launches = live[0]
        g_par = parity(g_rays)
        ctx[0] = rnds
        g_roof = roofline(args, g_kms, g_local / g_launches, args.numerics, gen[0].kernel_info())
        other_walk = {"walk": "linear-program interpreter (MRT_NO_SIG=1)", "numerics": args.numerics,
                      "kernel_features": gen[0].kernel_info()["kernel_features"],
                      "value": round(g_rays / g_secs / 1e6, 2), "ms_per_step": round(g_secs / args.steps * 1e3, 3),
                      "kernel_ms": round(g_kms, 3), "vgprs": g_roof["vgprs"], "parity": g_par,
                      "note": "VALU per ray differs from the specialised walk: no PMC for it, frac not priced"}
        for r in gen:
            r.close()

    if rank == 0:
        res = {
            "metric": METRIC,
            "value": round(nrays / secs / 1e6, 2),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(secs / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic scene (reference scene builder, deterministic seeds)",
            "config": {"workload": f"{WORKLOAD.get(args.scene, 'scene')}: scene {args.scene}, {args.width}x{args.height}, "
                                   f"{desc.sqrt_samples ** 2} spp, depth {args.depth}, draw() accumulation",
                       "scene": args.scene, "width": args.width, "height": args.height,
                       "spp": desc.sqrt_samples ** 2, "depth": args.depth, "parallelism": f"tiles{world}",
                       "tile_size": args.tile_size, "pipeline": npipe, **({"gather": args.gather} if multi else {}), "fold": "lean" if lean_fold else ("async" if async_fold else "full"), "numerics": args.numerics,
                       **({"emulated_share": f"rank {d_rank} of {d_world}" + (", + rank 0's scatter" if eg is not None else "")}
                          if d_world != world else {}),
                       "rays_per_step": nrays // args.steps},
            "roofline": roof,
            "parity": par,
            "cpu_baseline": None,
            "other_numerics": other,
            "other_walk": other_walk,
        }
        if verified is not None:
            res["verify_bit_exact"] = verified
        if step_times[0] is not None:
            res["step_times"] = step_times[0]
        if world == 1 and not args.no_cpu_baseline:
            try:
                res["cpu_baseline"] = cpu_baseline(args)
            except Exception as e:  # the baseline never blocks the GPU number
                res["cpu_baseline"] = {"error": str(e)[:200]}
        print(json.dumps(res), flush=True)
    if comm is not None:
        torch.cuda.synchronize(dev)
        comm.close()
    if multi:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
